cd $GRAFT_REPO_ROOT
for F in 8 16 32 64 128 4096; do timeout -k 10 120 python -u tools/onepass_perf.py $F 20 onepass 2>&1 | grep -E "^onepass |  onepass "; done

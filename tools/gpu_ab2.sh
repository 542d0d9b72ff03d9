# A/B of library builds x range-pass mode: tools/gpu_ab2.sh "lib1 lib2" "1 0" [rounds]
cd $GRAFT_REPO_ROOT
for r in $(seq ${3:-2}); do
  for n in $1; do for m in $2; do
    echo -n "$n pair=$m: "
    FMCW_ONEPASS_PAIR=$m FMCW_LIB=ab/$n.so timeout -k 10 120 python -u tools/onepass_perf.py 4096 20 onepass 2>&1 | grep -E "^onepass" || exit 1
  done; done
done

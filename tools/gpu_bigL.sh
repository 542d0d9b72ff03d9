set -u
cd $GRAFT_REPO_ROOT
for L in 65536 262144 940000; do timeout -k 10 200 python -u tools/stft_bigL.py $L 2>&1 | grep -v amdgpu.ids | tail -1 || exit 1; done

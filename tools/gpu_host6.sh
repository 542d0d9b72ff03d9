set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/host6; mkdir -p $O
timeout -k 10 200 python -u tools/host_probe.py 5 3 2>&1 | grep -v amdgpu.ids | tail -1
timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace --memory-copy-trace --stats -d $O/tr -o run --output-format csv -- python -u tools/host_probe.py 3 3 > $O/tr.log 2>&1; rc=$?; tail -1 $O/tr.log; exit $rc

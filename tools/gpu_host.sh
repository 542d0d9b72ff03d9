set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/host; mkdir -p $O
timeout -k 10 120 python -u tools/host_probe.py 300 2>&1 | grep -v amdgpu.ids | tail -2
timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace --memory-copy-trace --stats -d $O/tr -o run --output-format csv -- python -u tools/host_probe.py 100 > $O/tr.log 2>&1; rc=$?; tail -2 $O/tr.log; exit $rc

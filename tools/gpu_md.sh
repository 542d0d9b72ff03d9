set -u
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_multidev.py -v --timeout 120 --timeout-method thread > gpurun_out/md.log 2>&1; rc=$?
grep -E "PASSED|FAILED|SKIPPED|Error" gpurun_out/md.log | head -20; exit $rc

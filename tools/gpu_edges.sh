set -u
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_edges.py -v --timeout 120 --timeout-method thread > gpurun_out/edges.log 2>&1; rc=$?
grep -E "PASSED|FAILED|Error|assert" gpurun_out/edges.log | head -30; exit $rc

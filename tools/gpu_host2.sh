set -u
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/tests.log 2>&1; rc=$?
echo "tests rc=$rc: $(tail -1 gpurun_out/tests.log)"; [ $rc -ne 0 ] && { grep -E "Error|FAILED" gpurun_out/tests.log | head -20; exit $rc; }
for i in 1 2 3; do timeout -k 10 120 python -u tools/host_probe.py 300 2>&1 | grep -v amdgpu.ids | tail -1; done

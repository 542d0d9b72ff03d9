# the full GPU suite (one process), then nothing else
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_gpu.log 2>&1
rc=$?; tail -25 gpurun_out/t_gpu.log; exit $rc

# quick GPU check of the single-pass tree: its parity tests, then an A/B against ab/base.so
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_golden.py tests/test_gpu_onepass.py tests/test_gpu_device_path.py tests/test_gpu_parity.py -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/t_quick.log 2>&1; rc=$?
tail -3 gpurun_out/t_quick.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_ab.sh "$1" 4096 10 2

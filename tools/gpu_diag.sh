set -u
cd $GRAFT_REPO_ROOT
T="python -u -m pytest -q --timeout 120 --timeout-method thread"
timeout -k 10 300 $T tests/test_gpu_fullsize.py > gpurun_out/fs1.log 2>&1; echo "alone rc=$?: $(tail -1 gpurun_out/fs1.log)"; grep "Error:" gpurun_out/fs1.log | head -5
timeout -k 10 300 $T tests/test_gpu_device_path.py tests/test_gpu_fullsize.py > gpurun_out/fs2.log 2>&1; echo "after device_path rc=$?: $(tail -1 gpurun_out/fs2.log)"; grep "Error:" gpurun_out/fs2.log | head -5
timeout -k 10 300 $T tests/test_gpu_coresidency.py tests/test_gpu_fullsize.py > gpurun_out/fs3.log 2>&1; echo "after coresidency rc=$?: $(tail -1 gpurun_out/fs3.log)"; grep "Error:" gpurun_out/fs3.log | head -5
echo done

set -u
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_stft_coarse.py tests/test_gpu_parity.py tests/test_gpu_radar.py tests/test_gpu_multidev.py -v --timeout 120 --timeout-method thread > gpurun_out/coarse.log 2>&1; rc=$?
grep -E "FAILED|Error|passed|failed" gpurun_out/coarse.log | tail -8; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  echo -n "coarse: "; timeout -k 10 200 python -u tools/host_probe.py 5 3 2>&1 | grep -v amdgpu.ids | tail -1
  echo -n "full:   "; FMCW_STFT_COARSE=0 timeout -k 10 200 python -u tools/host_probe.py 5 3 2>&1 | grep -v amdgpu.ids | tail -1
done

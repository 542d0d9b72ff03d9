set -u
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_stft_coarse.py tests/test_gpu_parity.py -k "coarse or stft" -v --timeout 120 --timeout-method thread > gpurun_out/coarse.log 2>&1; rc=$?
grep -E "PASSED|FAILED|Error|assert" gpurun_out/coarse.log | head -30; [ $rc -ne 0 ] && exit $rc
for L in 262144 940000; do
  echo -n "coarse: "; FMCW_STFT_DEBUG=1 timeout -k 10 200 python -u tools/stft_bigL.py $L 2>&1 | grep -v amdgpu.ids | tail -2 | tr '\n' ' '; echo
  echo -n "full:   "; FMCW_STFT_COARSE=0 timeout -k 10 200 python -u tools/stft_bigL.py $L 2>&1 | grep -v amdgpu.ids | tail -1
done

cd $GRAFT_REPO_ROOT
for lib in fmcw_radar_processing_amd/libfmcw.so ab/plain.so; do
  echo "== $lib"; FMCW_LIB=$PWD/$lib timeout -k 10 300 python -u -m pytest tests/test_golden.py tests/test_gpu_onepass.py -m gpu -q --timeout 120 --timeout-method thread 2>&1 | grep -E "passed|failed|Error|assert np" | head -8
done
bash tools/gpu_ab.sh "plain wt" 4096 10 2

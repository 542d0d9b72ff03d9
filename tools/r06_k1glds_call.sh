# Round-6 K1 LDS-DMA A/B (ab/k1glds.so: -DK1_GLDS -DK1_WAVES=2; cur = the shipped K1): the range-FFT and
# streams parity tests on the variant, then the config-2 gap sweep (tools/place_probe.py k1) per library,
# alternating, then bench.py's config-2 line (placed + default allocation) per library.
cd $GRAFT_REPO_ROOT
FMCW_LIB=ab/k1glds.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -q -x \
  --timeout 120 --timeout-method thread > gpurun_out/k1glds_tests.log 2>&1; rc=$?
echo "k1glds tests rc=$rc: $(tail -1 gpurun_out/k1glds_tests.log)"; [ $rc -ne 0 ] && { tail -30 gpurun_out/k1glds_tests.log; exit $rc; }
for r in 1 2; do for n in cur k1glds; do
  lib=ab/$n.so; [ "$n" = cur ] && lib=fmcw_radar_processing_amd/libfmcw.so
  echo "== $n round $r"
  FMCW_LIB=$lib timeout -k 10 200 python3 -u tools/place_probe.py k1 > gpurun_out/k1p_${n}_$r.log 2>&1 || { tail -5 gpurun_out/k1p_${n}_$r.log; exit 1; }
  grep -v amdgpu gpurun_out/k1p_${n}_$r.log | tail -20
done; done
AB="cur k1glds" ROUNDS="1" timeout -k 10 400 bash tools/ab_bench.sh

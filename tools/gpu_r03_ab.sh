# Round-3 A/B call: the copy floor probe, then library variants under ab/ (tools/ab_build.sh)
# timed back to back (tools/onepass_perf.py, XCD schedule), each variant's k_rdx parity tests first.
#   tools/gpu_r03_ab.sh "name1 name2 ..." [rounds]
set -u
cd $GRAFT_REPO_ROOT
names=$1; N=${2:-2}
if [ -x tools/copy_probe.bin ] && [ "${NOCOPY:-0}" != "1" ]; then
  timeout -k 10 120 tools/copy_probe.bin > gpurun_out/copy_probe.log 2>&1; rc=$?
  cat gpurun_out/copy_probe.log; [ $rc -ne 0 ] && { echo "copy probe rc=$rc"; exit $rc; }
fi
for n in ${TESTS:-$names}; do
  FMCW_LIB=ab/$n.so timeout -k 10 300 python -u -m pytest tests/test_gpu_onepass.py -q -x -k "${KEXPR:-xcd}" --timeout 120 \
    --timeout-method thread > gpurun_out/abt_$n.log 2>&1; rc=$?
  echo "$n tests rc=$rc: $(tail -1 gpurun_out/abt_$n.log)"
  [ $rc -ne 0 ] && { tail -30 gpurun_out/abt_$n.log; exit $rc; }
done
for n in ${FULLTEST:-}; do
  FMCW_LIB=ab/$n.so timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 120 \
    --timeout-method thread > gpurun_out/abft_$n.log 2>&1; rc=$?
  echo "$n full gpu tests rc=$rc: $(tail -1 gpurun_out/abft_$n.log)"
  [ $rc -ne 0 ] && { tail -30 gpurun_out/abft_$n.log; exit $rc; }
done
for i in $(seq $N); do
  for n in $names; do
    echo -n "$n: "
    FMCW_LIB=ab/$n.so timeout -k 10 120 python -u tools/onepass_perf.py 4096 20 xcd > gpurun_out/ab_$n.log 2>&1 || { tail -5 gpurun_out/ab_$n.log; exit 1; }
    grep -E "^xcd| onepass |xk-stamps|sclk" gpurun_out/ab_$n.log | tr -s ' ' | tr '\n' ' '; echo
  done
done
for i in $(seq $N); do
  for n in ${K1:-}; do
    echo -n "$n: "
    FMCW_LIB=ab/$n.so timeout -k 10 120 python -u tools/k1_perf.py > gpurun_out/k1_$n.log 2>&1 || { tail -5 gpurun_out/k1_$n.log; exit 1; }
    grep "^k1" gpurun_out/k1_$n.log
  done
done
for i in $(seq $N); do
  for n in ${FP16NAMES:-}; do
    echo -n "$n fp16: "
    FP16=1 FMCW_LIB=ab/$n.so timeout -k 10 120 python -u tools/onepass_perf.py 4096 20 xcd > gpurun_out/ab16_$n.log 2>&1 || { tail -5 gpurun_out/ab16_$n.log; exit 1; }
    grep -E "^xcd| onepass " gpurun_out/ab16_$n.log | tr -s ' ' | tr '\n' ' '; echo
  done
done

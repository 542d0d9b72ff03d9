# K1 (config 2) A/B: library variants under ab/ (tools/ab_build.sh), parity tests then
# tools/k1_perf.py alternating.   tools/gpu_k1ab.sh "base nopf3 ..." [rounds]
set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/k1ab
mkdir -p $O
names=$1; N=${2:-3}
for n in $names; do
  FMCW_LIB=ab/$n.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -x -k "range_fft_only or process_matches or fp16" \
    --timeout 120 --timeout-method thread > $O/t_$n.log 2>&1; rc=$?
  echo "$n tests rc=$rc: $(tail -1 $O/t_$n.log)"; [ $rc -ne 0 ] && { tail -30 $O/t_$n.log; exit $rc; }
done
for i in $(seq $N); do
  for n in $names; do
    echo -n "$n: "
    FMCW_LIB=ab/$n.so timeout -k 10 120 python -u tools/k1_perf.py 4096 50 > $O/k1_$n.$i.log 2>&1 || { tail -5 $O/k1_$n.$i.log; exit 1; }
    grep "^k1" $O/k1_$n.$i.log
  done
done
echo call done

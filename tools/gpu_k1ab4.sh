# K1 A/B 4: taps from global memory (ab/tg) vs LDS (in-tree), at cpt 8 / 4.
set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/k1ab4
mkdir -p $O
FMCW_LIB=ab/tg.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -x -k "range_fft" --timeout 120 --timeout-method thread > $O/t.log 2>&1
rc=$?; echo "tests rc=$rc: $(tail -1 $O/t.log)"; [ $rc -ne 0 ] && { tail -30 $O/t.log; exit $rc; }
for i in 1 2 3; do
  for c in 8 4; do
    echo -n "lds cpt$c: "; FMCW_K1_CPT=$c timeout -k 10 120 python -u tools/k1_perf.py 4096 50 2>&1 | grep "^k1"
    echo -n "tg cpt$c: "; FMCW_LIB=ab/tg.so FMCW_K1_CPT=$c timeout -k 10 120 python -u tools/k1_perf.py 4096 50 2>&1 | grep "^k1"
  done
done
echo call done

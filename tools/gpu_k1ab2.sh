# K1 A/B 2: the LDS profile combine (in-tree build) at cpt 16 / 4 / 2 against ab/k1base (per-team
# atomics, cpt 16); parity tests of the combine first.
set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/k1ab2
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -x -k "range_fft" --timeout 120 --timeout-method thread > $O/t.log 2>&1
rc=$?; echo "tests rc=$rc: $(tail -1 $O/t.log)"; [ $rc -ne 0 ] && { tail -30 $O/t.log; exit $rc; }
for i in 1 2 3; do
  echo -n "k1base cpt16: "; FMCW_LIB=ab/k1base.so timeout -k 10 120 python -u tools/k1_perf.py 4096 50 2>&1 | grep "^k1"
  for c in 16 4 2; do
    echo -n "lds cpt$c: "; FMCW_K1_CPT=$c timeout -k 10 120 python -u tools/k1_perf.py 4096 50 2>&1 | grep "^k1"
  done
done
echo call done
timeout -k 10 200 tools/r04_probe.bin 9 > $O/probe9.log 2>&1; rc=$?
cat $O/probe9.log; [ $rc -ne 0 ] && { echo "probe rc=$rc"; exit $rc; }
echo probe done

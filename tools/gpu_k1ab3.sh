# K1 A/B 3: per-workgroup profile partials + reduction at cpt 8 / 4 against cpt 16 (whole-frame
# workgroups); parity tests of the combine first.
set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/k1ab3
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -x -k "range_fft" --timeout 120 --timeout-method thread > $O/t.log 2>&1
rc=$?; echo "tests rc=$rc: $(tail -1 $O/t.log)"; [ $rc -ne 0 ] && { tail -30 $O/t.log; exit $rc; }
for i in 1 2 3; do
  for c in 16 8 4 2; do
    echo -n "cpt$c: "; FMCW_K1_CPT=$c timeout -k 10 120 python -u tools/k1_perf.py 4096 50 2>&1 | grep "^k1"
  done
done
echo call done

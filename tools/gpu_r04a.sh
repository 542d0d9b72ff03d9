# Round-4 first GPU call: GPU suite and bench on the round-3 tree, then tools/r04_probe
# (copy ceiling, hand-off variants, store policies) with FETCH/WRITE/TCC passes.
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r04a
O=gpurun_out/r04a
if [ "${NOTESTS:-0}" != 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > $O/tests.log 2>&1
  rc=$?; echo "tests rc=$rc: $(tail -1 $O/tests.log)"; [ $rc -ne 0 ] && { tail -30 $O/tests.log; exit $rc; }
fi
if [ "${NOBENCH:-0}" != 1 ]; then
  timeout -k 10 400 python -u bench.py > $O/bench.log 2>&1; rc=$?
  echo "bench rc=$rc"; tail -c 600 $O/bench.log; [ $rc -ne 0 ] && exit $rc
fi
timeout -k 10 200 tools/r04_probe.bin ${PARTS:-0} > $O/probe.log 2>&1; rc=$?
cat $O/probe.log; [ $rc -ne 0 ] && { echo "probe rc=$rc"; exit $rc; }
for part in ${PMCPARTS:-2 3}; do
  for c in FETCH_SIZE WRITE_SIZE "TCC_HIT_sum TCC_MISS_sum"; do
    tag=$(echo $c | cut -d' ' -f1)
    timeout -s KILL 150 rocprofv3 --pmc $c --kernel-trace -d $O/p${part}_$tag -o run --output-format csv -- tools/r04_probe.bin $part > $O/p${part}_$tag.log 2>&1 || { echo "pmc $part $c failed"; tail -3 $O/p${part}_$tag.log; exit 1; }
  done
done
echo call done

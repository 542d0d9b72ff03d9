# One GPU call: full GPU suite on the in-tree library, then A/B timing of ab/ variants
# (tools/gpu_r03_ab.sh) and LDS counters (tools/pmc_lds.sh).  Env: AB="a b", PMC="a b", N=rounds
set -u
cd $GRAFT_REPO_ROOT
if [ "${NOTESTS:-0}" != 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/tests.log 2>&1
  rc=$?; echo "tests rc=$rc: $(tail -1 gpurun_out/tests.log)"; [ $rc -ne 0 ] && { tail -30 gpurun_out/tests.log; exit $rc; }
fi
if [ -n "${AB:-}" ]; then NOCOPY=1 bash tools/gpu_r03_ab.sh "$AB" ${N:-2} || exit 1; fi
if [ -n "${PMC:-}" ]; then bash tools/pmc_lds.sh "$PMC" || exit 1; fi
echo call done

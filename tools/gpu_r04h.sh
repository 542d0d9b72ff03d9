# Round-4 GPU round on the final tree: full GPU suite + smoke, the bench line (with CPU baseline
# and every check leg), then rocprofv3 stats + PMC passes (tools/profile_run.sh).
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
run() { local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > gpurun_out/$n.log 2>&1; local rc=$?
  echo "$n rc=$rc"; grep -v amdgpu.ids gpurun_out/$n.log | tail -${TAILN:-4} | cut -c1-400
  if [ $rc -ne 0 ]; then echo "STOP after $n"; exit $rc; fi; }
TAG=${1:-r04h}
run tests 900 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread
run smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
TAILN=1 run bench 600 python -u bench.py
[ "${NOPROF:-0}" = "1" ] || run prof 1100 bash tools/profile_run.sh $TAG
echo call done

# One GPU round: parity tests, the bench line, rocprof summaries into profiles/.
set -u
cd $GRAFT_REPO_ROOT
run() { local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > gpurun_out/$n.log 2>&1; local rc=$?
  echo "$n rc=$rc"; grep -v amdgpu.ids gpurun_out/$n.log | tail -${TAILN:-6}
  if [ $rc -ne 0 ]; then echo "STOP after $n"; exit $rc; fi; }
TAG=${1:-${TAG:-r02}}
run tests 900 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread
TAILN=2 run bench 600 python -u bench.py
[ "${NOPROF:-0}" = "1" ] || run prof 1100 bash tools/profile_run.sh $TAG

# One GPU round for the XCD schedule: full parity suite, the bench line, the
# stamps breakdown of k_rdx, then rocprof summaries (tools/profile_run.sh).
set -u
cd $GRAFT_REPO_ROOT
run() { local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > gpurun_out/$n.log 2>&1; local rc=$?
  echo "$n rc=$rc"; grep -v amdgpu.ids gpurun_out/$n.log | tail -${TAILN:-4} | cut -c1-400
  if [ $rc -ne 0 ]; then echo "STOP after $n"; exit $rc; fi; }
TAG=${1:-r02e}
run tests 900 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread
TAILN=1 run bench 600 python -u bench.py
[ -f ab/xst.so ] && { FMCW_LIB=ab/xst.so timeout -k 10 120 python -u tools/onepass_perf.py 4096 3 xcd > gpurun_out/stamps.log 2>&1; grep xk-stamps gpurun_out/stamps.log | tail -2; }
[ "${NOPROF:-0}" = "1" ] || run prof 1100 bash tools/profile_run.sh $TAG

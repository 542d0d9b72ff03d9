set -u
cd $GRAFT_REPO_ROOT
run() { local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > gpurun_out/$n.log 2>&1; local rc=$?
  echo "$n rc=$rc"; grep -v amdgpu.ids gpurun_out/$n.log | tail -${TAILN:-12}
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP after $n"; exit $rc; fi; }
run tests 900 python -m pytest tests -m gpu -q -x
run probe 300 python tools/perf_probe.py ${PROBE_ARGS:-streams range}

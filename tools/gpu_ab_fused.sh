set -u
cd $GRAFT_REPO_ROOT
run() { # name, timeout, cmd...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > gpurun_out/$n.log 2>&1; local rc=$?
  echo "$n rc=$rc"; tail -${TAILN:-3} gpurun_out/$n.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP after $n"; exit $rc; fi
  return 0
}
run fused_tests 600 python -m pytest tests/test_gpu_fused.py -x -q
TAILN=40 run probe 600 python tools/perf_probe.py streams fused:2 fused:3 fused:4 range
run all_gpu_tests 900 python -m pytest tests -m gpu -q

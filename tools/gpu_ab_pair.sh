set -u
cd $GRAFT_REPO_ROOT
run() { local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > gpurun_out/$n.log 2>&1; local rc=$?
  echo "$n rc=$rc"; grep -v amdgpu.ids gpurun_out/$n.log | tail -${TAILN:-12}
  if [ $rc -ne 0 ]; then echo "STOP after $n"; exit $rc; fi; }
FMCW_PAIR=0 run pair0 300 python tools/perf_probe.py streams range
FMCW_PAIR=1 run pair1 300 python tools/perf_probe.py streams range
FMCW_PAIR=0 run pair0b 300 python tools/perf_probe.py streams range
FMCW_PAIR=1 run pair1b 300 python tools/perf_probe.py streams range

set -u
cd $GRAFT_REPO_ROOT
run() { local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > gpurun_out/$n.log 2>&1; local rc=$?
  echo "$n rc=$rc"; grep -v amdgpu.ids gpurun_out/$n.log | tail -${TAILN:-12}
  if [ $rc -ne 0 ]; then echo "STOP after $n"; exit $rc; fi; }
run s3 300 python tools/perf_probe.py streams range
FMCW_ONE_STREAM=1 run s1 300 python tools/perf_probe.py streams
run s3b 300 python tools/perf_probe.py streams
FMCW_ONE_STREAM=1 run s1b 300 python tools/perf_probe.py streams

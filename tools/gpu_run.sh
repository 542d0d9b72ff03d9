#!/bin/bash
# One GPU call made of steps, each under its own time limit, stopping at the first failure
# (no GPU step runs after a fault, an abort or a time limit).  Output: gpurun_out/<name>.log.
#   tools/gpu_run.sh 'tests' 'tests1 tests/test_gpu_slow_leg.py' 'bench' 'bench2 --stft-form direct' \
#                    'prof r05b' 'perf xcd' 'cmd name python -u tools/x.py'
# step forms (the first word names the log; a digit suffix tells repeated steps apart):
#   tests[N] [pytest args]   GPU tests (default: the whole -m gpu suite)
#   bench[N] [bench args]    bench.py line (last line printed)
#   prof <tag> [bench args]  rocprofv3 stats + PMC passes (tools/profile_run.sh)
#   perf[N] <schedules>      tools/onepass_perf.py 4096 20 <schedules> (FMCW_LIB / FP16 from the env)
#   cmd <name> <command...>  any command, 300 s
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for step in "$@"; do
  set -- $step
  kind=$1; shift
  case $kind in
    tests*) name=$kind; lim=900
            [ $# -eq 0 ] && set -- tests -m gpu
            cmd=(python -u -m pytest -q -x --timeout 120 --timeout-method thread "$@");;
    bench*) name=$kind; lim=600; cmd=(python -u bench.py "$@");;
    prof)   name=prof_$1; lim=1100; cmd=(bash tools/profile_run.sh "$@");;
    perf*)  name=$kind; lim=200; cmd=(python -u tools/onepass_perf.py 4096 20 "${1:-xcd}");;
    cmd)    name=$1; shift; lim=300; cmd=("$@");;
    *) echo "unknown step '$step'"; exit 2;;
  esac
  timeout -k 10 $lim "${cmd[@]}" > gpurun_out/$name.log 2>&1
  rc=$?
  echo "== $name rc=$rc"
  grep -v amdgpu.ids gpurun_out/$name.log | tail -${TAILN:-3} | cut -c1-600
  if [ $rc -ne 0 ]; then echo "STOP after $name"; exit $rc; fi
done
echo "== all steps done"

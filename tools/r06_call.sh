#!/bin/bash
# Round-6 GPU call driver: steps chained, each under its own limit, stop at the first failure.
#   tools/r06_call.sh tests | ab "<names>" [bench args] | trace <tag> | clock <tag> <cmd...> | bench
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
step=$1; shift
case $step in
  tests) timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread "$@" > gpurun_out/tests.log 2>&1
         rc=$?; echo "tests rc=$rc: $(tail -1 gpurun_out/tests.log)"; [ $rc -ne 0 ] && tail -30 gpurun_out/tests.log; exit $rc;;
  ab)    names=$1; shift; AB="$names" ROUNDS="${ROUNDS:-1 2}" bash tools/ab_bench.sh "$@"; exit $?;;
  trace) bash tools/trace_gaps.sh "$@"; exit $?;;
  clock) bash tools/clock_pmc.sh "$@"; exit $?;;
  bench) timeout -k 10 600 python -u bench.py "$@" > gpurun_out/bench.log 2>&1; rc=$?; tail -c 600 gpurun_out/bench.log; exit $rc;;
  *) echo "unknown step $step"; exit 2;;
esac

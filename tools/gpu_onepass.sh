# Single-pass schedule check on one GPU: its parity tests, then the schedule A/B probe.
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
run() { local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > gpurun_out/$n.log 2>&1; local rc=$?
  echo "$n rc=$rc"; grep -v amdgpu.ids gpurun_out/$n.log | tail -${TAILN:-8}
  if [ $rc -ne 0 ]; then echo "STOP after $n"; exit $rc; fi; }
TAILN=15 run op_tests 300 python -u -m pytest tests/test_gpu_onepass.py -m gpu -x -v --timeout 120 --timeout-method thread
TAILN=20 run op_perf 300 python -u tools/onepass_perf.py 4096 10
TAILN=6 run all_tests 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread

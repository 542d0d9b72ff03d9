# Round-4 GPU call: full GPU suite, then an A/B of k_rdx's cooperative vs plain launch
# (bench.py headline step only, alternating on one box).
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r04c
mkdir -p $O
if [ "${NOTESTS:-0}" != 1 ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > $O/tests.log 2>&1
  rc=$?; echo "tests rc=$rc: $(tail -1 $O/tests.log)"; [ $rc -ne 0 ] && { tail -30 $O/tests.log; exit $rc; }
fi
B="python -u bench.py --cpu-seconds 0 --no-extras --no-check --steps 20"
for i in 1 2; do
  for m in 1 0; do
    FMCW_XCD_PLAIN_LAUNCH=$m timeout -k 10 200 $B > $O/ab_plain$m.$i.log 2>&1; rc=$?
    [ $rc -ne 0 ] && { echo "bench plain=$m rc=$rc"; tail -5 $O/ab_plain$m.$i.log; exit $rc; }
    python3 -c "
import json,sys
for l in open('$O/ab_plain$m.$i.log'):
    if l.startswith('{'):
        d=json.loads(l); print('plain=$m', d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'], d['stages_ms_per_step'])"
  done
done
echo call done

#!/bin/bash
# Soak of the headline step: 2000 timed config-4 steps (8.19 M frames) per storage format, one process each;
# bench.py exits non-zero on any k_rdx hand-off timeout (fmcw_synchronize after the timed steps) and on a
# full-size check failure.  -> one line per run: frames/s, ms per step, k_rdx us (HIP events)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for v in "fp32" "fp16 --fp16"; do
  set -- $v; n=$1; shift
  timeout -k 10 300 python3 -u bench.py --steps 2000 --warmup 10 --no-extras --cpu-seconds 0 "$@" > gpurun_out/soak_$n.log 2>&1
  rc=$?
  echo "$n rc=$rc $(python3 -c "
import json,sys
d=json.loads([l for l in open('gpurun_out/soak_$n.log').read().splitlines() if l.startswith('{')][-1])
print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'], {k: v['pass'] for k, v in (d.get('checked') or {}).items()})
" 2>/dev/null)"
  [ $rc -ne 0 ] && { tail -5 gpurun_out/soak_$n.log; exit $rc; }
done
exit 0

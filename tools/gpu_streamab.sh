# A/B: bench.py on one explicit torch stream (current) vs the engine's own stream (bench_prev.py)
set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/streamab; mkdir -p $O
for i in 1 2; do
  for v in bench bench_prev; do
    timeout -k 10 300 python -u $v.py --cpu-seconds 0 --no-check --no-host-path --steps 20 > $O/$v.$i.log 2>&1; rc=$?
    [ $rc -ne 0 ] && { echo "$v rc=$rc"; tail -5 $O/$v.$i.log; exit $rc; }
    python3 -c "
import json
for l in open('$O/$v.$i.log'):
    if l.startswith('{'):
        d=json.loads(l); print('$v', d['value'], d['roofline']['avg_launch_us'], 'cfg2', d['config2_range_fft']['roofline']['avg_launch_us'], 'fp16', d['fp16_storage']['roofline']['avg_launch_us'])"
  done
done

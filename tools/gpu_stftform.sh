set -u
cd $GRAFT_REPO_ROOT
for i in 1 2 3; do
  for f in stored direct; do
    timeout -k 10 200 python -u bench.py --cpu-seconds 0 --no-extras --steps 20 --stft-form $f > gpurun_out/sf_$f.$i.log 2>&1 || { echo "$f failed"; tail -3 gpurun_out/sf_$f.$i.log; exit 1; }
    python3 -c "
import json
for l in open('gpurun_out/sf_$f.$i.log'):
    if l.startswith('{'):
        d=json.loads(l); print('$f', d['value'], d['stages_ms_per_step'], d['checked']['config4_f32']['pass'])"
  done
done

# Round-4 GPU call: K1 occupancy A/B (ab/ variants), probe part E (hand-off traffic vs sync),
# STFT leg direct-dB vs stored-P A/B (bench.py headline step).
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r04d
mkdir -p $O
bash tools/gpu_k1ab.sh "${K1NAMES:-base nopf3 nopf2 pf3}" 3 || exit 1
timeout -k 10 200 tools/r04_probe.bin 5 > $O/probe5.log 2>&1; rc=$?
cat $O/probe5.log; [ $rc -ne 0 ] && { echo "probe rc=$rc"; exit $rc; }
B="python -u bench.py --cpu-seconds 0 --no-extras --steps 20"
for i in 1 2; do
  for f in direct stored; do
    timeout -k 10 300 $B --stft-form $f > $O/stft_$f.$i.log 2>&1; rc=$?
    [ $rc -ne 0 ] && { echo "bench $f rc=$rc"; tail -5 $O/stft_$f.$i.log; exit $rc; }
    python3 -c "
import json
for l in open('$O/stft_$f.$i.log'):
    if l.startswith('{'):
        d=json.loads(l); c=d['checked']['config4_f32']
        print('$f', d['value'], d['ms_per_step'], d['stages_ms_per_step'], 'stft_db', c['stft_max_abs_db'], c['pass'])"
  done
done
echo call done

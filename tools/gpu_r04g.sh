# Round-4 GPU call: STFT changes (general-nfft MFMA, pmax pre-check): tests, STFT-form A/B,
# then one full bench (extras + host path + CPU baseline).
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r04g
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_stft_mfma.py tests/test_gpu_device_path.py tests/test_gpu_parity.py tests/test_gpu_radar.py tests/test_gpu_multidev.py -q -x --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc: $(tail -1 $O/tests.log)"; [ $rc -ne 0 ] && { tail -30 $O/tests.log; exit $rc; }
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
timeout -k 10 500 python -u bench.py > $O/bench_full.log 2>&1; rc=$?
echo "full bench rc=$rc"; [ $rc -ne 0 ] && { tail -5 $O/bench_full.log; exit $rc; }
python3 -c "
import json
for l in open('$O/bench_full.log'):
    if l.startswith('{'):
        d=json.loads(l); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['stages_ms_per_step']); print(json.dumps(d.get('host_path'))[:1500])"
echo call done

# Round-4 GPU call: MFMA STFT (direct dB) tests, bench A/B of the STFT leg forms.
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r04f
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_stft_mfma.py tests/test_gpu_device_path.py tests/test_gpu_parity.py -q -x --timeout 120 --timeout-method thread > $O/tests.log 2>&1
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
echo call done

# Round-4 GPU call: probe part F (k_rdx's protocol with deferred group, by unit size), GPU suite
# (3-wave K1, MFMA STFT), config-2 K1 timing, bench with the MFMA STFT vs the VALU one.
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r04e
mkdir -p $O
timeout -k 10 200 tools/r04_probe.bin 6 > $O/probe6.log 2>&1; rc=$?
cat $O/probe6.log; [ $rc -ne 0 ] && { echo "probe rc=$rc"; exit $rc; }
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc: $(tail -1 $O/tests.log)"; [ $rc -ne 0 ] && { tail -30 $O/tests.log; exit $rc; }
for i in 1 2; do timeout -k 10 120 python -u tools/k1_perf.py 4096 50 2>&1 | grep "^k1"; done
B="python -u bench.py --cpu-seconds 0 --no-extras --steps 20"
for i in 1 2; do
  for m in 1 0; do
    FMCW_STFT_MFMA=$m timeout -k 10 300 $B > $O/stft_m$m.$i.log 2>&1; rc=$?
    [ $rc -ne 0 ] && { echo "bench mfma=$m rc=$rc"; tail -5 $O/stft_m$m.$i.log; exit $rc; }
    python3 -c "
import json
for l in open('$O/stft_m$m.$i.log'):
    if l.startswith('{'):
        d=json.loads(l); c=d['checked']['config4_f32']
        print('mfma=$m', d['value'], d['ms_per_step'], d['stages_ms_per_step'], 'stft_db', c['stft_max_abs_db'], c['pass'])"
  done
done
echo call done

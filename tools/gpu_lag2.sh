# k_rdx poll lag 2 (4 slots, ab/lag2.so) against lag 1 (ab/base.so): parity tests, then the bench step alternating
set -u
cd $GRAFT_REPO_ROOT
O=gpurun_out/lag2; mkdir -p $O
FMCW_LIB=ab/lag2.so timeout -k 10 300 python -u -m pytest tests/test_gpu_onepass.py tests/test_gpu_fullsize.py tests/test_gpu_coresidency.py -q -x --timeout 120 --timeout-method thread > $O/t.log 2>&1
rc=$?; echo "lag2 tests rc=$rc: $(tail -1 $O/t.log)"; [ $rc -ne 0 ] && { tail -30 $O/t.log; exit $rc; }
B="python -u bench.py --cpu-seconds 0 --no-check --no-host-path --steps 20"
for i in 1 2 3; do
  for v in base lag2; do
    FMCW_LIB=ab/$v.so timeout -k 10 200 $B > $O/ab_$v.$i.log 2>&1; rc=$?
    [ $rc -ne 0 ] && { echo "bench $v rc=$rc"; tail -5 $O/ab_$v.$i.log; exit $rc; }
    python3 -c "
import json
for l in open('$O/ab_$v.$i.log'):
    if l.startswith('{'):
        d=json.loads(l); print('$v', d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'], 'fp16', d['fp16_storage']['roofline']['avg_launch_us'])"
  done
done
echo call done

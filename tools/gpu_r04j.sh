# Round-4 probe part J: slot reuse proven by done counters (1-slot ring), with PMC.
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r04j
mkdir -p $O
for r in 1 2; do
  timeout -k 10 120 tools/r04_probe.bin 10 > $O/probe10_$r.log 2>&1; rc=$?
  cat $O/probe10_$r.log; [ $rc -ne 0 ] && { echo "probe rc=$rc"; exit $rc; }
done
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --kernel-trace -d $O/p10_$c -o run --output-format csv -- tools/r04_probe.bin 10 > $O/p10_$c.log 2>&1 || { echo "pmc failed"; tail -3 $O/p10_$c.log; exit 1; }
done
echo call done
# k_rdx with one slot and a done counter (ab/done.so) against the same tree's 2-slot ring (ab/base.so)
FMCW_LIB=ab/done.so timeout -k 10 300 python -u -m pytest tests/test_gpu_onepass.py -q -x --timeout 120 --timeout-method thread > $O/t_done.log 2>&1
rc=$?; echo "done tests rc=$rc: $(tail -1 $O/t_done.log)"; [ $rc -ne 0 ] && { tail -30 $O/t_done.log; exit $rc; }
B="python -u bench.py --cpu-seconds 0 --no-extras --no-check --steps 20"
for i in 1 2 3; do
  for v in base done; do
    FMCW_LIB=ab/$v.so timeout -k 10 200 $B > $O/ab_$v.$i.log 2>&1; rc=$?
    [ $rc -ne 0 ] && { echo "bench $v rc=$rc"; tail -5 $O/ab_$v.$i.log; exit $rc; }
    python3 -c "
import json
for l in open('$O/ab_$v.$i.log'):
    if l.startswith('{'):
        d=json.loads(l); print('$v', d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'])"
  done
done
for c in FETCH_SIZE WRITE_SIZE; do
  FMCW_LIB=ab/done.so timeout -s KILL 200 rocprofv3 --pmc $c --kernel-trace -d $O/pd_$c -o run --output-format csv -- python -u bench.py --cpu-seconds 0 --no-extras --no-check --steps 3 --warmup 1 > $O/pd_$c.log 2>&1 || { echo "pmc failed"; tail -3 $O/pd_$c.log; exit 1; }
done
echo call2 done

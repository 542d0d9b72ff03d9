# Round-4 GPU call: cooperative-launch k_rdx (co-residency test + XCD tests + bench), then
# tools/r04_probe part D (cache policies / unit size) with FETCH/WRITE/TCC passes.
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r04b
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_coresidency.py tests/test_gpu_onepass.py -v -s -x --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc: $(tail -1 $O/tests.log)"; grep -E "hold|PASS|FAIL" $O/tests.log | head -20; [ $rc -ne 0 ] && { tail -30 $O/tests.log; exit $rc; }
timeout -k 10 400 python -u bench.py --cpu-seconds 0 --no-host-path > $O/bench.log 2>&1; rc=$?
echo "bench rc=$rc"; tail -c 1500 $O/bench.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 tools/r04_probe.bin 4 > $O/probe.log 2>&1; rc=$?
cat $O/probe.log; [ $rc -ne 0 ] && { echo "probe rc=$rc"; exit $rc; }
for c in FETCH_SIZE WRITE_SIZE "TCC_HIT_sum TCC_MISS_sum"; do
  tag=$(echo $c | cut -d' ' -f1)
  timeout -s KILL 150 rocprofv3 --pmc $c --kernel-trace -d $O/p4_$tag -o run --output-format csv -- tools/r04_probe.bin 4 > $O/p4_$tag.log 2>&1 || { echo "pmc $c failed"; tail -3 $O/p4_$tag.log; exit 1; }
done
echo call done

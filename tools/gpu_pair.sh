# pair-exchange single pass: GPU tests, then perf pair vs 8-tile, then stamps
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_onepass.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_onepass.log 2>&1
rc=$?; tail -15 gpurun_out/t_onepass.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP rc=$rc"; exit $rc; fi
for r in 1 2; do
  for m in 1 0; do echo -n "pair=$m: "; FMCW_ONEPASS_PAIR=$m timeout -k 10 120 python -u tools/onepass_perf.py 4096 20 onepass 2>&1 | grep -E "^onepass" || exit 1; done
done
FMCW_LIB=ab/stamps.so timeout -k 10 120 python -u tools/onepass_perf.py 4096 3 onepass > gpurun_out/st_pair.log 2>&1; grep stamps gpurun_out/st_pair.log | tail -1

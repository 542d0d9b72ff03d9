cd $GRAFT_REPO_ROOT
FMCW_ONEPASS_PAIR=0 FMCW_LIB=ab/rot1.so timeout -k 10 400 python -u -m pytest tests/test_gpu_onepass.py -x -q --timeout 120 --timeout-method thread -k "not range_pass_modes and not handoff" > gpurun_out/t_rot.log 2>&1
rc=$?; tail -5 gpurun_out/t_rot.log
if [ $rc -ne 0 ]; then echo "STOP rc=$rc"; exit $rc; fi
bash tools/gpu_ab2.sh "rot0 rot1 rot4" "0" 2
FMCW_ONEPASS_PAIR=0 FMCW_LIB=ab/stamps_rot1.so timeout -k 10 120 python -u tools/onepass_perf.py 4096 3 onepass 2>&1 | grep stamps | tail -1

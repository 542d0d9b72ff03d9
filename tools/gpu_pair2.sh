cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 -L > gpurun_out/counters.txt 2>&1
for m in 1 0; do
  FMCW_ONEPASS_PAIR=$m FMCW_LIB=ab/stamps.so timeout -k 10 120 python -u tools/onepass_perf.py 4096 3 onepass > gpurun_out/st_pair$m.log 2>&1; grep stamps gpurun_out/st_pair$m.log | tail -2
done
for m in 1 0; do
  out=gpurun_out/sq_pair$m; mkdir -p $out
  FMCW_ONEPASS_PAIR=$m timeout -k 10 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT --kernel-trace -d $out/sq -o run --output-format csv -- python3 tools/onepass_perf.py 2048 3 onepass > $out/sq.log 2>&1 || exit 14
  FMCW_ONEPASS_PAIR=$m timeout -k 10 200 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD GRBM_GUI_ACTIVE --kernel-trace -d $out/sq2 -o run --output-format csv -- python3 tools/onepass_perf.py 2048 3 onepass > $out/sq2.log 2>&1 || exit 16
  python3 tools/pmc_summary.py $out > $out/summary.txt 2>&1; grep -E "k_rd1p" $out/summary.txt
done

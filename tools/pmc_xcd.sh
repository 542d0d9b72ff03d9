#!/bin/bash
# PMC passes (one counter group each) over tools/onepass_perf.py for one schedule:
#   tools/pmc_xcd.sh <mode: xcd|onepass> <tag>  -> gpurun_out/pmc_<tag>_<group>/
cd $GRAFT_REPO_ROOT
mode=$1; tag=$2
export TMPDIR=/tmp
P="python3 tools/onepass_perf.py 4096 2 $mode"
i=0
for g in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum" "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $g --kernel-trace -d gpurun_out/pmc_${tag}_$i -o run --output-format csv -- $P > gpurun_out/pmc_${tag}_$i.log 2>&1 || { echo "pass $i ($g) failed"; tail -5 gpurun_out/pmc_${tag}_$i.log; exit 1; }
done
echo pmc done

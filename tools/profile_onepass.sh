#!/bin/bash
# rocprofv3 passes over tools/onepass_perf.py (single-pass schedule only):
# kernel stats, then one PMC group per pass.  usage: tools/profile_onepass.sh <tag> [F reps]
set -o pipefail
tag=$1; shift
out=gpurun_out/op_$tag
mkdir -p $out
export TMPDIR=/tmp
F=${1:-2048}; R=${2:-3}
P="python3 tools/onepass_perf.py $F $R onepass"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $out/stats -o run --output-format csv -- $P > $out/stats.log 2>&1 || exit 11
timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $out/fetch -o run --output-format csv -- $P > $out/fetch.log 2>&1 || exit 12
timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $out/write -o run --output-format csv -- $P > $out/write.log 2>&1 || exit 13
timeout -k 10 200 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT --kernel-trace -d $out/sq -o run --output-format csv -- $P > $out/sq.log 2>&1 || exit 14
timeout -k 10 200 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE --kernel-trace -d $out/tcc -o run --output-format csv -- $P > $out/tcc.log 2>&1 || exit 15
timeout -k 10 200 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INSTS_FLAT SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD --kernel-trace -d $out/sq2 -o run --output-format csv -- $P > $out/sq2.log 2>&1 || exit 16
python3 tools/pmc_summary.py $out > $out/summary.txt 2>&1
echo done

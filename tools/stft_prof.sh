#!/bin/bash
# STFT leg under rocprofv3 (tools/stft_perf.py): kernel stats for the folded and the k_stft64m
# forms, one SQ counter pass and one clock pass on the folded form, and the folded form's timing
# at 1, 2 and 4 blocks per CU.  Output: gpurun_out/stp_*.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
o=gpurun_out
step() { n=$1; shift; timeout -k 10 ${LIM:-150} "$@" > $o/stp_$n.log 2>&1; rc=$?; echo "== $n rc=$rc"; grep -E "us per call" $o/stp_$n.log; [ $rc -ne 0 ] && { tail -5 $o/stp_$n.log; exit $rc; }; return 0; }
F=${FORMS:-max,direct,stored}
step stats_fold rocprofv3 --kernel-trace --stats -d $o/stp_stats_fold -o run --output-format csv -- python3 tools/stft_perf.py 20 $F
step stats_m env FMCW_STFT64_FOLD=0 rocprofv3 --kernel-trace --stats -d $o/stp_stats_m -o run --output-format csv -- python3 tools/stft_perf.py 20 $F
LIM=60 step sq timeout -s KILL 60 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT --kernel-trace -d $o/stp_sq -o run --output-format csv -- python3 tools/stft_perf.py 3 $F
LIM=60 step clk timeout -s KILL 60 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace -d $o/stp_clk -o run --output-format csv -- python3 tools/stft_perf.py 3 $F
for b in ${BPCS:-1 2 4}; do step bpc$b env FMCW_STFT64_BPC=$b python3 -u tools/stft_perf.py 50 $F; done
echo "== stft_prof done"

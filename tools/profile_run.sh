#!/bin/bash
# rocprofv3 passes over bench.py: kernel stats (+ the bench's own JSON line),
# then one PMC group per pass (FETCH_SIZE and WRITE_SIZE cannot share a pass).
# Writes gpurun_out/prof_<tag>/ (merged back by gpurun); tools/collect_profiles.sh
# then writes the judged summaries under profiles/ in the build container.
# usage: tools/profile_run.sh <tag> [bench args...]
set -o pipefail
tag=$1; shift
out=gpurun_out/prof_$tag
mkdir -p $out
export TMPDIR=/tmp
B="python3 bench.py --cpu-seconds 0 --no-fanout --no-host-path --no-check"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/stats -o run --output-format csv -- $B --steps 20 --warmup 30 "$@" > $out/stats.log 2>&1 || exit 11
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $out/fetch -o run --output-format csv -- $B --steps 2 --warmup 1 "$@" > $out/fetch.log 2>&1 || exit 12
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $out/write -o run --output-format csv -- $B --steps 2 --warmup 1 "$@" > $out/write.log 2>&1 || exit 13
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT --kernel-trace -d $out/sq -o run --output-format csv -- $B --steps 2 --warmup 1 "$@" > $out/sq.log 2>&1 || exit 14
timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE --kernel-trace -d $out/tcc -o run --output-format csv -- $B --steps 2 --warmup 1 "$@" > $out/tcc.log 2>&1 || exit 15
echo done

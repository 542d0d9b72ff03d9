#!/bin/bash
# Copy the judged summaries of a GPU round (gpurun_out/prof_<tag>, merged back
# by gpurun) into profiles/.  usage: tools/collect_profiles.sh <tag> [--fp16]
set -e
tag=$1
out=gpurun_out/prof_$tag
js=profiles/bench_pmc.json

mkdir -p profiles
python3 tools/pmc_summary.py $out --json $js --bench-log $out/stats.log > profiles/${tag}_summary.txt
cp $out/stats/run_kernel_stats.csv profiles/${tag}_kernel_stats.csv
grep '^{' $out/stats.log > profiles/${tag}_bench_under_rocprof.json || true
[ -f gpurun_out/bench.log ] && grep '^{' gpurun_out/bench.log > profiles/${tag}_bench.json || true
echo "profiles/: $(ls profiles | tr '\n' ' ')"

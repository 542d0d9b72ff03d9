#!/bin/bash
# The headline step's dispatch gaps, measured: rocprofv3 kernel trace + HIP API
# trace of a short bench.py run (no PMC in this pass), then tools/gap_report.py lines up each steady
# step's host enqueue times with its kernels' start / end.  usage: tools/trace_gaps.sh <tag> [bench args]
# -> gpurun_out/trace_<tag>/ (+ gap_<tag>.txt)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tag=$1; shift
out=gpurun_out/trace_$tag
mkdir -p $out
timeout -k 10 240 rocprofv3 --kernel-trace --hip-trace --memory-copy-trace -d $out -o run --output-format csv -- \
  python3 bench.py --steps 12 --warmup 6 --cpu-seconds 0 --no-fanout --no-host-path --no-check --no-extras \
  --no-stage-timing --no-copy-ceiling "$@" > $out/bench.log 2>&1 || { echo "trace $tag failed"; tail -5 $out/bench.log; exit 1; }
python3 tools/gap_report.py $out > gpurun_out/gap_$tag.txt 2>&1 || { echo "gap report failed"; tail -5 gpurun_out/gap_$tag.txt; exit 1; }
tail -25 gpurun_out/gap_$tag.txt

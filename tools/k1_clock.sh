#!/bin/bash
# Config-2 K1 on this box: its event time (tools/k1_perf.py) and, in a separate rocprofv3 pass, its
# effective shader clock and the copy kernel's (tools/clock_pmc.sh), one line each, so that K1's
# box-to-box spread can be set against the clock.  usage: tools/k1_clock.sh <tag>
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tag=$1
timeout -k 10 120 python3 -u tools/k1_perf.py > gpurun_out/k1t_$tag.log 2>&1 || { echo "k1_perf failed"; tail -3 gpurun_out/k1t_$tag.log; exit 1; }
bash tools/clock_pmc.sh k1$tag python3 tools/k1_perf.py > gpurun_out/k1c_$tag.log 2>&1 || { echo "clock pass failed"; tail -3 gpurun_out/k1c_$tag.log; exit 1; }
echo "$tag: $(grep '^k1' gpurun_out/k1t_$tag.log | tail -1)"
grep -E 'k_range|k_copy16' gpurun_out/k1c_$tag.log | sed 's/  */ /g' | cut -c1-160

#!/bin/bash
# K1 (config 2) A/B over builds x chirps per team: tools/k1_perf.py with FMCW_LIB=ab/<name>.so and
# FMCW_K1_CPT, alternating rounds.  tools/k1_ab2.sh "base tapsg" "8 4" [rounds]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
names=$1; cpts=$2; N=${3:-2}
for r in $(seq $N); do for n in $names; do for c in $cpts; do
  FMCW_LIB=ab/$n.so FMCW_K1_CPT=$c timeout -k 10 120 python3 -u tools/k1_perf.py > gpurun_out/k1b_${n}_${c}_$r.log 2>&1 || { echo "$n $c failed"; tail -5 gpurun_out/k1b_${n}_${c}_$r.log; exit 1; }
  echo "$r $n cpt $c: $(grep '^k1' gpurun_out/k1b_${n}_${c}_$r.log)"
done; done; done

#!/bin/bash
# STFT leg A/B of library builds (tools/stft_perf.py under FMCW_LIB=ab/<name>.so, alternating).
#   tools/stft_ab.sh "base variant" [rounds] [forms]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
names=$1; N=${2:-3}; F=${3:-max,direct,stored}
for r in $(seq $N); do for n in $names; do
  FMCW_LIB=ab/$n.so timeout -k 10 120 python3 -u tools/stft_perf.py 50 $F > gpurun_out/sab_${n}_$r.log 2>&1 || { echo "$n failed"; tail -5 gpurun_out/sab_${n}_$r.log; exit 1; }
  echo "$r $n: $(grep 'us per call' gpurun_out/sab_${n}_$r.log | tr -s ' ' | tr '\n' '|')"
done; done

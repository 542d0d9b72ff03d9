#!/bin/bash
# K1 (config 2) order A/B: the interleaved team walk at cpt 16 and 8 against the team-contiguous
# order (FMCW_K1_ILV=0, cpt 8: the round-4 default), alternating rounds in one call
# (tools/k1_perf.py).  Output: gpurun_out/k1ab_*.log.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for r in ${ROUNDS:-1 2}; do
  for v in "ilv16 FMCW_K1_ILV=1 FMCW_K1_CPT=16" "ilv8 FMCW_K1_ILV=1 FMCW_K1_CPT=8" "seq8 FMCW_K1_ILV=0 FMCW_K1_CPT=8"; do
    set -- $v; n=$1; shift
    env "$@" timeout -k 10 120 python3 -u tools/k1_perf.py > gpurun_out/k1ab_${n}_$r.log 2>&1 || { echo "$n failed"; tail -5 gpurun_out/k1ab_${n}_$r.log; exit 1; }
    echo "$r $n: $(grep -v amdgpu gpurun_out/k1ab_${n}_$r.log | tail -1)"
  done
done

#!/bin/bash
# bench.py A/B over library builds, alternating rounds in one call:
#   AB="sysfence cur" ROUNDS="1 2" tools/ab_bench.sh [extra bench args]
# a name is ab/<name>.so (tools/ab_build.sh), "cur" the in-tree libfmcw.so.  One summary line per run:
# value, ms per step, k_rdx us, outside-k_rdx ms, sclk, fp16 k_rdx us, config-2 K1 us.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in ${ROUNDS:-1 2}; do for n in ${AB:-base new}; do
  # a name is a library (ab/<name>.so, cur = in-tree), optionally +VAR=value for one environment setting
  lib=${n%%+*}; envset=; [ "$lib" != "$n" ] && envset=${n#*+}
  [ "$lib" = cur ] && lib=fmcw_radar_processing_amd/libfmcw.so || lib=ab/$lib.so
  env $envset FMCW_LIB=$lib timeout -k 10 300 python3 -u bench.py --cpu-seconds 0 --no-host-path "$@" > gpurun_out/abb_${n}_$r.log 2>&1 || { echo "$n failed"; tail -5 gpurun_out/abb_${n}_$r.log; exit 1; }
  python3 - gpurun_out/abb_${n}_$r.log $n $r <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]).read().splitlines() if l.startswith("{")][-1]); r = d["roofline"]
f16 = (d.get("fp16_storage") or {}).get("roofline") or {}
c2 = (d.get("config2_range_fft") or {}).get("roofline") or {}
print(f"{sys.argv[3]} {sys.argv[2]:10s} value {d['value']:10.1f} step {d['ms_per_step']:.4f} k_rdx {r['avg_launch_us']:8.2f} "
      f"outside {d['ms_per_step'] - r['avg_launch_us'] / 1e3:.4f} sclk {r.get('sclk_mhz')} fp16 {f16.get('avg_launch_us')} "
      f"k1 {c2.get('avg_launch_us')} k1frac {c2.get('frac')} ok {all(v.get('pass', True) for v in (d.get('checked') or {}).values())}")
PY
done; done

set -u
cd $GRAFT_REPO_ROOT
for r in 1 2; do for n in base new; do
  FMCW_LIB=ab/$n.so timeout -k 10 300 python3 -u bench.py --cpu-seconds 0 --no-host-path > gpurun_out/abb_${n}_$r.log 2>&1 || { echo "$n failed"; tail -5 gpurun_out/abb_${n}_$r.log; exit 1; }
  python3 - gpurun_out/abb_${n}_$r.log $n <<'PY'
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d["roofline"]
print(sys.argv[2], d["value"], d["ms_per_step"], r["avg_launch_us"], round(d["ms_per_step"]-r["avg_launch_us"]/1e3,4), d["stages_ms_per_step"].get("detect"))
PY
done; done

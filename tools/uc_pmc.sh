#!/bin/bash
# FETCH_SIZE and WRITE_SIZE (separate rocprofv3 passes) of k_rdx with its input / RD map allocated
# default or uncached (tools/uc_probe.py): tools/uc_pmc.sh "default:default uncached:uncached"
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for pair in $1; do
  fin=${pair%:*}; fout=${pair#*:}; n=uc_${fin}_${fout}
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 120 rocprofv3 --pmc $c --kernel-trace -d gpurun_out/pmc_${n}_$c -o run --output-format csv -- \
      python3 tools/uc_probe.py rdx $fin $fout 3 > gpurun_out/pmc_${n}_$c.log 2>&1 || { echo "pmc $n $c failed"; tail -3 gpurun_out/pmc_${n}_$c.log; exit 1; }
  done
  python3 - gpurun_out/pmc_${n} $n <<'PY'
import csv, glob, sys
base, n = sys.argv[1], sys.argv[2]
val = {}
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    f = glob.glob(f"{base}_{c}/**/*counter_collection.csv", recursive=True)[0]
    rows = [r for r in csv.DictReader(open(f)) if "k_rdx" in r["Kernel_Name"] and r["Counter_Name"] == c]
    v = sorted(float(r["Counter_Value"]) for r in rows)
    val[c] = v[len(v) // 2] * 1024 if v else 0.0       # KiB -> bytes, median launch
print(f"{n}: FETCH x2 {2 * val['FETCH_SIZE'] / 1e9:.2f} GB + WRITE {val['WRITE_SIZE'] / 1e9:.2f} GB = {(2 * val['FETCH_SIZE'] + val['WRITE_SIZE']) / 1e9:.2f} GB")
PY
done

# A/B timing plus FETCH_SIZE per k_rd1p launch for library builds: tools/gpu_pmc_ab.sh "name1 name2"
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/gpu_ab.sh "$1" 4096 10 2 || exit 1
for n in $1; do
  FMCW_LIB=$PWD/ab/$n.so timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmc_$n -o run --output-format csv -- python3 tools/onepass_perf.py 4096 3 onepass > gpurun_out/pmc_$n.log 2>&1 || { echo "pmc $n failed"; exit 1; }
  python3 - $n <<'PY'
import csv, sys, glob
n = sys.argv[1]
f = glob.glob(f"gpurun_out/pmc_{n}/**/run_counter_collection.csv", recursive=True)[0]
v = [float(r["Counter_Value"]) for r in csv.DictReader(open(f)) if "k_rd1p" in r["Kernel_Name"] and r["Counter_Name"] == "FETCH_SIZE"]
print(f"{n}: FETCH_SIZE x2 per k_rd1p launch {2 * sum(v) / len(v) / 1024 / 1024:.2f} GB over {len(v)} launches")
PY
done

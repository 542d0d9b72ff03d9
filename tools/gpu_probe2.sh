# xcd_probe2 timings, then FETCH/WRITE per variant (separate rocprofv3 --pmc passes)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 120 tools/xcd_probe2.bin ${1:-0} > gpurun_out/probe2.log 2>&1; rc=$?; cat gpurun_out/probe2.log; [ $rc -ne 0 ] && exit $rc
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --kernel-trace -d gpurun_out/probe2_$c -o run --output-format csv -- tools/xcd_probe2.bin ${1:-0} > gpurun_out/probe2_$c.log 2>&1 || { echo "pmc $c failed"; tail -3 gpurun_out/probe2_$c.log; exit 1; }
done
python3 - <<'PY'
import csv, glob, collections
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    acc = collections.defaultdict(list)
    for fn in glob.glob(f"gpurun_out/probe2_{c}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(fn)):
            acc[r["Kernel_Name"][:60]].append(float(r["Counter_Value"]))
    for k, v in acc.items():
        print(c, k, "%.3f GB" % (sum(v) / len(v) / 1e6), "(kB units: KB->GB)")
PY

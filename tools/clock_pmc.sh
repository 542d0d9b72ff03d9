#!/bin/bash
# Effective shader clock per kernel: GRBM_GUI_ACTIVE (summed over the 8 XCDs) / 8 / dispatch time
# (MI355X_MICROARCH.md, DVFS give-back).  usage: tools/clock_pmc.sh tag cmd...
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
tag=$1; shift
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES --kernel-trace -d gpurun_out/clk_$tag -o run --output-format csv -- "$@" > gpurun_out/clk_$tag.log 2>&1 || { echo "clock pmc $tag failed"; tail -3 gpurun_out/clk_$tag.log; exit 1; }
python3 - gpurun_out/clk_$tag <<'PY'
import csv, glob, sys, collections
d = sys.argv[1]
cc = glob.glob(d + '/**/*counter_collection.csv', recursive=True)[0]
rows = list(csv.DictReader(open(cc)))
acc = collections.defaultdict(lambda: [0.0, 0.0, 0])
for r in rows:
    if r['Counter_Name'] != 'GRBM_GUI_ACTIVE':
        continue
    dur = (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) * 1e-9 if 'End_Timestamp' in r else None
    if not dur or dur < 2e-4:
        continue
    a = acc[r['Kernel_Name'][:50]]
    a[0] += float(r['Counter_Value']); a[1] += dur; a[2] += 1
for k, (g, t, n) in acc.items():
    print(f"{d.split('/')[-1]:14s} {k:50s} n={n} avg {t / n * 1e3:.3f} ms  clock {g / 8 / t / 1e9:.3f} GHz")
PY

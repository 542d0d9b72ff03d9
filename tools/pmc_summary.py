"""Summarise rocprofv3 CSV output per kernel (development + profiles/ summaries).

usage: python tools/pmc_summary.py <prof_dir>   (the -d directory of tools/profile_run.sh)
FETCH_SIZE / WRITE_SIZE are in KiB per dispatch.  On gfx950 FETCH_SIZE counts
half the bytes of wide coalesced streaming reads (MI355X_MICROARCH.md, HBM):
the 'fetch_x2' column applies that documented x2 correction.
"""
import csv
import collections
import os
import sys


def short(name):
    name = name.replace("HIP_vector_type<float, 2u>", "c64").replace("__half2", "c32h")
    return name.split("(")[0].replace("void ", "")[:70]


def load_counters(path):
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    dur = collections.defaultdict(list)
    with open(path) as fh:
        for r in csv.DictReader(fh):
            k = short(r["Kernel_Name"])
            per[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
            dur[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    return per, dur


def main(d):
    rows = collections.OrderedDict()
    stats = os.path.join(d, "stats", "run_kernel_stats.csv")
    if os.path.exists(stats):
        print("== kernel stats (rocprofv3 --kernel-trace --stats) ==")
        print(f"{'kernel':72s} {'calls':>6s} {'avg_us':>9s} {'total_ms':>9s} {'pct':>6s}")
        with open(stats) as fh:
            for r in csv.DictReader(fh):
                print(f"{short(r['Name']):72s} {int(r['Calls']):6d} {float(r['AverageNs'])/1e3:9.2f} "
                      f"{float(r['TotalDurationNs'])/1e6:9.2f} {float(r['Percentage']):6.2f}")
    for sub in ("fetch", "write", "sq", "tcc"):
        p = os.path.join(d, sub, "run_counter_collection.csv")
        if not os.path.exists(p):
            continue
        per, dur = load_counters(p)
        for k, cs in per.items():
            row = rows.setdefault(k, {})
            for c, vals in cs.items():
                row[c] = sum(vals) / len(vals)
    if rows:
        print("\n== PMC per dispatch (averages; FETCH/WRITE in MB, fetch_x2 = gfx950 x2 read correction) ==")
        for k, r in rows.items():
            if "FETCH_SIZE" not in r and "SQ_WAVES" not in r and "SQ_WAVE_CYCLES" not in r:
                continue
            parts = []
            if "FETCH_SIZE" in r:
                parts.append(f"fetch {r['FETCH_SIZE']/1024:.2f} MB (x2 {2*r['FETCH_SIZE']/1024:.2f})")
            if "WRITE_SIZE" in r:
                parts.append(f"write {r['WRITE_SIZE']/1024:.2f} MB")
            if "TCC_HIT_sum" in r and (r["TCC_HIT_sum"] + r.get("TCC_MISS_sum", 0)) > 0:
                parts.append(f"L2 hit {r['TCC_HIT_sum']/(r['TCC_HIT_sum']+r['TCC_MISS_sum']):.2f}")
            if "SQ_WAVE_CYCLES" in r and r["SQ_WAVE_CYCLES"] > 0:
                wc = r["SQ_WAVE_CYCLES"]
                parts.append(f"wait {r.get('SQ_WAIT_ANY',0)/wc:.2f} issue-stall {r.get('SQ_WAIT_INST_ANY',0)/wc:.2f} "
                             f"active {r.get('SQ_ACTIVE_INST_ANY',0)/wc:.2f} valu {r.get('SQ_ACTIVE_INST_VALU',0)/wc:.2f}")
            if "SQ_LDS_BANK_CONFLICT" in r:
                parts.append(f"lds_conf {r['SQ_LDS_BANK_CONFLICT']:.0f}")
            if "GRBM_GUI_ACTIVE" in r:
                parts.append(f"gui_active {r['GRBM_GUI_ACTIVE']:.0f}")
            print(f"{k:72s} " + " | ".join(parts))


if __name__ == "__main__":
    main(sys.argv[1])

"""Summarise rocprofv3 CSV output per kernel (development + profiles/ summaries).

usage: python tools/pmc_summary.py <prof_dir> [--json OUT --bench-log LOG]
  (<prof_dir>: the -d directory of tools/profile_run.sh; --json writes the
  per-kernel HBM traffic that bench.py reports as roofline.traffic)
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
    """Per kernel name, the dispatches of its LARGEST grid only (a kernel launched at
    several sizes, e.g. k_rdx for the 4096-frame step and for a small host-path
    chunk, would otherwise average unlike launches)."""
    rows = list(csv.DictReader(open(path)))
    big = collections.defaultdict(int)
    for r in rows:
        k = short(r["Kernel_Name"])
        big[k] = max(big[k], int(r["Grid_Size"]))
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    dur = collections.defaultdict(list)
    for r in rows:
        k = short(r["Kernel_Name"])
        if int(r["Grid_Size"]) != big[k]:
            continue
        per[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
        dur[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    return per, dur


def trace_avg_us(path):
    """(avg us, calls) per kernel name over the dispatches of its largest grid (kernel trace)."""
    rows = list(csv.DictReader(open(path)))
    big = collections.defaultdict(int)
    for r in rows:
        g = int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"])
        big[short(r["Kernel_Name"])] = max(big[short(r["Kernel_Name"])], g)
    acc = collections.defaultdict(list)
    for r in rows:
        k = short(r["Kernel_Name"])
        if int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"]) == big[k]:
            acc[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    return {k: (sum(v) / len(v), len(v)) for k, v in acc.items()}


LABELS = ("k_range", "k_doppler", "k_detect_1p", "k_detect", "k_rdx", "k_slow_fix", "k_rd_fused", "k_compact", "k_stft_power", "k_stft_db")


def label(k):
    for lb in LABELS:
        if k.startswith("fmcw::" + lb + "<") or k == "fmcw::" + lb:
            return lb
    return None


def main(d, json_out=None, bench_log=None):
    rows = collections.OrderedDict()
    stat_us = {}
    stats = os.path.join(d, "stats", "run_kernel_stats.csv")
    if os.path.exists(stats):
        print("== kernel stats (rocprofv3 --kernel-trace --stats) ==")
        print(f"{'kernel':72s} {'calls':>6s} {'avg_us':>9s} {'total_ms':>9s} {'pct':>6s}")
        with open(stats) as fh:
            for r in csv.DictReader(fh):
                stat_us[short(r['Name'])] = (float(r['AverageNs']) / 1e3, int(r['Calls']))
                print(f"{short(r['Name']):72s} {int(r['Calls']):6d} {float(r['AverageNs'])/1e3:9.2f} "
                      f"{float(r['TotalDurationNs'])/1e6:9.2f} {float(r['Percentage']):6.2f}")
    trace = os.path.join(d, "stats", "run_kernel_trace.csv")
    if os.path.exists(trace):
        stat_us.update(trace_avg_us(trace))        # per kernel: its largest launch only
    for sub in ("fetch", "write", "sq", "tcc", "sq2"):
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
            if "SQ_INSTS_VMEM_RD" in r:
                parts.append("insts " + " ".join(f"{c[9:].lower()}={r[c]:.0f}" for c in
                             ("SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR", "SQ_INSTS_LDS", "SQ_INSTS_SALU", "SQ_INSTS_FLAT")
                             if c in r) + f" valu={r.get('SQ_INSTS_VALU', 0):.0f}")
                wc = r.get("SQ_WAVE_CYCLES", 0)
                if wc:
                    parts.append(f"wait_lds {r.get('SQ_WAIT_INST_LDS', 0)/wc:.2f} active_lds {r.get('SQ_ACTIVE_INST_LDS', 0)/wc:.2f} "
                                 f"vmem_rd_cyc {r.get('SQ_INST_CYCLES_VMEM_RD', 0)/wc:.2f}")
            if "GRBM_GUI_ACTIVE" in r:
                parts.append(f"gui_active {r['GRBM_GUI_ACTIVE']:.0f}")
            print(f"{k:72s} " + " | ".join(parts))
    if json_out:
        import json
        bench = {}
        if bench_log and os.path.exists(bench_log):
            for line in open(bench_log):
                if line.startswith("{") and '"metric"' in line:
                    bench = json.loads(line)
        # every roofline object of the bench line names its kernel and launch size
        roofs = {}
        def walk(o):
            if isinstance(o, dict):
                if o.get("kernel_name") and "frames_per_launch" in o:
                    roofs[o["kernel_name"]] = o
                for v in o.values():
                    walk(v)
        walk(bench)
        out = {"prof_dir": d, "bench_line": {k: bench.get(k) for k in ("value", "ms_per_step", "dtype", "config")},
               "note": "hbm_bytes_per_launch = (2 x FETCH_SIZE + WRITE_SIZE) per dispatch; FETCH_SIZE x2 is the "
                       "gfx950 correction of MI355X_MICROARCH.md (HBM section); separate --pmc passes",
               "kernels": {}, "by_name": {}}
        for k, r in rows.items():
            if "FETCH_SIZE" in r and "WRITE_SIZE" in r:
                e = {"fetch_kib": round(r["FETCH_SIZE"], 1), "write_kib": round(r["WRITE_SIZE"], 1),
                     "hbm_bytes_per_launch": int((2 * r["FETCH_SIZE"] + r["WRITE_SIZE"]) * 1024)}
                if k in stat_us:
                    e["rocprof_avg_us"], e["rocprof_calls"] = round(stat_us[k][0], 2), stat_us[k][1]
                    e["rocprof_avg_note"] = "kernel trace, dispatches of the kernel's largest grid"
                if k in roofs:
                    e["frames_per_launch"] = roofs[k]["frames_per_launch"]
                    e["bench_event_avg_us"] = roofs[k]["avg_launch_us"]
                    e["alg_bytes_per_launch"] = roofs[k]["alg_bytes_per_launch"]
                out["by_name"][k] = e
            lb = label(k)
            if not lb or "FETCH_SIZE" not in r or "WRITE_SIZE" not in r:
                continue
            e = {"name": k, "fetch_kib": round(r["FETCH_SIZE"], 1), "write_kib": round(r["WRITE_SIZE"], 1),
                 "hbm_bytes_per_launch": int((2 * r["FETCH_SIZE"] + r["WRITE_SIZE"]) * 1024)}
            if k in stat_us:
                e["rocprof_avg_us"], e["rocprof_calls"] = round(stat_us[k][0], 2), stat_us[k][1]
            # keyed by the full instantiation name: k_rdx<.., H = true, ..> (fp16 storage) and the fp32
            # k_rdx share the label, and one must not overwrite the other; the bench's event time is
            # attached only to the instantiation its roofline names
            e["label"] = lb
            if k in roofs:
                e["frames_per_launch"] = roofs[k]["frames_per_launch"]
                e["bench_event_avg_us"] = roofs[k]["avg_launch_us"]
            out["kernels"][k] = e
        with open(json_out, "w") as fh:
            json.dump(out, fh, indent=1)
        print(f"wrote {json_out}")


if __name__ == "__main__":
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--json")
    ap.add_argument("--bench-log")
    a = ap.parse_args()
    main(a.dir, a.json, a.bench_log)

"""Line up the headline step's kernels with the host calls that enqueued them.

python tools/gap_report.py <rocprofv3 -d dir>   (a --kernel-trace --hip-trace run of bench.py,
tools/trace_gaps.sh).  For the last steady steps (k_rdx to k_rdx) it prints every kernel with its
duration and the idle gap before it, and for every gap the HIP calls the host made around it: when
the host enqueued the next kernel long before the gap ended, the gap is not the host's enqueue.
"""
import collections
import csv
import glob
import os
import sys


def load(d, pat):
    fs = glob.glob(os.path.join(d, "**", pat), recursive=True)
    rows = []
    for f in fs:
        rows += list(csv.DictReader(open(f)))
    return rows


def short(n):
    n = n.split("(")[0]
    for k in ("k_rdx<", "k_stft64f<", "k_detect_1p", "k_copy16", "__amd_rocclr_fillBuffer", "k_synth"):
        if k in n:
            i = n.find(k)
            return n[i:i + 40]
    return n[-40:]


def main(d):
    ks = load(d, "*kernel_trace.csv")
    api = load(d, "*hip_api_trace.csv")
    if not ks:
        print("no kernel trace under", d)
        return 1
    ks.sort(key=lambda r: int(r["Start_Timestamp"]))
    by_corr = {r["Correlation_Id"]: r for r in api}
    rdx = [i for i, r in enumerate(ks) if "k_rdx" in r["Kernel_Name"]]
    print(f"kernels {len(ks)}, k_rdx launches {len(rdx)}, hip api records {len(api)}")
    if len(rdx) < 3:
        return 1
    api_sorted = sorted(api, key=lambda r: int(r["Start_Timestamp"]))
    gaps = collections.defaultdict(list)
    for s_i in range(max(0, len(rdx) - 5), len(rdx) - 1):
        a, b = rdx[s_i], rdx[s_i + 1]
        print(f"\n-- step {s_i}: kernels {a}..{b}")
        t_prev_end = None
        for i in range(a, b + 1):
            r = ks[i]
            t0, t1 = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
            gap = (t0 - t_prev_end) / 1e3 if t_prev_end is not None else 0.0
            c = by_corr.get(r["Correlation_Id"])
            enq = f"enqueued {(t0 - int(c['End_Timestamp'])) / 1e3:9.1f} us before start by {c['Function']}" if c else "no api record"
            nm = short(r["Kernel_Name"])
            print(f"  gap {gap:7.1f} | {nm:40s} {(t1 - t0) / 1e3:9.1f} us | {enq}")
            if t_prev_end is not None and i <= b:
                gaps[(short(ks[i - 1]["Kernel_Name"]), nm)].append(gap)
                # host calls whose span overlaps the gap
                calls = [x for x in api_sorted if int(x["End_Timestamp"]) >= t_prev_end - 2000 and int(x["Start_Timestamp"]) <= t0]
                if gap > 3 and calls:
                    print("      host calls during the gap:", ", ".join(
                        f"{x['Function']}@{(int(x['Start_Timestamp']) - t_prev_end) / 1e3:+.1f}" for x in calls[:12]))
            t_prev_end = t1
    print("\nmean gap before each kernel (steady steps):")
    for k, v in gaps.items():
        print(f"  {k[0]:40s} -> {k[1]:40s} {sum(v) / len(v):7.2f} us (n={len(v)})")
    # host-side: time between consecutive k_rdx enqueues vs GPU step
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1]))

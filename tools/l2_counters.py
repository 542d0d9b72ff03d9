"""Summarise the PMC passes of tools/pmc_xcd.sh (one per schedule) into the L2 evidence table
committed as profiles/r02_l2_counters.txt: per launch of the largest dispatch of each single-pass
kernel, TCP->TCC read/write requests and bytes (128-B reads / 64-B writes), TCC hits and misses,
HBM-side FETCH (x2, gfx950 correction) and WRITE, and the SQ busy/VALU figures.

python tools/l2_counters.py gpurun_out/pmc_x gpurun_out/pmc_o > profiles/r02_l2_counters.txt
"""
import collections
import csv
import sys

ALG = 4096 * 4198400          # algorithmic bytes per 4096-frame launch (input + RD + profile)


def load(prefix):
    out = collections.defaultdict(float)
    name = None
    for i in range(1, 6):
        rows = list(csv.DictReader(open(f"{prefix}_{i}/run_counter_collection.csv")))
        per = collections.defaultdict(lambda: collections.defaultdict(float))
        for r in rows:
            k = r["Kernel_Name"]
            if "k_rdx" in k:
                per[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
                name = k
        big = max(per.values(), key=lambda v: sum(v.values()))
        for c, v in big.items():
            out[c] = v
    return name, out


def main(*prefixes):
    print("L2 evidence per 4096-frame launch (rocprofv3 --pmc, one counter group per pass; tools/pmc_xcd.sh)")
    print(f"algorithmic bytes per launch: {ALG / 1e9:.2f} GB (input 8.59 + RD map 8.59 + profile 0.02)\n")
    for p in prefixes:
        name, c = load(p)
        rd = c["TCP_TCC_READ_REQ_sum"] * 128 / 1e9
        wr = c["TCP_TCC_WRITE_REQ_sum"] * 64 / 1e9
        hit, miss = c["TCC_HIT_sum"], c["TCC_MISS_sum"]
        print(f"{name}")
        print(f"  L1->L2 (TCP->TCC) reads  {c['TCP_TCC_READ_REQ_sum'] / 1e6:8.1f} M requests = {rd:6.1f} GB "
              f"({rd / (ALG / 2 / 1e9):.1f} x the input)")
        print(f"  L1->L2 (TCP->TCC) writes {c['TCP_TCC_WRITE_REQ_sum'] / 1e6:8.1f} M requests = {wr:6.1f} GB")
        print(f"  TCC hits {hit / 1e6:.1f} M, misses {miss / 1e6:.1f} M (hit rate {hit / (hit + miss):.2f})")
        print(f"  HBM side: FETCH x2 {c['FETCH_SIZE'] * 2 / 1e6:.2f} GB, WRITE {c['WRITE_SIZE'] / 1e6:.2f} GB")
        print(f"  SQ: busy cycles {c['SQ_BUSY_CYCLES'] / 1e6:.1f} M, VALU instructions {c['SQ_INSTS_VALU'] / 1e6:.1f} M, "
              f"active VALU / wave cycles {c['SQ_ACTIVE_INST_VALU'] / c['SQ_WAVE_CYCLES']:.3f}, "
              f"wait / wave cycles {c['SQ_WAIT_ANY'] / c['SQ_WAVE_CYCLES']:.3f}, LDS bank conflicts {c['SQ_LDS_BANK_CONFLICT']:.0f}")
        print()


if __name__ == "__main__":
    main(*sys.argv[1:])

#!/usr/bin/env python3
"""Per-phase counters of the common-mode kernel from one ``cm_probe.py --pmc-pass`` rocprofv3 run.

After one correctness launch, the probe launches calib_cm 3 times per flags value, in the order 0 (memory phases only),
1 (+ row medians), 2 (+ column medians), 3 (both), on 32 epix10k2M frames; this prints, per flags
value, the mean per-frame value of every counter (summed over the dispatch's instances), and the
row / column phase deltas (flags 1 - 0, 2 - 0).

    python tools/pmc_cm.py gpurun_out/ab/pmc_base [--frames 32]
"""
import argparse
import collections
import csv
import glob
import os


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--frames", type=int, default=32)
    a = ap.parse_args()
    agg = collections.defaultdict(float)
    for f in glob.glob(os.path.join(a.dir, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if "calib_cm" not in r.get("Kernel_Name", ""):
                continue
            agg[(int(r["Dispatch_Id"]), r["Counter_Name"])] += float(r["Counter_Value"])
    disp = sorted({k[0] for k in agg})
    names = sorted({k[1] for k in agg})
    if len(disp) < 12:
        raise SystemExit(f"expected 12 calib_cm dispatches, found {len(disp)}")
    disp = disp[-12:]   # the probe's correctness launch (flags 3) comes first
    per = {}
    for flags in range(4):
        ds = disp[3 * flags:3 * flags + 3]
        per[flags] = {n: sum(agg[(d, n)] for d in ds) / len(ds) / a.frames for n in names}
    print("counter (per frame) | flags0 | flags1 | flags2 | flags3 | rows (1-0) | cols (2-0)")
    for n in names:
        v = [per[f][n] for f in range(4)]
        print(f"{n} | " + " | ".join(f"{x:,.0f}" for x in v) + f" | {v[1] - v[0]:,.0f} | {v[2] - v[0]:,.0f}")


if __name__ == "__main__":
    main()

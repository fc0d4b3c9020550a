"""Summarise rocprofv3 --pmc CSV output (one directory per pass) into a per-kernel markdown table:
mean counter value per dispatch, plus derived HBM bytes / LDS conflict rate where the inputs exist.

    python tools/pmc_summary.py gpurun_out/pmc_a gpurun_out/pmc_b ... > profiles/pmc_kernels_r1.md
"""
import csv
import glob
import os
import re
import sys
from collections import defaultdict


def short(name: str) -> str:
    n = re.sub(r"\(.*$", "", name)
    n = n.replace("void ", "").replace("pr::", "")
    return n[:60]


def main(dirs):
    vals = defaultdict(lambda: defaultdict(list))   # kernel -> counter -> values
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            with open(f) as fh:
                for row in csv.DictReader(fh):
                    k = short(row.get("Kernel_Name", "?"))
                    c = row.get("Counter_Name", "?")
                    try:
                        vals[k][c].append(float(row.get("Counter_Value", "nan")))
                    except ValueError:
                        pass
    counters = sorted({c for k in vals for c in vals[k]})
    keep = [k for k in vals if not k.startswith("at::") and "elementwise" not in k and "reduce_kernel" not in k]
    print("| kernel | " + " | ".join(counters) + " |")
    print("|---|" + "---|" * len(counters))
    for k in sorted(keep):
        cells = []
        for c in counters:
            v = vals[k].get(c)
            cells.append(f"{sum(v) / len(v):,.0f}" if v else "")
        print(f"| `{k}` | " + " | ".join(cells) + " |")
    print()
    print("Derived (per dispatch, 32 epix10k2M frames; FETCH_SIZE doubled for gfx950's half-count of wide "
          "streaming reads, MI355X_MICROARCH.md:298):")
    print()
    print("| kernel | HBM read MB (2xFETCH) | HBM write MB | LDS conflict cycles / LDS instr |")
    print("|---|---|---|---|")
    for k in sorted(keep):
        v = vals[k]
        rd = 2 * sum(v["FETCH_SIZE"]) / len(v["FETCH_SIZE"]) / 1024 if v.get("FETCH_SIZE") else None
        wr = sum(v["WRITE_SIZE"]) / len(v["WRITE_SIZE"]) / 1024 if v.get("WRITE_SIZE") else None
        lc = None
        if v.get("SQ_LDS_BANK_CONFLICT") and v.get("SQ_INSTS_LDS"):
            ins = sum(v["SQ_INSTS_LDS"])
            lc = sum(v["SQ_LDS_BANK_CONFLICT"]) / ins if ins else 0.0
        f = lambda x, p=1: "" if x is None else f"{x:,.{p}f}"  # noqa: E731
        print(f"| `{k}` | {f(rd)} | {f(wr)} | {f(lc, 3)} |")


if __name__ == "__main__":
    main(sys.argv[1:])

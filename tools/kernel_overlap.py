#!/usr/bin/env python3
"""Concurrency of two kernel families in a rocprofv3 kernel trace (CSV): how much of the consumer's
peak-finder time overlaps the producer's common-mode kernels (co-residency on the same GPU).

    python tools/kernel_overlap.py <dir with *kernel_trace.csv> [name_a] [name_b]
"""
import csv
import glob
import json
import sys


def intervals(rows, key):
    return sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows if key in r["Kernel_Name"])


def union(iv):
    out = []
    for s, e in iv:
        if out and s <= out[-1][1]:
            out[-1][1] = max(out[-1][1], e)
        else:
            out.append([s, e])
    return out


def overlap(a, b):
    i = j = tot = 0
    while i < len(a) and j < len(b):
        s, e = max(a[i][0], b[j][0]), min(a[i][1], b[j][1])
        tot += max(0, e - s)
        if a[i][1] < b[j][1]:
            i += 1
        else:
            j += 1
    return tot


def main():
    d = sys.argv[1]
    na = sys.argv[2] if len(sys.argv) > 2 else "calib_cm"
    nb = sys.argv[3] if len(sys.argv) > 3 else "peakfind"
    files = glob.glob(d + "/**/*kernel_trace.csv", recursive=True)
    rows = [r for f in files for r in csv.DictReader(open(f))]
    a, b = union(intervals(rows, na)), union(intervals(rows, nb))
    ta, tb = sum(e - s for s, e in a), sum(e - s for s, e in b)
    ov = overlap(a, b)
    span = (max(a[-1][1], b[-1][1]) - min(a[0][0], b[0][0])) if a and b else 0
    print(json.dumps({"a": na, "b": nb, "a_busy_ms": ta / 1e6, "b_busy_ms": tb / 1e6, "overlap_ms": ov / 1e6,
                      "b_overlapped_fraction": round(ov / max(tb, 1), 3), "span_ms": span / 1e6,
                      "n_a": len(intervals(rows, na)), "n_b": len(intervals(rows, nb))}))


if __name__ == "__main__":
    main()

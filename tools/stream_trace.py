#!/usr/bin/env python3
"""Per-queue / per-stream view of a rocprofv3 kernel trace (CSV) of the device-resident pipeline:
which hardware queue and HIP stream every kernel family ran on, its median duration, and how the
producer's common-mode launches sit against each other (concurrent / back-to-back / gaps).

    python tools/stream_trace.py <dir with *kernel_trace.csv>
"""
import collections
import csv
import glob
import json
import statistics
import sys


def family(name):
    for k in ("calib_cm", "peakfind", "copy", "image", "calib"):
        if k in name:
            return k
    return name.split("(")[0][-40:]


def main():
    files = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)
    rows = [r for f in files for r in csv.DictReader(open(f))]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    by = collections.defaultdict(list)
    for r in rows:
        by[(family(r["Kernel_Name"]), r.get("Queue_Id", "?"), r.get("Stream_Id", "?"))].append(r)
    out = {"placement": []}
    for (fam, q, s), rs in sorted(by.items()):
        d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rs]
        out["placement"].append({"kernel": fam, "queue": q, "stream": s, "n": len(rs),
                                 "median_us": round(statistics.median(d), 1)})
    cm = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows if "calib_cm" in r["Kernel_Name"]]
    if len(cm) > 2:
        # start of launch i+1 relative to the end of launch i: < 0 concurrent, >= 0 gap
        rel = [(cm[i + 1][0] - cm[i][1]) / 1e3 for i in range(len(cm) - 1)]
        conc = [x for x in rel if x < 0]
        out["cm_next_start_minus_end_us"] = {"median": round(statistics.median(rel), 1),
                                             "concurrent_fraction": round(len(conc) / len(rel), 3),
                                             "gaps_over_5us": sum(1 for x in rel if x > 5)}
        span = (cm[-1][1] - cm[0][0]) / 1e3
        busy = sum(e - s for s, e in cm) / 1e3
        out["cm_span_us"] = round(span, 1)
        out["cm_sum_of_durations_us"] = round(busy, 1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()

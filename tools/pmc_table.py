#!/usr/bin/env python3
"""Per-kernel counter table of tools/pmc_workload.py runs.

    python tools/pmc_table.py PHASES.json TRACE_DIR PASS_DIR [PASS_DIR ...] > table.md
    python tools/pmc_table.py --cm-phases PASS_DIR [FRAMES]      (per-phase common-mode counters)

TRACE_DIR: a ``--kernel-trace`` run (durations); PASS_DIRs: ``--pmc`` runs.  Dispatches are
labelled by the phase list pmc_workload.py wrote (the LAST dispatches of each kernel family, in phase
order).  Bytes: FETCH_SIZE x 2 (gfx950 tallies a wide coalesced stream's 128-B requests at 64 B,
/opt/skills/guides/MI355X_MICROARCH.md:297-299), WRITE_SIZE as reported; both in KB per dispatch.
Mean waves per SIMD = 4 x SQ_WAVE_CYCLES (quad-cycles) / (cycles x 1024 SIMDs), cycles =
GRBM_GUI_ACTIVE / 8 XCDs."""
import argparse
import collections
import csv
import glob
import json
import os
import sys

FAMILY = {"cm": "calib_cm_net_kernel", "cm_image": "calib_cm_net_kernel", "peakfind": "peakfind_range_kernel",
          "h2d": "copy_h2d_kernel", "xcopy": "copy_runs_kernel"}


def rows(d, pat):
    out = []
    for f in glob.glob(f"{d}/**/*{pat}", recursive=True):
        out += list(csv.DictReader(open(f)))
    return out


def label(dispatches, phases):
    """dispatch id -> phase name: walk the phases backwards over each family's dispatches."""
    by_fam = collections.defaultdict(list)
    for did, name in sorted(dispatches.items()):
        for fam in set(FAMILY.values()):
            if fam in name:
                by_fam[fam].append(did)
    lab = {}
    taken = collections.Counter()
    for ph in reversed(phases):
        fam = FAMILY[ph["name"]]
        ids = by_fam[fam]
        n = ph["dispatches"]
        end = len(ids) - taken[fam]
        for did in ids[max(0, end - n):end]:
            lab[did] = ph["name"]
        taken[fam] += n
    return lab


def main():
    phases = json.load(open(sys.argv[1]))
    trace = rows(sys.argv[2], "kernel_trace.csv")
    names = {int(r["Dispatch_Id"]): r["Kernel_Name"] for r in trace}
    lab = label(names, phases)
    dur = collections.defaultdict(list)
    for r in trace:
        d = int(r["Dispatch_Id"])
        if d in lab:
            dur[lab[d]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3)
    ctr = collections.defaultdict(lambda: collections.defaultdict(list))
    for pdir in sys.argv[3:]:
        cr = rows(pdir, "counter_collection.csv")
        cnames = {int(r["Dispatch_Id"]): r["Kernel_Name"] for r in cr}
        clab = label(cnames, phases)
        per = collections.defaultdict(float)
        for r in cr:
            d = int(r["Dispatch_Id"])
            if d in clab:
                per[(d, r["Counter_Name"])] += float(r["Counter_Value"])
        for (d, c), v in per.items():
            ctr[clab[d]][c].append(v)
    mean = lambda v: sum(v) / len(v) if v else float("nan")
    print("| kernel (phase) | frames / dispatch | us / frame | read MB / frame (FETCH x2) | write MB / frame | "
          "TB/s (read + write) | of 6.29 TB/s | waves / SIMD | VALU insts / frame | LDS bank conflicts |")
    print("|---|---|---|---|---|---|---|---|---|---|")
    out = {}
    for ph in phases:
        n = ph["name"]
        F = ph["frames"]
        us = mean(dur[n])
        c = ctr[n]
        fetch = 2 * mean(c.get("FETCH_SIZE", [])) * 1024 / F / 1e6
        write = mean(c.get("WRITE_SIZE", [])) * 1024 / F / 1e6
        tbs = (fetch + write) * 1e6 * F / (us * 1e-6) / 1e12 if us == us else float("nan")
        g = mean(c.get("GRBM_GUI_ACTIVE", []))
        wc = mean(c.get("SQ_WAVE_CYCLES", []))
        occ = 4 * wc / (g / 8 * 1024) if g == g and g > 0 else float("nan")
        valu = mean(c.get("SQ_INSTS_VALU", [])) / F
        ldsc = mean(c.get("SQ_LDS_BANK_CONFLICT", [])) / F
        out[n] = {"us_per_frame": us / F, "read_MB_per_frame": fetch, "write_MB_per_frame": write, "TBps": tbs,
                  "waves_per_simd": occ, "valu_per_frame": valu, "lds_conflicts_per_frame": ldsc,
                  "dispatch_us": us, "n_dispatches_timed": len(dur[n]), "nominal": ph["bytes_per_frame_nominal"]}
        print(f"| {FAMILY[n]} ({n}) | {F} | {us / F:.3f} | {fetch:.2f} | {write:.2f} | {tbs:.2f} | "
              f"{tbs / 6.29:.0%} | {occ:.2f} | {valu:,.0f} | {ldsc:,.0f} |")
    print()
    print("```json")
    print(json.dumps(out, indent=1))
    print("```")


def cm_phases(argv):
    """One ``cm_probe.py --pmc-pass`` run: after its correctness launch the probe launches calib_cm 3
    times per flags value, in the order 0 (memory phases only), 1 (+ row medians), 2 (+ column
    medians), 3 (both), on 32 epix10k2M frames; prints per flags value the mean per-frame value of
    every counter (summed over the dispatch's instances) and the row / column phase deltas."""
    a = argparse.Namespace(dir=argv[0], frames=int(argv[1]) if len(argv) > 1 else 32)
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
    if len(sys.argv) > 1 and sys.argv[1] == "--cm-phases":
        cm_phases(sys.argv[2:])
        sys.exit(0)
    main()

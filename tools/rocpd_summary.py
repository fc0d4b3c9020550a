#!/usr/bin/env python3
"""Summarise a rocprofv3 rocpd SQLite database (kernel stats + memory copies) as markdown/JSON."""
import glob
import json
import sqlite3
import sys


def summarize(path):
    dbs = glob.glob(path + "/**/*.db", recursive=True) if not path.endswith(".db") else [path]
    out = {}
    for db in dbs:
        con = sqlite3.connect(db)
        cols = [r[1] for r in con.execute("pragma table_info(kernels)")]
        rows = con.execute("select * from kernels").fetchall()
        ks = {}
        ni, si, ei = cols.index("name"), cols.index("start"), cols.index("end")
        for r in rows:
            name = r[ni].split("(")[0]
            d = ks.setdefault(name, [0, 0.0, 1e30, 0.0])
            dur = (r[ei] - r[si]) / 1e3
            d[0] += 1
            d[1] += dur
            d[2] = min(d[2], dur)
            d[3] = max(d[3], dur)
        tot = sum(v[1] for v in ks.values())
        kern = sorted(([k, v[0], v[1], v[1] / v[0], v[2], v[3], 100 * v[1] / max(tot, 1e-9)] for k, v in ks.items()),
                      key=lambda x: -x[2])
        mc = []
        try:
            mcols = [r[1] for r in con.execute("pragma table_info(memory_copies)")]
            mrows = con.execute("select * from memory_copies").fetchall()
            agg = {}
            for r in mrows:
                d = dict(zip(mcols, r))
                key = d.get("name") or d.get("kind") or "copy"
                a = agg.setdefault(key, [0, 0.0, 0])
                a[0] += 1
                a[1] += (d["end"] - d["start"]) / 1e3
                a[2] += d.get("size", 0) or 0
            mc = [[k, v[0], v[1], v[2] / max(v[1], 1e-9) / 1e3] for k, v in agg.items()]
        except Exception:
            pass
        marks = []
        try:   # roctx ranges (--marker-trace): message in regions.extdata
            agg = {}
            for ext, st, en in con.execute("select extdata, start, end from regions"):
                try:
                    msg = json.loads(ext).get("message", "?")
                except Exception:
                    msg = "?"
                agg.setdefault(msg, []).append((en - st) / 1e3)
            for k, v in agg.items():
                v.sort()
                marks.append([k, len(v), sum(v), sum(v) / len(v), v[len(v) // 2], v[-1]])
            marks.sort(key=lambda x: -x[2])
        except Exception:
            pass
        out[db] = {"kernels": kern, "copies": mc, "ranges": marks}
    return out


def to_markdown(s):
    lines = []
    for db, d in s.items():
        lines.append("| kernel | calls | total us | avg us | min us | max us | % |")
        lines.append("|---|---|---|---|---|---|---|")
        for k in d["kernels"]:
            lines.append(f"| `{k[0][:90]}` | {k[1]} | {k[2]:.1f} | {k[3]:.2f} | {k[4]:.2f} | {k[5]:.2f} | {k[6]:.1f} |")
        if d["copies"]:
            lines.append("")
            lines.append("| copy | calls | total us | GB/s |")
            lines.append("|---|---|---|---|")
            for c in d["copies"]:
                lines.append(f"| {c[0]} | {c[1]} | {c[2]:.1f} | {c[3]:.1f} |")
        if d.get("ranges"):
            lines.append("")
            lines.append("| roctx range | n | total us | mean us | p50 us | max us |")
            lines.append("|---|---|---|---|---|---|")
            for m in d["ranges"]:
                lines.append(f"| `{m[0]}` | {m[1]} | {m[2]:.1f} | {m[3]:.1f} | {m[4]:.1f} | {m[5]:.1f} |")
    return "\n".join(lines)


if __name__ == "__main__":
    s = summarize(sys.argv[1])
    print(to_markdown(s))
    if len(sys.argv) > 2:
        with open(sys.argv[2], "w") as f:
            json.dump(s, f, indent=1)

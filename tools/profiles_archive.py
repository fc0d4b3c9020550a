#!/usr/bin/env python3
"""Pack / unpack the raw A/B results under profiles/ (<= 300 tracked files).

Files a document cites by path (README.md, docs/, profiles/**/README.md, sources)
and every Markdown file stay as they are.  Every other file of a directory is packed into that
directory's ``ARCHIVE.jsonl`` (one line per file: {"file": name, "text": contents}), so a cited
directory still exists and still holds its numbers.

    python tools/profiles_archive.py pack [DIR...]   # rewrite the tree, or only DIRs (git rm / add by hand)
    python tools/profiles_archive.py unpack DIR      # restore DIR's files next to its archive
    python tools/profiles_archive.py cat DIR/FILE    # print one packed file
"""
import json
import os
import re
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
TEXT = (".md", ".py", ".sh", ".hip", ".cpp", ".h", ".toml", ".txt", ".ini")


def cited(tracked):
    prof = {f for f in tracked if f.startswith("profiles/")}
    pat = re.compile(r"profiles/[A-Za-z0-9_./\-]+")
    keep = {p for p in prof if p.endswith(".md")}
    for f in tracked:
        if not f.endswith(TEXT):
            continue
        s = (ROOT / f).read_text(errors="ignore")
        cands = [m.rstrip(".,);:`'\"") for m in pat.findall(s)]
        if f.startswith("profiles/"):
            base = os.path.dirname(f)
            for m in re.findall(r"(?<![A-Za-z0-9_/])([A-Za-z0-9_\-]+(?:/[A-Za-z0-9_.\-]+)+/?)", s):
                cands.append(os.path.join(base, m.rstrip(".,);:`'\"")))
            for m in re.findall(r"`([A-Za-z0-9_.\-]+\.(?:csv|json|jsonl|txt|log|md))`", s):
                cands.append(os.path.join(base, m))
        keep.update(c for c in cands if c in prof)
    return keep


def pack(dirs=()):
    """Every directory of profiles/ (no ``dirs``), or only the given directories."""
    tracked = subprocess.run(["git", "ls-files"], cwd=ROOT, capture_output=True, text=True, check=True).stdout.split()
    keep = cited(tracked)
    want = {d.rstrip("/") for d in dirs}
    groups = {}
    for f in tracked:
        if f.startswith("profiles/") and f not in keep and not f.endswith("ARCHIVE.jsonl"):
            if want and not any(f.startswith(d + "/") for d in want):
                continue
            groups.setdefault(os.path.dirname(f), []).append(f)
    for d, fs in sorted(groups.items()):
        arc = ROOT / d / "ARCHIVE.jsonl"
        lines = []
        if arc.exists():
            lines = [x for x in arc.read_text().splitlines() if x.strip()]
        for f in sorted(fs):
            lines.append(json.dumps({"file": os.path.basename(f), "text": (ROOT / f).read_text(errors="replace")}))
            (ROOT / f).unlink()
        arc.write_text("\n".join(lines) + "\n")
    print(f"packed {sum(len(v) for v in groups.values())} files into {len(groups)} archives; kept {len(keep)} cited")


def unpack(d):
    arc = ROOT / d / "ARCHIVE.jsonl"
    for line in arc.read_text().splitlines():
        if line.strip():
            e = json.loads(line)
            (ROOT / d / e["file"]).write_text(e["text"])
            print(ROOT / d / e["file"])


def cat(path):
    d, name = os.path.split(path)
    for line in (ROOT / d / "ARCHIVE.jsonl").read_text().splitlines():
        if line.strip() and json.loads(line)["file"] == name:
            sys.stdout.write(json.loads(line)["text"])
            return
    raise SystemExit(f"{name} is not in {d}/ARCHIVE.jsonl")


if __name__ == "__main__":
    if len(sys.argv) < 2:
        raise SystemExit(__doc__)
    {"pack": lambda: pack(sys.argv[2:]), "unpack": lambda: unpack(sys.argv[2]), "cat": lambda: cat(sys.argv[2])}[sys.argv[1]]()

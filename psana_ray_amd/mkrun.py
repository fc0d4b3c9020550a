"""``psana-ray-mkrun``: write a synthetic run that ``psana-ray-producer`` picks up via ``--data_dir`` /
``$PSANA_RAY_DATA``: XTC2-style bigdata + smalldata files (default; psana's SMD layout, see
source/xtc2.py) or a fixed-record raw-run file (``--format praw``).

    psana-ray-mkrun --data_dir /data --exp mfxl1038923 --run 58 --detector_name epix10k2M --num_events 1000
"""
from __future__ import annotations

import argparse
import sys


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--data_dir", required=True)
    ap.add_argument("--exp", required=True)
    ap.add_argument("--run", type=int, required=True)
    ap.add_argument("--detector_name", required=True)
    ap.add_argument("--num_events", type=int, default=100)
    ap.add_argument("--format", choices=["xtc2", "praw"], default="xtc2")
    a = ap.parse_args(argv)
    if a.format == "xtc2":
        from .source.xtc2 import make_synthetic_xtc2_run

        big, smd = make_synthetic_xtc2_run(a.data_dir, a.exp, a.run, a.detector_name, a.num_events)
        print(big)
        print(smd)
        return 0
    from .source.rawfile import make_synthetic_run

    p = make_synthetic_run(a.data_dir, a.exp, a.run, a.detector_name, a.num_events)
    print(p)
    return 0


if __name__ == "__main__":
    sys.exit(main())

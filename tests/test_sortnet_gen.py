"""the common-mode kernel's generated networks (csrc/sortnet_gen.h) are re-derived
and verified here -- every merge node of every sort tree exhaustively on 0-1 inputs, V-merges
exhaustively on 0-1 V-shaped inputs, sorts / selections on random inputs -- and the committed
header must be exactly what the generator writes."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_generator_checks_and_header_is_current():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "sortnet_gen.py"), "--check", "--diff"],
                       capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    assert "matches the generator" in r.stdout

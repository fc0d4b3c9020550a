"""the common-mode kernel's NaN fill is ``fmed3(x, s, x)`` with x itself as the
third operand.  It is only correct while LLVM keeps that call as a v_med3_f32 (hardware: a NaN
operand makes med3 return min3 of its operands, which drops NaNs) instead of folding it to x.  This
test compiles csrc/common_mode.hip for gfx950 (device code only, no GPU needed) and checks that
the repeated-operand med3 instructions are in the ISA, so a compiler upgrade that folds them fails
here rather than silently in the data."""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = "/opt/rocm/bin/hipcc"


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not installed")
def test_nan_fill_med3_survives_compilation(tmp_path):
    out = tmp_path / "cm.s"
    r = subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off",
                        f"-I{ROOT}/csrc", "-x", "hip", "--cuda-device-only", "-S",
                        os.path.join(ROOT, "csrc", "common_mode.hip"), "-o", str(out)],
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    asm = out.read_text()
    same = re.findall(r"v_med3_f32 v\d+, (v\d+), v\d+, \1\s*$", asm, flags=re.M)
    assert len(same) >= 64, f"only {len(same)} NaN-fill med3 instructions (x, s, x) survived"

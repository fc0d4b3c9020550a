"""Host-side race / memory-safety checks of the native runtime (SURVEY §5 "Race detection").

tools/sanitize_host.sh builds tests/cpp/slotpool_stress.cpp + csrc/runtime.cpp + csrc/fabric.cpp
with ThreadSanitizer or AddressSanitizer+UBSan (host pass only) and runs producer / fabric /
consumer threads against the slot pool state machine and the link protocol (including a consumer
that leaves mid-stream)."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(not os.path.exists("/opt/rocm/lib/llvm/bin/clang++"), reason="ROCm clang not installed")
@pytest.mark.parametrize("san", ["thread", "address"])
def test_runtime_under_sanitizer(san, tmp_path):
    env = dict(os.environ, TMPDIR=str(tmp_path))
    r = subprocess.run(["bash", os.path.join(ROOT, "tools", "sanitize_host.sh"), san, "5000"], env=env,
                       capture_output=True, text=True, timeout=600)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert "SLOTPOOL_STRESS_OK" in r.stdout
    assert "WARNING: ThreadSanitizer" not in out and "ERROR: AddressSanitizer" not in out, out[-4000:]

"""Native threads stop before the process tears down (csrc/lifecycle.h).

A queue-fabric progress thread that is still running when the interpreter exits would keep calling
into the (HIP) runtime while its static destructors run.  The extension's loader registers
``halt_native_threads`` with atexit; these tests check that it stops and joins every live fabric
thread, that a halted fabric still destroys cleanly, and that a process which LEAKS running fabrics
exits with status 0."""
import os
import subprocess
import sys
import textwrap
import time

from tests.test_fabric_links import _member

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_halt_native_threads_stops_running_fabrics(native):
    C = native
    tok = f"/psq-halt-{os.getpid()}-{time.monotonic_ns() % 100000}"
    pp, pr_, pf = _member(C, tok, 0, 8, 0, 256, 0)
    cp, cr, cf = _member(C, tok, 1, 0, 8, 256, 0)
    name = f"{tok}-0-1"
    cf.add_in_link(0, name)
    pf.add_out_link(1, name)
    pf.start()
    cf.start()
    assert pf.running and cf.running
    C.halt_native_threads()
    assert not pf.running and not cf.running
    C.halt_native_threads()          # idempotent
    assert pf.join(1.0) and cf.join(1.0)
    del pf, cf                       # destructors after a halt: nothing left to join


def test_process_with_leaked_running_fabrics_exits_cleanly():
    code = textwrap.dedent(f"""
        import os, sys, time
        sys.path.insert(0, {REPO!r})
        from psana_ray_amd.ops import _ext
        from tests.test_fabric_links import _member
        C = _ext.load()
        tok = "/psq-leak-" + str(os.getpid())
        keep = []
        for r in range(3):
            pool, ring, fab = _member(C, tok, r, 4, 4, 256, 0)
            fab.start()
            keep.append((pool, ring, fab))
        sys.modules["__leak__"] = keep     # still referenced at interpreter exit
        time.sleep(0.2)
        print("ok", flush=True)
    """)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120, cwd=REPO)
    assert r.returncode == 0, (r.returncode, r.stdout[-2000:], r.stderr[-2000:])
    assert r.stdout.strip().endswith("ok")

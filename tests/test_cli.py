"""Producer/consumer CLI parity (psana_ray/producer.py:17-33) and end-to-end runs of the
installed entry points as separate processes (CPU, gloo)."""
import os
import random
import subprocess
import sys

import pytest

from psana_ray_amd import producer
from psana_ray_amd.config import DEFAULT_QUEUE_NAME, DEFAULT_RAY_NAMESPACE
from psana_ray_amd.data_reader import DataReader

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

REFERENCE_FLAGS = {
    # flag: (type, default, required)
    "--exp": (str, None, True), "--run": (int, None, True), "--detector_name": (str, None, True),
    "--calib": (bool, False, False), "--uses_bad_pixel_mask": (bool, False, False),
    "--manual_mask_path": (str, None, False), "--ray_address": (str, "auto", False),
    "--ray_namespace": (str, "default", False), "--queue_name": (str, "my", False),
    "--queue_size": (int, 100, False), "--num_consumers": (int, 1, False), "--max_steps": (int, None, False),
    "--log_level": (str, "INFO", False),
}


def test_reference_flags_identical():
    p = producer.build_parser()
    acts = {a.option_strings[0]: a for a in p._actions if a.option_strings}
    for flag, (typ, default, req) in REFERENCE_FLAGS.items():
        a = acts[flag]
        assert a.default == default, flag
        assert a.required == req, flag
        if typ is bool:
            assert a.const is True and a.nargs == 0, flag
        else:
            assert a.type is typ, flag
    assert acts["--log_level"].choices == ["DEBUG", "INFO", "WARNING", "ERROR", "CRITICAL"]


def test_readme_command_line_parses():
    a = producer.parse_arguments("--exp mfxl1038923 --run 58 --detector_name epix10k2M --queue_size 400".split())
    assert (a.exp, a.run, a.detector_name, a.queue_size, a.calib) == ("mfxl1038923", 58, "epix10k2M", 400, False)


def test_consumer_defaults_match_producer_defaults():
    """Q-3 fixed: DataReader() finds the queue a default producer creates."""
    r = DataReader()
    a = producer.parse_arguments(["--exp", "x", "--run", "1", "--detector_name", "epix10k2M"])
    assert (r.queue_name, r.ray_namespace) == (a.queue_name, a.ray_namespace) == (DEFAULT_QUEUE_NAME,
                                                                                  DEFAULT_RAY_NAMESPACE)


def test_backoff_schedule_matches_reference():
    assert [producer.backoff_delays(r)[0] for r in range(7)] == [0.1, 0.2, 0.4, 0.8, 1.6, 2.0, 2.0]
    assert producer.backoff_delays(0)[1] == 0.5


def test_read_before_connect_raises():
    with pytest.raises(RuntimeError):
        DataReader().read()


def test_in_process_queue_reader():
    from psana_ray_amd.shared_queue import create_queue, drop_queue

    q = create_queue("cfg1", "test", maxsize=4)
    q.put([0, 0, "frame", 9.5])
    with DataReader(queue_name="cfg1", ray_namespace="test") as r:
        assert r.read() == [0, 0, "frame", 9.5]
        assert r.read() is None
    drop_queue("cfg1", "test")


def _env(extra=None):
    env = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    env["PYTHONPATH"] = ROOT + os.pathsep + env.get("PYTHONPATH", "")
    env.update(extra or {})
    return env


@pytest.mark.parametrize("n_prod,n_cons", [(1, 1), (2, 2)])
def test_cli_end_to_end_cpu(native, tmp_path, n_prod, n_cons):
    port = random.randint(30000, 45000)
    addr = f"127.0.0.1:{port}"
    n_events = 12
    prods = []
    for r in range(n_prod):
        env = _env({"RANK": str(r), "WORLD_SIZE": str(n_prod), "LOCAL_RANK": str(r)})
        prods.append(subprocess.Popen(
            [sys.executable, "-m", "psana_ray_amd.producer", "--exp", "synthetic", "--run", "3", "--detector_name",
             "tiny_epix", "--calib", "--num_events", str(n_events), "--ray_address", addr, "--num_consumers",
             str(n_cons), "--queue_size", "6", "--device", "cpu", "--uses_bad_pixel_mask", "--timeout", "60"],
            env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True))
    cons = [subprocess.Popen([sys.executable, "-m", "psana_ray_amd.consumer", str(c), "--ray_address", addr,
                              "--device", "cpu", "--timeout", "60"],
                             env=_env(), stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
            for c in range(n_cons)]
    outs = []
    try:
        for p in prods + cons:
            out, _ = p.communicate(timeout=180)
            outs.append((p.returncode, out))
    finally:
        for p in prods + cons:
            if p.poll() is None:
                p.kill()
    for rc, out in outs:
        assert rc == 0, out[-3000:]
    processed = [l for _, out in outs[n_prod:] for l in out.splitlines() if "processed:" in l]
    assert len(processed) == n_events
    for l in processed:
        assert "shape=(2, 32, 48)" in l


def test_calibrate_on_read_cpu(native):
    """Capacity tier: the producer queues RAW frames (--calibrate_on_read) and the DataReader
    calibrates them on read with the same constants, mask and common mode."""
    port = random.randint(30000, 45000)
    addr = f"127.0.0.1:{port}"
    n_events = 10
    prod = subprocess.Popen(
        [sys.executable, "-m", "psana_ray_amd.producer", "--exp", "synthetic", "--run", "4", "--detector_name",
         "tiny_epix", "--calib", "--num_events", str(n_events), "--ray_address", addr, "--num_consumers", "1",
         "--queue_size", "4", "--device", "cpu", "--uses_bad_pixel_mask", "--common_mode", "default",
         "--calibrate_on_read", "--timeout", "60"],
        env=_env({"RANK": "0", "WORLD_SIZE": "1", "LOCAL_RANK": "0"}), stdout=subprocess.PIPE,
        stderr=subprocess.STDOUT, text=True)
    cons = subprocess.Popen([sys.executable, os.path.join(ROOT, "tests", "_cor_consumer.py"), addr, "1", "tiny_epix",
                             "4"], env=_env(), stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    try:
        pout, _ = prod.communicate(timeout=180)
        cout, _ = cons.communicate(timeout=180)
    finally:
        for p in (prod, cons):
            if p.poll() is None:
                p.kill()
    assert prod.returncode == 0, pout[-3000:]
    assert cons.returncode == 0, cout[-3000:]
    assert f"COR_OK {n_events}" in cout


def test_sigint_on_endless_producer_ends_stream_cleanly(native):
    """R-03 / Q-14: Ctrl+C on an endless producer (no --num_events) stops production, advertises
    EOS and exits 0; the consumer sees the end of stream (reference: only rank 0 handled SIGINT,
    with ray.shutdown(); exit(0), psana_ray/producer.py:73-76,142-143, so consumers polled forever)."""
    import signal
    import threading

    port = random.randint(30000, 45000)
    addr = f"127.0.0.1:{port}"
    prod = subprocess.Popen(
        [sys.executable, "-m", "psana_ray_amd.producer", "--exp", "synthetic", "--run", "5", "--detector_name",
         "tiny_epix", "--calib", "--ray_address", addr, "--num_consumers", "1", "--queue_size", "4",
         "--device", "cpu", "--timeout", "60"],
        env=_env({"RANK": "0", "WORLD_SIZE": "1", "LOCAL_RANK": "0"}), stdout=subprocess.PIPE,
        stderr=subprocess.STDOUT, text=True)
    cons = subprocess.Popen([sys.executable, "-m", "psana_ray_amd.consumer", "0", "--ray_address", addr,
                             "--device", "cpu", "--timeout", "60"],
                            env=_env(), stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    lines, seen = [], threading.Event()

    def pump():
        for line in cons.stdout:
            lines.append(line)
            if sum("processed:" in l for l in lines) >= 5:
                seen.set()

    t = threading.Thread(target=pump, daemon=True)
    t.start()
    try:
        assert seen.wait(120), "consumer never received frames:\n" + "".join(lines)[-3000:]
        prod.send_signal(signal.SIGINT)
        pout, _ = prod.communicate(timeout=120)
        cons.wait(timeout=120)
        t.join(timeout=10)
    finally:
        for p in (prod, cons):
            if p.poll() is None:
                p.kill()
    assert prod.returncode == 0, pout[-3000:]
    assert "Ctrl+C pressed" in pout
    out = "".join(lines)
    assert cons.returncode == 0, out[-3000:]
    assert "end of stream" in out, out[-3000:]
    idx = [int(l.split("idx=")[1].split()[0]) for l in lines if "processed:" in l]
    assert idx == list(range(len(idx))), "frames lost or duplicated before EOS"


def test_consumer_without_a_store_fails_with_one_line():
    """No rendezvous store at the address: the consumer CLI ends with one clear error line and
    rc 1 (no traceback)."""
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, PYTHONPATH=root)
    p = subprocess.run([sys.executable, "-m", "psana_ray_amd.consumer", "--ray_address", f"127.0.0.1:{port}",
                        "--timeout", "2", "--metrics_interval", "0"], env=env, cwd=root, capture_output=True,
                       text=True, timeout=120)
    assert p.returncode == 1, p.stdout + p.stderr
    assert "Traceback" not in p.stderr, p.stderr
    assert "could not join the queue" in p.stderr and f"127.0.0.1:{port}" in p.stderr, p.stderr

"""Elastic membership of one named shared queue (the Ray named/detached actor analog).

Reference behaviour (SURVEY R-02, R-10, R-11, C-04, P-02):
  * the first producer job creates the named queue, a later job with the same
    ``(ray_namespace, queue_name)`` reuses it (psana_ray/producer.py:39-48, shared_queue.py:33-35);
  * producers put immediately -- the actor buffers up to ``maxsize`` items with nobody reading
    (producer.py:98-111);
  * any number of consumers attach whenever they like (data_reader.py:11-24, README.md:23-35);
    ``--num_consumers`` is only the number of end-of-stream sentinels (producer.py:29,121-126);
  * a consumer crash affects nobody else; only the actor's death stops producers (producer.py:112-114).

Here a queue is a SESSION in the rendezvous store (``torch.distributed.TCPStore``) keyed by
``psana_ray/<namespace>/<queue>``: ``meta`` (frame shape, dtype, device kind, queue_size and a
random ``token`` naming the session's shared-memory mailboxes) plus one record per MEMBER
process (role, pid, host, boot id, device) under a monotonically growing member id.  Every
member runs a watcher thread that
  * heartbeats (cross-host liveness) and publishes its state (running / draining / done / closed),
  * discovers members that joined after it and asks the native fabric (csrc/fabric.h) for the
    links that pair it with them (producer -> consumer),
  * notices members that died (pid gone on this host, stale heartbeat elsewhere) so the fabric
    takes back what they held.
Nothing is fixed at creation: producers start without consumers, consumers come and go, a second
producer job attaches to a live session (a stale session -- no live member -- is replaced).
Links are node-local (shared memory + HIP IPC); members on another host are reported and ignored.
"""
from __future__ import annotations

import json
import logging
import os
import socket
import threading
import time
import uuid
from typing import Callable, Dict, Optional

log = logging.getLogger(__name__)

HEARTBEAT_S = 1.0
STALE_S = 10.0          # heartbeat age after which a member on another host counts as dead
CREATE_GRACE_S = 10.0   # a freshly created session counts as live before its members registered
PRODUCER_ROLES = ("producer", "prosumer", "keeper")
CONSUMER_ROLES = ("consumer", "prosumer", "keeper")   # keeper: psana_ray_amd/keeper.py


def queue_key(namespace: str, queue_name: str) -> str:
    return f"psana_ray/{namespace}/{queue_name}"


def boot_id() -> str:
    try:
        with open("/proc/sys/kernel/random/boot_id") as f:
            return f.read().strip()
    except OSError:
        return ""


def _pid_alive(pid: int) -> bool:
    from ..ops import _ext

    return bool(_ext.load().pid_alive(int(pid)))


class QueueMismatch(RuntimeError):
    """A live queue with this name carries frames of another shape / dtype / device kind."""


def _get_json(store, key: str) -> Optional[dict]:
    if not store.check([key]):
        return None
    return json.loads(store.get(key).decode())


def member_alive(store, base_s: str, mid: int, info: dict, here_boot: str) -> bool:
    if info.get("boot") == here_boot and here_boot:
        return _pid_alive(int(info["pid"]))
    try:
        hb = float(store.get(f"{base_s}/hb/{mid}").decode())
    except Exception:  # noqa: BLE001
        return False
    return time.time() - hb < STALE_S


def session_live(store, base: str, meta: dict) -> bool:
    """Any member of the session still alive (or the session was created moments ago)?"""
    if time.time() - float(meta.get("created", 0)) < CREATE_GRACE_S:
        return True
    base_s = f"{base}/s{meta['session']}"
    n = store.add(f"{base_s}/mids", 0)
    here = boot_id()
    for mid in range(n):
        info = _get_json(store, f"{base_s}/m/{mid}")
        if info is None:
            continue
        st = store.get(f"{base_s}/st/{mid}").decode() if store.check([f"{base_s}/st/{mid}"]) else "running"
        if st in ("done", "closed", "failed"):
            continue
        if member_alive(store, base_s, mid, info, here):
            return True
    return False


def _compatible(a: dict, b: dict) -> bool:
    return (list(a["frame_shape"]) == list(b["frame_shape"]) and a["dtype"] == b["dtype"]
            and a["device_kind"] == b["device_kind"])


def create_or_attach(store, namespace: str, queue_name: str, meta: dict, timeout_s: float = 60.0) -> dict:
    """Producer side: the live session of this queue (attach-if-exists, producer.py:43-45) or a new
    one.  Concurrent creators agree through compare-and-set."""
    base = queue_key(namespace, queue_name)
    key = f"{base}/meta"
    deadline = time.time() + timeout_s
    while True:
        cur = store.get(key).decode() if store.check([key]) else None
        if cur is not None:
            m = json.loads(cur)
            if session_live(store, base, m):
                if not _compatible(m, meta):
                    raise QueueMismatch(
                        f"queue {queue_name!r} (namespace {namespace!r}) is live with frames {m['frame_shape']} "
                        f"{m['dtype']} on {m['device_kind']}; this job produces {list(meta['frame_shape'])} "
                        f"{meta['dtype']} on {meta['device_kind']}")
                return m
        new = dict(meta)
        new["frame_shape"] = list(meta["frame_shape"])
        new["session"] = int(store.add(f"{base}/session_counter", 1))
        new["token"] = uuid.uuid4().hex[:10]
        new["created"] = time.time()
        js = json.dumps(new)
        got = store.compare_set(key, cur if cur is not None else "", js).decode()
        if got == js:
            log.info("Shared queue %s created (namespace %s, queue_size=%s, session %d).", queue_name, namespace,
                     new.get("queue_size"), new["session"])
            return new
        if time.time() > deadline:
            raise TimeoutError(f"could not create or attach queue {queue_name!r}")


def wait_meta(store, namespace: str, queue_name: str, timeout_s: float) -> dict:
    """Consumer side: the live session of this queue, waiting up to ``timeout_s`` for one."""
    base = queue_key(namespace, queue_name)
    deadline = time.time() + timeout_s
    while True:
        m = _get_json(store, f"{base}/meta")
        if m is not None and session_live(store, base, m):
            return m
        if time.time() > deadline:
            raise TimeoutError(f"queue {queue_name!r} in namespace {namespace!r} has no live producer "
                               f"(waited {timeout_s:.0f} s)")
        time.sleep(0.2)


class QueueSession:
    """This process's membership of a queue session (see module docstring)."""

    def __init__(self, store, namespace: str, queue_name: str, meta: dict, role: str, device: int = -1,
                 job: Optional[str] = None, rank: Optional[int] = None, own_store: bool = False):
        assert role in ("producer", "consumer", "prosumer", "keeper"), role
        self.store = store
        self.namespace, self.queue_name = namespace, queue_name
        self.meta = meta
        self.role = role
        self.base = queue_key(namespace, queue_name)
        self.base_s = f"{self.base}/s{meta['session']}"
        self.token = meta["token"]
        self.own_store = own_store
        self.boot = boot_id()
        self.host = socket.gethostname()
        self.mid = int(store.add(f"{self.base_s}/mids", 1)) - 1
        self.consumer_seq = int(store.add(f"{self.base_s}/cseq", 1)) - 1 if role in CONSUMER_ROLES else -1
        info = {"role": role, "pid": os.getpid(), "host": self.host, "boot": self.boot, "device": device,
                "job": job, "rank": rank, "t": time.time()}
        self.info = info
        store.set(f"{self.base_s}/hb/{self.mid}", repr(time.time()))
        store.set(f"{self.base_s}/st/{self.mid}", "running")
        store.set(f"{self.base_s}/m/{self.mid}", json.dumps(info))
        # global registry: lets a detached store server exit once no member is left
        reg = int(store.add("psana_ray/_reg_n", 1)) - 1
        store.set(f"psana_ray/_reg/{reg}", json.dumps({"pid": os.getpid(), "boot": self.boot}))
        self.members: Dict[int, dict] = {}
        self.states: Dict[int, str] = {}
        self.dead: set = set()
        self._known = 0
        self._state = "running"
        self._lock = threading.Lock()
        self._poll_lock = threading.Lock()
        self._stop = threading.Event()
        self._thread: Optional[threading.Thread] = None
        self.store_lost = False
        self._warned_remote: set = set()
        self.on_member: Optional[Callable[[int, dict], None]] = None
        self.on_dead: Optional[Callable[[int], None]] = None
        self.on_tick: Optional[Callable[[], None]] = None

    # ------------------------------------------------------------------------ naming
    def link_name(self, producer_mid: int, consumer_mid: int) -> str:
        return f"/psq-{self.token}-{producer_mid}-{consumer_mid}"

    def ring_name(self) -> str:
        return f"/psq-{self.token}-r{self.mid}"

    # ------------------------------------------------------------------------ state
    def set_state(self, state: str):
        self._state = state
        try:
            self.store.set(f"{self.base_s}/st/{self.mid}", state)
        except Exception as e:  # noqa: BLE001 - the store host may be gone at the very end
            log.debug("member %d: could not publish state %s: %r", self.mid, state, e)

    def producers(self) -> Dict[int, dict]:
        with self._lock:
            return {m: i for m, i in self.members.items() if i["role"] in PRODUCER_ROLES}

    def state(self, mid: int) -> str:
        with self._lock:
            return self.states.get(mid, "running")

    def finished(self, mid: int) -> bool:
        """Producer member ``mid`` will send nothing more (done, failed, left, or dead)."""
        with self._lock:
            return mid in self.dead or self.states.get(mid) in ("done", "closed", "failed")

    # ------------------------------------------------------------------------ watcher
    def start(self, on_member: Callable[[int, dict], None], on_dead: Callable[[int], None],
              on_tick: Optional[Callable[[], None]] = None):
        self.on_member, self.on_dead, self.on_tick = on_member, on_dead, on_tick
        self.poll()   # members already present are linked before the first frame moves
        self._thread = threading.Thread(target=self._run, name=f"psana-ray-session-{self.mid}", daemon=True)
        self._thread.start()
        from ..ops import _ext

        _ext.on_exit(self)   # a session left open stops its watcher before the native threads halt
        return self

    def stop_at_exit(self):
        """Process exit: stop the watcher thread (its callbacks drive the native fabric)."""
        self._stop.set()
        if self._thread is not None and self._thread is not threading.current_thread():
            self._thread.join(2)

    def _run(self):
        last_hb = 0.0
        while not self._stop.wait(0.1):
            try:
                now = time.time()
                if now - last_hb >= HEARTBEAT_S:
                    self.store.set(f"{self.base_s}/hb/{self.mid}", repr(now))
                    last_hb = now
                if self.on_tick is not None:
                    self.on_tick()
                self.poll()
                if self.store_lost:
                    log.info("member %d: rendezvous store is reachable again", self.mid)
                    self.store_lost = False
            except Exception as e:  # noqa: BLE001 - the store host left: keep the links we have
                if not self.store_lost:
                    log.warning("member %d: rendezvous store unreachable (%r); existing links keep working",
                                self.mid, e)
                self.store_lost = True

    def poll(self):
        with self._poll_lock:
            self._poll()

    def _poll(self):
        st = self.store
        n = int(st.add(f"{self.base_s}/mids", 0))
        for mid in range(self._known, n):
            key = f"{self.base_s}/m/{mid}"
            if not st.check([key]):
                break   # registered its id but not its record yet: next poll
            info = json.loads(st.get(key).decode())
            self._known = mid + 1
            if mid == self.mid:
                continue
            with self._lock:
                self.members[mid] = info
                self.states[mid] = "running"
            if info.get("boot") != self.boot or not self.boot:
                if mid not in self._warned_remote:
                    log.warning("member %d of queue %s runs on host %s: links are node-local, it is ignored", mid,
                                self.queue_name, info.get("host"))
                    self._warned_remote.add(mid)
                continue
            if self.on_member is not None:
                self.on_member(mid, info)
        # states + liveness of the members we know
        with self._lock:
            mids = list(self.members)
        for mid in mids:
            if mid in self.dead:
                continue
            try:
                s = st.get(f"{self.base_s}/st/{mid}").decode()
            except Exception:  # noqa: BLE001
                s = "running"
            with self._lock:
                self.states[mid] = s
            info = self.members[mid]
            if not member_alive(st, self.base_s, mid, info, self.boot):
                with self._lock:
                    self.dead.add(mid)
                if s not in ("done", "closed"):
                    log.warning("queue %s: member %d (%s, pid %s) died", self.queue_name, mid, info["role"],
                                info["pid"])
                if self.on_dead is not None:
                    self.on_dead(mid)

    def close(self, state: str = "closed"):
        self._stop.set()
        if self._thread is not None:
            self._thread.join(5)
        self.set_state(state)

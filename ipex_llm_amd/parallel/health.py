"""Rank-failure detection for multi-process serving.

Reference: the reference relies on the oneCCL / torch process-group timeout
and its API server's /health route (``serving/fastapi/api_server.py``);
a dead pipeline rank leaves the other ranks blocked in a collective until
that timeout fires.

Here every rank runs a :class:`Heartbeat` thread that stamps
``illm/hb/<rank>`` in the job's c10d key-value store (the same TCPStore the
process group rendezvoused on, so no extra port) once per ``interval``.
A :class:`RankMonitor` on the driving rank reads the stamps; a rank silent
for ``timeout`` seconds (or whose process is gone, so its heartbeat socket
errors) is declared dead.  The serving loops check the monitor before every
tick -- a collective is never entered with a dead peer -- and on failure
abort the process group (so a rank already blocked inside a collective
returns), finish every in-flight request with ``finish_reason="error: ..."``
(streams are woken, clients do not hang) and report it on /health.
"""
from __future__ import annotations

import threading
import time
from typing import Dict, List, Optional


class RankFailureError(RuntimeError):
    pass


def default_store():
    """the default process group's c10d store (None without torch.distributed)"""
    try:
        import torch.distributed as dist
        from torch.distributed import distributed_c10d as c10d
        if not dist.is_initialized():
            return None
        return c10d._get_default_store()
    except Exception:  # pragma: no cover - older torch layouts
        return None


class Heartbeat:
    def __init__(self, store, rank: int, interval: float = 0.5, prefix: str = "illm/hb"):
        self.store, self.rank, self.interval, self.prefix = store, rank, interval, prefix
        self._stop = threading.Event()
        self.thread = threading.Thread(target=self._run, daemon=True, name=f"illm-heartbeat-{rank}")

    def start(self):
        self._beat()
        self.thread.start()
        return self

    def _beat(self):
        self.store.set(f"{self.prefix}/{self.rank}", repr(time.time()))

    def _run(self):
        while not self._stop.wait(self.interval):
            try:
                self._beat()
            except Exception:       # store gone (job tearing down): stop quietly
                return

    def stop(self):
        self._stop.set()
        try:
            self.store.set(f"{self.prefix}/{self.rank}", "stopped")
        except Exception:
            pass


class RankMonitor:
    """Watches the heartbeats of ``ranks``; ``check()`` raises
    :class:`RankFailureError` naming the dead ranks."""

    def __init__(self, store, ranks: List[int], timeout: float = 5.0, prefix: str = "illm/hb",
                 poll: float = 0.5):
        self.store, self.ranks, self.timeout, self.prefix = store, list(ranks), timeout, prefix
        self.poll = poll
        self.dead: List[int] = []
        self.reason: Optional[str] = None
        self._last_poll = 0.0
        self._stamp: Dict[int, float] = {}
        self.t0 = time.time()

    def _read(self, r: int) -> Optional[float]:
        key = f"{self.prefix}/{r}"
        if not self.store.check([key]):
            return None
        v = self.store.get(key).decode()
        return -1.0 if v == "stopped" else float(v)

    def poll_now(self) -> List[int]:
        now = time.time()
        dead = []
        for r in self.ranks:
            try:
                t = self._read(r)
            except Exception as e:           # store unreachable: the store host (rank 0) itself is gone
                self.reason = f"heartbeat store unreachable: {e!r}"
                return list(self.ranks)
            if t is None:
                if now - self.t0 > self.timeout:
                    dead.append(r)
                continue
            if t < 0:
                continue                     # stopped cleanly
            self._stamp[r] = t
            if now - t > self.timeout:
                dead.append(r)
        self.dead = dead
        if dead:
            self.reason = f"rank(s) {dead} missed heartbeats for > {self.timeout:.1f}s"
        return dead

    def check(self):
        now = time.time()
        if now - self._last_poll >= self.poll:
            self._last_poll = now
            self.poll_now()
        if self.dead:
            raise RankFailureError(self.reason)

    @property
    def healthy(self) -> bool:
        return not self.dead


def abort_process_group(group=None):
    """best effort: make collectives blocked on a dead peer return"""
    try:
        from torch.distributed import distributed_c10d as c10d
        fn = getattr(c10d, "_abort_process_group", None)
        if fn is not None:
            fn(group) if group is not None else fn()
            return True
    except Exception:
        pass
    return False

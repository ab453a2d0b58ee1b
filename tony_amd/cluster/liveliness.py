"""Heartbeat liveliness monitor (T/ApplicationMaster.java:202-222, Hadoop AbstractLivelinessMonitor).

Tasks register when they pass ``registerWorkerSpec`` and ping every
``tony.task.heartbeat-interval-ms``; a task not heard from for
``interval * max(3, tony.task.max-missed-heartbeats)`` ms is declared dead and
``on_expired(task_id)`` fires once (the coordinator fails the session).  A task
that reports its execution result is unregistered first, which is what closes
the completion-vs-expiry race TonY documents (ApplicationMaster.java:928-956).
"""
from __future__ import annotations

import logging
import threading
import time
from typing import Callable, Dict

LOG = logging.getLogger(__name__)


class HeartbeatMonitor:
    def __init__(self, hb_interval_ms: int, max_missed: int, on_expired: Callable[[str], None]):
        self.expire_s = hb_interval_ms * max(3, max_missed) / 1000.0
        self.check_s = max(0.05, 3 * hb_interval_ms / 1000.0 / 4)
        self.on_expired = on_expired
        self._last: Dict[str, float] = {}
        self._lock = threading.Lock()
        self._stop = threading.Event()
        self._thread = threading.Thread(target=self._run, name="tony-hb-monitor", daemon=True)

    def start(self):
        self._thread.start()

    def stop(self):
        self._stop.set()

    def register(self, task_id: str) -> None:
        with self._lock:
            self._last[task_id] = time.monotonic()

    def received_ping(self, task_id: str) -> bool:
        with self._lock:
            if task_id not in self._last:
                return False
            self._last[task_id] = time.monotonic()
            return True

    def unregister(self, task_id: str) -> None:
        with self._lock:
            self._last.pop(task_id, None)

    def reset(self) -> None:
        with self._lock:
            self._last.clear()

    def _run(self):
        while not self._stop.wait(self.check_s):
            now = time.monotonic()
            expired = []
            with self._lock:
                for tid, t in list(self._last.items()):
                    if now - t > self.expire_s:
                        expired.append(tid)
                        del self._last[tid]
            for tid in expired:
                LOG.error("task %s missed heartbeats for %.1fs", tid, self.expire_s)
                try:
                    self.on_expired(tid)
                except Exception:  # noqa: BLE001
                    LOG.exception("expiry callback failed")

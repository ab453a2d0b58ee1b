"""History maintenance: mover (mark crashed jobs KILLED, move finished jobs) and purger.

Parity: tony-portal app/history/HistoryFileMover.java:35-170 and
HistoryFilePurger.java:26-113.  YARN told TonY's mover which apps were KILLED;
here the coordinator leaves an ``coordinator.owner`` file (host, pid, process
start time) in its intermediate job dir, and a job whose jhist is still
``.inprogress`` while its owner process is gone is the "killed app".
"""
from __future__ import annotations

import datetime as _dt
import json
import logging
import os
import re
import shutil
import socket
import threading
import time
from typing import Callable, List, Optional

from .. import constants as C
from ..events.history import completed_time_from_file_name, get_jhist_file_path, year_month_day_dir

LOG = logging.getLogger("tony.portal.history")
OWNER_FILE = "coordinator.owner"


def write_owner(job_dir: str, staging_job_dir: Optional[str] = None) -> None:
    """Called by the coordinator when it creates its intermediate history dir.

    ``staging_job_dir`` (where the per-task logs live) lets the portal link logs."""
    info = {"host": socket.gethostname(), "pid": os.getpid(), "start": _proc_start(os.getpid()),
            "jobDir": staging_job_dir}
    with open(os.path.join(job_dir, OWNER_FILE), "w") as f:
        json.dump(info, f)


def read_owner(job_dir: str) -> dict:
    try:
        with open(os.path.join(job_dir, OWNER_FILE)) as f:
            return json.load(f)
    except (OSError, ValueError):
        return {}


def _proc_start(pid: int) -> Optional[float]:
    try:
        import psutil

        return psutil.Process(pid).create_time()
    except Exception:  # noqa: BLE001
        return None


def owner_alive(job_dir: str) -> Optional[bool]:
    """True/False when decidable from this host, None when the owner lives elsewhere / is unknown."""
    info = read_owner(job_dir)
    if not info:
        return None
    if info.get("host") != socket.gethostname():
        return None
    pid = int(info.get("pid", -1))
    if pid <= 0:
        return None
    try:
        os.kill(pid, 0)
    except ProcessLookupError:
        return False
    except PermissionError:
        pass
    start = info.get("start")
    now_start = _proc_start(pid)
    if start is not None and now_start is not None and abs(now_start - start) > 1.0:
        return False  # pid reused by another process
    return True


def killed_file_name(inprogress_path: str, now_ms: int) -> str:
    """``<id>-<start>-<user>.jhist.inprogress`` -> ``<id>-<start>-<now>-<user>-KILLED.jhist``."""
    d, name = os.path.split(inprogress_path)
    head, tail = name.rsplit("-", 1)
    user = tail.split(".")[0]
    return os.path.join(d, f"{head}-{now_ms}-{user}-{C.KILLED}.{C.HISTFILE_SUFFIX}")


class HistoryFileMover:
    def __init__(self, intermediate: str, finished: str, tz: str = "UTC",
                 is_killed: Optional[Callable[[str], bool]] = None,
                 on_job_dir: Optional[Callable[[str], None]] = None):
        self.intermediate = intermediate
        self.finished = finished
        self.tz = tz
        self.is_killed = is_killed or (lambda d: owner_alive(d) is False)
        self.on_job_dir = on_job_dir
        self._stop = threading.Event()

    def _job_dirs(self) -> List[str]:
        try:
            return [os.path.join(self.intermediate, d) for d in sorted(os.listdir(self.intermediate))
                    if os.path.isdir(os.path.join(self.intermediate, d))]
        except OSError:
            return []

    def rename_killed_apps(self, dirs: List[str]) -> List[str]:
        renamed = []
        for d in dirs:
            path = get_jhist_file_path(d)
            if path is None or not path.endswith(C.INPROGRESS) or not self.is_killed(d):
                continue
            dst = killed_file_name(path, int(time.time() * 1000))
            try:
                os.rename(path, dst)
                renamed.append(dst)
                LOG.info("marked killed: %s", dst)
            except OSError:
                LOG.exception("failed to rename killed app %s", path)
        return renamed

    def move_intermediate_to_finished(self, dirs: List[str]) -> List[str]:
        moved = []
        for d in dirs:
            if self.on_job_dir is not None:
                self.on_job_dir(d)
            path = get_jhist_file_path(d)
            if path is None or not path.endswith(C.HISTFILE_SUFFIX):
                continue
            dst_root = year_month_day_dir(self.finished, completed_time_from_file_name(path), self.tz)
            dst = os.path.join(dst_root, os.path.basename(d))
            try:
                os.makedirs(dst_root, mode=0o770, exist_ok=True)
                if os.path.exists(dst):
                    shutil.rmtree(dst)
                shutil.move(d, dst)
                moved.append(dst)
            except OSError:
                LOG.exception("failed to move %s to %s", d, dst)
        return moved

    def run_once(self) -> List[str]:
        dirs = self._job_dirs()
        self.rename_killed_apps(dirs)
        return self.move_intermediate_to_finished(dirs)

    def start(self, interval_ms: int) -> threading.Thread:
        def loop():
            while not self._stop.is_set():
                try:
                    self.run_once()
                except Exception:  # noqa: BLE001
                    LOG.exception("history mover failed")
                self._stop.wait(interval_ms / 1000.0)

        t = threading.Thread(target=loop, name="tony-history-mover", daemon=True)
        t.start()
        return t

    def stop(self) -> None:
        self._stop.set()


def _last_day_of_month(y: int, m: int) -> _dt.date:
    nxt = _dt.date(y + (m == 12), m % 12 + 1, 1)
    return nxt - _dt.timedelta(days=1)


def purge_finished_dir(finished: str, cutoff: _dt.date) -> List[str]:
    """Delete yyyy / MM / dd dirs entirely before ``cutoff`` (HistoryFilePurger.purgeFinishedDir)."""
    gone = []

    def ls(p, pat):
        try:
            return sorted(n for n in os.listdir(p) if re.fullmatch(pat, n) and os.path.isdir(os.path.join(p, n)))
        except OSError:
            return []

    for y in ls(finished, r"\d{4}"):
        yp = os.path.join(finished, y)
        if _dt.date(int(y), 12, 31) < cutoff:
            shutil.rmtree(yp, ignore_errors=True)
            gone.append(yp)
            continue
        for m in ls(yp, r"\d{2}"):
            mp = os.path.join(yp, m)
            if _last_day_of_month(int(y), int(m)) < cutoff:
                shutil.rmtree(mp, ignore_errors=True)
                gone.append(mp)
                continue
            for d in ls(mp, r"\d{2}"):
                dp = os.path.join(mp, d)
                try:
                    if _dt.date(int(y), int(m), int(d)) < cutoff:
                        shutil.rmtree(dp, ignore_errors=True)
                        gone.append(dp)
                except ValueError:
                    continue
    return gone


def purge_intermediate_dir(intermediate: str, cutoff: _dt.date) -> List[str]:
    """Delete intermediate job dirs last modified before ``cutoff``."""
    gone = []
    try:
        names = os.listdir(intermediate)
    except OSError:
        return gone
    for n in names:
        p = os.path.join(intermediate, n)
        try:
            if _dt.date.fromtimestamp(os.path.getmtime(p)) < cutoff:
                shutil.rmtree(p, ignore_errors=True) if os.path.isdir(p) else os.remove(p)
                gone.append(p)
        except OSError:
            continue
    return gone


class HistoryFilePurger:
    def __init__(self, intermediate: str, finished: str, retention_sec: int, tz: str = "UTC"):
        self.intermediate, self.finished = intermediate, finished
        self.retention_sec = retention_sec
        self.tz = tz
        self._stop = threading.Event()

    def cutoff(self) -> _dt.date:
        now = _dt.datetime.now(_dt.timezone.utc)
        if self.tz and self.tz.upper() != "UTC":
            try:
                from zoneinfo import ZoneInfo

                now = now.astimezone(ZoneInfo(self.tz))
            except Exception:  # noqa: BLE001
                pass
        return (now - _dt.timedelta(seconds=self.retention_sec)).date()

    def run_once(self) -> List[str]:
        c = self.cutoff()
        return purge_finished_dir(self.finished, c) + purge_intermediate_dir(self.intermediate, c)

    def start(self, interval_ms: int) -> threading.Thread:
        def loop():
            while not self._stop.is_set():
                try:
                    self.run_once()
                except Exception:  # noqa: BLE001
                    LOG.exception("history purger failed")
                self._stop.wait(interval_ms / 1000.0)

        t = threading.Thread(target=loop, name="tony-history-purger", daemon=True)
        t.start()
        return t

    def stop(self) -> None:
        self._stop.set()

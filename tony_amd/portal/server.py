"""History portal: job list, config, events and log pages over the local history dir.

Parity: tony-portal conf/routes:1-5 (``/``, ``/config/:jobId``, ``/jobs/:jobId``,
``/logs/:jobId``), app/controllers/*PageController.java (sorting rules),
app/cache/CacheWrapper.java:28-132 (bounded caches warmed from the finished +
intermediate dirs).  Pages are plain HTML tables (no Play / Bootstrap); every
page also answers ``?format=json`` for scripting.  Log links point at the
per-task log dirs the coordinator writes (``<job dir>/logs/<container>``).
"""
from __future__ import annotations

import html
import json
import logging
import os
import threading
from collections import OrderedDict
from dataclasses import asdict
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from typing import Dict, List, Optional
from urllib.parse import parse_qs, urlparse

from .. import constants as C
from .history import read_owner
from ..events.history import (DEFAULT_JOB_ID_REGEX, JobMetadata, find_job_dirs, map_event_to_job_log,
                              parse_config, parse_events, parse_metadata)

LOG = logging.getLogger("tony.portal")


class _LRU:
    def __init__(self, max_entries: int):
        self.max = max(1, int(max_entries))
        self._d: "OrderedDict[str, object]" = OrderedDict()
        self._lock = threading.Lock()

    def get(self, k):
        with self._lock:
            if k not in self._d:
                return None
            self._d.move_to_end(k)
            return self._d[k]

    def put(self, k, v) -> None:
        with self._lock:
            self._d[k] = v
            self._d.move_to_end(k)
            while len(self._d) > self.max:
                self._d.popitem(last=False)

    def values(self):
        with self._lock:
            return list(self._d.values())

    def __len__(self):
        return len(self._d)


class CacheWrapper:
    """Metadata / config / event / log caches keyed by job id."""

    def __init__(self, intermediate: str, finished: str, max_entries: int = 1000,
                 logs_root: Optional[str] = None, job_id_regex: str = DEFAULT_JOB_ID_REGEX):
        self.intermediate, self.finished = intermediate, finished
        self.logs_root = logs_root
        self.regex = job_id_regex
        self.metadata = _LRU(max_entries)
        self.config = _LRU(max_entries)
        self.events = _LRU(max_entries)
        self.logs = _LRU(max_entries)
        self._dirs: Dict[str, str] = {}

    def update_caches(self, job_dir: str) -> None:
        job_id = os.path.basename(job_dir.rstrip("/"))
        md = parse_metadata(job_dir, self.regex)
        if md is None:
            return
        self._dirs[job_id] = job_dir
        self.metadata.put(job_id, md)
        self.config.put(job_id, parse_config(job_dir))
        evs = parse_events(job_dir)
        self.events.put(job_id, evs)
        logs_root = self.logs_root or self._staging_logs(job_dir, job_id)
        self.logs.put(job_id, [lg for lg in (map_event_to_job_log(e, logs_root) for e in evs) if lg is not None])

    @staticmethod
    def _staging_logs(job_dir: str, job_id: str) -> Optional[str]:
        """The coordinator records its staging job dir (holding ``logs/<container>``) in its owner file."""
        staging = read_owner(job_dir).get("jobDir")
        return os.path.join(staging, "logs") if staging else None

    def warm(self) -> int:
        """(Re)load job dirs not cached yet, moved since, or still running."""
        n = 0
        for root in (self.finished, self.intermediate):
            for d in find_job_dirs(root, self.regex):
                job_id = os.path.basename(d)
                if self._dirs.get(job_id) == d and self.metadata.get(job_id) is not None \
                        and not self._is_running(job_id):
                    continue
                self.update_caches(d)
                n += 1
        return n

    def _ensure(self, job_id: str) -> bool:
        if self.metadata.get(job_id) is not None and not self._is_running(job_id):
            return True
        d = self._dirs.get(job_id)
        if d is None or not os.path.isdir(d):
            for root in (self.intermediate, self.finished):
                for jd in find_job_dirs(root, self.regex):
                    if os.path.basename(jd) == job_id:
                        d = jd
                        break
                if d is not None and os.path.isdir(d):
                    break
        if d is None or not os.path.isdir(d):
            return False
        self.update_caches(d)
        return self.metadata.get(job_id) is not None

    def _is_running(self, job_id: str) -> bool:
        md = self.metadata.get(job_id)
        return md is not None and md.status == C.RUNNING

    # -- page models -------------------------------------------------------------------------
    def jobs(self) -> List[JobMetadata]:
        """Sorted like JobsMetadataPageController.java:22-31: completed desc, started desc, user."""
        self.warm()
        return sorted(self.metadata.values(), key=lambda m: (-m.completed, -m.started, m.user))

    def job_config(self, job_id: str):
        return self.config.get(job_id) if self._ensure(job_id) else None

    def job_events(self, job_id: str):
        return self.events.get(job_id) if self._ensure(job_id) else None

    def job_logs(self, job_id: str):
        return self.logs.get(job_id) if self._ensure(job_id) else None


_CSS = ("body{font-family:sans-serif;margin:1.5em}table{border-collapse:collapse}"
        "td,th{border:1px solid #ccc;padding:3px 8px;text-align:left}th{background:#eee}")


def _page(title: str, header: List[str], rows: List[List[str]]) -> str:
    th = "".join(f"<th>{html.escape(h)}</th>" for h in header)
    body = "".join("<tr>" + "".join(f"<td>{c}</td>" for c in r) + "</tr>" for r in rows)
    return (f"<!DOCTYPE html><html><head><meta charset='utf-8'><title>{html.escape(title)}</title>"
            f"<style>{_CSS}</style></head><body><h2>{html.escape(title)}</h2>"
            f"<p><a href='/'>all jobs</a></p><table><tr>{th}</tr>{body}</table></body></html>")


def _ms(ts: int) -> str:
    import datetime as _dt

    if ts is None or ts < 0:
        return "-"
    return _dt.datetime.fromtimestamp(ts / 1000, tz=_dt.timezone.utc).strftime("%Y-%m-%d %H:%M:%S UTC")


class _Handler(BaseHTTPRequestHandler):
    cache: CacheWrapper = None  # set on the subclass

    def log_message(self, fmt, *args):
        LOG.debug(fmt, *args)

    def _send(self, code: int, body: str, ctype: str) -> None:
        data = body.encode()
        self.send_response(code)
        self.send_header("Content-Type", ctype)
        self.send_header("Content-Length", str(len(data)))
        self.end_headers()
        self.wfile.write(data)

    def do_GET(self):  # noqa: N802
        u = urlparse(self.path)
        as_json = parse_qs(u.query).get("format", [""])[0] == "json"
        parts = [p for p in u.path.split("/") if p]
        try:
            if not parts:
                return self._jobs(as_json)
            if len(parts) == 2 and parts[0] in (C.JOBS_SUFFIX, C.CONFIG_SUFFIX, C.LOGS_SUFFIX):
                return {C.JOBS_SUFFIX: self._events, C.CONFIG_SUFFIX: self._config,
                        C.LOGS_SUFFIX: self._logs}[parts[0]](parts[1], as_json)
        except Exception as e:  # noqa: BLE001
            LOG.exception("portal error")
            return self._send(500, f"error: {html.escape(str(e))}", "text/plain")
        self._send(404, "not found", "text/plain")

    def _missing(self, job_id: str, as_json: bool):
        if as_json:
            return self._send(404, json.dumps({"error": f"no history for {job_id}"}), "application/json")
        return self._send(404, f"no history for {html.escape(job_id)}", "text/plain")

    def _jobs(self, as_json: bool):
        jobs = self.cache.jobs()
        if as_json:
            return self._send(200, json.dumps([asdict(j) for j in jobs]), "application/json")
        rows = [[f"<a href='{j.job_link}'>{html.escape(j.id)}</a>", f"<a href='{j.config_link}'>config</a>",
                 f"<a href='/{C.LOGS_SUFFIX}/{j.id}'>logs</a>", _ms(j.started), _ms(j.completed),
                 html.escape(j.status), html.escape(j.user)] for j in jobs]
        self._send(200, _page("TonY jobs", ["Job", "Config", "Logs", "Started", "Completed", "Status", "User"],
                              rows), "text/html")

    def _config(self, job_id: str, as_json: bool):
        cfg = self.cache.job_config(job_id)
        if cfg is None:
            return self._missing(job_id, as_json)
        if as_json:
            return self._send(200, json.dumps([asdict(c) for c in cfg]), "application/json")
        rows = [[html.escape(c.name), html.escape(c.value), str(c.final).lower(), html.escape(c.source or "")]
                for c in cfg]
        self._send(200, _page(f"Config of {job_id}", ["Name", "Value", "Final", "Source"], rows), "text/html")

    def _events(self, job_id: str, as_json: bool):
        evs = self.cache.job_events(job_id)
        if evs is None:
            return self._missing(job_id, as_json)
        if as_json:
            return self._send(200, json.dumps([{"type": e.type, "event": e.event, "timestamp": e.timestamp}
                                               for e in evs], default=str), "application/json")
        rows = [[html.escape(e.type), html.escape(json.dumps(e.event, default=str)), e.date] for e in evs]
        self._send(200, _page(f"Events of {job_id}", ["Type", "Event", "Time"], rows), "text/html")

    def _logs(self, job_id: str, as_json: bool):
        logs = self.cache.job_logs(job_id)
        if logs is None:
            return self._missing(job_id, as_json)
        if as_json:
            return self._send(200, json.dumps([asdict(lg) for lg in logs]), "application/json")
        rows = [[html.escape(lg.container_id), html.escape(lg.host),
                 f"<a href='file://{html.escape(lg.log_link)}'>{html.escape(lg.log_link)}</a>"] for lg in logs]
        self._send(200, _page(f"Logs of {job_id}", ["Container", "Host", "Log"], rows), "text/html")


class PortalServer:
    def __init__(self, cache: CacheWrapper, host: str = "127.0.0.1", port: int = 0):
        handler = type("PortalHandler", (_Handler,), {"cache": cache})
        self.cache = cache
        self.httpd = ThreadingHTTPServer((host, port), handler)
        self.port = self.httpd.server_address[1]
        self._thread: Optional[threading.Thread] = None

    def start(self) -> int:
        self._thread = threading.Thread(target=self.httpd.serve_forever, name="tony-portal", daemon=True)
        self._thread.start()
        return self.port

    def serve_forever(self) -> None:
        self.httpd.serve_forever()

    def stop(self) -> None:
        self.httpd.shutdown()
        self.httpd.server_close()

"""Background history writer (behavioural parity with T/events/EventHandler.java:22-157).

Events are queued by the coordinator and appended by one thread to an Avro
container file ``<job dir>/<appId>-<started>-<user>.jhist.inprogress``; ``stop``
drains the queue, closes the file and renames it to the final
``…-<completed>-<user>-<STATUS>.jhist``.  Failures to write never fail the job
(they are logged), as in TonY.
"""
from __future__ import annotations

import logging
import os
import queue
import threading
from typing import Optional

from .avro import DataFileWriter
from .history import JobMetadata, generate_file_name
from .schema import event_schema

LOG = logging.getLogger(__name__)


class EventHandler:
    def __init__(self):
        self._q: "queue.Queue" = queue.Queue()
        self._thread: Optional[threading.Thread] = None
        self._stopped = threading.Event()
        self._writer: Optional[DataFileWriter] = None
        self.in_progress_file: Optional[str] = None
        self.final_file: Optional[str] = None
        self.emitted = 0

    def set_up(self, job_dir: Optional[str], md: JobMetadata) -> bool:
        if job_dir is None:
            return True
        try:
            os.makedirs(job_dir, exist_ok=True)
            self.in_progress_file = os.path.join(job_dir, generate_file_name(md))
            self._writer = DataFileWriter(open(self.in_progress_file, "wb"), event_schema(), sync_interval=1)
        except OSError:
            LOG.exception("Failed to set up history writer")
            self.in_progress_file = None
            return False
        return True

    def start(self) -> None:
        self._thread = threading.Thread(target=self._run, name="tony-event-handler", daemon=True)
        self._thread.start()

    def emit(self, event: dict) -> None:
        LOG.debug("Emitting event: %s", event)
        self._q.put(event)

    def _append(self, ev) -> None:
        try:
            self._writer.append(ev)
            self._writer.flush()
            self.emitted += 1
        except Exception:  # noqa: BLE001
            LOG.exception("Failed to append event %s", ev)

    def _run(self) -> None:
        if self.in_progress_file is None:
            return
        while not self._stopped.is_set():
            try:
                ev = self._q.get(timeout=0.1)
            except queue.Empty:
                continue
            self._append(ev)
        while True:  # drain
            try:
                self._append(self._q.get_nowait())
            except queue.Empty:
                break

    def stop(self, job_dir: Optional[str], md: JobMetadata) -> Optional[str]:
        if self.in_progress_file is None:
            return None
        self._stopped.set()
        if self._thread is not None:
            self._thread.join(timeout=10)
        try:
            self._writer.close()
        except Exception:  # noqa: BLE001
            LOG.exception("Failed to close writer")
        self.final_file = os.path.join(job_dir, generate_file_name(md))
        try:
            os.replace(self.in_progress_file, self.final_file)
        except OSError:
            LOG.exception("Failed to move %s to %s", self.in_progress_file, self.final_file)
        return self.final_file

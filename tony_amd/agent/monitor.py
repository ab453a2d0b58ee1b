"""Task resource monitor (behavioural parity with T/TaskMonitor.java:25-192).

Every ``tony.task.metrics-interval-ms`` it samples the RSS of the task's process
tree (psutil) and, for the GPUs the coordinator pinned to the task (TonY
averages over *all* GPUs of the node), busy %, VRAM-used % and memory-engine
busy % via amd-smi, plus MI355X power / temperature; keeps running max and
average, and pushes them to the coordinator's metrics RPC.  Also the xGMI traffic of the pinned GPUs
(GB/s read / written over all links, from amd-smi's accumulated per-link counters).  GPU sampling stops
after ``MAX_REPEATED_GPU_ERROR_ALLOWED`` consecutive failures.
"""
from __future__ import annotations

import logging
import threading
import time
from typing import Callable, Dict, List, Optional

from .. import constants as C
from .. import native

LOG = logging.getLogger(__name__)


class RunningStat:
    def __init__(self):
        self.max = 0.0
        self.sum = 0.0
        self.n = 0

    def add(self, v: float) -> None:
        self.max = max(self.max, v)
        self.sum += v
        self.n += 1

    @property
    def avg(self) -> float:
        return self.sum / self.n if self.n else 0.0


def tree_rss_bytes(pid: int) -> int:
    try:
        import psutil
    except ImportError:  # pragma: no cover
        return 0
    try:
        p = psutil.Process(pid)
        procs = [p] + p.children(recursive=True)
    except psutil.Error:
        return 0
    total = 0
    for q in procs:
        try:
            total += q.memory_info().rss
        except psutil.Error:
            pass
    return total


class TaskMonitor:
    def __init__(self, pid_fn: Callable[[], Optional[int]], gpu_ids: List[int], interval_ms: int,
                 push: Callable[[Dict[str, float]], None], gpu_metrics: bool = True,
                 on_fault: Optional[Callable[[str], None]] = None, memory_limit_bytes: int = 0):
        self.pid_fn = pid_fn
        self.gpu_ids = gpu_ids
        self.interval_s = max(0.05, interval_ms / 1000.0)
        self.push = push
        self.gpu_metrics = gpu_metrics and bool(gpu_ids)
        self.mem = RunningStat()
        self.util = RunningStat()
        self.fb = RunningStat()
        self.main = RunningStat()
        self.power = RunningStat()
        self.temp = RunningStat()
        self.xgmi_rd = RunningStat()   # GB/s read over the xGMI links of the pinned GPUs (interval deltas)
        self.xgmi_wr = RunningStat()
        self._xgmi_last = None         # (time, read KB, write KB) of the previous sample
        self.ecc_base = None      # uncorrectable ECC count of the pinned GPUs when the task started
        self.ecc_new = 0          # uncorrectable errors raised since (a GPU fault: SURVEY.md §5.3)
        self.gpu_errors = 0
        self.on_fault = on_fault              # called once with a diagnostic on a GPU fault / over-limit memory
        self.memory_limit = int(memory_limit_bytes)
        self.fault: Optional[str] = None
        self._stop = threading.Event()
        self._thread = threading.Thread(target=self._run, name="tony-task-monitor", daemon=True)

    def start(self):
        self._thread.start()

    def stop(self):
        self._stop.set()
        self.refresh()
        self._push()

    def refresh(self) -> None:
        pid = self.pid_fn()
        if pid:
            rss = float(tree_rss_bytes(pid))
            self.mem.add(rss)
            if self.memory_limit and rss > self.memory_limit:
                self._raise_fault(f"memory limit: process tree RSS {rss / 2 ** 20:.0f} MiB > "
                                  f"{self.memory_limit / 2 ** 20:.0f} MiB", C.EXIT_MEMORY_LIMIT)
        if self.gpu_metrics and self.gpu_errors < C.MAX_REPEATED_GPU_ERROR_ALLOWED:
            samples = [native.smi_sample(g) for g in self.gpu_ids]
            samples = [s for s in samples if s is not None]
            if not samples:
                self.gpu_errors += 1
                return
            self.gpu_errors = 0
            n = len(samples)
            self.util.add(sum(s.gfx_busy_pct for s in samples) / n)
            self.fb.add(sum(100.0 * s.vram_used_mb / s.vram_total_mb for s in samples if s.vram_total_mb) / n)
            self.main.add(sum(s.mem_busy_pct for s in samples) / n)
            self.power.add(sum(s.power_w for s in samples))
            self.temp.add(max(s.temp_c for s in samples))
            rd, wr = sum(s.xgmi_read_kb for s in samples), sum(s.xgmi_write_kb for s in samples)
            now = time.monotonic()
            if self._xgmi_last is not None and now > self._xgmi_last[0] and rd >= self._xgmi_last[1]:
                dt = now - self._xgmi_last[0]
                self.xgmi_rd.add((rd - self._xgmi_last[1]) / dt / 1e6)   # KB/s -> GB/s
                self.xgmi_wr.add((wr - self._xgmi_last[2]) / dt / 1e6)
            self._xgmi_last = (now, rd, wr)
            ecc = sum(s.ecc_uncorrectable for s in samples)
            if self.ecc_base is None:
                self.ecc_base = ecc
            elif ecc > self.ecc_base + self.ecc_new:
                LOG.error("GPU(s) %s raised %d new uncorrectable ECC error(s)", self.gpu_ids,
                          ecc - self.ecc_base - self.ecc_new)
                self.ecc_new = ecc - self.ecc_base
                self._raise_fault(f"GPU fault: {self.ecc_new} uncorrectable ECC error(s) on GPU(s) {self.gpu_ids}",
                                  C.EXIT_GPU_FAULT)

    def _raise_fault(self, message: str, code: int) -> None:
        """First fault wins: record it and let the agent stop the task."""
        if self.fault is not None:
            return
        self.fault = message
        self.fault_code = code
        LOG.error("%s", message)
        if self.on_fault is not None:
            try:
                self.on_fault(message)
            except Exception:  # noqa: BLE001
                LOG.exception("fault handler failed")

    def metrics(self) -> Dict[str, float]:
        m = {C.MAX_MEMORY_BYTES: self.mem.max, C.AVG_MEMORY_BYTES: self.mem.avg}
        if self.gpu_metrics:
            m.update({C.MAX_GPU_UTILIZATION: self.util.max, C.AVG_GPU_UTILIZATION: self.util.avg,
                      C.MAX_GPU_FB_MEMORY_USAGE: self.fb.max, C.AVG_GPU_FB_MEMORY_USAGE: self.fb.avg,
                      C.MAX_GPU_MAIN_MEMORY_USAGE: self.main.max, C.AVG_GPU_MAIN_MEMORY_USAGE: self.main.avg,
                      C.MAX_GPU_POWER_WATTS: self.power.max, C.AVG_GPU_POWER_WATTS: self.power.avg,
                      C.MAX_GPU_TEMPERATURE: self.temp.max, C.GPU_ECC_UNCORRECTABLE: float(self.ecc_new),
                      C.MAX_XGMI_READ_GBPS: self.xgmi_rd.max, C.AVG_XGMI_READ_GBPS: self.xgmi_rd.avg,
                      C.MAX_XGMI_WRITE_GBPS: self.xgmi_wr.max, C.AVG_XGMI_WRITE_GBPS: self.xgmi_wr.avg})
        return m

    def _push(self):
        try:
            self.push(self.metrics())
        except Exception:  # noqa: BLE001
            LOG.debug("metrics push failed", exc_info=True)

    def _run(self):
        while not self._stop.wait(self.interval_s):
            self.refresh()
            self._push()

"""Native replay of a captured training step (csrc/plan.hip).

A step is captured once with ``torch.cuda.graph`` into a hipGraph that is never instantiated
(``CUDAGraph(keep_graph=True)``); :class:`StepPlan` walks it in C++ and re-issues its kernels,
memsets and copies onto the compute stream and the side / branch streams the eager step uses, with
event edges only where the captured dependencies cross streams.  One fast call per replay instead of
~600 Python-issued launches (eager) or one ``hipGraphLaunch`` that costs as much host time and runs
slower on the GPU (see the header of csrc/plan.hip for the measurements that motivated it).

Memory and arguments: the kernels' argument blocks live in the graph's nodes and the tensors they
point at in the capture's private memory pool, so the plan holds the ``CUDAGraph`` object for its
whole life -- exactly the lifetime rule of a replayed ``torch.cuda.CUDAGraph``.

Segments: ``mark(i)`` captured inside the step (``tony_plan_mark``) splits the plan; ``replay(seg,
side)`` issues one segment and forks the marker's stream into ``side`` so host-issued work (a
gradient bucket's RCCL collective, which stays outside the graph) can follow it.

Reference parity: TonY hands step execution to the framework's runtime; this is the
MI355X-native runtime piece that replaces a tracing compiler's launch path.
"""
from __future__ import annotations

import ctypes
from typing import Dict, List, Optional, Sequence

import torch

from . import _lib

STAT_KEYS = ("kernels", "memsets", "memcpys", "waits", "records", "streams_used", "markers", "graph_nodes",
             "false_deps", "empty_nodes", "node_graphs")


class PlanUnsupported(RuntimeError):
    """The captured graph holds a node kind the native replay does not issue (host, child graph...)."""


class StepPlan:
    def __init__(self, graph: torch.cuda.CUDAGraph, streams: Sequence[torch.cuda.Stream]):
        if not 1 <= len(streams) <= 8:
            raise ValueError("a plan uses 1..8 streams (the first is the one replay() is issued on)")
        handles = [s.cuda_stream for s in streams]
        if len(set(handles)) != len(handles):
            raise ValueError("plan streams must be distinct")
        L = _lib.lib()
        arr = (ctypes.c_uint64 * len(handles))(*handles)
        stats = (ctypes.c_int * len(STAT_KEYS))()
        out = ctypes.c_uint64(0)
        rc = L.tony_plan_build(graph.raw_cuda_graph(), arr, len(handles), ctypes.byref(out), stats)
        if rc < 0:
            raise PlanUnsupported(f"tony_plan_build: {rc}")
        _lib.check(rc, "tony_plan_build")
        self.graph = graph  # node argument blocks + the capture pool stay alive with the plan
        self.streams = list(streams)
        self.handle = out.value
        self.stats: Dict[str, int] = dict(zip(STAT_KEYS, stats))
        self.segments = L.tony_plan_segments(self.handle)
        self._replay = L.tony_plan_replay

    def replay(self, seg: int = -1, side: Optional[torch.cuda.Stream] = None) -> None:
        """Issue segment ``seg`` (every segment when < 0) on the plan's streams; the caller's current
        stream must be ``streams[0]``."""
        rc = self._replay(self.handle, seg, None if side is None else side.cuda_stream)
        if rc:
            f = (ctypes.c_int * 3)()
            _lib.lib().tony_plan_failure(self.handle, f)
            kinds = ("kernel", "memset", "memcpy", "wait", "record", "marker", "one-node graph")
            kind = kinds[f[1]] if 0 <= f[1] < len(kinds) else str(f[1])
            _lib.check(rc, f"tony_plan_replay (segment {seg}: op {f[0]} of {len(self.ops())}, a {kind} on plan "
                           f"stream {f[2]})")

    def ops(self) -> List[tuple]:
        """(kind, stream, event-or-marker) per issued op: kinds 0 kernel, 1 memset, 2 memcpy, 3 wait,
        4 record, 5 marker, 6 one-node graph (tests / tracing)."""
        L = _lib.lib()
        n = L.tony_plan_ops(self.handle, None, 0)
        buf = (ctypes.c_int * (3 * max(n, 1)))()
        L.tony_plan_ops(self.handle, buf, n)
        return [tuple(buf[3 * i:3 * i + 3]) for i in range(n)]

    def close(self) -> None:
        if self.handle:
            _lib.lib().tony_plan_destroy(self.handle)
            self.handle = 0

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001 - interpreter teardown
            pass


def mark(i: int, stream: Optional[torch.cuda.Stream] = None) -> None:
    """Capture a segment boundary on ``stream`` (default: the current stream)."""
    s = stream if stream is not None else torch.cuda.current_stream()
    _lib.check(_lib.lib().tony_plan_mark(int(i), s.cuda_stream), "tony_plan_mark")

"""Step-phase tracing and hang diagnostics.

* ``trace_range(name)`` pushes a roctx range (``torch.cuda.nvtx`` is roctx on ROCm builds) around
  a phase of the step -- forward, backward, PS push/apply/pull, bucket i -- when ``TONY_TRACE=1``;
  ``rocprofv3 --marker-trace`` (or the ``tony.amd.profile`` task wrapper with marker tracing)
  then shows the phases on the kernel timeline.  Off, it costs one dict lookup.
* ``hang_watchdog(seconds)`` makes a gang hang visible: every ``seconds`` without a
  ``heartbeat()`` call, all Python thread stacks are dumped to stderr (faulthandler), so the
  task log shows which collective / barrier each rank is blocked in.  Enabled for every
  process group formed through tony_amd.parallel.bootstrap when ``TONY_HANG_DUMP_S`` is set.
"""
from __future__ import annotations

import contextlib
import faulthandler
import os
import sys

_ENABLED = os.environ.get("TONY_TRACE", "0") == "1"
_WATCHDOG_S = [0.0]


def enabled() -> bool:
    return _ENABLED


def set_enabled(on: bool) -> None:
    global _ENABLED
    _ENABLED = bool(on)


@contextlib.contextmanager
def trace_range(name: str):
    if not _ENABLED:
        yield
        return
    import torch

    pushed = False
    try:
        if torch.cuda.is_available() and not torch.cuda.is_current_stream_capturing():
            torch.cuda.nvtx.range_push(name)
            pushed = True
    except Exception:  # noqa: BLE001 - tracing must never break a step
        pushed = False
    try:
        yield
    finally:
        if pushed:
            torch.cuda.nvtx.range_pop()


def hang_watchdog(seconds: float, file=None) -> None:
    """(Re)arm the stack-dump watchdog; ``seconds <= 0`` disarms it."""
    faulthandler.cancel_dump_traceback_later()
    _WATCHDOG_S[0] = float(seconds)
    if seconds > 0:
        faulthandler.dump_traceback_later(seconds, repeat=True, file=file or sys.stderr)


def heartbeat() -> None:
    """Progress was made: push the next dump ``seconds`` into the future."""
    if _WATCHDOG_S[0] > 0:
        faulthandler.cancel_dump_traceback_later()
        faulthandler.dump_traceback_later(_WATCHDOG_S[0], repeat=True, file=sys.stderr)


def arm_from_env() -> None:
    s = os.environ.get("TONY_HANG_DUMP_S")
    if s:
        try:
            hang_watchdog(float(s))
        except ValueError:
            pass

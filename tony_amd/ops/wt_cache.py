"""Per-step transposed conv weights for the backward-data GEMMs, refreshed in ONE batched launch.

Every dgrad (implicit-GEMM conv dgrad, and the 1x1 / fused-head backward GEMMs) reads the weight
as [Ci][R][S][Co].  Transposing inside each backward costs one small torch copy kernel per conv
(≈70 per Inception-v3 step, ≈6 µs each).  Weights only change at the optimizer step, so while a
``Trainer`` runs, the convs look their transposed copy up here and the trainer refreshes ALL of
them with one ``tony_transpose_batch`` launch right after the PS apply/pull (csrc/transpose.hip).

A weight seen for the first time (an eager warm-up step) gets a fresh copy made on the spot and
joins the batch.  Outside a trainer (``enabled`` False: tests, inference, other optimizers) the
lookup returns None and callers transpose on the fly, so no stale copy is ever read.
"""
from __future__ import annotations

import struct
from typing import Dict, Optional

import torch

from . import _lib

_DESC = struct.Struct("<QQiiiiii")  # csrc/transpose.hip TDesc
_T = 64


def _crsk(weight: torch.Tensor) -> torch.Tensor:
    return weight.permute(1, 2, 3, 0).contiguous()


class TransposedWeights:
    def __init__(self, device):
        self.device = _norm(device)
        if _lib.lib().tony_transpose_desc_bytes() != _DESC.size:
            raise _lib.KernelError("transpose descriptor layout differs between Python and the kernels")
        self.entries: Dict[int, tuple] = {}
        self.enabled = False
        self.frozen = False  # set once a HIP graph captured refresh(): the work list must not change
        self.desc: Optional[torch.Tensor] = None
        self.n_desc = 0
        self.total_tiles = 0

    def get(self, weight: torch.Tensor) -> Optional[torch.Tensor]:
        """[Ci, R, S, Co]-contiguous copy of ``weight`` valid for the current step, or None."""
        if not self.enabled or not isinstance(weight, torch.nn.Parameter) or weight.dim() != 4:
            return None
        e = self.entries.get(id(weight))
        if e is not None and e[0] is weight and e[2] == weight.data_ptr():
            return e[1]
        if self.frozen or torch.cuda.is_current_stream_capturing():
            return None  # registration (a host->device descriptor upload) happens in eager steps only
        co, ci, r, s = weight.shape
        if not weight.is_contiguous(memory_format=torch.channels_last) or weight.dtype != torch.bfloat16:
            return None
        buf = _crsk(weight)
        self.entries[id(weight)] = (weight, buf, weight.data_ptr())
        self._build()
        return buf

    def _build(self):
        parts, tiles = [], 0
        for w, buf, _ in self.entries.values():
            co, ci, r, s = w.shape
            tci, tco = (ci + _T - 1) // _T, (co + _T - 1) // _T
            parts.append(_DESC.pack(w.data_ptr(), buf.data_ptr(), co, r * s, ci, tci, tco, tiles))
            tiles += r * s * tci * tco
        raw = torch.frombuffer(bytearray(b"".join(parts)), dtype=torch.uint8)
        self.desc = raw.to(self.device)
        self.n_desc = len(parts)
        self.total_tiles = tiles

    def refresh(self) -> None:
        """Re-transpose every registered weight (call after each optimizer step)."""
        if not self.n_desc:
            return
        L = _lib.lib()
        rc = L.tony_transpose_batch(self.desc.data_ptr(), self.n_desc, self.total_tiles,
                                    _lib.stream_ptr(self.device))
        _lib.check(rc, "tony_transpose_batch")


_ACTIVE: list = [None]


def _norm(device) -> torch.device:
    d = torch.device(device)
    if d.type == "cuda" and d.index is None:
        d = torch.device("cuda", torch.cuda.current_device())
    return d


def activate(cache: Optional[TransposedWeights]) -> None:
    """Make ``cache`` the one the conv backward passes consult (None: transpose on the fly)."""
    _ACTIVE[0] = cache


def transposed(weight: torch.Tensor) -> torch.Tensor:
    """weight [Co, Ci, R, S] as a [Ci][R][S][Co]-contiguous tensor (cached copy when a trainer runs)."""
    c = _ACTIVE[0]
    if c is not None and c.enabled and c.device == _norm(weight.device):
        t = c.get(weight)
        if t is not None:
            return t
    return _crsk(weight)

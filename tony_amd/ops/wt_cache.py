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


_XDESC = struct.Struct("<QQQiiiiiiii")  # csrc/x3.hip XDesc


class X3Weights:
    """The fp32 model's x3 weight planes (ops/x3.py), both layouts, for the current step: the forward
    planes [Co][R][S][3cp] and the backward-data planes [C][R][S][3Co] of every conv weight, refreshed
    by ONE ``tony_x3_weights_batch`` launch right after the optimizer step instead of a split launch per
    conv and pass on the critical path.  Same protocol as TransposedWeights: a weight seen for the first
    time in an eager step is split on the spot and joins the batch; None outside a trainer."""

    def __init__(self, device):
        self.device = _norm(device)
        if _lib.lib().tony_x3_desc_bytes() != _XDESC.size:
            raise _lib.KernelError("x3 weight descriptor layout differs between Python and the kernels")
        self.entries: Dict[int, tuple] = {}
        self.enabled = False
        self.frozen = False
        self.desc: Optional[torch.Tensor] = None
        self.n_desc = 0
        self.total_tiles = 0

    def _entry(self, weight: torch.Tensor):
        if not self.enabled or not isinstance(weight, torch.nn.Parameter) or weight.dim() != 4:
            return None
        e = self.entries.get(id(weight))
        if e is not None and e[0] is weight and e[3] == weight.data_ptr():
            return e
        if self.frozen or torch.cuda.is_current_stream_capturing():
            return None
        co, c, r, s = weight.shape
        if weight.dtype != torch.float32 or co % 8 or not weight.is_contiguous(memory_format=torch.channels_last):
            return None
        from . import x3

        fwd = x3.split_weight(weight)        # [Co * R * S, 3cp]
        bwd = x3.split_weight_t(weight)      # [C, R, S, 3Co]
        e = (weight, fwd, bwd, weight.data_ptr())
        self.entries[id(weight)] = e
        self._build()
        return e

    def planes(self, weight: torch.Tensor) -> Optional[torch.Tensor]:
        e = self._entry(weight)
        return None if e is None else e[1]

    def planes_t(self, weight: torch.Tensor) -> Optional[torch.Tensor]:
        e = self._entry(weight)
        return None if e is None else e[2]

    def _build(self):
        parts, tiles = [], 0
        for w, fwd, bwd, _ in self.entries.values():
            co, c, r, s = w.shape
            cp = (c + 7) // 8 * 8
            tc, tco = (cp + _T - 1) // _T, (co + _T - 1) // _T
            parts.append(_XDESC.pack(w.data_ptr(), fwd.data_ptr(), bwd.data_ptr(), co, r * s, c, cp, tc, tco, tiles, 0))
            tiles += r * s * tc * tco
        raw = torch.frombuffer(bytearray(b"".join(parts)), dtype=torch.uint8)
        self.desc = raw.to(self.device)
        self.n_desc = len(parts)
        self.total_tiles = tiles

    def refresh(self) -> None:
        """Re-split every registered weight (call after each optimizer step)."""
        if not self.n_desc:
            return
        rc = _lib.lib().tony_x3_weights_batch(self.desc.data_ptr(), self.n_desc, self.total_tiles,
                                              _lib.stream_ptr(self.device))
        _lib.check(rc, "tony_x3_weights_batch")


_ACTIVE: list = [None]
_ACTIVE_X3: list = [None]


def _norm(device) -> torch.device:
    d = torch.device(device)
    if d.type == "cuda" and d.index is None:
        d = torch.device("cuda", torch.cuda.current_device())
    return d


def activate(cache: Optional[TransposedWeights], x3cache: Optional[X3Weights] = None) -> None:
    """Make ``cache`` the one the conv backward passes consult (None: transpose on the fly), and
    ``x3cache`` the fp32 model's weight planes (None: split on the fly)."""
    _ACTIVE[0] = cache
    _ACTIVE_X3[0] = x3cache


def x3_planes(weight: torch.Tensor) -> Optional[torch.Tensor]:
    """The forward x3 planes of ``weight`` for this step (None: no trainer cache, split on the fly)."""
    c = _ACTIVE_X3[0]
    if c is not None and c.enabled and c.device == _norm(weight.device):
        return c.planes(weight)
    return None


def x3_planes_t(weight: torch.Tensor) -> Optional[torch.Tensor]:
    """The backward-data x3 planes of ``weight`` for this step (None: split on the fly)."""
    c = _ACTIVE_X3[0]
    if c is not None and c.enabled and c.device == _norm(weight.device):
        return c.planes_t(weight)
    return None


def transposed(weight: torch.Tensor) -> torch.Tensor:
    """weight [Co, Ci, R, S] as a [Ci][R][S][Co]-contiguous tensor (cached copy when a trainer runs)."""
    c = _ACTIVE[0]
    if c is not None and c.enabled and c.device == _norm(weight.device):
        t = c.get(weight)
        if t is not None:
            return t
    return _crsk(weight)

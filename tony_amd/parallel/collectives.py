"""Collective helpers over torch.distributed (RCCL over xGMI on the GPU, gloo on CPU).

On MI355X every rank is one process pinned to one GPU and the ``nccl`` backend
IS RCCL, which runs its rings/trees over the fully-connected 8-GPU xGMI mesh.
The helpers pick the flat, single-launch collective when the backend has it
(``reduce_scatter_tensor`` / ``all_gather_into_tensor``) and emulate it with the
generic ops on gloo, so the same parameter-server / data-parallel code is
exercised by the multi-process CPU tests.
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist

# TONY_COLLECTIVE=hip (conf tony.amd.collective, exported by the coordinator; bench.py
# --collective hip) routes the flat GPU collectives of the default group through tony_amd's xGMI
# peer-memory kernels (xgmi.py), whatever the process group's backend (a gloo group only carries
# the IPC-handle exchange: the one-GPU multi-process rehearsal of that path)
_XGMI = [None]


_FALLBACKS = [0]


def use_hip() -> bool:
    """TONY_COLLECTIVE asks for tony_amd's xGMI peer-memory kernels instead of RCCL."""
    return os.environ.get("TONY_COLLECTIVE", "rccl").lower() in ("hip", "xgmi")


def fallback_count() -> int:
    """Collectives that TONY_COLLECTIVE=xgmi asked for but that ran on RCCL (dtype / size / group)."""
    return _FALLBACKS[0]


def _xgmi(t: torch.Tensor, group):
    """The XgmiComm to use for tensor t, or None for the torch.distributed (RCCL / gloo) path."""
    if os.environ.get("TONY_COLLECTIVE", "rccl").lower() not in ("hip", "xgmi") or not t.is_cuda:
        return None
    if group is not None or t.dtype not in (torch.bfloat16, torch.float32) or (t.numel() * t.element_size()) % 16:
        _FALLBACKS[0] += 1
        return None
    if _XGMI[0] is None:
        from .xgmi import XgmiComm, XgmiError

        try:
            _XGMI[0] = XgmiComm()  # checks itself against the process group's all-reduce first
            _STATUS["xgmi_collectives"] = "verified"
        except XgmiError as e:  # every rank raises together: every rank falls back together
            import warnings

            warnings.warn(f"TONY_COLLECTIVE=xgmi: {e}; the collectives fall back to {dist.get_backend()}",
                          RuntimeWarning)
            _STATUS["xgmi_collectives"] = f"failed: {e}"
            _XGMI[0] = False
    if _XGMI[0] is False:
        _FALLBACKS[0] += 1
        return None
    return _XGMI[0]


# first-use verification of the hand data planes (bench.py records it): None = not used
_STATUS = {"xgmi_collectives": None, "ps_plane": None}


def data_plane_status() -> dict:
    return dict(_STATUS)


def world(group=None) -> int:
    return dist.get_world_size(group) if dist.is_available() and dist.is_initialized() else 1


def rank(group=None) -> int:
    return dist.get_rank(group) if dist.is_available() and dist.is_initialized() else 0


def _is_gloo(group=None) -> bool:
    return dist.get_backend(group) == "gloo"


def reduce_scatter_flat(out: torch.Tensor, inp: torch.Tensor, group=None, async_op=False):
    """out (= inp.numel()/world elements) <- sum over ranks of this rank's slice of inp."""
    if world(group) == 1:
        if out.data_ptr() != inp.data_ptr():
            out.copy_(inp)
        return None
    x = _xgmi(inp, group)  # before the gloo emulation: a gloo group can carry the xGMI handshake
    if x is not None:
        x.reduce_scatter(out, inp)
        return None
    if _is_gloo(group):
        dist.all_reduce(inp, group=group)
        r = rank(group)
        n = out.numel()
        out.copy_(inp[r * n:(r + 1) * n])
        return None
    return dist.reduce_scatter_tensor(out, inp, group=group, async_op=async_op)


def all_gather_flat(out: torch.Tensor, inp: torch.Tensor, group=None, async_op=False):
    """out (world * inp.numel()) <- concat over ranks of inp."""
    if world(group) == 1:
        if out.data_ptr() != inp.data_ptr():
            out.copy_(inp)
        return None
    x = _xgmi(inp, group)
    if x is not None:
        x.all_gather(out, inp)
        return None
    if _is_gloo(group):
        n = inp.numel()
        parts = [out[i * n:(i + 1) * n] for i in range(world(group))]
        src = inp.clone() if any(p.data_ptr() == inp.data_ptr() for p in parts) else inp
        dist.all_gather(parts, src, group=group)
        return None
    return dist.all_gather_into_tensor(out, inp, group=group, async_op=async_op)


def all_reduce(t: torch.Tensor, op=None, group=None, async_op=False, average: bool = False):
    """Sum (``average``: mean) of ``t`` over the ranks, in place.  TONY_COLLECTIVE=hip runs it on the
    xGMI kernels (one launch; the average is a scale inside the reduction), else RCCL (AVG op) / gloo
    (SUM, then a scale)."""
    if world(group) == 1:
        return None
    x = _xgmi(t, group) if op in (None, dist.ReduceOp.SUM) else None
    if x is not None and t.is_contiguous():
        x.all_reduce(t, average=average)
        return None
    if average:
        if op not in (None, dist.ReduceOp.SUM):
            raise ValueError("average=True is a SUM scaled by 1/world")
        if not _is_gloo(group):
            return dist.all_reduce(t, op=dist.ReduceOp.AVG, group=group, async_op=async_op)
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
        t.mul_(1.0 / world(group))
        return None
    return dist.all_reduce(t, op=op or dist.ReduceOp.SUM, group=group, async_op=async_op)


def broadcast(t: torch.Tensor, src: int, group=None, async_op=False):
    if world(group) == 1:
        return None
    x = _xgmi(t, group)
    if x is not None and t.is_contiguous():
        x.broadcast(t, src)
        return None
    return dist.broadcast(t, src, group=group, async_op=async_op)


def max_over_ranks(v: float, device=None) -> float:
    if world() == 1:
        return float(v)
    t = torch.tensor([float(v)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())

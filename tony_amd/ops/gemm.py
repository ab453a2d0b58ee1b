"""MFMA bf16 GEMM (csrc/gemm.hip) and the NHWC 1x1 convolution built on it.

A stride-1, unpadded 1x1 convolution on a channels_last tensor is exactly a GEMM
over rows: Y[NHW, Cout] = X[NHW, Cin] . W[Cout, Cin]^T.  Forward and the
backward-data GEMM run on the hand-written MFMA kernel; the weight gradient
(a reduction over all NHW rows into a tiny Cout x Cin matrix) runs on the
split-K MFMA kernel that reads its operands with ds_read_b64_tr_b16
(``tony_gemm_tn_bf16``).
"""
from __future__ import annotations

import ctypes
import os

import torch

from . import _lib, tape, tune
from .arena import zeros_f32
from .bn import _as_rows, _rows_view


def gemm_nt(a: torch.Tensor, b: torch.Tensor, out: torch.Tensor | None = None, stats: torch.Tensor | None = None,
            vflags: int = 0):
    """out[M,N] = a[M,K] @ b[N,K]^T for bf16 CUDA 2-D tensors with unit inner stride (``vflags``: tile
    variant bits, ops/tune.py; 0 = the built-in heuristic)."""
    if not (a.is_cuda and b.is_cuda) or a.dtype != torch.bfloat16 or b.dtype != torch.bfloat16:
        raise TypeError("gemm_nt takes bf16 CUDA tensors")
    if a.stride(1) != 1:
        a = a.contiguous()
    if b.stride(1) != 1:
        b = b.contiguous()
    M, K = a.shape
    N, K2 = b.shape
    if K != K2:
        raise ValueError(f"inner dims differ: {a.shape} x {b.shape}^T")
    if out is None:
        out = torch.empty((M, N), dtype=torch.bfloat16, device=a.device)
    if stats is not None:
        stats.zero_()  # the epilogue accumulates into it
    rc = _lib.lib().tony_gemm_bf16(a.data_ptr(), b.data_ptr(), out.data_ptr(), M, N, K, a.stride(0) if M > 1 else K,
                                   b.stride(0) if N > 1 else K, out.stride(0) if M > 1 else N,
                                   (1 if stats is not None else 0) | vflags, _lib.ptr(stats), 0,
                                   _lib.stream_ptr(a.device))
    _lib.check(rc, "tony_gemm_bf16")
    return out


def _gemm_rows(a_ptr, lda, b, M, N, K, out_ptr, ldc, device):
    rc = _lib.lib().tony_gemm_bf16(a_ptr, b.data_ptr(), out_ptr, M, N, K, lda, b.stride(0), ldc, 0, 0, 0,
                                   _lib.stream_ptr(device))
    _lib.check(rc, "tony_gemm_bf16")


# The split-K wgrad kernels size their grid as 2 workgroups per "CU" they are told about; telling
# them occ x the real CU count keeps more splits in flight per CU (bigger slab, more latency hiding,
# more combine traffic).  The best occ depends on the shape (tools/conv_bench.py --tony: 4 beats 1
# on the 147x147 stem, changes nothing at 17x17), so it is autotuned per shape (ops/tune.py).
# In the training step the wgrads run on a side stream beside the BN passes, and more splits also
# mean more fp32 partials through HBM (~1 GB of slab per step at the tuned 2-4x): restricting the
# search to occ = 1 measured 14.43 / 14.47 vs 14.55 / 14.62 ms of GPU time per step
# (profiles/r2s3_wgrad_occ_ab.log).  TONY_WGRAD_OCC=1,2,4,8 restores the isolated-speed search.
# Fractions (TONY_WGRAD_OCC=0.5) plan fewer workgroups than CUs: fewer splits, less slab traffic for the
# combine, fewer CUs taken from the data-gradient chain the wgrads overlap with.
# Default 0.5 (one workgroup per CU instead of two): 14.16 / 14.34 vs 14.40 / 14.38 ms/step mean over
# two A/Bs of three repetitions, GPU-ahead time 14.24 vs 14.41 (profiles/r5_ab_wgrad_occ.log).
WGRAD_OCC = tuple((float(o) if "." in o else int(o)) for o in os.environ.get("TONY_WGRAD_OCC", "0.5").split(","))
# TONY_WGRAD_OCC_BIG: the plan for wgrads over >= TONY_WGRAD_BIG_ROWS rows (the stem layers, whose
# wgrads close the backward pass with little left to overlap them); empty: TONY_WGRAD_OCC.  Default 2
# above 600 K rows (Inception's 147x147 / 73x73 stem): 14.04 vs 14.13 ms/step over 4 repetitions; at
# 400 K rows it also took ResNet-50's mid-network 56x56 layers and cost 0.45 % there
# (profiles/r5_ab_wgrad_occ.log)
def _occ_list(v: str):
    return tuple((float(o) if "." in o else int(o)) for o in v.split(",") if o)


WGRAD_OCC_BIG = _occ_list(os.environ.get("TONY_WGRAD_OCC_BIG", "2"))
WGRAD_BIG_ROWS = int(os.environ.get("TONY_WGRAD_BIG_ROWS", "600000"))


def occ_choices(rows: int):
    """The split plans (workgroups per CU) a weight gradient over ``rows`` reduction rows may use."""
    return WGRAD_OCC_BIG if WGRAD_OCC_BIG and rows >= WGRAD_BIG_ROWS else WGRAD_OCC


# the x3 (fp32) weight gradients' plan (ops/x3.py conv_wgrad); 0.5 (one workgroup per two CUs, fewer slab
# partials): 31.14 vs 31.36 ms per fp32 step over 3 repetitions with the weight-gradient batch of 4
# (profiles/r6_ab_fp32_wb4.log)
X3_WGRAD_OCC = float(os.environ.get("TONY_X3_WGRAD_OCC", "0.5"))
# 2 on the stem-size layers: 32.32 vs 32.42 ms per fp32 step (profiles/r5_ab_wgrad_occ.log); 0: X3_WGRAD_OCC
X3_WGRAD_OCC_BIG = float(os.environ.get("TONY_X3_WGRAD_OCC_BIG", "2") or 0)


def x3_occ(rows: int) -> float:
    """The split plan of an x3 weight gradient over ``rows`` reduction rows."""
    return X3_WGRAD_OCC_BIG if X3_WGRAD_OCC_BIG > 0 and rows >= WGRAD_BIG_ROWS else X3_WGRAD_OCC


def wgrad_cus(device, occ: float = 1) -> int:
    return max(1, int(round(_lib.num_cus(device) * occ)))


# TONY_SPLITK_FOLD=1: the last workgroup of each dW tile sums the split partials inside the wgrad
# kernel (mfma_common.h splitk_fold_tile) instead of a separate combine launch.  Off by default:
# measured on MI355X it serialises each tile's ~100-split reduction on ONE workgroup -- the Inception
# wgrads went from 74 to 404 us (profiles/r2_rejected_splitk_fold_bn_onepass_prof.md).
SPLITK_FOLD = os.environ.get("TONY_SPLITK_FOLD", "0") == "1"
# TONY_SPLITK_TREE=1: the splits of each dW tile meet pairwise inside the wgrad launch
# (mfma_common.h splitk_tree_fold: a binary tree over the split index, each workgroup reads at most
# one partner's partial per level) -- no tony_splitk_reduce launch.  Off by default: measured on
# MI355X every level is a 64 KB read-add-write by ONE workgroup (~100-200 GB/s per CU) behind a
# ticket, so the 5-9 levels add 25-45 us to each wgrad where the chip-wide combine takes ~8 us:
# Inception conv time 11.47 -> 14.58 ms/step, step 14.22 -> 15.03 ms (profiles/r5_rejected_splitk_tree.log)
SPLITK_TREE = os.environ.get("TONY_SPLITK_TREE", "0") == "1"


def splitk_combine(launch, n: int, ntiles: int, device, dst: torch.Tensor | None = None, occ: int = 1,
                   pairs: int = 1):
    """Run a split-K weight-gradient kernel in slab mode and sum its splits.

    ``launch(slab_ptr, slab_cap, splits_ref, fold_counters, fold_dst, fold_flags)`` launches the
    kernel; its M splits store dense partials of the ``n``-float result into the slab and, with
    fold counters, the last split of every tile sums them into ``fold_dst`` in the same launch
    (else csrc/splitk.hip's combine kernel does).  The sum is ADDED into ``dst`` (a bf16 or fp32
    flat-gradient slot in the kernel's element order) and None returned, or returned as a new
    fp32 tensor of n floats.  The split count never exceeds ceil(2 * CUs / ntiles) (the kernels'
    2-workgroups-per-CU plan), which bounds the slab; ``pairs``: plane pairs of an x3 launch
    (csrc/conv.hip tony_conv_wgrad_x3), each with its own splits of that plan divided by ``pairs``."""
    cus = wgrad_cus(device, occ)
    bound = pairs * max(1, -(-2 * cus // (pairs * ntiles)))
    tree = SPLITK_TREE and pairs == 1
    # the tree's workspace: a 128 x 128 fp32 slot per workgroup; the kernel's grid is at most
    # 2 * cus + its tile count (its tiles may be 4x narrower than the 128-row ntiles the caller counts)
    wgs = 2 * cus + 4 * ntiles + 8
    slab = torch.empty(max(bound * n, wgs * 128 * 128) if tree else bound * n, dtype=torch.float32, device=device)
    splits = ctypes.c_int(0)
    out = dst if dst is not None else torch.empty(n, dtype=torch.float32, device=device)
    flags = int(out.dtype == torch.bfloat16) | (2 if dst is not None else 0)
    if tree:
        counters = zeros_f32(4 * wgs, device)  # 4 words per workgroup
        rc = launch(slab.data_ptr(), slab.numel(), ctypes.addressof(splits), counters.data_ptr(), out.data_ptr(),
                    flags | 4)
        if rc == 0:
            return None if dst is not None else out
        if rc != -3:  # -3: no tree for this launch (x3 plane pairs, 2 GB slab): the combine below
            _lib.check(rc, "split-K wgrad (tree)")
    if SPLITK_FOLD and pairs == 1:
        counters = zeros_f32(ntiles, device)  # zero bits = zero uint32 arrival counters
        _lib.check(launch(slab.data_ptr(), slab.numel(), ctypes.addressof(splits), counters.data_ptr(), out.data_ptr(),
                          flags), "split-K wgrad (fold)")
        return None if dst is not None else out
    _lib.check(launch(slab.data_ptr(), slab.numel(), ctypes.addressof(splits), 0, 0, 0), "split-K wgrad")
    rc = _lib.lib().tony_splitk_reduce(slab.data_ptr(), splits.value, n, out.data_ptr(), int(out.dtype == torch.bfloat16),
                                       int(dst is not None), cus, _lib.stream_ptr(device))
    _lib.check(rc, "tony_splitk_reduce")
    return None if dst is not None else out


def wgrad_tn(a_ptr, lda, b_ptr, ldb, M, n1, n2, device, dst: torch.Tensor | None = None):
    """fp32 [n1, n2] = A^T B for row-major A [M, n1], B [M, n2] (split-K MFMA kernel), or, with
    ``dst`` (a contiguous [n1, n2]-ordered gradient slot), that product added into dst (returns None)."""
    L = _lib.lib()
    stream = _lib.stream_ptr(device)
    ntiles = -(-n1 // 128) * -(-n2 // 128)

    def run(occ, dst_=None):
        return splitk_combine(lambda slab, cap, sp, fc, fd, ff: L.tony_gemm_tn_bf16(
            a_ptr, b_ptr, 0, M, n1, n2, lda, ldb, n2, slab, cap, sp, wgrad_cus(device, occ), fc, fd, ff, stream),
                              n1 * n2, ntiles, device, dst_, occ)

    occ = tune.pick_choice(("wgrad_tn", M, n1, n2, lda, ldb), occ_choices(M), run)
    out = run(occ, dst)
    return None if out is None else out.view(n1, n2)


def gemm_tn(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """fp32 a^T @ b for bf16 CUDA a [M, n1], b [M, n2] with unit inner stride."""
    if a.stride(1) != 1:
        a = a.contiguous()
    if b.stride(1) != 1:
        b = b.contiguous()
    return wgrad_tn(a.data_ptr(), a.stride(0), b.data_ptr(), b.stride(0), a.shape[0], a.shape[1], b.shape[1],
                    a.device)


class _Conv1x1Fn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight):
        cout, cin = weight.shape[0], weight.shape[1]
        x, (M, C, ldx) = _as_rows(x)
        if C != cin:
            raise ValueError("channel mismatch")
        w2 = weight.reshape(cout, cin)
        if w2.stride(1) != 1 or w2.stride(0) != cin:
            w2 = w2.contiguous()
        n, _, h, w = x.shape
        y = torch.empty((n, cout, h, w), dtype=x.dtype, device=x.device, memory_format=torch.channels_last)
        _gemm_rows(x.data_ptr(), ldx, w2, M, cout, cin, y.data_ptr(), cout, x.device)
        ctx.save_for_backward(x, weight)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, weight = ctx.saved_tensors
        cout, cin = weight.shape[0], weight.shape[1]
        M, _, ldx = _rows_view(x)
        dy, (_, _, lddy) = _as_rows(dy)
        dx = None
        if ctx.needs_input_grad[0]:
            wt = weight.reshape(cout, cin).t().contiguous()  # [Cin, Cout]
            dx = torch.empty(x.shape, dtype=x.dtype, device=x.device, memory_format=torch.channels_last)
            _gemm_rows(dy.data_ptr(), lddy, wt, M, cin, cout, dx.data_ptr(), cin, x.device)
        dw = None
        if ctx.needs_input_grad[1]:
            dw = wgrad_tn(dy.data_ptr(), lddy, x.data_ptr(), ldx, M, cout, cin, x.device)
            dw = dw.to(weight.dtype).reshape(weight.shape)
        return dx, dw


def conv1x1(x: torch.Tensor, weight: torch.Tensor) -> torch.Tensor:
    """Stride-1 unpadded 1x1 convolution of a channels_last bf16 tensor."""
    if x.is_cuda:
        if x.dtype != torch.bfloat16 or weight.dtype != torch.bfloat16:
            raise TypeError("conv1x1 MFMA path takes bf16 activations and weights")
        return tape.apply(_Conv1x1Fn, x, weight)
    return torch.nn.functional.conv2d(x, weight)

"""Per-shape tile-variant autotuning for the NT MFMA kernels (1x1-conv GEMM, implicit-GEMM conv).

The NT kernels (csrc/gemm.hip, csrc/conv.hip) take a tile variant in flags bits 8..15
(``kNtVariants`` in csrc/mfma_common.h: rows per tile x column-tile cap; 0 = built-in heuristic).
Which one is fastest depends on the shape: Inception-v3 runs the same kernels on M = 682k rows
(a 128-row tile gives 5,300 tiles) and on M = 8,192 rows (64 tiles of 128 rows leave 3/4 of the
256 CUs idle), with N from 48 to 1,344 and K from 64 to 2,048.  The first eager call of each
(kernel, shape) times every variant on the real operands and caches the fastest; a HIP-graph
capture replays the cached decision (nothing is timed while capturing).  ``TONY_CONV_AUTOTUNE=0``
pins the heuristic.
"""
from __future__ import annotations

import os
from typing import Callable, Dict, Hashable

import torch

AUTOTUNE = os.environ.get("TONY_CONV_AUTOTUNE", "1") != "0"
# csrc/mfma_common.h kNtVariants (0-8) + 9: conv.hip halo-tile 3x3 path, 10: conv.hip persistent
# direct 3x3 kernel (32/64 channels), 11-15: conv.hip LDS-DMA kernels, 16-19: their 8-wave 256-row
# tiles, 20-24: interleaved-issue forms (igemm.h kGldsVariants; TONY_CONV_GLDS=0 leaves them all out of
# the search, TONY_CONV_GLDS8=0 the 8-wave and interleaved ones, TONY_CONV_GLDS_IL=0 the interleaved)
_N_GLDS = (25 if os.environ.get("TONY_CONV_GLDS_IL", "1") != "0" else 20) \
    if os.environ.get("TONY_CONV_GLDS8", "1") != "0" else 16
_BASE = tuple(range(_N_GLDS if os.environ.get("TONY_CONV_GLDS", "1") != "0" else 11))
# 25-31: the LDS-DMA tiles at several workgroups per CU (igemm.h conv_glds_occ_kernel: a register budget of
# 2-4 waves per SIMD; TONY_CONV_OCC=0 leaves them out of the search)
if os.environ.get("TONY_CONV_OCC", "1") != "0" and os.environ.get("TONY_CONV_GLDS", "1") != "0":
    _BASE = _BASE + tuple(range(25, 32))
# + stream-K forms of the LDS-DMA variants (csrc/igemm.h SplitK): candidate v + 256 * m, i.e. flags bits
# 16..19 = m, a grid of m x CUs workgroups sharing the (tile, K-step) iterations.  Only launches whose
# tiles leave a poorly filled last wave take it (the kernel refuses it when the tiles are a multiple of
# the grid or more than 4x it).  Off by default: on every 17x17 / 8x8 / 35x35 Inception layer the
# stream-K forms ran 0.72-0.85x of the best plain launch (the fold's partial tiles, 100-200 KB per
# workgroup through L2, cost more than the idle CUs of the plain grid; profiles/r5_streamk_ab.md) except
# the 8x8 448->384 3x3 forward (1.03-1.04x) and the whole-input aux-head GEMMs (the K = R*S*C reduction
# of 6-25 tiles).  TONY_STREAMK=1,2,3: the grid multiples offered to the tuner.
STREAM_MS = tuple(int(x) for x in os.environ.get("TONY_STREAMK", "").split(",") if x.strip() not in ("", "0"))
NT_VARIANTS = _BASE + tuple(v + 256 * m for m in STREAM_MS for v in _BASE if v >= 11)
# 40: csrc/band.hip -- the 1 x T / T x 1 stride-1 convs (forward, backward-data) on whole-line halo tiles (it
# declines every other shape).  Opt-in (TONY_CONV_BAND=1 offers it to the conv tuner): measured 0.68-0.85x of
# the best LDS-DMA tile on every Inception 1-D shape (profiles/r6_band_bench.log) -- the halo cuts the A
# re-gather but every tile still streams the 7-tap filter slice, and the register-staged prefetch (192
# VGPRs, one workgroup per CU) leaves the CU waiting on each chunk's loads
BAND_CODE = 40
CONV_VARIANTS = NT_VARIANTS + ((BAND_CODE,) if os.environ.get("TONY_CONV_BAND", "0") == "1" else ())
# the x3 (fp32) convs: their K is three planes deep, so a tile's K loop is 3x the bf16 one and the fold's
# partial tiles cost relatively less -- stream-K over one CU-grid is offered there (fp32 step A/B
# 37.64 vs 37.95 ms, profiles/r5_x3_wgrad_fused.md); TONY_X3_STREAMK=0: plain launches only
X3_STREAM_MS = tuple(int(x) for x in os.environ.get("TONY_X3_STREAMK", "1").split(",") if x.strip() not in ("", "0"))
# the fused-plane x3 tiles (igemm.h kX3Variants, codes 32-37: A hi / lo and B hi / lo staged once per K-step,
# three products on the same accumulators) for operands whose plane width is a multiple of 32;
# TONY_X3_FUSED=0 leaves them out (A/B)
X3F_CODES = tuple(range(32, 38)) if os.environ.get("TONY_X3_FUSED", "1") != "0" else ()
X3_VARIANTS = _BASE + tuple(v + 256 * m for m in X3_STREAM_MS for v in _BASE if v >= 11)
X3F_VARIANTS = X3F_CODES + tuple(v + 256 * m for m in X3_STREAM_MS for v in X3F_CODES)
# the whole-input (aux-head) GEMMs: a handful of tiles over a long K -- stream-K spreads K over the CUs
# (conv_bench --tony: fwd 30 -> 17 us, dgrad 163 -> 68 us)
SMALL_GEMM_VARIANTS = _BASE + tuple(v + 256 * m for m in (1, 2) for v in _BASE if v >= 11)


def stream_of(vflags: int) -> int:
    """Stream-K grid (in CUs) encoded in variant flags (0: plain launch)."""
    return (vflags >> 16) & 15
_CACHE: Dict[Hashable, int] = {}


def time_ms(fn: Callable[[], object], reps: int = 5) -> float:
    """GPU time of ``fn`` (ms).  A spin kernel keeps the GPU busy while the host enqueues the reps, so
    the events bracket back-to-back kernels: the host cost of a Python/ctypes launch (tens of us, as
    long as a small kernel) would otherwise be measured instead of the kernel and make the choice
    between candidates random for small shapes."""
    fn()
    torch.cuda.synchronize()
    start, end = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda._sleep(4_000_000)  # ~2 ms of spinning: longer than enqueueing the reps
    start.record()
    for _ in range(reps):
        fn()
    end.record()
    end.synchronize()
    return start.elapsed_time(end) / reps


def pick(key: Hashable, launch: Callable[[int], int], variants=NT_VARIANTS) -> int:
    """Return the flags bits (variant << 8) of the fastest tile variant for ``key``.

    ``launch(vflags)`` runs the kernel once with those variant bits and returns its status code
    (non-zero: the variant does not apply to this shape and is skipped)."""
    v = _CACHE.get(key)
    if v is not None:
        return v << 8
    if not AUTOTUNE or torch.cuda.is_current_stream_capturing():
        return 0
    best, best_t = 0, float("inf")
    for cand in variants:
        if launch(cand << 8) != 0:
            continue
        t = time_ms(lambda: launch(cand << 8))
        if t < best_t:
            best, best_t = cand, t
    _CACHE[key] = best
    return best << 8


def pick_choice(key: Hashable, choices, run: Callable[[object], object]):
    """The fastest of ``choices`` for ``key``: ``run(choice)`` executes the op once with it (timed
    on the first eager call, cached; the first choice while capturing or with tuning off)."""
    c = _CACHE.get(key)
    if c is not None:
        return c
    if not AUTOTUNE or torch.cuda.is_current_stream_capturing():
        return choices[0]
    times = {ch: time_ms(lambda: run(ch)) for ch in choices}
    best = min(times, key=times.get)
    _CACHE[key] = best
    return best


def cached(key: Hashable):
    """The variant bits already chosen for ``key``, 0 when tuning is off or capturing, else None."""
    v = _CACHE.get(key)
    if v is not None:
        return v << 8
    if not AUTOTUNE or torch.cuda.is_current_stream_capturing():
        return 0
    return None


def choices() -> Dict[Hashable, int]:
    """Variant decisions so far (for logs / profiles)."""
    return dict(_CACHE)


def gemm_flags(a: torch.Tensor, b: torch.Tensor, c: torch.Tensor, M: int, N: int, K: int, lda: int,
               stats: bool, variants=NT_VARIANTS) -> int:
    """Variant bits for ``tony_gemm_bf16`` C[M,N] = A[M,K] B[N,K]^T (B and C dense, ld K and N).

    Timing runs write C (the caller overwrites it right after) and statistics into a scratch
    buffer, never into the caller's accumulators."""
    from . import _lib

    key = ("gemm", M, N, K, lda, bool(stats))
    if key in _CACHE or not AUTOTUNE or torch.cuda.is_current_stream_capturing():
        return pick(key, lambda vf: 0)
    L = _lib.lib()
    dev = c.device
    stream = _lib.stream_ptr(dev)
    scratch = torch.zeros(_lib.stat_floats(N), dtype=torch.float32, device=dev)
    base = 1 if stats else 0
    return pick(key, lambda vf: L.tony_gemm_bf16(a.data_ptr(), b.data_ptr(), c.data_ptr(), M, N, K, lda, K, N,
                                                 base | vf, scratch.data_ptr(), 2 * N, stream), variants)


# ---- persistent decisions (the MIOpen find-db idea for tony_amd's own choices) -------------------
def save(path: str) -> int:
    """Write every decision made so far -- tile variants / split plans (this module) and the
    tony-vs-MIOpen choice per conv pass and shape (ops/conv.py) -- to a JSON file; returns the count.
    Keys are the repr of the in-process tuple keys (ints, strings, tuples, bools only)."""
    import json

    from . import conv

    rec = {"tune": {repr(k): v for k, v in _CACHE.items()}, "conv": {repr(k): v for k, v in conv._CHOICE.items()}}
    with open(path, "w") as f:
        json.dump(rec, f, indent=0, sort_keys=True)
    return len(rec["tune"]) + len(rec["conv"])


def load(path: str) -> int:
    """Seed the decision caches from ``save()``'s file (same hardware: the choices are only about
    speed, every variant computes the same result).  Returns how many decisions were loaded."""
    import ast
    import json

    from . import conv

    with open(path) as f:
        rec = json.load(f)
    for k, v in rec.get("tune", {}).items():
        _CACHE[ast.literal_eval(k)] = v
    for k, v in rec.get("conv", {}).items():
        conv._CHOICE[ast.literal_eval(k)] = v
    return len(rec.get("tune", {})) + len(rec.get("conv", {}))


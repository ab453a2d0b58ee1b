"""ctypes binding of ``_tony_kernels.so`` (the gfx950 HIP kernels).

torch is imported first on purpose: it loads its bundled HIP runtime, whose
SONAME (``libamdhip64.so.7``) the kernel library then resolves to, so both share
one runtime, one device context and the same stream handles.

On a machine with a GPU the library is REQUIRED: ``lib()`` raises if it is
missing or fails to load, so no test or benchmark silently runs an eager
PyTorch fallback.  On a CPU-only container ops called with CPU tensors use the
reference implementations in ``tony_amd.ops.reference``.
"""
from __future__ import annotations

import ctypes
import os
import threading
import weakref
from typing import Dict

import torch  # noqa: F401  (must precede the dlopen below)

_HERE = os.path.dirname(os.path.abspath(__file__))
SO_PATH = os.environ.get("TONY_KERNELS_SO") or os.path.join(_HERE, "_tony_kernels.so")  # override: A/B of builds

_lock = threading.Lock()
_lib = None

c_void_p = ctypes.c_void_p
c_int = ctypes.c_int
c_int64 = ctypes.c_int64
c_float = ctypes.c_float
c_int_p = ctypes.POINTER(ctypes.c_int)
c_void_pp = ctypes.POINTER(ctypes.c_void_p)
c_u8_p = ctypes.POINTER(ctypes.c_uint8)
c_u64_p = ctypes.POINTER(ctypes.c_uint64)

_SIGNATURES = {
    "tony_bn_fwd_train": [c_void_p, c_int64, c_int, c_int64, c_void_p, c_int64, c_void_p, c_void_p, c_int,
                          c_float, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_float, c_void_p],
    "tony_bn_fwd_infer": [c_void_p, c_int64, c_int, c_int64, c_void_p, c_int64, c_void_p, c_void_p, c_int,
                          c_float, c_int, c_void_p, c_void_p, c_void_p],
    "tony_bn_bwd": [c_void_p, c_int64, c_void_p, c_int64, c_void_p, c_int64, c_int64, c_int, c_void_p, c_void_p,
                    c_void_p, c_void_p, c_int, c_int, c_void_p, c_void_p, c_void_p, c_int, c_void_p],
    # statistics buffers: shard 0 pointers + the shard stride in floats (STAT_SHARDS copies)
    "tony_stat_shards": [],
    "tony_bn_stats": [c_void_p, c_int64, c_int, c_int64, c_void_p, c_void_p, c_int64, c_void_p],
    "tony_bn_apply": [c_void_p, c_int64, c_int, c_int64, c_void_p, c_int64, c_void_p, c_void_p, c_int64, c_void_p,
                      c_void_p, c_int, c_float, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_float,
                      c_void_p],
    "tony_bn_apply_segs": [c_void_p, c_int64, c_int, c_int64, c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p,
                           c_void_p, c_void_p, c_int64, c_int64, c_int64, c_int64, c_void_p, c_void_p, c_int64,
                           c_void_p, c_void_p, c_int, c_float, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p,
                           c_float, c_void_p],
    "tony_bn_bwd_reduce_segs": [c_void_p, c_int64, c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p,
                                c_void_p, c_int64, c_int64, c_int64, c_int64, c_int64, c_int, c_void_p, c_void_p,
                                c_void_p, c_void_p, c_int, c_int, c_void_p, c_void_p, c_int64, c_void_p],
    "tony_bn_bwd_apply_segs": [c_void_p, c_int64, c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p,
                               c_void_p, c_int64, c_int64, c_int64, c_int64, c_void_p, c_int64, c_int64, c_int,
                               c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_void_p, c_void_p, c_int64,
                               c_void_p, c_void_p, c_int, c_void_p],
    "tony_bn_relu_maxpool": [c_void_p, c_int64, c_void_p, c_void_p, c_int64, c_void_p, c_void_p, c_int, c_float,
                             c_void_p, c_void_p, c_void_p, c_void_p, c_float, c_void_p, c_int64, c_void_p, c_int,
                             c_int, c_int, c_int, c_int, c_int, c_int, c_void_p],
    "tony_bn_bwd_reduce": [c_void_p, c_int64, c_void_p, c_int64, c_int64, c_int, c_void_p, c_void_p, c_void_p,
                           c_void_p, c_int, c_int, c_void_p, c_void_p, c_int64, c_void_p],
    "tony_bn_bwd_apply": [c_void_p, c_int64, c_void_p, c_int64, c_void_p, c_int64, c_int64, c_int, c_void_p,
                          c_void_p, c_void_p, c_void_p, c_int, c_int, c_void_p, c_void_p, c_int64, c_void_p,
                          c_void_p, c_int, c_void_p],
    "tony_bn_apply_f32_x3": [c_void_p, c_int64, c_int, c_int64, c_void_p, c_int64, c_void_p, c_void_p, c_int64,
                             c_void_p, c_void_p, c_int, c_float, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p,
                             c_float, c_void_p],
    "tony_bn_apply_res": [c_void_p, c_int64, c_int, c_int64, c_void_p, c_int64, c_void_p, c_int64, c_void_p,
                          c_void_p, c_int64, c_void_p, c_void_p, c_int, c_float, c_int, c_int, c_void_p, c_void_p,
                          c_void_p, c_void_p, c_float, c_void_p],
    "tony_bn_apply_res_m": [c_void_p, c_int64, c_int, c_int64, c_void_p, c_int64, c_void_p, c_int64, c_void_p,
                            c_void_p, c_int64, c_void_p, c_void_p, c_int, c_float, c_int, c_int, c_void_p, c_void_p,
                            c_void_p, c_void_p, c_float, c_void_p, c_int64, c_void_p],
    "tony_bn_bwd_res": [c_void_p, c_int64, c_void_p, c_int64, c_void_p, c_int64, c_void_p, c_int64, c_void_p, c_int64,
                        c_int64, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_void_p,
                        c_int, c_void_p],
    "tony_bn_bwd_res_m": [c_void_p, c_int64, c_void_p, c_int64, c_void_p, c_int64, c_void_p, c_int64, c_void_p,
                          c_int64, c_int64, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_void_p,
                          c_void_p, c_int, c_void_p],
    "tony_bn_bwd_onepass": [c_void_p, c_int64, c_void_p, c_int64, c_void_p, c_int64, c_int64, c_int, c_void_p,
                            c_void_p, c_void_p, c_void_p, c_int, c_int, c_void_p, c_void_p, c_void_p, c_int,
                            c_void_p, c_int, c_void_p],
    "tony_add_f32": [c_void_p, c_int, c_void_p, c_int64, c_void_p],
    "tony_sgd_step": [c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_int64, c_void_p, c_void_p],
    "tony_adam_step": [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_int64, c_void_p, c_void_p],
    "tony_grad_stats": [c_void_p, c_int, c_int64, c_void_p, c_void_p],
    "tony_xent_fwd": [c_void_p, c_int, c_int64, c_int, c_int64, c_void_p, c_float, c_void_p, c_void_p, c_void_p],
    "tony_xent_bwd": [c_void_p, c_int, c_int64, c_int, c_int64, c_void_p, c_float, c_void_p, c_void_p, c_void_p,
                      c_int64, c_void_p],
    "tony_dropout_fwd": [c_void_p, c_void_p, c_void_p, c_int64, c_int, c_float, c_void_p, c_void_p],
    "tony_dropout_bwd": [c_void_p, c_void_p, c_void_p, c_int64, c_int, c_float, c_void_p],
    "tony_counter_bump": [c_void_p, c_void_p],
    "tony_gemm_bf16": [c_void_p, c_void_p, c_void_p, c_int64, c_int64, c_int64, c_int64, c_int64, c_int64,
                       c_int, c_void_p, c_int64, c_void_p],
    "tony_gemm_bf16_bnact": [c_void_p, c_void_p, c_void_p, c_int64, c_int64, c_int64, c_int64, c_int64, c_int64,
                             c_int, c_void_p, c_int64, c_void_p, c_void_p],
    "tony_gemm_tn_bf16": [c_void_p, c_void_p, c_void_p, c_int64, c_int64, c_int64, c_int64, c_int64, c_int64,
                          c_void_p, c_int64, c_void_p, c_int, c_void_p, c_void_p, c_int, c_void_p],
    "tony_splitk_reduce": [c_void_p, c_int, c_int64, c_void_p, c_int, c_int, c_int, c_void_p],
    "tony_splitk_workspace": [c_void_p, c_int64, c_void_p, c_int64],
    "tony_conv_fwd": [c_void_p, c_int, c_int, c_int, c_int, c_int64, c_void_p, c_int, c_int, c_int, c_int, c_int,
                      c_int, c_int, c_void_p, c_int, c_int, c_int64, c_int, c_void_p, c_int64, c_void_p],
    "tony_stem_fwd": [c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_int, c_int, c_int, c_int, c_int, c_int,
                      c_int, c_void_p, c_int, c_int, c_int64, c_int, c_void_p, c_int64, c_int, c_void_p],
    "tony_stem_wgrad": [c_void_p, c_int64, c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int,
                        c_int, c_int, c_int, c_int, c_void_p, c_int64, c_void_p, c_int, c_void_p],
    "tony_conv_dgrad": [c_void_p, c_int, c_int, c_int, c_int, c_int64, c_void_p, c_int, c_int, c_int, c_int, c_int,
                        c_void_p, c_int, c_int, c_int64, c_int, c_void_p, c_void_p],
    "tony_conv_dgrad_strided": [c_void_p, c_int, c_int, c_int, c_int, c_int64, c_void_p, c_int, c_int, c_int, c_int,
                                c_int, c_int, c_int, c_void_p, c_int, c_int, c_int64, c_int, c_void_p, c_void_p],
    "tony_conv_wgrad": [c_void_p, c_int64, c_void_p, c_int, c_int, c_int, c_int, c_int64, c_int, c_int, c_int, c_int,
                        c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_int64, c_void_p, c_int, c_void_p,
                        c_void_p, c_int, c_void_p],
    "tony_conv_wgrad_x3": [c_void_p, c_int64, c_void_p, c_int, c_int, c_int, c_int, c_int64, c_int, c_int, c_int,
                           c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_void_p, c_int64, c_void_p, c_int,
                           c_void_p],
    "tony_x3_wgrad_mode": [c_int],
    "tony_dgrad_one_launch": [c_int],
    "tony_wgrad_pf": [c_int],
    "tony_kv_copy_blocks": [c_int64],
    "tony_kv_copy_flag": [c_void_p, c_void_p, c_int64, c_void_p, c_void_p],
    "tony_kv_wait": [c_void_p, ctypes.c_uint32, c_void_p, ctypes.c_double, c_void_p],
    "tony_conv_wgrad_direct": [c_void_p, c_int64, c_void_p, c_int, c_int, c_int, c_int, c_int64, c_int, c_int, c_int,
                               c_int, c_int, c_void_p, c_int64, c_void_p, c_int, c_void_p],
    "tony_avgpool3_s1p1": [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int64, c_int64, c_void_p],
    "tony_maxpool_fwd": [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int64, c_int64,
                         c_void_p],
    "tony_maxpool_bwd": [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int64, c_int64,
                         c_void_p],
    "tony_bn_bwd_pool_apply": [c_void_p, c_int64, c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_void_p,
                               c_int64, c_void_p, c_int64, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int,
                               c_void_p, c_int64, c_void_p, c_void_p, c_int, c_void_p],
    "tony_maxpool_bwd_acc": [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int64, c_int64,
                         c_void_p],
    "tony_maxpool_bwd_bnred": [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int64,
                               c_int64, c_void_p, c_int64, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int,
                               c_void_p, c_int64, c_int, c_void_p],
    "tony_avgpool_fwd": [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_int64, c_int64, c_void_p],
    "tony_avgpool_bwd": [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_int64, c_int64, c_void_p],
    "tony_transpose_desc_bytes": [],
    "tony_x3_desc_bytes": [],
    "tony_x3_weights_batch": [c_void_p, c_int, c_int, c_void_p],
    "tony_transpose_batch": [c_void_p, c_int, c_int, c_void_p],
    # cross-stream forks / joins of the eager step (csrc/streams.hip, ops/streams.py)
    "tony_event_pool": [c_int, c_u64_p],
    "tony_fork": [c_void_p, c_void_p, c_void_p],
    # fp32 forms of the BN / pool kernels and the x3 operand split (csrc/x3.hip, ops/x3.py)
    "tony_bn_stats_f32": [c_void_p, c_int64, c_int, c_int64, c_void_p, c_void_p, c_int64, c_void_p],
    "tony_bn_apply_f32": [c_void_p, c_int64, c_int, c_int64, c_void_p, c_int64, c_void_p, c_void_p, c_int64, c_void_p,
                      c_void_p, c_int, c_float, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_float,
                      c_void_p],
    "tony_bn_bwd_reduce_f32": [c_void_p, c_int64, c_void_p, c_int64, c_int64, c_int, c_void_p, c_void_p, c_void_p,
                           c_void_p, c_int, c_int, c_void_p, c_void_p, c_int64, c_void_p],
    "tony_bn_bwd_apply_f32": [c_void_p, c_int64, c_void_p, c_int64, c_void_p, c_int64, c_int64, c_int, c_void_p,
                          c_void_p, c_void_p, c_void_p, c_int, c_int, c_void_p, c_void_p, c_int64, c_void_p,
                          c_void_p, c_int, c_void_p],
    "tony_bn_bwd_apply_f32_x3": [c_void_p, c_int64, c_void_p, c_int64, c_void_p, c_int64, c_int64, c_int, c_void_p,
                          c_void_p, c_void_p, c_void_p, c_int, c_int, c_void_p, c_void_p, c_int64, c_void_p,
                          c_void_p, c_int, c_void_p],
    "tony_bn_bwd_apply_f32_x3p": [c_void_p, c_int64, c_void_p, c_int64, c_void_p, c_int64, c_int64, c_int64, c_int,
                                  c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_void_p, c_void_p, c_int64,
                                  c_void_p, c_void_p, c_int, c_void_p],
    "tony_avgpool3_s1p1_f32": [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int64, c_int64, c_void_p],
    "tony_avgpool3_s1p1_x3p": [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int64, c_int64, c_int64, c_void_p],
    "tony_avgpool3_s1p1_acc": [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int64, c_int64, c_int, c_void_p],
    "tony_avgpool3_s1p1_x3": [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int64, c_void_p],
    "tony_maxpool_fwd_f32": [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int64, c_int64,
                         c_void_p],
    "tony_maxpool_bwd_f32": [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int64, c_int64,
                         c_void_p],
    "tony_maxpool_bwd_acc_f32": [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int64, c_int64,
                         c_void_p],
    "tony_avgpool_fwd_f32": [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_int64, c_int64, c_void_p],
    "tony_avgpool_bwd_f32": [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_int64, c_int64, c_void_p],
    "tony_x3_split": [c_void_p, c_int64, c_int64, c_int, c_int, c_void_p, c_int64, c_int, c_void_p],
    "tony_x3_split_slice": [c_void_p, c_int64, c_int64, c_int, c_void_p, c_int64, c_int, c_int, c_void_p],
    "tony_bn_apply_f32_p3": [c_void_p, c_int64, c_int, c_int64, c_void_p, c_int64, c_void_p, c_int64, c_int64,
                             c_void_p, c_void_p, c_int64, c_void_p, c_void_p, c_int, c_float, c_int, c_int, c_void_p,
                             c_void_p, c_void_p, c_void_p, c_float, c_void_p],
    "tony_x3_weights_t": [c_void_p, c_int, c_int, c_int, c_void_p, c_void_p],
    # native replay of a captured step (csrc/plan.hip, ops/plan.py)
    "tony_plan_mark": [c_int, c_void_p],
    "tony_plan_build": [c_void_p, c_u64_p, c_int, c_u64_p, c_int_p],
    "tony_plan_replay": [c_void_p, c_int, c_void_p],
    "tony_plan_segments": [c_void_p],
    "tony_plan_failure": [c_void_p, c_int_p],
    "tony_plan_ops": [c_void_p, c_int_p, c_int],
    "tony_plan_destroy": [c_void_p],
    # parameter-server data plane over xGMI windows (csrc/ps_plane.hip, parallel/ps_plane.py)
    "tony_ps_header_bytes": [],
    "tony_kv_copy": [c_void_p, c_void_p, c_int64, c_void_p, c_void_p],
    "tony_ps_max_buckets": [],
    "tony_ps_max_blocks": [],
    "tony_ps_land_entry_bytes": [],
    "tony_ps_window_alloc": [c_int64, c_void_pp, c_u8_p],
    "tony_ps_push": [c_void_p, c_int, c_void_p, c_int64, c_int, c_int64, c_int, c_int, ctypes.c_uint32, c_int,
                     c_void_p],
    "tony_ps_apply": [c_void_p, c_int64, c_int64, c_int, c_int, c_int64, c_int64, c_void_p, c_void_p, c_void_p,
                      c_void_p, c_int, c_u64_p, c_void_p, c_int, c_int, ctypes.c_uint32, c_int, ctypes.c_double,
                      c_int, c_void_p],
    "tony_ps_land": [c_void_p, c_void_p, c_int, c_void_p, c_int, ctypes.c_uint32, ctypes.c_double, c_void_p],
    "tony_ps_error_async": [c_void_p, c_void_p, c_void_p],
    "tony_ps_error": [c_void_p, c_int_p],
    # xGMI peer-memory collectives (csrc/xgmi.hip, parallel/xgmi.py)
    "tony_xgmi_max_ranks": [],
    "tony_xgmi_handle_bytes": [],
    "tony_xgmi_alloc": [c_int64, c_void_pp, c_u8_p],
    "tony_xgmi_open": [c_u8_p, c_void_pp],
    "tony_xgmi_close": [c_void_p],
    "tony_xgmi_free": [c_void_p],
    "tony_xgmi_error": [c_void_p, c_int_p],
    "tony_xgmi_error_async": [c_void_p, c_void_p, c_void_p],
    "tony_xgmi_collective": [c_u64_p, c_int, c_int, c_int64, c_int, c_void_p, c_void_p, c_int64, c_int, c_int,
                             c_float, ctypes.c_uint32, c_int, c_void_p],
}


class BnRed(ctypes.Structure):
    """csrc/conv.hip ``BnRed``: the BatchNorm-backward reduction a backward-data kernel fuses into its
    epilogue (z = layer L's BN input, the dgrad's output is dY of layer L); ``done`` is set when the
    launched kernel reduced (a tile variant without the fused epilogue leaves it 0)."""
    _fields_ = [("z", c_void_p), ("ldz", c_int64), ("mean", c_void_p), ("invstd", c_void_p), ("gamma", c_void_p),
                ("beta", c_void_p), ("pb", c_int), ("relu", c_int), ("dsum", c_void_p), ("sstride", c_int64),
                ("done", c_int)]


class _SignedLib:
    """The loaded library, exposing ONLY the functions declared in _SIGNATURES.

    ctypes passes an undeclared function's Python-int arguments as 32-bit C ints, which silently
    truncates device pointers and streams (a GPU fault far from the call); refuse such calls."""

    def __init__(self, h):
        self._h = h
        for name, argtypes in _SIGNATURES.items():
            fn = getattr(h, name, None)
            if fn is None:
                continue
            fn.argtypes = argtypes
            fn.restype = c_int
            setattr(self, name, fn)
        # the generated METH_FASTCALL wrappers (ops/fastcall.py) replace the ctypes calls where built
        self.fastcall = 0
        if os.environ.get("TONY_FASTCALL", "1") != "0":
            try:
                from . import _tony_fastcall, fastcall
            except ImportError:
                _tony_fastcall = None
            if _tony_fastcall is not None:
                for name, w in fastcall.bind_all(_tony_fastcall, h, _SIGNATURES).items():
                    setattr(self, name, w)
                    self.fastcall += 1
        # the NT conv / GEMM entry points take a stream-K grid in flags bits 16..19: give those launches
        # their workspace (csrc/igemm.h SplitK) wherever they are made from
        set_ws = self.__dict__.get("tony_splitk_workspace")
        if set_ws is not None:
            for name, fpos in _SPLITK_ENTRIES.items():
                fn = self.__dict__.get(name)
                if fn is not None:
                    setattr(self, name, _splitk_entry(fn, set_ws, fpos))

    def __getattr__(self, name):
        raise KernelError(f"{name}: not exported by {SO_PATH} or missing from _lib._SIGNATURES")


class KernelError(RuntimeError):
    pass


# entry point -> position of its flags argument (bits 16..19: stream-K grid in CUs, csrc/igemm.h SplitK)
_SPLITK_ENTRIES = {"tony_gemm_bf16": 9, "tony_conv_fwd": 18, "tony_conv_dgrad": 16}
SPLITK_MAX_TILES = 4096  # csrc/igemm.h kStreamMaxTiles: counters of a stream-K launch


def splitk_slab_floats(m: int, cus: int) -> int:
    """Partial tiles of a stream-K launch over m x cus workgroups: 2 per workgroup, each at most the
    largest LDS-DMA tile (256 x 192)."""
    return 2 * m * cus * 256 * 192


def _splitk_entry(fn, set_ws, fpos: int):
    def call(*a):
        s = (a[fpos] >> 16) & 15
        if not s:
            return fn(*a)
        from .arena import zeros_f32

        dev = torch.device("cuda", torch.cuda.current_device())
        # on the launch's (current) stream: the caching allocator keeps the slab for that stream's later work
        slab = torch.empty(splitk_slab_floats(s, num_cus(dev)), dtype=torch.float32, device=dev)
        cnt = zeros_f32(2 * SPLITK_MAX_TILES, dev)  # ticket + done counters per tile (zero bits = zero uint32)
        check(set_ws(slab.data_ptr(), slab.numel(), cnt.data_ptr(), cnt.numel()), "tony_splitk_workspace")
        try:
            return fn(*a)
        finally:
            set_ws(0, 0, 0, 0)

    call.__name__ = getattr(fn, "__name__", "splitk_entry")
    call.__wrapped__ = fn
    return call


# BatchNorm statistics are accumulated into STAT_SHARDS copies (csrc/common.h kStatShards): a
# statistics buffer for C channels is STAT_SHARDS x [sum C | sumsq C] floats, shard stride 2C.
STAT_SHARDS = 8


def stat_floats(c: int) -> int:
    """Floats of a zeroed statistics buffer for ``c`` channels ([sum | sumsq] x STAT_SHARDS)."""
    return STAT_SHARDS * 2 * c


def check_stat_buffer(buf, c: int) -> None:
    """Refuse a statistics buffer too small for the kernels' STAT_SHARDS copies (they would write past it)."""
    if buf is not None and (buf.dtype != torch.float32 or buf.numel() < stat_floats(c) or not buf.is_contiguous()):
        raise ValueError(f"statistics buffer for {c} channels must be {stat_floats(c)} contiguous fp32 "
                         f"(STAT_SHARDS={STAT_SHARDS} x [sum | sumsq]); got {buf.dtype} x {buf.numel()}")


# TONY_BN_ONEPASS=1: BatchNorm backward in ONE launch (reduce -> grid barrier -> apply,
# csrc/bn_act.hip; the arrival counter is the word after the statistics floats of the zeroed
# workspace).  Off by default: its grid must stay co-resident (<= 2 workgroups per CU), which starves
# the memory pipeline -- measured 109 us per layer vs 43 us for the reduce + apply pair
# (profiles/r2_rejected_splitk_fold_bn_onepass_prof.md).
BN_ONEPASS = os.environ.get("TONY_BN_ONEPASS", "0") == "1"
# ... only for layers whose activation (M x C bf16) is at most this many MB (0: every layer): the small
# 17x17 / 8x8 layers pay two launch ramps for 14 MB of data, and their second read hits the L2 / MALL
BN_ONEPASS_MAX_BYTES = int(os.environ.get("TONY_BN_ONEPASS_MAX_MB", "0")) << 20


def bn_bwd_ws_floats(c: int) -> int:
    """Floats of a zeroed BN-backward workspace: the sharded [dsum | dsumx] + the barrier counter."""
    return stat_floats(c) + 4


def bn_bwd(x, ldx: int, dy, lddy: int, dx, lddx: int, M: int, C: int, mean, invstd, gamma, beta, pb: int,
           relu: bool, ws, dgamma, dbeta, accumulate: bool, device, sums=None) -> None:
    """dx (and dgamma/dbeta, added into when ``accumulate``) of y = relu?(bn(x)) from dy.  ``sums``:
    the sharded [dsum | dsumx] already reduced by the kernel that produced dy (a dgrad epilogue,
    csrc/conv.hip BnRed): only the apply pass runs."""
    L = lib()
    if sums is not None:
        rc = L.tony_bn_bwd_apply(x.data_ptr(), ldx, dy.data_ptr(), lddy, dx.data_ptr(), lddx, M, C, mean.data_ptr(),
                                 invstd.data_ptr(), ptr(gamma), ptr(beta), pb, int(relu), sums.data_ptr(),
                                 sums.data_ptr() + 4 * C, 2 * C, ptr(dgamma), ptr(dbeta), int(accumulate),
                                 stream_ptr(device))
        check(rc, "tony_bn_bwd_apply")
        return
    if BN_ONEPASS and ws.numel() >= stat_floats(C) + 1 and (BN_ONEPASS_MAX_BYTES == 0 or
                                                             2 * M * C <= BN_ONEPASS_MAX_BYTES):
        rc = L.tony_bn_bwd_onepass(x.data_ptr(), ldx, dy.data_ptr(), lddy, dx.data_ptr(), lddx, M, C,
                                   mean.data_ptr(), invstd.data_ptr(), ptr(gamma), ptr(beta), pb, int(relu),
                                   ws.data_ptr(), ptr(dgamma), ptr(dbeta), int(accumulate),
                                   ws.data_ptr() + 4 * stat_floats(C), num_cus(device), stream_ptr(device))
        check(rc, "tony_bn_bwd_onepass")
        return
    rc = L.tony_bn_bwd(x.data_ptr(), ldx, dy.data_ptr(), lddy, dx.data_ptr(), lddx, M, C, mean.data_ptr(),
                       invstd.data_ptr(), ptr(gamma), ptr(beta), pb, int(relu), ws.data_ptr(), ptr(dgamma), ptr(dbeta),
                       int(accumulate), stream_ptr(device))
    check(rc, "tony_bn_bwd")


def fold_stats(buf, c: int):
    """[sum | sumsq] (2c floats) of a sharded statistics buffer (sums the STAT_SHARDS copies)."""
    return buf[:stat_floats(c)].view(STAT_SHARDS, 2 * c).sum(0)


def lib():
    """Load (once) and return the kernel library; raise loudly if unavailable."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(SO_PATH):
            raise KernelError(
                f"{SO_PATH} is missing: run `python -m tony_amd.ops.build` (or __graft_entry__.build())")
        h = _SignedLib(ctypes.CDLL(SO_PATH, mode=ctypes.RTLD_LOCAL))
        n = h.tony_stat_shards()
        if n != STAT_SHARDS:
            raise KernelError(f"{SO_PATH} accumulates BN statistics in {n} shards, the Python side expects "
                              f"{STAT_SHARDS}: rebuild the kernels")
        _lib = h
    return _lib


def available() -> bool:
    try:
        lib()
        return True
    except (KernelError, OSError):
        return False


_RAW_STREAM = getattr(torch._C, "_cuda_getCurrentRawStream", None)


def stream_ptr(device=None) -> int:
    """The current HIP stream of ``device`` as an integer (the raw binding: every kernel launch asks)."""
    if _RAW_STREAM is not None:
        idx = getattr(device, "index", None)
        return _RAW_STREAM(torch.cuda.current_device() if idx is None else idx)
    return torch.cuda.current_stream(device).cuda_stream


def check(rc: int, name: str):
    if rc != 0:
        raise KernelError(f"{name} failed with code {rc}")


_NUM_CUS = {}


def num_cus(device) -> int:
    idx = device.index if device.index is not None else torch.cuda.current_device()
    if idx not in _NUM_CUS:
        _NUM_CUS[idx] = torch.cuda.get_device_properties(idx).multi_processor_count
    return _NUM_CUS[idx]


_INPLACE_GRADS = [True]


def set_inplace_grads(enabled: bool) -> None:
    """When on (default), fused ops ADD parameter gradients straight into an
    existing ``param.grad`` (the flat gradient buffer of tony_amd.parallel) and
    return None to autograd, which removes one AccumulateGrad add kernel and one
    temporary per parameter per step.  Turn off for hook-driven gradient
    bucketing that must observe every AccumulateGrad."""
    _INPLACE_GRADS[0] = bool(enabled)


_SLOT_OK: Dict[int, tuple] = {}  # id(param) -> (weakref to its .grad, whether that tensor passed the checks)


def grad_slot(param):
    """The tensor to accumulate ``param``'s gradient into, or None.  The dtype / shape / layout checks
    of a given ``.grad`` tensor are memoised (~200 lookups per Inception step): a hit requires the
    very same gradient tensor object (FlatParams' slot views are rebound, never mutated in place)."""
    if not _INPLACE_GRADS[0] or param is None or not isinstance(param, torch.nn.Parameter):
        return None
    g = param.grad
    if g is None:
        return None
    hit = _SLOT_OK.get(id(param))
    if hit is not None and hit[0]() is g:
        return g if hit[1] else None
    ok = (g.dtype == param.dtype and g.shape == param.shape
          and (g.is_contiguous() or (g.dim() == 4 and g.is_contiguous(memory_format=torch.channels_last))))
    if len(_SLOT_OK) > 65536:
        _SLOT_OK.clear()
    _SLOT_OK[id(param)] = (weakref.ref(g), ok)  # weak: never keeps a dropped gradient buffer alive
    return g if ok else None


_GRAD_LISTENERS: "weakref.WeakSet" = weakref.WeakSet()


def add_grad_listener(listener) -> None:
    """Register an object whose ``ready(params)`` is told when fused ops finish writing gradients
    in place (the gradient-bucket engines of tony_amd.parallel.buckets); held weakly."""
    _GRAD_LISTENERS.add(listener)


def remove_grad_listener(listener) -> None:
    _GRAD_LISTENERS.discard(listener)


def grads_ready(*params) -> None:
    """Called by a fused op's backward, after its last kernel is enqueued, for every parameter whose
    gradient it accumulated in place (those never reach AccumulateGrad or its hooks)."""
    if _GRAD_LISTENERS:
        ps = [p for p in params if p is not None]
        for lst in list(_GRAD_LISTENERS):
            lst.ready(ps)


def report_inplace(params, returned) -> None:
    """``grads_ready`` for the trainable ``params`` whose gradient a backward node returned as None,
    i.e. accumulated in place into the flat gradient buffer."""
    if _GRAD_LISTENERS:
        grads_ready(*[p for p, g in zip(params, returned)
                      if g is None and isinstance(p, torch.nn.Parameter) and p.requires_grad])


def ptr(t) -> int:
    return 0 if t is None else t.data_ptr()


def check_f32_stats(*tensors) -> None:
    """BatchNorm running statistics are fp32 device buffers that the kernels update in place.

    ``model.to(torch.bfloat16)`` also casts them; passing those to a kernel that writes fp32
    would overrun the buffer, so refuse loudly (use tony_amd.models.layers.cast_model)."""
    for t in tensors:
        if t is not None and t.dtype != torch.float32:
            raise TypeError(f"BatchNorm running statistics must be float32, got {t.dtype}; "
                            "cast models with tony_amd.models.layers.cast_model(model, dtype)")

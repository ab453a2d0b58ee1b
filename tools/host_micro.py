#!/usr/bin/env python3
"""Host cost of the building blocks of an eager tony_amd step (GPU box): what one torch.empty, one
fastcall kernel launch, one autograd Function round trip, one nn.Module call, one stream fork and
one arena slice cost on this host.  Decides where host-issue work pays (README, round 3).

usage: python tools/host_micro.py [--iters 20000]
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def bench(fn, iters):
    for _ in range(min(200, iters)):
        fn()
    t = time.perf_counter()
    for _ in range(iters):
        fn()
    return (time.perf_counter() - t) / iters * 1e6


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20000)
    a = ap.parse_args()
    from tony_amd.ops import _lib, arena, streams

    dev = torch.device("cuda", 0)
    L = _lib.lib()
    cl = torch.channels_last
    x = torch.zeros((8, 64, 17, 17), dtype=torch.bfloat16, device=dev).contiguous(memory_format=cl)
    out = {}
    out["torch.empty_cl_us"] = bench(lambda: torch.empty((8, 64, 17, 17), dtype=torch.bfloat16, device=dev,
                                                         memory_format=cl), a.iters)
    out["torch.empty_1d_us"] = bench(lambda: torch.empty(64, dtype=torch.float32, device=dev), a.iters)
    out["empty_like_us"] = bench(lambda: torch.empty_like(x), a.iters)
    out["data_ptr_us"] = bench(lambda: x.data_ptr(), a.iters)
    out["shape_stride_us"] = bench(lambda: (x.shape, x.stride()), a.iters)
    st = _lib.stream_ptr(dev)
    out["stream_ptr_us"] = bench(lambda: _lib.stream_ptr(dev), a.iters)
    y = torch.empty_like(x)
    # a tiny real kernel launch through the fastcall binding (avg-pool 3x3 on a small map)
    out["fastcall_launch_us"] = bench(lambda: L.tony_avgpool3_s1p1(x.data_ptr(), y.data_ptr(), 8, 17, 17, 64, 64,
                                                                   64, st), a.iters)
    torch.cuda.synchronize()

    class Nop(torch.autograd.Function):
        @staticmethod
        def forward(ctx, t):
            return t.view_as(t)

        @staticmethod
        def backward(ctx, g):
            return g

    xr = x.clone().requires_grad_(True)
    out["function_apply_fwd_us"] = bench(lambda: Nop.apply(xr), a.iters // 4)
    out["function_fwd_bwd_us"] = bench(lambda: Nop.apply(xr).sum().backward(), a.iters // 20)
    out["sum_backward_baseline_us"] = bench(lambda: xr.sum().backward(), a.iters // 20)
    m = torch.nn.Identity()
    out["module_call_us"] = bench(lambda: m(x), a.iters)
    s = torch.cuda.Stream()
    ev = torch.cuda.Event()

    def fork():
        ev.record(torch.cuda.current_stream())
        s.wait_event(ev)

    out["event_fork_us"] = bench(fork, a.iters)
    main = torch.cuda.current_stream()
    out["native_fork_us"] = bench(lambda: streams.fork(main, s), a.iters)
    out["set_stream_pair_us"] = bench(lambda: (torch.cuda.set_stream(s), torch.cuda.set_stream(main)), a.iters)
    out["current_stream_us"] = bench(lambda: torch.cuda.current_stream(), a.iters)
    ar = arena.for_device(dev)
    ar.begin_step()
    out["arena_slice_us"] = bench(lambda: arena.zeros_f32(128, dev), 2000)
    ar.end_step()
    out["torch_zeros_us"] = bench(lambda: torch.zeros(128, device=dev), a.iters)
    torch.cuda.synchronize()
    out["streams_enabled"] = streams.ENABLED
    print(json.dumps({k: (round(v, 3) if isinstance(v, float) else v) for k, v in out.items()}), flush=True)


if __name__ == "__main__":
    main()

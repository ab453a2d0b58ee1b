#!/usr/bin/env python3
"""Graph capture of ONE fp32 (x3) Inception block's forward + backward with its fast form on (branch
streams, concat slots, GradJoin), as the trainer captures the step: names the block (and the toggle)
whose capture fails.  One block per process (a capture crash ends the process).

usage: python tools/x3_capture_diag.py <A|B|C|D|E> [--no-join] [--no-branches]
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    from tony_amd.models import inception_v3 as I
    from tony_amd.ops import streams

    name = sys.argv[1]
    I.JOIN = "--no-join" not in sys.argv
    branches = "--no-branches" not in sys.argv
    dev = torch.device("cuda", 0)
    mk = {"A": lambda: (I.InceptionA(192, 32, x3=True), 35), "B": lambda: (I.InceptionB(288, x3=True), 35),
          "C": lambda: (I.InceptionC(768, 128, x3=True), 17), "D": lambda: (I.InceptionD(768, x3=True), 17),
          "E": lambda: (I.InceptionE(1280, x3=True), 8)}
    torch.manual_seed(0)
    blk, hw = mk[name]()
    blk = blk.to(dev).to(memory_format=torch.channels_last).train()
    cin = {"A": 192, "B": 288, "C": 768, "D": 768, "E": 1280}[name]
    x0 = torch.randn(8, cin, hw, hw, device=dev).contiguous(memory_format=torch.channels_last).requires_grad_(True)

    def step():
        on = streams.begin(dev, branches=branches)
        try:
            y = blk(x0 * 1.0)
            y.backward(torch.ones_like(y))
        finally:
            if on:
                streams.end()

    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            step()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    print(f"block {name}: eager ok", flush=True)
    if "--bt" in sys.argv:  # native call stack on a crash (tools/native/segv_bt.cpp), installed last
        import ctypes

        ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "native", "libsegv_bt.so")).segv_bt_install()
    g = torch.cuda.CUDAGraph(keep_graph=True)
    with torch.cuda.graph(g):
        step()
    print(f"block {name}: capture ok", flush=True)
    g.instantiate()
    g.replay()
    torch.cuda.synchronize()
    print(f"block {name}: replay ok", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())

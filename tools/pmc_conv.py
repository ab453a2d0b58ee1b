#!/usr/bin/env python3
"""Hardware-counter table of the Inception-v3 step's top conv kernels (MI355X, rocprofv3 --pmc).

Workload (``--run``): the heaviest conv kernels of the bf16 step, each pinned to the tile variant the
autotuner picks for it at batch 128 (``--variants`` overrides), 5 launches each, nothing else on the
GPU -- the 17x17 1x7 forward (LDS-DMA 8-wave 256x192, interleaved issue), its backward-data, a 35x35 3x3
forward, the 17x17 split-K weight gradient (conv_wgrad_glds_kernel<96>) and a 1x1 weight gradient
(gemm_tn_glds_kernel).  Three counter passes, each its own rocprofv3 run (tools/pmc_conv.sh), then
``--summarize DIR`` prints one row per kernel:

* wave cycles split into issuing / waiting at s_waitcnt + barrier (SQ_WAIT_ANY) / issue-stalled
  (SQ_WAIT_INST_ANY, of which LDS-issue stalls SQ_WAIT_INST_LDS);
* MFMA busy ~ SQ_VALU_MFMA_BUSY_CYCLES / (kernel cycles x 1024 SIMDs), kernel cycles = GRBM_GUI_ACTIVE / 8;
* LDS busy ~ SQ_LDS_IDX_ACTIVE / (kernel cycles x 256 CUs), bank-conflict share of it;
* VALU / MFMA / LDS / VMEM instruction counts per MFMA; L2 hit rate.

usage: python3 tools/pmc_conv.py --run          (the workload; under rocprofv3)
       python3 tools/pmc_conv.py --summarize gpurun_out/pmc_conv
"""
import argparse
import csv
import glob
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

# (label, pass, (N, Cin, H, W, Cout, k, pad), variant flags)
CASES = [
    ("fwd 17x17 192->192 1x7", "fwd", (128, 192, 17, 17, 192, (1, 7), (0, 3)), 23 << 8),
    ("dgrad 17x17 192->192 1x7", "dgrad", (128, 192, 17, 17, 192, (1, 7), (0, 3)), 23 << 8),
    ("fwd 35x35 96->96 3x3", "fwd", (128, 96, 35, 35, 96, (3, 3), (1, 1)), 24 << 8),
    ("wgrad 17x17 192->192 1x7", "wgrad", (128, 192, 17, 17, 192, (1, 7), (0, 3)), None),
    ("wgrad 17x17 768->192 1x1", "wgrad", (128, 768, 17, 17, 192, (1, 1), (0, 0)), None),
]


def run() -> int:
    import torch

    from tony_amd.ops import _lib
    from tony_amd.ops import conv as C

    _lib.set_inplace_grads(False)
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)

    def nhwc(t):
        return t.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)

    for _, pas, (n, ci, h, w, co, k, p), vf in CASES:
        x = nhwc(torch.randn(n, ci, h, w, device=dev))
        wt = nhwc(torch.randn(co, ci, *k, device=dev) / (ci * k[0] * k[1]) ** 0.5)
        y = C.conv_fwd(x, wt, 1, p, None, vflags=23 << 8 if vf is None else vf)
        dy = nhwc(torch.randn(y.shape, device=dev))
        stats = torch.zeros(_lib.stat_floats(co), device=dev)
        for _ in range(5):
            if pas == "fwd":
                stats.zero_()
                C.conv_fwd(x, wt, 1, p, stats, vflags=vf)
            elif pas == "dgrad":
                C.conv_dgrad(dy, wt, x.shape, 1, p, vflags=vf)
            else:
                C.conv_wgrad(dy, x, wt.shape, 1, p)
        torch.cuda.synchronize()
    print("ok")
    return 0


def summarize(d: str) -> int:
    acc = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                name = row.get("Kernel_Name", "")
                if "conv_" not in name and "gemm_" not in name and "splitk" not in name:
                    continue
                short = name.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
                acc[short][row["Counter_Name"]] += float(row["Counter_Value"])
                disp[short].add((f, row.get("Dispatch_Id")))
    if not acc:
        print(f"no counter rows under {d}")
        return 1
    print("| kernel | dispatches | issuing / waitcnt+barrier / issue-stalled (LDS) | MFMA busy | LDS busy (conflict) "
          "| VALU / LDS / VMEM per MFMA | L2 hit |")
    print("|---|---|---|---|---|---|---|")
    for k, c in sorted(acc.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0)):
        wc = c.get("SQ_WAVE_CYCLES", 0) or float("nan")
        cyc = c.get("GRBM_GUI_ACTIVE", 0) / 8 or float("nan")
        mf = c.get("SQ_INSTS_MFMA", 0) or float("nan")
        hit = c.get("TCC_HIT_sum", 0)
        miss = c.get("TCC_MISS_sum", 0)
        print(f"| `{k}` | {len(disp[k])} | {c.get('SQ_ACTIVE_INST_ANY', 0) / wc:.2f} / {c.get('SQ_WAIT_ANY', 0) / wc:.2f} / "
              f"{c.get('SQ_WAIT_INST_ANY', 0) / wc:.2f} ({c.get('SQ_WAIT_INST_LDS', 0) / wc:.2f}) | "
              f"{c.get('SQ_VALU_MFMA_BUSY_CYCLES', 0) / (cyc * 1024):.2f} | "
              f"{c.get('SQ_LDS_IDX_ACTIVE', 0) / (cyc * 256):.2f} "
              f"({c.get('SQ_LDS_BANK_CONFLICT', 0) / max(1.0, c.get('SQ_LDS_IDX_ACTIVE', 0)):.3f}) | "
              f"{c.get('SQ_INSTS_VALU', 0) / mf:.2f} / {c.get('SQ_INSTS_LDS', 0) / mf:.2f} / "
              f"{c.get('SQ_INSTS_VMEM', 0) / mf:.2f} | "
              f"{hit / (hit + miss) if hit + miss else float('nan'):.3f} |")
    return 0


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--run", action="store_true")
    ap.add_argument("--summarize", default=None)
    a = ap.parse_args()
    sys.exit(run() if a.run else summarize(a.summarize) if a.summarize else 2)

#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel trace into a compact markdown table (steady state only).

usage: prof_summary.py <prof_dir> [--top N] [--skip W] [--by-grid]

--by-grid: one row per (kernel, grid size) instead of per kernel -- the same kernel on different
layer shapes launches different grids, so this separates e.g. the 35x35 from the 17x17 convs.

Reads *kernel_trace.csv under <prof_dir> (rocprofv3 --kernel-trace --output-format csv).
Every training step launches exactly one fused optimizer kernel (sgd_kernel /
adam_kernel), so those launches delimit steps: kernels before the end of the W-th
optimizer launch (warmup, MIOpen solver search, first-call compiles) are dropped and
the remaining window is reported per step, grouped into tony_amd HIP kernels vs
MIOpen / hipBLASLt / PyTorch-native kernels.
"""
import csv
import glob
import os
import sys


def classify(name):
    n = name.lower()
    if "bn_fwd" in n or "bn_bwd" in n:
        return "tony HIP: fused BN+ReLU"
    if "bn_relu_maxpool" in n:
        return "tony HIP: fused BN+ReLU+maxpool (stem)"
    if "gemm_nt_kernel" in n or "gemm_tn_splitk" in n or "gemm_tn_glds" in n:
        return "tony HIP: MFMA GEMM (1x1 conv fwd/dgrad/wgrad)"
    if "conv_nt_kernel" in n or "conv_wgrad_kernel" in n or "conv_wgrad_glds" in n or "conv_halo" in n \
            or "conv_direct_kernel" in n or "conv_glds_kernel" in n or "conv_glds_occ" in n or "conv_wgrad_direct" in n or "conv_wgrad_x3f" in n:
        return "tony HIP: implicit-GEMM conv (fwd/dgrad/wgrad)"
    if "stem_fwd_kernel" in n or "stem_wgrad_kernel" in n:
        return "tony HIP: MFMA image-stem conv (fwd/wgrad)"
    if "add_f32_kernel" in n:
        return "tony HIP: in-place grad accumulate"
    if "box3_kernel" in n or "maxpool_" in n or "avgpool_" in n:
        return "tony HIP: pooling"
    if "sgd_kernel" in n or "adam_kernel" in n or "grad_stats" in n:
        return "tony HIP: fused optimizer"
    if "xent" in n:
        return "tony HIP: fused xent"
    if "tony" in n or "conv_nhwc" in n or "pool_nhwc" in n or "cat_nhwc" in n:
        return "tony HIP: other"
    if "nccl" in n or "rccl" in n:
        return "RCCL"
    if "batch_norm" in n or "batchnorm" in n:
        return "PyTorch/MIOpen BN"
    if "naive_conv" in n or "igemm" in n or "conv" in n or "gridwise" in n or "xdlops" in n or "ck::" in n \
            or "_zn2ck" in n:
        return "MIOpen conv (CK / igemm / naive)"
    if "cijk" in n or "gemm" in n or "rocblas" in n or "hipblaslt" in n:
        return "hipBLASLt/rocBLAS GEMM"
    if "pool" in n:
        return "PyTorch pooling"
    if "splitk_reduce" in n:
        return "tony HIP: split-K wgrad combine"
    if "cat" in n or "copy" in n or "elementwise" in n or "vectorized" in n or "reduce" in n or "fill" in n \
            or "subtensor" in n:
        return "PyTorch elementwise/copy/fill"
    return "other"


def col(r, *names):
    for n in names:
        if n in r:
            return r[n]
    raise KeyError(names)


def main():
    d = sys.argv[1]
    top = int(sys.argv[sys.argv.index("--top") + 1]) if "--top" in sys.argv else 30
    skip = int(sys.argv[sys.argv.index("--skip") + 1]) if "--skip" in sys.argv else 3
    files = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    if not files:
        print(f"no kernel_trace.csv under {d}")
        return 1
    ks = []
    for f in files:
        with open(f) as fh:
            for r in csv.DictReader(fh):
                name = col(r, "Kernel_Name", "Name", "name")
                if "--by-grid" in sys.argv:
                    grid = "x".join(r[k] for k in sorted(r) if k.startswith("Grid_Size") and r[k] not in ("", "1"))
                    short = name.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
                    name = f"{short} grid={grid or r.get('Grid_Size', '?')}"
                ks.append((int(col(r, "Start_Timestamp", "start")), int(col(r, "End_Timestamp", "end")), name))
    ks.sort()
    opt_ends = [e for s, e, n in ks if "sgd_kernel" in n or "adam_kernel" in n]
    if len(opt_ends) <= skip:
        print(f"only {len(opt_ends)} optimizer launches, cannot skip {skip}")
        return 1
    t0, t1 = opt_ends[skip - 1], opt_ends[-1]
    steps = len(opt_ends) - skip
    # the harness's spin kernels (bench.py host-ahead window, tune.time_ms) are not step work
    win = [(s, e, n) for s, e, n in ks if s > t0 and e <= t1 and "spin_kernel" not in n]
    if "--sequence" in sys.argv:
        # one steady-state step in dispatch order: index, start offset, duration, gap to previous end
        one = [(s, e, n) for s, e, n in ks if s > opt_ends[-2] and e <= t1]
        prev = one[0][0] if one else 0
        for i, (s, e, n) in enumerate(one):
            print(f"{i:4d} {(s - one[0][0]) / 1e3:9.1f} {(e - s) / 1e3:8.1f} {(s - prev) / 1e3:6.1f}  {n[:110]}")
            prev = e
        return 0
    busy = sum(e - s for s, e, _ in win)
    wall = t1 - t0
    by_name, groups = {}, {}
    for s, e, n in win:
        a = by_name.setdefault(n, [0, 0])
        a[0] += 1
        a[1] += e - s
        g = classify(n)
        groups[g] = groups.get(g, 0) + (e - s)
    print(f"steady-state window: {steps} steps, wall {wall / 1e6 / steps:.2f} ms/step, "
          f"kernel busy {busy / 1e6 / steps:.2f} ms/step, {len(win) // max(steps, 1)} launches/step")
    print()
    print("| group | ms/step | share of kernel time |")
    print("|---|---|---|")
    for g, v in sorted(groups.items(), key=lambda kv: -kv[1]):
        print(f"| {g} | {v / 1e6 / steps:.3f} | {100 * v / busy:.1f}% |")
    print()
    print("| kernel | calls/step | ms/step | avg us | share |")
    print("|---|---|---|---|---|")
    for n, (c, t) in sorted(by_name.items(), key=lambda kv: -kv[1][1])[:top]:
        name = n if len(n) <= 100 else n[:97] + "..."
        name = name.replace("|", "\\|")
        print(f"| `{name}` | {c / steps:.1f} | {t / 1e6 / steps:.3f} | {t / c / 1e3:.1f} | {100 * t / busy:.1f}% |")
    return 0


if __name__ == "__main__":
    sys.exit(main())

#!/usr/bin/env python3
"""Kernel-by-kernel comparison of one steady-state step issued eagerly and replayed by the native plan
(ops/plan.py), from two rocprofv3 kernel traces (CSV) of bench.py --mode eager / --mode graph.

The plan re-issues the captured step in capture order, so the k-th kernel of a plan step is the k-th kernel
of the eager step.  For each kernel: the stream it ran on in either mode, its duration in either mode and
the time it waited after its predecessor on the same stream finished (a dependency on another stream, or
the queue).  Summaries: duration sums, how often the plan put consecutive chain kernels on different
streams, and the kernels whose start slipped most relative to the step start.

usage: python tools/plan_vs_eager.py EAGER_kernel_trace.csv PLAN_kernel_trace.csv [--step 2] [--top 25]
"""
import argparse
import csv
from collections import defaultdict


def short(n):
    return n.replace("(anonymous namespace)::", "").replace("tony::glds::", "").split("(")[0][:70]


def steps(path):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r.get("Dispatch_Id", r.get("Correlation_Id", 0))), int(r["Start_Timestamp"]),
                         int(r["End_Timestamp"]), r["Stream_Id"], r["Kernel_Name"]))
    rows.sort()  # dispatch (issue) order
    out, cur = [], []
    for r in rows:
        cur.append(r)
        if "sgd_kernel" in r[4] or "adam_kernel" in r[4]:
            out.append(cur)
            cur = []
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("eager")
    ap.add_argument("plan")
    ap.add_argument("--step", type=int, default=-2, help="which complete step (default: the second last)")
    ap.add_argument("--top", type=int, default=25)
    a = ap.parse_args()
    es, ps = steps(a.eager), steps(a.plan)
    E, P = es[a.step], ps[a.step]
    ne, np_ = [short(r[4]) for r in E], [short(r[4]) for r in P]
    print(f"eager step: {len(E)} kernels, {(max(r[2] for r in E) - min(r[1] for r in E)) / 1e3:.3f} ms span; "
          f"plan step: {len(P)} kernels, {(max(r[2] for r in P) - min(r[1] for r in P)) / 1e3:.3f} ms span")
    if ne != np_:
        # align by name where the sequences differ (a kernel only one mode issues)
        print("kernel sequences differ; comparing the common prefix")
    n = min(len(E), len(P))
    e0, p0 = min(r[1] for r in E), min(r[1] for r in P)
    de = sum(r[2] - r[1] for r in E[:n]) / 1e3
    dp = sum(r[2] - r[1] for r in P[:n]) / 1e3
    print(f"sum of kernel durations: eager {de:.3f} ms, plan {dp:.3f} ms")
    for name, rows in (("eager", E), ("plan", P)):
        busy = defaultdict(float)
        cnt = defaultdict(int)
        for r in rows:
            busy[r[3]] += (r[2] - r[1]) / 1e3
            cnt[r[3]] += 1
        print(f"  {name}: " + ", ".join(f"stream {s}: {cnt[s]} kernels {busy[s]:.2f} ms" for s in sorted(busy)))
    # stream mapping: how the plan's streams correspond to the eager ones
    pairs = defaultdict(int)
    for i in range(n):
        pairs[(E[i][3], P[i][3])] += 1
    print("eager stream -> plan stream (kernel counts): " + ", ".join(f"{k[0]}->{k[1]}: {v}" for k, v in
                                                                     sorted(pairs.items(), key=lambda kv: -kv[1])))
    # per-kernel slip: start offset from the step start, plan minus eager
    slips = []
    prev_e, prev_p = defaultdict(int), defaultdict(int)
    for i in range(n):
        re_, rp = E[i], P[i]
        wait_e = max(0, re_[1] - prev_e[re_[3]]) if prev_e[re_[3]] else 0
        wait_p = max(0, rp[1] - prev_p[rp[3]]) if prev_p[rp[3]] else 0
        prev_e[re_[3]] = re_[2]
        prev_p[rp[3]] = rp[2]
        slips.append((i, ne[i], (rp[1] - p0 - (re_[1] - e0)) / 1e3, (re_[2] - re_[1]) / 1e3, (rp[2] - rp[1]) / 1e3,
                      wait_e / 1e3, wait_p / 1e3, re_[3], rp[3]))
    print(f"\nkernels by plan-minus-eager growth of the start offset (first {a.top} jumps):")
    last = 0.0
    jumps = []
    for s in slips:
        jumps.append((s[2] - last, s))
        last = s[2]
    for dj, s in sorted(jumps, key=lambda t: -t[0])[:a.top]:
        print(f"  #{s[0]:3d} {s[1]:70s} slip +{dj * 1e3:7.1f} us (total {s[2]:6.3f} ms)  dur e/p "
              f"{s[3] * 1e3:6.1f}/{s[4] * 1e3:6.1f} us  wait e/p {s[5] * 1e3:6.1f}/{s[6] * 1e3:6.1f} us  "
              f"stream e/p {s[7]}/{s[8]}")
    print("\nlargest duration differences (plan - eager):")
    for s in sorted(slips, key=lambda s: -(s[4] - s[3]))[:a.top]:
        print(f"  #{s[0]:3d} {s[1]:70s} dur e/p {s[3] * 1e3:6.1f}/{s[4] * 1e3:6.1f} us  stream e/p {s[7]}/{s[8]}")
    return 0


if __name__ == "__main__":
    raise SystemExit(main())

#!/usr/bin/env python3
"""Per-step GPU busy time from a rocprofv3 kernel trace: wall, summed kernel time and the union of
kernel intervals (the GPU-bound step time when streams overlap).  Steps are delimited by the
loss kernel (xent_fwd, 2 launches per Inception step: main + aux head).

Usage: python tools/step_union.py <trace dir> [--per-step-marker xent_fwd --markers-per-step 2]
"""
import argparse
import csv
import glob
import os


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace_dir")
    ap.add_argument("--marker", default="xent_fwd")
    ap.add_argument("--markers-per-step", type=int, default=2)
    a = ap.parse_args()
    path = glob.glob(os.path.join(a.trace_dir, "**", "*kernel_trace.csv"), recursive=True)[0]
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    marks = [i for i, r in enumerate(rows) if a.marker in r["Kernel_Name"]][::a.markers_per_step]
    for lo, hi in zip(marks, marks[1:]):
        iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows[lo:hi])
        wall = int(rows[hi]["Start_Timestamp"]) - iv[0][0]
        busy = sum(e - s for s, e in iv)
        u, (cs, ce) = 0, iv[0]
        for s, e in iv[1:]:
            if s > ce:
                u, cs, ce = u + ce - cs, s, e
            else:
                ce = max(ce, e)
        u += ce - cs
        print(f"{hi - lo:5d} kernels  wall {wall / 1e6:7.2f} ms  kernel-sum {busy / 1e6:7.2f} ms  "
              f"union {u / 1e6:7.2f} ms")


if __name__ == "__main__":
    main()

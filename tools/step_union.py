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
    ap.add_argument("--per-queue", action="store_true", help="busy time per queue + the busiest queue's gaps")
    ap.add_argument("--gaps", type=int, default=12)
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
        if a.per_queue:
            per_queue(rows[lo:hi], a.gaps)


def per_queue(rows, ngaps):
    """Busy time per hardware queue / stream of one step and the longest idle gaps of the busiest
    one (the critical chain: a gap there is time the chain waited on the host or another stream)."""
    key = "Stream_Id" if "Stream_Id" in rows[0] else "Queue_Id"
    qs = {}
    for r in rows:
        qs.setdefault(r.get(key, "?"), []).append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    main_q = max(qs, key=lambda q: sum(e - s for s, e, _ in qs[q]))
    for q, iv in sorted(qs.items(), key=lambda kv: -len(kv[1])):
        busy = sum(e - s for s, e, _ in iv)
        span = iv[-1][1] - iv[0][0]
        print(f"    {key} {q}: {len(iv)} kernels, busy {busy / 1e6:.2f} ms over {span / 1e6:.2f} ms"
              + ("  <- busiest" if q == main_q else ""))
    for q, ivs in qs.items():
        by = {}
        for s_, e_, name in ivs:
            k = name.replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0][:70]
            t, c = by.get(k, (0, 0))
            by[k] = (t + e_ - s_, c + 1)
        print(f"    top kernels of {key} {q}:")
        for k, (t, c) in sorted(by.items(), key=lambda kv: -kv[1][0])[:14]:
            print(f"      {t / 1e3:8.1f} us {c:4d}x  {k}")
    iv = sorted(qs[main_q])
    gaps = sorted(((b[0] - a[1], a[2][:60], b[2][:60]) for a, b in zip(iv, iv[1:])), reverse=True)
    tot = sum(g for g, _, _ in gaps if g > 0)
    print(f"    busiest queue: {tot / 1e6:.2f} ms of gaps between its kernels; longest:")
    for g, a_, b_ in gaps[:ngaps]:
        print(f"      {g / 1e3:8.1f} us  after {a_}  before {b_}")


if __name__ == "__main__":
    main()

"""Critical-path view of steady-state steps from a rocprofv3 kernel trace (CSV): for the steps issued
with the host far ahead (bench.py's host-ahead window, after its spin kernel), per step: forward /
backward split on the compute stream (the first BN-backward kernel starts the backward), each
stream's busy time, the compute stream's idle gaps and what the other streams run meanwhile.

usage: python tools/crit_path.py gpurun_out/trace/run_kernel_trace.csv
"""
import csv
import sys
from collections import defaultdict


def short(n):
    n = n.replace("(anonymous namespace)::", "")
    return n.split("(")[0][:60]


def main():
    rows = []
    with open(sys.argv[1]) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), int(r["Stream_Id"]), r["Kernel_Name"]))
    rows.sort()
    spins = [i for i, r in enumerate(rows) if "spin_kernel" in r[3]]
    # the host-ahead window: after the last long spin kernel
    start = max(spins, key=lambda i: rows[i][1] - rows[i][0]) + 1
    win = rows[start:]
    ends = [r[1] for r in win if "sgd_kernel" in r[3]]
    if len(ends) < 3:
        print("not enough steps after the spin kernel")
        return 1
    for si in range(1, min(len(ends), 4)):
        t0, t1 = ends[si - 1], ends[si]
        step = [r for r in win if r[0] >= t0 and r[1] <= t1]
        main_s = 0
        busy = defaultdict(int)
        for s, e, st, n in step:
            busy[st] += e - s
        bwd0 = min((s for s, e, st, n in step if "bn_bwd" in n or "xent_bwd" in n), default=t1)
        print(f"step {si}: {(t1 - t0) / 1e3:.2f} ms  forward {(bwd0 - t0) / 1e3:.2f} ms  backward+update "
              f"{(t1 - bwd0) / 1e3:.2f} ms")
        for st in sorted(busy):
            print(f"   stream {st}: busy {busy[st] / 1e3:.2f} ms")
        ms = [r for r in step if r[2] == main_s]
        gaps = []
        prev = t0
        for s, e, st, n in ms:
            if s - prev > 20000:  # > 20 us idle
                others = defaultdict(int)
                for s2, e2, st2, n2 in step:
                    if st2 != main_s and e2 > prev and s2 < s:
                        others[short(n2)] += min(e2, s) - max(s2, prev)
                gaps.append((s - prev, prev - t0, short(n), sorted(others.items(), key=lambda kv: -kv[1])[:3]))
            prev = max(prev, e)
        tot = sum(g[0] for g in gaps)
        print(f"   compute-stream gaps > 20 us: {len(gaps)}, {tot / 1e3:.2f} ms; largest:")
        for g in sorted(gaps, reverse=True)[:8]:
            print(f"     {g[0] / 1e3:6.3f} ms at +{g[1] / 1e3:6.2f} before {g[2]}; others: "
                  + ", ".join(f"{k} {v / 1e3:.2f}" for k, v in g[3]))
    return 0


if __name__ == "__main__":
    sys.exit(main())

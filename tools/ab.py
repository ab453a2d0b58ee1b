#!/usr/bin/env python3
"""Alternating A/B of bench.py over environment toggles (one GPU).

    python tools/ab.py [--reps 2] [--mode eager] [--bench-args "..."] NAME=VAR=VAL[,VAR=VAL] ...

``base`` (no extra environment) always runs first in every repetition.  Each arm is one bench.py
process (its own autotune), so the spread between repetitions of the same arm is the noise floor.
Prints one line per run and a summary (best / mean ms_per_step per arm) and writes the JSON records to
gpurun_out/ab.json.
"""
import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--mode", default="eager")
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--timeout", type=int, default=300)
    ap.add_argument("--bench-args", default="")
    ap.add_argument("arms", nargs="*")
    a = ap.parse_args()
    arms = [("base", {})]
    for spec in a.arms:
        name, _, rest = spec.partition("=")
        env, last = {}, None
        for kv in rest.split(","):
            if "=" in kv:
                last, val = kv.split("=", 1)
                env[last] = val
            elif kv and last is not None:  # a comma inside a value (TONY_STREAMK=1,2)
                env[last] += "," + kv
        arms.append((name, env))
    out = {}
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    for rep in range(a.reps):
        for name, env in arms:
            cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--steps", str(a.steps), "--warmup", "6",
                   "--mode", a.mode] + a.bench_args.split()
            t = time.time()
            p = subprocess.run(cmd, env={**os.environ, **env}, capture_output=True, text=True, timeout=a.timeout)
            line = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
            if p.returncode != 0 or not line:
                print(f"{name} rep {rep}: FAILED rc={p.returncode}\n{p.stderr[-2000:]}", flush=True)
                return 1
            d = json.loads(line[-1])
            c = d["config"]
            out.setdefault(name, []).append(d)
            print(f"{name:14s} rep {rep}: {d['value']:9.1f} img/s  {d['ms_per_step']:7.3f} ms/step  host "
                  f"{c.get('host_ms_per_step')}  gpu_ahead {c.get('gpu_ms_per_step_host_ahead')}  "
                  f"({time.time() - t:.0f}s)", flush=True)
    print("summary (ms/step): arm, best, mean")
    for name, recs in out.items():
        ms = [r["ms_per_step"] for r in recs]
        print(f"  {name:14s} {min(ms):7.3f} {sum(ms) / len(ms):7.3f}")
    with open(os.path.join(ROOT, "gpurun_out", "ab.json"), "w") as f:
        json.dump(out, f)
    return 0


if __name__ == "__main__":
    sys.exit(main())

#!/usr/bin/env python3
"""Same-box A/B of whole source trees: bench.py of each tree, alternating, on one GPU.

    python tools/ab_trees.py [--reps 2] [--bench-args "..."] NAME=TREE_DIR [NAME=TREE_DIR ...]
                             [--arm NAME=TREE_DIR:VAR=VAL,VAR=VAL]

Every tree must hold its own built kernels (each tree's ``__graft_entry__.build()``); ``.`` is this tree.
A regression that box-to-box spread hides (boxes differ by 3-5 %) shows up here as a gap between arms
measured minutes apart on the same GPU.  Prints one line per run and a per-arm summary, and writes the
JSON records to gpurun_out/ab_trees.json.
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
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=6)
    ap.add_argument("--timeout", type=int, default=400)
    ap.add_argument("--bench-args", default="")
    ap.add_argument("arms", nargs="+")
    a = ap.parse_args()
    arms = []
    for spec in a.arms:
        name, _, rest = spec.partition("=")
        tree, _, envs = rest.partition(":")
        env = dict(kv.split("=", 1) for kv in envs.split(",") if "=" in kv)
        arms.append((name, os.path.abspath(os.path.join(ROOT, tree)), env))
    out = {}
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    for rep in range(a.reps):
        for name, tree, env in arms:
            cmd = [sys.executable, os.path.join(tree, "bench.py"), "--steps", str(a.steps), "--warmup",
                   str(a.warmup), "--fp32-row", "0"] + a.bench_args.split()
            t = time.time()
            p = subprocess.run(cmd, cwd=tree, env={**os.environ, **env}, capture_output=True, text=True,
                               timeout=a.timeout)
            line = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
            if p.returncode != 0 or not line:
                print(f"{name} rep {rep}: FAILED rc={p.returncode}\n{p.stderr[-2000:]}", flush=True)
                return 1
            d = json.loads(line[-1])
            c = d["config"]
            out.setdefault(name, []).append(d)
            print(f"{name:14s} rep {rep}: {d['value']:9.1f} img/s  {d['ms_per_step']:7.3f} ms/step  mode "
                  f"{c.get('step_mode')}  setup {c.get('mode_setup_ms')}  host {c.get('host_ms_per_step')}  "
                  f"gpu_ahead {c.get('gpu_ms_per_step_host_ahead')}  ({time.time() - t:.0f}s)", flush=True)
    print("summary (ms/step): arm, best, mean")
    for name, recs in out.items():
        ms = [r["ms_per_step"] for r in recs]
        print(f"  {name:14s} {min(ms):7.3f} {sum(ms) / len(ms):7.3f}")
    with open(os.path.join(ROOT, "gpurun_out", "ab_trees.json"), "w") as f:
        json.dump(out, f)
    return 0


if __name__ == "__main__":
    sys.exit(main())

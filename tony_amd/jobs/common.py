"""Shared plumbing of the reference jobs: device choice, synthetic data, metric lines, checkpoint dir."""
from __future__ import annotations

import json
import os
import sys
import time

import torch


def log(msg: str) -> None:
    print(f"[{os.environ.get('JOB_NAME', 'job')}:{os.environ.get('TASK_INDEX', '0')}] {msg}", flush=True)


def metric(**kv) -> None:
    """One machine-readable line per report (the training-metrics side channel)."""
    print("TONY_METRIC " + json.dumps(kv, sort_keys=True), flush=True)


def working_dir(default: str = "model") -> str:
    """Where checkpoints go: $TONY_WORKING_DIR, else <job dir>/<default> (shared by every task and
    by every session of a retried job, so a relaunched gang resumes), else ./<default>."""
    if os.environ.get("TONY_WORKING_DIR"):
        return os.environ["TONY_WORKING_DIR"]
    return os.path.join(os.environ.get("TONY_JOB_DIR", os.getcwd()), default)


class Throughput:
    def __init__(self, device: torch.device):
        self.device = device
        self.t0 = None
        self.n = 0

    def start(self):
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)
        self.t0 = time.perf_counter()
        self.n = 0

    def add(self, items: int):
        self.n += items

    def rate(self) -> float:
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)
        dt = time.perf_counter() - self.t0
        return self.n / dt if dt > 0 else 0.0


def synthetic_images(n: int, res: int, classes: int, device, dtype=torch.bfloat16, seed: int = 0):
    """Device-side RNG fill of an NHWC ImageNet-shaped batch."""
    g = torch.Generator(device=device).manual_seed(seed)
    x = torch.randn(n, 3, res, res, device=device, generator=g).to(dtype).contiguous(
        memory_format=torch.channels_last)
    y = torch.randint(0, classes, (n,), device=device, generator=g)
    return x, y


def exit_code(ok: bool) -> None:
    sys.exit(0 if ok else 1)

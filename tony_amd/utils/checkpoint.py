"""Checkpoint / resume helpers for the reference jobs.

TonY itself never checkpoints; its jobs rely on the framework (MonitoredTrainingSession's
``checkpoint_dir``, Estimator ``RunConfig(save_checkpoints_steps=1000, keep_checkpoint_max=3)``,
Horovod's rank-0 ``tf.train.Checkpoint``) writing to a shared path, and on the AM retry loop
relaunching the gang (``NUM_AM_RETRIES`` / ``SESSION_ID``).  ``CheckpointManager`` is that
framework piece here:

* ``save`` on the chief only (rank 0), every ``save_steps`` steps; tensors are copied
  device->host into pinned buffers on the calling stream and the file is written by a
  background thread, so the training loop only pays the D2H copy;
* files are written to ``ckpt-<step>.pt.tmp`` then renamed (a crash never leaves a
  half-written "latest"); only the newest ``keep_max`` are kept;
* ``restore`` loads with ``torch.load(weights_only=True)`` (no pickled code is executed).
"""
from __future__ import annotations

import os
import re
import threading
from typing import Any, Dict, List, Optional, Tuple

import torch

_NAME = re.compile(r"^ckpt-(\d+)\.pt$")


def _to_host(obj):
    if torch.is_tensor(obj):
        if obj.is_cuda:
            h = torch.empty(obj.shape, dtype=obj.dtype, pin_memory=True)
            h.copy_(obj, non_blocking=True)
            return h
        return obj.detach().clone()
    if isinstance(obj, dict):
        return {k: _to_host(v) for k, v in obj.items()}
    if isinstance(obj, (list, tuple)):
        return type(obj)(_to_host(v) for v in obj)
    return obj


class CheckpointManager:
    def __init__(self, directory: str, keep_max: int = 3, save_steps: int = 1000, rank: Optional[int] = None,
                 async_write: bool = True):
        self.dir = directory
        self.keep_max = max(1, int(keep_max))
        self.save_steps = int(save_steps)
        if rank is None:
            import torch.distributed as dist

            rank = dist.get_rank() if dist.is_available() and dist.is_initialized() else 0
        self.rank = rank
        self.async_write = async_write
        self._thread: Optional[threading.Thread] = None
        if self.is_chief:
            os.makedirs(directory, exist_ok=True)

    @property
    def is_chief(self) -> bool:
        return self.rank == 0

    def checkpoints(self) -> List[Tuple[int, str]]:
        try:
            names = os.listdir(self.dir)
        except OSError:
            return []
        out = []
        for n in names:
            m = _NAME.match(n)
            if m:
                out.append((int(m.group(1)), os.path.join(self.dir, n)))
        return sorted(out)

    def latest(self) -> Optional[Tuple[int, str]]:
        c = self.checkpoints()
        return c[-1] if c else None

    def should_save(self, step: int) -> bool:
        return self.save_steps > 0 and step > 0 and step % self.save_steps == 0

    def _write(self, step: int, state: Dict[str, Any]) -> None:
        path = os.path.join(self.dir, f"ckpt-{step}.pt")
        torch.save(state, path + ".tmp")
        os.replace(path + ".tmp", path)
        for _, old in self.checkpoints()[:-self.keep_max]:
            try:
                os.remove(old)
            except OSError:
                pass

    def save(self, step: int, state: Dict[str, Any], force: bool = False) -> Optional[str]:
        if not self.is_chief or not (force or self.should_save(step)):
            return None
        self.wait()
        host = _to_host(dict(state, step=step))
        if torch.cuda.is_available():
            torch.cuda.current_stream().synchronize()  # the pinned D2H copies above
        if self.async_write:
            self._thread = threading.Thread(target=self._write, args=(step, host), name="tony-ckpt", daemon=True)
            self._thread.start()
        else:
            self._write(step, host)
        return os.path.join(self.dir, f"ckpt-{step}.pt")

    def wait(self) -> None:
        if self._thread is not None:
            self._thread.join()
            self._thread = None

    def restore(self, map_location=None) -> Optional[Dict[str, Any]]:
        lt = self.latest()
        if lt is None:
            return None
        return torch.load(lt[1], map_location=map_location, weights_only=True)


def training_state(model: Optional[torch.nn.Module] = None, optimizer=None, ps=None, **extra) -> Dict[str, Any]:
    """The usual checkpoint payload: module state, torch/flat optimizer state or a ParameterServer."""
    st: Dict[str, Any] = dict(extra)
    if model is not None:
        st["model"] = model.state_dict()
    if optimizer is not None:
        st["optimizer"] = optimizer.state_dict()
    if ps is not None:
        st["ps"] = ps.state_dict()
    return st


def resume_step(state: Optional[Dict[str, Any]]) -> int:
    return int(state["step"]) if state else 0

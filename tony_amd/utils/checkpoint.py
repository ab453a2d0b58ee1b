"""Checkpoint / resume helpers for the reference jobs.

TonY itself never checkpoints; its jobs rely on the framework (MonitoredTrainingSession's
``checkpoint_dir``, Estimator ``RunConfig(save_checkpoints_steps=1000, keep_checkpoint_max=3)``,
Horovod's rank-0 ``tf.train.Checkpoint``) writing to a shared path, and on the AM retry loop
relaunching the gang (``NUM_AM_RETRIES`` / ``SESSION_ID``; reference
``T/ApplicationMaster.java:406-422``, ``EX/mnist-tensorflow/mnist_distributed.py:237-241``).
``CheckpointManager`` is that framework piece here:

* ``save`` every ``save_steps`` steps -- on the chief only (rank 0), or, with ``sharded=True``, on
  EVERY rank: each rank of a sharded parameter server owns different variables' fp32 master copy
  and optimizer state, so each writes ``ckpt-<step>-shard<r>-of-<N>.pt`` (TF's PS checkpoints are
  likewise one shard per ps task);
* tensors are copied device->host into pinned buffers on the calling stream and the file is
  written by a background thread, so the training loop only pays the D2H copy;
* files are written to ``*.tmp`` then renamed (a crash never leaves a half-written checkpoint);
  a sharded step counts only once all N shards exist, and ranks agree on the newest complete
  step before restoring; only the newest ``keep_max`` are kept;
* ``restore`` loads with ``torch.load(weights_only=True)`` (no pickled code is executed).
"""
from __future__ import annotations

import os
import re
import threading
from typing import Any, Dict, List, Optional, Tuple

import torch

_NAME = re.compile(r"^ckpt-(\d+)\.pt$")
_SHARD = re.compile(r"^ckpt-(\d+)-shard(\d+)-of-(\d+)\.pt$")


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


def _dist():
    import torch.distributed as dist

    return dist if dist.is_available() and dist.is_initialized() else None


class CheckpointManager:
    def __init__(self, directory: str, keep_max: int = 3, save_steps: int = 1000, rank: Optional[int] = None,
                 async_write: bool = True, sharded: bool = False, world: Optional[int] = None):
        self.dir = directory
        self.keep_max = max(1, int(keep_max))
        self.save_steps = int(save_steps)
        d = _dist()
        if rank is None:
            rank = d.get_rank() if d else 0
        if world is None:
            world = d.get_world_size() if d else 1
        self.rank = rank
        self.world = int(world)
        self.sharded = bool(sharded)
        self.async_write = async_write
        self._thread: Optional[threading.Thread] = None
        if self.is_chief or self.sharded:
            os.makedirs(directory, exist_ok=True)

    @property
    def is_chief(self) -> bool:
        return self.rank == 0

    def _path(self, step: int, rank: Optional[int] = None) -> str:
        if not self.sharded:
            return os.path.join(self.dir, f"ckpt-{step}.pt")
        r = self.rank if rank is None else rank
        return os.path.join(self.dir, f"ckpt-{step}-shard{r}-of-{self.world}.pt")

    def checkpoints(self) -> List[Tuple[int, str]]:
        """(step, path of THIS rank's file) of every complete checkpoint, oldest first."""
        try:
            names = os.listdir(self.dir)
        except OSError:
            return []
        out = []
        if not self.sharded:
            for n in names:
                m = _NAME.match(n)
                if m:
                    out.append((int(m.group(1)), os.path.join(self.dir, n)))
            return sorted(out)
        shards: Dict[int, set] = {}
        for n in names:
            m = _SHARD.match(n)
            if m and int(m.group(3)) == self.world:
                shards.setdefault(int(m.group(1)), set()).add(int(m.group(2)))
        for step, have in shards.items():
            if have == set(range(self.world)):
                out.append((step, self._path(step)))
        return sorted(out)

    def latest(self) -> Optional[Tuple[int, str]]:
        c = self.checkpoints()
        return c[-1] if c else None

    def should_save(self, step: int) -> bool:
        return self.save_steps > 0 and step > 0 and step % self.save_steps == 0

    def _write(self, step: int, state: Dict[str, Any]) -> None:
        path = self._path(step)
        torch.save(state, path + ".tmp")
        os.replace(path + ".tmp", path)
        if self.sharded:  # prune this rank's own old shards only
            mine = sorted(int(m.group(1)) for m in (_SHARD.match(n) for n in os.listdir(self.dir))
                          if m and int(m.group(2)) == self.rank and int(m.group(3)) == self.world)
            old = [self._path(s) for s in mine[:-self.keep_max]]
        else:
            old = [p for _, p in self.checkpoints()[:-self.keep_max]]
        for p in old:
            try:
                os.remove(p)
            except OSError:
                pass

    def save(self, step: int, state: Dict[str, Any], force: bool = False) -> Optional[str]:
        if not (self.is_chief or self.sharded) or not (force or self.should_save(step)):
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
        return self._path(step)

    def wait(self) -> None:
        if self._thread is not None:
            self._thread.join()
            self._thread = None

    def agreed_latest(self, device=None) -> Optional[Tuple[int, str]]:
        """The newest step complete for every rank (collective when a process group is up)."""
        lt = self.latest()
        d = _dist()
        if not self.sharded or d is None or d.get_world_size() == 1:
            return lt
        dev = device if device is not None else (
            torch.device("cuda", torch.cuda.current_device()) if d.get_backend() == "nccl" else torch.device("cpu"))
        t = torch.tensor([lt[0] if lt else -1], dtype=torch.int64, device=dev)
        d.all_reduce(t, op=d.ReduceOp.MIN)
        step = int(t.item())
        if step < 0:
            return None
        return step, self._path(step)

    def restore(self, map_location=None, device=None) -> Optional[Dict[str, Any]]:
        lt = self.agreed_latest(device) if self.sharded else self.latest()
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

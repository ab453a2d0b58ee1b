"""Horovod-compatible API on torch.distributed (RCCL over xGMI), for jobs launched by the horovod runtime.

``import tony_amd.hvd as hvd`` gives the calls the reference's Horovod examples
use (EX/horovod-on-tony/tensorflow2_mnist.py:32-101, tensorflow2_keras_mnist.py:55-75):
``init / rank / size / local_rank / local_size / cross_rank / cross_size``,
``allreduce(_async)(_)``, ``allgather``, ``broadcast(_)``, ``alltoall``,
``broadcast_parameters``, ``broadcast_optimizer_state``, ``broadcast_object``,
``allgather_object``, ``DistributedOptimizer`` (fusion-buffer gradient averaging
overlapped with backward), ``Compression``, ``join``, ``barrier``, ``shutdown``.

Rendezvous: the horovod runtime exports ``HOROVOD_RANK/SIZE/LOCAL_RANK/...`` and
``HOROVOD_GLOO_RENDEZVOUS_ADDR/PORT`` (T/runtime/HorovodRuntime.java:318-349);
rank 0 serves a TCPStore and publishes it in that HTTP KV.  The data plane is
RCCL (``nccl`` backend) on GPU ranks and gloo on CPU ranks -- Horovod's own
``HOROVOD_CPU_OPERATIONS=gloo`` is honoured by using gloo for CPU tensors.
"""
from __future__ import annotations

import io
import os
from typing import Dict, Iterable, List, Optional, Tuple

import torch
import torch.distributed as dist

from . import bootstrap
from .ddp import DEFAULT_BUCKET_MB, BucketedAllReduce
from .flat import FlatParams


class _Op:
    def __init__(self, name):
        self.name = name

    def __repr__(self):
        return self.name


Average, Sum, Adasum, Min, Max, Product = (_Op(n) for n in ("Average", "Sum", "Adasum", "Min", "Max", "Product"))

_state: Dict[str, object] = {"init": False}


class Compression:
    """Wire compression for gradients (horovod.torch.Compression)."""

    class none:  # noqa: N801
        dtype = None

    class fp16:  # noqa: N801
        dtype = torch.float16

    class bf16:  # noqa: N801 - the native MI355X choice
        dtype = torch.bfloat16


def init(comm=None) -> None:  # noqa: ARG001 - MPI communicators do not exist here
    if _state["init"]:
        return
    env = os.environ
    if "HOROVOD_RANK" in env:
        rank, size = int(env["HOROVOD_RANK"]), int(env["HOROVOD_SIZE"])
        local, local_size = int(env.get("HOROVOD_LOCAL_RANK", rank)), int(env.get("HOROVOD_LOCAL_SIZE", size))
        cross, cross_size = int(env.get("HOROVOD_CROSS_RANK", 0)), int(env.get("HOROVOD_CROSS_SIZE", 1))
        store = None
        if size > 1:
            key = f"tony/torch-store/{env.get('SESSION_ID', '0')}"
            store = bootstrap.store_via_kv(env["HOROVOD_GLOO_RENDEZVOUS_ADDR"],
                                           int(env["HOROVOD_GLOO_RENDEZVOUS_PORT"]), rank, size, key)
        dev = bootstrap.init_process_group(rank, size, store=store or dist.HashStore(), local_rank=local)
    else:
        rank, size, local, dev = bootstrap.init_from_env()
        local_size, cross, cross_size = int(env.get("LOCAL_WORLD_SIZE", size)), 0, 1
    _state.update(init=True, rank=rank, size=size, local_rank=local, local_size=local_size, cross_rank=cross,
                  cross_size=cross_size, device=dev, handles={}, next_handle=0)


def _need_init():
    if not _state["init"]:
        raise ValueError("Horovod has not been initialized; use hvd.init().")


def is_initialized() -> bool:
    return bool(_state["init"])


def rank() -> int:
    _need_init()
    return _state["rank"]


def size() -> int:
    _need_init()
    return _state["size"]


def local_rank() -> int:
    _need_init()
    return _state["local_rank"]


def local_size() -> int:
    _need_init()
    return _state["local_size"]


def cross_rank() -> int:
    _need_init()
    return _state["cross_rank"]


def cross_size() -> int:
    _need_init()
    return _state["cross_size"]


def device() -> torch.device:
    _need_init()
    return _state["device"]


def mpi_threads_supported() -> bool:
    return False


def mpi_enabled() -> bool:
    return False


def gloo_enabled() -> bool:
    return True


def nccl_built() -> bool:
    return True  # RCCL


def rocm_built() -> bool:
    return True


def cuda_built() -> bool:
    return False


def _reduce_op(op) -> Tuple[dist.ReduceOp, bool]:
    """(torch op, divide-by-size afterwards)."""
    if op is None or op is Average:
        return dist.ReduceOp.SUM, True
    if op is Adasum:
        raise NotImplementedError("Adasum is not supported; use Average or Sum")
    return {Sum: dist.ReduceOp.SUM, Min: dist.ReduceOp.MIN, Max: dist.ReduceOp.MAX,
            Product: dist.ReduceOp.PRODUCT}[op], False


def _resolve_op(average, op):
    if average is not None:
        return Average if average else Sum
    return op if op is not None else Average


class _Handle:
    def __init__(self, work, out, post):
        self.work, self.out, self.post = work, out, post


def allreduce_async_(tensor: torch.Tensor, average=None, name=None, op=None, prescale_factor=1.0,
                     postscale_factor=1.0, process_set=None) -> int:  # noqa: ARG001
    _need_init()
    op = _resolve_op(average, op)
    top, div = _reduce_op(op)
    if prescale_factor != 1.0:
        tensor.mul_(prescale_factor)
    work = dist.all_reduce(tensor, op=top, async_op=True) if _state["size"] > 1 else None
    scale = postscale_factor / (_state["size"] if div else 1)
    h = _state["next_handle"]
    _state["next_handle"] = h + 1
    _state["handles"][h] = _Handle(work, tensor, scale)
    return h


def synchronize(handle: int) -> torch.Tensor:
    h = _state["handles"].pop(handle)
    if h.work is not None:
        h.work.wait()
    if h.post != 1.0:
        if h.out.is_floating_point():
            h.out.mul_(h.post)
        else:
            h.out.copy_(torch.div(h.out, round(1 / h.post), rounding_mode="floor"))
    return h.out


def poll(handle: int) -> bool:
    h = _state["handles"].get(handle)
    return h is None or h.work is None or h.work.is_completed()


def allreduce_(tensor, average=None, name=None, op=None, **kw):
    return synchronize(allreduce_async_(tensor, average, name, op, **kw))


def allreduce_async(tensor, average=None, name=None, op=None, **kw) -> int:
    return allreduce_async_(tensor.clone(), average, name, op, **kw)


def allreduce(tensor, average=None, name=None, compression=Compression.none, op=None, **kw):
    wire = tensor.to(compression.dtype) if compression.dtype is not None and tensor.is_floating_point() \
        else tensor.clone()
    out = allreduce_(wire, average, name, op, **kw)
    return out.to(tensor.dtype)


def grouped_allreduce(tensors: List[torch.Tensor], average=None, name=None, op=None, **kw):
    """One fused collective over a list: pack into one buffer, reduce, unpack."""
    if not tensors:
        return []
    flat = torch.cat([t.reshape(-1) for t in tensors])
    allreduce_(flat, average, name, op, **kw)
    out, off = [], 0
    for t in tensors:
        out.append(flat[off:off + t.numel()].view_as(t))
        off += t.numel()
    return out


def allgather(tensor: torch.Tensor, name=None) -> torch.Tensor:  # noqa: ARG001
    """Concatenate along dim 0; the first dimension may differ between ranks."""
    _need_init()
    n = _state["size"]
    if n == 1:
        return tensor.clone()
    dim0 = torch.tensor([tensor.shape[0]], dtype=torch.int64, device=tensor.device)
    sizes = [torch.zeros_like(dim0) for _ in range(n)]
    dist.all_gather(sizes, dim0)
    sizes = [int(s.item()) for s in sizes]
    mx = max(sizes)
    pad = torch.zeros((mx,) + tuple(tensor.shape[1:]), dtype=tensor.dtype, device=tensor.device)
    pad[:tensor.shape[0]] = tensor
    parts = [torch.empty_like(pad) for _ in range(n)]
    dist.all_gather(parts, pad)
    return torch.cat([p[:s] for p, s in zip(parts, sizes)])


def broadcast_(tensor: torch.Tensor, root_rank: int, name=None) -> torch.Tensor:  # noqa: ARG001
    _need_init()
    if _state["size"] > 1:
        dist.broadcast(tensor, root_rank)
    return tensor


def broadcast(tensor: torch.Tensor, root_rank: int, name=None) -> torch.Tensor:
    return broadcast_(tensor.clone(), root_rank, name)


def alltoall(tensor: torch.Tensor, splits: Optional[List[int]] = None, name=None):  # noqa: ARG001
    _need_init()
    n = _state["size"]
    if splits is None:
        if tensor.shape[0] % n:
            raise ValueError("tensor dim 0 must divide evenly without splits")
        splits = [tensor.shape[0] // n] * n
    send = torch.tensor(splits, dtype=torch.int64, device=tensor.device)
    recv = torch.empty_like(send)
    if n == 1:
        return tensor.clone()
    dist.all_to_all_single(recv, send)
    rsplits = [int(v) for v in recv.tolist()]
    out = torch.empty((sum(rsplits),) + tuple(tensor.shape[1:]), dtype=tensor.dtype, device=tensor.device)
    dist.all_to_all_single(out, tensor.contiguous(), rsplits, list(splits))
    return out


def barrier() -> None:
    _need_init()
    if _state["size"] > 1:
        dist.barrier()


def join(device=None) -> int:  # noqa: ARG001
    """All ranks reached the end; returns the last rank to join (here: a barrier)."""
    barrier()
    return _state["size"] - 1


def broadcast_object(obj, root_rank: int = 0, name=None):  # noqa: ARG001
    _need_init()
    if _state["size"] == 1:
        return obj
    box = [obj if _state["rank"] == root_rank else None]
    dist.broadcast_object_list(box, src=root_rank)
    return box[0]


def allgather_object(obj, name=None) -> list:  # noqa: ARG001
    _need_init()
    out = [None] * _state["size"]
    if _state["size"] == 1:
        return [obj]
    dist.all_gather_object(out, obj)
    return out


def broadcast_parameters(params, root_rank: int = 0) -> None:
    """``params``: a state_dict / named_parameters() / list of (name, tensor)."""
    items = sorted(params.items()) if isinstance(params, dict) else list(params)
    for _, p in items:
        t = p.data if isinstance(p, torch.nn.Parameter) else p
        if torch.is_tensor(t):
            broadcast_(t, root_rank)


def broadcast_optimizer_state(optimizer: torch.optim.Optimizer, root_rank: int = 0) -> None:
    """Make every rank's optimizer state (slots + hyper-parameters) equal to ``root_rank``'s."""
    sd = optimizer.state_dict()
    # materialise slots that only exist after a first step so every rank has the same structure
    buf = io.BytesIO()
    torch.save(sd, buf) if _state["rank"] == root_rank else None
    payload = broadcast_object(buf.getvalue() if _state["rank"] == root_rank else None, root_rank)
    if _state["rank"] != root_rank:
        dev = next((p.device for g in optimizer.param_groups for p in g["params"]), torch.device("cpu"))
        new = torch.load(io.BytesIO(payload), map_location=dev, weights_only=True)
        optimizer.load_state_dict(new)


class _DistributedOptimizer:
    """Wraps a torch optimizer: gradients are averaged (bucketed, overlapped) before ``step``.

    Parameters are re-homed into one flat buffer per dtype (rank 0's values),
    each dtype group gets a :class:`BucketedAllReduce` whose buckets launch from
    the gradient hooks during backward.
    """

    def __init__(self, optimizer, named_parameters=None, compression=Compression.none,
                 backward_passes_per_step: int = 1, op=Average, bucket_mb: float = DEFAULT_BUCKET_MB,
                 gradient_predivide_factor: float = 1.0, fused: Optional[bool] = None):
        _need_init()
        if op not in (Average, Sum):
            raise ValueError("DistributedOptimizer supports op=Average or op=Sum")
        self.optimizer = optimizer
        self.backward_passes_per_step = int(backward_passes_per_step)
        params = [p for g in optimizer.param_groups for p in g["params"] if p.requires_grad]
        if named_parameters is not None:  # Horovod's check: names must cover every optimized parameter
            named = list(named_parameters)
            names = [n for n, _ in named]
            if len(set(names)) != len(names):
                raise ValueError("named_parameters has duplicate names")
            known = {id(p) for _, p in named}
            missing = [i for i, p in enumerate(params) if id(p) not in known]
            if missing:
                raise ValueError(f"named_parameters does not cover {len(missing)} optimizer parameter(s)")
        by_dtype: Dict[torch.dtype, List[torch.nn.Parameter]] = {}
        for p in params:
            by_dtype.setdefault(p.dtype, []).append(p)
        self.groups = []
        for dt, ps in by_dtype.items():
            m = torch.nn.Module()
            for i, p in enumerate(ps):
                m.register_parameter(f"p{i}", p)
            flat = FlatParams(m, dtype=dt, world=1)
            if _state["size"] > 1:
                dist.broadcast(flat.data, 0)
            red = BucketedAllReduce(flat, bucket_mb, average=(op is Average), compression=compression.dtype,
                                    predivide=gradient_predivide_factor if op is Average else 1.0)
            red.passes_per_reduce = self.backward_passes_per_step
            red.register_hooks()
            self.groups.append((flat, red))
        # fused apply: a single-group torch SGD on GPU tensors becomes ONE fused HIP SGD-momentum launch
        # per flat buffer (fp32 master + momentum, writes the bf16 compute copy; ops/optim.py)
        self._fused = []
        can_fuse = (isinstance(optimizer, torch.optim.SGD) and len(optimizer.param_groups) == 1
                    and all(f.device.type == "cuda" for f, _ in self.groups)
                    and not optimizer.param_groups[0].get("dampening", 0)
                    and not optimizer.param_groups[0].get("maximize", False))
        if fused is None:
            fused = can_fuse
        elif fused and not can_fuse:
            raise ValueError("fused=True needs a single-group, dampening-free torch.optim.SGD on GPU tensors")
        if fused:
            from ..ops.optim import FlatSGD

            g = optimizer.param_groups[0]
            for flat, _ in self.groups:
                # an fp32 flat buffer IS the master (nothing to keep in sync); a bf16 one gets an fp32
                # master that re-seeds from any element changed behind the optimizer's back (resync)
                master = flat.data if flat.data.dtype == torch.float32 else flat.data.float().clone()
                self._fused.append((flat, FlatSGD(master, g["lr"], momentum=g["momentum"],
                                                  weight_decay=g["weight_decay"], nesterov=g["nesterov"],
                                                  resync=master is not flat.data)))
            # torch-SGD state index of every parameter -> (flat buffer, slot)
            slot_of = {}
            for fi, (flat, _) in enumerate(self.groups):
                for slot, p in zip(flat.slots, flat.params):
                    slot_of[id(p)] = (fi, slot)
            self._slots = [slot_of.get(id(p)) for p in optimizer.param_groups[0]["params"]]

    # torch.optim.Optimizer surface
    @property
    def param_groups(self):
        return self.optimizer.param_groups

    @property
    def state(self):
        return self.optimizer.state

    def state_dict(self):
        """torch.optim.SGD's state_dict format; with the fused apply the momentum buffers are views of
        the flat fp32 momentum (the wrapped optimizer never steps, so its own state is empty)."""
        sd = self.optimizer.state_dict()
        if not self._fused:
            return sd
        state = {}
        for i, fs in enumerate(self._slots):
            if fs is None:  # a frozen parameter: no state
                continue
            fi, slot = fs
            opt = self._fused[fi][1]
            if opt.step_count and self.optimizer.param_groups[0]["momentum"]:
                state[i] = {"momentum_buffer": slot.view(opt.v).clone()}
        sd["state"] = state
        return sd

    def load_state_dict(self, sd):
        self.optimizer.load_state_dict(sd)
        if not self._fused:
            return
        g = self.optimizer.param_groups[0]
        for fi, (_, opt) in enumerate(self._fused):
            opt.v.zero_()
            opt.lr, opt.momentum, opt.weight_decay = g["lr"], g["momentum"], g["weight_decay"]
        for i, st in sd.get("state", {}).items():
            buf = st.get("momentum_buffer") if isinstance(st, dict) else None
            if buf is None:
                continue
            fs = self._slots[int(i)]
            if fs is None:
                continue
            fi, slot = fs
            opt = self._fused[fi][1]
            with torch.no_grad():
                slot.view(opt.v).copy_(buf.to(device=opt.v.device, dtype=torch.float32))
            opt.step_count = max(opt.step_count, 1)

    def zero_grad(self, set_to_none: bool = False):  # noqa: ARG002 - grads are views of the flat buffers
        for flat, _ in self.groups:
            flat.zero_grad()
            flat.rebind_grads()

    def synchronize(self):
        """Grads are already averaged when backward returns; kept for API parity."""

    def step(self, closure=None):
        """Call after ``backward_passes_per_step`` backward passes (their sum is averaged)."""
        if not self._fused:
            return self.optimizer.step(closure)
        loss = closure() if closure is not None else None
        g = self.optimizer.param_groups[0]  # lr schedules edit the wrapped optimizer's group
        for flat, opt in self._fused:
            opt.lr, opt.momentum, opt.weight_decay = g["lr"], g["momentum"], g["weight_decay"]
            if opt.w is flat.data:
                opt.step(flat.grad)  # fp32: updated in place
            else:
                opt.step(flat.grad, out_bf16=flat.data)
        return loss

    def __getattr__(self, name):
        return getattr(self.optimizer, name)


def DistributedOptimizer(optimizer, named_parameters=None, compression=Compression.none,  # noqa: N802
                         backward_passes_per_step: int = 1, op=Average, **kw):
    """Horovod's DistributedOptimizer: bucketed gradient averaging overlapped with backward; a plain
    torch SGD on GPU tensors is applied by the fused HIP kernel (``fused=False`` keeps torch's)."""
    return _DistributedOptimizer(optimizer, named_parameters, compression, backward_passes_per_step, op, **kw)


def shutdown() -> None:
    if _state["init"] and dist.is_initialized():
        dist.destroy_process_group()
    _state.clear()
    _state["init"] = False


def allreduce_parameters_stats(params: Iterable[torch.Tensor]) -> List[torch.Tensor]:
    """MetricAverageCallback equivalent: average a list of scalars/tensors across ranks."""
    return [allreduce(torch.as_tensor(p, dtype=torch.float32)) for p in params]

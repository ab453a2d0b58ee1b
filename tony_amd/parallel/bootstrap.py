"""Process-group bootstrap from the env contracts the TonY runtimes inject.

One process per GPU, ``torch.distributed`` with the ``nccl`` backend (= RCCL
over xGMI) when the process sees a GPU, ``gloo`` otherwise.  Every runtime of
``tony_amd.runtime`` gives the user process enough to form the group:

pytorch     MASTER_ADDR / MASTER_PORT / RANK / WORLD_SIZE / LOCAL_RANK
            (plus TonY's INIT_METHOD / RANK / WORLD, T/runtime/PyTorchRuntime.java:45-56)
tensorflow  TF_CONFIG (T/runtime/TFRuntime.java:45-59) -> see :mod:`tony_amd.parallel.tf_config`
horovod     HOROVOD_RANK / SIZE / LOCAL_RANK + HOROVOD_GLOO_RENDEZVOUS_ADDR/PORT
            (T/runtime/HorovodRuntime.java:318-349): rank 0 serves a TCPStore and
            publishes its address in the rendezvous KV
mxnet       DMLC_ROLE / DMLC_PS_ROOT_URI / DMLC_PS_ROOT_PORT (T/runtime/MXNetRuntime.java:44-66)
            -> see :mod:`tony_amd.parallel.kvstore`
"""
from __future__ import annotations

import datetime
import os
import time
from typing import Optional

import torch
import torch.distributed as dist

DEFAULT_TIMEOUT = datetime.timedelta(seconds=int(os.environ.get("TONY_DIST_TIMEOUT_S", "1800")))


def default_backend() -> str:
    forced = os.environ.get("TONY_DIST_BACKEND")
    if forced:
        return forced
    return "nccl" if torch.cuda.is_available() else "gloo"


def pick_device(local_rank: int) -> torch.device:
    """The task's GPU: the first of TONY_HIP_ORDINALS when the launcher pinned it with every GPU
    visible (visible-devices-mode none, the default), else ``local_rank`` (index 0 under a per-task
    HIP_VISIBLE_DEVICES, or torchrun's LOCAL_RANK)."""
    if not torch.cuda.is_available():
        return torch.device("cpu")
    n = torch.cuda.device_count()
    ords = [int(o) for o in os.environ.get("TONY_HIP_ORDINALS", "").split(",") if o.strip()]
    if ords and os.environ.get("TONY_VISIBLE_MODE", "none") == "none" and ords[0] < n:
        dev = torch.device("cuda", ords[0])
    else:
        dev = torch.device("cuda", local_rank % n)
    torch.cuda.set_device(dev)
    from ..gpu.inventory import verify_visible_device

    verify_visible_device(dev.index)  # the coordinator's pinned BDF == the device HIP shows (raises if not)
    return dev


def _advertised_host() -> str:
    # same rule as the coordinator's cluster spec (utils.core.current_host): loopback on one node
    return os.environ.get("TONY_ADVERTISE_HOST") or os.environ.get("TONY_HOST", "127.0.0.1")


def store_via_kv(kv_addr: str, kv_port: int, rank: int, world: int, key: str = "tony/torch-store",
                 timeout: datetime.timedelta = DEFAULT_TIMEOUT) -> dist.TCPStore:
    """Rank 0 serves a TCPStore on an ephemeral port and publishes ``host:port`` in the HTTP KV."""
    from ..horovod.rendezvous import kv_get, kv_put

    if rank == 0:
        host = _advertised_host()
        store = dist.TCPStore("0.0.0.0", 0, world, True, timeout=timeout, wait_for_workers=False)
        kv_put(kv_addr, kv_port, key, f"{host}:{store.port}".encode())
        return store
    addr = kv_get(kv_addr, kv_port, key, timeout.total_seconds()).decode()
    host, port = addr.rsplit(":", 1)
    return dist.TCPStore(host, int(port), world, False, timeout=timeout)


def init_process_group(rank: int, world: int, store: Optional[dist.Store] = None, master_addr: Optional[str] = None,
                       master_port: Optional[int] = None, backend: Optional[str] = None,
                       timeout: datetime.timedelta = DEFAULT_TIMEOUT, local_rank: Optional[int] = None):
    """Form the world group once; returns the device of this rank."""
    dev = pick_device(rank if local_rank is None else local_rank)
    if dist.is_initialized():
        return dev
    backend = backend or default_backend()
    kw = {}
    if backend == "nccl" and dev.type == "cuda":
        kw["device_id"] = dev  # eager RCCL communicator init, bound to this rank's GPU
    if store is None:
        if master_addr is None:
            raise ValueError("need a store or master_addr/master_port")
        store = dist.TCPStore(master_addr, int(master_port), world, rank == 0, timeout=timeout,
                              wait_for_workers=False)
    dist.init_process_group(backend, store=store, rank=rank, world_size=world, timeout=timeout, **kw)
    from ..utils.tracing import arm_from_env

    arm_from_env()  # TONY_HANG_DUMP_S: dump every thread's stack when a rank stops making progress
    return dev


def init_from_env(backend: Optional[str] = None):
    """Initialise from whichever contract is present.  Returns (rank, world, local_rank, device).  A process
    group that already exists (e.g. torch.distributed.run's env:// rendezvous) is used as it is."""
    env = os.environ
    if dist.is_initialized():
        rank, world = dist.get_rank(), dist.get_world_size()
        local = int(env.get("LOCAL_RANK", env.get("HOROVOD_LOCAL_RANK", rank)))
        dev = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else pick_device(local)
        return rank, world, local, dev
    if "HOROVOD_RANK" in env:
        rank, world = int(env["HOROVOD_RANK"]), int(env["HOROVOD_SIZE"])
        local = int(env.get("HOROVOD_LOCAL_RANK", rank))
        store = store_via_kv(env["HOROVOD_GLOO_RENDEZVOUS_ADDR"], int(env["HOROVOD_GLOO_RENDEZVOUS_PORT"]),
                             rank, world) if world > 1 else None
    elif "TF_CONFIG" in env:
        from .tf_config import TFConfig

        tc = TFConfig.from_env()
        rank, world, local = tc.rank, tc.world, tc.local_rank
        store = None
        if world > 1:
            host, port = tc.master_address
            store = dist.TCPStore(host, port, world, rank == 0, timeout=DEFAULT_TIMEOUT, wait_for_workers=False)
    elif "WORLD_SIZE" in env or "WORLD" in env:
        world = int(env.get("WORLD_SIZE", env.get("WORLD", "1")))
        rank = int(env.get("RANK", "0"))
        local = int(env.get("LOCAL_RANK", rank))
        store = None
        if world > 1:
            addr, port = env.get("MASTER_ADDR"), env.get("MASTER_PORT")
            if addr is None and env.get("INIT_METHOD", "").startswith("tcp://"):
                addr, port = env["INIT_METHOD"][len("tcp://"):].rsplit(":", 1)
            store = dist.TCPStore(addr, int(port), world, rank == 0, timeout=DEFAULT_TIMEOUT,
                                  wait_for_workers=False)
    else:
        rank, world, local, store = 0, 1, 0, None
    if world == 1 and store is None:
        store = dist.HashStore()
    dev = init_process_group(rank, world, store=store, backend=backend, local_rank=local)
    return rank, world, local, dev


def init_from_tf_config(tc, backend: Optional[str] = None):
    """Group over ``tc``'s rank table (see TFConfig.without_ps).  Returns (rank, world, device)."""
    rank, world = tc.rank, tc.world
    if rank < 0:
        raise ValueError(f"{tc.task_type}:{tc.task_index} is not a member of the training group")
    store = dist.HashStore()
    if world > 1:
        host, port = tc.master_address
        store = dist.TCPStore(host if rank else "0.0.0.0", port, world, rank == 0, timeout=DEFAULT_TIMEOUT,
                              wait_for_workers=False)
    dev = init_process_group(rank, world, store=store, backend=backend, local_rank=tc.local_rank)
    return rank, world, dev


def wait_for(predicate, timeout_s: float, poll_s: float = 0.01) -> bool:
    end = time.time() + timeout_s
    while time.time() < end:
        if predicate():
            return True
        time.sleep(poll_s)
    return predicate()

"""MXNet-style key-value store (``mx.kv``) for jobs launched by TonY's mxnet runtime.

TonY's mxnet runtime (T/runtime/MXNetRuntime.java:44-66) starts ``scheduler``,
``server`` and ``worker`` tasks with ``DMLC_ROLE / DMLC_PS_ROOT_URI /
DMLC_PS_ROOT_PORT / DMLC_NUM_SERVER / DMLC_NUM_WORKER``; the reference job
(EX/linearregression-mxnet/src/mxnet_dist_ex.py:35,61-68) trains through
``mx.kv.create('dist_async')``.  MXNet/ps-lite are not part of this stack, so
this module implements the kvstore semantics itself:

``local`` / ``device``
    one process; ``push`` sums the pushed list, the updater (if set) runs on
    the stored value, ``pull`` copies it out.
``dist_sync``
    servers own the keys (key id mod #servers).  A push round completes when
    every worker has pushed a key; the server then applies the optimizer to
    the *sum* (or stores the sum), and a worker's pull issued after its own
    push waits for that round -- the BSP semantics of ps-lite's sync mode.
``dist_async``
    every push is applied on arrival; pulls return the current value.
``dist_device_sync``
    no servers in the data path: the workers all-reduce the pushed gradients
    with RCCL (the xGMI path for GPU tensors) and run the same updater on
    every worker (replicated, deterministic).

Transport for the server modes: one torch.distributed (gloo) group over
servers + workers; the scheduler task hosts its TCPStore on
``DMLC_PS_ROOT_PORT`` and exits when every member has finished.  Requests are
an int64 header ``[op, key, numel, dtype]`` followed by the payload.

GPU payload plane (``TONY_KV_PLANE=xgmi``, the default when every member sees a GPU): every member
allocates an IPC-mapped window on its GPU (csrc/ps_plane.hip) and maps its peers' -- a worker the
servers', a server the workers'.  A pushed GPU tensor is stored by a copy kernel straight into its
row of the owning server's window and only the header goes over gloo; the server replies to a pull
by storing the value into the worker's landing area.  Neither side waits on the host: every copy
kernel's workgroups add to a u32 counter in the consumer's window header after their bytes
(``tony_kv_copy_flag``), and the consumer's stream waits on the device for the counter to reach the
copy's cumulative total (``tony_kv_wait``, bounded by ``TONY_KV_WAIT_S``; a timeout sets the window's
error word, which ``barrier`` / ``close`` raise) before the kernel that reads the bytes.  The payload
bytes never leave the GPUs (xGMI between devices; the server may share a worker's GPU, like TonY's
0-GPU ps).  Keys that do not fit the windows (``TONY_KV_WINDOW_MB``) or the flag tables, and CPU
tensors, keep the gloo payload.  A worker re-pushing a key before pulling it (its last row may not have
been read yet) sends that push over gloo: the pull's reply is what orders the server's read of the row
before the worker's next store into it (the server reads the row on its stream before it stores the
reply; the worker's next push is issued behind its wait for that reply).
"""
from __future__ import annotations

import datetime
import json
import os
import time
from typing import Dict, List, Optional, Union

import torch
import torch.distributed as dist

OP_INIT, OP_PUSH, OP_PULL, OP_OPT, OP_STOP, OP_PUSH_X, OP_PULL_X = range(7)  # _X: payload on the GPU plane
TAG_HDR, TAG_DATA, TAG_REPLY = 1, 2, 3
_DTYPES = [torch.float32, torch.float16, torch.bfloat16, torch.float64, torch.int64, torch.int32, torch.uint8]
_EXIT_KEY = "tony/kv/exited"


def _dcode(dt: torch.dtype) -> int:
    return _DTYPES.index(dt)


# -- optimizers (server- or worker-side updater) -----------------------------------------------
class Optimizer:
    """``mx.optimizer`` subset: sgd (momentum, wd, rescale_grad, clip_gradient) and adam."""

    def __init__(self, name: str = "sgd", learning_rate: float = 0.01, momentum: float = 0.0, wd: float = 0.0,
                 rescale_grad: float = 1.0, clip_gradient: Optional[float] = None, beta1: float = 0.9,
                 beta2: float = 0.999, epsilon: float = 1e-8):
        self.name = name.lower()
        if self.name not in ("sgd", "adam"):
            raise ValueError(f"unsupported optimizer {name!r}")
        self.cfg = dict(name=self.name, learning_rate=learning_rate, momentum=momentum, wd=wd,
                        rescale_grad=rescale_grad, clip_gradient=clip_gradient, beta1=beta1, beta2=beta2,
                        epsilon=epsilon)
        self.state: Dict[int, dict] = {}

    def to_json(self) -> str:
        return json.dumps(self.cfg)

    @classmethod
    def from_json(cls, s: str) -> "Optimizer":
        return cls(**json.loads(s))

    def update(self, key: int, weight: torch.Tensor, grad: torch.Tensor) -> None:
        c = self.cfg
        g = grad.float() * c["rescale_grad"]
        if c["clip_gradient"] is not None:
            g.clamp_(-c["clip_gradient"], c["clip_gradient"])
        w = weight if weight.dtype == torch.float32 else weight.float()
        g.add_(w, alpha=c["wd"])
        st = self.state.setdefault(key, {"t": 0})
        lr = c["learning_rate"]
        if self.name == "sgd":
            if c["momentum"]:
                m = st.setdefault("mom", torch.zeros_like(w))
                m.mul_(c["momentum"]).add_(g, alpha=-lr)
                w.add_(m)
            else:
                w.add_(g, alpha=-lr)
        else:
            st["t"] += 1
            m = st.setdefault("m", torch.zeros_like(w))
            v = st.setdefault("v", torch.zeros_like(w))
            m.mul_(c["beta1"]).add_(g, alpha=1 - c["beta1"])
            v.mul_(c["beta2"]).addcmul_(g, g, value=1 - c["beta2"])
            t = st["t"]
            lr_t = lr * (1 - c["beta2"] ** t) ** 0.5 / (1 - c["beta1"] ** t)
            w.addcdiv_(m, v.sqrt().add_(c["epsilon"]), value=-lr_t)
        if w is not weight:
            weight.copy_(w)

    def state_dict(self):
        return {"cfg": self.cfg, "state": self.state}


def create_optimizer(name: str = "sgd", **kw) -> Optimizer:
    return Optimizer(name, **kw)


def _as_list(v) -> List[torch.Tensor]:
    return list(v) if isinstance(v, (list, tuple)) else [v]


def _merge(vals: List[torch.Tensor]) -> torch.Tensor:
    out = vals[0].detach().clone()
    for v in vals[1:]:
        out.add_(v.to(out.device))
    return out


class _KeyIds:
    def __init__(self):
        self.ids: Dict[object, int] = {}

    def __call__(self, key) -> int:
        if isinstance(key, int):
            return key
        if key not in self.ids:
            self.ids[key] = len(self.ids) + (1 << 40)  # string keys live above int keys
        return self.ids[key]


# -- local ----------------------------------------------------------------------------------------
class KVStore:
    def __init__(self, kind: str = "local"):
        self.type = kind
        self._store: Dict[int, torch.Tensor] = {}
        self._opt: Optional[Optimizer] = None
        self._key = _KeyIds()

    @property
    def rank(self) -> int:
        return 0

    @property
    def num_workers(self) -> int:
        return 1

    def _keys_vals(self, key, value):
        if isinstance(key, (list, tuple)):
            return list(key), list(value)
        return [key], [value]

    def init(self, key, value) -> None:
        for k, v in zip(*self._keys_vals(key, value)):
            self._store[self._key(k)] = _as_list(v)[0].detach().clone()

    def push(self, key, value, priority: int = 0) -> None:  # noqa: ARG002
        for k, v in zip(*self._keys_vals(key, value)):
            kid = self._key(k)
            g = _merge(_as_list(v))
            self._apply(kid, g)

    def _apply(self, kid: int, merged: torch.Tensor) -> None:
        if kid not in self._store:
            raise KeyError(f"key {kid} was not initialised")
        if self._opt is not None:
            self._opt.update(kid, self._store[kid], merged.to(self._store[kid].device))
        else:
            self._store[kid].copy_(merged)

    def pull(self, key, out=None, priority: int = 0, ignore_sparse: bool = True):  # noqa: ARG002
        keys, outs = self._keys_vals(key, out)
        for k, o in zip(keys, outs):
            src = self._store[self._key(k)]
            for t in _as_list(o):
                t.copy_(src.to(t.device))

    def pushpull(self, key, value, out=None, priority: int = 0) -> None:
        self.push(key, value, priority)
        self.pull(key, out if out is not None else value, priority)

    def set_optimizer(self, optimizer: Optimizer) -> None:
        self._opt = optimizer

    def set_gradient_compression(self, params: dict) -> None:
        if params.get("type") not in (None, "none"):
            raise NotImplementedError("gradient compression is not supported by this kvstore")

    def barrier(self) -> None:
        pass

    def save_optimizer_states(self, fname: str, dump_optimizer: bool = False) -> None:  # noqa: ARG002
        if self._opt is None:
            raise RuntimeError("no optimizer set")
        torch.save({"cfg": json.dumps(self._opt.cfg), "state": self._opt.state}, fname)

    def load_optimizer_states(self, fname: str) -> None:
        sd = torch.load(fname, weights_only=True)
        self._opt = Optimizer.from_json(sd["cfg"])
        self._opt.state = sd["state"]

    def close(self) -> None:
        pass


# -- dist (servers) -------------------------------------------------------------------------------
def _env_int(name: str, default: int) -> int:
    try:
        return int(os.environ.get(name, default))
    except ValueError:
        return default


class _Topology:
    def __init__(self):
        e = os.environ
        self.role = e.get("DMLC_ROLE", "worker")
        self.num_servers = _env_int("DMLC_NUM_SERVER", 0)
        self.num_workers = _env_int("DMLC_NUM_WORKER", 1)
        self.root_uri = e.get("DMLC_PS_ROOT_URI", "127.0.0.1")
        self.root_port = _env_int("DMLC_PS_ROOT_PORT", 0)
        self.index = _env_int("TASK_INDEX", 0)

    @property
    def world(self) -> int:
        return self.num_servers + self.num_workers

    @property
    def rank(self) -> int:
        return self.index if self.role == "server" else self.num_servers + self.index

    def server_of(self, kid: int) -> int:
        return kid % self.num_servers


def _connect(topo: _Topology, timeout_s: float = 1800.0) -> dist.TCPStore:
    return dist.TCPStore(topo.root_uri, topo.root_port, topo.world + 1, False,
                         timeout=datetime.timedelta(seconds=timeout_s))


def _init_group(topo: _Topology):
    store = _connect(topo)
    if not dist.is_initialized():
        dist.init_process_group("gloo", store=dist.PrefixStore("tony-kv", store), rank=topo.rank,
                                world_size=topo.world)
    workers = dist.new_group(list(range(topo.num_servers, topo.world)))
    return store, workers


def _pad16(n: int) -> int:
    return (n + 15) // 16 * 16


# device flag tables in a plane window's header (csrc/ps_plane.hip: the first 1 MiB is the PS plane's
# arrival table, unused by a kvstore process): a server's push counters [key slot][worker], a worker's
# reply counters [server][key slot]
_MAX_SLOTS, _MAX_KV_WORKERS = 4096, 64
_REPLY_FLAGS = 4 * _MAX_SLOTS * _MAX_KV_WORKERS


def _push_flag(slot: int, worker: int) -> int:
    return 4 * (slot * _MAX_KV_WORKERS + worker)


def _reply_flag(topo: "_Topology", server: int, slot: int) -> int:
    return _REPLY_FLAGS + 4 * (server * (_MAX_SLOTS // max(1, topo.num_servers)) + slot)


def _wait_budget_s() -> float:
    return float(os.environ.get("TONY_KV_WAIT_S", "300"))


def _plane_wanted() -> bool:
    mode = os.environ.get("TONY_KV_PLANE", "auto").lower()
    if mode in ("gloo", "0", "off"):
        return False
    if mode == "xgmi" and not torch.cuda.is_available():
        raise RuntimeError("TONY_KV_PLANE=xgmi but this task sees no GPU")
    return torch.cuda.is_available()


class _KvLayout:
    """Where each key's bytes live in the plane windows, computed identically by a server and every worker
    from the keys in init order (a server sees only its own keys, which is all its part depends on):
    server s's window holds, per key it owns, one receive row per worker; a worker's window is split in one
    landing region per server, each holding that server's keys back to back."""

    def __init__(self, topo: "_Topology", window_bytes: int):
        self.topo, self.bytes = topo, window_bytes
        self.region = window_bytes // max(1, topo.num_servers) // 16 * 16  # a worker's landing region per server
        self.row_used = [0] * topo.num_servers
        self.land_used = [0] * topo.num_servers
        self.slots = [0] * topo.num_servers
        self.keys: Dict[int, tuple] = {}  # kid -> (server, nbytes, row_off, land_off, flag slot)

    def add_key(self, kid: int, nbytes: int) -> bool:
        s = self.topo.server_of(kid)
        rows = self.topo.num_workers * _pad16(nbytes)
        if (self.row_used[s] + rows > self.bytes or self.land_used[s] + _pad16(nbytes) > self.region
                or self.slots[s] >= _MAX_SLOTS // max(1, self.topo.num_servers)
                or self.topo.num_workers > _MAX_KV_WORKERS):
            return False  # stays on the gloo payload path (decided identically on every member)
        self.keys[kid] = (s, nbytes, self.row_used[s], s * self.region + self.land_used[s], self.slots[s])
        self.row_used[s] += rows
        self.land_used[s] += _pad16(nbytes)
        self.slots[s] += 1
        return True


class _KvPlane:
    """The GPU payload windows of one server / worker (module docstring), laid out by _KvLayout."""

    def __init__(self, topo: "_Topology", device: torch.device):
        import ctypes

        from ..ops import _lib

        self.topo, self.device, self.L = topo, device, _lib.lib()
        self.bytes = int(os.environ.get("TONY_KV_WINDOW_MB", "64")) << 20
        hsize = self.L.tony_xgmi_handle_bytes()
        win, handle = ctypes.c_void_p(), (ctypes.c_uint8 * hsize)()
        with torch.cuda.device(device):
            rc = self.L.tony_ps_window_alloc(self.bytes, ctypes.byref(win), handle)
        self.window = win.value if rc == 0 else None
        self._opened: List[int] = []
        hdr = self.L.tony_ps_header_bytes()
        allh: List[Optional[bytes]] = [None] * topo.world
        dist.all_gather_object(allh, bytes(handle) if rc == 0 else b"")  # every member joins, even on failure
        _lib.check(rc, "tony_ps_window_alloc")
        if not all(allh):
            raise RuntimeError("a peer could not allocate its window")
        self.base = self.window + hdr
        self.peer: Dict[int, int] = {}
        self.peer_win: Dict[int, int] = {}  # window bases (flag tables) of the peers
        peers = range(topo.num_servers, topo.world) if topo.role == "server" else range(topo.num_servers)
        for r in peers:
            p = ctypes.c_void_p()
            buf = (ctypes.c_uint8 * hsize).from_buffer_copy(allh[r])
            with torch.cuda.device(device):
                _lib.check(self.L.tony_xgmi_open(buf, ctypes.byref(p)), f"tony_xgmi_open(rank {r})")
            self.peer[r] = p.value + hdr
            self.peer_win[r] = p.value
            self._opened.append(p.value)
        self.layout = _KvLayout(topo, self.bytes)
        self.keys = self.layout.keys
        self._side: Dict[int, "torch.cuda.Stream"] = {}  # server: per pushing worker, waits + row reads
        self._arrived: Dict[tuple, int] = {}  # server: (kid, worker) -> flag counts expected so far
        # the window's error word, copied to pinned host memory behind every POLL_EVERY-th copy: a timed-out
        # device wait surfaces within a few calls on both sides without a device synchronisation
        self._err_host = torch.zeros(1, dtype=torch.int32, pin_memory=True)
        self._polls = 0

    POLL_EVERY = 8

    def poll(self) -> None:
        """Raise if an earlier asynchronous read of the error word saw a timed-out wait; queue a new read."""
        from ..ops import _lib

        if int(self._err_host[0]):
            self.check()
        _lib.check(self.L.tony_ps_error_async(self.window, self._err_host.data_ptr(), _lib.stream_ptr(self.device)),
                   "tony_ps_error_async")

    def add_key(self, kid: int, nbytes: int) -> bool:
        return self.layout.add_key(kid, nbytes)

    def copy(self, dst: int, src: int, nbytes: int) -> None:
        """Stream-ordered local copy out of this rank's window behind a wait: skipped on the device when a
        wait of this window timed out (no stale or partial payload is merged or pulled), and the error is
        raised by the next check."""
        from ..ops import _lib

        with torch.cuda.device(self.device):
            _lib.check(self.L.tony_kv_copy(dst, src, nbytes, self.window, _lib.stream_ptr(self.device)),
                       "tony_kv_copy")
            self._polls += 1
            if self._polls % self.POLL_EVERY == 0:  # a cheap asynchronous read of the error word
                self.poll()

    def send(self, dst: int, src: int, nbytes: int, flag: int) -> int:
        """Copy into a peer's window and count it on the peer's flag at window offset ``flag`` (no host
        wait); returns the count the copy adds (the consumer's target grows by it)."""
        from ..ops import _lib

        with torch.cuda.device(self.device):
            _lib.check(self.L.tony_kv_copy_flag(dst, src, nbytes, flag, _lib.stream_ptr(self.device)),
                       "tony_kv_copy_flag")
        return self.L.tony_kv_copy_blocks(nbytes)

    def take(self, kid: int, w: int, numel: int, dtype: torch.dtype):
        """Server: worker w's pushed row of kid as a new tensor, and the event after its read.  The row has
        landed once the worker's copy counted all its workgroups on the key's push flag.  The wait and
        the read run on the worker's own stream: the bytes may depend on a reply this server has yet to
        store (the worker pushes behind its wait for its last pull), so nothing else may queue behind
        the wait.  The worker rewrites the row only behind its wait for a later reply, which the server
        stores after merging this round -- no host wait on either side."""
        _, nbytes, row_off, _, slot = self.keys[kid]
        side = self._side.get(w)
        if side is None:
            side = self._side[w] = torch.cuda.Stream(self.device)
        main = torch.cuda.current_stream(self.device)
        with torch.cuda.stream(side):
            buf = torch.empty(numel, dtype=dtype, device=self.device)
            n = self._arrived[(kid, w)] = self._arrived.get((kid, w), 0) + self.L.tony_kv_copy_blocks(nbytes)
            self.wait(_push_flag(slot, w), n)
            self.copy(buf.data_ptr(), self.base + row_off + w * _pad16(nbytes), nbytes)
            ev = torch.cuda.Event()
            ev.record(side)
        buf.record_stream(main)
        return buf, ev

    def wait(self, flag_off: int, target: int) -> None:
        """Hold this rank's stream until the counter at ``flag_off`` of its window reaches ``target``."""
        from ..ops import _lib

        with torch.cuda.device(self.device):
            _lib.check(self.L.tony_kv_wait(self.window + flag_off, target & 0xFFFFFFFF, self.window,
                                           _wait_budget_s(), _lib.stream_ptr(self.device)), "tony_kv_wait")

    def check(self) -> None:
        """Raise if one of this rank's device waits timed out (synchronises the device)."""
        import ctypes

        from ..ops import _lib

        with torch.cuda.device(self.device):
            torch.cuda.synchronize(self.device)
            err = ctypes.c_int(0)
            _lib.check(self.L.tony_ps_error(self.window, ctypes.byref(err)), "tony_ps_error")
        if err.value:
            raise RuntimeError(f"kvstore plane: a device wait timed out after {_wait_budget_s()} s "
                               "(TONY_KV_WAIT_S): a peer never delivered its payload")

    def close(self) -> None:
        """Unmap the peers and free the window; raises afterwards if a device wait of this rank timed out
        (the copies behind it were skipped, so the run's payloads are not trustworthy)."""
        err = None
        if getattr(self, "window", None) is not None:
            torch.cuda.synchronize(self.device)  # no copy into or out of a window is left in flight
            try:
                self.check()
            except RuntimeError as e:
                err = e
        for p in self._opened:
            self.L.tony_xgmi_close(p)
        self._opened = []
        if getattr(self, "window", None) is not None:
            self.L.tony_xgmi_free(self.window)
            self.window = None
        if err is not None:
            raise err


def _make_plane(topo: "_Topology", device: Optional[torch.device]) -> Optional[_KvPlane]:
    """Collective over servers + workers: the plane when every member wants it (else None everywhere)."""
    want = device is not None and _plane_wanted()
    allw: List[Optional[bool]] = [None] * topo.world
    dist.all_gather_object(allw, want)
    if not all(allw):
        return None
    plane, err = None, ""
    try:
        plane = _KvPlane(topo, device)
    except Exception as e:  # noqa: BLE001 - e.g. a peer GPU this task cannot see: agree on gloo everywhere
        err = f"{type(e).__name__}: {e}"
    errs: List[Optional[str]] = [None] * topo.world
    dist.all_gather_object(errs, err)
    if any(errs):
        if plane is not None:
            plane.close()
        import sys

        print(f"[tony kvstore] GPU payload plane unavailable, payloads over gloo: "
              f"{'; '.join(f'rank {r}: {e}' for r, e in enumerate(errs) if e)}", file=sys.stderr, flush=True)
        return None
    return plane


def run_scheduler(poll_s: float = 0.05) -> int:
    """The scheduler role: host the rendezvous store until every server and worker exited."""
    topo = _Topology()
    store = dist.TCPStore("0.0.0.0", topo.root_port, topo.world + 1, True,
                          timeout=datetime.timedelta(seconds=1800), wait_for_workers=False)
    while store.add(_EXIT_KEY, 0) < topo.world:
        time.sleep(poll_s)
    return 0


class _Server:
    def __init__(self, topo: _Topology, sync: bool, plane: Optional[_KvPlane] = None):
        self.topo = topo
        self.sync = sync
        self.plane = plane
        self.values: Dict[int, torch.Tensor] = {}
        self.pushed: Dict[int, set] = {}
        self.deferred: Dict[int, List[int]] = {}
        self.opt: Optional[Optimizer] = None
        self.early: Dict[int, list] = {}
        self.sends = []
        self.applied = 0
        self.round: Dict[int, list] = {}  # kid -> [(worker, arrival, payload, event)] of the open round

    def _reply(self, kid: int, worker: int, via_plane: bool = False) -> None:
        if via_plane:  # the value into the worker's landing area, counted on the worker's reply flag
            srv, nbytes, _, land_off, slot = self.plane.keys[kid]
            v = self.values[kid].contiguous()
            self.plane.send(self.plane.peer[worker] + land_off, v.data_ptr(), nbytes,
                            self.plane.peer_win[worker] + _reply_flag(self.topo, srv, slot))
            return
        self.sends.append(dist.isend(self.values[kid].contiguous().cpu(), worker, tag=TAG_REPLY))

    def _merge_round(self, kid: int) -> torch.Tensor:
        """The open round's pushes of kid summed in worker order (deterministic), on this stream after
        every plane push's row read (device events: the host never waits for a payload)."""
        v = self.values[kid]
        merged = None
        for _, _, b, ev in sorted(self.round.pop(kid), key=lambda e: (e[0], e[1])):
            if ev is not None:
                torch.cuda.current_stream(v.device).wait_event(ev)
            b = b.to(v.device, v.dtype)  # every payload buffer is this server's own: summed in place
            merged = b if merged is None else merged.add_(b)
        return merged

    def _finish_round(self, kid: int) -> None:
        merged = self._merge_round(kid)
        if self.opt is not None:
            self.opt.update(kid, self.values[kid], merged)
        else:
            self.values[kid].copy_(merged)
        self.applied += 1
        self.pushed[kid] = set()
        for w, via in self.deferred.pop(kid, []):
            self._reply(kid, w, via)

    def handle(self, worker: int, hdr: List[int], buf: Optional[torch.Tensor] = None) -> bool:
        op, kid, numel, dcode = hdr
        if op in (OP_INIT, OP_PUSH, OP_OPT) and buf is None:
            buf = torch.empty(numel, dtype=_DTYPES[dcode])
            dist.recv(buf, worker, tag=TAG_DATA)
        via = op == OP_PULL_X
        if op in (OP_PUSH, OP_PULL, OP_PUSH_X, OP_PULL_X) and kid not in self.values:
            # raced ahead of worker 0's INIT (it is sent before the workers' barrier, but the server
            # may poll this worker first): replay once the key exists.  A plane push is parked with its
            # raw header: the key has no window row in this server's layout until the INIT adds it, and
            # the worker does not rewrite that row before its next pull (DistKVStore._unread)
            self.early.setdefault(kid, []).append((worker, hdr, buf))
            return True
        ev = None
        if op == OP_PUSH_X:  # the payload is in this worker's receive row of the window: take it now
            buf, ev = self.plane.take(kid, worker - self.topo.num_servers, numel, _DTYPES[dcode])
            op = OP_PUSH
        elif op == OP_PULL_X:
            op = OP_PULL
        if op in (OP_INIT, OP_PUSH, OP_OPT):
            if op == OP_INIT:
                if self.plane is not None and self.plane.add_key(kid, buf.numel() * buf.element_size()):
                    buf = buf.to(self.plane.device)  # the key's value lives on the server's GPU
                self.values[kid] = buf
                self.pushed[kid] = set()
                for w, h, b in self.early.pop(kid, []):
                    self.handle(w, h, b)
            elif op == OP_OPT:
                self.opt = Optimizer.from_json(bytes(buf.tolist()).decode())
            else:
                r = self.round.setdefault(kid, [])
                r.append((worker, len(r), buf, ev))
                if not self.sync:
                    self._finish_round(kid)
                    return True
                self.pushed[kid].add(worker)
                if len(self.pushed[kid]) == self.topo.num_workers:
                    self._finish_round(kid)
        elif op == OP_PULL:
            if self.sync and worker in self.pushed.get(kid, ()):
                self.deferred.setdefault(kid, []).append((worker, via))
            else:
                self._reply(kid, worker, via)
        elif op == OP_STOP:
            return False
        return True

    def serve(self) -> None:
        """Receive request headers from ANY worker (gloo recv-anysource) until all sent STOP."""
        live = self.topo.num_workers
        hdr = torch.empty(4, dtype=torch.int64)
        while live:
            w = dist.recv(hdr, tag=TAG_HDR)
            if not self.handle(w, [int(x) for x in hdr.tolist()]):
                live -= 1
                if self.plane is not None:  # a worker finished: nothing it sent may have timed out
                    self.plane.check()
            if len(self.sends) > 64:
                for s in self.sends:
                    s.wait()
                self.sends = []
        for s in self.sends:
            s.wait()


def run_server(sync: Optional[bool] = None) -> int:
    """The server role: own keys until every worker sent STOP."""
    topo = _Topology()
    store, _ = _init_group(topo)
    dev = None
    if torch.cuda.is_available():  # a server may share a worker's GPU (TonY's servers ask for none)
        dev = torch.device("cuda", _env_int("TONY_KV_DEVICE", topo.index % torch.cuda.device_count()))
    plane = _make_plane(topo, dev)
    if sync is None:  # every worker announces its kvstore type before its first request
        sync = store.get("tony/kv/type").decode() != "dist_async"
    _Server(topo, sync, plane).serve()
    dist.barrier()
    if plane is not None:
        plane.close()
    store.add(_EXIT_KEY, 1)
    return 0


class DistKVStore(KVStore):
    """Worker side of ``dist_sync`` / ``dist_async``."""

    def __init__(self, kind: str):
        super().__init__(kind)
        self.topo = _Topology()
        if self.topo.num_servers < 1:
            raise ValueError(f"{kind} needs DMLC_NUM_SERVER >= 1 server task")
        self.store, self.workers = _init_group(self.topo)
        dev = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else None
        self.plane = _make_plane(self.topo, dev)
        self.store.set("tony/kv/type", kind)
        self._shapes: Dict[int, torch.Size] = {}
        self._unread: set = set()  # keys pushed on the plane and not pulled since (their row may be unread)
        self._replies: Dict[int, int] = {}  # kid -> reply copies counted on this worker's flag (target)
        # kid -> event after the last plane pull's copy out of the landing area: a repeat pull with no push
        # in between must not let the server overwrite that area before the copy read it
        self._landed: Dict[int, "torch.cuda.Event"] = {}
        self.plane_ops = [0, 0]  # pushes / pulls whose payload went over the GPU plane (tests)
        self._closed = False

    @property
    def rank(self) -> int:
        return self.topo.index

    @property
    def num_workers(self) -> int:
        return self.topo.num_workers

    def _send(self, op: int, kid: int, payload: Optional[torch.Tensor] = None) -> int:
        srv = self.topo.server_of(kid) if op != OP_STOP else kid
        n, dc = (payload.numel(), _dcode(payload.dtype)) if payload is not None else (0, 0)
        dist.send(torch.tensor([op, kid, n, dc], dtype=torch.int64), srv, tag=TAG_HDR)
        if payload is not None:
            dist.send(payload, srv, tag=TAG_DATA)
        return srv

    def init(self, key, value) -> None:
        for k, v in zip(*self._keys_vals(key, value)):
            kid = self._key(k)
            t = _as_list(v)[0].detach()
            self._shapes[kid] = t.shape
            if self.plane is not None:
                self.plane.add_key(kid, t.numel() * t.element_size())
            if self.rank == 0:
                self._send(OP_INIT, kid, t.reshape(-1).cpu().contiguous())
        self.barrier()

    def _on_plane(self, kid: int, t: torch.Tensor) -> bool:
        return self.plane is not None and kid in self.plane.keys and t.is_cuda

    def push(self, key, value, priority: int = 0) -> None:  # noqa: ARG002
        for k, v in zip(*self._keys_vals(key, value)):
            kid = self._key(k)
            g = _merge(_as_list(v)).reshape(-1)
            if self._on_plane(kid, g) and kid not in self._unread:
                srv, nbytes, row_off, _, slot = self.plane.keys[kid]
                g = g.to(self.plane.device).contiguous()
                if g.data_ptr() % 16:  # the copy kernel moves 16-B aligned addresses: a view at an odd offset
                    g = g.clone()
                # into this worker's row of the server's window, counted on the key's push flag there; the
                # header may overtake the bytes: the server's stream waits for the flag before reading
                self.plane.send(self.plane.peer[srv] + row_off + self.rank * _pad16(nbytes), g.data_ptr(), nbytes,
                                self.plane.peer_win[srv] + _push_flag(slot, self.rank))
                dist.send(torch.tensor([OP_PUSH_X, kid, g.numel(), _dcode(g.dtype)], dtype=torch.int64), srv,
                          tag=TAG_HDR)
                self._unread.add(kid)
                self.plane_ops[0] += 1
                continue
            self._send(OP_PUSH, kid, g.cpu().contiguous())

    def pull(self, key, out=None, priority: int = 0, ignore_sparse: bool = True):  # noqa: ARG002
        keys, outs = self._keys_vals(key, out)
        for k, o in zip(keys, outs):
            kid = self._key(k)
            first = _as_list(o)[0]
            if self._on_plane(kid, first):
                srv, nbytes, _, land_off, slot = self.plane.keys[kid]
                prev = self._landed.pop(kid, None)
                if prev is not None and kid not in self._unread:
                    # no push since the last pull: nothing orders the server's next reply store after that
                    # pull's copy-out (a push would -- the server answers only after reading it, and the push
                    # copy queues behind the copy-out); wait for the copy-out before asking again
                    prev.synchronize()
                dist.send(torch.tensor([OP_PULL_X, kid, 0, 0], dtype=torch.int64), srv, tag=TAG_HDR)
                # the reply lands in this worker's landing area, counted on its reply flag: this stream waits
                # for it on the device, then copies it out -- the host moves on at once
                n = self._replies[kid] = self._replies.get(kid, 0) + self.plane.L.tony_kv_copy_blocks(nbytes)
                self.plane.wait(_reply_flag(self.topo, srv, slot), n)
                buf = torch.empty(first.numel(), dtype=first.dtype, device=self.plane.device)
                self.plane.copy(buf.data_ptr(), self.plane.base + land_off, nbytes)
                ev = torch.cuda.Event()
                ev.record(torch.cuda.current_stream(self.plane.device))
                self._landed[kid] = ev
                self._unread.discard(kid)  # the server answered: it consumed this worker's earlier rows
                self.plane_ops[1] += 1
            else:
                srv = self._send(OP_PULL, kid)
                buf = torch.empty(first.numel(), dtype=first.dtype)
                dist.recv(buf, srv, tag=TAG_REPLY)
                self._unread.discard(kid)
            for t in _as_list(o):
                t.copy_(buf.view(t.shape).to(t.device))

    def set_optimizer(self, optimizer: Optimizer) -> None:
        """Ship the optimizer to every server (MXNet pickles it; here it is a JSON config)."""
        if self.rank == 0:
            payload = torch.tensor(list(optimizer.to_json().encode()), dtype=torch.uint8)
            for s in range(self.topo.num_servers):
                self._send_to(s, OP_OPT, payload)
        self.barrier()

    def _send_to(self, srv: int, op: int, payload: torch.Tensor) -> None:
        dist.send(torch.tensor([op, srv, payload.numel(), _dcode(payload.dtype)], dtype=torch.int64), srv,
                  tag=TAG_HDR)
        dist.send(payload, srv, tag=TAG_DATA)

    def barrier(self) -> None:
        if self.plane is not None:
            self.plane.check()
        dist.barrier(group=self.workers)

    def save_optimizer_states(self, fname: str, dump_optimizer: bool = False) -> None:
        raise NotImplementedError("optimizer states live on the servers in dist modes")

    def close(self) -> None:
        """Tell every server this worker is done (MXNet does this at process exit)."""
        if self._closed:
            return
        self._closed = True
        self.barrier()
        for s in range(self.topo.num_servers):
            dist.send(torch.tensor([OP_STOP, s, 0, 0], dtype=torch.int64), s, tag=TAG_HDR)
        dist.barrier()
        if self.plane is not None:
            self.plane.close()
        self.store.add(_EXIT_KEY, 1)


class DeviceSyncKVStore(KVStore):
    """``dist_device_sync``: RCCL all-reduce of pushes among workers + replicated updater."""

    def __init__(self, kind: str = "dist_device_sync", group=None):
        super().__init__(kind)
        if not dist.is_initialized():
            from .bootstrap import init_from_env

            init_from_env()
        self.group = group

    @property
    def rank(self) -> int:
        return dist.get_rank(self.group)

    @property
    def num_workers(self) -> int:
        return dist.get_world_size(self.group)

    def init(self, key, value) -> None:
        for k, v in zip(*self._keys_vals(key, value)):
            t = _as_list(v)[0].detach().clone()
            dist.broadcast(t, 0, group=self.group)
            self._store[self._key(k)] = t

    def push(self, key, value, priority: int = 0) -> None:  # noqa: ARG002
        for k, v in zip(*self._keys_vals(key, value)):
            g = _merge(_as_list(v))
            dist.all_reduce(g, group=self.group)
            self._apply(self._key(k), g)

    def barrier(self) -> None:
        dist.barrier(group=self.group)


def create(name: str = "local") -> KVStore:
    name = name.lower()
    if name in ("local", "device", "local_allreduce_cpu", "local_allreduce_device"):
        return KVStore(name)
    if name in ("dist_sync", "dist_async", "dist"):
        return DistKVStore("dist_sync" if name == "dist" else name)
    if name in ("dist_device_sync", "dist_sync_device"):
        return DeviceSyncKVStore("dist_device_sync")
    raise ValueError(f"unknown kvstore type {name!r}")


def run_role() -> bool:
    """Run the scheduler / server loop if this task is one; True when the caller should exit.

    ``import mxnet`` does this implicitly for non-worker roles (mxnet_dist_ex.py:10-13).
    """
    role = os.environ.get("DMLC_ROLE", "worker")
    if role == "scheduler":
        run_scheduler()
        return True
    if role == "server":
        run_server()
        return True
    return False


Value = Union[torch.Tensor, List[torch.Tensor]]

"""The dedicated parameter server's data plane over xGMI peer memory (csrc/ps_plane.hip, H16).

TonY's TF-PS topology (``ps`` tasks own the variables and apply the optimizer, workers push
gradients and pull variables every step: /root/reference/tony-examples/mnist-tensorflow/
mnist_distributed.py:206-241) on one MI355X node, with every byte moved by GPU kernels over
IPC-mapped windows instead of RCCL reduce / broadcast rings:

* push  -- a worker's communication stream stores each bucket's gradient (cast to the wire dtype
  on the way) straight into its row of the owning ps GPU's receive window, as soon as backward
  finished the bucket (parallel/buckets.py), and raises per-chunk arrival flags there;
* apply -- the ps GPU applies the fused optimizer chunk by chunk as the rows land (sync: once every
  worker's chunk is there, async: each worker's chunk on its own) and stores the new variables
  straight into every worker's landing window (the ps drives its links to all workers at once);
* land  -- after backward, a worker copies its landing window into its flat parameters once the
  ps flagged each chunk.

The ps GPU has an xGMI link to every other GPU, so the fan-in of N workers and the fan-out of the
new variables run over N links in parallel, and the ps applies as arrivals complete -- the apply
hides behind the workers' backward.  HBM sizing: the ps window holds one receive row per worker
for every bucket it owns (7 workers x 109 MB of fp32 Inception-v3 gradients = 763 MB of the ps
GPU's 288 GB), so no row is ever reused within a step.

Selected by ``ParameterServer(mode="dedicated", plane="xgmi")`` (the default on GPUs; ``plane=
"rccl"`` keeps the reduce / broadcast form for A/B runs).  Every rank must map every peer's memory:
the launcher leaves all GPUs visible for such jobs (visible-devices-mode auto -> none, cluster/
coordinator.py).  A ps and a worker may share one GPU (two processes; TonY's 0-GPU ps is placed on a
worker's GPU, tony.amd.ps-share-gpu); one process cannot be both.  At init a canary bucket goes
through push / apply / land and is checked on every worker (``verified``); a mismatch raises on every
rank and the ParameterServer falls back to the collective plane.

Shared GPUs: every wait here is a kernel spinning on a flag, so the processes on one GPU must all get
their queues serviced.  The landing walks its chunks on at most one workgroup per CU (two workers' landings
of the fp32 Inception buckets once filled every workgroup slot and starved the ps's apply), and the
one-GPU rehearsal of 1 ps + 2 x3 workers with their branch / weight-gradient streams still stalled a
worker until the wait budget ran out (profiles/r6_x3_ps_dedicated_shared_gpu.log) -- one GPU per rank,
or the ps sharing ONE worker's GPU, is the supported placement; the budget turns a stall into an error.
"""
from __future__ import annotations

import ctypes
import os
from typing import Dict, List, Optional

import torch
import torch.distributed as dist

from ..ops import _lib

# seconds a kernel waits for a peer before it gives up and flags an error (the first step of a job
# autotunes its kernels for a while, so this is generous)
SPIN_S = float(os.environ.get("TONY_PS_SPIN_S", "300"))


class PSPlaneError(RuntimeError):
    pass


def blocks_for(nbytes: int, cap: int) -> int:
    """Workgroups per bucket: one per ~64 KiB of gradient, 4..cap (256: an 8 MB bucket's apply spreads
    over 128 workgroups, so its fan-out of the new variables keeps requests in flight on every link).
    A pure function of the bucket size: pusher and ps must agree on the chunking."""
    return max(4, min(cap, nbytes >> 16))


CANARY_N = 1024  # elements of the init-time canary bucket (its own rows / landing area)


class XgmiPSPlane:
    def __init__(self, flat, buckets, owner_of, ps_ranks: List[int], worker_ranks: List[int], rank: int,
                 wire_dtype: torch.dtype, group=None, sync: bool = True):
        L = _lib.lib()
        if len(buckets) > L.tony_ps_max_buckets() - 1:  # the last bucket index is the canary's
            raise PSPlaneError(f"{len(buckets)} buckets > {L.tony_ps_max_buckets()}: raise the bucket size")
        if len(worker_ranks) > 8:
            raise PSPlaneError("at most 8 workers per ps on one node")
        self.flat, self.buckets, self.group = flat, buckets, group
        self.rank, self.sync = rank, sync
        self.ps_ranks, self.worker_ranks = list(ps_ranks), list(worker_ranks)
        self.owner = {b.index: owner_of(b) for b in buckets}
        self.wire_dtype = wire_dtype
        self.wesz = torch.empty((), dtype=wire_dtype).element_size()
        self.pesz = flat.data.element_size()
        self.device = flat.device
        self.is_ps = rank in self.ps_ranks
        self.is_worker = rank in self.worker_ranks
        self.widx = self.worker_ranks.index(rank) if self.is_worker else -1
        cap = L.tony_ps_max_blocks()
        self.blocks = {b.index: blocks_for(b.numel * self.wesz, cap) for b in buckets}
        # receive-row layout of every ps (all ranks compute it: workers need the offsets)
        self.row_off: Dict[int, int] = {}
        self.row_stride: Dict[int, int] = {}
        for p in self.ps_ranks:
            off = 0
            for b in buckets:
                if self.owner[b.index] == p:
                    self.row_off[b.index] = off
                    off += (b.numel * self.wesz + 15) // 16 * 16
            self.row_stride[p] = off
        # canary areas after the real ones: CANARY_N wire elements per worker in every ps window, CANARY_N
        # parameter elements at flat element canary_lo of every worker's landing zone
        self.canary_bytes = (CANARY_N * self.wesz + 15) // 16 * 16
        self.canary_lo = (flat.numel + 7) // 8 * 8
        payload = 0
        if self.is_ps:
            payload += len(self.worker_ranks) * (self.row_stride[rank] + self.canary_bytes)
        if self.is_worker:
            payload += (self.canary_lo + CANARY_N) * self.pesz  # the landing zone (+ the canary's)
        if self.is_ps and self.is_worker:
            raise PSPlaneError("a rank cannot be both ps and worker on the xGMI plane (use mode='colocated')")
        hsize = L.tony_xgmi_handle_bytes()
        window = ctypes.c_void_p()
        handle = (ctypes.c_uint8 * hsize)()
        with torch.cuda.device(self.device):
            _lib.check(L.tony_ps_window_alloc(payload, ctypes.byref(window), handle), "tony_ps_window_alloc")
        self.window = window.value
        handles: List[Optional[bytes]] = [None] * dist.get_world_size(group)
        dist.all_gather_object(handles, bytes(handle), group=group)
        # map what this rank writes into: a worker maps the ps windows, a ps maps the worker windows
        self.mapped: Dict[int, int] = {rank: self.window}
        self._opened: List[int] = []
        peers = self.ps_ranks if self.is_worker else self.worker_ranks
        for r in peers:
            p = ctypes.c_void_p()
            buf = (ctypes.c_uint8 * hsize).from_buffer_copy(handles[r])
            with torch.cuda.device(self.device):
                _lib.check(L.tony_xgmi_open(buf, ctypes.byref(p)), f"tony_xgmi_open(rank {r})")
            self.mapped[r] = p.value
            self._opened.append(p.value)
        if self.is_ps:
            self._worker_windows = (ctypes.c_uint64 * len(self.worker_ranks))(
                *[self.mapped[w] for w in self.worker_ranks])
        if self.is_worker:
            import struct

            ent = struct.Struct("<qqii")
            assert ent.size == L.tony_ps_land_entry_bytes()
            raw = b"".join(ent.pack(b.lo, b.numel, self.blocks[b.index], b.index) for b in buckets)
            self._land_table = torch.frombuffer(bytearray(raw), dtype=torch.uint8).to(self.device)
        self._err_host = torch.zeros(1, dtype=torch.int32, pin_memory=True)
        self.pushed = 0
        self.dead = None  # set once a wait timed out: the plane refuses every later call
        dist.barrier(group=group)
        self.verified = False
        self._canary()

    # -- first-use check ------------------------------------------------------------------------
    def _canary(self) -> None:
        """Push / apply / land of a small random bucket through every ps, checked against the
        expected sum on every worker before any real gradient moves: the windows are mapped across
        real devices, fine-grained stores reach the peer, the flags order them.  Raises PSPlaneError on
        every rank if any rank saw a mismatch or a timeout (the ParameterServer then falls back to the
        collective plane, loudly); sets ``verified`` otherwise."""
        L = _lib.lib()
        cb = L.tony_ps_max_buckets() - 1
        blocks = 4
        stream = _lib.stream_ptr(self.device)
        gdt = self.flat.grad.dtype
        pats = [torch.randn(CANARY_N, generator=torch.Generator().manual_seed(777 + w)).to(gdt)
                for w in range(len(self.worker_ranks))]
        wire = self.wire_dtype
        want = sum(p.to(wire).float() for p in pats).to(self.flat.data.dtype).float()
        bad = []
        hp = torch.tensor([-1.0, 0.0, 0.0, 1.0, 0.0, 0.0, 0.0, 1.0, 0.0], device=self.device)  # SGD lr -1: w = sum g
        for k, p in enumerate(self.ps_ranks):
            value = k + 1
            rows_off = len(self.worker_ranks) * self.row_stride[p]
            if self.is_worker:
                g = pats[self.widx].to(self.device)
                _lib.check(L.tony_ps_push(g.data_ptr(), int(gdt == torch.bfloat16), self.mapped[p],
                                          rows_off + self.widx * self.canary_bytes, int(wire == torch.bfloat16),
                                          CANARY_N, cb, self.widx, value, blocks, stream), "tony_ps_push (canary)")
            if self.rank == p:
                master = torch.zeros(CANARY_N, device=self.device)
                mom = torch.zeros(CANARY_N, device=self.device)
                _lib.check(L.tony_ps_apply(self.window, rows_off, self.canary_bytes, len(self.worker_ranks),
                                           int(wire == torch.bfloat16), CANARY_N, self.canary_lo, master.data_ptr(),
                                           mom.data_ptr(), None, hp.data_ptr(), 0, self._worker_windows, None,
                                           int(self.flat.data.dtype == torch.bfloat16), cb, value, 0, 60.0,
                                           blocks, stream), "tony_ps_apply (canary)")
            if self.is_worker:
                import struct

                ent = struct.Struct("<qqii").pack(self.canary_lo, CANARY_N, blocks, cb)
                tab = torch.frombuffer(bytearray(ent), dtype=torch.uint8).to(self.device)
                out = torch.empty(CANARY_N, dtype=self.flat.data.dtype, device=self.device)
                base = out.data_ptr() - self.canary_lo * self.pesz  # the kernel adds the bucket's offset
                _lib.check(L.tony_ps_land(self.window, tab.data_ptr(), 1, base,
                                          int(self.flat.data.dtype == torch.bfloat16), value, 60.0, stream),
                           "tony_ps_land (canary)")
                torch.cuda.synchronize(self.device)
                tol = 2e-2 if self.flat.data.dtype == torch.bfloat16 else 1e-5
                got = out.float().cpu()
                if not torch.allclose(got, want, rtol=tol, atol=tol):
                    bad.append(f"ps {p}: max |diff| {float((got - want).abs().max()):.3g}")
            torch.cuda.synchronize(self.device)
            dist.barrier(group=self.group)
        err = ctypes.c_int(0)
        _lib.check(L.tony_ps_error(self.window, ctypes.byref(err)), "tony_ps_error")
        if err.value:
            bad.append("a canary wait timed out")
        allbad: List[Optional[list]] = [None] * dist.get_world_size(self.group)
        dist.all_gather_object(allbad, bad, group=self.group)
        msgs = [f"rank {r}: {m}" for r, b in enumerate(allbad) for m in (b or [])]
        if msgs:
            self.close()
            raise PSPlaneError("xGMI PS plane canary mismatch: " + "; ".join(msgs))
        self.verified = True

    # -- errors ---------------------------------------------------------------------------------
    def _poll_error(self, stream) -> None:
        if self.dead is not None:
            raise PSPlaneError(self.dead)
        if int(self._err_host[0]):
            self.check_error()
        _lib.check(_lib.lib().tony_ps_error_async(self.window, self._err_host.data_ptr(), stream),
                   "tony_ps_error_async")

    def check_error(self) -> None:
        torch.cuda.synchronize(self.device)
        err = ctypes.c_int(0)
        _lib.check(_lib.lib().tony_ps_error(self.window, ctypes.byref(err)), "tony_ps_error")
        self._err_host.zero_()
        if err.value:
            # the plane is unusable from here on: the kernels of this rank are poisoned (they do nothing
            # once the error word was set) and every later call raises this
            self.dead = (f"rank {self.rank}: a peer of the parameter-server plane never arrived within "
                         f"{SPIN_S:.0f} s: this step's variables are invalid")
            raise PSPlaneError(self.dead)

    # -- the three kernels ----------------------------------------------------------------------
    def push(self, b, step: int) -> None:
        """Worker: bucket b's gradient into its row of the owner's window (current stream)."""
        if self.dead is not None:
            raise PSPlaneError(self.dead)
        g = self.flat.grad[b.lo:b.hi]
        owner = self.owner[b.index]
        row = self.widx * self.row_stride[owner] + self.row_off[b.index]  # this worker's row of bucket b
        rc = _lib.lib().tony_ps_push(g.data_ptr(), int(g.dtype == torch.bfloat16), self.mapped[owner],
                                     row, int(self.wire_dtype == torch.bfloat16), b.numel, b.index,
                                     self.widx, (step + 1) & 0xFFFFFFFF, self.blocks[b.index],
                                     _lib.stream_ptr(self.device))
        _lib.check(rc, "tony_ps_push")
        self.pushed += b.numel * self.wesz

    def apply(self, b, step: int, opt, m: int, local_params: Optional[torch.Tensor] = None) -> None:
        """PS: apply bucket b from the landed rows (``opt``: FlatSGD / FlatAdam over this ps's masters,
        ``m``: the bucket's offset in them) and land the new variables in every worker's window."""
        from ..ops.optim import FlatAdam

        if self.dead is not None:
            raise PSPlaneError(self.dead)
        adam = isinstance(opt, FlatAdam)
        s0 = opt.m if adam else opt.v
        s1 = opt.v if adam else None
        stream = _lib.stream_ptr(self.device)
        rc = _lib.lib().tony_ps_apply(
            self.window, self.row_off[b.index], self.row_stride[self.rank], len(self.worker_ranks),
            int(self.wire_dtype == torch.bfloat16), b.numel, b.lo, opt.w.data_ptr() + 4 * m, s0.data_ptr() + 4 * m,
            None if s1 is None else s1.data_ptr() + 4 * m, opt._hp_dev.data_ptr(), int(adam), self._worker_windows,
            None if local_params is None else local_params.data_ptr(), int(self.flat.data.dtype == torch.bfloat16),
            b.index, (step + 1) & 0xFFFFFFFF, int(not self.sync), SPIN_S, self.blocks[b.index], stream)
        _lib.check(rc, "tony_ps_apply")

    def land(self, step: int) -> None:
        """Worker: wait for every bucket's new variables and copy them into the flat parameters."""
        stream = _lib.stream_ptr(self.device)
        rc = _lib.lib().tony_ps_land(self.window, self._land_table.data_ptr(), len(self.buckets),
                                     self.flat.data.data_ptr(), int(self.flat.data.dtype == torch.bfloat16),
                                     (step + 1) & 0xFFFFFFFF, SPIN_S, stream)
        _lib.check(rc, "tony_ps_land")
        self._poll_error(stream)

    def end_step(self) -> None:
        """PS: queue the error-word check after this step's applies."""
        self._poll_error(_lib.stream_ptr(self.device))

    def close(self) -> None:
        if self.window is None:
            return
        torch.cuda.synchronize(self.device)
        dist.barrier(group=self.group)  # nobody writes into a window after this
        L = _lib.lib()
        for p in self._opened:
            L.tony_xgmi_close(p)
        L.tony_xgmi_free(self.window)
        self.window = None
        self._opened = []

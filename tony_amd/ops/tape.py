"""Tape segments: one autograd node for a whole sub-network of tony_amd ops.

Every fused op (conv+BN+ReLU, fused 1x1 heads, pools, zero-copy concat, ...) is a Python
``torch.autograd.Function``.  Through ``Function.apply`` each costs ~10 us of host time in the
forward (node creation, input unpacking, SavedVariable packing, output wrapping) and again in the
backward (the engine's PyNode call, output validation), ~900 nodes per Inception-v3 step: with the
GPU step at ~14 ms the host issue time had become the limit (bench ``host_ms_per_step_unblocked``).

``segment(run, x, params)`` runs ``run(x)`` -- e.g. an Inception block -- as ONE autograd node:
inside it the ops' ``forward`` staticmethods are called directly on a light context object and
recorded on a tape (``apply`` below is what the ops' wrappers call instead of ``Fn.apply``); the
node's backward replays the tape in reverse, calling each op's ``backward`` with the gradients of
its outputs and routing the returned input gradients (summed when a tensor feeds several ops).
Semantics kept from the autograd engine:

* streams -- an op's backward runs on the stream its forward ran on (the Inception branch
  streams, ops/streams.py); a gradient produced on another stream is waited for with an event and
  held until ``streams.end()`` (its block belongs to the producer stream's allocator pool);
* memory -- each op's recorded context is dropped as soon as its backward has been issued, so the
  activations are recycled in the same order as under autograd;
* ``needs_input_grad`` -- true for the segment input (if it requires grad), every tensor produced
  on the tape and every parameter that requires grad;
* undefined output gradients are materialised as zeros (``set_materialize_grads`` default);
* parameter gradients an op returns (no in-place gradient slot) are summed per parameter and
  returned by the segment node, so autograd accumulates them into ``.grad`` as usual.

Measured on MI355X (bench.py eager, alternating A/B, profiles/r2s3_tape_segments_ab.log): correct
(tests/test_tape_gpu.py) but the step ran 15.05-15.30 ms with tapes vs 14.26-14.68 ms without, the
GPU time itself 0.8 ms longer, and no measurable host saving -- so segments are opt-in
(``TONY_TAPE=1``).

Reference parity: TonY leaves the training step to the framework; this is the
host-side half of running that step at MI355X speed.
"""
from __future__ import annotations

import os
from typing import Callable, Dict, List, Optional, Sequence

import torch

from . import streams

ENABLED = os.environ.get("TONY_TAPE", "0") == "1"

_active: List[Optional["Tape"]] = [None]


class _Ctx:
    """The subset of the autograd ctx API the tony_amd ops use."""

    __slots__ = ("_saved", "needs_input_grad", "__dict__")

    def __init__(self, needs):
        self._saved = ()
        self.needs_input_grad = needs

    def save_for_backward(self, *tensors):
        self._saved = tensors

    @property
    def saved_tensors(self):
        return self._saved


class UntrackedTensorError(RuntimeError):
    """A recorded op received a tensor no recorded op produced: some code in the segment ran a plain
    PyTorch op on an activation, whose gradient the tape cannot route."""


class Tape:
    __slots__ = ("entries", "diff", "params", "stream", "known")

    def __init__(self, x: torch.Tensor, params: Sequence[torch.Tensor], buffers: Sequence[torch.Tensor] = ()):
        self.entries: list = []
        self.diff = set()  # ids of tensors gradients flow to (the input, tape outputs)
        if x.requires_grad:
            self.diff.add(id(x))
        self.params = {id(p): i for i, p in enumerate(params)}
        for p in params:
            if p.requires_grad:
                self.diff.add(id(p))
        # tensors that may enter an op without being produced on the tape: the input, the parameters,
        # the modules' buffers (BN running statistics)
        self.known = {id(x), *self.params, *(id(b) for b in buffers)}
        self.stream = torch.cuda.current_stream(x.device) if x.is_cuda else None

    def record(self, fn, args):
        diff, known = self.diff, self.known
        for a in args:
            if isinstance(a, torch.Tensor) and id(a) not in diff and id(a) not in known:
                raise UntrackedTensorError(f"{fn.__name__} got a tensor {tuple(a.shape)} produced outside the "
                                           "segment's recorded ops")
        needs = tuple(isinstance(a, torch.Tensor) and id(a) in diff for a in args)
        ctx = _Ctx(needs)
        out = fn.forward(ctx, *args)
        outs = out if isinstance(out, tuple) else (out,)
        for o in outs:
            if isinstance(o, torch.Tensor):
                diff.add(id(o))
        stream = torch.cuda.current_stream() if self.stream is not None else None
        self.entries.append((fn, ctx, args, outs, stream))
        return out

    def backward(self, x: torch.Tensor, out: int, dout: torch.Tensor, nparams: int):
        """(dx, [d param]) from the gradient of the segment output (``out``: its id)."""
        home = self.stream
        grads: Dict[int, list] = {out: [dout, home]}  # id -> [gradient, stream it was produced on]
        dparams: List[Optional[torch.Tensor]] = [None] * nparams
        pid = self.params
        entries = self.entries
        for n in range(len(entries) - 1, -1, -1):
            fn, ctx, args, outs, stream = entries[n]
            entries[n] = None  # the op's saved activations go back to the allocator as in autograd
            gs = [grads.pop(id(o) if not isinstance(o, _Ref) else o.id, None)
                  if isinstance(o, (torch.Tensor, _Ref)) else None for o in outs]
            if all(e is None for e in gs):
                continue  # nothing flows back through this op
            if stream is not None:
                for e in gs:
                    if e is not None and e[1] is not stream:
                        _wait(stream, e[1])
                        streams.keep(e[0])  # read on this stream, allocated on the producer's
            gl = [e[0] if e is not None else (torch.zeros_like(o) if isinstance(o, torch.Tensor) else
                                             o.zeros() if isinstance(o, _Ref) else None)
                  for e, o in zip(gs, outs)]
            prev = None
            if stream is not None and stream is not torch.cuda.current_stream():
                prev = torch.cuda.current_stream()
                torch.cuda.set_stream(stream)
            try:
                ins = fn.backward(ctx, *gl)
                if not isinstance(ins, tuple):
                    ins = (ins,)
                for a, g in zip(args, ins):
                    if g is None or not isinstance(a, torch.Tensor):
                        continue
                    k = id(a)
                    i = pid.get(k)
                    if i is not None:  # a parameter without an in-place gradient slot
                        dparams[i] = g if dparams[i] is None else dparams[i] + g
                        continue
                    cur = grads.get(k)
                    if cur is not None:
                        if cur[1] is not stream:
                            _wait(stream, cur[1])
                            streams.keep(cur[0])
                        g = cur[0] + g
                    grads[k] = [g, stream]
            finally:
                if prev is not None:
                    torch.cuda.set_stream(prev)
        e = grads.pop(id(x), None)
        dx = None
        if e is not None:
            if e[1] is not home:
                _wait(home, e[1])
                streams.keep(e[0])
            dx = e[0]
        return dx, dparams


class _Ref:
    """Stands in for the segment's output in the tape (the output holds the segment node, which holds
    the tape: a strong reference back would be a cycle only the cyclic GC could free)."""

    __slots__ = ("id", "shape", "stride", "dtype", "device")

    def __init__(self, t: torch.Tensor):
        self.id, self.shape, self.stride = id(t), tuple(t.shape), t.stride()
        self.dtype, self.device = t.dtype, t.device

    def zeros(self) -> torch.Tensor:
        return torch.empty_strided(self.shape, self.stride, dtype=self.dtype, device=self.device).zero_()


def _wait(stream: Optional[torch.cuda.Stream], producer: Optional[torch.cuda.Stream]) -> None:
    if stream is None or producer is None or producer is stream:
        return
    streams.fork(producer, stream)


def recording() -> bool:
    """Inside a segment's forward (autograd's grad mode is off there, but the ops are differentiated)."""
    return _active[0] is not None


def apply(fn, *args):
    """``fn.apply(*args)``, or -- inside a segment -- ``fn.forward`` recorded on the segment's tape."""
    t = _active[0]
    if t is None:
        return fn.apply(*args)
    return t.record(fn, args)


class _SegmentFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, run, buffers, x, *params):
        tape = Tape(x, params, buffers)
        prev = _active[0]
        _active[0] = tape
        try:
            out = run(x)
        finally:
            _active[0] = prev
        if not isinstance(out, torch.Tensor):
            raise TypeError("a tape segment returns one tensor")
        if not tape.entries or not any(o is out for o in tape.entries[-1][3]):
            raise ValueError("a tape segment must end with a recorded op that returns its output")
        fn, lctx, args, outs, stream = tape.entries[-1]
        tape.entries[-1] = (fn, lctx, args, tuple(_Ref(o) if o is out else o for o in outs), stream)
        ctx.tape = tape
        ctx.x = x
        ctx.out = id(out)
        ctx.nparams = len(params)
        return out

    @staticmethod
    def backward(ctx, dout):
        tape = ctx.tape
        dx, dparams = tape.backward(ctx.x, ctx.out, dout, ctx.nparams)
        ctx.tape = None  # drop the recorded contexts and activations now
        return (None, None, dx, *dparams)


def segment(run: Callable[[torch.Tensor], torch.Tensor], x: torch.Tensor, params: Sequence[torch.Tensor],
            buffers: Sequence[torch.Tensor] = ()):
    """``run(x)`` as one autograd node (see the module docstring); plain ``run(x)`` when tapes are off,
    grad mode is off or a tape is already recording.  ``params`` / ``buffers``: every parameter and
    buffer the ops of ``run`` take.  Every op in ``run`` must go through ``apply`` (a plain PyTorch op
    on an activation raises UntrackedTensorError when the next recorded op consumes its result)."""
    if not ENABLED or not torch.is_grad_enabled() or _active[0] is not None:
        return run(x)
    return _SegmentFn.apply(run, tuple(buffers), x, *params)

"""Fused optimizers over flat parameter shards (HIP kernels in csrc/optim.hip).

``FlatSGD`` / ``FlatAdam`` own an fp32 master copy of a flat parameter shard
plus its optimizer state, consume a flat gradient (bf16 or fp32) and write the
updated bf16 compute copy in the same pass.  The PS shard (``tony_amd.parallel.ps``)
and the data-parallel engine use them directly; on CPU tensors the same update
is computed with PyTorch ops (used by the CPU test-suite and local mode).

Hyper-parameters are kept in a device tensor that is refreshed (a 36-byte H2D
copy) before each step, so a captured HIP graph sees the current lr / step.
"""
from __future__ import annotations

import torch

from . import _lib


class _FlatOptimizer:
    n_hp = 0

    def __init__(self, master: torch.Tensor, lr: float, weight_decay: float = 0.0):
        if master.dtype != torch.float32 or master.dim() != 1:
            raise TypeError("master shard must be a flat fp32 tensor")
        if master.numel() % 4:
            raise ValueError("flat shard length must be a multiple of 4 (pad the buffer)")
        self.w = master
        self.lr = float(lr)
        self.weight_decay = float(weight_decay)
        self.grad_scale = 1.0
        self.step_count = 0
        dev = master.device
        self._hp_last = None
        self._hp_dev = torch.zeros(self.n_hp, dtype=torch.float32, device=dev)

    def _hp_values(self):
        raise NotImplementedError

    def _push_hp(self):
        if self.w.is_cuda and torch.cuda.is_current_stream_capturing():
            return  # graph capture: the Trainer refreshes hp before every replay
        vals = [float(v) for v in self._hp_values()]
        if vals == self._hp_last:
            return  # unchanged (constant-lr SGD): no H2D traffic at all
        # pageable source: the copy is staged before copy_ returns, so the host
        # may rewrite its values for the next step without racing the DMA
        self._hp_dev.copy_(torch.tensor(vals, dtype=torch.float32), non_blocking=True)
        self._hp_last = vals

    def begin_step(self):
        """Advance the step counter and push this step's hyper-parameters (before any apply_range)."""
        self.step_count += 1
        if self.w.is_cuda:
            self._push_hp()

    def apply_range(self, grad: torch.Tensor, lo: int = 0, out_bf16: torch.Tensor | None = None):
        raise NotImplementedError

    def step(self, grad: torch.Tensor, out_bf16: torch.Tensor | None = None):
        """One whole-shard update: ``begin_step`` + ``apply_range`` over every element."""
        if grad.numel() != self.w.numel():
            raise ValueError("grad / shard size mismatch")
        self.begin_step()
        self.apply_range(grad, 0, out_bf16)

    def state_dict(self):
        raise NotImplementedError


class FlatSGD(_FlatOptimizer):
    """SGD with (Nesterov) momentum: v = mu*v + g + wd*w ; w -= lr*v (TF MomentumOptimizer semantics)."""

    n_hp = 6

    def __init__(self, master, lr, momentum=0.9, weight_decay=0.0, nesterov=False, resync=False):
        super().__init__(master, lr, weight_decay)
        self.momentum = float(momentum)
        self.nesterov = bool(nesterov)
        # resync: the bf16 compute copy (``out_bf16``) is the parameters users see and may overwrite
        # (load_state_dict, broadcast_parameters); elements changed there re-seed the fp32 master
        # before the update (csrc/optim.hip sgd_kernel).  Off for the PS, whose masters are the truth.
        self.resync = bool(resync)
        self.v = torch.zeros_like(master)

    def _hp_values(self):
        return [self.lr, self.momentum, self.weight_decay, self.grad_scale, 1.0 if self.nesterov else 0.0,
                1.0 if self.resync else 0.0]

    def apply_range(self, grad: torch.Tensor, lo: int = 0, out_bf16: torch.Tensor | None = None):
        """Update master elements [lo, lo + grad.numel()) (one bucket of a sharded PS) with ``grad``;
        hyper-parameters are those pushed by the last ``begin_step``."""
        n = grad.numel()
        if lo < 0 or lo + n > self.w.numel() or lo % 4 or n % 4:
            raise ValueError(f"range [{lo}, {lo + n}) outside the {self.w.numel()}-element shard or not 4-aligned")
        if self.w.is_cuda:
            rc = _lib.lib().tony_sgd_step(self.w.data_ptr() + 4 * lo, self.v.data_ptr() + 4 * lo, grad.data_ptr(),
                                          int(grad.dtype == torch.bfloat16), _lib.ptr(out_bf16), n,
                                          self._hp_dev.data_ptr(), _lib.stream_ptr(self.w.device))
            _lib.check(rc, "tony_sgd_step")
            return
        w, v = self.w[lo:lo + n], self.v[lo:lo + n]
        if self.resync and out_bf16 is not None:
            changed = out_bf16 != w.to(out_bf16.dtype)
            w.copy_(torch.where(changed, out_bf16.float(), w))
        g = grad.float() * self.grad_scale + self.weight_decay * w
        v.mul_(self.momentum).add_(g)
        upd = g + self.momentum * v if self.nesterov else v
        w.add_(upd, alpha=-self.lr)
        if out_bf16 is not None:
            out_bf16.copy_(w)

    def state_dict(self):
        return {"kind": "sgd", "step": self.step_count, "momentum_buffer": self.v, "lr": self.lr}

    def load_state_dict(self, sd):
        self.step_count = int(sd["step"])
        self.v.copy_(sd["momentum_buffer"])
        self.lr = float(sd.get("lr", self.lr))


class FlatAdam(_FlatOptimizer):
    """Adam / AdamW (``decoupled=True``) with bias correction."""

    n_hp = 9

    def __init__(self, master, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0, decoupled=False):
        super().__init__(master, lr, weight_decay)
        self.b1, self.b2 = float(betas[0]), float(betas[1])
        self.eps = float(eps)
        self.decoupled = bool(decoupled)
        self.m = torch.zeros_like(master)
        self.v = torch.zeros_like(master)

    def _hp_values(self):
        t = self.step_count
        return [self.lr, self.b1, self.b2, self.eps, self.weight_decay, self.grad_scale,
                1.0 - self.b1 ** t, 1.0 - self.b2 ** t, 1.0 if self.decoupled else 0.0]

    def apply_range(self, grad: torch.Tensor, lo: int = 0, out_bf16: torch.Tensor | None = None):
        n = grad.numel()
        if lo < 0 or lo + n > self.w.numel() or lo % 4 or n % 4:
            raise ValueError(f"range [{lo}, {lo + n}) outside the {self.w.numel()}-element shard or not 4-aligned")
        if self.w.is_cuda:
            rc = _lib.lib().tony_adam_step(self.w.data_ptr() + 4 * lo, self.m.data_ptr() + 4 * lo,
                                           self.v.data_ptr() + 4 * lo, grad.data_ptr(),
                                           int(grad.dtype == torch.bfloat16), _lib.ptr(out_bf16), n,
                                           self._hp_dev.data_ptr(), _lib.stream_ptr(self.w.device))
            _lib.check(rc, "tony_adam_step")
            return
        t = self.step_count
        w, m, v = self.w[lo:lo + n], self.m[lo:lo + n], self.v[lo:lo + n]
        g = grad.float() * self.grad_scale
        if self.decoupled:
            w.mul_(1.0 - self.lr * self.weight_decay)
        else:
            g = g + self.weight_decay * w
        m.mul_(self.b1).add_(g, alpha=1 - self.b1)
        v.mul_(self.b2).addcmul_(g, g, value=1 - self.b2)
        denom = (v.sqrt() / (1 - self.b2 ** t) ** 0.5).add_(self.eps)
        w.addcdiv_(m, denom, value=-self.lr / (1 - self.b1 ** t))
        if out_bf16 is not None:
            out_bf16.copy_(w)

    def state_dict(self):
        return {"kind": "adam", "step": self.step_count, "exp_avg": self.m, "exp_avg_sq": self.v, "lr": self.lr}

    def load_state_dict(self, sd):
        self.step_count = int(sd["step"])
        self.m.copy_(sd["exp_avg"])
        self.v.copy_(sd["exp_avg_sq"])
        self.lr = float(sd.get("lr", self.lr))


def grad_stats(grad: torch.Tensor):
    """Return a device tensor [sum(g^2), any_nonfinite] for a flat gradient (H12)."""
    if grad.is_cuda:
        out = torch.empty(2, dtype=torch.float32, device=grad.device)
        rc = _lib.lib().tony_grad_stats(grad.data_ptr(), int(grad.dtype == torch.bfloat16), grad.numel(),
                                        out.data_ptr(), _lib.stream_ptr(grad.device))
        _lib.check(rc, "tony_grad_stats")
        return out
    g = grad.float()
    return torch.stack([(g * g).sum(), (~torch.isfinite(g)).any().float()])

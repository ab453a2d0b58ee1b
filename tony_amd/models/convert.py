"""State-dict conversion between the stock Inception-v3 graph and the fused one.

``inception_v3(fused=True)`` merges the 1x1 convs that read an Inception block's input (and the
avg-pool branch's 1x1) into one ``FusedHead`` (ops/fused.py): one conv weight and one BatchNorm
whose output channels are the concatenation of the branches' ``(b1 | b5[0] | b3[0] | bp)``, and the
branch chains lose their first layer.  ``stock_to_fused`` / ``fused_to_stock`` move parameters and
BN buffers between the two layouts, so a checkpoint of either trains in the other, and the fused
model can be checked layer by layer against the stock fp32 graph (tests/test_model_fp32_gpu.py).
"""
from __future__ import annotations

from typing import Dict, List, Tuple

import torch

from .inception_v3 import InceptionA, InceptionC, InceptionD, InceptionE, InceptionV3

_BN = ("weight", "bias", "running_mean", "running_var")

# per block type: (stock layers feeding the fused head, in split order), {fused chain layer: stock layer}
_HEADS = {
    InceptionA: (["b1", "b5.0", "b3.0", "bp"], {"b5": "b5.1", "b3.0": "b3.1", "b3.1": "b3.2"}),
    InceptionC: (["b1", "b7.0", "bd.0", "bp"], {"b7.0": "b7.1", "b7.1": "b7.2", "bd.0": "bd.1", "bd.1": "bd.2",
                                                "bd.2": "bd.3", "bd.3": "bd.4"}),
    InceptionD: (["b3.0", "b7.0"], {"b3": "b3.1", "b7.0": "b7.1", "b7.1": "b7.2", "b7.2": "b7.3"}),
    InceptionE: (["b1", "b3", "bd.0", "bp"], {"bd": "bd.1"}),
}


def _blocks(model: InceptionV3) -> List[Tuple[str, type]]:
    out = []
    for name, mod in model.named_modules():
        for t in _HEADS:
            if type(mod) is t:
                out.append((name, t))
    return out


def stock_to_fused(stock_sd: Dict[str, torch.Tensor], fused_model: InceptionV3) -> Dict[str, torch.Tensor]:
    """The fused model's state dict built from a stock (``fused=False``) Inception-v3 state dict."""
    out = dict(stock_sd)
    for name, t in _blocks(fused_model):
        heads, chain = _HEADS[t]
        srcs = [f"{name}.{h}" for h in heads]
        out[f"{name}.head.conv.weight"] = torch.cat([stock_sd[f"{s}.conv.weight"] for s in srcs], 0)
        for k in _BN:
            out[f"{name}.head.bn.{k}"] = torch.cat([stock_sd[f"{s}.bn.{k}"] for s in srcs], 0)
        out[f"{name}.head.bn.num_batches_tracked"] = stock_sd[f"{srcs[0]}.bn.num_batches_tracked"]
        for s in srcs:
            for k in list(out):
                if k.startswith(s + "."):
                    del out[k]
        moved = {}
        for dst, src in chain.items():
            for k, v in stock_sd.items():
                if k.startswith(f"{name}.{src}."):
                    moved[f"{name}.{dst}." + k[len(f"{name}.{src}."):]] = v
        for src in chain.values():
            for k in list(out):
                if k.startswith(f"{name}.{src}."):
                    del out[k]
        out.update(moved)
    want = set(fused_model.state_dict())
    missing, extra = want - set(out), set(out) - want
    if missing or extra:
        raise KeyError(f"stock -> fused conversion: missing {sorted(missing)[:5]} extra {sorted(extra)[:5]}")
    return out


def fused_to_stock(fused_sd: Dict[str, torch.Tensor], fused_model: InceptionV3,
                   stock_model: InceptionV3) -> Dict[str, torch.Tensor]:
    """The stock model's state dict from a fused one (inverse of ``stock_to_fused``)."""
    ssd = stock_model.state_dict()
    out = {k: v for k, v in fused_sd.items()}
    for name, t in _blocks(fused_model):
        heads, chain = _HEADS[t]
        widths = [ssd[f"{name}.{h}.conv.weight"].shape[0] for h in heads]
        moved = {}
        for dst, src in chain.items():
            for k, v in fused_sd.items():
                if k.startswith(f"{name}.{dst}."):
                    moved[f"{name}.{src}." + k[len(f"{name}.{dst}."):]] = v
        for k in list(out):  # the fused block's own keys go; the stock ones are written below
            if k.startswith(f"{name}.head.") or any(k.startswith(f"{name}.{dst}.") for dst in chain):
                del out[k]
        for key in ["conv.weight"] + [f"bn.{k}" for k in _BN]:
            parts = torch.split(fused_sd[f"{name}.head.{key}"], widths, 0)
            for h, p in zip(heads, parts):
                out[f"{name}.{h}.{key}"] = p.clone()
        for h in heads:
            out[f"{name}.{h}.bn.num_batches_tracked"] = fused_sd[f"{name}.head.bn.num_batches_tracked"]
        out.update(moved)
    want = set(ssd)
    missing, extra = want - set(out), set(out) - want
    if missing or extra:
        raise KeyError(f"fused -> stock conversion: missing {sorted(missing)[:5]} extra {sorted(extra)[:5]}")
    return out


def fused_grads_to_stock(fused_model: InceptionV3, stock_model: InceptionV3) -> Dict[str, torch.Tensor]:
    """Parameter gradients of the fused model in the stock model's parameter names (for checks)."""
    g = {k: p.grad for k, p in fused_model.named_parameters() if p.grad is not None}
    full = dict(fused_model.state_dict())
    full.update(g)
    conv = fused_to_stock(full, fused_model, stock_model)
    return {k: conv[k] for k, _ in stock_model.named_parameters()}

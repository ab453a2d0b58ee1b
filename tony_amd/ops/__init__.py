"""MI355X (gfx950) compute kernels of tony_amd.

Hand-written HIP kernels (``csrc/*.hip``) built in-tree into
``_tony_kernels.so`` and bound with ctypes:

* ``bn``     -- NHWC BatchNorm(+ReLU) training/inference fwd+bwd (H3/H4)
* ``loss``   -- fused softmax cross-entropy fwd+bwd (H9)
* ``optim``  -- flat-shard fused SGD-momentum / Adam(W) apply, grad stats (H10-H12)
* ``gemm``   -- MFMA bf16 GEMM (LDS-tiled, XCD-aware) for 1x1 convs / FC (H1/H8)
"""
from ._lib import KernelError, available, lib  # noqa: F401
from .bn import BatchNormAct2d, bn_act  # noqa: F401
from .loss import cross_entropy  # noqa: F401
from .optim import FlatAdam, FlatSGD, grad_stats  # noqa: F401

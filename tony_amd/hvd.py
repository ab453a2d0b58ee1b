"""``import tony_amd.hvd as hvd``: the Horovod-compatible API (implemented in tony_amd.parallel.hvd)."""
import sys

from .parallel import hvd as _impl

sys.modules[__name__] = _impl

"""``import tony_amd.kv as kv``: the MXNet-style kvstore (implemented in tony_amd.parallel.kvstore)."""
import sys

from .parallel import kvstore as _impl

sys.modules[__name__] = _impl

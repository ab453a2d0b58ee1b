"""Node GPU inventory and GPU/CPU slot allocation (the RM/NM resource model on one MI355X node).

TonY asks YARN for ``yarn.io/gpu`` resources and YARN's NodeManager isolates them
(T/util/Utils.java:193-211, HadoopCompatibleAdapter.existGPUResource).  On a
single MI355X node the coordinator owns that decision:

* inventory  -- amd-smi (native binding: BDF, UUID, NUMA node, VRAM) or, when
  ``tony.amd.fake-gpus >= 0``, a fake inventory for CI / local mode (SURVEY.md §4:
  "TONY_FAKE_GPUS"); ``/sys/class/kfd`` is the fallback when amd-smi is absent;
* allocation -- each task asking ``tony.<job>.gpus = g`` gets ``g`` free GPUs,
  preferring GPUs that share a NUMA node (the 8 GPUs of an MI355X node hang off
  2 sockets; all pairs are xGMI-connected, so NUMA locality of the host side is
  the placement criterion that matters);
* CPU pinning -- the task's CPUs are the cores of its first GPU's NUMA node.
"""
from __future__ import annotations

import glob
import logging
import os
import threading
from dataclasses import dataclass
from typing import Dict, List, Optional

from .. import native
from ..native import GpuDevice

LOG = logging.getLogger(__name__)


def _parse_cpulist(s: str) -> List[int]:
    out: List[int] = []
    for part in s.strip().split(","):
        if not part:
            continue
        if "-" in part:
            a, b = part.split("-")
            out.extend(range(int(a), int(b) + 1))
        else:
            out.append(int(part))
    return out


def numa_cpus(node: int) -> List[int]:
    try:
        with open(f"/sys/devices/system/node/node{node}/cpulist") as f:
            return _parse_cpulist(f.read())
    except OSError:
        return []


def num_numa_nodes() -> int:
    return max(1, len(glob.glob("/sys/devices/system/node/node[0-9]*")))


def _kfd_devices() -> List[GpuDevice]:
    out = []
    for props in sorted(glob.glob("/sys/class/kfd/kfd/topology/nodes/*/properties")):
        try:
            kv = dict(line.split() for line in open(props) if len(line.split()) == 2)
        except (OSError, ValueError):
            continue
        if int(kv.get("simd_count", "0")) <= 0:
            continue
        out.append(GpuDevice(len(out), numa_node=int(kv.get("numa_node", "-1"))))
    return out


def discover(fake_gpus: int = -1) -> List[GpuDevice]:
    """GPUs on this node.  ``fake_gpus >= 0`` returns that many fake devices."""
    if fake_gpus is not None and fake_gpus >= 0:
        nodes = num_numa_nodes()
        per = max(1, (fake_gpus + nodes - 1) // nodes)
        return [GpuDevice(i, bdf=f"fake:{i:02x}", uuid=f"fake-{i}", numa_node=min(i // per, nodes - 1),
                          vram_total_mb=288 * 1024, fake=True) for i in range(fake_gpus)]
    env = os.environ.get("TONY_FAKE_GPUS")
    if env is not None:
        return discover(int(env))
    devs = native.smi_devices()
    if not devs:
        devs = _kfd_devices()
    return devs


@dataclass
class Slot:
    gpus: List[int]
    numa_node: int
    cpus: List[int]


class GpuAllocator:
    def __init__(self, devices: List[GpuDevice]):
        self.devices = devices
        self._free = [d.index for d in devices]
        self._owner: Dict[int, str] = {}
        self._lock = threading.Lock()

    @property
    def total(self) -> int:
        return len(self.devices)

    def free_count(self) -> int:
        with self._lock:
            return len(self._free)

    def allocate(self, owner: str, n: int) -> Optional[Slot]:
        """Reserve ``n`` GPUs for ``owner`` (NUMA-local first); None if not enough are free."""
        if n <= 0:
            return Slot([], -1, [])
        with self._lock:
            if len(self._free) < n:
                return None
            by_node: Dict[int, List[int]] = {}
            for g in self._free:
                by_node.setdefault(self.devices[g].numa_node, []).append(g)
            # smallest NUMA group that fits, else fill from the largest groups
            fitting = sorted((len(v), k) for k, v in by_node.items() if len(v) >= n)
            if fitting:
                chosen = sorted(by_node[fitting[0][1]])[:n]
            else:
                chosen = []
                for _, k in sorted(((len(v), k) for k, v in by_node.items()), reverse=True):
                    chosen.extend(sorted(by_node[k])[: n - len(chosen)])
                    if len(chosen) == n:
                        break
            for g in chosen:
                self._free.remove(g)
                self._owner[g] = owner
        node = self.devices[chosen[0]].numa_node
        return Slot(chosen, node, numa_cpus(node) if node >= 0 else [])

    def release(self, owner: str) -> None:
        with self._lock:
            for g, o in list(self._owner.items()):
                if o == owner:
                    del self._owner[g]
                    self._free.append(g)
            self._free.sort()

    def owners(self) -> Dict[int, str]:
        with self._lock:
            return dict(self._owner)

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
* CPU pinning -- a task gets ``tony.<job>.vcores`` CPUs of its first GPU's NUMA node, sliced so that
  tasks on the same node get disjoint CPUs while there are enough (YARN's vcores as a cpuset);
* device ordinals -- amd-smi enumerates GPUs in its own order, HIP in KFD-topology order;
  ``hip_ordinals`` maps one to the other by PCI BDF so ``HIP_VISIBLE_DEVICES`` names the GPU the
  allocator picked (and the NUMA binding matches it); the task re-checks the BDF it sees
  (``verify_visible_device``, TONY_GPU_BDFS).
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


KFD_TOPOLOGY = "/sys/class/kfd/kfd/topology/nodes"


def _kfd_node_id(path: str) -> int:
    try:
        return int(os.path.basename(os.path.dirname(path)))
    except ValueError:
        return 1 << 30


def kfd_gpu_bdfs(root: str = KFD_TOPOLOGY) -> List[str]:
    """PCI BDFs ("dddd:bb:dd.f") of the GPU agents in KFD topology-node order -- the order in which
    ROCr/HIP number devices (HIP ordinal i = i-th GPU node)."""
    out = []
    for props in sorted(glob.glob(os.path.join(root, "*", "properties")), key=_kfd_node_id):
        try:
            kv = dict(line.split() for line in open(props) if len(line.split()) == 2)
        except (OSError, ValueError):
            continue
        if int(kv.get("simd_count", "0")) <= 0:
            continue
        loc, dom = int(kv.get("location_id", "0")), int(kv.get("domain", "0"))
        out.append(f"{dom:04x}:{(loc >> 8) & 0xff:02x}:{(loc >> 3) & 0x1f:02x}.{loc & 0x7}")
    return out


def _norm_bdf(bdf: str) -> str:
    """Canonical lower-case dddd:bb:dd.f (amd-smi may print without the domain or the function)."""
    b = bdf.strip().lower()
    if b.count(":") == 1:
        b = "0000:" + b
    if "." not in b:
        b += ".0"
    return b


def hip_ordinals(devices: List[GpuDevice], kfd_bdfs: Optional[List[str]] = None) -> Dict[int, int]:
    """amd-smi index -> HIP ordinal, matched by BDF.  Identity for fake inventories; raises when a
    real GPU's BDF is not among the HIP-visible devices (wrong pinning must not pass silently)."""
    if not devices or all(d.fake for d in devices):
        return {d.index: d.index for d in devices}
    kfd = [_norm_bdf(b) for b in (kfd_bdfs if kfd_bdfs is not None else kfd_gpu_bdfs())]
    if not kfd:
        LOG.warning("KFD topology unreadable: assuming amd-smi order == HIP order")
        return {d.index: d.index for d in devices}
    pos = {b: i for i, b in enumerate(kfd)}
    out = {}
    for d in devices:
        if not d.bdf:
            raise RuntimeError(f"GPU {d.index} has no PCI BDF: cannot map it to a HIP ordinal")
        b = _norm_bdf(d.bdf)
        if b not in pos:
            raise RuntimeError(f"GPU {d.index} ({b}) is not among the HIP-visible devices {kfd}")
        out[d.index] = pos[b]
    return out


def verify_visible_device(device_index: int = 0) -> Optional[str]:
    """In a task: the BDF torch/HIP sees for ``device_index`` vs the one the coordinator pinned
    (TONY_GPU_BDFS, same order as HIP_VISIBLE_DEVICES).  Returns the BDF; raises on a mismatch."""
    want = [b for b in os.environ.get("TONY_GPU_BDFS", "").split(",") if b]
    if not want or any(b.startswith("fake") for b in want):
        return None  # local mode's fake inventory (tony.amd.fake-gpus): nothing real to verify against
    mode = os.environ.get("TONY_VISIBLE_MODE") or ("hip" if os.environ.get("HIP_VISIBLE_DEVICES") is not None
                                                   else "")
    if mode in ("hip", "rocr"):
        pos = device_index  # the task sees only its GPUs, in allocation order
    elif mode == "none":   # every GPU visible: the task's GPUs are the ordinals the coordinator named
        ords = [int(o) for o in os.environ.get("TONY_HIP_ORDINALS", "").split(",") if o.strip()]
        if device_index not in ords:
            raise RuntimeError(f"HIP device {device_index} is not among this task's GPUs {ords} "
                               "(TONY_HIP_ORDINALS)")
        pos = ords.index(device_index)
    else:
        return None
    if pos >= len(want):
        return None
    import torch

    p = torch.cuda.get_device_properties(device_index)
    got = f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}.0"
    exp = _norm_bdf(want[pos])
    if exp.rsplit(".", 1)[0] != got.rsplit(".", 1)[0]:
        raise RuntimeError(f"HIP device {device_index} is {got} but the coordinator pinned {exp}: "
                           f"the {mode} pinning does not select the allocated GPU")
    return got


def _kfd_devices() -> List[GpuDevice]:
    out = []
    for props in sorted(glob.glob(os.path.join(KFD_TOPOLOGY, "*", "properties")), key=_kfd_node_id):
        try:
            kv = dict(line.split() for line in open(props) if len(line.split()) == 2)
        except (OSError, ValueError):
            continue
        if int(kv.get("simd_count", "0")) <= 0:
            continue
        loc, dom = int(kv.get("location_id", "0")), int(kv.get("domain", "0"))
        bdf = f"{dom:04x}:{(loc >> 8) & 0xff:02x}:{(loc >> 3) & 0x1f:02x}.{loc & 0x7}"
        out.append(GpuDevice(len(out), bdf=bdf, numa_node=int(kv.get("numa_node", "-1"))))
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


def rank_cpus(hip_ordinal: int, local_ranks_ordinals: List[int], devices: Optional[List[GpuDevice]] = None,
              cpus_of_node=None, allowed: Optional[List[int]] = None) -> List[int]:
    """CPUs for the rank driving HIP device ``hip_ordinal`` when one process per GPU runs on this node
    (bench.py --gpus N, torchrun): the CPUs of that GPU's NUMA node that this process may use, split evenly
    among the local ranks whose GPUs share the node (``local_ranks_ordinals``: every local rank's HIP
    ordinal, in local-rank order), so ranks do not contend for one core and each issues its kernels from
    CPUs next to its GPU -- what the coordinator's slot allocator does for launcher tasks
    (GpuAllocator._take_cpus; TaskExecutor.java:189-238 owns placement per task in the reference).
    ``devices``: the GPUs in HIP-ordinal order (default: the KFD topology).  Empty when nothing is known
    (no NUMA information, or none of the node's CPUs allowed): the caller then leaves affinity alone."""
    devs = devices if devices is not None else _kfd_devices()
    cpus_of_node = cpus_of_node or numa_cpus
    if hip_ordinal < 0 or hip_ordinal >= len(devs):
        return []
    node = devs[hip_ordinal].numa_node
    if node is None or node < 0:
        return []
    ok = set(allowed if allowed is not None else (os.sched_getaffinity(0) if hasattr(os, "sched_getaffinity")
                                                    else []))
    cpus = [c for c in cpus_of_node(node) if not ok or c in ok]
    if not cpus:
        return []
    peers = [o for o in local_ranks_ordinals if 0 <= o < len(devs) and devs[o].numa_node == node]
    if hip_ordinal not in peers or len(peers) <= 1:
        return cpus
    k, n = peers.index(hip_ordinal), len(peers)
    share = len(cpus) // n
    if share < 1:
        return cpus
    return cpus[k * share:(k + 1) * share]


@dataclass
class Slot:
    gpus: List[int]
    numa_node: int
    cpus: List[int]


class GpuAllocator:
    def __init__(self, devices: List[GpuDevice], cpus_of_node=None):
        self.devices = devices
        self._free = [d.index for d in devices]
        self._owner: Dict[int, str] = {}
        self._sharers: Dict[int, List[str]] = {}
        self._cpu_owner: Dict[int, str] = {}
        self._cpus_of_node = cpus_of_node or numa_cpus
        self._lock = threading.Lock()

    @property
    def total(self) -> int:
        return len(self.devices)

    def free_count(self) -> int:
        with self._lock:
            return len(self._free)

    def allocate(self, owner: str, n: int, vcores: int = 0) -> Optional[Slot]:
        """Reserve ``n`` GPUs for ``owner`` (NUMA-local first) and ``vcores`` CPUs of their NUMA node
        (0: the whole node); None if not enough GPUs are free."""
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
        return Slot(chosen, node, self._take_cpus(owner, node, vcores) if node >= 0 else [])

    def share(self, owner: str, gpu: int, vcores: int = 0) -> Slot:
        """A slot on GPU ``gpu`` that another task owns (the 0-GPU ps placed beside a worker,
        utils/core.ps_shares_worker_gpu): the GPU stays owned by its task; ``owner`` is recorded as a
        sharer (``sharers``) and gets ``vcores`` CPUs of the GPU's NUMA node."""
        with self._lock:
            self._sharers.setdefault(gpu, []).append(owner)
        node = self.devices[gpu].numa_node
        return Slot([gpu], node, self._take_cpus(owner, node, vcores) if node >= 0 else [])

    def sharers(self) -> Dict[int, List[str]]:
        with self._lock:
            return {g: list(o) for g, o in self._sharers.items()}

    def _take_cpus(self, owner: str, node: int, vcores: int) -> List[int]:
        """``vcores`` CPUs of ``node`` for ``owner``: unowned ones first, then (oversubscribed) the
        least recently handed out; the whole node when vcores <= 0."""
        cpus = self._cpus_of_node(node)
        if vcores <= 0 or vcores >= len(cpus):
            return list(cpus)
        with self._lock:
            free = [c for c in cpus if c not in self._cpu_owner]
            take = free[:vcores]
            if len(take) < vcores:
                shared = [c for c in cpus if c not in take]
                take += shared[:vcores - len(take)]
            for c in take:
                self._cpu_owner.setdefault(c, owner)
        return sorted(take)

    def release(self, owner: str) -> None:
        """Return ``owner``'s GPUs and CPUs.  A GPU stays off the free list while a task that shares it
        (``share``) is still alive, even after its owner left: it goes back when its last sharer does."""
        with self._lock:
            for g in list(self._sharers):
                self._sharers[g] = [o for o in self._sharers[g] if o != owner]
                if not self._sharers[g]:
                    del self._sharers[g]
                    if g not in self._owner and g not in self._free:  # its owner already left
                        self._free.append(g)
            for g, o in list(self._owner.items()):
                if o == owner:
                    del self._owner[g]
                    if g not in self._sharers:
                        self._free.append(g)
            self._free.sort()
            for c, o in list(self._cpu_owner.items()):
                if o == owner:
                    del self._cpu_owner[c]

    def owners(self) -> Dict[int, str]:
        with self._lock:
            return dict(self._owner)

"""Horovod-on-TonY pieces: slot planning, the rendezvous KV server and the driver.

Parity map: SlotInfo (T/horovod/SlotInfo.java:21-98), HorovodClusterSpec
(T/horovod/HorovodClusterSpec.java), DriverCallbackInfo
(T/horovod/DriverCallbackInfo.java), the driver process
(TR/horovod_driver.py + T/horovod/HorovodDriver.java:48-331).
Horovod itself is not installed: the rendezvous server is implemented here and
the worker data plane is tony_amd.parallel.hvd (RCCL over xGMI).
"""
from __future__ import annotations

import json
from dataclasses import asdict, dataclass
from typing import Dict, List, Sequence, Tuple


@dataclass
class SlotInfo:
    hostname: str
    rank: int
    localRank: int  # noqa: N815 (wire names)
    crossRank: int  # noqa: N815
    size: int
    localSize: int  # noqa: N815
    crossSize: int  # noqa: N815

    @classmethod
    def from_dict(cls, d) -> "SlotInfo":
        return cls(d["hostname"], int(d["rank"]), int(d["localRank"]), int(d["crossRank"]), int(d["size"]),
                   int(d["localSize"]), int(d["crossSize"]))


def parse_hosts(worker_list: str) -> List[Tuple[str, int]]:
    """"h1:2,h2:1" -> [("h1", 2), ("h2", 1)]."""
    out = []
    for item in worker_list.split(","):
        item = item.strip()
        if not item:
            continue
        host, n = item.rsplit(":", 1)
        out.append((host, int(n)))
    return out


def host_assignments(hosts: Sequence[Tuple[str, int]], min_np: int = 1) -> List[SlotInfo]:
    """Horovod's static slot plan: ranks fill hosts in order; cross_rank = the host's
    position among hosts that have this local rank."""
    size = sum(n for _, n in hosts)
    if size < min_np:
        raise ValueError(f"need at least {min_np} slots, have {size}")
    slots: List[SlotInfo] = []
    rank = 0
    for host, n in hosts:
        for local in range(n):
            cross_hosts = [h for h, m in hosts if m > local]
            slots.append(SlotInfo(host, rank, local, cross_hosts.index(host), size, n, len(cross_hosts)))
            rank += 1
    return slots


def fake_host_plan(worker_list: str) -> List[SlotInfo]:
    """Test-mode plan of TR/horovod_driver.py:44-65 (two slots on the first host)."""
    host = worker_list.split(":")[0]
    return [SlotInfo(host, 0, 0, 0, 2, 2, 1), SlotInfo(host, 1, 1, 1, 2, 2, 1)]


def slots_json(slots: Sequence[SlotInfo]) -> str:
    return json.dumps([asdict(s) for s in slots])


@dataclass
class DriverCallbackInfo:
    port: str
    host: str
    slotInfos: List[Dict]  # noqa: N815

    def to_json(self) -> str:
        return json.dumps(asdict(self))

    @classmethod
    def from_json(cls, s: str) -> "DriverCallbackInfo":
        d = json.loads(s)
        return cls(str(d["port"]), d["host"], list(d["slotInfos"]))


@dataclass
class HorovodClusterSpec:
    slotInfos: List[Dict]  # noqa: N815
    port: str
    amHost: str  # noqa: N815
    sameHostTaskIndexList: List[int]  # noqa: N815

    def to_json(self) -> str:
        return json.dumps(asdict(self))

    @classmethod
    def from_json(cls, s: str) -> "HorovodClusterSpec":
        d = json.loads(s)
        return cls(list(d["slotInfos"]), str(d["port"]), d["amHost"], [int(i) for i in d["sameHostTaskIndexList"]])

"""ctypes binding of the native host runtime (tony_native.cpp -> _tony_native.so).

``spawn`` / ``kill_tree`` / ``reserve_port`` and the amd-smi GPU inventory.  The
library is built in-tree by ``tony_amd.ops.build`` (``__graft_entry__.build()``).
If it is missing (e.g. a source checkout that was never built) the process
helpers fall back to the Python standard library, logged once; the amd-smi
binding then reports "no GPUs", so inventories must come from
``tony.amd.fake-gpus`` or ``/sys/class/kfd``.
"""
from __future__ import annotations

import ctypes
import logging
import os
import signal
import socket
import subprocess
from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence

LOG = logging.getLogger(__name__)
SO_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_tony_native.so")

_lib = None
_load_failed = False


class _GpuInfo(ctypes.Structure):
    _fields_ = [("bdf", ctypes.c_char * 32), ("uuid", ctypes.c_char * 64), ("numa_node", ctypes.c_int32),
                ("vram_total_mb", ctypes.c_uint32)]


class _GpuSample(ctypes.Structure):
    _fields_ = [("gfx_busy_pct", ctypes.c_uint32), ("mem_busy_pct", ctypes.c_uint32),
                ("vram_used_mb", ctypes.c_uint32), ("vram_total_mb", ctypes.c_uint32), ("power_w", ctypes.c_double),
                ("temp_c", ctypes.c_double), ("ecc_correctable", ctypes.c_uint64),
                ("ecc_uncorrectable", ctypes.c_uint64), ("xgmi_read_kb", ctypes.c_uint64),
                ("xgmi_write_kb", ctypes.c_uint64), ("xgmi_link_speed_gbps", ctypes.c_uint32),
                ("xgmi_link_width", ctypes.c_uint32)]


def lib():
    global _lib, _load_failed
    if _lib is not None or _load_failed:
        return _lib
    try:
        h = ctypes.CDLL(SO_PATH)
    except OSError as e:
        _load_failed = True
        LOG.warning("native runtime %s unavailable (%s); using Python fallbacks", SO_PATH, e)
        return None
    c_char_pp = ctypes.POINTER(ctypes.c_char_p)
    h.tony_spawn.argtypes = [c_char_pp, c_char_pp, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int,
                             ctypes.POINTER(ctypes.c_int)]
    h.tony_kill_tree.argtypes = [ctypes.c_int, ctypes.c_int]
    h.tony_reserve_port.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_int)]
    h.tony_release_port.argtypes = [ctypes.c_int]
    h.tony_smi_init.argtypes = []
    h.tony_smi_info.argtypes = [ctypes.c_int, ctypes.POINTER(_GpuInfo)]
    h.tony_smi_sample.argtypes = [ctypes.c_int, ctypes.POINTER(_GpuSample)]
    h.tony_smi_link.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_int)]
    h.tony_smi_shutdown.restype = None
    _lib = h
    return _lib


def available() -> bool:
    return lib() is not None


# -- processes --------------------------------------------------------------------------
def _cstr_array(items: Sequence[str]):
    arr = (ctypes.c_char_p * (len(items) + 1))()
    arr[:-1] = [s.encode() for s in items]
    arr[-1] = None
    return arr


def spawn(argv: Sequence[str], env: Dict[str, str], cwd: Optional[str] = None, stdout: Optional[str] = None,
          stderr: Optional[str] = None, new_session: bool = True) -> int:
    """Start ``argv`` in its own session (pgid == pid); returns the pid."""
    L = lib()
    if L is not None:
        pid = ctypes.c_int(-1)
        envp = _cstr_array([f"{k}={v}" for k, v in env.items()])
        rc = L.tony_spawn(_cstr_array(list(argv)), envp, (cwd or "").encode(), (stdout or "").encode(),
                          (stderr or "").encode(), int(new_session), ctypes.byref(pid))
        if rc != 0:
            raise OSError(-rc, f"spawn {argv[0]}: {os.strerror(-rc)}")
        return pid.value
    out = open(stdout, "ab") if stdout else None
    err = open(stderr, "ab") if stderr else None
    try:
        p = subprocess.Popen(list(argv), env=env, cwd=cwd, stdout=out, stderr=err, stdin=subprocess.DEVNULL,
                             start_new_session=new_session)
    finally:
        for f in (out, err):
            if f:
                f.close()
    return p.pid


def kill_tree(pgid: int, sig: int = signal.SIGKILL) -> bool:
    L = lib()
    if L is not None:
        return L.tony_kill_tree(int(pgid), int(sig)) == 0
    try:
        os.killpg(pgid, sig)
        return True
    except (ProcessLookupError, PermissionError):
        return False


class PortReservation:
    """A bound (and listening) TCP port held until ``release()``."""

    def __init__(self, port: int = 0, reuse_port: bool = False):
        self.reuse_port = reuse_port
        L = lib()
        self._sock = None
        self._fd = -1
        if L is not None:
            fd = ctypes.c_int(-1)
            rc = L.tony_reserve_port(int(port), int(reuse_port), ctypes.byref(fd))
            if rc < 0:
                raise OSError(-rc, f"reserve port {port}: {os.strerror(-rc)}")
            self.port = rc
            self._fd = fd.value
        else:
            s = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
            s.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
            if reuse_port:
                s.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEPORT, 1)
            s.bind(("", port))
            s.listen(16)
            self._sock = s
            self.port = s.getsockname()[1]

    def release(self):
        if self._sock is not None:
            self._sock.close()
            self._sock = None
        if self._fd >= 0:
            lib().tony_release_port(self._fd)
            self._fd = -1

    @property
    def held(self) -> bool:
        return self._sock is not None or self._fd >= 0

    def __del__(self):
        try:
            self.release()
        except Exception:  # noqa: BLE001
            pass


# -- GPUs -------------------------------------------------------------------------------
@dataclass
class GpuDevice:
    index: int
    bdf: str = ""
    uuid: str = ""
    numa_node: int = -1
    vram_total_mb: int = 0
    fake: bool = False


@dataclass
class GpuSample:
    gfx_busy_pct: float = 0.0
    mem_busy_pct: float = 0.0
    vram_used_mb: float = 0.0
    vram_total_mb: float = 0.0
    power_w: float = 0.0
    temp_c: float = 0.0
    ecc_correctable: int = 0
    ecc_uncorrectable: int = 0
    xgmi_read_kb: int = 0      # accumulated over all links since boot
    xgmi_write_kb: int = 0
    xgmi_link_speed_gbps: int = 0


def smi_devices() -> List[GpuDevice]:
    """GPUs reported by amd-smi (empty when amd-smi / a GPU is unavailable)."""
    L = lib()
    if L is None:
        return []
    n = L.tony_smi_init()
    out = []
    for i in range(max(n, 0)):
        info = _GpuInfo()
        if L.tony_smi_info(i, ctypes.byref(info)) == 0:
            out.append(GpuDevice(i, info.bdf.decode(), info.uuid.decode(), int(info.numa_node),
                                 int(info.vram_total_mb)))
    return out


def smi_sample(index: int) -> Optional[GpuSample]:
    L = lib()
    if L is None or L.tony_smi_init() <= index:
        return None
    s = _GpuSample()
    if L.tony_smi_sample(int(index), ctypes.byref(s)) != 0:
        return None
    return GpuSample(s.gfx_busy_pct, s.mem_busy_pct, s.vram_used_mb, s.vram_total_mb, s.power_w, s.temp_c,
                     int(s.ecc_correctable), int(s.ecc_uncorrectable), int(s.xgmi_read_kb), int(s.xgmi_write_kb),
                     int(s.xgmi_link_speed_gbps))


def smi_link(a: int, b: int):
    """(kind, hops) with kind in {"xgmi", "pcie", "unknown"}, or None."""
    L = lib()
    if L is None or L.tony_smi_init() <= max(a, b):
        return None
    hops = ctypes.c_int(0)
    rc = L.tony_smi_link(a, b, ctypes.byref(hops))
    if rc < 0:
        return None
    return {2: "xgmi", 1: "pcie"}.get(rc, "unknown"), hops.value

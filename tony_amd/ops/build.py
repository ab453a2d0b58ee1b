"""In-tree build of the tony_amd native libraries.

Two shared objects are produced next to their Python loaders:

* ``tony_amd/ops/_tony_kernels.so`` -- every ``csrc/*.hip`` translation unit,
  compiled by ``hipcc --offload-arch=gfx950`` and linked against the HIP
  runtime that PyTorch-ROCm already loaded (torch ships its own
  ``libamdhip64.so`` without a SONAME; linking to ``/opt/rocm``'s
  ``libamdhip64.so.7`` would put a second HIP runtime in the process and stream
  handles would not be shared).
* ``tony_amd/ops/_tony_fastcall*.so`` -- generated CPython METH_FASTCALL wrappers of the kernel
  entry points (ops/fastcall.py), ~20x cheaper per launch than ctypes.
* ``tony_amd/native/_tony_native.so`` -- host-only C++ runtime pieces (process
  launcher / gang spawner, port reservation, amd-smi GPU inventory + metrics).

The build is incremental (mtime based) and needs no GPU: hipcc cross-compiles
gfx950 code objects on the CPU container.  ``python -m tony_amd.ops.build``.
"""
from __future__ import annotations

import glob
import os
import shutil
import subprocess
import sys

ARCH = os.environ.get("TONY_OFFLOAD_ARCH", "gfx950")
HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.dirname(HERE)
ROOT = os.path.dirname(PKG)
BUILD_DIR = os.path.join(ROOT, "build", "native")
KERNELS_SO = os.path.join(HERE, "_tony_kernels.so")
NATIVE_SO = os.path.join(PKG, "native", "_tony_native.so")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")

HIPCC_FLAGS = [
    f"--offload-arch={ARCH}",
    "-O3",
    "-fPIC",
    "-std=c++17",
    "-fno-gpu-rdc",
    "-munsafe-fp-atomics",  # fp32 atomicAdd -> global_atomic_add_f32 (memory side)
    "-Wall",
    "-Wno-unused-function",
]


def _torch_lib_dir() -> str:
    import importlib.util

    spec = importlib.util.find_spec("torch")
    if spec is None or spec.origin is None:
        raise RuntimeError("torch is required to locate the HIP runtime it loads")
    return os.path.join(os.path.dirname(spec.origin), "lib")


def _newer(target: str, deps) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def _run(cmd, verbose):
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        sys.stderr.write(r.stdout + r.stderr)
        raise RuntimeError(f"build step failed ({r.returncode}): {' '.join(cmd[:3])} ...")
    return r


def build_kernels(verbose: bool = False, force: bool = False) -> str:
    hipcc = shutil.which("hipcc") or os.path.join(ROCM, "bin", "hipcc")
    srcs = sorted(glob.glob(os.path.join(HERE, "csrc", "*.hip")))
    headers = sorted(glob.glob(os.path.join(HERE, "csrc", "*.h")))
    os.makedirs(BUILD_DIR, exist_ok=True)
    objs = []
    # compile translation units in parallel (each hipcc is single threaded)
    procs = []
    for src in srcs:
        obj = os.path.join(BUILD_DIR, os.path.basename(src) + f".{ARCH}.o")
        objs.append(obj)
        if force or _newer(obj, [src] + headers):
            cmd = [hipcc, *HIPCC_FLAGS, "-c", src, "-o", obj]
            if verbose:
                print(" ".join(cmd), flush=True)
            procs.append((cmd, subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)))
    failed = []
    for cmd, p in procs:
        out, _ = p.communicate()
        if p.returncode != 0:
            failed.append((cmd, out))
    if failed:
        for cmd, out in failed:
            sys.stderr.write(out)
        raise RuntimeError(f"hipcc failed for {[c[-3] for c, _ in failed]}")
    if force or _newer(KERNELS_SO, objs):
        tlib = _torch_lib_dir()
        cmd = [
            "g++", "-shared", "-o", KERNELS_SO, *objs,
            f"-L{tlib}", "-l:libamdhip64.so", f"-Wl,-rpath,{tlib}", "-Wl,--no-undefined",
        ]
        _run(cmd, verbose)
    return KERNELS_SO


def build_fastcall(verbose: bool = False, force: bool = False) -> str:
    """Generate (ops/fastcall.py) and compile the CPython fast-call wrappers of the kernel entry points."""
    import sysconfig

    from . import fastcall
    from ._lib import _SIGNATURES

    out = os.path.join(HERE, "_tony_fastcall" + sysconfig.get_config_var("EXT_SUFFIX"))
    src = os.path.join(BUILD_DIR, "_tony_fastcall.c")
    os.makedirs(BUILD_DIR, exist_ok=True)
    code = fastcall.generate(_SIGNATURES)
    old = open(src).read() if os.path.exists(src) else None
    if old != code:
        with open(src, "w") as fh:
            fh.write(code)
    if force or old != code or _newer(out, [src]):
        cmd = ["gcc", "-O2", "-fPIC", "-shared", "-Wall", f"-I{sysconfig.get_paths()['include']}", src, "-o", out]
        _run(cmd, verbose)
    return out


def build_native(verbose: bool = False, force: bool = False) -> str:
    ndir = os.path.join(PKG, "native")
    srcs = sorted(glob.glob(os.path.join(ndir, "*.cpp")))
    headers = sorted(glob.glob(os.path.join(ndir, "*.h")))
    if not srcs:
        return ""
    if force or _newer(NATIVE_SO, srcs + headers):
        cmd = [
            "g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-Wall", "-o", NATIVE_SO, *srcs,
            f"-I{ROCM}/include", "-ldl", "-lpthread",
        ]
        _run(cmd, verbose)
    # stand-alone helper executables (no Python between fork and exec in the task agent)
    for src in sorted(glob.glob(os.path.join(ndir, "launcher", "*.cpp"))):
        exe = os.path.join(ndir, os.path.splitext(os.path.basename(src))[0])
        if force or _newer(exe, [src]):
            _run(["g++", "-O2", "-std=c++17", "-Wall", "-o", exe, src], verbose)
    return NATIVE_SO


def build_all(verbose: bool = False, force: bool = False):
    kernels = build_kernels(verbose, force)
    build_fastcall(verbose, force)
    return kernels, build_native(verbose, force)


if __name__ == "__main__":
    print(build_all(verbose="-v" in sys.argv, force="-f" in sys.argv))

#!/usr/bin/env python3
"""Per-kernel register / LDS / spill table of a built HIP object (the gfx950 code object's metadata notes).

    python tools/kernel_regs.py build/native/conv.hip.gfx950.o [NAME_SUBSTRING]
"""
import os
import re
import subprocess
import sys
import tempfile

B = "/opt/rocm/lib/llvm/bin"


def notes(obj: str) -> str:
    with tempfile.TemporaryDirectory() as d:
        fb, co = os.path.join(d, "fb"), os.path.join(d, "co")
        subprocess.run([f"{B}/llvm-objcopy", "-O", "binary", "--only-section=.hip_fatbin", obj, fb], check=True)
        subprocess.run([f"{B}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fb}",
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True)
        return subprocess.run([f"{B}/llvm-readelf", "--notes", co], capture_output=True, text=True).stdout


def main():
    obj, pat = sys.argv[1], (sys.argv[2] if len(sys.argv) > 2 else "")
    txt = notes(obj)
    for blk in re.split(r"\n\s+- \.agpr_count", txt)[1:]:
        name = re.search(r"\.name:\s+(\S+)", blk)
        if not name or pat not in name.group(1):
            continue
        get = lambda k: (re.search(rf"\.{k}:\s+(\S+)", blk) or [None, "?"])[1]  # noqa: E731
        dm = subprocess.run(["c++filt"], input=name.group(1), capture_output=True, text=True).stdout.strip()
        print(f"vgpr {get('vgpr_count'):>4} agpr {blk.split(None, 1)[0] if blk else '?':>4} sgpr {get('sgpr_count'):>4} "
              f"vspill {get('vgpr_spill_count'):>3} lds {get('group_segment_fixed_size'):>6}  {dm[:160]}")


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Instruction mix of the innermost loops around the MFMAs of a kernel in a gfx950 disassembly.

    /opt/rocm/lib/llvm/bin/llvm-objdump -d --no-show-raw-insn CODE_OBJECT > k.s
    python tools/isa_loops.py k.s 'conv_glds_kernel<256, 192, 4, 32, true, 4'

For each matching kernel: every backward branch whose body holds MFMAs, with its counts of MFMA, LDS reads,
LDS-DMA, waits, barriers, VALU / SALU and scratch (spill) instructions.
"""
import re
import subprocess
import sys


def functions(path):
    funcs, cur = {}, None
    for line in open(path):
        m = re.match(r"^([0-9a-f]+) <(.*)>:$", line.strip())
        if m:
            cur = m.group(2)
            funcs[cur] = []
            continue
        if cur is not None and line.startswith("\t"):
            funcs[cur].append(line.rstrip("\n"))
    return funcs


def main():
    path, pat = sys.argv[1], sys.argv[2]
    for name, body in functions(path).items():
        dm = subprocess.run(["c++filt"], input=name, capture_output=True, text=True).stdout.strip()
        if pat not in dm:
            continue
        off = {}
        for i, l in enumerate(body):
            m = re.search(r"<[^>]*\+0x([0-9a-f]+)>", l)
            a = re.search(r"//\s*([0-9A-Fa-f]+):", l)
            if a:
                off[int(a.group(1), 16)] = i
        base = min(off) if off else 0
        loops = []
        for i, l in enumerate(body):
            if "s_cbranch" not in l and "s_branch" not in l:
                continue
            m = re.search(r"<[^>]*\+0x([0-9a-f]+)>", l)
            if not m:
                continue
            t = off.get(base + int(m.group(1), 16))
            if t is not None and t < i:
                loops.append((t, i))
        print(dm[:150])
        for a, b in sorted(loops):
            seg = body[a:b + 1]
            c = lambda p: sum(1 for x in seg if re.search(p, x))  # noqa: E731
            nm = c(r"\sv_mfma")
            if not nm:
                continue
            pats = [("mfma", r"\sv_mfma"), ("ds_read", "ds_read"), ("ds_write", "ds_write"), ("lds-dma", "global_load_lds"),
                    ("waitcnt", "s_waitcnt"), ("barrier", "s_barrier"), ("valu", r"^\s+v_(?!mfma)"),
                    ("salu", r"^\s+s_(?!waitcnt|barrier|nop|cbranch|branch)"), ("nop", r"^\s+s_nop"),
                    ("scratch", "scratch_"), ("global", r"global_(load|store)_(?!lds)")]
            print(f"  loop [{a},{b}] {b - a + 1} insts: " + "  ".join(f"{k} {c(p)}" for k, p in pats))


if __name__ == "__main__":
    main()

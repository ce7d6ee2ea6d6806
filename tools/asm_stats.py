#!/usr/bin/env python3
"""Instruction mix of one kernel in a hipcc -S (gfx950) assembly file.

usage: asm_stats.py FILE.s SYMBOL_SUBSTRING [--dump]
Prints the kernel's VGPR/SGPR/occupancy metadata and counts instructions by class
(VALU, SALU, VMEM, SMEM, LDS, branches) overall and per basic block.
"""
import re
import sys


def kernel_body(path, sub):
    lines = open(path).read().split("\n")
    start = None
    for i, l in enumerate(lines):
        if start is None and l.startswith("_Z") and ":" in l and sub in l.split(":")[0]:
            start = i
        elif start is not None and l.startswith(".Lfunc_end"):
            return lines[start:i], lines[i:i + 60]
    raise SystemExit(f"{sub} not found")


def klass(op):
    if op.startswith(("global_load", "buffer_load", "flat_load")):
        return "vmem_load"
    if op.startswith(("global_store", "buffer_store", "flat_store")):
        return "vmem_store"
    if op.startswith("global_atomic"):
        return "vmem_atomic"
    if op.startswith("s_load") or op.startswith("s_buffer_load"):
        return "smem"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("s_cbranch", "s_branch")):
        return "branch"
    if op.startswith("s_waitcnt"):
        return "waitcnt"
    if op.startswith("s_"):
        return "salu"
    if op.startswith("v_"):
        return "valu"
    return "other"


def main():
    path, sub = sys.argv[1], sys.argv[2]
    body, meta = kernel_body(path, sub)
    print(body[0])
    blocks, cur = [], ["entry", {}]
    for l in body[1:]:
        s = l.strip()
        if re.match(r"^\.LBB\d+_\d+:", s):
            blocks.append(cur)
            cur = [s.split(":")[0], {}]
            continue
        if not s or s.startswith((";", ".", "//")):
            continue
        op = s.split()[0]
        k = klass(op)
        cur[1][k] = cur[1].get(k, 0) + 1
        cur[1]["_ops"] = cur[1].get("_ops", []) + [op]
    blocks.append(cur)
    for name, c in blocks:
        ops = c.pop("_ops", [])
        print(f"{name:14s} " + " ".join(f"{k}={v}" for k, v in sorted(c.items())))
        if "--dump" in sys.argv:
            vals = {}
            for o in ops:
                vals[o] = vals.get(o, 0) + 1
            print("    " + ", ".join(f"{k}:{v}" for k, v in sorted(vals.items(), key=lambda x: -x[1])))
    for l in body:
        if any(k in l for k in ("NumVgprs", "NumSgprs", "Occupancy", "ScratchSize")):
            print(l.strip())


if __name__ == "__main__":
    main()

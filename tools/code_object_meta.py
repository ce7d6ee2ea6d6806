#!/usr/bin/env python3
"""Kernel metadata (registers, LDS, occupancy inputs) of the gfx950 code objects inside a
HIP shared library.

usage: code_object_meta.py LIB.so [KERNEL_SUBSTRING]

The library's .hip_fatbin section holds one offload bundle per translation unit; each
gfx950 code object's AMDGPU metadata note lists every kernel with .vgpr_count,
.agpr_count, .sgpr_count and .group_segment_fixed_size.  Used by
tests/test_generated_chain_loop.py to check that k_sgd_chains_x keeps its
one-wave-per-SIMD allocation (DESIGN.md §9 "Chains on SIMDs of their own")."""
import json
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
TARGET = "hipv4-amdgcn-amd-amdhsa--gfx950"


def _code_objects(lib: str, d: str) -> list:
    """Paths of the gfx950 code objects unbundled from the library's .hip_fatbin into d."""
    cos = []
    fb = os.path.join(d, "fb.bin")
    subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fb}", lib,
                    os.path.join(d, "junk")], check=True, capture_output=True)
    data = open(fb, "rb").read()
    starts = [m.start() for m in re.finditer(re.escape(MAGIC), data)] + [len(data)]
    for i in range(len(starts) - 1):
        part = os.path.join(d, f"b{i}.bin")
        with open(part, "wb") as f:
            f.write(data[starts[i]:starts[i + 1]])
        co = os.path.join(d, f"b{i}.co")
        r = subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o",
                            f"--input={part}", f"--targets={TARGET}", f"--output={co}"],
                           capture_output=True)
        if r.returncode == 0 and os.path.getsize(co):
            cos.append(co)
    return cos


def disassembly(lib: str) -> dict:
    """{kernel symbol: its gfx950 disassembly} over every code object of the library
    (llvm-objdump -d; a function's text runs from its `<symbol>:` line to the next one)."""
    out = {}
    with tempfile.TemporaryDirectory() as d:
        for co in _code_objects(lib, d):
            text = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--no-show-raw-insn", co],
                                  check=True, capture_output=True, text=True).stdout
            name, buf = None, []
            for line in text.splitlines():
                m = re.match(r"^[0-9a-f]+ <([^>]+)>:$", line)
                if m:
                    if name:
                        out[name] = out.get(name, "") + "\n".join(buf)
                    name, buf = m.group(1), []
                elif name:
                    buf.append(line)
            if name:
                out[name] = out.get(name, "") + "\n".join(buf)
    return out


def kernels(lib: str) -> list:
    """[{name, vgpr_count, agpr_count, sgpr_count, lds}] over every gfx950 code object."""
    out = []
    with tempfile.TemporaryDirectory() as d:
        fb = os.path.join(d, "fb.bin")
        subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fb}", lib,
                        os.path.join(d, "junk")], check=True, capture_output=True)
        data = open(fb, "rb").read()
        starts = [m.start() for m in re.finditer(re.escape(MAGIC), data)] + [len(data)]
        for i in range(len(starts) - 1):
            part = os.path.join(d, f"b{i}.bin")
            with open(part, "wb") as f:
                f.write(data[starts[i]:starts[i + 1]])
            co = os.path.join(d, f"b{i}.co")
            r = subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o",
                                f"--input={part}", f"--targets={TARGET}", f"--output={co}"],
                               capture_output=True)
            if r.returncode != 0 or not os.path.getsize(co):
                continue
            notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], check=True,
                                   capture_output=True, text=True).stdout
            out += parse_notes(notes)
    return out


def parse_notes(text: str) -> list:
    """Kernel records from llvm-readelf's YAML dump of the amdhsa.kernels metadata."""
    ks, cur = [], None
    for line in text.splitlines():
        s = line.strip()
        m = re.match(r"^-?\s*\.(\w+):\s*(.*)$", s)
        if not m:
            continue
        key, val = m.group(1), m.group(2).strip()
        if key == "agpr_count" and s.startswith("- "):
            cur = {}
            ks.append(cur)
        if cur is None:
            continue
        if key in ("agpr_count", "vgpr_count", "sgpr_count", "group_segment_fixed_size",
                   "private_segment_fixed_size"):
            cur[key] = int(val)
        elif key in ("name", "symbol"):
            cur.setdefault(key, val.strip("'\""))
    return [k for k in ks if "name" in k]


def main():
    lib = sys.argv[1]
    sub = sys.argv[2] if len(sys.argv) > 2 else ""
    for k in kernels(lib):
        if sub in k["name"]:
            print(json.dumps(k))


if __name__ == "__main__":
    main()

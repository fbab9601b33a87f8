#!/usr/bin/env python
"""Per-kernel register / spill / scratch / LDS figures of the gfx950 code objects inside a built
library (the AMDGPU metadata note), optionally against a second library.

    python tools/kernel_resources.py [LIB] [--vs OTHER_LIB] [--grep REGEX]

Host-only: unbundles .hip_fatbin (tests/test_abi_cpu.py's ELF reader) and runs llvm-readobj
--notes on each code object.  Prints one line per kernel: VGPR, AGPR, SGPR, VGPR / SGPR spills,
scratch bytes, LDS bytes; with --vs, only the kernels whose figures differ.
"""
import argparse
import os
import re
import subprocess
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tests.test_abi_cpu import _gfx950_code_objects  # noqa: E402

READOBJ = "/opt/rocm/lib/llvm/bin/llvm-readobj"
KEYS = (".vgpr_count", ".agpr_count", ".sgpr_count", ".vgpr_spill_count", ".sgpr_spill_count",
        ".private_segment_fixed_size", ".group_segment_fixed_size")


def resources(lib):
    with open(lib, "rb") as f:
        so = f.read()
    out = {}
    for co in _gfx950_code_objects(so):
        with tempfile.NamedTemporaryFile(suffix=".co") as t:
            t.write(co)
            t.flush()
            notes = subprocess.run([READOBJ, "--notes", t.name], capture_output=True, text=True).stdout
        cur = None
        for line in notes.splitlines():
            m = re.match(r"\s*-?\s*\.name:\s+(\S+)", line)
            if m:
                cur = out.setdefault(m.group(1), {})
                continue
            m = re.match(r"\s*-?\s*(\.\w+):\s+(\d+)\s*$", line)
            if m and cur is not None and m.group(1) in KEYS:
                cur[m.group(1)] = int(m.group(2))
    return out


def fmt(name, r):
    v = [r.get(k, -1) for k in KEYS]
    return f"v{v[0]:4d} a{v[1]:4d} s{v[2]:4d} spill v{v[3]} s{v[4]} scratch {v[5]:5d} lds {v[6]:6d}  {name}"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("lib", nargs="?", default="fp8_quantization_amd/lib/libfp8approx.so")
    ap.add_argument("--vs")
    ap.add_argument("--grep", default="")
    a = ap.parse_args()
    r = resources(a.lib)
    rx = re.compile(a.grep)
    if not a.vs:
        for n in sorted(r):
            if rx.search(n):
                print(fmt(n, r[n]))
        return
    o = resources(a.vs)
    for n in sorted(set(r) | set(o)):
        if not rx.search(n) or r.get(n) == o.get(n):
            continue
        print("new", fmt(n, r.get(n, {})))
        print("old", fmt(n, o.get(n, {})))


if __name__ == "__main__":
    main()

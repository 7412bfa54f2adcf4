#!/usr/bin/env python3
"""Disassemble every gfx950 code object linked into a HIP shared library and count instructions
per kernel.  A hipcc-linked .so carries one clang offload bundle per compilation unit, back to
back in its .hip_fatbin section; each bundle holds a host entry and the gfx950 code object.

    python tools/isa_scan.py image_compression_amd/lib/libimgcomp.so 'v_pk_(add|mul|fma)_f32'

prints, per kernel with hits, the count (the packed-fp32 rule of DESIGN.md 9a is that there are
none).  tests/test_isa_scan.py runs the same scan on the in-tree library (CPU only)."""
import os
import re
import struct
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def _section(path, name):
    """(bytes) of ELF section `name` of `path` (64-bit little-endian ELF)."""
    with open(path, "rb") as f:
        data = f.read()
    assert data[:4] == b"\x7fELF" and data[4] == 2 and data[5] == 1, path
    shoff, = struct.unpack_from("<Q", data, 0x28)
    shentsize, shnum, shstrndx = struct.unpack_from("<HHH", data, 0x3A)
    sh = [struct.unpack_from("<IIQQQQIIQQ", data, shoff + i * shentsize) for i in range(shnum)]
    stro = sh[shstrndx][4]
    for s in sh:
        nm = data[stro + s[0]:data.index(b"\0", stro + s[0])].decode()
        if nm == name:
            return data[s[4]:s[4] + s[5]]
    raise KeyError(f"{path}: no section {name}")


def code_objects(path, target="gfx950"):
    """Every device code object for `target` in the library's .hip_fatbin, in link order."""
    fat = _section(path, ".hip_fatbin")
    out = []
    pos = fat.find(MAGIC)
    while pos >= 0:
        n, = struct.unpack_from("<Q", fat, pos + 24)
        q = pos + 32
        for _ in range(n):
            off, size, tl = struct.unpack_from("<QQQ", fat, q)
            triple = fat[q + 24:q + 24 + tl].decode()
            q += 24 + tl
            if triple.endswith(target):
                out.append(fat[pos + off:pos + off + size])
        pos = fat.find(MAGIC, pos + 32)
    return out


def disassemble(path, target="gfx950"):
    """{kernel symbol: [instruction lines]} over all code objects of the library."""
    kernels = {}
    with tempfile.TemporaryDirectory() as d:
        for i, co in enumerate(code_objects(path, target)):
            fn = os.path.join(d, f"co{i}.o")
            with open(fn, "wb") as f:
                f.write(co)
            txt = subprocess.run([os.path.join(LLVM, "llvm-objdump"), "-d", f"--mcpu={target}", fn],
                                 check=True, capture_output=True, text=True).stdout
            cur = None
            for line in txt.splitlines():
                m = re.match(r"^[0-9a-f]+ <(.+)>:$", line)
                if m:
                    cur = m.group(1)
                    kernels.setdefault(cur, [])
                elif cur is not None and line.startswith("\t"):
                    kernels[cur].append(line.strip())
    return kernels


def count(kernels, pattern):
    rx = re.compile(pattern)
    return {k: sum(1 for ln in v if rx.match(ln)) for k, v in kernels.items()}


def main():
    lib = sys.argv[1] if len(sys.argv) > 1 else "image_compression_amd/lib/libimgcomp.so"
    pat = sys.argv[2] if len(sys.argv) > 2 else r"v_pk_(add|mul|fma)_f32"
    ks = disassemble(lib)
    hits = {k: n for k, n in count(ks, pat).items() if n}
    print(f"{len(ks)} kernels, {sum(len(v) for v in ks.values())} instructions; '{pat}' in {len(hits)} kernels")
    for k, n in sorted(hits.items(), key=lambda t: -t[1]):
        print(f"{n:6d}  {k}")


if __name__ == "__main__":
    main()

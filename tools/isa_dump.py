#!/usr/bin/env python3
"""Disassemble the gfx950 code object embedded in a HIP shared library (no GPU needed).

The library's `.hip_fatbin` section holds a clang offload bundle; the gfx950 entry is an AMDGPU ELF
that `llvm-objdump -d` disassembles.  Used by tests/test_attention_isa.py (hazard distances of the
hand-written MFMAs) and for reading kernels' instruction streams.

    python tools/isa_dump.py [LIB] [--kernel SUBSTRING]      (prints the disassembly)
"""
from __future__ import annotations

import argparse
import re
import struct
import subprocess
import sys
import tempfile
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"
READELF = "/opt/rocm/lib/llvm/bin/llvm-readelf"
_MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def code_objects(lib: Path) -> list:
    """[(target triple, ELF bytes)] of every offload bundle in the library (one per source file)."""
    data = lib.read_bytes()
    out = []
    pos = data.find(_MAGIC)
    while pos >= 0:
        n = struct.unpack_from("<Q", data, pos + 24)[0]
        p = pos + 32
        for _ in range(n):
            off, size, tlen = struct.unpack_from("<QQQ", data, p)
            triple = data[p + 24:p + 24 + tlen].decode()
            p += 24 + tlen
            if size:
                out.append((triple, data[pos + off:pos + off + size]))
        pos = data.find(_MAGIC, pos + 1)
    return out


def disassemble(lib: Path, arch: str = "gfx950") -> str:
    objs = [b for t, b in code_objects(lib) if arch in t]
    if not objs:
        raise RuntimeError(f"no {arch} code object in {lib}")
    texts = []
    for b in objs:
        with tempfile.NamedTemporaryFile(suffix=".co") as f:
            f.write(b)
            f.flush()
            r = subprocess.run([OBJDUMP, "-d", f"--mcpu={arch}", f.name], capture_output=True, text=True, check=True)
            texts.append(r.stdout)
    return "\n".join(texts)


def kernel_resources(lib: Path, arch: str = "gfx950") -> dict:
    """{kernel name: {vgpr, agpr, sgpr, lds (static bytes), max_wg, spills}} from the AMDGPU metadata
    note of every code object (``llvm-readelf --notes``)."""
    import yaml
    out = {}
    for _, b in ((t, b) for t, b in code_objects(lib) if arch in t):
        with tempfile.NamedTemporaryFile(suffix=".co") as f:
            f.write(b)
            f.flush()
            r = subprocess.run([READELF, "--notes", f.name], capture_output=True, text=True, check=True)
        text = r.stdout
        i = text.find("---")
        j = text.find("\n...", i)
        meta = yaml.safe_load(text[i:j if j > 0 else None])
        for k in meta.get("amdhsa.kernels", []):
            out[k[".name"]] = {"vgpr": k.get(".vgpr_count", 0), "agpr": k.get(".agpr_count", 0),
                               "sgpr": k.get(".sgpr_count", 0), "lds": k.get(".group_segment_fixed_size", 0),
                               "max_wg": k.get(".max_flat_workgroup_size", 0),
                               "spills": k.get(".vgpr_spill_count", 0)}
    return out


def vgpr_alloc(res: dict) -> int:
    """VGPRs one wave of the kernel takes from its SIMD's 512 (arch VGPRs 4-aligned, then the
    AGPRs, in granules of 8)."""
    v, a = res["vgpr"], res["agpr"]
    t = ((v + 3) // 4 * 4 + a) if a else v
    return (t + 7) // 8 * 8


def kernel_bodies(disasm: str, name_substr: str) -> dict:
    """{symbol: instruction lines} of every function whose symbol contains name_substr."""
    out, cur = {}, None
    for ln in disasm.splitlines():
        m = re.match(r"^[0-9a-f]+ <(.+)>:$", ln)
        if m:
            cur = m.group(1) if name_substr in m.group(1) else None
            if cur is not None:
                out[cur] = []
            continue
        if cur is not None and ln.strip():
            out[cur].append(ln.split("//")[0].strip())
    return out


def kernel_body(disasm: str, name_substr: str) -> list:
    """Instruction lines of the first function whose symbol contains name_substr."""
    bodies = kernel_bodies(disasm, name_substr)
    return next(iter(bodies.values()), [])


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("lib", nargs="?", default=str(ROOT / "pytorch_operator_amd" / "_lib" / "libpto_hip.so"))
    ap.add_argument("--kernel", default=None)
    a = ap.parse_args(argv)
    d = disassemble(Path(a.lib))
    print("\n".join(kernel_body(d, a.kernel)) if a.kernel else d)
    return 0


if __name__ == "__main__":
    sys.exit(main())

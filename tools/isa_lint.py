#!/usr/bin/env python
"""Static hazard lint of the gfx950 code objects inside ``_kafka_hip*.so``.

Every HIP translation unit embeds a clang offload bundle; this tool unpacks
the gfx950 ELF of each, disassembles it with ``llvm-objdump`` and checks the
MFMA operand hazard that inline assembly once had to pad by hand
(csrc/kf_gp_mfma.h history): a VALU instruction that writes a VGPR read by a
following ``v_mfma*`` as SrcA or SrcB needs at least 2 wait states between
them (independent instructions or ``s_nop``).  Within a straight-line block
the scan is exact; across a label the predecessor is unknown and the scan
stops (the compiler pads block entries itself).

    python tools/isa_lint.py [--resources] [path/to/_kafka_hip.so]    # exit 1 on a violation
"""
from __future__ import annotations

import os
import re
import struct
import subprocess
import sys
import tempfile
from pathlib import Path

MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
OBJDUMP = Path(os.environ.get("ROCM_PATH", "/opt/rocm")) / "lib" / "llvm" / "bin" / "llvm-objdump"
REQUIRED_WAIT = 2

_REG = re.compile(r"\bv\[(\d+):(\d+)\]|\bv(\d+)\b")


def bundles(blob: bytes):
    """Yield (triple, code object bytes) of every offload bundle entry."""
    pos = blob.find(MAGIC)
    while pos >= 0:
        n = struct.unpack_from("<Q", blob, pos + len(MAGIC))[0]
        o = pos + len(MAGIC) + 8
        for _ in range(n):
            off, size, tlen = struct.unpack_from("<QQQ", blob, o)
            o += 24
            triple = blob[o:o + tlen].decode()
            o += tlen
            yield triple, blob[pos + off:pos + off + size]
        pos = blob.find(MAGIC, pos + 1)


def regs(op: str) -> set[int]:
    out = set()
    for m in _REG.finditer(op):
        if m.group(3) is not None:
            out.add(int(m.group(3)))
        else:
            out.update(range(int(m.group(1)), int(m.group(2)) + 1))
    return out


def parse(asm: str):
    """[(kind, mnemonic, operands)] per line of one disassembly; kind 'label' or 'inst'."""
    out = []
    for line in asm.splitlines():
        if re.match(r"^[0-9a-f]+ <.*>:$", line.strip()) or line.strip().endswith(">:"):
            out.append(("label", line.strip(), []))
            continue
        m = re.match(r"^\s+([a-z_0-9]+)(?:\s+([^/]*))?(?://.*)?$", line)
        if not m:
            continue
        mnem = m.group(1)
        ops = [o.strip() for o in (m.group(2) or "").split(",")] if m.group(2) else []
        out.append(("inst", mnem, ops))
    return out


def lint_listing(insts, name="") -> list[str]:
    bad = []
    for i, (kind, mnem, ops) in enumerate(insts):
        if kind != "inst" or not mnem.startswith("v_mfma") or len(ops) < 3:
            continue
        src = regs(ops[1]) | regs(ops[2])
        waits = 0
        for j in range(i - 1, -1, -1):
            k2, m2, o2 = insts[j]
            if k2 == "label" or m2.startswith("s_branch") or m2.startswith("s_cbranch"):
                break
            if waits >= REQUIRED_WAIT:
                break
            if m2.startswith("v_") and not m2.startswith("v_mfma") and o2:
                dst = o2[0].split()[0]
                if regs(dst) & src:
                    bad.append(f"{name}: {m2} {', '.join(o2)} -> {mnem} {', '.join(ops)} after {waits} wait states")
                    break
            if m2 == "s_nop":
                waits += int(o2[0], 0) + 1 if o2 else 1
            else:
                waits += 1
    return bad


READELF = OBJDUMP.with_name("llvm-readelf")


def kernel_resources(path: Path) -> dict[str, dict]:
    """{mangled kernel name: {vgpr, agpr, scratch, sgpr_spill}} from the
    code-object metadata notes of every gfx950 bundle in ``path``."""
    blob = path.read_bytes()
    out = {}
    with tempfile.TemporaryDirectory() as td:
        for i, (triple, code) in enumerate(bundles(blob)):
            if "gfx950" not in triple:
                continue
            f = Path(td) / f"co{i}.elf"
            f.write_bytes(code)
            notes = subprocess.run([str(READELF), "--notes", str(f)], capture_output=True, text=True,
                                   check=True).stdout
            cur = {}
            for line in notes.splitlines():
                m = re.match(r"\s+\.(name|vgpr_count|agpr_count|private_segment_fixed_size|sgpr_spill_count):\s+(\S+)",
                             line)
                if not m:
                    continue
                key, val = m.groups()
                if key == "name":
                    cur = out.setdefault(val, {})
                else:
                    cur[{"vgpr_count": "vgpr", "agpr_count": "agpr", "private_segment_fixed_size": "scratch",
                         "sgpr_spill_count": "sgpr_spill"}[key]] = int(val)
    return out


def waves_per_simd(vgpr: int, agpr: int = 0) -> int:
    """Waves per SIMD allowed by the unified VGPR+AGPR file (granule 8, 512 per lane)."""
    alloc = -(-(vgpr + agpr) // 8) * 8
    return min(8, 512 // max(alloc, 8))


def lint_so(path: Path) -> tuple[int, list[str]]:
    blob = path.read_bytes()
    n_mfma, bad = 0, []
    with tempfile.TemporaryDirectory() as td:
        for i, (triple, code) in enumerate(bundles(blob)):
            if "gfx950" not in triple:
                continue
            f = Path(td) / f"co{i}.elf"
            f.write_bytes(code)
            asm = subprocess.run([str(OBJDUMP), "-d", "--mcpu=gfx950", str(f)], capture_output=True, text=True,
                                 check=True).stdout
            insts = parse(asm)
            n_mfma += sum(1 for k, m, _ in insts if k == "inst" and m.startswith("v_mfma"))
            bad += lint_listing(insts, f"{path.name}#{i}")
    return n_mfma, bad


def main(argv):
    paths = [Path(a) for a in argv[1:] if not a.startswith("--")] or sorted((Path(__file__).resolve().parents[1] /
                                                   "kafka_inferenceengine_amd").glob("_kafka_hip*.so"))
    rc = 0
    for p in paths:
        if "--resources" in argv:
            for name, r in sorted(kernel_resources(p).items()):
                if "analysis" in name or "gain" in name:
                    print(f"{name[:80]:80s} vgpr={r.get('vgpr')} scratch={r.get('scratch')} "
                          f"waves/SIMD={waves_per_simd(r.get('vgpr', 0), r.get('agpr', 0))}")
        n, bad = lint_so(p)
        print(f"{p.name}: {n} MFMA instructions, {len(bad)} SrcA/SrcB wait-state violations")
        for b in bad[:20]:
            print("  " + b)
        rc |= bool(bad)
    return rc


if __name__ == "__main__":
    sys.exit(main(sys.argv))

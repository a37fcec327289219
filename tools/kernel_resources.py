#!/usr/bin/env python3
"""Register / LDS / spill summary of the gfx950 kernels in libpicocsum.so (build-time check).

    python tools/kernel_resources.py [name-substring]

Extracts the .hip_fatbin bundle, unbundles the gfx950 code object and reads its
AMDGPU metadata notes (llvm-readelf --notes)."""
from __future__ import annotations

import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LLVM = "/opt/rocm/lib/llvm/bin"


def kernels(so: str = os.path.join(ROOT, "picotcp_amd", "libpicocsum.so")):
    magic = b"__CLANG_OFFLOAD_BUNDLE__"
    notes = ""
    with tempfile.TemporaryDirectory() as d:
        fb = os.path.join(d, "fatbin")
        subprocess.run(["objcopy", "-O", "binary", "--only-section=.hip_fatbin", so, fb], check=True)
        blob = open(fb, "rb").read()
        starts = [i for i in range(len(blob)) if blob.startswith(magic, i)] if len(blob) < (1 << 20) else None
        if starts is None:                      # large section: find the bundles with bytes.find
            starts, i = [], blob.find(magic)
            while i >= 0:
                starts.append(i)
                i = blob.find(magic, i + 1)
        for k, a in enumerate(starts):          # one bundle per kernel TU
            b = starts[k + 1] if k + 1 < len(starts) else len(blob)
            part, co = os.path.join(d, f"b{k}"), os.path.join(d, f"k{k}.co")
            open(part, "wb").write(blob[a:b])
            subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={part}",
                            "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True)
            notes += subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], check=True, capture_output=True,
                                    text=True).stdout
    out = []
    for e in notes.split("- .agpr_count")[1:]:
        def g(k, e=e):
            m = re.search(rf"\.{k}:\s+(\S+)", e)
            return m.group(1) if m else "?"
        out.append(dict(name=g("name"), vgpr=g("vgpr_count"), vspill=g("vgpr_spill_count"),
                        sgpr=g("sgpr_count"), sspill=g("sgpr_spill_count"), lds=g("group_segment_fixed_size"),
                        scratch=g("private_segment_fixed_size")))
    return out


if __name__ == "__main__":
    sub = sys.argv[1] if len(sys.argv) > 1 else ""
    for k in kernels():
        if sub in k["name"]:
            print(f'{k["name"][:90]:90s} vgpr {k["vgpr"]:>4} vspill {k["vspill"]:>3} sgpr {k["sgpr"]:>3} '
                  f'sspill {k["sspill"]:>3} lds {k["lds"]:>6} scratch {k["scratch"]}')


def disasm(kernel_substr: str, so: str = os.path.join(ROOT, "picotcp_amd", "libpicocsum.so")) -> str:
    """llvm-objdump of the first kernel whose symbol contains kernel_substr."""
    magic = b"__CLANG_OFFLOAD_BUNDLE__"
    with tempfile.TemporaryDirectory() as d:
        fb = os.path.join(d, "fatbin")
        subprocess.run(["objcopy", "-O", "binary", "--only-section=.hip_fatbin", so, fb], check=True)
        blob = open(fb, "rb").read()
        starts, i = [], blob.find(magic)
        while i >= 0:
            starts.append(i)
            i = blob.find(magic, i + 1)
        for k, a in enumerate(starts):
            b = starts[k + 1] if k + 1 < len(starts) else len(blob)
            part, co = os.path.join(d, f"b{k}"), os.path.join(d, f"k{k}.co")
            open(part, "wb").write(blob[a:b])
            subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={part}",
                            "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True)
            txt = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--no-show-raw-insn", co], check=True,
                                 capture_output=True, text=True).stdout
            blocks = txt.split("\n\n")
            for blk in blocks:
                head = blk.strip().split("\n", 1)[0]
                if kernel_substr in head and head.endswith(">:"):
                    return blk
    return ""

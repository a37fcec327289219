"""Drop-in proof: the reference's own caller
code, compiled unmodified, binds to libpicocsum's pico_dualbuffer_checksum /
pico_checksum once pico_frame.o's two definitions are renamed away, and gives the
same results as the reference build on 20 000 frames.  CPU only; needs
/root/reference to compile the reference objects (skipped elsewhere)."""
from __future__ import annotations

import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = os.path.join(ROOT, "oracle", "_ref")


@pytest.fixture(scope="module")
def dropin_built():
    if not os.path.isdir("/root/reference/stack"):
        pytest.skip("reference sources absent (the GPU box): drop-in libraries are built where they exist")
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "dropin"], check=True)
    return REF


def test_reference_udp_caller_binds_to_libpicocsum(dropin_built):
    r = subprocess.run([os.path.join(dropin_built, "dropin_check"),
                        os.path.join(dropin_built, "libref_udp_dropin.so"),
                        os.path.join(dropin_built, "libref_udp_native.so")],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    words = r.stdout.split()
    bound = words[words.index("bound") + 1]
    assert os.path.realpath(bound) == os.path.realpath(os.path.join(ROOT, "picotcp_amd", "libpicocsum.so"))
    assert int(words[words.index("frames") + 1]) == 20001
    assert int(words[words.index("mismatches") + 1]) == 0


def test_weakened_symbol_recipe_does_not_interpose(dropin_built, tmp_path):
    """Why INTEGRATION.md renames instead of weakening: a weak definition left in an
    object of the executable still wins over libpicocsum.so's strong one."""
    weak = tmp_path / "pico_frame_weak.o"
    subprocess.run(["objcopy", "--weaken-symbol=pico_checksum", "--weaken-symbol=pico_dualbuffer_checksum",
                    os.path.join(dropin_built, "pico_frame.o"), str(weak)], check=True)
    src = tmp_path / "m.c"
    src.write_text('#define _GNU_SOURCE\n#include <dlfcn.h>\n#include <stdio.h>\n#include <stdint.h>\n'
                   'uint16_t pico_checksum(void *, uint32_t);\n'
                   'int main(void){Dl_info d; dladdr((void*)pico_checksum,&d); puts(d.dli_fname); return 0;}\n')
    exe = tmp_path / "m"
    lib = os.path.join(ROOT, "picotcp_amd")
    subprocess.run(["gcc", str(src), str(weak), f"-L{lib}", "-lpicocsum", f"-Wl,-rpath,{lib}", "-ldl", "-o", str(exe)],
                   check=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.strip()
    assert os.path.realpath(out) == os.path.realpath(str(exe))

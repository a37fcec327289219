"""CPU tests of the C-ABI boundary: libpicocsum.so loads, exports exactly what
include/pico_csum.h declares, validates arguments, and refuses (loudly) to run
the batched path without a HIP device.  No compute is launched here."""
from __future__ import annotations

import ctypes
import os
import re
import subprocess

import pytest
import torch

from picotcp_amd import _lib

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
HEADER = os.path.join(ROOT, "include", "pico_csum.h")


def declared_functions() -> set[str]:
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    names = set()
    for m in re.finditer(r"^[A-Za-z_][\w\s\*]*?\b(pico_\w+)\s*\(", src, flags=re.M):
        names.add(m.group(1))
    return names


def test_header_declares_the_exported_list():
    assert declared_functions() == set(_lib.EXPORTED)


def test_library_exports_every_declared_symbol():
    lib = _lib.load()
    for name in declared_functions():
        assert hasattr(lib, name), name
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True,
                         check=True).stdout
    defined = {line.split()[-1] for line in out.splitlines() if line.strip()}
    missing = declared_functions() - defined
    assert not missing, missing


def test_reference_symbol_signatures_are_drop_in():
    """pico_checksum / pico_dualbuffer_checksum have the reference's exact prototypes
    (include/pico_frame.h:106-107 of the reference)."""
    src = open(HEADER).read()
    assert "uint16_t pico_checksum(void *inbuf, uint32_t len);" in src
    assert "uint16_t pico_dualbuffer_checksum(void *inbuf1, uint32_t len1, void *inbuf2, uint32_t len2);" in src


def test_abi_version():
    assert _lib.load().pico_csum_abi_version() == _lib.ABI_VERSION == 4
    src = open(HEADER).read()
    assert re.search(r"#define PICO_CSUM_ABI_VERSION 4\b", src)
    for name, val in (("F_NXTHDR_DISPATCH", 8), ("V_FRAG", 16), ("V_EXPIRED", 16), ("V_MALFORMED", 8),
                      ("V_LOCAL_SRC", 32), ("V_DUPLICATE", 64)):
        m = re.search(rf"#define PICO_CSUM_{name}\s+(0x[0-9a-fA-F]+|[0-9]+)u", src)
        assert m and int(m.group(1), 0) == val, name
        assert getattr(_lib, name) == val


def test_header_compiles_as_c_and_cpp(tmp_path):
    c = tmp_path / "t.c"
    c.write_text('#include "pico_csum.h"\nint main(void){ struct pico_csum_desc d; (void)d; '
                 'return (int)sizeof(struct pico_csum_desc) - 16; }\n')
    exe = tmp_path / "t"
    subprocess.run(["gcc", "-std=c99", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"), str(c), "-o", str(exe)],
                   check=True)
    assert subprocess.run([str(exe)]).returncode == 0
    subprocess.run(["g++", "-fsyntax-only", "-x", "c++", "-I", os.path.join(ROOT, "include"), str(c)], check=True)


def test_argument_validation():
    lib = _lib.load()
    vp = ctypes.c_void_p
    # odd crc_off
    assert lib.pico_checksum_batch_dev(vp(0x1000), 1 << 20, vp(0x2000), 4, 3, 0, vp(0x3000), None, None) \
        == -_lib.EINVAL
    # misaligned descriptors
    assert lib.pico_checksum_batch_dev(vp(0x1000), 1 << 20, vp(0x2008), 4, -1, 0, vp(0x3000), None, None) \
        == -_lib.EINVAL
    # F_WRITE without a crc field
    assert lib.pico_checksum_batch_dev(vp(0x1000), 1 << 20, vp(0x2000), 4, -1, _lib.F_WRITE, vp(0x3000), None,
                                       None) == -_lib.EINVAL
    # F_WRITE on an RX ipv4 batch
    assert lib.pico_ipv4_checksum_batch_dev(vp(0x1000), 1 << 20, vp(0x2000), 4, _lib.F_WRITE, None, None, None,
                                            None) == -_lib.EINVAL
    assert lib.pico_ipv6_checksum_batch_dev(vp(0x1000), 1 << 20, vp(0x2000), 4, _lib.F_WRITE, None, None,
                                            None) == -_lib.EINVAL
    assert lib.pico_ipv6_checksum_batch_dev(vp(0x1000), 1 << 20, vp(0x2004), 4, 0, None, None, None) \
        == -_lib.EINVAL
    # F_NXTHDR_DISPATCH is an IPv6 / Ethernet RX option
    assert lib.pico_ipv6_checksum_batch_dev(vp(0x1000), 1 << 20, vp(0x2000), 4, _lib.F_TX | _lib.F_NXTHDR_DISPATCH,
                                            None, None, None) == -_lib.EINVAL
    assert lib.pico_eth_checksum_batch_dev(vp(0x1000), 1 << 20, vp(0x2000), 4, _lib.F_TX | _lib.F_NXTHDR_DISPATCH,
                                           None, None, None, None, None) == -_lib.EINVAL
    assert lib.pico_ipv4_checksum_batch_dev(vp(0x1000), 1 << 20, vp(0x2000), 4, _lib.F_NXTHDR_DISPATCH, None, None,
                                            None, None) == -_lib.EINVAL
    # ABI 1's dispatch bit 0x4 (the opposite meaning) is refused, never silently reinterpreted
    assert lib.pico_ipv6_checksum_batch_dev(vp(0x1000), 1 << 20, vp(0x2000), 4, 0x4, None, None, None) \
        == -_lib.EINVAL
    assert "retired" in lib.pico_csum_last_error().decode()
    assert lib.pico_eth_checksum_batch_dev(vp(0x1000), 1 << 20, vp(0x2000), 4, 0x4, None, None, None, None,
                                           None) == -_lib.EINVAL
    # forwarding: the verdict array is required, at most 32 host addresses, an aligned state
    loc = (ctypes.c_uint32 * 33)()
    assert lib.pico_ipv4_forward_batch_dev(vp(0x1000), 1 << 20, vp(0x2000), 4, None, 0, None, None, None) \
        == -_lib.EINVAL
    assert lib.pico_ipv4_forward_batch_dev(vp(0x1000), 1 << 20, vp(0x2000), 4, loc, 33, None, vp(0x3000), None) \
        == -_lib.EINVAL
    assert lib.pico_ipv4_forward_batch_dev(vp(0x1000), 1 << 20, vp(0x2000), 4, None, 1, None, vp(0x3000), None) \
        == -_lib.EINVAL
    assert lib.pico_ipv4_forward_batch_dev(vp(0x1000), 1 << 20, vp(0x2000), 4, loc, 2, vp(0x4002), vp(0x3000),
                                           None) == -_lib.EINVAL
    # reassembly: flags (IPv6: F_NXTHDR_DISPATCH only), alignment, NULL buffers
    ra = (vp(0x1000), 1 << 20, vp(0x2000), 4, vp(0x3000), 2, vp(0x4000), 1 << 20, vp(0x5000), None, None, None)
    assert lib.pico_ipv6_reassemble_batch_dev(*ra, _lib.F_TX, None) == -_lib.EINVAL
    assert lib.pico_ipv6_reassemble_batch_dev(*ra, 0x4, None) == -_lib.EINVAL
    assert lib.pico_ipv6_reassemble_batch_dev(*ra[:6], vp(0x4002), *ra[7:], 0, None) == -_lib.EINVAL
    assert lib.pico_ipv4_reassemble_batch_dev(*ra[:8], vp(0x5008), None, None, None, None) == -_lib.EINVAL
    assert lib.pico_ipv4_reassemble_batch_dev(None, *ra[1:], None) == -_lib.EINVAL
    # NULL buffers
    assert lib.pico_checksum_batch_uniform_dev(None, 6000, 1500, 1500, 4, 0, vp(0x3000), None) == -_lib.EINVAL
    # frames past base_len
    assert lib.pico_checksum_batch_uniform_dev(vp(0x1000), 5999, 1500, 1500, 4, 0, vp(0x3000), None) \
        == -_lib.EINVAL
    # n == 0 is a no-op
    assert lib.pico_checksum_batch_uniform_dev(None, 0, 1500, 1500, 0, 0, None, None) == 0
    msg = lib.pico_csum_last_error().decode()
    assert isinstance(msg, str)


def test_launch_override_validation():
    lib = _lib.load()
    # uniform rings: group 4..64
    assert lib.pico_csum_set_launch_override(12, 2, 1, 16, 0, 0) == -_lib.EINVAL
    assert lib.pico_csum_set_launch_override(16, 3, 1, 16, 0, 1) == -_lib.EINVAL   # 3 / 5-7: pipelined only
    assert lib.pico_csum_set_launch_override(4, 6, 1, 16, 0, 0) == -_lib.EINVAL    # ... and group >= 8
    assert lib.pico_csum_set_launch_override(16, 6, 2, 16, 0, 0) == -_lib.EINVAL   # cpl * unroll <= 8
    assert lib.pico_csum_set_launch_override(16, 9, 1, 16, 0, 0) == -_lib.EINVAL
    assert lib.pico_csum_set_launch_override(16, 6, 1, 16, 2, 2) == 0
    assert lib.pico_csum_set_launch_override(32, 3, 1, 16, 2, 0) == 0
    assert lib.pico_csum_set_launch_override(16, 2, 1, 6, 0, 0) == -_lib.EINVAL
    assert lib.pico_csum_set_launch_override(16, 4, 4, 16, 0, 0) == -_lib.EINVAL
    assert lib.pico_csum_set_launch_override(16, 2, 1, 16, 4, 0) == -_lib.EINVAL
    assert lib.pico_csum_set_launch_override(16, 2, 1, 16, 1, 4) == -_lib.EINVAL
    assert lib.pico_csum_set_launch_override(16, 2, 1, 16, 1, 3) == 0
    assert lib.pico_csum_set_launch_override(16, 2, 4, 16, 2, 2) == 0
    assert lib.pico_csum_set_launch_override(4, 16, 1, 16, 2, 0) == -_lib.EINVAL
    # descriptor batches: group 2, fpw only; the flat (1) and adaptive (3) kernels are gone
    assert lib.pico_csum_set_launch_override(2, 8, 0, 37, 2, 0) == 0
    assert lib.pico_csum_set_launch_override(2, 0, 0, 64, 0, 0) == 0
    assert lib.pico_csum_set_launch_override(2, 0, 0, 65, 0, 0) == -_lib.EINVAL
    assert lib.pico_csum_set_launch_override(2, 0, 0, 0, 0, 0) == -_lib.EINVAL
    assert lib.pico_csum_set_launch_override(1, 4, 1, 7, 1, 0) == -_lib.EINVAL
    assert lib.pico_csum_set_launch_override(3, 8, 0, 16, 1, 0) == -_lib.EINVAL
    assert lib.pico_csum_set_launch_override(0, 0, 0, 0, 0, 0) == 0


@pytest.mark.skipif(torch.cuda.is_available(), reason="checks the no-device error path")
def test_batch_path_fails_loudly_without_gpu():
    """No CPU fallback: without a HIP device the batched API returns -ENODEV."""
    lib = _lib.load()
    vp = ctypes.c_void_p
    rc = lib.pico_checksum_batch_uniform_dev(vp(0x1000), 6000, 1500, 1500, 4, 0, vp(0x3000), None)
    assert rc == -_lib.ENODEV
    assert "HIP device" in lib.pico_csum_last_error().decode()
    from picotcp_amd import batch
    with pytest.raises(ValueError):
        batch.checksum_uniform(torch.zeros(6000, dtype=torch.uint8), 1500, 1500, 4)
    # (ABI 4) the scratch release has nothing to free and says why
    assert lib.pico_csum_release_thread_scratch() == -_lib.ENODEV


def test_kernel_image_is_gfx950():
    """The shared library's fat binary carries gfx950 code objects and no other target."""
    blob = open(_lib.LIB_PATH, "rb").read()
    targets = set(re.findall(rb"amdgcn-amd-amdhsa--(gfx[0-9a-z]+)", blob))
    assert targets == {b"gfx950"}, targets

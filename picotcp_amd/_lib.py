"""ctypes binding of libpicocsum.so (include/pico_csum.h).

The shared library is the product: a C-ABI drop-in for picoTCP's checksum path
whose batched entry points run HIP kernels on gfx950.  This module only loads
it and declares argument types.  There is no Python or CPU fallback for the
batched path: if the library is missing, importing the batch helpers raises.
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libpicocsum.so")
# A/B measurement only (tools/ab_lib.sh): another build of the same library
if os.environ.get("PICO_CSUM_LIB"):
    LIB_PATH = os.path.abspath(os.environ["PICO_CSUM_LIB"])

# Public symbols declared by include/pico_csum.h (checked by tests/test_abi.py).
EXPORTED = (
    "pico_checksum",
    "pico_dualbuffer_checksum",
    "pico_checksum_partial",
    "pico_ipv4_pseudo_partial",
    "pico_ipv6_pseudo_partial",
    "pico_checksum_batch_dev",
    "pico_checksum_batch_uniform_dev",
    "pico_ipv4_checksum_batch_dev",
    "pico_ipv6_checksum_batch_dev",
    "pico_eth_checksum_batch_dev",
    "pico_ipv4_forward_batch_dev",
    "pico_ipv4_nat_batch_dev",
    "pico_ipv4_reassemble_batch_dev",
    "pico_ipv6_reassemble_batch_dev",
    "pico_csum_ctx_create",
    "pico_csum_ctx_destroy",
    "pico_checksum_batch_uniform_host",
    "pico_checksum_batch_host",
    "pico_ipv4_checksum_batch_host",
    "pico_ipv6_checksum_batch_host",
    "pico_eth_checksum_batch_host",
    "pico_csum_host_register",
    "pico_csum_host_unregister",
    "pico_csum_host_device_pointer",
    "pico_csum_abi_version",
    "pico_csum_last_error",
    "pico_csum_set_launch_override",
    "pico_csum_set_uniform_stream",
    "pico_csum_set_host_in_place",
    "pico_csum_set_reasm_flat",
    "pico_csum_release_thread_scratch",
)

F_WRITE = 0x1
F_TX = 0x2
F_NXTHDR_DISPATCH = 0x8   # IPv6 RX: TCP / UDP by next header, not the reference's byte 9 (include/pico_csum.h)
V_ACCEPT, V_NET_BAD, V_L4_BAD, V_MALFORMED, V_EXPIRED = 1, 2, 4, 8, 16
V_FRAG = 16                # RX / TX batches (V_EXPIRED: the forwarding batch)
ABI_VERSION = 4
V_DROP_L2, V_ARP, V_IPV6 = 32, 64, 128
V_UNTOUCHED = 32            # NAT batch (same bit as V_DROP_L2)
V_LOCAL_SRC, V_DUPLICATE = 32, 64   # forwarding batch (same bits as V_DROP_L2 / V_ARP)
EINVAL, ENODEV, EIO, ENOMEM = 22, 19, 5, 12


class PicoCsumError(RuntimeError):
    def __init__(self, fn: str, rc: int, msg: str):
        super().__init__(f"{fn} failed ({rc}): {msg}")
        self.rc = rc


_lib = None


def load() -> ctypes.CDLL:
    """Load libpicocsum.so once; raise loudly if it was not built."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"{LIB_PATH} not found: build it with `make -C picotcp_amd/csrc` "
            "(or __graft_entry__.build()); the batched checksum path has no fallback")
    lib = ctypes.CDLL(LIB_PATH)
    u8p = ctypes.c_void_p
    vp = ctypes.c_void_p
    u16, u32, u64, i32 = ctypes.c_uint16, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int32

    def sig(name, res, *args):
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = list(args)

    sig("pico_checksum", u16, vp, u32)
    sig("pico_dualbuffer_checksum", u16, vp, u32, vp, u32)
    sig("pico_checksum_partial", u32, u32, vp, u32)
    sig("pico_ipv4_pseudo_partial", u32, u32, u32, ctypes.c_uint8, ctypes.c_uint16)
    sig("pico_ipv6_pseudo_partial", u32, vp, vp, ctypes.c_uint8, u32)
    sig("pico_checksum_batch_dev", ctypes.c_int, vp, u64, vp, u32, i32, u32, vp, vp, vp)
    sig("pico_checksum_batch_uniform_dev", ctypes.c_int, vp, u64, u64, u32, u32, u32, vp, vp)
    sig("pico_ipv4_checksum_batch_dev", ctypes.c_int, vp, u64, vp, u32, u32, vp, vp, vp, vp)
    sig("pico_ipv6_checksum_batch_dev", ctypes.c_int, vp, u64, vp, u32, u32, vp, vp, vp)
    sig("pico_eth_checksum_batch_dev", ctypes.c_int, vp, u64, vp, u32, u32, vp, vp, vp, vp, vp)
    sig("pico_ipv4_forward_batch_dev", ctypes.c_int, vp, u64, vp, u32, vp, u32, vp, vp, vp)
    sig("pico_ipv4_nat_batch_dev", ctypes.c_int, vp, u64, vp, u32, vp, vp, vp, vp, vp)
    sig("pico_ipv4_reassemble_batch_dev", ctypes.c_int, vp, u64, vp, u32, vp, u32, vp, u64, vp, vp, vp, vp, vp)
    sig("pico_ipv6_reassemble_batch_dev", ctypes.c_int, vp, u64, vp, u32, vp, u32, vp, u64, vp, vp, vp, vp, u32, vp)
    sig("pico_csum_ctx_create", vp, ctypes.c_int, u64)
    sig("pico_csum_ctx_destroy", None, vp)
    sig("pico_checksum_batch_uniform_host", ctypes.c_int, vp, vp, u64, u32, u32, u32, vp)
    sig("pico_checksum_batch_host", ctypes.c_int, vp, vp, u64, vp, u32, i32, u32, vp)
    sig("pico_ipv4_checksum_batch_host", ctypes.c_int, vp, vp, u64, vp, u32, u32, vp, vp, vp)
    sig("pico_ipv6_checksum_batch_host", ctypes.c_int, vp, vp, u64, vp, u32, u32, vp, vp)
    sig("pico_eth_checksum_batch_host", ctypes.c_int, vp, vp, u64, vp, u32, u32, vp, vp, vp, vp)
    sig("pico_csum_host_register", ctypes.c_int, vp, u64)
    sig("pico_csum_host_unregister", ctypes.c_int, vp)
    sig("pico_csum_host_device_pointer", vp, vp)
    sig("pico_csum_abi_version", ctypes.c_int)
    sig("pico_csum_last_error", ctypes.c_char_p)
    sig("pico_csum_set_launch_override", ctypes.c_int, u32, u32, u32, u32, u32, u32)
    if hasattr(lib, "pico_csum_set_uniform_stream"):     # (an A/B build of an older round may lack it)
        sig("pico_csum_set_uniform_stream", ctypes.c_int, u32, u32)
    if hasattr(lib, "pico_csum_set_host_in_place"):
        sig("pico_csum_set_host_in_place", ctypes.c_int, u32)
    if hasattr(lib, "pico_csum_set_reasm_flat"):
        sig("pico_csum_set_reasm_flat", ctypes.c_int, u32)
    if hasattr(lib, "pico_csum_release_thread_scratch"):
        sig("pico_csum_release_thread_scratch", ctypes.c_int)
    del u8p
    if lib.pico_csum_abi_version() != ABI_VERSION:
        raise ImportError(f"{LIB_PATH} has ABI {lib.pico_csum_abi_version()}, this binding {ABI_VERSION}: rebuild it")
    _lib = lib
    return lib


def check(fn: str, rc: int) -> None:
    if rc != 0:
        msg = load().pico_csum_last_error().decode(errors="replace")
        raise PicoCsumError(fn, rc, msg)

"""TEST INFRASTRUCTURE ONLY: ctypes access to the CPU oracle.

  liboracle.so       -- C restatement (oracle/pico_csum_oracle.c), the checker.
  _ref/libpicoref.so -- the reference's own stack/pico_frame.c compiled from
                        /root/reference by oracle/Makefile (present here and,
                        prebuilt, on the GPU box).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
this module.  The product (picotcp_amd/) never does.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ORACLE_SO = os.path.join(HERE, "liboracle.so")
REF_SO = os.path.join(HERE, "_ref", "libpicoref.so")
REF_OS_SO = os.path.join(HERE, "_ref", "libpicoref_Os.so")

DESC_DTYPE = np.dtype([("off", "<u8"), ("len", "<u4"), ("seed", "<u4")])
ORACLE_IPV4_TX = 1
ORACLE_NXTHDR_DISPATCH = 4   # IPv6 RX: TCP / UDP by next header (default: the reference's byte-9 dispatch)

_vp = ctypes.c_void_p
_u16, _u32, _u64, _i32 = ctypes.c_uint16, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int32


def build() -> None:
    """Compile liboracle.so (and oracle/_ref when /root/reference is present)."""
    subprocess.run(["make", "-s", "-C", HERE, "all"], check=True)
    if os.path.isdir("/root/reference/stack"):
        subprocess.run(["make", "-s", "-C", HERE, "ref"], check=True)


_olib = None


def lib() -> ctypes.CDLL:
    global _olib
    if _olib is None:
        if not os.path.exists(ORACLE_SO):
            build()
        L = ctypes.CDLL(ORACLE_SO)
        L.oracle_checksum_adder.restype = _u32
        L.oracle_checksum_adder.argtypes = [_u32, _vp, _u32]
        L.oracle_checksum_finalize.restype = _u16
        L.oracle_checksum_finalize.argtypes = [_u32]
        L.oracle_checksum.restype = _u16
        L.oracle_checksum.argtypes = [_vp, _u32]
        L.oracle_dualbuffer_checksum.restype = _u16
        L.oracle_dualbuffer_checksum.argtypes = [_vp, _u32, _vp, _u32]
        L.oracle_ipv4_pseudo_sum.restype = _u32
        L.oracle_ipv4_pseudo_sum.argtypes = [_vp, _vp, ctypes.c_uint8, ctypes.c_uint16]
        L.oracle_batch_raw.restype = None
        L.oracle_batch_raw.argtypes = [_vp, _vp, _u32, _vp, _i32]
        L.oracle_batch_uniform.restype = None
        L.oracle_batch_uniform.argtypes = [_vp, _u64, _u32, _u32, _u32, _vp]
        L.oracle_batch_ipv4.restype = None
        L.oracle_batch_ipv4.argtypes = [_vp, _vp, _u32, _vp, _vp, _vp, _u32]
        L.oracle_ipv6_pseudo_sum.restype = _u32
        L.oracle_ipv6_pseudo_sum.argtypes = [_vp, _vp, ctypes.c_uint8, _u32]
        L.oracle_batch_ipv6.restype = None
        L.oracle_batch_ipv6.argtypes = [_vp, _vp, _u32, _vp, _vp, _u32]
        L.oracle_ipv6_walk.restype = ctypes.c_int
        L.oracle_ipv6_walk.argtypes = [_vp, _u32, _vp, _vp]
        L.oracle_batch_eth.restype = None
        L.oracle_batch_eth.argtypes = [_vp, _vp, _u32, _vp, _vp, _vp, _vp, _u32]
        L.oracle_ipv4_reassemble.restype = None
        L.oracle_ipv4_reassemble.argtypes = [_vp, _vp, _u32, _vp, _u32, _vp, _vp, _vp, _vp, _vp]
        L.oracle_ipv6_reassemble.restype = None
        L.oracle_ipv6_reassemble.argtypes = [_vp, _vp, _u32, _vp, _u32, _vp, _vp, _vp, _vp, _vp, _u32]
        L.oracle_ipv6_walk_frag.restype = ctypes.c_int
        L.oracle_ipv6_walk_frag.argtypes = [_vp, _u32, _vp, _vp, _vp]
        L.oracle_batch_ipv4_forward.restype = None
        L.oracle_batch_ipv4_forward.argtypes = [_vp, _vp, _u32, _vp, _u32, _vp, _vp]
        L.oracle_batch_ipv4_nat.restype = None
        L.oracle_batch_ipv4_nat.argtypes = [_vp, _vp, _u32, _vp, _vp, _vp, _vp]
        L.oracle_uniform_mt.restype = ctypes.c_double
        L.oracle_uniform_mt.argtypes = [_vp, _vp, _u64, _u32, _u32, _vp, _u32]
        _olib = L
    return _olib


def _p(a: np.ndarray) -> ctypes.c_void_p:
    return ctypes.c_void_p(a.ctypes.data)


def _buf(b) -> np.ndarray:
    return np.ascontiguousarray(np.frombuffer(bytes(b), dtype=np.uint8) if isinstance(b, (bytes, bytearray))
                                else b, dtype=np.uint8)


def checksum(b) -> int:
    a = _buf(b)
    return lib().oracle_checksum(_p(a), a.size)


def dualbuffer_checksum(b1, b2) -> int:
    a1, a2 = _buf(b1), _buf(b2)
    return lib().oracle_dualbuffer_checksum(_p(a1), a1.size, _p(a2), a2.size)


def adder(s: int, b) -> int:
    a = _buf(b)
    return lib().oracle_checksum_adder(s & 0xFFFFFFFF, _p(a), a.size)


def ipv4_pseudo_sum(src: bytes, dst: bytes, proto: int, tl: int) -> int:
    s, d = _buf(src), _buf(dst)
    return lib().oracle_ipv4_pseudo_sum(_p(s), _p(d), proto, tl)


def ipv6_pseudo_sum(src: bytes, dst: bytes, nxt: int, tl: int) -> int:
    s, d = _buf(src), _buf(dst)
    return lib().oracle_ipv6_pseudo_sum(_p(s), _p(d), nxt, tl)


def batch_raw(base: np.ndarray, desc: np.ndarray, crc_off: int = -1) -> np.ndarray:
    desc = np.ascontiguousarray(desc, dtype=DESC_DTYPE)
    out = np.zeros(desc.shape[0], dtype=np.uint16)
    lib().oracle_batch_raw(_p(base), _p(desc), desc.shape[0], _p(out), crc_off)
    return out


def batch_uniform(base: np.ndarray, stride: int, length: int, n: int, seed: int = 0) -> np.ndarray:
    out = np.zeros(n, dtype=np.uint16)
    lib().oracle_batch_uniform(_p(base), stride, length, n, seed & 0xFFFFFFFF, _p(out))
    return out


def batch_ipv4(base: np.ndarray, desc: np.ndarray, tx: bool = False):
    desc = np.ascontiguousarray(desc, dtype=DESC_DTYPE)
    n = desc.shape[0]
    on, ol, v = np.zeros(n, np.uint16), np.zeros(n, np.uint16), np.zeros(n, np.uint8)
    lib().oracle_batch_ipv4(_p(base), _p(desc), n, _p(on), _p(ol), _p(v), ORACLE_IPV4_TX if tx else 0)
    return on, ol, v


def batch_ipv6(base: np.ndarray, desc: np.ndarray, tx: bool = False, nxthdr_dispatch: bool = False):
    desc = np.ascontiguousarray(desc, dtype=DESC_DTYPE)
    n = desc.shape[0]
    ol, v = np.zeros(n, np.uint16), np.zeros(n, np.uint8)
    lib().oracle_batch_ipv6(_p(base), _p(desc), n, _p(ol), _p(v),
                            (ORACLE_IPV4_TX if tx else 0) | (ORACLE_NXTHDR_DISPATCH if nxthdr_dispatch else 0))
    return ol, v


WALK_DROP, WALK_PROTO, WALK_FRAG, WALK_BAD = 0, 1, 2, -1


def ipv6_walk(dgram) -> tuple:
    """oracle_ipv6_walk on one IPv6 datagram: (kind, net_len, proto)."""
    a = _buf(dgram)
    nl, pr = ctypes.c_uint32(0), ctypes.c_uint8(0)
    k = lib().oracle_ipv6_walk(_p(a), a.size, ctypes.byref(nl), ctypes.byref(pr))
    return k, nl.value, pr.value


def batch_eth(base: np.ndarray, desc: np.ndarray, mac: bytes | None = None, tx: bool = False,
              nxthdr_dispatch: bool = False):
    """Ethernet dispatch + fused IPv4 / IPv6 (oracle_batch_eth); mac None = no destination filter."""
    desc = np.ascontiguousarray(desc, dtype=DESC_DTYPE)
    n = desc.shape[0]
    on, ol, v = np.zeros(n, np.uint16), np.zeros(n, np.uint16), np.zeros(n, np.uint8)
    m = None if mac is None else _buf(mac)
    lib().oracle_batch_eth(_p(base), _p(desc), n, None if m is None else _p(m), _p(on), _p(ol), _p(v),
                           (ORACLE_IPV4_TX if tx else 0) | (ORACLE_NXTHDR_DISPATCH if nxthdr_dispatch else 0))
    return on, ol, v


def ipv4_reassemble(base: np.ndarray, desc: np.ndarray, groups: np.ndarray, out: np.ndarray, out_desc: np.ndarray):
    """oracle_ipv4_reassemble: writes into `out` (uint8, writable); returns (out_len, out_l4, verdict)."""
    desc = np.ascontiguousarray(desc, dtype=DESC_DTYPE)
    od = np.ascontiguousarray(out_desc, dtype=DESC_DTYPE)
    grp = np.ascontiguousarray(groups, dtype=np.uint32).reshape(-1)
    ng = grp.size // 2
    ol, l4, v = np.zeros(ng, np.uint32), np.zeros(ng, np.uint16), np.zeros(ng, np.uint8)
    lib().oracle_ipv4_reassemble(_p(base), _p(desc), desc.shape[0], _p(grp), ng, _p(out), _p(od), _p(ol), _p(l4),
                                 _p(v))
    return ol, l4, v


def ipv6_reassemble(base: np.ndarray, desc: np.ndarray, groups: np.ndarray, out: np.ndarray, out_desc: np.ndarray,
                    nxthdr_dispatch: bool = False):
    """oracle_ipv6_reassemble: writes into `out` (uint8, writable); returns (out_len, out_l4, verdict)."""
    desc = np.ascontiguousarray(desc, dtype=DESC_DTYPE)
    od = np.ascontiguousarray(out_desc, dtype=DESC_DTYPE)
    grp = np.ascontiguousarray(groups, dtype=np.uint32).reshape(-1)
    ng = grp.size // 2
    ol, l4, v = np.zeros(ng, np.uint32), np.zeros(ng, np.uint16), np.zeros(ng, np.uint8)
    lib().oracle_ipv6_reassemble(_p(base), _p(desc), desc.shape[0], _p(grp), ng, _p(out), _p(od), _p(ol), _p(l4),
                                 _p(v), ORACLE_NXTHDR_DISPATCH if nxthdr_dispatch else 0)
    return ol, l4, v


def ipv6_walk_frag(dgram) -> tuple:
    """oracle_ipv6_walk_frag: (kind, net_len, proto, frag field)."""
    a = _buf(dgram)
    nl, pr, om = ctypes.c_uint32(0), ctypes.c_uint8(0), ctypes.c_uint16(0)
    k = lib().oracle_ipv6_walk_frag(_p(a), a.size, ctypes.byref(nl), ctypes.byref(pr), ctypes.byref(om))
    return k, nl.value, pr.value, om.value


FWD_STATE_DTYPE = np.dtype([("src", "<u4"), ("dst", "<u4"), ("id", "<u2"), ("proto", "<u2"), ("reserved", "<u4")])


def fwd_state() -> np.ndarray:
    """A forwarding state at the reference's initial value (zeros)."""
    return np.zeros(1, FWD_STATE_DTYPE)


def batch_ipv4_forward(base: np.ndarray, desc: np.ndarray, local=(), state: np.ndarray | None = None) -> np.ndarray:
    """pico_ipv4_pre_forward_checks in batch order, in place on `base` (a writable uint8 array);
    `local` = the stack's link addresses as stored (uint32 little-endian views of the 4 bytes),
    `state` (fwd_state(), updated) carries the last forwarded tuple between calls; verdicts."""
    desc = np.ascontiguousarray(desc, dtype=DESC_DTYPE)
    loc = np.ascontiguousarray(np.asarray(local, dtype=np.uint32))
    st = fwd_state() if state is None else state
    assert st.dtype == FWD_STATE_DTYPE and st.flags.c_contiguous
    v = np.zeros(desc.shape[0], np.uint8)
    lib().oracle_batch_ipv4_forward(_p(base), _p(desc), desc.shape[0], _p(loc), loc.size, _p(st), _p(v))
    return v


NAT_DTYPE = np.dtype([("addr", "<u4"), ("port", "<u2"), ("dir", "u1"), ("reserved", "u1")])
NAT_NONE, NAT_OUTBOUND, NAT_INBOUND = 0, 1, 2


def batch_ipv4_nat(base: np.ndarray, desc: np.ndarray, nat: np.ndarray):
    """pico_ipv4_nat_outbound / _inbound's frame work (oracle_batch_ipv4_nat), in place on
    `base` (a writable uint8 array); returns (out_net, out_l4, verdict)."""
    desc = np.ascontiguousarray(desc, dtype=DESC_DTYPE)
    nat = np.ascontiguousarray(nat, dtype=NAT_DTYPE)
    n = desc.shape[0]
    assert nat.shape[0] == n
    on, ol, v = np.zeros(n, np.uint16), np.zeros(n, np.uint16), np.zeros(n, np.uint8)
    lib().oracle_batch_ipv4_nat(_p(base), _p(desc), n, _p(nat), _p(on), _p(ol), _p(v))
    return on, ol, v


# ---------------------------------------------------------------- reference

_rlibs: dict = {}


def ref_available(os_flags: bool = False) -> bool:
    return os.path.exists(REF_OS_SO if os_flags else REF_SO)


def ref_lib(os_flags: bool = False) -> ctypes.CDLL:
    path = REF_OS_SO if os_flags else REF_SO
    if path not in _rlibs:
        if not os.path.exists(path):
            raise FileNotFoundError(f"{path} missing: run `make -C oracle ref` where /root/reference exists")
        L = ctypes.CDLL(path)
        L.pico_checksum.restype = _u16
        L.pico_checksum.argtypes = [_vp, _u32]
        L.pico_dualbuffer_checksum.restype = _u16
        L.pico_dualbuffer_checksum.argtypes = [_vp, _u32, _vp, _u32]
        _rlibs[path] = L
    return _rlibs[path]


def ref_checksum(b) -> int:
    a = _buf(b)
    return ref_lib().pico_checksum(_p(a), a.size)


def ref_dualbuffer_checksum(b1, b2) -> int:
    a1, a2 = _buf(b1), _buf(b2)
    return ref_lib().pico_dualbuffer_checksum(_p(a1), a1.size, _p(a2), a2.size)


def uniform_mt(base: np.ndarray, stride: int, length: int, n: int, nthreads: int,
               kind: str = "reference", os_flags: bool = False):
    """Time `n` uniform frames through pico_checksum on `nthreads` pthreads.
    kind="reference": the compiled reference pico_frame.c; "port": the restatement.
    Returns (seconds, out)."""
    out = np.zeros(n, dtype=np.uint16)
    if kind == "reference":
        fn = ctypes.cast(ref_lib(os_flags).pico_checksum, ctypes.c_void_p)
    else:
        fn = ctypes.cast(lib().oracle_checksum, ctypes.c_void_p)
    secs = lib().oracle_uniform_mt(fn, _p(base), stride, length, n, _p(out), nthreads)
    return secs, out


REF_CALLERS_SO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_ref", "libref_callers.so")
RC_RX4, RC_RX6, RC_TX4, RC_ETH = 0, 1, 2, 3


def ref_callers_available() -> bool:
    return os.path.exists(REF_CALLERS_SO)


def ref_callers_batch(base: np.ndarray, desc: np.ndarray, mode: int, threads: int):
    """The reference's own per-datagram work (oracle/ref_callers_shim.c rc_batch_mt: pico_checksum
    of the IPv4 header + pico_tcp/udp_checksum_ipv4/_ipv6, the compiled reference modules) over a
    batch on `threads` pthreads.  TX (RC_TX4) writes the values into `base`.  Returns (seconds,
    out_net, out_l4)."""
    import time
    if "callers" not in _rlibs:
        L = ctypes.CDLL(REF_CALLERS_SO)
        L.rc_batch_mt.restype = ctypes.c_int
        L.rc_batch_mt.argtypes = [_vp, _vp, _u32, ctypes.c_int, ctypes.c_int, _vp, _vp]
        _rlibs["callers"] = L
    desc = np.ascontiguousarray(desc, dtype=DESC_DTYPE)
    n = desc.shape[0]
    on, ol = np.zeros(n, np.uint16), np.zeros(n, np.uint16)
    t0 = time.perf_counter()
    rc = _rlibs["callers"].rc_batch_mt(_p(base), _p(desc), n, mode, threads, _p(on), _p(ol))
    secs = time.perf_counter() - t0
    if rc != 0:
        raise RuntimeError(f"rc_batch_mt failed ({rc})")
    return secs, on, ol


REF_RX_O3_SO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_ref", "libref_rx_O3.so")


class _quiet:
    """fds 1 and 2 to /dev/null around calls into the reference stack, whose debug output (device
    and protocol registration, timer-heap warnings) must not reach a caller's stdout (bench.py
    prints one JSON line there); the C stdio buffers are flushed before the fds come back."""

    def __enter__(self):
        import sys
        sys.stdout.flush()
        sys.stderr.flush()
        self.saved = (os.dup(1), os.dup(2))
        self.null = os.open(os.devnull, os.O_WRONLY)
        os.dup2(self.null, 1)
        os.dup2(self.null, 2)
        return self

    def __exit__(self, *exc):
        ctypes.CDLL(None).fflush(None)
        os.dup2(self.saved[0], 1)
        os.dup2(self.saved[1], 2)
        for f in (*self.saved, self.null):
            os.close(f)
        return False


def ref_reasm_available() -> bool:
    return os.path.exists(REF_RX_O3_SO)


def ref_reasm_batch(v6: bool, base: np.ndarray, offs: np.ndarray, lens: np.ndarray, groups: np.ndarray):
    """The reference's own fragment path (oracle/ref_rx_driver.c rr_reasm_batch over the compiled
    reference stack at -O3: each fragment into a pico_frame, pico_ipv4_process_in /
    pico_ipv6_extension_headers, pico_ipv4/6_process_frag's tree and pico_fragments_reassemble,
    pico_transport_crc_check on the datagram handed on) over every group, on the calling thread.
    The datagrams' destination must be a local link (ref_reasm_link).  Returns (seconds,
    datagrams reassembled, transport checks passed)."""
    import time
    if "rx3" not in _rlibs:
        L = ctypes.CDLL(REF_RX_O3_SO)
        L.rr_init.restype = ctypes.c_int
        L.rr_ipv4_link.argtypes = [_u32]
        L.rr_ipv6_link.argtypes = [_vp]
        L.rr_reasm_batch.restype = ctypes.c_int
        L.rr_reasm_batch.argtypes = [ctypes.c_int, _vp, _vp, _vp, _vp, _u32, _vp]
        with _quiet():
            rc = L.rr_init()
        if rc != 0:
            raise RuntimeError("rr_init failed")
        _rlibs["rx3"] = L
    L = _rlibs["rx3"]
    offs = np.ascontiguousarray(offs, np.uint64)
    lens = np.ascontiguousarray(lens, np.uint32)
    groups = np.ascontiguousarray(groups, np.uint32)
    chk = np.zeros(1, np.uint32)
    with _quiet():
        t0 = time.perf_counter()
        done = L.rr_reasm_batch(int(v6), _p(base), _p(offs), _p(lens), _p(groups), groups.size // 2, _p(chk))
        secs = time.perf_counter() - t0
    return secs, int(done), int(chk[0])


def ref_reasm_link(v6: bool, addr: bytes) -> None:
    """Make `addr` (4 bytes as on the wire, or 16) a local link of the reference stack."""
    ref_reasm_batch(v6, np.zeros(1, np.uint8), np.zeros(0), np.zeros(0), np.zeros(0))   # (loads it)
    L = _rlibs["rx3"]
    with _quiet():
        if v6:
            a = np.frombuffer(addr, np.uint8).copy()
            L.rr_ipv6_link(_p(a))
        else:
            L.rr_ipv4_link(int.from_bytes(addr, "little"))


def fix_ipv4_header_crcs(buf: np.ndarray, offs: np.ndarray) -> None:
    """Store the header checksum (RFC 1071 over the 20-byte header, the field zeroed first) of the
    IPv4 header at each offset, in place: what a sender's pico_ipv4_frame_push leaves there."""
    offs = np.asarray(offs, np.int64)
    idx = offs[:, None] + np.arange(20)[None, :]
    h = buf[idx].astype(np.uint32)
    h[:, 10] = h[:, 11] = 0
    s = ((h[:, 0::2] << 8) | h[:, 1::2]).sum(axis=1)
    while (s >> 16).any():
        s = (s & 0xFFFF) + (s >> 16)
    c = (~s) & 0xFFFF
    buf[offs + 10] = (c >> 8).astype(np.uint8)
    buf[offs + 11] = (c & 0xFF).astype(np.uint8)

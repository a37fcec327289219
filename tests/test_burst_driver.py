"""The batched boundary through the compiled reference stack.

integration/pico_dev_burst.c is the driver a maintainer adds to picoTCP: one libpicocsum call
gives the verdicts of a whole Ethernet burst (pico_eth_checksum_batch_host), then every frame the
reference would accept goes on through pico_stack_recv into a stack built with CRC=0 (its
pico_ipv4_crc_check / pico_transport_crc_check compiled to the no-op variants,
modules/pico_ipv4.c:259-264, stack/pico_socket.c:1969-1975).  oracle/_ref/burst_main runs that
driver (tests/c_abi/burst_main.c) in front of the unmodified reference stack built with CRC=0
(oracle/_ref/libref_rx_crc0.so); the same burst goes through the same stack built with CRC=1
(libref_rx.so, a private copy) frame by frame.  The burst: every pinned frame of
tests/golden/ref_eth_cases.npz (IPv4 / IPv6 / ARP / other ethertypes, own / broadcast / multicast /
foreign destinations, valid and corrupted checksums, options, extension headers, fragments), with
the IPv4 and IPv6 destinations configured as the host's links so the datagrams are delivered
locally -- plus routed_frames(): datagrams to destinations that are NOT the host's (IPv4 inside a
link's /24, so routed out, and outside every route; IPv6 straight to TCP / UDP and behind a
hop-by-hop header, to the device's MAC and to a 33:33:00:00:00:01 multicast MAC -- the reference
forwards a hop-by-hop datagram only when the byte it reads as the routing type, which on RX is
the Ethernet frame's byte 2, is zero, pico_ipv6.c:845-853), each with a valid and a corrupted
transport checksum, so the driver's forwarded branch runs.  Asserted: for every frame, the protocol the CRC=0 stack
hands to the transport layer behind the driver equals what the CRC=1 stack hands on AND passes
its transport check, and the frames the CRC=0 stack routes on are the ones the CRC=1 stack
routes on -- with the GPU verdicts (-m gpu) and with the driver's host fallback (no device:
-ENODEV), which verifies with the scalar drop-in instead of dropping the burst.  A second stack
configuration adds a 0.0.0.0 link, which takes every non-local IPv4 datagram into UDP's queue
(pico_ipv4.c:353-361) where the transport is checked after all."""
from __future__ import annotations

import ctypes
import os
import shutil
import struct
import subprocess
import tempfile

import numpy as np
import pytest

from oracle import oracle as O
from tests import golden_data as G
from tests.golden import make_ref_rx as RX

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = os.path.join(ROOT, "oracle", "_ref")
BURST_MAIN = os.path.join(REF, "burst_main")
REF_RX = os.path.join(REF, "libref_rx.so")
need = pytest.mark.skipif(not (os.path.exists(BURST_MAIN) and os.path.exists(REF_RX)),
                          reason="oracle/_ref/burst_main or libref_rx.so not built (make -C oracle refrx burst)")


DST6_FOREIGN = bytes.fromhex("20010db8deadbeef0000000000000099")
MCAST6_MAC = bytes.fromhex("333300000001")


def _set16(b: bytearray, at: int, v: int) -> None:
    b[at], b[at + 1] = v >> 8, v & 0xFF


def _eth(mac: bytes, et: int, payload: bytes) -> bytes:
    return mac + bytes.fromhex("02aabbccddee") + et.to_bytes(2, "big") + payload


def _l4(proto: int, sport: int, n: int, rng) -> bytearray:
    t = bytearray(rng.integers(0, 256, n, dtype=np.uint8).tobytes())
    if proto == 6:
        t[12] = 0x50
    else:
        _set16(t, 4, n)
    _set16(t, 0, sport)
    return t


def _v4(mac, src, dst, proto, ident, n, rng, corrupt):
    t = _l4(proto, 1000 + ident, n, rng)
    h = bytearray(20)
    h[0], h[8], h[9] = 0x45, 64, proto
    _set16(h, 2, 20 + n)
    _set16(h, 4, ident)
    h[12:16], h[16:20] = src, dst
    fo = 16 if proto == 6 else 6
    t[fo] = t[fo + 1] = 0
    c = O.dualbuffer_checksum(np.frombuffer(bytes(src) + bytes(dst) + bytes([0, proto]) + (n).to_bytes(2, "big"),
                                            np.uint8), np.frombuffer(bytes(t), np.uint8))
    _set16(t, fo, c ^ (0x0101 if corrupt else 0))
    _set16(h, 10, O.checksum(np.frombuffer(bytes(h), np.uint8)))
    return _eth(mac, 0x0800, bytes(h) + bytes(t))


def _v6(mac, src, dst, proto, n, rng, corrupt, hbh=None):
    """hbh: None (transport first) or the hop-by-hop header's 6 option bytes (8-byte header)."""
    t = _l4(proto, 2000 + n, n, rng)
    ext = b"" if hbh is None else bytes([proto, 0]) + hbh
    h = bytearray(40)
    h[0], h[6], h[7] = 0x60, 0 if hbh is not None else proto, 64
    _set16(h, 4, len(ext) + n)
    h[8:24], h[24:40] = src, dst
    fo = 16 if proto == 6 else 6
    t[fo] = t[fo + 1] = 0
    ps = bytes(src) + bytes(dst) + n.to_bytes(4, "big") + bytes([0, 0, 0, proto])
    c = O.dualbuffer_checksum(np.frombuffer(ps, np.uint8), np.frombuffer(bytes(t), np.uint8))
    _set16(t, fo, c ^ (0x0101 if corrupt else 0))
    return _eth(mac, 0x86DD, bytes(h) + ext + bytes(t))


def routed_frames(mac: bytes) -> list:
    """Datagrams to destinations that are not the host's (see the module docstring)."""
    rng = np.random.default_rng(17)
    out, ident = [], 1
    src4 = bytes([172, 16, 3, 9])
    for dst in (bytes([192, 168, 7, 77]), bytes([10, 9, 8, 7])):   # inside a link's /24; no route
        for proto in (6, 17):
            for corrupt in (False, True):
                for n in (20 if proto == 6 else 8, 333):
                    out.append(_v4(mac, src4, dst, proto, ident, n, rng, corrupt))
                    ident += 1
    for m in (mac, MCAST6_MAC):
        for proto in (6, 17):
            src6 = bytes([0x20, proto, 0x0d, 0xb8]) + bytes(11) + b"\x05"      # byte 9 = the transport
            for hbh in (None, bytes(6), bytes([1, 4, 0, 0, 0, 0]), bytes([5, 2, 0, 0, 1, 0])):   # Pad1 / PadN / RA
                for corrupt in (False, True):
                    out.append(_v6(m, src6, DST6_FOREIGN, proto, 96 + 8 * len(out), rng, corrupt, hbh))
    return out


def burst():
    c = G.ref_eth_cases()
    pin = np.flatnonzero(c["pinned"])
    off, av, buf = c["off"][pin].astype(np.int64), c["avail"][pin], c["buf"]
    mac = c["mac"].tobytes()
    extra = routed_frames(mac)
    ring = np.concatenate([buf[o:o + a] for o, a in zip(off, av)] + [np.frombuffer(f, np.uint8) for f in extra])
    av = np.concatenate([av, np.array([len(f) for f in extra], av.dtype)])
    noff = np.concatenate([[0], np.cumsum(av.astype(np.int64))[:-1]]).astype(np.uint64)
    d6 = set()
    for o, a, l2 in zip(off, av, c["l2"][pin]):
        if l2 == 2 and a >= 54:
            d6.add(bytes(buf[o + 38:o + 54]))
    assert all(d[:8] != DST6_FOREIGN[:8] for d in d6)
    links4 = [int.from_bytes(d, "little") for d in RX.DSTS4]
    desc = np.zeros(noff.size, batch_desc_dtype())
    desc["off"], desc["len"] = noff, av
    _, _, want_v = O.batch_eth(ring, desc, mac=mac)
    want_v[:pin.size] = c["verdict"][pin]               # the reference's own verdicts where pinned
    return mac, ring, noff, av, links4, sorted(d6), want_v


def batch_desc_dtype():
    return np.dtype([("off", "<u8"), ("len", "<u4"), ("seed", "<u4")])


def write_burst(path, mac, ring, off, av, links4, links6):
    desc = np.zeros(off.size, np.dtype([("off", "<u8"), ("len", "<u4"), ("seed", "<u4")]))
    desc["off"], desc["len"] = off, av
    with open(path, "wb") as f:
        f.write(struct.pack("<III6sHQ", off.size, len(links4), len(links6), mac, 0, ring.size))
        f.write(np.array(links4, np.uint32).tobytes())
        f.write(b"".join(links6))
        f.write(desc.tobytes())
        f.write(ring.tobytes())


def run_driver(tmp_path, args, any_link=False):
    mac, ring, off, av, l4, l6, _ = burst()
    bp, op = tmp_path / "burst.bin", tmp_path / "out.bin"
    write_burst(bp, mac, ring, off, av, l4 + ([0] if any_link else []), l6)
    r = subprocess.run([BURST_MAIN, str(bp), str(op)] + args, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    raw = op.read_bytes()
    n = off.size
    used = struct.unpack("<i", raw[:4])[0]
    verdict = np.frombuffer(raw[4:4 + n], np.uint8)
    deliv = np.frombuffer(raw[4 + n:4 + 5 * n], np.int32)
    routed = np.frombuffer(raw[4 + 9 * n:4 + 13 * n], np.int32)
    return used, verdict, deliv, routed


def reference_crc1(any_link=False):
    """Every frame through the CRC=1 stack (a private copy of libref_rx.so: its own state):
    (delivered protocol whose transport check passed or -1, routed on 0/1) per frame."""
    mac, ring, off, av, l4, l6, _ = burst()
    l4 = l4 + ([0] if any_link else [])
    tmp = tempfile.NamedTemporaryFile(suffix=".so", delete=False)
    tmp.close()
    shutil.copyfile(REF_RX, tmp.name)
    R = ctypes.CDLL(tmp.name)
    os.unlink(tmp.name)
    R.rr_eth_init.argtypes = [ctypes.c_char_p]
    R.rr_ipv4_link.argtypes = [ctypes.c_uint32]
    R.rr_ipv6_link.argtypes = [ctypes.c_char_p]
    R.rr_stack_rx.argtypes = [ctypes.c_void_p, ctypes.c_uint32]
    R.rr_take_delivered.argtypes = [ctypes.POINTER(ctypes.c_int)]
    R.rr_take_forwarded.restype = ctypes.c_int
    assert R.rr_init() == 0 and R.rr_eth_init(mac) == 0
    for a in l4:
        R.rr_ipv4_link(a)
    for a in l6:
        R.rr_ipv6_link(a)
    out = np.full(off.size, -1, np.int32)
    routed = np.zeros(off.size, np.int32)
    chk = ctypes.c_int(0)
    for i, (o, a) in enumerate(zip(off.astype(np.int64), av)):
        fr = np.ascontiguousarray(ring[o:o + a])
        R.rr_stack_rx(fr.ctypes.data, int(a))
        p = R.rr_take_delivered(ctypes.byref(chk))
        if p >= 0 and (p not in (6, 17) or chk.value == 1):
            out[i] = p                                  # delivered and its transport check passed
        routed[i] = R.rr_take_forwarded()
    return out, routed


_ref_cache = {}


def ref_delivered(any_link=False):
    if any_link not in _ref_cache:
        _ref_cache[any_link] = reference_crc1(any_link)
    return _ref_cache[any_link]


def check_same(deliv, routed, any_link):
    want, want_r = ref_delivered(any_link)
    n_extra = len(routed_frames(b"\0" * 6))
    assert (want >= 0).sum() > 800                       # TCP / UDP / ICMP delivered locally (835)
    if not any_link:                                     # the routed frames are routed, both ways
        assert want_r[-n_extra:].sum() >= 32 and want_r[:-n_extra].sum() == 0
    else:                                                # the 0.0.0.0 link keeps IPv4 here
        assert (want[-n_extra:][:16] == 17).sum() == 8   # the valid half, via UDP's queue
    bad = np.flatnonzero((deliv != want) | (routed != want_r))
    assert bad.size == 0, (f"{bad.size} frames differ, e.g. {bad[:10]}: delivered {deliv[bad[:10]]} vs "
                           f"{want[bad[:10]]}, routed {routed[bad[:10]]} vs {want_r[bad[:10]]}")


@need
@pytest.mark.parametrize("any_link", [False, True])
def test_host_fallback_matches_crc1_stack(tmp_path, any_link):
    """No device here (or --no-gpu): the driver's scalar host verify, then the CRC=0 stack."""
    used, _, deliv, routed = run_driver(tmp_path, ["--no-gpu"], any_link)
    assert used == 0
    check_same(deliv, routed, any_link)


@need
@pytest.mark.gpu
@pytest.mark.parametrize("any_link", [False, True])
def test_gpu_verdicts_match_crc1_stack(tmp_path, any_link):
    """The GPU verdicts (pico_eth_checksum_batch_host), then the CRC=0 stack."""
    used, verdict, deliv, routed = run_driver(tmp_path, [], any_link)
    assert used == 1
    *_, want_v = burst()
    np.testing.assert_array_equal(verdict, want_v)       # the reference's pinned verdicts + the oracle's
    check_same(deliv, routed, any_link)

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
locally.  Asserted: for every frame, the protocol the CRC=0 stack hands to the transport layer
behind the driver equals what the CRC=1 stack hands on AND passes its transport check -- with the
GPU verdicts (-m gpu) and with the driver's host fallback (no device: -ENODEV), which verifies with
the scalar drop-in instead of dropping the burst."""
from __future__ import annotations

import ctypes
import os
import shutil
import struct
import subprocess
import tempfile

import numpy as np
import pytest

from tests import golden_data as G
from tests.golden import make_ref_rx as RX

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = os.path.join(ROOT, "oracle", "_ref")
BURST_MAIN = os.path.join(REF, "burst_main")
REF_RX = os.path.join(REF, "libref_rx.so")
need = pytest.mark.skipif(not (os.path.exists(BURST_MAIN) and os.path.exists(REF_RX)),
                          reason="oracle/_ref/burst_main or libref_rx.so not built (make -C oracle refrx burst)")


def burst():
    c = G.ref_eth_cases()
    pin = np.flatnonzero(c["pinned"])
    off, av, buf = c["off"][pin].astype(np.int64), c["avail"][pin], c["buf"]
    ring = np.concatenate([buf[o:o + a] for o, a in zip(off, av)])
    noff = np.concatenate([[0], np.cumsum(av.astype(np.int64))[:-1]]).astype(np.uint64)
    d6 = set()
    for o, a, l2 in zip(off, av, c["l2"][pin]):
        if l2 == 2 and a >= 54:
            d6.add(bytes(buf[o + 38:o + 54]))
    links4 = [int.from_bytes(d, "little") for d in RX.DSTS4]
    return c["mac"].tobytes(), ring, noff, av, links4, sorted(d6), c["verdict"][pin]


def write_burst(path, mac, ring, off, av, links4, links6):
    desc = np.zeros(off.size, np.dtype([("off", "<u8"), ("len", "<u4"), ("seed", "<u4")]))
    desc["off"], desc["len"] = off, av
    with open(path, "wb") as f:
        f.write(struct.pack("<III6sHQ", off.size, len(links4), len(links6), mac, 0, ring.size))
        f.write(np.array(links4, np.uint32).tobytes())
        f.write(b"".join(links6))
        f.write(desc.tobytes())
        f.write(ring.tobytes())


def run_driver(tmp_path, args):
    mac, ring, off, av, l4, l6, _ = burst()
    bp, op = tmp_path / "burst.bin", tmp_path / "out.bin"
    write_burst(bp, mac, ring, off, av, l4, l6)
    r = subprocess.run([BURST_MAIN, str(bp), str(op)] + args, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    raw = op.read_bytes()
    n = off.size
    used = struct.unpack("<i", raw[:4])[0]
    verdict = np.frombuffer(raw[4:4 + n], np.uint8)
    deliv = np.frombuffer(raw[4 + n:4 + 5 * n], np.int32)
    return used, verdict, deliv


def reference_crc1():
    """Every frame through the CRC=1 stack (a private copy of libref_rx.so: its own state)."""
    mac, ring, off, av, l4, l6, _ = burst()
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
    assert R.rr_init() == 0 and R.rr_eth_init(mac) == 0
    for a in l4:
        R.rr_ipv4_link(a)
    for a in l6:
        R.rr_ipv6_link(a)
    out = np.full(off.size, -1, np.int32)
    chk = ctypes.c_int(0)
    for i, (o, a) in enumerate(zip(off.astype(np.int64), av)):
        fr = np.ascontiguousarray(ring[o:o + a])
        R.rr_stack_rx(fr.ctypes.data, int(a))
        p = R.rr_take_delivered(ctypes.byref(chk))
        if p >= 0 and (p not in (6, 17) or chk.value == 1):
            out[i] = p                                  # delivered and its transport check passed
    return out


_ref_cache = {}


def ref_delivered():
    if "d" not in _ref_cache:
        _ref_cache["d"] = reference_crc1()
    return _ref_cache["d"]


@need
def test_host_fallback_matches_crc1_stack(tmp_path):
    """No device here (or --no-gpu): the driver's scalar host verify, then the CRC=0 stack."""
    used, _, deliv = run_driver(tmp_path, ["--no-gpu"])
    assert used == 0
    want = ref_delivered()
    assert (want >= 0).sum() > 800                       # TCP / UDP / ICMP delivered locally (835)
    bad = np.flatnonzero(deliv != want)
    assert bad.size == 0, f"{bad.size} frames differ, e.g. {bad[:10]}: {deliv[bad[:10]]} vs {want[bad[:10]]}"


@need
@pytest.mark.gpu
def test_gpu_verdicts_match_crc1_stack(tmp_path):
    """The GPU verdicts (pico_eth_checksum_batch_host), then the CRC=0 stack."""
    used, verdict, deliv = run_driver(tmp_path, [])
    assert used == 1
    *_, want_v = burst()
    np.testing.assert_array_equal(verdict, want_v)       # the reference's pinned verdicts
    want = ref_delivered()
    bad = np.flatnonzero(deliv != want)
    assert bad.size == 0, f"{bad.size} frames differ, e.g. {bad[:10]}: {deliv[bad[:10]]} vs {want[bad[:10]]}"

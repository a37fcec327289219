#!/usr/bin/env python3
"""Golden TX frames: the datagrams the compiled reference stack (CRC=1) itself emits.

Run here (where /root/reference exists):
    make -C oracle refrx && python tests/golden/make_ref_tx.py

oracle/_ref/libref_rx.so is the reference stack compiled unmodified (oracle/Makefile `refrx`).  Its
driver (oracle/ref_rx_driver.c) records every IPv4 datagram the stack hands to pico_datalink_send
(rr_tx_capture) while frames reach the real transport layer (rr_real_transport) and the public
socket API runs (rr_socket / rr_sendto / rr_accept / rr_write / rr_tick).  The traffic:
  * TCP from tcp_send (modules/pico_tcp.c:968-985, crc = short_be(pico_tcp_checksum)): the SYN-ACK
    of every connection a listening socket accepts (SYNs with and without MSS / window-scale /
    SACK-permitted / timestamp options), the data segments of the accepted connection after
    pico_socket_write (payloads of 1 .. several MSS, odd lengths), and the RST a SYN to a closed
    port gets;
  * UDP from pico_udp_push (crc = 0, modules/pico_udp.c:120), payloads 0 .. 1472 bytes;
  * ICMPv4 echo replies (pico_icmp4_checksum, modules/pico_icmp4.c:30-41), payloads of any length;
each behind pico_ipv4_frame_push's header checksum (pico_ipv4_checksum, modules/pico_ipv4.c:231-240,
:1079).  The incoming frames (SYN, ACK, echo request) are built here with valid checksums.

Output (data only): ref_tx_cases.npz
  buf uint8[] (the captured datagrams back to back), off uint64[n], len uint32[n], proto uint8[n]
"""
from __future__ import annotations

import ctypes
import os
import shutil
import struct
import sys
import tempfile

import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, ROOT)

from oracle import oracle as O  # noqa: E402

OUT = os.path.dirname(os.path.abspath(__file__))
REF_RX = os.path.join(ROOT, "oracle", "_ref", "libref_rx.so")
MAC = bytes.fromhex("02005e0a0b0c")
HOST = bytes([192, 168, 7, 1])


def ref_lib():
    """A private copy of libref_rx.so (its own stack state)."""
    tmp = tempfile.NamedTemporaryFile(suffix=".so", delete=False)
    tmp.close()
    shutil.copyfile(REF_RX, tmp.name)
    R = ctypes.CDLL(tmp.name)
    os.unlink(tmp.name)
    vp, u32, u16 = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint16
    R.rr_eth_init.argtypes = [ctypes.c_char_p]
    R.rr_ipv4_link.argtypes = [u32]
    R.rr_stack_rx.argtypes = [vp, u32]
    R.rr_tx_capture.argtypes = [vp, u32, vp, u32]
    R.rr_real_transport.argtypes = [ctypes.c_int]
    R.rr_socket.restype = vp
    R.rr_socket.argtypes = [ctypes.c_int, u32, u16, ctypes.c_int]
    R.rr_sendto.argtypes = [vp, vp, ctypes.c_int, u32, u16]
    R.rr_accept.restype = vp
    R.rr_accept.argtypes = [vp]
    R.rr_write.argtypes = [vp, vp, ctypes.c_int]
    R.rr_tick.argtypes = [ctypes.c_int]
    return R


def a32(b: bytes) -> int:
    return int.from_bytes(b, "little")          # struct pico_ip4 as stored


def be16(v: int) -> int:
    return ((v & 0xFF) << 8) | (v >> 8)         # a port in network order, as a native uint16


def ipv4(src: bytes, dst: bytes, proto: int, payload: bytes, ident: int) -> bytes:
    h = bytearray(20)
    h[0], h[8], h[9] = 0x45, 64, proto
    h[2:4] = (20 + len(payload)).to_bytes(2, "big")
    h[4:6] = (ident & 0xFFFF).to_bytes(2, "big")
    h[12:16], h[16:20] = src, dst
    c = O.checksum(np.frombuffer(bytes(h), np.uint8))
    h[10:12] = c.to_bytes(2, "big")
    return bytes(h) + payload


def eth(payload: bytes) -> bytes:
    return MAC + bytes.fromhex("02aabbccdd01") + b"\x08\x00" + payload


def l4_crc(src: bytes, dst: bytes, proto: int, t: bytearray, field: int) -> None:
    t[field:field + 2] = b"\0\0"
    ps = src + dst + bytes([0, proto]) + len(t).to_bytes(2, "big")
    c = O.dualbuffer_checksum(np.frombuffer(ps, np.uint8), np.frombuffer(bytes(t), np.uint8))
    t[field:field + 2] = c.to_bytes(2, "big")


def tcp_seg(src, dst, sport, dport, seq, ack, flags, opts=b"", data=b"", wnd=8192):
    hl = 20 + len(opts)
    t = bytearray(struct.pack("!HHIIBBHHH", sport, dport, seq, ack, (hl // 4) << 4, flags, wnd, 0, 0)) + opts + data
    l4_crc(src, dst, 6, t, 16)
    return t


OPTS = [b"", b"\x02\x04\x05\xb4", b"\x02\x04\x05\xb4\x01\x03\x03\x07",
        b"\x02\x04\x05\xb4\x04\x02\x08\x0a\x00\x00\x10\x00\x00\x00\x00\x00\x01\x03\x03\x02",
        b"\x01\x01\x04\x02", b"\x02\x04\x02\x18\x01\x01\x08\x0a\x01\x02\x03\x04\x00\x00\x00\x00"]


def capture(seed: int = 1, conns: int = 24):
    """Drive one fresh reference stack; returns the captured datagrams (list of bytes)."""
    rng = np.random.default_rng(seed)
    R = ref_lib()
    assert R.rr_init() == 0 and R.rr_eth_init(MAC) == 0
    assert R.rr_ipv4_link(a32(HOST)) == 0
    R.rr_real_transport(1)
    cap = np.zeros(8 << 20, np.uint8)
    lens = np.zeros(8192, np.uint32)
    R.rr_tx_capture(cap.ctypes.data, cap.size, lens.ctypes.data, lens.size)
    ident = 1

    def rx(frame: bytes):
        b = np.frombuffer(frame, np.uint8).copy()
        R.rr_stack_rx(b.ctypes.data, b.size)

    def last_frames(k0):
        n = R.rr_tx_capture(cap.ctypes.data, cap.size, lens.ctypes.data, lens.size)   # (restarts the buffer)
        out = []
        o = 0
        for i in range(n):
            out.append(bytes(cap[o:o + lens[i]]))
            o += int(lens[i])
        return out

    frames = []
    # UDP (crc 0 on the reference's TX)
    s = R.rr_socket(17, a32(HOST), be16(5000), 0)
    assert s
    for i, ln in enumerate([0, 1, 2, 7, 8, 64, 333, 1000, 1471, 1472] + list(rng.integers(0, 1473, 20))):
        data = rng.integers(0, 256, int(ln), dtype=np.uint8).tobytes()
        buf = np.frombuffer(data, np.uint8).copy() if ln else np.zeros(1, np.uint8)
        R.rr_sendto(s, buf.ctypes.data, int(ln), a32(bytes([192, 168, 7, 200 + i % 40])), be16(7000 + i))
        R.rr_tick(2)
    frames += last_frames(0)
    # ICMPv4 echo requests -> replies
    for i, ln in enumerate([0, 1, 2, 3, 56, 57, 1000, 1472] + list(rng.integers(0, 1473, 16))):
        data = rng.integers(0, 256, int(ln), dtype=np.uint8).tobytes()
        m = bytearray(b"\x08\x00\x00\x00" + struct.pack("!HH", 0x1234 + i, i) + data)
        c = O.checksum(np.frombuffer(bytes(m), np.uint8))
        m[2:4] = c.to_bytes(2, "big")
        rx(eth(ipv4(bytes([192, 168, 7, 50 + i]), HOST, 1, bytes(m), ident)))
        ident += 1
        R.rr_tick(2)
    frames += last_frames(0)
    # TCP: SYN -> SYN-ACK, ACK, accept, write -> data segments; SYN to a closed port -> RST
    lst = R.rr_socket(6, a32(HOST), be16(80), 1)
    assert lst
    for c in range(conns):
        peer = bytes([192, 168, 7, 100 + c])
        sport, x = 40000 + c, int(rng.integers(0, 1 << 32))
        opts = OPTS[c % len(OPTS)]
        rx(eth(ipv4(peer, HOST, 6, bytes(tcp_seg(peer, HOST, sport, 80, x, 0, 0x02, opts)), ident)))
        ident += 1
        R.rr_tick(2)
        got = last_frames(0)
        frames += got
        synack = [f for f in got if f[9] == 6 and f[16:20] == peer and (f[20 + 13] & 0x12) == 0x12]
        if not synack:
            continue
        y = int.from_bytes(synack[-1][24:28], "big")
        rx(eth(ipv4(peer, HOST, 6, bytes(tcp_seg(peer, HOST, sport, 80, x + 1, y + 1, 0x10, wnd=65535)), ident)))
        ident += 1
        R.rr_tick(2)
        child = R.rr_accept(lst)
        if child:
            ln = int(rng.integers(1, 4000))
            data = rng.integers(0, 256, ln, dtype=np.uint8)
            R.rr_write(child, data.ctypes.data, ln)
            R.rr_tick(4)
        frames += last_frames(0)
        # a SYN to a closed port: RST
        rx(eth(ipv4(peer, HOST, 6, bytes(tcp_seg(peer, HOST, sport + 1000, 81, x ^ 0x5555, 0, 0x02)), ident)))
        ident += 1
        R.rr_tick(2)
        frames += last_frames(0)
    R.rr_tx_capture(None, 0, None, 0)
    return [f for f in frames if f[0] >> 4 == 4 and f[9] in (1, 6, 17)]


def main() -> None:
    frames = capture()
    buf = np.frombuffer(b"".join(frames), np.uint8)
    lens = np.array([len(f) for f in frames], np.uint32)
    off = np.concatenate([[0], np.cumsum(lens[:-1].astype(np.int64))]).astype(np.uint64)
    proto = np.array([f[9] for f in frames], np.uint8)
    np.savez_compressed(os.path.join(OUT, "ref_tx_cases.npz"), buf=buf, off=off, len=lens, proto=proto)
    print(f"ref_tx_cases.npz: {lens.size} datagrams ({int((proto == 6).sum())} TCP, {int((proto == 17).sum())} UDP, "
          f"{int((proto == 1).sum())} ICMPv4), {buf.size} bytes")


if __name__ == "__main__":
    main()

"""Seeded synthetic frame batches.

Byte source: splitmix64 (Steele, Lea, Flood 2014): state_i = seed + (i+1)*0x9E3779B97F4A7C15,
z = mix(state_i), little-endian bytes of z concatenated.  Same definition in the
golden-fixture generator (tests/golden/make_golden.py), so fixtures store only
seeds and expected outputs.
"""
from __future__ import annotations

import numpy as np

GAMMA = np.uint64(0x9E3779B97F4A7C15)
M1 = np.uint64(0xBF58476D1CE4E5B9)
M2 = np.uint64(0x94D049BB133111EB)


def splitmix64(seed: int, count: int, start: int = 0) -> np.ndarray:
    with np.errstate(over="ignore"):
        i = np.arange(start + 1, start + count + 1, dtype=np.uint64)
        z = np.uint64(seed & 0xFFFFFFFFFFFFFFFF) + i * GAMMA
        z = (z ^ (z >> np.uint64(30))) * M1
        z = (z ^ (z >> np.uint64(27))) * M2
        return z ^ (z >> np.uint64(31))


def random_bytes(seed: int, nbytes: int) -> np.ndarray:
    words = splitmix64(seed, (nbytes + 7) // 8)
    return words.view(np.uint8)[:nbytes].copy()


def uniform_batch(n: int, length: int, stride: int | None = None, seed: int = 1) -> np.ndarray:
    """C1/C3/C4: n frames of `length` random bytes at `stride` (default packed)."""
    stride = length if stride is None else stride
    total = (n - 1) * stride + length if n else 0
    return random_bytes(seed, total)


SIMPLE_IMIX = ((64, 7), (576, 4), (1500, 1))


def imix_lengths(n: int, seed: int, mix=SIMPLE_IMIX) -> np.ndarray:
    """C2: frame sizes in the simple-IMIX ratio 7:4:1, seeded shuffle."""
    sizes = np.concatenate([np.full(w, s, dtype=np.uint32) for s, w in mix])
    reps = -(-n // sizes.size)
    lens = np.tile(sizes, reps)[:n]
    perm = np.argsort(splitmix64(seed ^ 0x5EED, n), kind="stable")
    return lens[perm]


def ipv4_batch(lengths: np.ndarray, seed: int = 2, proto: int = 6, eth: bool = True, ihl: int = 5,
               frag=None, slot: int = 0):
    """IPv4 datagrams of the given total lengths, packed back to back, each with a
    valid header (vhl = 0x40|ihl, len, ttl 64, proto, random id/addresses/ports/payload)
    and a transport header (TCP 20 B, UDP 8 B, ICMP 8 B).  frag = the flags / offset field
    (host order) of every datagram, or an array cycled over them; default DF (0x4000).
    Every crc field is zero:
    make them valid with the TX kernel (PICO_CSUM_F_TX | F_WRITE) or a host checker.
    eth=True puts a 14-byte Ethernet header in front of each datagram (pico_ethernet.c:183),
    so the IPv4 headers are 2-byte aligned as in the reference RX path.
    slot > 0: frame k starts at k * slot instead (a driver's ring of fixed slots; the rest of each
    slot holds random bytes).
    Returns (buffer uint8, net offsets uint64, available bytes uint32)."""
    lengths = np.asarray(lengths, dtype=np.uint32)
    n = lengths.size
    pre = 14 if eth else 0
    frame_len = lengths.astype(np.uint64) + pre
    starts = np.zeros(n, dtype=np.uint64)
    if slot:
        assert int(frame_len.max(initial=0)) <= slot, "frame larger than its slot"
        starts = np.arange(n, dtype=np.uint64) * np.uint64(slot)
        total = n * slot
    else:
        if n:
            starts[1:] = np.cumsum(frame_len)[:-1]
        total = int(frame_len.sum())
    buf = random_bytes(seed, total)
    net = starts + np.uint64(pre)
    hl = 4 * ihl
    rnd = splitmix64(seed ^ 0xABCDEF, n).view(np.uint8).reshape(n, 8)
    idx = net.astype(np.int64)

    def put(off, vals):
        buf[idx + off] = vals

    if eth:
        e = starts.astype(np.int64)
        buf[e + 12] = 0x08
        buf[e + 13] = 0x00
    put(0, np.uint8(0x40 | ihl))
    put(1, 0)
    put(2, (lengths >> 8).astype(np.uint8))
    put(3, (lengths & 0xFF).astype(np.uint8))
    put(4, rnd[:, 0]); put(5, rnd[:, 1])
    if frag is None:
        put(6, 0x40); put(7, 0)
    else:
        fr = np.resize(np.asarray(frag, dtype=np.uint16), n) if n else np.zeros(0, np.uint16)
        put(6, (fr >> 8).astype(np.uint8)); put(7, (fr & 0xFF).astype(np.uint8))
    put(8, 64)
    put(9, np.uint8(proto))
    put(10, 0); put(11, 0)
    # src 10.x.y.z / dst 192.168.y.z from the random word
    put(12, 10); put(13, rnd[:, 2]); put(14, rnd[:, 3]); put(15, rnd[:, 4])
    put(16, 192); put(17, 168); put(18, rnd[:, 5]); put(19, rnd[:, 6])
    for o in range(20, hl):               # options: NOP padding
        put(o, 1)
    t = idx + hl
    if proto == 6:
        buf[t + 12] = 0x50                  # data offset 5
        buf[t + 13] = 0x18                  # PSH|ACK
        buf[t + 16] = 0
        buf[t + 17] = 0
    elif proto == 17:
        ul = (lengths - hl).astype(np.uint32)
        buf[t + 4] = (ul >> 8).astype(np.uint8)
        buf[t + 5] = (ul & 0xFF).astype(np.uint8)
        buf[t + 6] = 0
        buf[t + 7] = 0
    elif proto == 1:
        buf[t + 0] = 8                      # echo request
        buf[t + 1] = 0
        buf[t + 2] = 0
        buf[t + 3] = 0
    avail = lengths.copy()
    return buf, net, avail


def ipv6_batch(lengths: np.ndarray, seed: int = 3, proto: int = 6, eth: bool = True, hbh: bool = False,
               icmp_type: int = 128, frag=None, destopt: bool = False, walked: bool = False):
    """IPv6 datagrams of the given total lengths (40-byte header + optional 8-byte extension
    headers + transport), packed back to back, crc fields zero.  proto 6 / 17 / 58 (ICMPv6 of
    `icmp_type`).  Extension headers, in RFC 8200 order: hop-by-hop (PadN) when `hbh`, a
    destination-options header (PadN) when `destopt`, a fragment header carrying `frag` (the
    offset / M field, host order; scalar or an array cycled over the datagrams) when frag is not
    None.  Returns (buffer, net offsets, available bytes, descriptor seeds): seed =
    net_len | proto << 16 when extension headers are present and not `walked` (what
    pico_ipv6_extension_headers leaves in the frame), else 0 (the kernel walks them)."""
    lengths = np.asarray(lengths, dtype=np.uint32)
    n = lengths.size
    pre = 14 if eth else 0
    frame_len = lengths.astype(np.uint64) + pre
    starts = np.zeros(n, dtype=np.uint64)
    if n:
        starts[1:] = np.cumsum(frame_len)[:-1]
    buf = random_bytes(seed, int(frame_len.sum()))
    net = starts + np.uint64(pre)
    idx = net.astype(np.int64)
    chain = (["hbh"] if hbh else []) + (["dst"] if destopt else []) + (["frag"] if frag is not None else [])
    net_len = 40 + 8 * len(chain)
    plen = (lengths - 40).astype(np.uint32)
    if eth:
        e = starts.astype(np.int64)
        buf[e + 12] = 0x86
        buf[e + 13] = 0xDD
    code = {"hbh": 0, "dst": 60, "frag": 44}
    buf[idx + 0] = 0x60
    buf[idx + 4] = (plen >> 8).astype(np.uint8)
    buf[idx + 5] = (plen & 0xFF).astype(np.uint8)
    buf[idx + 6] = code[chain[0]] if chain else proto
    buf[idx + 7] = 255 if proto == 58 else 64
    for k, c in enumerate(chain):
        o = idx + 40 + 8 * k
        buf[o] = code[chain[k + 1]] if k + 1 < len(chain) else proto   # next header
        if c == "frag":
            fr = np.resize(np.asarray(frag, dtype=np.uint16), n) if n else np.zeros(0, np.uint16)
            buf[o + 1] = 0
            buf[o + 2] = (fr >> 8).astype(np.uint8)
            buf[o + 3] = (fr & 0xFF).astype(np.uint8)
        else:
            buf[o + 1] = 0            # length: 8 bytes
            buf[o + 2] = 1            # PadN
            buf[o + 3] = 4
            for q in range(4, 8):
                buf[o + q] = 0
    t = idx + net_len
    if proto == 6:
        buf[t + 12] = 0x50
        buf[t + 13] = 0x18
        buf[t + 16] = 0
        buf[t + 17] = 0
    elif proto == 17:
        ul = (lengths - net_len).astype(np.uint32)
        buf[t + 4] = (ul >> 8).astype(np.uint8)
        buf[t + 5] = (ul & 0xFF).astype(np.uint8)
        buf[t + 6] = 0
        buf[t + 7] = 0
    elif proto == 58:
        buf[t + 0] = icmp_type
        buf[t + 1] = 0
        buf[t + 2] = 0
        buf[t + 3] = 0
    seeds = np.full(n, (net_len | (proto << 16)) if chain and not walked else 0, dtype=np.uint32)
    return buf, net, lengths.copy(), seeds


ETH_KINDS = ("ipv4_tcp", "ipv4_udp", "ipv4_icmp", "ipv6_tcp", "ipv6_udp", "ipv6_icmp", "ipv6_hbh_tcp", "arp",
             "lldp", "ipv4_bad_version", "ipv4_opt_tcp", "ipv4_opt_udp", "ipv4_frag", "ipv4_evil", "ipv6_frag",
             "ipv6_dst_tcp")


def interleave(parts, kinds: np.ndarray):
    """One burst from several packed ones: parts[k] = (buffer, frame starts, frame bytes); frame i of
    the result is the next unused frame of parts[kinds[i]], back to back.  Returns (buffer, starts
    uint64, bytes uint32)."""
    kinds = np.asarray(kinds)
    n = kinds.size
    lens = np.zeros(n, np.int64)
    src = np.zeros(n, np.int64)                      # source start, in the concatenated parts
    base = 0
    for k, (b, st, ln) in enumerate(parts):
        sel = np.flatnonzero(kinds == k)
        assert sel.size <= st.size
        lens[sel] = np.asarray(ln, np.int64)[:sel.size]
        src[sel] = np.asarray(st, np.int64)[:sel.size] + base
        base += b.size
    cat = np.concatenate([b for b, _, _ in parts])
    starts = np.concatenate([[0], np.cumsum(lens)[:-1]])
    seg = np.repeat(np.arange(n), lens)
    idx = (src - starts)[seg] + np.arange(int(lens.sum()))
    return cat[idx], starts.astype(np.uint64), lens.astype(np.uint32)


def eth_batch(n: int, seed: int = 11, mac: bytes = bytes.fromhex("02005e0a0b0c")):
    """A mixed Ethernet burst as a TAP / pico_device RX ring delivers it: n frames, each
    with a 14-byte Ethernet header, of the kinds in ETH_KINDS (IPv4 / IPv6 datagrams in
    IMIX sizes, ARP, an unknown ethertype, an IPv4 ethertype carrying version 6), in seeded
    order with 0-3 byte gaps (every alignment), and destination MACs drawn from {mac,
    broadcast, 01:00:5e IPv4 multicast, 33:33 IPv6 multicast, a foreign unicast}.  Transport
    crc fields are zero (TX input).  IPv4 fragments (first / middle / last) and evil-bit
    datagrams, IPv6 datagrams behind a fragment or a destination-options header left for the
    kernel to walk (seed 0).  Returns (buffer, frame offsets uint64, frame bytes uint32,
    descriptor seeds uint32 (IPv6 net_len | proto << 16 behind a hop-by-hop header, else 0),
    kind index uint8 into ETH_KINDS)."""
    rng = np.random.default_rng(seed)
    kind = rng.integers(0, len(ETH_KINDS), n).astype(np.uint8)
    frames, seeds = [], np.zeros(n, dtype=np.uint32)
    lens = imix_lengths(n, seed ^ 0x33)
    for i in range(n):
        k = ETH_KINDS[kind[i]]
        s = seed * 7919 + i
        if k.startswith("ipv4"):
            proto = {"ipv4_tcp": 6, "ipv4_udp": 17, "ipv4_icmp": 1, "ipv4_bad_version": 6, "ipv4_opt_tcp": 6,
                     "ipv4_opt_udp": 17, "ipv4_frag": 6, "ipv4_evil": 17}[k]
            ihl = int(rng.integers(6, 16)) if "opt" in k else 5
            fr = None
            if k == "ipv4_frag":       # first / middle / last fragments
                fr = int(rng.choice([0x2000, 0x2000 | int(rng.integers(1, 0x1FFF)), int(rng.integers(1, 0x1FFF))]))
            elif k == "ipv4_evil":
                fr = 0x8000 | 0x4000
            b, _, _ = ipv4_batch(np.array([max(int(lens[i]), 4 * ihl + 28)], np.uint32), seed=s, proto=proto, eth=True,
                                 ihl=ihl, frag=fr)
            if k == "ipv4_bad_version":
                b[14] = 0x65
        elif k.startswith("ipv6"):
            proto = 6 if ("tcp" in k or k == "ipv6_frag") else 17 if "udp" in k else 58
            fr = (int(rng.integers(0, 200)) << 3) | int(rng.integers(0, 2)) if k == "ipv6_frag" else None
            b, _, _, sd = ipv6_batch(np.array([max(int(lens[i]) + 20, 68)], np.uint32), seed=s, proto=proto,
                                     eth=True, hbh="hbh" in k, icmp_type=int(rng.choice([128, 129, 135, 136, 143])),
                                     frag=fr, destopt=k == "ipv6_dst_tcp", walked=k in ("ipv6_frag", "ipv6_dst_tcp"))
            seeds[i] = sd[0]
            if proto != 58 and rng.random() < 0.6:
                b[14 + 9] = proto        # the byte pico_transport_crc_check dispatches on (pico_socket.c:1923)
        elif k == "arp":
            b = random_bytes(s, 60)
            b[12], b[13] = 0x08, 0x06
        else:
            b = random_bytes(s, int(rng.integers(60, 300)))
            b[12], b[13] = 0x88, 0xCC
        d = int(rng.integers(0, 10))
        dst = (mac if d < 5 else b"\xff" * 6 if d == 5 else bytes([0x01, 0x00, 0x5e, 1, 2, 3]) if d == 6
               else bytes([0x33, 0x33, 0, 0, 0, 1]) if d == 7 else bytes([0x02, 0x11, 0x22, 0x33, 0x44, 0x55]))
        b[0:6] = np.frombuffer(dst, np.uint8)
        frames.append(b)
    gaps = rng.integers(0, 4, n)
    off = np.zeros(n, dtype=np.uint64)
    pos = 0
    for i in range(n):
        pos += int(gaps[i])
        off[i] = pos
        pos += frames[i].size
    buf = random_bytes(seed ^ 0xE7, pos + 16)
    for i in range(n):
        buf[int(off[i]):int(off[i]) + frames[i].size] = frames[i]
    flen = np.array([f.size for f in frames], dtype=np.uint32)
    return buf, off, flen, seeds, kind


def _ones_sum(data: np.ndarray, seed: int = 0) -> int:
    """pico_checksum_adder over data (LE 16-bit words, odd trailing byte low), mod 2^32."""
    n = data.size
    s = int(data[: n & ~1].view("<u2").astype(np.uint64).sum()) if n >= 2 else 0
    if n & 1:
        s += int(data[-1])
    return (seed + s) & 0xFFFFFFFF


def _finalize(s: int) -> int:
    while s >> 16:
        s = (s & 0xFFFF) + (s >> 16)
    c = ~s & 0xFFFF
    return ((c >> 8) | (c << 8)) & 0xFFFF


def ipv4_fragments(lengths, seed: int = 21, proto: int = 17, frag_payload: int = 1480, shuffle: bool = True,
                   valid: bool = True):
    """IPv4 datagrams of the given TRANSPORT lengths, each split into fragments of
    `frag_payload` bytes (a multiple of 8; the last one shorter) as a sender's
    pico_ipv4_fragment / an MTU-1500 path produces them, every fragment an IPv4 frame
    (14-byte Ethernet gap, 20-byte header: tot = 20 + payload, frag = MF | offset/8, same
    id / src / dst / proto).  With `valid` the transport carries a correct TCP / UDP
    checksum over the whole datagram.  Fragments of a datagram are placed in the buffer
    (and listed) in a seeded arrival order when `shuffle`.
    Returns (buffer, frag offsets uint64 (-> IPv4 header), frag bytes uint32, groups
    uint32[n, 2] = (first descriptor, count) per datagram)."""
    lengths = np.asarray(lengths, dtype=np.uint32)
    assert frag_payload % 8 == 0 and frag_payload > 0
    rng = np.random.default_rng(seed)
    pieces, groups = [], []
    for g, L in enumerate(lengths.tolist()):
        t = random_bytes(seed * 1000003 + g, L)
        src = bytes([10, int(rng.integers(256)), int(rng.integers(256)), 1])
        dst = bytes([192, 168, int(rng.integers(256)), 2])
        if proto == 6 and L >= 20:
            t[12], t[13], t[16], t[17] = 0x50, 0x18, 0, 0
        if proto == 17 and L >= 8:
            t[4], t[5], t[6], t[7] = (L >> 8) & 0xFF, L & 0xFF, 0, 0
        if valid and proto in (6, 17) and L >= (20 if proto == 6 else 8):
            ph = np.frombuffer(src + dst + bytes([0, proto, (L >> 8) & 0xFF, L & 0xFF]), np.uint8)
            c = _finalize(_ones_sum(t, _ones_sum(ph)))
            x = 16 if proto == 6 else 6
            t[x], t[x + 1] = c >> 8, c & 0xFF
        ident = int(rng.integers(1, 65536))
        offs = list(range(0, max(L, 1), frag_payload)) if L else [0]
        frs = []
        for o in offs:
            pl = min(frag_payload, L - o)
            h = np.zeros(20, np.uint8)
            h[0], h[2], h[3] = 0x45, ((20 + pl) >> 8) & 0xFF, (20 + pl) & 0xFF
            h[4], h[5], h[8], h[9] = ident >> 8, ident & 0xFF, 64, proto
            fr = (o >> 3) | (0x2000 if o + pl < L else 0)
            h[6], h[7] = fr >> 8, fr & 0xFF
            h[12:16] = np.frombuffer(src, np.uint8)
            h[16:20] = np.frombuffer(dst, np.uint8)
            frs.append(np.concatenate([h, t[o:o + pl]]))
        if shuffle:
            frs = [frs[i] for i in rng.permutation(len(frs))]
        groups.append((len(pieces), len(frs)))
        pieces.extend(frs)
    n = len(pieces)
    place = rng.permutation(n) if shuffle else np.arange(n)
    off = np.zeros(n, dtype=np.uint64)
    pos = 0
    for j in place.tolist():
        pos += 14
        off[j] = pos
        pos += pieces[j].size
    buf = random_bytes(seed ^ 0xF4A6, pos + 16)
    for j in range(n):
        buf[int(off[j]):int(off[j]) + pieces[j].size] = pieces[j]
    flen = np.array([p.size for p in pieces], dtype=np.uint32)
    return buf, off, flen, np.array(groups, dtype=np.uint32).reshape(-1, 2)


def ipv6_fragments(lengths, seed: int = 23, proto: int = 6, frag_payload: int = 1448, shuffle: bool = True,
                   valid: bool = True, hbh: bool = False, b9_proto: bool = True):
    """IPv6 datagrams of the given TRANSPORT lengths, each split into fragments of
    `frag_payload` bytes (a multiple of 8; the last one shorter) as pico_ipv6_frag_send / an
    MTU-1500 path produces them: every fragment an IPv6 frame (14-byte Ethernet gap, 40-byte
    header, an optional 8-byte hop-by-hop header (PadN) when `hbh`, the 8-byte fragment header:
    next header = proto, offset | M, a per-datagram id; payload length = the rest), same src /
    dst.  With `valid` the transport carries a correct TCP / UDP / ICMPv6 checksum over the whole
    datagram; `b9_proto` puts proto into header byte 9 (the source address's second byte, which
    pico_transport_crc_check dispatches on).  Fragments of a datagram are placed (and listed) in
    a seeded arrival order when `shuffle`.
    Returns (buffer, frag offsets uint64 (-> IPv6 header), frag bytes uint32, groups uint32[n, 2])."""
    lengths = np.asarray(lengths, dtype=np.uint32)
    assert frag_payload % 8 == 0 and frag_payload > 0
    rng = np.random.default_rng(seed)
    pieces, groups = [], []
    for g, L in enumerate(lengths.tolist()):
        t = random_bytes(seed * 1000003 + g, L)
        src = bytearray(random_bytes(seed * 7 + g, 16).tobytes())
        dst = bytes(random_bytes(seed * 11 + g, 16).tobytes())
        if b9_proto:
            src[1] = proto
        src = bytes(src)
        x = {6: 16, 17: 6, 58: 2}.get(proto)
        if proto == 6 and L >= 20:
            t[12], t[13], t[16], t[17] = 0x50, 0x18, 0, 0
        if proto == 17 and L >= 8:
            t[4], t[5], t[6], t[7] = (L >> 8) & 0xFF, L & 0xFF, 0, 0
        if proto == 58 and L >= 4:
            t[0], t[2], t[3] = 128, 0, 0
        if valid and x is not None and L >= x + 2:
            ph = np.frombuffer(src + dst + L.to_bytes(4, "big") + bytes([0, 0, 0, proto]), np.uint8)
            c = _finalize(_ones_sum(t, _ones_sum(ph)))
            t[x], t[x + 1] = c >> 8, c & 0xFF
        ident = int(rng.integers(1, 1 << 32))
        offs = list(range(0, max(L, 1), frag_payload)) if L else [0]
        frs = []
        for o in offs:
            pl = min(frag_payload, L - o)
            ext = 16 if hbh else 8
            h = np.zeros(40 + ext, np.uint8)
            h[0] = 0x60
            plen = ext + pl
            h[4], h[5] = plen >> 8, plen & 0xFF
            h[6], h[7] = (0 if hbh else 44), 64
            h[8:24] = np.frombuffer(src, np.uint8)
            h[24:40] = np.frombuffer(dst, np.uint8)
            f = 40
            if hbh:
                h[40:48] = [44, 0, 1, 4, 0, 0, 0, 0]
                f = 48
            om = o | (1 if o + pl < L else 0)
            h[f:f + 8] = [proto, 0, om >> 8, om & 0xFF, ident >> 24, (ident >> 16) & 0xFF, (ident >> 8) & 0xFF,
                          ident & 0xFF]
            frs.append(np.concatenate([h, t[o:o + pl]]))
        if shuffle:
            frs = [frs[i] for i in rng.permutation(len(frs))]
        groups.append((len(pieces), len(frs)))
        pieces.extend(frs)
    n = len(pieces)
    place = rng.permutation(n) if shuffle else np.arange(n)
    off = np.zeros(n, dtype=np.uint64)
    pos = 0
    for j in place.tolist():
        pos += 14
        off[j] = pos
        pos += pieces[j].size
    buf = random_bytes(seed ^ 0xF6A6, pos + 16)
    for j in range(n):
        buf[int(off[j]):int(off[j]) + pieces[j].size] = pieces[j]
    flen = np.array([p.size for p in pieces], dtype=np.uint32)
    return buf, off, flen, np.array(groups, dtype=np.uint32).reshape(-1, 2)

"""GPU: the device RX pipeline of INTEGRATION.md sections 2, 5a and 5c, end to end on one burst.

A burst of Ethernet frames as a TAP poll would read it: whole IPv4 / TCP datagrams (valid, and a
few with a flipped transport byte), the 1480-byte fragments of larger TCP / UDP datagrams
interleaved in arrival order (shuffled within each datagram), ARP frames and frames for a foreign
MAC.  Then, as the recipe says:
  1. pico_eth_checksum_batch_dev (RX, MAC filter) -- verdicts equal the oracle's;
  2. the host groups the V_FRAG frames by (src, dst, id, proto) in arrival order and hands them
     (descriptors at the IP header) to pico_ipv4_reassemble_batch_dev -- every datagram comes
     back whole, byte for byte the datagram the sender fragmented, with its transport check
     passed;
  3. the accepted whole datagrams go through pico_ipv4_nat_batch_dev (outbound) -- every byte
     as oracle_batch_ipv4_nat writes it, and the rewritten datagrams pass the RX batch again."""
from __future__ import annotations

import numpy as np
import pytest
import torch

from oracle import oracle as O
from picotcp_amd import batch, synth
from tests.test_gpu_parity import to_dev

pytestmark = pytest.mark.gpu

MAC = bytes.fromhex("02005e0a0b0c")


def eth(ip: np.ndarray, dst: bytes = MAC, etype: int = 0x0800, rng=None) -> np.ndarray:
    h = np.zeros(14, np.uint8)
    h[0:6] = np.frombuffer(dst, np.uint8)
    h[6:12] = rng.integers(0, 256, 6) if rng is not None else 0x11
    h[12], h[13] = etype >> 8, etype & 0xFF
    return np.concatenate([h, ip])


def whole_datagrams(rng, n):
    lens = synth.imix_lengths(n, 5)
    buf, net, avail = synth.ipv4_batch(lens, seed=9, proto=6, eth=False)
    desc = batch.make_desc(net, avail)
    on, ol, _ = O.batch_ipv4(buf, desc, tx=True)          # make every checksum valid
    out = []
    for i in range(n):
        o = int(net[i])
        d = buf[o:o + int(lens[i])].copy()
        d[10], d[11] = on[i] >> 8, on[i] & 0xFF
        d[36], d[37] = ol[i] >> 8, ol[i] & 0xFF            # TCP crc at 20 + 16
        out.append(d)
    return out


def test_rx_reassembly_nat_pipeline():
    rng = np.random.default_rng(2024)
    whole = whole_datagrams(rng, 3000)
    bad = set(rng.choice(len(whole), 60, replace=False).tolist())
    for i in bad:                                          # a flipped transport byte: V_L4_BAD
        whole[i][-1] ^= 0x5A
    big = rng.integers(3000, 20000, 40).tolist()
    fbuf, foff, flen, grp = synth.ipv4_fragments(big, seed=3, proto=6, frag_payload=1480, shuffle=True)
    fon, _, _ = O.batch_ipv4(fbuf, batch.make_desc(foff, flen), tx=True)   # valid header checksums
    for j in range(foff.size):
        fbuf[int(foff[j]) + 10], fbuf[int(foff[j]) + 11] = fon[j] >> 8, fon[j] & 0xFF
    frags = [fbuf[int(foff[j]):int(foff[j]) + int(flen[j])].copy() for j in range(foff.size)]
    # the burst: whole datagrams, fragments (each datagram's in its arrival order), ARP, foreign MACs
    items = [("w", i) for i in range(len(whole))]
    queues = [list(range(int(grp[g, 0]), int(grp[g, 0] + grp[g, 1]))) for g in range(len(big))]
    items += [("f", j) for q in queues for j in q]
    order = rng.permutation(len(items))
    seq = []
    fq = [list(q) for q in queues]
    qi = {j: g for g, q in enumerate(queues) for j in q}
    for k in order:                                        # keep arrival order within a datagram
        kind, idx = items[k]
        if kind == "f":
            g = qi[idx]
            idx = fq[g].pop(0)
        seq.append((kind, idx))
    frames, kinds = [], []
    for kind, idx in seq:
        frames.append(eth(whole[idx] if kind == "w" else frags[idx], rng=rng))
        kinds.append((kind, idx))
        if rng.random() < 0.01:
            frames.append(eth(rng.integers(0, 256, 28).astype(np.uint8), dst=b"\xff" * 6, etype=0x0806, rng=rng))
            kinds.append(("arp", -1))
        if rng.random() < 0.01:
            frames.append(eth(whole[0], dst=bytes.fromhex("020000000099"), rng=rng))
            kinds.append(("foreign", -1))
    off = np.zeros(len(frames), np.uint64)
    p = 0
    for i, f in enumerate(frames):
        off[i] = p
        p += f.size + 2                                     # a gap; headers land at any alignment
    ring = np.zeros(p + 16, np.uint8)
    for i, f in enumerate(frames):
        ring[int(off[i]):int(off[i]) + f.size] = f
    desc = batch.make_desc(off, np.array([f.size for f in frames], np.uint32))
    n = desc.size

    # 1. the Ethernet front end, RX
    d_ring = to_dev(ring)
    on, ol, v = batch.eth_checksum_batch(d_ring, batch.desc_to_device(desc, "cuda:0"), n, mac=MAC)
    torch.cuda.synchronize()
    v = v.cpu().numpy()
    won, wol, wv = O.batch_eth(ring, desc, mac=MAC)
    np.testing.assert_array_equal(v, wv)
    kinds_a = np.array([k for k, _ in kinds])
    assert (v[kinds_a == "arp"] == batch.V_ARP).all() and (v[kinds_a == "foreign"] == batch.V_DROP_L2).all()
    wi = np.array([k == "w" for k, _ in kinds])
    wbad = np.array([k == "w" and i in bad for k, i in kinds])
    assert (v[wi & ~wbad] == batch.V_ACCEPT).all() and (v[wbad] == batch.V_L4_BAD).all()
    assert (v[kinds_a == "f"] == batch.V_FRAG).all()

    # 2. fragments -> reassembly, grouped by (src, dst, id, proto) in arrival order
    fr = np.flatnonzero(v == batch.V_FRAG)
    ipo = off[fr] + 14
    key = {}
    for j, o in zip(fr.tolist(), ipo.tolist()):
        h = ring[o:o + 20]
        key.setdefault((bytes(h[12:20]), bytes(h[4:6]), int(h[9])), []).append(o)
    groups, fd = [], []
    for k_, offs in key.items():
        groups.append((len(fd), len(offs)))
        fd.extend(offs)
    fdesc = batch.make_desc(np.array(fd, np.uint64), np.array([int(ring[o + 2]) << 8 | int(ring[o + 3]) for o in fd],
                                                              np.uint32))
    ng = len(groups)
    cap = (20 + max(big) + 16 + 15) // 16 * 16           # output regions 16-byte aligned
    od = batch.make_desc(np.arange(ng, dtype=np.uint64) * cap, np.full(ng, cap, np.uint32))
    out = torch.zeros(ng * cap, dtype=torch.uint8, device="cuda:0")
    rl, rl4, rv = batch.ipv4_reassemble_batch(
        d_ring, batch.desc_to_device(fdesc, "cuda:0"), len(fd),
        to_dev(np.array(groups, np.uint32).reshape(-1).view(np.int32)), out, batch.desc_to_device(od, "cuda:0"))
    torch.cuda.synchronize()
    rv, rl, out_h = rv.cpu().numpy(), rl.cpu().numpy().view(np.uint32), out.cpu().numpy()
    assert ng == len(big) and (rv == batch.V_ACCEPT).all()
    sent = {}                                              # the sender's datagrams, by (addrs, id)
    for g in range(len(big)):
        j0 = int(grp[g, 0])
        h = fbuf[int(foff[j0]):int(foff[j0]) + 20]
        sent[(bytes(h[12:20]), bytes(h[4:6]), int(h[9]))] = g
    for gi, (k_, offs) in enumerate(key.items()):
        g = sent[k_]
        assert rl[gi] == big[g]
        parts = sorted(range(int(grp[g, 0]), int(grp[g, 0] + grp[g, 1])),
                       key=lambda j: (int(fbuf[int(foff[j]) + 6]) << 8 | int(fbuf[int(foff[j]) + 7])) & 0x1FFF)
        payload = np.concatenate([fbuf[int(foff[j]) + 20:int(foff[j]) + int(flen[j])] for j in parts])
        np.testing.assert_array_equal(out_h[gi * cap + 20:gi * cap + 20 + big[g]], payload)

    # 3. the accepted whole datagrams -> NAT outbound, then RX again
    acc = np.flatnonzero(wi & (v == batch.V_ACCEPT))
    ndesc = batch.make_desc(off[acc] + 14, desc["len"][acc] - 14)
    nat = np.zeros(acc.size, batch.NAT_DTYPE)
    nat["addr"] = int.from_bytes(bytes([198, 51, 100, 1]), "little")
    nat["port"] = rng.integers(1024, 65536, acc.size).astype(np.uint16)
    nat["dir"] = batch.NAT_OUTBOUND
    nn, nl, nv = batch.ipv4_nat_batch(d_ring, batch.desc_to_device(ndesc, "cuda:0"), acc.size,
                                      to_dev(nat.view(np.uint8)))
    torch.cuda.synchronize()
    after = ring.copy()
    O.batch_ipv4_nat(after, ndesc, nat)
    np.testing.assert_array_equal(d_ring.cpu().numpy(), after)
    assert (nv.cpu().numpy() == batch.V_ACCEPT).all()
    _, _, v2 = batch.ipv4_checksum_batch(d_ring, batch.desc_to_device(ndesc, "cuda:0"), acc.size)
    torch.cuda.synchronize()
    assert (v2.cpu().numpy() == batch.V_ACCEPT).all()

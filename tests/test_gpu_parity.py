"""GPU parity: the HIP kernels (through the C ABI) against the oracle and the
reference's golden fixtures, bit-exact.  Run on an MI355X with `-m gpu`."""
from __future__ import annotations

import numpy as np
import pytest
import torch

from oracle import oracle as O
from picotcp_amd import batch, synth
from tests import golden_data as G

pytestmark = pytest.mark.gpu

DEV = "cuda:0"
SHAPES = [(g, c) for g in (4, 8, 16, 32, 64) for c in (1, 2, 4, 8)] + \
    [(g, c) for g in (8, 16, 32, 64) for c in (3, 5, 6, 7)]     # (the pipelined kernel's extra shapes)
# descriptor batches: the sorted-rounds kernel, automatic or with a forced frames-per-wave
# (1: a wave per frame; 5 / 7 / 13: ragged waves; 64: full waves whatever the batch size)
FPWS = (1, 5, 7, 13, 64)
KERNELS = {"auto": None, **{f"fpw{f}": f for f in FPWS}}


def use_kernel(name):
    if KERNELS[name] is None:
        batch.set_launch_override(0)
    else:
        batch.set_launch_override(2, fpw=KERNELS[name])


def u16(t: torch.Tensor) -> np.ndarray:
    torch.cuda.synchronize()
    return t.cpu().numpy().view(np.uint16)


def to_dev(a: np.ndarray) -> torch.Tensor:
    return torch.from_numpy(np.ascontiguousarray(a)).to(DEV)


@pytest.fixture(autouse=True)
def _reset_override():
    yield
    batch.set_launch_override(0, 0, 0)


# ------------------------------------------------------------------ uniform

@pytest.mark.parametrize("name,stride", [("c1_1500_packed", 1500), ("c1_1500_stride1536", 1536)])
def test_uniform_golden(name, stride):
    case = G.raw_cases()[name]
    buf, _ = G.raw_case_inputs(case, lambda b: O.adder(0, b))
    n = case["off"].size
    got = u16(batch.checksum_uniform(to_dev(buf), stride, 1500, n))
    np.testing.assert_array_equal(got, case["expected"])


@pytest.mark.parametrize("g,c", SHAPES)
def test_uniform_every_shape(g, c):
    """Every compiled (group, chunks-per-lane) shape, several frames-per-wave, odd lengths,
    odd strides, a seed -- against the oracle."""
    rng = np.random.default_rng(g * 10 + c)
    for ln, stride in ((1500, 1500), (1501, 1503), (63, 64), (0, 8), (9000, 9001), (3, 5)):
        n = int(rng.integers(1, 700))
        buf = synth.uniform_batch(n, ln, stride, seed=ln + stride)
        if buf.size == 0:
            buf = np.zeros(16, np.uint8)
        seed = int(rng.integers(0, 1 << 32))
        want = O.batch_uniform(buf, stride, ln, n, seed)
        d = to_dev(buf)
        for fpw in sorted({64 // g, 64, (64 // g) * 3 if (64 // g) * 3 <= 64 else 64}):
            for pipe in ((2,) if c in (3, 5, 6, 7) else (1, 2)):   # (frames past one pass: multi-pass)
                batch.set_launch_override(g, c, fpw, 1, 2 if pipe == 2 else 1, pipe)
                got = u16(batch.checksum_uniform(d, stride, ln, n, seed=seed))
                np.testing.assert_array_equal(got, want, err_msg=f"g={g} c={c} fpw={fpw} pipe={pipe} len={ln} "
                                                                 f"stride={stride}")


def test_uniform_automatic_shapes_every_length_class():
    """The launcher's own shape (no override) over frame lengths that land on every lane-group
    width and every exact chunk count of the pipelined kernel (3, 5-7 chunks a lane as well as the
    powers of two), odd strides and a seed -- against the oracle."""
    rng = np.random.default_rng(77)
    for ln in list(range(1, 200, 13)) + list(range(200, 2200, 37)) + [1500, 1520, 1521, 1522, 4000, 8170]:
        stride = ln + int(rng.integers(0, 9))
        n = int(rng.integers(100, 1500))
        buf = synth.uniform_batch(n, ln, stride, seed=ln)
        seed = int(rng.integers(0, 1 << 32))
        want = O.batch_uniform(buf, stride, ln, n, seed)
        got = u16(batch.checksum_uniform(to_dev(buf), stride, ln, n, seed=seed))
        np.testing.assert_array_equal(got, want, err_msg=f"len={ln} stride={stride} n={n}")


def test_uniform_c1_full_size():
    """C1 at its full size: 256K x 1500 B, bit-exact against the oracle on every frame."""
    n, ln = 262144, 1500
    buf = synth.uniform_batch(n, ln, seed=2026)
    want = O.batch_uniform(buf, ln, ln, n)
    got = u16(batch.checksum_uniform(to_dev(buf), ln, ln, n))
    np.testing.assert_array_equal(got, want)


def test_uniform_c3_jumbo_full_size():
    """C3: 256K x 9000 B jumbo frames (2.2 GiB), bit-exact on every frame."""
    n, ln = 262144, 9000
    buf = synth.uniform_batch(n, ln, seed=2027)
    want = O.batch_uniform(buf, ln, ln, n)
    got = u16(batch.checksum_uniform(to_dev(buf), ln, ln, n))
    np.testing.assert_array_equal(got, want)
    del buf


# ------------------------------------------------------------------ descriptors

@pytest.mark.parametrize("name", ["mixed_align", "c2_imix_raw", "c3_9000", "c3_65536", "wrap_lengths",
                                  "c1_1500_packed"])
def test_desc_golden(name):
    case = G.raw_cases()[name]
    buf, desc = G.raw_case_inputs(case, lambda b: O.adder(0, b))
    got = u16(batch.checksum_batch(to_dev(buf), batch.desc_to_device(desc, DEV), desc.size))
    np.testing.assert_array_equal(got, case["expected"])


@pytest.mark.parametrize("fpw", FPWS)
def test_desc_every_fpw(fpw):
    case = G.raw_cases()["mixed_align"]
    buf, desc = G.raw_case_inputs(case, lambda b: O.adder(0, b))
    d_buf, d_desc = to_dev(buf), batch.desc_to_device(desc, DEV)
    batch.set_launch_override(2, fpw=fpw)
    got = u16(batch.checksum_batch(d_buf, d_desc, desc.size))
    np.testing.assert_array_equal(got, case["expected"], err_msg=f"fpw={fpw}")


@pytest.mark.parametrize("kernel", list(KERNELS))
def test_desc_big_regions(kernel):
    """Regions over 64K chunks (> 1 MiB) in 64-lane rounds, mixed with small ones, odd
    offsets, seeds and a crc field."""
    rng = np.random.default_rng(44)
    buf = synth.random_bytes(45, 12 << 20)
    offs = [1, 3 << 20, 5, (7 << 20) + 3, 100, 2000, 11 << 20]
    lens = [2 << 20, (3 << 20) + 1, 64, (1 << 20) + 17, 1500, 0, 123457]
    desc = batch.make_desc(offs, lens, rng.integers(0, 1 << 32, len(offs), dtype=np.uint64).astype(np.uint32))
    use_kernel(kernel)
    for crc in (-1, 10):
        want = O.batch_raw(buf, desc, crc_off=crc)
        got = u16(batch.checksum_batch(to_dev(buf), batch.desc_to_device(desc, DEV), len(offs), crc_off=crc))
        np.testing.assert_array_equal(got, want)


def test_desc_empty_and_edge_lengths():
    buf = synth.random_bytes(99, 4096)
    offs, lens = [], []
    for off in range(0, 33):
        for ln in (0, 1, 2, 3, 4, 15, 16, 17, 31, 32, 33):
            offs.append(off)
            lens.append(ln)
    desc = batch.make_desc(offs, lens)
    want = O.batch_raw(buf, desc)
    got = u16(batch.checksum_batch(to_dev(buf), batch.desc_to_device(desc, DEV), desc.size))
    np.testing.assert_array_equal(got, want)
    assert (want[np.array(lens) == 0] == 0xFFFF).all()


def test_desc_crc_field_and_write_roundtrip():
    """crc_off: the field reads as zero; F_WRITE stores short_be(ret) there; the
    region then verifies to 0 -- the TX insert / RX verify round trip."""
    rng = np.random.default_rng(12)
    n = 3000
    lens = rng.integers(12, 1500, n)
    offs = np.zeros(n, dtype=np.uint64)
    offs[1:] = np.cumsum(lens.astype(np.uint64) + rng.integers(0, 5, n).astype(np.uint64))[:-1]
    offs += 1
    buf = synth.random_bytes(7, int(offs[-1]) + int(lens[-1]) + 7)
    seeds = rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32)
    desc = batch.make_desc(offs, lens, seeds)
    want = O.batch_raw(buf, desc, crc_off=10)
    d_buf, d_desc = to_dev(buf), batch.desc_to_device(desc, DEV)
    got = u16(batch.checksum_batch(d_buf, d_desc, n, crc_off=10))
    np.testing.assert_array_equal(got, want)
    got = u16(batch.checksum_batch(d_buf, d_desc, n, crc_off=10, flags=batch.F_WRITE))
    np.testing.assert_array_equal(got, want)
    after = d_buf.cpu().numpy()
    f = offs.astype(np.int64) + 10
    np.testing.assert_array_equal(after[f], (want >> 8).astype(np.uint8))
    np.testing.assert_array_equal(after[f + 1], (want & 0xFF).astype(np.uint8))
    verify = u16(batch.checksum_batch(d_buf, d_desc, n))
    assert (verify == 0).all()
    # bytes outside the crc fields untouched
    mask = np.ones(after.size, bool)
    mask[f] = False
    mask[f + 1] = False
    np.testing.assert_array_equal(after[mask], buf[mask])


@pytest.mark.parametrize("kernel", list(KERNELS))
def test_desc_crc_write_every_kernel(kernel):
    rng = np.random.default_rng(21)
    n = 2000
    lens = rng.integers(0, 3000, n)
    offs = np.zeros(n, dtype=np.uint64)
    offs[1:] = np.cumsum(lens.astype(np.uint64) + rng.integers(0, 3, n).astype(np.uint64))[:-1]
    offs += 3
    buf = synth.random_bytes(17, int(offs[-1]) + int(lens[-1]) + 5)
    desc = batch.make_desc(offs, lens, rng.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32))
    want = O.batch_raw(buf, desc, crc_off=16)
    use_kernel(kernel)
    d_buf, d_desc = to_dev(buf), batch.desc_to_device(desc, DEV)
    got = u16(batch.checksum_batch(d_buf, d_desc, n, crc_off=16, flags=batch.F_WRITE))
    np.testing.assert_array_equal(got, want)
    verify = u16(batch.checksum_batch(d_buf, d_desc, n))
    has = lens >= 18
    assert (verify[has] == 0).all()


@pytest.mark.parametrize("kernel", list(KERNELS))
def test_desc_out_of_bounds_every_kernel(kernel):
    use_kernel(kernel)
    test_desc_out_of_bounds_regions_are_not_read()


def test_desc_out_of_bounds_regions_are_not_read():
    """Descriptors past the buffer: not read, result 0, counted in d_bad; the rest exact."""
    buf = synth.random_bytes(8, 10000)
    offs = [0, 9000, 9990, 10000, 10001, 1 << 40, 5000, 100]
    lens = [1500, 1000, 10, 0, 1, 16, 6000, 200]
    desc = batch.make_desc(offs, lens)
    bad = torch.zeros(1, dtype=torch.int32, device=DEV)
    got = u16(batch.checksum_batch(to_dev(buf), batch.desc_to_device(desc, DEV), len(offs), bad=bad))
    ok = [i for i in range(len(offs)) if offs[i] + lens[i] <= buf.size]
    want = O.batch_raw(buf, desc[ok])
    np.testing.assert_array_equal(got[ok], want)
    oob = [i for i in range(len(offs)) if i not in ok]
    assert (got[oob] == 0).all()
    assert int(bad.item()) == len(oob)


# ------------------------------------------------------------------ IPv4 fused

def test_ipv4_golden_rx_tx():
    c = G.ipv4_cases()
    desc = batch.desc_to_device(G.ipv4_desc(c["net"], c["avail"]), DEV)
    n = c["net"].size
    net, l4, v = batch.ipv4_checksum_batch(to_dev(c["buf"]), desc, n)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(v.cpu().numpy(), c["rx_verdict"])
    np.testing.assert_array_equal(u16(net), c["rx_net"])
    np.testing.assert_array_equal(u16(l4), c["rx_l4"])
    net, l4, v = batch.ipv4_checksum_batch(to_dev(c["tx_buf"]), desc, n, flags=batch.F_TX)
    np.testing.assert_array_equal(u16(net), c["tx_net"])
    np.testing.assert_array_equal(u16(l4), c["tx_l4"])
    np.testing.assert_array_equal(v.cpu().numpy(), c["tx_verdict"])


@pytest.mark.parametrize("fpw", FPWS)
def test_ipv4_every_fpw(fpw):
    """The fixture (valid, corrupted, fragments, the evil bit, IHL < 5, bad sources, options,
    truncations) with every wave shape, RX and TX."""
    cs = G.ipv4_cases()
    desc = batch.desc_to_device(G.ipv4_desc(cs["net"], cs["avail"]), DEV)
    n = cs["net"].size
    d_buf = to_dev(cs["buf"])
    batch.set_launch_override(2, fpw=fpw)
    net, l4, v = batch.ipv4_checksum_batch(d_buf, desc, n)
    np.testing.assert_array_equal(u16(net), cs["rx_net"], err_msg=f"fpw={fpw}")
    np.testing.assert_array_equal(u16(l4), cs["rx_l4"], err_msg=f"fpw={fpw}")
    np.testing.assert_array_equal(v.cpu().numpy(), cs["rx_verdict"], err_msg=f"fpw={fpw}")
    net, l4, v = batch.ipv4_checksum_batch(to_dev(cs["tx_buf"]), desc, n, flags=batch.F_TX)
    np.testing.assert_array_equal(u16(net), cs["tx_net"], err_msg=f"TX fpw={fpw}")
    np.testing.assert_array_equal(u16(l4), cs["tx_l4"], err_msg=f"TX fpw={fpw}")
    np.testing.assert_array_equal(v.cpu().numpy(), cs["tx_verdict"], err_msg=f"TX fpw={fpw}")


def test_ipv4_out_of_bounds_is_malformed():
    c = G.unit_socket_frames()
    net = np.array([0, 64 * 5, 64 * 5 + 1, 1 << 33], dtype=np.uint64)
    avail = np.array([64, 64, 64, 64], dtype=np.uint32)
    desc = batch.desc_to_device(G.ipv4_desc(net, avail), DEV)
    _, _, v = batch.ipv4_checksum_batch(to_dev(c["buf"]), desc, 4)
    np.testing.assert_array_equal(v.cpu().numpy(), [c["rx_verdict"][0], c["rx_verdict"][5], 8, 8])


def test_ipv4_unit_socket_frames():
    c = G.unit_socket_frames()
    desc = batch.desc_to_device(G.ipv4_desc(c["net"], c["avail"]), DEV)
    net, l4, v = batch.ipv4_checksum_batch(to_dev(c["buf"]), desc, c["net"].size)
    np.testing.assert_array_equal(v.cpu().numpy(), c["rx_verdict"])
    np.testing.assert_array_equal(u16(net), c["rx_net"])
    np.testing.assert_array_equal(u16(l4), c["rx_l4"])


@pytest.mark.parametrize("proto,eth,ihl", [(6, True, 5), (6, False, 7), (17, True, 5), (1, True, 5), (6, True, 15)])
def test_ipv4_tx_write_then_rx_accepts(proto, eth, ihl):
    """C2-style IMIX batch: TX compute + in-place write, then RX verify accepts every
    datagram; the written fields equal the oracle's TX outputs."""
    lens = synth.imix_lengths(20000, 5 + proto)
    lens = np.maximum(lens, 4 * ihl + 20).astype(np.uint32)
    buf, net_off, avail = synth.ipv4_batch(lens, seed=proto * 7 + ihl, proto=proto, eth=eth, ihl=ihl)
    desc_h = G.ipv4_desc(net_off, avail)
    want_net, want_l4, want_v = O.batch_ipv4(buf, desc_h, tx=True)
    assert (want_v == 1).all()
    d_buf, d_desc = to_dev(buf), batch.desc_to_device(desc_h, DEV)
    net, l4, v = batch.ipv4_checksum_batch(d_buf, d_desc, lens.size, flags=batch.F_TX | batch.F_WRITE)
    np.testing.assert_array_equal(u16(net), want_net)
    np.testing.assert_array_equal(u16(l4), want_l4)
    net, l4, v = batch.ipv4_checksum_batch(d_buf, d_desc, lens.size)
    assert (v.cpu().numpy() == 1).all()
    assert (u16(net) == 0).all()
    assert (u16(l4) == 0).all()
    # oracle agrees on the written buffer
    wb = d_buf.cpu().numpy()
    on, ol, ov = O.batch_ipv4(wb, desc_h, tx=False)
    assert (ov == 1).all()


def test_c2_full_size_rx():
    """C2 at full size: 256K IMIX IPv4/TCP datagrams, RX verify vs oracle, with 1/64 corrupted."""
    lens = synth.imix_lengths(262144, 2026)
    buf, net_off, avail = synth.ipv4_batch(lens, seed=11, proto=6, eth=True)
    desc_h = G.ipv4_desc(net_off, avail)
    d_buf, d_desc = to_dev(buf), batch.desc_to_device(desc_h, DEV)
    batch.ipv4_checksum_batch(d_buf, d_desc, lens.size, flags=batch.F_TX | batch.F_WRITE)
    torch.cuda.synchronize()
    h = d_buf.cpu().numpy()
    bad = net_off[::64].astype(np.int64) + 30
    h[bad] ^= 0x10
    want = O.batch_ipv4(h, desc_h, tx=False)
    got = batch.ipv4_checksum_batch(to_dev(h), d_desc, lens.size)
    np.testing.assert_array_equal(u16(got[0]), want[0])
    np.testing.assert_array_equal(u16(got[1]), want[1])
    np.testing.assert_array_equal(got[2].cpu().numpy(), want[2])
    assert (want[2][::64] != 1).all() and (np.delete(want[2], np.arange(0, lens.size, 64)) == 1).all()


# ------------------------------------------------------------------ host-resident

def test_host_batch_roundtrip():
    n, ln = 50000, 1500
    buf = synth.uniform_batch(n, ln, seed=31)
    want = O.batch_uniform(buf, ln, ln, n)
    hb = batch.HostBatch(0, staging_bytes=8 << 20)
    try:
        got = hb.checksum_uniform(buf, ln, ln, n)
    finally:
        hb.close()
    np.testing.assert_array_equal(got, want)


# ------------------------------------------------------------------ IPv6 fused

@pytest.mark.parametrize("kernel", list(KERNELS))
def test_ipv6_golden_rx_tx(kernel):
    """RX with the reference's byte-9 dispatch (default) and the next-header dispatch, TX."""
    cs = G.ipv6_cases()
    desc = batch.desc_to_device(G.ipv6_desc(cs), DEV)
    n = cs["net"].size
    use_kernel(kernel)
    l4, v = batch.ipv6_checksum_batch(to_dev(cs["buf"]), desc, n)
    np.testing.assert_array_equal(v.cpu().numpy(), cs["rx_verdict"])
    np.testing.assert_array_equal(u16(l4), cs["rx_l4"])
    l4, v = batch.ipv6_checksum_batch(to_dev(cs["buf"]), desc, n, flags=batch.F_NXTHDR_DISPATCH)
    np.testing.assert_array_equal(v.cpu().numpy(), cs["rx_verdict_nx"])
    np.testing.assert_array_equal(u16(l4), cs["rx_l4_nx"])
    l4, v = batch.ipv6_checksum_batch(to_dev(cs["tx_buf"]), desc, n, flags=batch.F_TX)
    np.testing.assert_array_equal(v.cpu().numpy(), cs["tx_verdict"])
    np.testing.assert_array_equal(u16(l4), cs["tx_l4"])


@pytest.mark.parametrize("proto,hbh,icmp_type", [(6, False, 0), (17, False, 0), (58, False, 135), (6, True, 0),
                                                 (58, True, 131)])
def test_ipv6_tx_write_then_rx_accepts(proto, hbh, icmp_type):
    lens = np.maximum(synth.imix_lengths(20000, 3 + proto), 48 + 20).astype(np.uint32)
    kw = dict(seed=proto + 7, proto=proto, eth=True, hbh=hbh)
    if proto == 58:
        kw["icmp_type"] = icmp_type
    buf, net_off, avail, seeds = synth.ipv6_batch(lens, **kw)
    desc_h = G.ipv4_desc(net_off, avail)
    desc_h["seed"] = seeds
    want_l4, want_v = O.batch_ipv6(buf, desc_h, tx=True)
    assert (want_v == 1).all()
    d_buf, d_desc = to_dev(buf), batch.desc_to_device(desc_h, DEV)
    l4, v = batch.ipv6_checksum_batch(d_buf, d_desc, lens.size, flags=batch.F_TX | batch.F_WRITE)
    np.testing.assert_array_equal(u16(l4), want_l4)
    l4, v = batch.ipv6_checksum_batch(d_buf, d_desc, lens.size, flags=batch.F_NXTHDR_DISPATCH)
    assert (v.cpu().numpy() == 1).all()
    assert (u16(l4) == 0).all()
    ol, ov = O.batch_ipv6(d_buf.cpu().numpy(), desc_h, nxthdr_dispatch=True)
    assert (ov == 1).all()
    # the reference's dispatch (byte 9) on the same bytes: whatever it checks, the oracle agrees
    wl, wv = O.batch_ipv6(d_buf.cpu().numpy(), desc_h)
    l4, v = batch.ipv6_checksum_batch(d_buf, d_desc, lens.size)
    np.testing.assert_array_equal(v.cpu().numpy(), wv)
    np.testing.assert_array_equal(u16(l4), wl)


# ------------------------------------------------------------------ reassembly-size datagrams

@pytest.mark.parametrize("proto", [6, 17])
@pytest.mark.parametrize("kernel", ["auto", "fpw7"])
def test_ipv4_frag_max_datagrams(proto, kernel):
    """64512 B (PICO_IPV4_FRAG_MAX_SIZE) IPv4 datagrams, as pico_fragments_reassemble hands
    them on: TX compute + write, then RX verify accepts; both against the oracle, with a
    few corrupted datagrams and odd (Ethernet) header alignment."""
    use_kernel(kernel)
    n = 48
    lens = np.full(n, 64512, dtype=np.uint32)
    lens[::7] = 64511                              # odd lengths too
    buf, net_off, avail = synth.ipv4_batch(lens, seed=61 + proto, proto=proto, eth=True)
    desc_h = G.ipv4_desc(net_off, avail)
    want_tx = O.batch_ipv4(buf, desc_h, tx=True)
    d_buf, d_desc = to_dev(buf), batch.desc_to_device(desc_h, DEV)
    net, l4, v = batch.ipv4_checksum_batch(d_buf, d_desc, n, flags=batch.F_TX | batch.F_WRITE)
    np.testing.assert_array_equal(v.cpu().numpy(), want_tx[2])
    np.testing.assert_array_equal(u16(net), want_tx[0])
    np.testing.assert_array_equal(u16(l4), want_tx[1])
    h = d_buf.cpu().numpy()
    h[net_off[::5].astype(np.int64) + 1000] ^= 0x40
    want = O.batch_ipv4(h, desc_h, tx=False)
    net, l4, v = batch.ipv4_checksum_batch(to_dev(h), d_desc, n)
    np.testing.assert_array_equal(v.cpu().numpy(), want[2])
    np.testing.assert_array_equal(u16(net), want[0])
    np.testing.assert_array_equal(u16(l4), want[1])
    if proto == 6:      # UDP over IPv4 is sent with crc 0 (pico_udp.c:123): RX does not verify it
        assert (want[2][::5] != 1).all() and (np.delete(want[2], np.arange(0, n, 5)) == 1).all()
    else:
        assert (want[2] == 1).all()


def test_c2_full_size_tx_compute():
    """C2 compute mode at full size: 256K IMIX datagrams, TX checksums vs the oracle and the
    in-place writes byte-exact."""
    lens = synth.imix_lengths(262144, 77)
    buf, net_off, avail = synth.ipv4_batch(lens, seed=78, proto=6, eth=True)
    desc_h = G.ipv4_desc(net_off, avail)
    want = O.batch_ipv4(buf, desc_h, tx=True)
    d_buf, d_desc = to_dev(buf), batch.desc_to_device(desc_h, DEV)
    net, l4, v = batch.ipv4_checksum_batch(d_buf, d_desc, lens.size, flags=batch.F_TX | batch.F_WRITE)
    np.testing.assert_array_equal(v.cpu().numpy(), want[2])
    np.testing.assert_array_equal(u16(net), want[0])
    np.testing.assert_array_equal(u16(l4), want[1])
    wb = d_buf.cpu().numpy()
    ip = net_off.astype(np.int64)
    np.testing.assert_array_equal(wb[ip + 10], (want[0] >> 8).astype(np.uint8))
    np.testing.assert_array_equal(wb[ip + 11], (want[0] & 0xFF).astype(np.uint8))
    np.testing.assert_array_equal(wb[ip + 20 + 16], (want[1] >> 8).astype(np.uint8))
    np.testing.assert_array_equal(wb[ip + 20 + 17], (want[1] & 0xFF).astype(np.uint8))


@pytest.mark.parametrize("v6", [False, True])
def test_short_transports_every_alignment(v6):
    """Transports shorter than the field the reference reads (UDP tl < 8: the crc at 6-7 lies
    past the region; ICMPv6 tl 1-3), at every start alignment: the region sum must stop at the
    region's end even when the head window reads further (regression: r03 fuzz)."""
    rng = np.random.default_rng(606 + v6)
    parts, offs, avs, pos = [], [], [], 0
    for a in range(16):
        for tl in range(0, 12):
            for proto in ((17, 58, 6) if v6 else (17, 6)):
                hl = 40 if v6 else 20
                d = bytearray(rng.integers(0, 256, hl + max(tl, 8) + 8).astype(np.uint8).tobytes())
                if v6:
                    d[0], d[4], d[5], d[6], d[9] = 0x60, 0, tl, proto, proto
                else:
                    d[0], d[2], d[3], d[6], d[7], d[9] = 0x45, 0, hl + tl, 0x40, 0, proto
                    d[12] = 10
                    d[10:12] = b"\0\0"
                    c = O.checksum(bytes(d[:20]))
                    d[10], d[11] = c >> 8, c & 0xFF
                pos += (a - pos) % 16
                offs.append(pos)
                avs.append(len(d))
                parts.append((pos, bytes(d)))
                pos += len(d)
    buf = np.zeros(pos + 16, np.uint8)
    for o, d in parts:
        buf[o:o + len(d)] = np.frombuffer(d, np.uint8)
    desc = batch.make_desc(np.array(offs, np.uint64), np.array(avs, np.uint32))
    d_desc = batch.desc_to_device(desc, DEV)
    for fpw in (None, 1, 64):
        use_kernel("auto" if fpw is None else f"fpw{fpw}")
        if v6:
            wl, wv = O.batch_ipv6(buf, desc)
            l4, v = batch.ipv6_checksum_batch(to_dev(buf), d_desc, len(offs))
        else:
            wn, wl, wv = O.batch_ipv4(buf, desc)
            net, l4, v = batch.ipv4_checksum_batch(to_dev(buf), d_desc, len(offs))
            np.testing.assert_array_equal(u16(net), wn)
        np.testing.assert_array_equal(v.cpu().numpy(), wv, err_msg=f"fpw={fpw}")
        np.testing.assert_array_equal(u16(l4), wl, err_msg=f"fpw={fpw}")
    assert (wv == 4).sum() > 100

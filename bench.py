#!/usr/bin/env python3
"""bench.py -- device-resident checksummed GiB/s on MI355X (BASELINE.json metric).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config <one of the configs below>]
  torchrun --nproc-per-node N ... bench.py --gpus N      (one rank per GPU)

A step = one pass of the hot path over one batch resident in HBM:
  c1 (default, the metric's config): 256K x 1500 B frames, raw pico_checksum per frame
  c1_s1536: the same frames at stride 1536 (each on a 128 B line)
  c2: 256K simple-IMIX {64,576,1500} IPv4/TCP datagrams, fused header + pseudo-header RX verify
  c2slot: the same datagrams each in its own 2 KiB slot (a driver's slot ring), RX verify
  c2tx: the same datagrams, fused TX (checksums computed and written in place)
  c2tx_nw: fused TX computed and returned only (F_TX without F_WRITE: the driver's header write-out)
  c2nat: the same datagrams through the NAT batch (address / port rewrite + full checksum recompute)
  c2v6: 256K IMIX+20 B IPv6/TCP datagrams, fused IPv6 pseudo-header RX verify
  c2eth: the C2 frames through the Ethernet front end (one launch: ethertype dispatch + RX verify)
  c2ethmix: a mixed IPv4 / IPv6 Ethernet burst through the same front end
  c3_frag: 16K x 64512 B IPv4/TCP datagrams (reassembly maximum), fused RX verify
  c3_reasm: 4K x 64512 B datagrams reassembled from 1480 B fragments + TCP check in the same pass
  c3_reasm6: the same for IPv6 (1448 B fragments behind a fragment header)
  c3_reasm_il / _retx / _576: c3_reasm with the fragments interleaved across datagrams / a
      retransmitted fragment in every datagram / 552 B fragments (a 576 B MTU)
  c3: 256K x 9000 B jumbo frames;  c3_64k: 16K x 64 KiB reassembled buffers
  c4: 4M x 1500 B frames sharded over the ranks (strong scaling)
c1/c2/c3 are weak-scaled: every rank checksums its own batch of that size (frame batches
are independent shards; no collective touches the data path -- RCCL only carries the
barrier and the max-over-ranks timing).

Rank 0 prints ONE JSON line.  `verified` checks the outputs of the timed region against the CPU
oracle (every frame of the uniform configs, every datagram of the fused ones); any mismatch
makes the run exit non-zero.  `value` = the bytes of all ranks / the max over ranks of each
rank's timed region (from a common start barrier to its own device synchronize; the closing
barrier is outside it).  `roofline` is the checksum kernel's achieved algorithmic HBM
bandwidth (HIP events bracketing the K timed launches on the launch stream; elapsed / K =
average launch duration) against the 8.0 TB/s HBM3E peak; `traffic` is the PMC-measured HBM bytes per launch
from profiles/pmc_traffic.json (FETCH_SIZE x2, calibrated to 128 B per touched line by tools/fetch_calib.py,
+ WRITE_SIZE; separate rocprofv3 passes recorded earlier, named in `traffic_source`) when recorded for this config;
`cpu_baseline` times the reference's own pico_checksum (compiled from stack/pico_frame.c,
oracle/_ref) on the host cores over a bounded sample of the same frames.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from picotcp_amd import batch, synth  # noqa: E402
from picotcp_amd.shard import shard_range  # noqa: E402

METRIC = "device-resident checksummed GiB/s, 1500B-frame batches, 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec peak, GB/s (MI355X_MICROARCH.md)
GIB = float(1 << 30)

CONFIGS = {
    "c1": dict(kind="uniform", frames=262144, frame_bytes=1500,
               workload="C1: 256K x 1500 B (Ethernet MTU) frames, raw pico_checksum per frame, packed stride 1500"),
    "c1_s1536": dict(kind="uniform", frames=262144, frame_bytes=1500, stride=1536,
                     workload="C1, the aligned variant (SURVEY 8d): 256K x 1500 B frames at stride 1536 (every "
                              "frame on a 128 B line), raw pico_checksum per frame"),
    "c2": dict(kind="ipv4", frames=262144,
               workload="C2: 256K simple-IMIX {64,576,1500} B IPv4/TCP datagrams (14 B Ethernet header in front), "
                        "fused IPv4 header + TCP pseudo-header RX verify"),
    "c2slot": dict(kind="ipv4", frames=262144, slot=2048,
                   workload="C2 on a slot ring: the 256K simple-IMIX {64,576,1500} B IPv4/TCP datagrams each "
                            "in its own 2 KiB slot (14 B Ethernet header first), as a batching TAP driver lays "
                            "out a burst (modules/pico_dev_tap.c:63-75), fused IPv4 header + TCP pseudo-header "
                            "RX verify"),
    "c2v6": dict(kind="ipv6", frames=262144,
                 workload="C2 (IPv6, SURVEY 8f row 3): 256K simple-IMIX {64,576,1500}+20 B IPv6/TCP datagrams "
                          "(14 B Ethernet header in front), fused IPv6 pseudo-header TCP RX verify"),
    "c2tx": dict(kind="ipv4", frames=262144, tx=True,
                 workload="C2 compute mode: 256K simple-IMIX {64,576,1500} B IPv4/TCP datagrams, fused TX: IPv4 "
                          "header and TCP checksums computed with the crc fields read as zero and written in place"),
    "c2tx_nw": dict(kind="ipv4", frames=262144, tx=True, write=False,
                    workload="C2 compute-only TX: 256K simple-IMIX {64,576,1500} B IPv4/TCP datagrams, IPv4 header "
                             "and TCP checksums computed with the crc fields read as zero and returned (F_TX "
                             "without F_WRITE: the driver writes them with its headers)"),
    "c2nat": dict(kind="ipv4", frames=262144, nat=True,
                  workload="C2 NAT (SURVEY 8f row 4): 256K simple-IMIX {64,576,1500} B IPv4/TCP datagrams, "
                           "pico_ipv4_nat_outbound / _inbound's frame work per record (address + port rewritten, "
                           "TCP and IPv4 header checksums recomputed over the whole datagram, all in place)"),
    "c3_frag": dict(kind="ipv4", frames=16384, frame_bytes=64512,
                    workload="C3 reassembled: 16K x 64512 B (PICO_IPV4_FRAG_MAX_SIZE) IPv4/TCP datagrams, fused "
                             "IPv4 header + TCP pseudo-header RX verify"),
    "c2eth": dict(kind="eth", frames=262144,
                  workload="C2 through the Ethernet front end (SURVEY 8f row 1): the 256K simple-IMIX IPv4/TCP "
                           "frames, descriptors at the Ethernet header, ethertype dispatch + destination-MAC filter "
                           "+ fused IPv4 / TCP RX verify in one launch"),
    "c2ethmix": dict(kind="eth", frames=262144, mix=True,
                     workload="C2 as a mixed Ethernet burst (SURVEY 8f rows 1 and 3): 256K frames, IPv4/TCP "
                              "(simple IMIX {64,576,1500} B) and IPv6/TCP (IMIX + 20 B) in seeded random order "
                              "back to back, one launch: ethertype dispatch + destination-MAC filter + fused "
                              "IPv4 / IPv6 / TCP RX verify"),
    "c3_reasm": dict(kind="frag", frames=4096, frame_bytes=64512,
                     workload="C3 reassembly (SURVEY 8f row 4): 4K x 64512 B IPv4/TCP datagrams arriving as 1480 B "
                              "fragments (44 per datagram, 14 B Ethernet gap each), gathered into reassembled "
                              "buffers with the TCP pseudo-header check of each datagram in the same pass"),
    "c3_reasm6": dict(kind="frag", frames=4096, frame_bytes=64512, v6=True,
                      workload="C3 reassembly, IPv6 (SURVEY 8f row 4): 4K x 64512 B IPv6/TCP datagrams arriving as "
                               "1448 B fragments (45 per datagram, 40 B header + 8 B fragment header, 14 B Ethernet "
                               "gap each), each fragment's extension headers walked, gathered into reassembled "
                               "buffers with the TCP pseudo-header check of each datagram in the same pass"),
    "c3_reasm_il": dict(kind="frag", frames=4096, frame_bytes=64512, interleave=True,
                        workload="C3 reassembly, fragments of the 4K datagrams interleaved as a NIC receives "
                                 "concurrent flows (fragment k of every datagram, then k + 1, ...), otherwise as "
                                 "c3_reasm"),
    "c3_reasm_576": dict(kind="frag", frames=4096, frame_bytes=64512, frag_payload=552,
                         workload="C3 reassembly over a 576 B MTU: 4K x 64512 B IPv4/TCP datagrams arriving as 552 B "
                                  "fragments (117 per datagram: past the flat grid's 64 a wave, one workgroup per "
                                  "datagram), otherwise as c3_reasm"),
    "c3_reasm_retx": dict(kind="frag", frames=4096, frame_bytes=64512, retx=True,
                          workload="C3 reassembly with retransmissions: as c3_reasm, every datagram's middle "
                                   "fragment arriving a second time, last (45 fragments, one repeated offset each)"),
    "c3": dict(kind="uniform", frames=262144, frame_bytes=9000,
               workload="C3: 256K x 9000 B jumbo frames, raw pico_checksum per frame"),
    "c3_64k": dict(kind="uniform", frames=16384, frame_bytes=65536,
                   workload="C3: 16K x 64 KiB reassembled-fragment buffers, raw pico_checksum per buffer"),
    "c4": dict(kind="uniform", frames=4194304, frame_bytes=1500, strong=True,
               workload="C4: 4M x 1500 B frames sharded contiguously over the ranks (strong scaling)"),
}


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=200)
    p.add_argument("--warmup", type=int, default=20)
    p.add_argument("--config", default="c1", choices=sorted(CONFIGS))
    p.add_argument("--rotate", type=int, default=0, help="rotating batch copies (0 = enough for >= 1 GiB)")
    p.add_argument("--cpu-seconds", type=float, default=4.0, help="target CPU-baseline wall per leg")
    p.add_argument("--no-cpu", action="store_true")
    p.add_argument("--no-e2e", action="store_true")
    p.add_argument("--no-verify", action="store_true", help="skip the parity check of the timed outputs")
    p.add_argument("--shape", default="", help="G,CPL,FPW,U,NT launch override (sweeps)")
    p.add_argument("--stream", default="", help="MODE,FPW the uniform rings' stream waves "
                                                  "(pico_csum_set_uniform_stream: 1 on, 255 off; frames per wave)")
    p.add_argument("--reasm-flat", type=int, default=0,
                   help="reassembly grid (pico_csum_set_reasm_flat: 0 auto, 1 flat, 2 one workgroup per datagram)")
    p.add_argument("--no-graph", action="store_true",
                   help="launch the K timed steps one by one from Python instead of replaying them as one "
                        "captured HIP graph")
    return p.parse_args()


def make_uniform(n, ln, device, seed):
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    nbytes = n * ln
    return torch.randint(0, 256, (nbytes,), dtype=torch.uint8, device=device, generator=g)


IMIX_MEAN = 354          # simple-IMIX mean datagram length (7:4:1 of 64/576/1500 B)


def rotation(batch_bytes: int) -> int:
    """Batch copies to rotate so that >= 1 GiB lies between two uses of one batch: the
    256 MiB Infinity Cache then cannot serve a repeat (MI355X_MICROARCH.md, L3)."""
    return max(3, -(-(1 << 30) // max(1, batch_bytes)))


def make_c2(n, device, seed, frame_bytes=0, keep_host=True, slot=0):
    lens = synth.imix_lengths(n, seed) if not frame_bytes else np.full(n, frame_bytes, dtype=np.uint32)
    buf, net, avail = synth.ipv4_batch(lens, seed=seed + 1, proto=6, eth=True, slot=slot)
    desc = batch.make_desc(net, avail)
    d_buf = torch.from_numpy(buf).to(device)
    d_desc = batch.desc_to_device(desc, device)
    # make every datagram valid with the TX kernel (untimed setup), so RX verify accepts
    batch.ipv4_checksum_batch(d_buf, d_desc, n, flags=batch.F_TX | batch.F_WRITE)
    torch.cuda.synchronize(device)
    # the host copy is the batch as the timed steps see it (valid checksums), for the CPU leg
    return d_buf, d_desc, int(lens.sum()), (d_buf.cpu().numpy(), desc) if keep_host else None


def make_c2v6(n, device, seed, keep_host=True):
    lens = (synth.imix_lengths(n, seed) + 20).astype(np.uint32)
    buf, net, avail, seeds = synth.ipv6_batch(lens, seed=seed + 1, proto=6, eth=True)
    desc = batch.make_desc(net, avail, seeds)
    d_buf = torch.from_numpy(buf).to(device)
    d_desc = batch.desc_to_device(desc, device)
    batch.ipv6_checksum_batch(d_buf, d_desc, n, flags=batch.F_TX | batch.F_WRITE)
    torch.cuda.synchronize(device)
    return d_buf, d_desc, int(lens.sum()), (d_buf.cpu().numpy(), desc) if keep_host else None


MAC = bytes.fromhex("02005e0a0b0c")


def make_c2eth(n, device, seed, keep_host=True, mix=False):
    """The C2 datagrams as Ethernet frames addressed to MAC (descriptors at the frame start); mix:
    IPv4 and IPv6 (IMIX + 20 B) frames in seeded random order, back to back."""
    lens = synth.imix_lengths(n, seed)
    buf, net, avail = synth.ipv4_batch(lens, seed=seed + 1, proto=6, eth=True)
    if mix:
        b6, n6, a6, _ = synth.ipv6_batch((lens + 20).astype(np.uint32), seed=seed + 2, proto=6, eth=True)
        kinds = np.random.default_rng(seed).integers(0, 2, n)
        buf, st, fl = synth.interleave([(buf, net - np.uint64(14), avail + 14), (b6, n6 - np.uint64(14), a6 + 14)],
                                       kinds)
        net, avail = st + np.uint64(14), fl - 14
        lens = avail
    e = net.astype(np.int64) - 14
    for k, b in enumerate(MAC):
        buf[e + k] = b
    desc = batch.make_desc(net - np.uint64(14), avail + 14)
    d_buf = torch.from_numpy(buf).to(device)
    d_desc = batch.desc_to_device(desc, device)
    batch.eth_checksum_batch(d_buf, d_desc, n, flags=batch.F_TX | batch.F_WRITE)
    torch.cuda.synchronize(device)
    return d_buf, d_desc, int(lens.sum()) + 14 * n, (d_buf.cpu().numpy(), desc) if keep_host else None


FRAG = 1480                 # IPv4 fragment payload (MTU 1500 - 20 B header)
FRAG6 = 1448                # IPv6 fragment payload (MTU 1500 - 40 B header - 8 B fragment header, 8-aligned)


def make_frag(n, tl, device, seed, v6=False, interleave=False, frag_payload=0, retx=False):
    """n IPv4/TCP (IPv6/TCP) datagrams of tl transport bytes as in-order 1480 B (1448 B)
    fragments (frag_payload: another payload size, a multiple of 8), each behind a 14 B gap, built
    on the device (vectorized); the TCP checksum made valid with one untimed reassembly pass.
    retx: every datagram's middle fragment arrives a second time, last (a retransmission: the same
    bytes, a repeated offset the reference's fragment tree rejects).
    Returns (buffer, fragment descriptors, groups, out, out descriptors, fragment count, payload
    bytes)."""
    fr, hl = (FRAG6, 48) if v6 else (FRAG, 20)
    if frag_payload:
        fr = frag_payload
    nf = -(-tl // fr)
    pl = np.full(nf, fr, np.int64)
    pl[-1] = tl - fr * (nf - 1)
    fsz = 14 + hl + pl                                   # bytes per fragment slot
    per = int(fsz.sum())
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    buf = torch.randint(0, 256, (n * per,), dtype=torch.uint8, device=device, generator=g)
    rel = np.concatenate([[0], np.cumsum(fsz)[:-1]]) + 14          # header offsets in one datagram
    net = (np.arange(n, dtype=np.int64)[:, None] * per + rel[None, :]).reshape(-1)
    if interleave:     # arrival order fragment-major: fragment k of datagrams 0..n-1, then k + 1
        kstart = np.concatenate([[0], np.cumsum(fsz * n)[:-1]])     # where fragment k's run starts
        net = (kstart[None, :] + np.arange(n, dtype=np.int64)[:, None] * fsz[None, :] + 14).reshape(-1)
    hdr = np.zeros((n, nf, hl), np.uint8)
    tot = hl + pl
    if v6:
        plen = 8 + pl
        hdr[:, :, 0] = 0x60
        hdr[:, :, 4], hdr[:, :, 5] = (plen >> 8)[None, :], (plen & 0xFF)[None, :]
        hdr[:, :, 6], hdr[:, :, 7] = 44, 64
        hdr[:, :, 8:24] = [0x20, 6, 0x0d, 0xb8, 0, 0, 0, 1, 0, 0, 0, 0, 0, 0, 0, 1]   # byte 9 = 6 (TCP)
        hdr[:, :, 24:40] = [0x20, 1, 0x0d, 0xb8, 0, 0, 0, 2, 0, 0, 0, 0, 0, 0, 0, 2]
        om = np.arange(nf) * fr | np.where(np.arange(nf) < nf - 1, 1, 0)
        hdr[:, :, 40], hdr[:, :, 42], hdr[:, :, 43] = 6, (om >> 8)[None, :], (om & 0xFF)[None, :]
        ident = np.arange(n, dtype=np.int64) * 7 + seed
        for k in range(4):
            hdr[:, :, 44 + k] = ((ident >> (24 - 8 * k)) & 0xFF)[:, None]
    else:
        hdr[:, :, 0] = 0x45
        hdr[:, :, 2], hdr[:, :, 3] = (tot >> 8)[None, :], (tot & 0xFF)[None, :]
        ident = (np.arange(n) * 7 + seed) & 0xFFFF
        hdr[:, :, 4], hdr[:, :, 5] = (ident >> 8)[:, None], (ident & 0xFF)[:, None]
        frag = ((np.arange(nf) * fr) >> 3) | np.where(np.arange(nf) < nf - 1, 0x2000, 0)
        hdr[:, :, 6], hdr[:, :, 7] = (frag >> 8)[None, :], (frag & 0xFF)[None, :]
        hdr[:, :, 8], hdr[:, :, 9] = 64, 6
        hdr[:, :, 12:16] = [10, 1, 2, 3]
        hdr[:, :, 16:20] = [192, 168, 4, 5]
    idx = torch.from_numpy((net[:, None] + np.arange(hl)[None, :]).reshape(-1)).to(device)
    buf[idx] = torch.from_numpy(hdr.reshape(-1)).to(device)
    crc = torch.from_numpy(np.stack([net[::nf] + hl + 16, net[::nf] + hl + 17], 1).reshape(-1)).to(device)
    buf[crc] = 0                                         # TCP crc of each datagram (first fragment)
    flen = np.repeat(tot[None, :], n, 0)
    if retx:                                             # + fragment nf // 2 again, last
        net2 = np.concatenate([net.reshape(n, nf), net.reshape(n, nf)[:, nf // 2:nf // 2 + 1]], 1).reshape(-1)
        flen = np.concatenate([flen, flen[:, nf // 2:nf // 2 + 1]], 1)
        desc = batch.make_desc(net2.astype(np.uint64), flen.reshape(-1))
        grp = np.stack([np.arange(n) * (nf + 1), np.full(n, nf + 1)], 1).astype(np.uint32).reshape(-1)
    else:
        desc = batch.make_desc(net.astype(np.uint64), flen.reshape(-1))
        grp = np.stack([np.arange(n) * nf, np.full(n, nf)], 1).astype(np.uint32).reshape(-1)
    H = 40 if v6 else 20
    cap = (H + tl + 15) // 16 * 16 + 16
    # each reassembled datagram at (16 - H % 16) mod 16, so that its transport (behind the H B
    # header) is 16-byte aligned: the gather then stores whole 16-byte units
    od = batch.make_desc(np.arange(n, dtype=np.uint64) * cap + np.uint64(8 if v6 else 12), np.full(n, cap - 12))
    d_desc, d_od = batch.desc_to_device(desc, device), batch.desc_to_device(od, device)
    d_grp = torch.from_numpy(grp.view(np.int32)).to(device)
    out = torch.empty(n * cap, dtype=torch.uint8, device=device)
    fn = batch.ipv6_reassemble_batch if v6 else batch.ipv4_reassemble_batch
    nfr = n * (nf + 1) if retx else n * nf
    _, l4, _ = fn(buf, d_desc, nfr, d_grp, out, d_od)
    c = l4.view(torch.int16).to(torch.int32) & 0xFFFF                # value to store: short_be(c)
    buf[crc[0::2]] = (c >> 8).to(torch.uint8)
    buf[crc[1::2]] = (c & 0xFF).to(torch.uint8)
    torch.cuda.synchronize(device)
    return buf, d_desc, d_grp, out, d_od, nfr, n * tl


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return os.uname().machine


def cpu_threads() -> tuple[int, int]:
    """(threads used, usable cores).  The GPU box gives one GPU's job a 16-core share of
    the host (OMP_NUM_THREADS=16 there; sched_getaffinity shows the whole machine, whose
    other cores run other jobs, and the box's rules size worker pools to that share), so
    the multi-thread leg runs on that share, capped at the usable cores."""
    cores = len(os.sched_getaffinity(0))
    return max(1, min(cores, int(os.environ.get("OMP_NUM_THREADS", cores)))), cores


def cgroup_cpu() -> str | None:
    """The CPU quota of this job's cgroup (cgroup v2 cpu.max: "<quota> <period>" or "max ...")."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            return f.read().strip()
    except OSError:
        return None


def cpu_baseline(sample: np.ndarray, ln: int, target_s: float, stride: int = 0):
    """The reference's pico_checksum (oracle/_ref: stack/pico_frame.c built -O3 = the
    reference's PERF=1, and -Os = its release default) over a bounded sample of the same
    frames, on 1 thread and on the job's host-core share."""
    from oracle import oracle as O
    kind = "reference" if O.ref_available() else "port"
    stride = stride or ln
    n = (sample.size - ln) // stride + 1
    threads, cores = cpu_threads()
    res = {}
    legs = [(1, False), (threads, False)]
    if kind == "reference" and O.ref_available(os_flags=True):
        legs += [(1, True), (threads, True)]
    for t, osf in legs:
        secs, _ = O.uniform_mt(sample, stride, ln, n, t, kind=kind, os_flags=osf)   # page-in / warm
        reps = max(1, int(target_s / max(secs, 1e-3)))
        tot = 0.0
        for _ in range(reps):
            secs, _ = O.uniform_mt(sample, stride, ln, n, t, kind=kind, os_flags=osf)
            tot += secs
        res[(t, osf)] = (n * ln * reps / tot / GIB, reps)
    out = {
        "value": round(res[(threads, False)][0], 3), "unit": "GiB/s", "cores": threads, "kind": kind,
        "single_core_value": round(res[(1, False)][0], 3),
        "sample": f"{n} x {ln} B frames{f' at stride {stride}' if stride != ln else ''} ({n * ln / 2**20:.0f} MiB, "
                  f"DRAM-resident), reference stack/pico_frame.c "
                  f"pico_checksum built -O3 (PERF=1), pthreads over contiguous frame ranges; "
                  f"{res[(threads, False)][1]} passes on {threads} threads, {res[(1, False)][1]} on 1 thread",
        "cpu_model": cpu_model(), "usable_cores": cores, "cgroup_cpu_max": cgroup_cpu(),
        "share": f"{threads} threads = the host share the GPU box grants one GPU's job (OMP_NUM_THREADS); "
                 f"sched_getaffinity shows {cores} cores of a machine other jobs share",
    }
    if (1, True) in res:
        out["Os_value"] = round(res[(threads, True)][0], 3)
        out["Os_single_core_value"] = round(res[(1, True)][0], 3)
    return out


def cpu_baseline_fused(host, kind: str, tx: bool, target_s: float, nat=None):
    """The reference's own per-datagram work on the host cores: oracle/_ref/libref_callers.so
    (rc_batch_mt over the compiled reference modules: pico_checksum of the IPv4 header +
    pico_tcp_checksum_ipv4 / _ipv6, f->sock NULL on RX; TX zeroes the crc fields, computes with a
    socket carrying the header's addresses and stores both, as tcp_send + pico_ipv4_frame_push do;
    the Ethernet burst by ethertype) over the batch as the timed steps see it, on 1 thread and on
    the job's host-core share.  Where that library is absent (or for NAT, which has no single
    reference entry point), the oracle's fused restatement on 1 thread (kind "port")."""
    from oracle import oracle as O
    buf, desc = host
    threads, cores = cpu_threads()
    if nat is None and O.ref_callers_available():
        mode = {"ipv4": O.RC_TX4 if tx else O.RC_RX4, "ipv6": O.RC_RX6, "eth": O.RC_ETH}[kind]
        if not (tx and kind != "ipv4"):
            nbytes = int(desc["len"].astype(np.int64).sum())
            work = buf.copy() if tx else buf
            res = {}
            for t in (1, threads):
                secs, on, ol = O.ref_callers_batch(work, desc, mode, t)        # page-in / warm
                reps = max(1, int(target_s / max(secs, 1e-3)))
                tot = 0.0
                for _ in range(reps):
                    secs, on, ol = O.ref_callers_batch(work, desc, mode, t)
                    tot += secs
                res[t] = (nbytes * reps / tot / GIB, reps)
            # the reference's values on this batch: every datagram is valid, so an RX pass gives 0 / 0
            ok = int(((on == 0) & (ol == 0)).sum()) if not tx else None
            what = {"ipv4": "IPv4 TX (crc fields zeroed, pico_tcp_checksum_ipv4 + pico_checksum of the header, stored)"
                    if tx else "IPv4 RX (pico_checksum of the header + pico_tcp_checksum_ipv4)",
                    "ipv6": "IPv6 RX (pico_tcp_checksum_ipv6)",
                    "eth": "Ethernet burst RX (ethertype, then the IPv4 / IPv6 RX work)"}[kind]
            out = {"value": round(res[threads][0], 3), "unit": "GiB/s", "cores": threads, "kind": "reference",
                   "single_core_value": round(res[1][0], 3),
                   "sample": f"all {desc.size} datagrams of the batch ({nbytes / 2**20:.0f} MiB), the reference's "
                             f"compiled modules (oracle/_ref/libref_callers.so, gcc -O3), {what}, a struct pico_frame "
                             f"per thread on the datagram in place; {res[threads][1]} passes on {threads} threads, "
                             f"{res[1][1]} on 1 thread",
                   "cpu_model": cpu_model(), "usable_cores": cores, "cgroup_cpu_max": cgroup_cpu()}
            if ok is not None:
                out["reference_accepts"] = ok
            return out
    k = min(desc.size, 65536)
    sample, nbytes = desc[:k], int(desc["len"][:k].astype(np.int64).sum())
    fn = {"ipv6": lambda: O.batch_ipv6(buf, sample, tx=tx), "ipv4": lambda: O.batch_ipv4(buf, sample, tx=tx),
          "eth": lambda: O.batch_eth(buf, sample, mac=MAC, tx=tx)}[kind]
    if nat is not None:                                  # in place on a copy (idempotent: same records)
        nbuf = buf.copy()
        fn = lambda: O.batch_ipv4_nat(nbuf, sample, nat[:k])  # noqa: E731
    t0 = time.perf_counter()
    fn()
    reps = max(1, int(target_s / max(time.perf_counter() - t0, 1e-3)))
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    dt = (time.perf_counter() - t0) / reps
    return {"value": round(nbytes / dt / GIB, 3), "unit": "GiB/s", "cores": 1, "kind": "port",
            "sample": f"first {k} datagrams of the batch ({nbytes / 2**20:.0f} MiB), oracle "
                      + ("NAT restatement (oracle_batch_ipv4_nat: rewrite + full recompute, as pico_nat.c)"
                         if nat is not None else
                         f"fused { {'ipv6': 'IPv6', 'ipv4': 'IPv4', 'eth': 'Ethernet + IPv4/IPv6'}[kind]} "
                         f"{'TX' if tx else 'RX'} restatement")
                      + f", gcc -O3, 1 thread, {reps} passes"}


def cpu_baseline_frag(st, target_s: float, v6: bool = False):
    """The reference's own fragment path on 1 host core over the first 256 datagrams of the batch:
    oracle/_ref/libref_rx_O3.so (the reference stack at -O3; rr_reasm_batch: every fragment into a
    frame of its own, pico_ipv4_process_in / pico_ipv6_extension_headers, pico_ipv4/6_process_frag,
    pico_fragments_reassemble, pico_transport_crc_check on the datagram handed on, a
    pico_stack_tick per datagram; the stack is not thread-safe, hence one thread).  The IPv4
    fragments' header checksums (zero in the synthetic batch, which the kernels do not check)
    are filled in on the host copy first, as pico_ipv4_process_in drops a bad one.  Without the
    reference build: the oracle's restatement (kind "port")."""
    from oracle import oracle as O
    fn = O.ipv6_reassemble if v6 else O.ipv4_reassemble
    b, d, gr, o, od, nfr, payload = st
    n = gr.numel() // 2
    k = min(n, 256)
    grp = gr.cpu().numpy().view(np.uint32)[:2 * k]
    nf_used = int(grp[-2] + grp[-1])
    desc = d.cpu().numpy().view(batch.DESC_DTYPE)[:nf_used]
    hi = int((desc["off"] + desc["len"].astype(np.uint64)).max())   # (retx: the last descriptor is a repeat)
    host = b[:hi].cpu().numpy()
    nbytes = payload // n * k
    if O.ref_reasm_available():
        host = host.copy()
        offs = desc["off"].astype(np.uint64)
        if not v6:
            O.fix_ipv4_header_crcs(host, offs)
        o0 = int(offs[0])
        O.ref_reasm_link(v6, bytes(host[o0 + 24:o0 + 40]) if v6 else bytes(host[o0 + 16:o0 + 20]))
        secs, done, chk = O.ref_reasm_batch(v6, host, offs, desc["len"], grp)      # (warm)
        reps = max(3, int(target_s / max(secs, 1e-3)))
        times = []
        for _ in range(reps):
            secs, done, chk = O.ref_reasm_batch(v6, host, offs, desc["len"], grp)
            times.append(secs)
        dt = float(np.median(times))
        return {"value": round(nbytes / dt / GIB, 3), "unit": "GiB/s", "cores": 1, "kind": "reference",
                "sample": f"first {k} datagrams ({nbytes / 2**20:.0f} MiB of payload, {nf_used} fragments), the "
                          f"reference's {'IPv6' if v6 else 'IPv4'} fragment path (oracle/_ref/libref_rx_O3.so "
                          f"rr_reasm_batch: frame per fragment, {'pico_ipv6_extension_headers' if v6 else 'pico_ipv4_process_in'}, "
                          f"pico_fragments_reassemble, pico_transport_crc_check), gcc -O3, 1 thread (the stack is "
                          f"not thread-safe), median of {reps} passes; {done} reassembled, {chk} transport checks "
                          f"passed"}
    odh = od.cpu().numpy().view(batch.DESC_DTYPE)[:k]
    outh = np.zeros(int(odh["off"][-1]) + int(odh["len"][-1]), np.uint8)
    t0 = time.perf_counter()
    fn(host, desc, grp, outh, odh)
    reps = max(1, int(target_s / max(time.perf_counter() - t0, 1e-3)))
    t0 = time.perf_counter()
    for _ in range(reps):
        fn(host, desc, grp, outh, odh)
    dt = (time.perf_counter() - t0) / reps
    return {"value": round(nbytes / dt / GIB, 3), "unit": "GiB/s", "cores": 1, "kind": "port",
            "sample": f"first {k} datagrams ({nbytes / 2**20:.0f} MiB of payload), oracle {'IPv6' if v6 else 'IPv4'} "
                      f"reassembly restatement (sort, memcpy gather, pico_checksum of the transport), gcc -O3, "
                      f"1 thread, {reps} passes"}


def verify(kind: str, cfg: dict, slot, out, host, threads: int) -> dict:
    """Parity evidence carried by the bench line itself: the outputs the timed region produced
    for rotation slot 0 against the CPU oracle (oracle/pico_csum_oracle.c, the checker; never
    the measured path).  uniform: every frame of the batch (the restatement on `threads`
    pthreads); fused IPv4 / IPv6 / Ethernet: every datagram, on the device buffer as the timed
    steps left it (TX: the values and the crc fields written in place); reassembly: every
    datagram (lengths, checksums, verdicts and the reassembled bytes)."""
    from oracle import oracle as O
    t0 = time.perf_counter()
    if kind == "uniform":
        b, ln, n = slot
        stride = cfg.get("stride", ln)
        hb = b.cpu().numpy()
        _, want = O.uniform_mt(hb, stride, ln, n, threads, kind="port")
        got = out.cpu().numpy().view(np.uint16)
        frames, bad = n, int((got != want).sum())
        what = f"every frame, oracle_checksum on {threads} threads"
    elif kind == "frag":
        b, d, gr, o, od, nfr, payload = slot
        n = gr.numel() // 2
        k = n
        grp = gr.cpu().numpy().view(np.uint32)[:2 * k]
        nf_used = int(grp[-2] + grp[-1])
        desc = d.cpu().numpy().view(batch.DESC_DTYPE)[:nf_used]
        hi = int((desc["off"] + desc["len"].astype(np.uint64)).max())     # (retx: the last descriptor is a repeat)
        odh = od.cpu().numpy().view(batch.DESC_DTYPE)[:k]
        outh = np.zeros(int(odh["off"][-1]) + int(odh["len"][-1]), np.uint8)
        v6 = bool(cfg.get("v6"))
        H = 40 if v6 else 20
        wl, wl4, wv = (O.ipv6_reassemble if v6 else O.ipv4_reassemble)(b[:hi].cpu().numpy(), desc, grp, outh, odh)
        gl, gl4, gv = (x.cpu().numpy()[:k] for x in out)
        gout = o[:outh.size].cpu().numpy()
        bad = int(((gl.view(np.uint32) != wl) | (gl4.view(np.uint16) != wl4) | (gv != wv)).sum())
        for g in range(k):
            if wl[g]:
                a = int(odh["off"][g])
                bad += int(not np.array_equal(gout[a:a + H + int(wl[g])], outh[a:a + H + int(wl[g])]))
        frames = k
        what = (f"every datagram ({k}): lengths, checksums, verdicts and reassembled bytes vs "
                f"oracle_ipv{6 if v6 else 4}_reassemble")
    else:
        b, d = slot[0], slot[1]
        hbuf, hdesc = host
        tx = bool(cfg.get("tx"))
        now = b.cpu().numpy()
        src = hbuf if tx else now                   # TX: the pre-write bytes are the input
        nat_bytes = None
        if kind == "ipv4" and cfg.get("nat"):
            after = cfg["_nat_before"].copy()
            want = O.batch_ipv4_nat(after, hdesc, cfg["_nat_host"])
            nat_bytes = int((now != after).sum())
        elif kind == "ipv4":
            want = O.batch_ipv4(src, hdesc, tx=tx)
        elif kind == "eth":
            want = O.batch_eth(src, hdesc, mac=MAC, tx=tx)
        else:
            want = O.batch_ipv6(src, hdesc, tx=tx)
        got = [x.cpu().numpy() for x in out]
        if kind == "ipv6":
            got = [got[0].view(np.uint16), got[1]]
        else:
            got = [got[0].view(np.uint16), got[1].view(np.uint16), got[2]]
        miss = np.zeros(hdesc.size, bool)
        for g_, w_ in zip(got, want):
            miss |= g_ != w_
        frames, bad = int(hdesc.size), int(miss.sum())
        if nat_bytes is not None:
            bad += int(nat_bytes > 0)
        if tx and cfg.get("write", True):           # the in-place writes: oracle RX on them accepts
            rx = O.batch_ipv4(now, hdesc) if kind == "ipv4" else None
            if rx is not None:
                bad += int(((want[2] == 1) & (rx[2] != 1)).sum())
        what = f"every datagram vs the oracle's fused {kind} {'TX' if tx else 'RX'} restatement" + \
            (" (+ RX of the written bytes)" if tx and kind == "ipv4" and cfg.get("write", True) else "")
        if nat_bytes is not None:
            what = "every datagram vs oracle_batch_ipv4_nat: checksums, verdicts and every byte of the rewritten batch"
    return {"frames": frames, "mismatches": bad, "checker": what, "seconds": round(time.perf_counter() - t0, 2)}


def seq_copy_lib():
    """tools/bin/libgather_ceiling.so (a measurement aid built by __graft_entry__.build(), never the
    product): its seq_copy_launch is the hand-written sequential copy the reassembly is priced
    against.  None when it is not built."""
    path = os.path.join(ROOT, "tools", "bin", "libgather_ceiling.so")
    if not os.path.exists(path):
        return None
    lib = ctypes.CDLL(path)
    lib.seq_copy_launch.restype = ctypes.c_int
    lib.seq_copy_launch.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p,
                                    ctypes.c_uint64, ctypes.c_void_p]
    return lib


# (variant, units per lane, workgroups): 0 non-temporal loads + stores, 1 cached, 2 nt loads + cached
# stores; workgroups 0 = one trip each, else a striding grid (8192 = 32 per CU)
SEQ_COPY_SHAPES = ((0, 4, 0), (0, 8, 0), (1, 4, 0), (2, 4, 0), (0, 4, 8192), (2, 8, 8192))
# the same copy with its loads 2 bytes off the 16-byte grid (as the reassembly's payload loads), reported
# beside the ceiling, not as it: 3 cached loads + stores, 4 nt loads + cached stores, 5 cached loads + nt
# stores (the reassembly's policy)
SEQ_COPY_UNALIGNED = ((3, 4, 0), (4, 4, 0), (5, 4, 0))


def copy_ceiling(nbytes: int, dev) -> dict:
    """The device's own contiguous copy of the payload bytes the reassembly moves (read + write),
    timed the same way: the practical ceiling of a gather.  A hand-written 16-byte-per-lane copy
    (tools/gather_ceiling.hip seq_copy, several shapes, the fastest reported); torch copy_ beside it."""
    nbytes &= ~15
    rot = max(3, -(-(1 << 30) // nbytes))
    src = [torch.empty(nbytes, dtype=torch.uint8, device=dev) for _ in range(rot)]
    dst = [torch.empty(nbytes, dtype=torch.uint8, device=dev) for _ in range(rot)]
    stream = torch.cuda.current_stream(dev)
    lib = seq_copy_lib()

    def timed(f, k=30):
        for i in range(5):
            f(i)
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ev0.record(stream)
        for i in range(k):
            f(i)
        ev1.record(stream)
        torch.cuda.synchronize(dev)
        return ev0.elapsed_time(ev1) / k * 1e3

    shapes = {}
    if lib is not None:
        h = ctypes.c_void_p(stream.cuda_stream)
        for var, u, blocks in SEQ_COPY_SHAPES:
            def f(i, var=var, u=u, blocks=blocks):
                assert lib.seq_copy_launch(var, u, blocks, dst[i % rot].data_ptr(), src[i % rot].data_ptr(), nbytes, h) == 0
            shapes[f"v{var}_u{u}_g{blocks}"] = round(timed(f), 2)
    unal = {}
    if lib is not None:
        for var, u, blocks in SEQ_COPY_UNALIGNED:
            def f(i, var=var, u=u, blocks=blocks):
                assert lib.seq_copy_launch(var, u, blocks, dst[i % rot].data_ptr(), src[i % rot].data_ptr(), nbytes, h) == 0
            unal[f"v{var}_u{u}_g{blocks}"] = round(timed(f), 2)
    torch_us = timed(lambda i: dst[i % rot].copy_(src[i % rot]))
    if shapes:
        best = min(shapes, key=shapes.get)
        us = shapes[best]
        what = (f"hand-written 16 B/lane copy (tools/gather_ceiling.hip seq_copy, fastest of {len(shapes)} shapes: "
                f"{best}) of {nbytes} B (read + write), {rot} rotating buffers, HIP events")
    else:
        us = torch_us
        what = f"torch copy_ of {nbytes} B (read + write), {rot} rotating buffers, HIP events (seq_copy not built)"
    return {"copy_us": round(us, 2), "copy_GBs": round(2 * nbytes / us / 1e3, 1), "what": what,
            "shapes_us": shapes, "unaligned_source_us": unal, "torch_copy_us": round(torch_us, 2)}


def e2e_rate_desc(host):
    """Host-resident fused IPv4 path (pico_ipv4_checksum_batch_host) on the C2 burst in pinned host
    memory, the caller's descriptors and result arrays in pageable memory.  The default routes a
    device-addressable burst in place (the kernel reads it over PCIe through its device alias; only
    descriptors and results staged); `staged` forces the staged path (chunked H2D of the span ->
    fused kernel -> D2H of the results, 32 MiB chunks, three slots).  Three warm calls before the
    five timed ones, each path."""
    buf, desc = host
    pinned = torch.from_numpy(buf).pin_memory()
    hb = batch.HostBatch(torch.cuda.current_device(), staging_bytes=32 << 20)
    nbytes = int(desc["len"].astype(np.int64).sum())
    n = int(desc.size)
    # a driver's pinned rings: descriptors and result arrays page-locked too
    kd = torch.from_numpy(np.ascontiguousarray(desc).view(np.uint8).copy()).pin_memory()
    pdesc = kd.numpy().view(batch.DESC_DTYPE)
    kout = [torch.empty(n, dtype=dt).pin_memory() for dt in (torch.int16, torch.int16, torch.uint8)]
    pout = (kout[0].numpy().view(np.uint16), kout[1].numpy().view(np.uint16), kout[2].numpy())

    def rate(in_place, d, out):
        batch.set_host_in_place(in_place)
        try:
            for _ in range(3):
                hb.ipv4_checksum_batch(pinned.numpy(), d, out=out)
            reps = 5
            t0 = time.perf_counter()
            for _ in range(reps):
                hb.ipv4_checksum_batch(pinned.numpy(), d, out=out)
            return nbytes / ((time.perf_counter() - t0) / reps) / GIB
        finally:
            batch.set_host_in_place(True)
    try:
        rings = rate(True, pdesc, pout)
        in_place = rate(True, desc, None)
        staged = rate(False, desc, None)
    finally:
        hb.close()
    return {"value": round(staged, 3), "unit": "GiB/s", "datagrams": n,
            "path": "pico_ipv4_checksum_batch_host staged (pico_csum_set_host_in_place(0)): pinned burst -> H2D of the "
                    "span in 32 MiB chunks -> fused IPv4/TCP RX kernel -> D2H of out_net/out_transport/verdict, "
                    "3 staging slots / streams; descriptors and results in pageable memory",
            "in_place": {"value": round(in_place, 3), "unit": "GiB/s",
                         "path": "the same call with the default routing: the pinned burst read in place by the kernel "
                                 "(PCIe), descriptors H2D and results D2H through the staging slots, 128K descriptors "
                                 "a chunk"},
            "pinned_rings": {"value": round(rings, 3), "unit": "GiB/s",
                             "path": "the same call with descriptors and result arrays page-locked too: one launch on "
                                     "the device aliases of all of them, nothing staged"},
            "zero_copy": e2e_zero_copy(pinned, desc)}


def e2e_zero_copy(pinned: torch.Tensor, desc: np.ndarray):
    """Zero-copy ingress (pico_csum_host_device_pointer): the same pinned burst, its descriptors and
    the result arrays in pinned host memory, read / written by the fused kernel over PCIe in place."""
    from picotcp_amd import _lib
    lib = _lib.load()
    n = int(desc.size)
    hd = torch.from_numpy(np.ascontiguousarray(desc).view(np.uint8).copy()).pin_memory()
    res = [torch.empty(k * n, dtype=torch.uint8).pin_memory() for k in (2, 2, 1)]
    dp = [lib.pico_csum_host_device_pointer(t.data_ptr()) for t in [pinned, hd] + res]
    if not all(dp):
        return {"error": lib.pico_csum_last_error().decode()}
    def run():
        rc = lib.pico_ipv4_checksum_batch_dev(dp[0], pinned.numel(), dp[1], n, 0, dp[2], dp[3], dp[4], None)
        _lib.check("pico_ipv4_checksum_batch_dev", rc)
        torch.cuda.synchronize()
    run()
    reps = 5
    t0 = time.perf_counter()
    for _ in range(reps):
        run()
    dt = (time.perf_counter() - t0) / reps
    nbytes = int(desc["len"].astype(np.int64).sum())
    return {"value": round(nbytes / dt / GIB, 3), "unit": "GiB/s",
            "path": "zero copy: burst, descriptors and results in pinned host memory, the fused IPv4/TCP RX "
                    "kernel on their device aliases (pico_csum_host_device_pointer), frames read over PCIe"}


def e2e_rate(n, ln):
    """Host-resident path (pinned host -> H2D -> kernel -> D2H, chunked, 2 streams)."""
    host = torch.randint(0, 256, (n * ln,), dtype=torch.uint8).pin_memory()
    hb = batch.HostBatch(torch.cuda.current_device(), staging_bytes=64 << 20)
    out = np.empty(n, dtype=np.uint16)
    try:
        hb.checksum_uniform(host, ln, ln, n, out=out)
        reps = 5
        t0 = time.perf_counter()
        for _ in range(reps):
            hb.checksum_uniform(host, ln, ln, n, out=out)
        dt = (time.perf_counter() - t0) / reps
    finally:
        hb.close()
    return {"value": round(n * ln / dt / GIB, 3), "unit": "GiB/s",
            "path": "pico_checksum_batch_uniform_host: pinned host frames -> H2D -> kernel -> D2H results, "
                    "64 MiB chunks double-buffered on 2 streams"}


def load_traffic(config: str):
    """(HBM bytes per launch, source) from profiles/pmc_traffic.json: rocprofv3 PMC passes of this
    config recorded on an earlier box (FETCH_SIZE x2 calibrated to 128 B per touched line, plus
    WRITE_SIZE); not measured by this run -- PMC counters need their own rocprofv3 passes."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if not os.path.exists(path):
        return None, None
    try:
        with open(path) as f:
            rec = json.load(f).get(config)
        if rec is None:
            return None, None
        return rec.get("hbm_bytes_per_launch"), (f"profiles/pmc_traffic.json round {rec.get('round')}: rocprofv3 "
                                                  "--pmc FETCH_SIZE (x2, line-calibrated) + WRITE_SIZE, separate "
                                                  "passes of this config, recorded earlier (not this run)")
    except Exception:
        return None, None


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(a) -> None:
    """`--gpus N` is honoured, never silently dropped.  Under torch.distributed.run
    (WORLD_SIZE set) it must equal WORLD_SIZE.  Without a launcher and N > 1, this
    process starts the N ranks itself (one per GPU, 127.0.0.1 rendezvous) as a child
    `torch.distributed.run`, before anything here touches the GPU, and exits with its
    status.  torch.cuda.device_count() does not initialise the device."""
    same_dev = os.environ.get("PICO_BENCH_SAME_DEVICE") == "1"
    if a.gpus < 1:
        sys.exit(f"bench.py: --gpus must be >= 1 (got {a.gpus})")
    ws = os.environ.get("WORLD_SIZE")
    if ws is not None:
        if int(ws) != a.gpus:
            sys.exit(f"bench.py: --gpus {a.gpus} but WORLD_SIZE={ws}: refusing to measure a different GPU count")
        return
    if a.gpus == 1:
        return
    have = torch.cuda.device_count()
    if have < a.gpus and not same_dev:
        sys.exit(f"bench.py: --gpus {a.gpus} but only {have} HIP device(s) visible")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={a.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"))
    sys.exit(subprocess.call(cmd, env=env))


def main():
    a = parse()
    launch_ranks(a)
    if os.environ.get("PICO_BENCH_DRY") == "1":      # launcher test (tests/test_bench_launch.py): no GPU use
        print(json.dumps({"rank": int(os.environ.get("RANK", 0)), "world": int(os.environ.get("WORLD_SIZE", 1)),
                          "gpus": a.gpus}), flush=True)
        return
    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    # Rehearsal knobs for a 1-GPU box (never set by the driver): every rank on GPU 0,
    # timing collectives over gloo (RCCL cannot put two ranks on one GPU).
    if os.environ.get("PICO_BENCH_SAME_DEVICE") == "1":
        local = 0
    backend = os.environ.get("PICO_BENCH_DIST_BACKEND", "nccl")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
    red_dev = dev if backend == "nccl" else torch.device("cpu")
    if a.shape:
        batch.set_launch_override(*[int(x) for x in a.shape.split(",")])
    if a.stream:
        batch.set_uniform_stream(*[int(x) for x in a.stream.split(",")])
    if a.reasm_flat:
        batch.set_reasm_flat(a.reasm_flat)
    cfg = CONFIGS[a.config]

    # ---- batches resident in HBM (rotated so the 256 MiB MALL cannot serve repeats)
    if cfg["kind"] == "uniform":
        ln = cfg["frame_bytes"]
        stride = cfg.get("stride", ln)
        if cfg.get("strong"):
            first, n = shard_range(cfg["frames"], rank, world)
        else:
            first, n = rank * cfg["frames"], cfg["frames"]
        per = n * ln
        rot = a.rotate or rotation(n * stride)
        bufs = [make_uniform(n, stride, dev, 1000 + 17 * rank + i) for i in range(rot)]
        outs = [torch.empty(n, dtype=torch.int16, device=dev) for _ in range(rot)]

        def step(i):
            batch.checksum_uniform(bufs[i % rot], stride, ln, n, out=outs[i % rot])
        frame_bytes = per
        algo_bytes = per + 2 * n                            # frames read + uint16 results written
    elif cfg["kind"] == "ipv4":
        n = cfg["frames"]
        ln = cfg.get("frame_bytes", 0)
        rot = a.rotate or rotation(n * (cfg.get("slot") or (ln or IMIX_MEAN) + 14))
        sets = [make_c2(n, dev, 500 + 13 * rank + i, ln, keep_host=i == 0, slot=cfg.get("slot", 0)) for i in range(rot)]
        wr = cfg.get("tx") and cfg.get("write", True)
        fl = (batch.F_TX | (batch.F_WRITE if wr else 0)) if cfg.get("tx") else 0
        outs = [(torch.empty(n, dtype=torch.int16, device=dev), torch.empty(n, dtype=torch.int16, device=dev),
                 torch.empty(n, dtype=torch.uint8, device=dev)) for _ in range(rot)]

        def step(i):
            b, d, _, _ = sets[i % rot]
            batch.ipv4_checksum_batch(b, d, n, flags=fl, out=outs[i % rot])
        frame_bytes = sets[0][2]
        # datagrams + descriptors + (2+2+1) B results (+ the two 2-byte crc fields written in place on TX)
        algo_bytes = frame_bytes + 16 * n + 5 * n + (4 * n if wr else 0)
        if cfg.get("nat"):
            # NAT records (8 B: addr, port, dir): outbound / inbound halves, a few without a tuple
            g = np.random.default_rng(31 + rank)
            nat_host = np.zeros(n, batch.NAT_DTYPE)
            nat_host["addr"] = g.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32)
            nat_host["port"] = g.integers(0, 1 << 16, n).astype(np.uint16)
            nat_host["dir"] = g.choice(np.array([0, 1, 2], np.uint8), n, p=[0.02, 0.49, 0.49])
            nat_dev = torch.from_numpy(nat_host.view(np.uint8)).to(dev)
            cfg["_nat_host"] = nat_host                  # for the parity check and the CPU leg
            cfg["_nat_before"] = sets[0][0].cpu().numpy()  # slot 0 as the NAT first sees it

            def step(i):                                 # noqa: F811 (the NAT batch instead)
                b, d, _, _ = sets[i % rot]
                batch.ipv4_nat_batch(b, d, n, nat_dev, out=outs[i % rot])
            # datagrams + descriptors + records read, (2+2+1) B results, 10 B written in place per
            # translated datagram (address 4, port 2, two checksums 4)
            algo_bytes = frame_bytes + 16 * n + 8 * n + 5 * n + 10 * int((nat_host["dir"] != 0).sum())
    elif cfg["kind"] == "eth":
        n = cfg["frames"]
        ln = 0
        rot = a.rotate or rotation(n * (IMIX_MEAN + 14))
        sets = [make_c2eth(n, dev, 500 + 13 * rank + i, keep_host=i == 0, mix=bool(cfg.get("mix")))
                for i in range(rot)]
        outs = [(torch.empty(n, dtype=torch.int16, device=dev), torch.empty(n, dtype=torch.int16, device=dev),
                 torch.empty(n, dtype=torch.uint8, device=dev)) for _ in range(rot)]

        def step(i):
            b, d, _, _ = sets[i % rot]
            batch.eth_checksum_batch(b, d, n, mac=MAC, out=outs[i % rot])
        frame_bytes = sets[0][2]
        algo_bytes = frame_bytes + 16 * n + 5 * n            # frames + descriptors + (2+2+1) B results
    elif cfg["kind"] == "frag":
        n, ln = cfg["frames"], cfg["frame_bytes"]
        rot = a.rotate or max(2, rotation(2 * n * ln))
        v6 = bool(cfg.get("v6"))
        sets = [make_frag(n, ln, dev, 900 + 13 * rank + i, v6, bool(cfg.get("interleave")), cfg.get("frag_payload", 0),
                          bool(cfg.get("retx"))) for i in range(rot)]
        res = [(torch.empty(n, dtype=torch.int32, device=dev), torch.empty(n, dtype=torch.int16, device=dev),
                torch.empty(n, dtype=torch.uint8, device=dev)) for _ in range(rot)]

        def step(i):
            b, d, gr, o, od, nfr, _ = sets[i % rot]
            if v6:
                batch.ipv6_reassemble_batch(b, d, nfr, gr, o, od, results=res[i % rot])
            else:
                batch.ipv4_reassemble_batch(b, d, nfr, gr, o, od, results=res[i % rot])
        frame_bytes = sets[0][6]
        nfr = sets[0][5]
        # payload read + written, fragment headers (20 B / 48 B) + descriptors (16 B) read,
        # 2 x 4 B group, 20 B / 40 B header written, (4+2+1) B results
        hl, H = (48, 40) if v6 else (20, 20)
        algo_bytes = 2 * frame_bytes + (hl + 16) * nfr + 8 * n + H * n + 7 * n
    else:
        n = cfg["frames"]
        ln = 0
        rot = a.rotate or rotation(n * (IMIX_MEAN + 20 + 14))
        sets = [make_c2v6(n, dev, 700 + 13 * rank + i, keep_host=i == 0) for i in range(rot)]
        outs = [(torch.empty(n, dtype=torch.int16, device=dev), torch.empty(n, dtype=torch.uint8, device=dev))
                for _ in range(rot)]

        def step(i):
            b, d, _, _ = sets[i % rot]
            batch.ipv6_checksum_batch(b, d, n, out=outs[i % rot])
        frame_bytes = sets[0][2]
        algo_bytes = frame_bytes + 16 * n + 3 * n           # datagrams + descriptors + (2+1) B results

    stream = torch.cuda.current_stream(dev)
    for i in range(a.warmup):
        step(i)
    torch.cuda.synchronize(dev)
    # The K timed steps (each one full pass of the kernel over one resident batch, the batches
    # rotating) are captured once as a HIP graph and replayed: a serving loop over a fixed ring
    # of burst buffers does the same, and the replay removes the Python launch path and part of
    # the per-kernel dispatch gap from the timeline (tools/burst_sweep.py).  --no-graph times
    # the same K launches issued one by one.
    graph = None
    if not a.no_graph:
        graph = torch.cuda.CUDAGraph()
        cap = torch.cuda.Stream(dev)
        cap.wait_stream(stream)
        with torch.cuda.stream(cap):
            with torch.cuda.graph(graph, stream=cap):
                for i in range(a.steps):
                    step(i)
        stream.wait_stream(cap)
        graph.replay()                                   # upload + one untimed pass
        torch.cuda.synchronize(dev)

    # HIP events on the launch stream bracket the timed region: their elapsed
    # time / K is the average launch duration (kernel + the dependent kernel
    # boundary), the figure the roofline fraction uses.
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    ev0.record(stream)
    if graph is not None:
        graph.replay()
    else:
        for i in range(a.steps):
            step(i)
    ev1.record(stream)
    torch.cuda.synchronize(dev)
    wall = time.perf_counter() - t0                  # this rank's region: its closing barrier is not in it
    kern_ms = ev0.elapsed_time(ev1) / a.steps
    if world > 1:
        dist.barrier()

    # ... and whole-job time = max over ranks (each rank's wall from the common start barrier)
    t = torch.tensor([wall, kern_ms], dtype=torch.float64, device=red_dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    wall, kern_max_ms = float(t[0]), float(t[1])
    ms_per_step = wall / a.steps * 1e3
    total_bytes = frame_bytes * (world if not cfg.get("strong") else 1)
    if cfg.get("strong"):
        tb = torch.tensor([float(frame_bytes)], dtype=torch.float64, device=red_dev)
        if world > 1:
            dist.all_reduce(tb)
        total_bytes = float(tb[0])
    value = total_bytes / (ms_per_step / 1e3) / GIB

    achieved = algo_bytes / (kern_ms / 1e3) / 1e9
    traffic, traffic_src = load_traffic(a.config)

    # ---- parity of what the timed region produced (every rank checks its own slot 0)
    ver = None
    if not a.no_verify:
        threads = cpu_threads()[0]
        if cfg["kind"] == "uniform":
            ver = verify("uniform", cfg, (bufs[0], ln, n), outs[0], None, threads)
        elif cfg["kind"] == "frag":
            ver = verify("frag", cfg, sets[0], res[0], None, threads)
        else:
            ver = verify(cfg["kind"], cfg, sets[0], outs[0], sets[0][3], threads)
        vt = torch.tensor([ver["frames"], ver["mismatches"]], dtype=torch.float64, device=red_dev)
        if world > 1:
            dist.all_reduce(vt)
        ver["frames"], ver["mismatches"] = int(vt[0]), int(vt[1])
        if world > 1:
            ver["ranks"] = world
    out = None
    if rank == 0:
        out = {
            "metric": METRIC, "value": round(value, 2), "unit": "GiB/s", "n_gpus": world, "steps": a.steps,
            "warmup": a.warmup, "ms_per_step": round(ms_per_step, 5), "higher_is_better": True,
            "scaling": "strong" if cfg.get("strong") else "weak", "vs_baseline": None, "dtype": "u16",
            "data": "synthetic (seeded random frame bytes; C2: valid IPv4/TCP headers written by the TX kernel)",
            "config": {"workload": cfg["workload"], "frames_per_gpu": n, "frame_bytes": ln or "imix",
                       "batch_bytes_per_gpu": frame_bytes, "rotating_batches": rot,
                       "launch": "K steps replayed as one captured HIP graph" if graph is not None
                       else "K launches from Python",
                       "parallelism": f"shard{world}" if world > 1 else "single",
                       "device": torch.cuda.get_device_name(dev),
                       "device_cus": torch.cuda.get_device_properties(dev).multi_processor_count},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic, "traffic_source": traffic_src,
                         "kernel_avg_us": round(kern_ms * 1e3, 2), "kernel_avg_us_max_rank": round(kern_max_ms * 1e3, 2),
                         "algorithmic_bytes_per_launch": algo_bytes},
        }
        if cfg["kind"] == "frag":         # batches of >= 512 datagrams: flat gather + finish
            flat = a.reasm_flat == 1 or (a.reasm_flat == 0 and n >= 512)
            out["roofline"]["kernels_per_step"] = 2 if flat else 1
        if ver is not None:
            out["verified"] = ver
    if rank == 0 and world == 1 and cfg["kind"] == "uniform":
        if not a.no_cpu:
            sample_frames = min(n, 262144)
            sample = bufs[0][: (sample_frames - 1) * stride + ln].cpu().numpy()
            out["cpu_baseline"] = cpu_baseline(sample, ln, a.cpu_seconds, stride)
        if not a.no_e2e and stride == ln:
            out["e2e_host_to_host"] = e2e_rate(n, ln)
    elif rank == 0 and world == 1 and cfg["kind"] in ("ipv4", "ipv6", "eth"):
        if not a.no_cpu:
            out["cpu_baseline"] = cpu_baseline_fused(sets[0][3], cfg["kind"], bool(cfg.get("tx")),
                                                     a.cpu_seconds / 2, nat=cfg.get("_nat_host"))
        if (not a.no_e2e and cfg["kind"] == "ipv4" and not cfg.get("tx") and not cfg.get("nat") and not ln
                and not cfg.get("slot")):
            out["e2e_host_to_host"] = e2e_rate_desc(sets[0][3])
    elif rank == 0 and world == 1 and cfg["kind"] == "frag":
        if not a.no_cpu:
            out["cpu_baseline"] = cpu_baseline_frag(sets[0], a.cpu_seconds / 2, bool(cfg.get("v6")))
        out["roofline"]["copy_ceiling"] = copy_ceiling(sets[0][6], dev)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    if ver is not None and ver["mismatches"]:
        sys.exit(f"bench.py: {ver['mismatches']} of {ver['frames']} outputs differ from the oracle")


if __name__ == "__main__":
    main()

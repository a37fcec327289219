"""Host-side (Python) mirror of the batched checksum API over torch device tensors.

Each function is a thin call into libpicocsum.so (include/pico_csum.h); the
work happens in the HIP kernels.  Frame buffers are uint8 tensors on a HIP
device; descriptor arrays are uint8 tensors of n*16 bytes (struct
pico_csum_desc); results are int16 tensors holding the uint16 checksum bits
(view them as uint16 with `.cpu().numpy().view(np.uint16)`).

Reference interfaces mirrored (per frame in the reference, per batch here):
  checksum_uniform / checksum_batch  <- pico_checksum, pico_dualbuffer_checksum
                                        (stack/pico_frame.c:312-328)
  ipv4_checksum_batch                <- pico_ipv4_checksum / pico_ipv4_crc_check
                                        (modules/pico_ipv4.c:231-257), pico_ipv4_process_in
                                        (:381-456: source, evil bit, IHL, fragments),
                                        pico_tcp_checksum_ipv4 (pico_tcp.c:422),
                                        pico_udp_checksum_ipv4 (pico_udp.c:36),
                                        pico_icmp4_checksum (pico_icmp4.c:30),
                                        pico_transport_crc_check (pico_socket.c:1916)
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import _lib
from ._lib import (F_NXTHDR_DISPATCH, F_TX, F_WRITE, V_ACCEPT, V_ARP, V_DROP_L2, V_DUPLICATE,  # noqa: F401
                   V_EXPIRED, V_FRAG, V_IPV6, V_L4_BAD, V_LOCAL_SRC, V_MALFORMED, V_NET_BAD, V_UNTOUCHED)

DESC_DTYPE = np.dtype([("off", "<u8"), ("len", "<u4"), ("seed", "<u4")])
# struct pico_csum_nat (include/pico_csum.h): the NAT batch's per-datagram record
NAT_DTYPE = np.dtype([("addr", "<u4"), ("port", "<u2"), ("dir", "u1"), ("reserved", "u1")])
NAT_NONE, NAT_OUTBOUND, NAT_INBOUND = 0, 1, 2
assert DESC_DTYPE.itemsize == 16


def make_desc(offsets, lengths, seeds=None) -> np.ndarray:
    """Host descriptor array (struct pico_csum_desc[n])."""
    offsets = np.asarray(offsets, dtype=np.uint64)
    d = np.zeros(offsets.shape[0], dtype=DESC_DTYPE)
    d["off"] = offsets
    d["len"] = np.asarray(lengths, dtype=np.uint32)
    if seeds is not None:
        d["seed"] = np.asarray(seeds, dtype=np.uint32)
    return d


def desc_to_device(desc: np.ndarray, device) -> torch.Tensor:
    """Copy a descriptor array to the device (fresh allocation: 16-B aligned)."""
    raw = np.ascontiguousarray(desc).view(np.uint8).reshape(-1)
    return torch.from_numpy(raw.copy()).to(device)


def _stream_handle(stream) -> ctypes.c_void_p:
    if stream is None:
        stream = torch.cuda.current_stream()
    return ctypes.c_void_p(stream.cuda_stream)


def _ptr(t: torch.Tensor | None) -> ctypes.c_void_p:
    return ctypes.c_void_p(t.data_ptr() if t is not None else 0)


def _require_device(t: torch.Tensor, name: str) -> None:
    if not t.is_cuda:
        raise ValueError(f"{name} must be a HIP device tensor (the batched path is GPU-only)")


def _check_out(out: torch.Tensor, n: int, name: str, device, itemsize: int = 2) -> None:
    """A caller-supplied result tensor: on the batch's device, contiguous, the right
    element size and at least n elements (the kernels write n results through its pointer)."""
    _require_device(out, name)
    if out.device != device:
        raise ValueError(f"{name} is on {out.device}, the batch on {device}")
    if not out.is_contiguous() or out.element_size() != itemsize:
        raise ValueError(f"{name} must be a contiguous tensor of {itemsize}-byte elements")
    if out.numel() < n:
        raise ValueError(f"{name} has {out.numel()} elements, the batch {n}")


def checksum_uniform(base: torch.Tensor, stride: int, length: int, n: int, seed: int = 0,
                     out: torch.Tensor | None = None, stream=None) -> torch.Tensor:
    """out[i] = pico_checksum(base + i*stride, length) (+ seed as pico_dualbuffer_checksum's
    first buffer); device-resident, asynchronous on `stream`."""
    _require_device(base, "base")
    if n and (n - 1) * stride + length > base.numel():
        raise ValueError("frames exceed the base tensor")
    if out is None:
        out = torch.empty(n, dtype=torch.int16, device=base.device)
    _check_out(out, n, "out", base.device)
    lib = _lib.load()
    _lib.check("pico_checksum_batch_uniform_dev",
               lib.pico_checksum_batch_uniform_dev(_ptr(base), base.numel(), stride, length, n, seed & 0xFFFFFFFF,
                                                   _ptr(out), _stream_handle(stream)))
    return out


def checksum_batch(base: torch.Tensor, desc: torch.Tensor, n: int, crc_off: int = -1, flags: int = 0,
                   out: torch.Tensor | None = None, bad: torch.Tensor | None = None, stream=None) -> torch.Tensor:
    """out[i] = finalize(adder(desc[i].seed, base + desc[i].off, desc[i].len)); crc field
    at crc_off read as zero (and written with F_WRITE).  Regions outside `base` are not
    read (out 0); `bad` (int32[1] on the device) counts them when given."""
    _require_device(base, "base")
    _require_device(desc, "desc")
    if desc.numel() < 16 * n:
        raise ValueError("descriptor tensor shorter than n entries")
    if out is None:
        out = torch.empty(n, dtype=torch.int16, device=base.device)
    _check_out(out, n, "out", base.device)
    if bad is not None:
        _check_out(bad, 1, "bad", base.device, itemsize=4)
    lib = _lib.load()
    _lib.check("pico_checksum_batch_dev",
               lib.pico_checksum_batch_dev(_ptr(base), base.numel(), _ptr(desc), n, crc_off, flags, _ptr(out),
                                           _ptr(bad), _stream_handle(stream)))
    return out


def ipv4_checksum_batch(base: torch.Tensor, desc: torch.Tensor, n: int, flags: int = 0, stream=None, out=None):
    """Fused IPv4 header + transport checksums (RX verify, or TX compute with F_TX).
    Returns (out_net int16[n], out_transport int16[n], verdict uint8[n]); `out` may pass
    that triple preallocated."""
    _require_device(base, "base")
    _require_device(desc, "desc")
    if desc.numel() < 16 * n:
        raise ValueError("descriptor tensor shorter than n entries")
    dev = base.device
    if out is None:
        out = (torch.empty(n, dtype=torch.int16, device=dev), torch.empty(n, dtype=torch.int16, device=dev),
               torch.empty(n, dtype=torch.uint8, device=dev))
    out_net, out_l4, verdict = out
    for t, nm, sz in ((out_net, "out_net", 2), (out_l4, "out_transport", 2), (verdict, "verdict", 1)):
        _check_out(t, n, nm, dev, sz)
    lib = _lib.load()
    _lib.check("pico_ipv4_checksum_batch_dev",
               lib.pico_ipv4_checksum_batch_dev(_ptr(base), base.numel(), _ptr(desc), n, flags, _ptr(out_net),
                                                _ptr(out_l4), _ptr(verdict), _stream_handle(stream)))
    return out_net, out_l4, verdict


def ipv6_checksum_batch(base: torch.Tensor, desc: torch.Tensor, n: int, flags: int = 0, stream=None, out=None):
    """Fused IPv6 transport checksums (TCP / UDP / ICMPv6; RX verify, or TX compute with
    F_TX).  desc.seed = net_len | proto << 16 (0: no extension headers).
    Returns (out_transport int16[n], verdict uint8[n]); `out` may pass that pair
    preallocated."""
    _require_device(base, "base")
    _require_device(desc, "desc")
    if desc.numel() < 16 * n:
        raise ValueError("descriptor tensor shorter than n entries")
    dev = base.device
    if out is None:
        out = (torch.empty(n, dtype=torch.int16, device=dev), torch.empty(n, dtype=torch.uint8, device=dev))
    out_l4, verdict = out
    for t, nm, sz in ((out_l4, "out_transport", 2), (verdict, "verdict", 1)):
        _check_out(t, n, nm, dev, sz)
    lib = _lib.load()
    _lib.check("pico_ipv6_checksum_batch_dev",
               lib.pico_ipv6_checksum_batch_dev(_ptr(base), base.numel(), _ptr(desc), n, flags, _ptr(out_l4),
                                                _ptr(verdict), _stream_handle(stream)))
    return out_l4, verdict


_MACS: dict = {}


def _mac_buf(mac: bytes):
    """A ctypes copy of a 6-byte MAC, built once per address (launch overhead stays below the kernel's)."""
    b = _MACS.get(mac)
    if b is None:
        b = _MACS[mac] = ctypes.create_string_buffer(mac, 6)
    return b


def eth_checksum_batch(base: torch.Tensor, desc: torch.Tensor, n: int, flags: int = 0, mac: bytes | None = None,
                       stream=None, out=None):
    """Ethernet front end + fused IPv4 / IPv6 checksums in one launch (pico_ethernet.c:180-235):
    desc.off -> Ethernet header, desc.len = frame bytes, desc.seed = IPv6 net_len | proto << 16.
    mac = the device address (6 bytes) for the RX destination filter, None = no filter.
    Returns (out_net int16[n], out_transport int16[n], verdict uint8[n])."""
    _require_device(base, "base")
    _require_device(desc, "desc")
    if desc.numel() < 16 * n:
        raise ValueError("descriptor tensor shorter than n entries")
    if mac is not None and len(mac) != 6:
        raise ValueError("mac must be 6 bytes")
    dev = base.device
    if out is None:
        out = (torch.empty(n, dtype=torch.int16, device=dev), torch.empty(n, dtype=torch.int16, device=dev),
               torch.empty(n, dtype=torch.uint8, device=dev))
    out_net, out_l4, verdict = out
    for t, nm, sz in ((out_net, "out_net", 2), (out_l4, "out_transport", 2), (verdict, "verdict", 1)):
        _check_out(t, n, nm, dev, sz)
    lib = _lib.load()
    m = None if mac is None else _mac_buf(bytes(mac))
    _lib.check("pico_eth_checksum_batch_dev",
               lib.pico_eth_checksum_batch_dev(_ptr(base), base.numel(), _ptr(desc), n, flags, m, _ptr(out_net),
                                               _ptr(out_l4), _ptr(verdict), _stream_handle(stream)))
    return out_net, out_l4, verdict


FWD_STATE_BYTES = 16          # struct pico_csum_fwd_state


def fwd_state(device) -> torch.Tensor:
    """A forwarding state (struct pico_csum_fwd_state) at the reference's initial value (zeros)."""
    return torch.zeros(FWD_STATE_BYTES, dtype=torch.uint8, device=device)


def ipv4_forward_batch(base: torch.Tensor, desc: torch.Tensor, n: int, *, state: torch.Tensor | None, local=(),
                       verdict: torch.Tensor | None = None, stream=None) -> torch.Tensor:
    """pico_ipv4_pre_forward_checks (pico_ipv4.c:1535-1574) in batch order, in place on n datagrams:
    ttl - 1, then unless the TTL expired the reference's crc++, the local-source check against
    `local` (the host's link addresses as stored: uint32 little-endian views, <= 32) and the
    duplicate check against the last forwarded tuple, carried in `state` (fwd_state()).  `state`
    is required: a sequence split over several calls must pass the same state tensor to each, as
    the reference's statics carry the last tuple; `state=None` is the explicit one-shot mode (the
    reference's zero initial state, nothing kept).  Descriptors of one batch must not overlap
    (two descriptors on one header would race on its TTL / crc).  Returns the verdicts (V_ACCEPT
    = forwarded, V_EXPIRED, V_LOCAL_SRC, V_DUPLICATE, V_MALFORMED)."""
    _require_device(base, "base")
    _require_u8(base, "base")
    _require_device(desc, "desc")
    if desc.numel() < 16 * n:
        raise ValueError("descriptor tensor shorter than n entries")
    if verdict is None:
        verdict = torch.empty(n, dtype=torch.uint8, device=base.device)
    _check_out(verdict, n, "verdict", base.device, 1)
    if state is not None:
        _require_device(state, "state")
        if state.numel() * state.element_size() < FWD_STATE_BYTES or not state.is_contiguous():
            raise ValueError("state must be a contiguous 16-byte tensor (fwd_state())")
    loc = np.ascontiguousarray(np.asarray(local, dtype=np.uint32))
    lib = _lib.load()
    _lib.check("pico_ipv4_forward_batch_dev",
               lib.pico_ipv4_forward_batch_dev(_ptr(base), base.numel(), _ptr(desc), n,
                                               loc.ctypes.data if loc.size else None, loc.size,
                                               _ptr(state) if state is not None else None, _ptr(verdict),
                                               _stream_handle(stream)))
    return verdict


def ipv4_nat_batch(base: torch.Tensor, desc: torch.Tensor, n: int, nat: torch.Tensor, stream=None, out=None):
    """NAT rewrite (pico_ipv4_nat_outbound / _inbound's frame work, pico_nat.c:424-545) in place on
    n IPv4 datagrams: nat = 8-byte records {addr u32, port u16, dir u8, 0} as uint8 / int64 tensor
    (NAT_DTYPE layout).  Returns (out_net int16[n], out_transport int16[n], verdict uint8[n]):
    V_ACCEPT translated, V_UNTOUCHED, V_FRAG, V_MALFORMED."""
    _require_device(base, "base")
    _require_u8(base, "base")
    _require_device(desc, "desc")
    _require_device(nat, "nat")
    if desc.numel() < 16 * n:
        raise ValueError("descriptor tensor shorter than n entries")
    if nat.numel() * nat.element_size() < 8 * n or not nat.is_contiguous():
        raise ValueError("nat must be a contiguous tensor of n 8-byte records")
    dev = base.device
    if out is None:
        out = (torch.empty(n, dtype=torch.int16, device=dev), torch.empty(n, dtype=torch.int16, device=dev),
               torch.empty(n, dtype=torch.uint8, device=dev))
    out_net, out_l4, verdict = out
    for t, nm, sz in ((out_net, "out_net", 2), (out_l4, "out_transport", 2), (verdict, "verdict", 1)):
        _check_out(t, n, nm, dev, sz)
    lib = _lib.load()
    _lib.check("pico_ipv4_nat_batch_dev",
               lib.pico_ipv4_nat_batch_dev(_ptr(base), base.numel(), _ptr(desc), n, _ptr(nat), _ptr(out_net),
                                           _ptr(out_l4), _ptr(verdict), _stream_handle(stream)))
    return out_net, out_l4, verdict


def _require_u8(t: torch.Tensor, name: str) -> None:
    if t.dtype != torch.uint8 or not t.is_contiguous():
        raise ValueError(f"{name} must be a contiguous uint8 tensor")


def ipv4_reassemble_batch(base: torch.Tensor, frag_desc: torch.Tensor, n_frag: int, groups: torch.Tensor,
                          out: torch.Tensor, out_desc: torch.Tensor, stream=None, results=None):
    """IPv4 reassembly gather + transport check (pico_fragments.c:216-358): groups = uint32
    (first, count) pairs per datagram (int32 tensor of 2*n), out = uint8 device buffer the
    datagrams are written into at out_desc[g].off.  Returns (out_len int32[n], out_transport
    int16[n], verdict uint8[n])."""
    return _reassemble(False, base, frag_desc, n_frag, groups, out, out_desc, 0, stream, results)


def ipv6_reassemble_batch(base: torch.Tensor, frag_desc: torch.Tensor, n_frag: int, groups: torch.Tensor,
                          out: torch.Tensor, out_desc: torch.Tensor, flags: int = 0, stream=None, results=None):
    """IPv6 reassembly gather + transport check (pico_fragments.c:432-498, 304-358): as
    ipv4_reassemble_batch, descriptors at each fragment's IPv6 header; flags F_NXTHDR_DISPATCH."""
    return _reassemble(True, base, frag_desc, n_frag, groups, out, out_desc, flags, stream, results)


def _reassemble(v6, base, frag_desc, n_frag, groups, out, out_desc, flags, stream, results):
    for t, nm in ((base, "base"), (frag_desc, "frag_desc"), (groups, "groups"), (out, "out"), (out_desc, "out_desc")):
        _require_device(t, nm)
        if t.device != base.device:
            raise ValueError(f"{nm} is on {t.device}, the batch on {base.device}")
    _require_u8(base, "base")
    _require_u8(out, "out")
    n = groups.numel() // 2
    if groups.element_size() != 4 or not groups.is_contiguous():
        raise ValueError("groups must be a contiguous 32-bit tensor of (first, count) pairs")
    if frag_desc.numel() * frag_desc.element_size() < 16 * n_frag or out_desc.numel() * out_desc.element_size() < 16 * n:
        raise ValueError("descriptor tensor shorter than its count")
    dev = base.device
    if results is None:
        results = (torch.empty(n, dtype=torch.int32, device=dev), torch.empty(n, dtype=torch.int16, device=dev),
                   torch.empty(n, dtype=torch.uint8, device=dev))
    ol, l4, v = results
    for t, nm, sz in ((ol, "out_len", 4), (l4, "out_transport", 2), (v, "verdict", 1)):
        _check_out(t, n, nm, dev, sz)
    lib = _lib.load()
    if v6:
        _lib.check("pico_ipv6_reassemble_batch_dev",
                   lib.pico_ipv6_reassemble_batch_dev(_ptr(base), base.numel(), _ptr(frag_desc), n_frag, _ptr(groups),
                                                      n, _ptr(out), out.numel(), _ptr(out_desc), _ptr(ol), _ptr(l4),
                                                      _ptr(v), flags, _stream_handle(stream)))
    else:
        _lib.check("pico_ipv4_reassemble_batch_dev",
                   lib.pico_ipv4_reassemble_batch_dev(_ptr(base), base.numel(), _ptr(frag_desc), n_frag, _ptr(groups),
                                                      n, _ptr(out), out.numel(), _ptr(out_desc), _ptr(ol), _ptr(l4),
                                                      _ptr(v), _stream_handle(stream)))
    return ol, l4, v


STREAM_OFF = 0xFF


def set_uniform_stream(mode: int = 0, frames_per_wave: int = 0) -> None:
    """Uniform rings' stream waves (tests / bench sweeps, this thread): mode 0 automatic, 1 on where
    the ring allows them, STREAM_OFF the lane-group kernels; frames per wave (0 = automatic).
    Results never depend on it (include/pico_csum.h)."""
    _lib.check("pico_csum_set_uniform_stream", _lib.load().pico_csum_set_uniform_stream(mode, frames_per_wave))


def set_host_in_place(on: bool = True) -> None:
    """Host-resident descriptor batches (this thread): read a device-addressable (page-locked) burst
    in place (True, the default) or always stage it (False).  Results never depend on it."""
    _lib.check("pico_csum_set_host_in_place", _lib.load().pico_csum_set_host_in_place(1 if on else 0))


def set_reasm_flat(mode: int = 0) -> None:
    """Reassembly batches' flat grid (tests / bench sweeps, this thread): 0 automatic (batches from
    512 datagrams), 1 always, 2 never.  Results never depend on it."""
    _lib.check("pico_csum_set_reasm_flat", _lib.load().pico_csum_set_reasm_flat(mode))


def set_launch_override(group: int = 0, cpl: int = 0, fpw: int = 0, unroll: int | None = None, nt: int = 0,
                        pipeline: int = 0) -> None:
    """Force a kernel launch shape (tests / bench sweeps): group 0 = automatic; 2 = descriptor
    batches with `fpw` frames per wave; 4..64 = uniform rings (lanes per frame, cpl, fpw,
    unroll, nt, pipeline as in include/pico_csum.h)."""
    if unroll is None:
        unroll = 0 if group == 2 else 1
    if group in (0, 2):
        unroll = cpl = nt = pipeline = 0
        if group == 0:
            fpw = 0
    _lib.check("pico_csum_set_launch_override",
               _lib.load().pico_csum_set_launch_override(group, cpl, unroll, fpw, nt, pipeline))


class HostBatch:
    """Host-resident batches (pico_checksum_batch_uniform_host and the descriptor batches
    pico_{checksum,ipv4_checksum,ipv6_checksum,eth_checksum}_batch_host): H2D, kernel and
    D2H chunked over two streams (staging_bytes per chunk)."""

    def __init__(self, device: int = 0, staging_bytes: int = 64 << 20):
        self._lib = _lib.load()
        self._ctx = self._lib.pico_csum_ctx_create(device, staging_bytes)
        if not self._ctx:
            raise _lib.PicoCsumError("pico_csum_ctx_create", -1,
                                     self._lib.pico_csum_last_error().decode(errors="replace"))

    def checksum_uniform(self, frames: np.ndarray | torch.Tensor, stride: int, length: int, n: int,
                         seed: int = 0, out: np.ndarray | None = None) -> np.ndarray:
        if out is None:
            out = np.empty(n, dtype=np.uint16)
        if not (isinstance(out, np.ndarray) and out.dtype == np.uint16 and out.flags.c_contiguous
                and out.size >= n):
            raise ValueError("out must be a contiguous uint16 array of at least n elements")
        need = (n - 1) * stride + length if n else 0
        if isinstance(frames, torch.Tensor):
            if frames.is_cuda:
                raise ValueError("HostBatch takes host memory")
            if not frames.is_contiguous():
                raise ValueError("frames must be contiguous")
            nbytes = frames.numel() * frames.element_size()
            src = frames.data_ptr()
        else:
            if not frames.flags.c_contiguous:
                raise ValueError("frames must be contiguous")
            nbytes = frames.nbytes
            src = frames.ctypes.data
        if nbytes < need:
            raise ValueError(f"frames hold {nbytes} bytes, the batch spans {need}")
        _lib.check("pico_checksum_batch_uniform_host",
                   self._lib.pico_checksum_batch_uniform_host(self._ctx, ctypes.c_void_p(src), stride, length, n,
                                                              seed & 0xFFFFFFFF,
                                                              ctypes.c_void_p(out.ctypes.data)))
        return out

    @staticmethod
    def _host(a: np.ndarray, name: str, dtype=None) -> int:
        if not isinstance(a, np.ndarray) or not a.flags.c_contiguous or (dtype is not None and a.dtype != dtype):
            raise ValueError(f"{name} must be a contiguous numpy array" + (f" of {dtype}" if dtype else ""))
        return a.ctypes.data

    def _desc_args(self, base: np.ndarray, desc: np.ndarray):
        if not (isinstance(base, np.ndarray) and base.dtype == np.uint8 and base.flags.c_contiguous):
            raise ValueError("base must be a contiguous uint8 numpy array (host memory)")
        d = np.ascontiguousarray(desc, dtype=DESC_DTYPE)
        return d, ctypes.c_void_p(base.ctypes.data), base.size, ctypes.c_void_p(d.ctypes.data), d.size

    def _outs(self, n, *spec):
        return [np.zeros(n, dtype=dt) for dt in spec]

    def checksum_batch(self, base: np.ndarray, desc: np.ndarray, crc_off: int = -1, flags: int = 0) -> np.ndarray:
        """pico_checksum_batch_host: raw descriptor batch from host memory (F_WRITE stores in `base`)."""
        d, b, bl, dp, n = self._desc_args(base, desc)
        (out,) = self._outs(n, np.uint16)
        _lib.check("pico_checksum_batch_host",
                   self._lib.pico_checksum_batch_host(self._ctx, b, bl, dp, n, crc_off, flags,
                                                      ctypes.c_void_p(out.ctypes.data)))
        return out

    def ipv4_checksum_batch(self, base: np.ndarray, desc: np.ndarray, flags: int = 0, out=None):
        """`out` may pass the (out_net uint16, out_transport uint16, verdict uint8) host arrays -- e.g.
        page-locked ones, which with a page-locked burst and descriptors make the call zero-copy."""
        d, b, bl, dp, n = self._desc_args(base, desc)
        if out is None:
            on, ol, v = self._outs(n, np.uint16, np.uint16, np.uint8)
        else:
            on, ol, v = out
            for a, nm, dt in ((on, "out_net", np.uint16), (ol, "out_transport", np.uint16), (v, "verdict", np.uint8)):
                self._host(a, nm, dt)
                if a.size < n:
                    raise ValueError(f"{nm} shorter than n")
        _lib.check("pico_ipv4_checksum_batch_host",
                   self._lib.pico_ipv4_checksum_batch_host(self._ctx, b, bl, dp, n, flags, on.ctypes.data,
                                                           ol.ctypes.data, v.ctypes.data))
        return on, ol, v

    def ipv6_checksum_batch(self, base: np.ndarray, desc: np.ndarray, flags: int = 0):
        d, b, bl, dp, n = self._desc_args(base, desc)
        ol, v = self._outs(n, np.uint16, np.uint8)
        _lib.check("pico_ipv6_checksum_batch_host",
                   self._lib.pico_ipv6_checksum_batch_host(self._ctx, b, bl, dp, n, flags, ol.ctypes.data,
                                                           v.ctypes.data))
        return ol, v

    def eth_checksum_batch(self, base: np.ndarray, desc: np.ndarray, flags: int = 0, mac: bytes | None = None):
        d, b, bl, dp, n = self._desc_args(base, desc)
        on, ol, v = self._outs(n, np.uint16, np.uint16, np.uint8)
        m = None if mac is None else ctypes.create_string_buffer(bytes(mac), 6)
        _lib.check("pico_eth_checksum_batch_host",
                   self._lib.pico_eth_checksum_batch_host(self._ctx, b, bl, dp, n, flags, m, on.ctypes.data,
                                                          ol.ctypes.data, v.ctypes.data))
        return on, ol, v

    def close(self) -> None:
        if self._ctx:
            self._lib.pico_csum_ctx_destroy(self._ctx)
            self._ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

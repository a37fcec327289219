// pico_csum_k_raw.hip -- uniform-ring and lane-group kernels (K1, K1p, K1a) and the first fused IPv4
// kernel; their launchers (called by pico_csum.c).
// Helpers, argument structs and the arithmetic contract: pico_csum_dev.h.
#include "pico_csum_dev.h"

namespace {

// RAW batch: per-frame pico_checksum / pico_dualbuffer_checksum.
// UNIFORM: frame i = base + i*stride, len, seed (no descriptors).
// Each lane group keeps U frames in flight: one pass issues U*CPL dwordx4 loads
// per lane before any of them is consumed, so a wave has U*CPL KiB (G=64) of
// reads outstanding while earlier frames are being reduced.
// One wave's frames [f0, f0 + cnt); lane j holds descriptor j (unless UNIFORM).
template <int G, int CPL, int U, bool UNIFORM, bool NT>
__device__ __forceinline__ void raw_wave(const RawArgs& p, uint64_t f0, uint32_t cnt, uint32_t d_lo, uint32_t d_hi,
                                         uint32_t d_len, uint32_t d_seed) {
    constexpr uint32_t NG = 64 / G;
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t g = lane / G, l = lane % G;
    uint32_t res = 0;
    for (uint32_t i = 0; i < cnt; i += NG * U) {
        uint8_t* fp[U];
        const uint8_t* a0[U];
        uint32_t r[U], nch[U], sel[U], seed[U], acc[U];
        uint64_t span[U];
        int64_t xr[U];
        bool oob[U], has_crc[U];
        uint32_t maxch = 0;
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t j = i + u * NG + g;
            uint64_t off;
            uint32_t len;
            if constexpr (UNIFORM) {
                off = (f0 + j) * p.stride;
                len = p.len;
                seed[u] = p.seed;
            } else {
                const uint32_t lo = (uint32_t)__shfl((int)d_lo, (int)j);
                const uint32_t hi = (uint32_t)__shfl((int)d_hi, (int)j);
                off = ((uint64_t)hi << 32) | lo;
                len = (uint32_t)__shfl((int)d_len, (int)j);
                seed[u] = (uint32_t)__shfl((int)d_seed, (int)j);
            }
            if (j >= cnt) len = 0;
            // a region outside the batch buffer is never read (include/pico_csum.h)
            oob[u] = !UNIFORM && j < cnt && (off > p.base_len || len > p.base_len - off);
            if (oob[u]) len = 0;
            fp[u] = p.base + off;
            const uintptr_t a = reinterpret_cast<uintptr_t>(fp[u]);
            r[u] = (uint32_t)(a & 15u);
            a0[u] = fp[u] - r[u];          // stays a global pointer: global_load, not flat_load
            span[u] = (uint64_t)r[u] + len;
            nch[u] = len ? (uint32_t)((span[u] + 15u) >> 4) : 0u;
            sel[u] = (a & 1u) ? SEL_ODD : SEL_EVEN;
            has_crc[u] = p.crc_off >= 0 && (uint64_t)p.crc_off + 2u <= len;
            xr[u] = has_crc[u] ? (int64_t)r[u] + p.crc_off : (int64_t)1 << 40;
            acc[u] = 0;
            maxch = max(maxch, nch[u]);
        }

        // Chunks [1, nch-2] lie wholly inside the frame: they are added unmasked.
        // The head chunk (k = 0), the tail chunk (k = nch-1) and the chunk(s)
        // holding the crc field are added unmasked too, then the bytes that do not
        // count are subtracted again (exact: every sum is mod 2^32).
        uint32_t xk0[U], xk1[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            xk0[u] = has_crc[u] ? (uint32_t)(xr[u] >> 4) : 0u;
            xk1[u] = has_crc[u] ? (uint32_t)((xr[u] + 1) >> 4) : 0u;
        }
        bool any_odd = false;
#pragma unroll
        for (int u = 0; u < U; ++u) any_odd |= (sel[u] != SEL_EVEN);
        any_odd = __builtin_amdgcn_ballot_w64(any_odd) != 0;

        auto pass = [&](auto perm_tag) {
            constexpr bool PERM = decltype(perm_tag)::value;
            for (uint32_t kb = 0; kb < maxch; kb += G * CPL) {
                uint4 v[U][CPL];
#pragma unroll
                for (int u = 0; u < U; ++u)
#pragma unroll
                    for (int c = 0; c < CPL; ++c) {
                        const uint32_t k = kb + l + G * c;
                        v[u][c] = k < nch[u] ? load_chunk_t<NT>(a0[u], k) : make_uint4(0, 0, 0, 0);
                    }
#pragma unroll
                for (int u = 0; u < U; ++u)
#pragma unroll
                    for (int c = 0; c < CPL; ++c) {
                        const uint32_t k = kb + l + G * c;
                        acc[u] = add_full<PERM>(v[u][c], sel[u], acc[u]);
                        const bool edge = k < nch[u] && (k == 0 || k + 1 == nch[u] || k == xk0[u] || k == xk1[u]);
                        if (edge) {
                            uint32_t m = chunk_range_mask(k, r[u], span[u]);
                            m = clear_field(m, xr[u] - ((int64_t)k << 4));
                            acc[u] -= add_chunk(v[u][c], ~m & 0xFFFFu, sel[u], 0u);
                        }
                    }
            }
        };
        if (any_odd) pass(std::integral_constant<bool, true>{});
        else pass(std::integral_constant<bool, false>{});
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const uint32_t j = i + u * NG + g;
            const uint32_t ret = oob[u] ? 0u : finalize(group_sum<G>(acc[u]) + seed[u]);
            if (l == G - 1 && j < cnt) {
                if ((p.flags & 1u) && has_crc[u]) store_crc(fp[u] + p.crc_off, ret);
                if (oob[u] && p.bad) atomicAdd(p.bad, 1u);
            }
            res = collect<G>(res, ret, lane, i + u * NG);
        }
    }
    if (lane < cnt) p.out[f0 + lane] = (uint16_t)res;
}

template <int G, int CPL, int U, bool UNIFORM, bool NT>
__global__ __launch_bounds__(256) void csum_raw_kernel(RawArgs p) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t wave = (uint64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    const uint64_t f0 = wave * p.fpw;
    if (f0 >= p.n) return;
    const uint32_t cnt = (uint32_t)min((uint64_t)p.fpw, (uint64_t)p.n - f0);
    uint32_t d_lo = 0, d_hi = 0, d_len = 0, d_seed = 0;
    if constexpr (!UNIFORM) {
        if (lane < cnt) {
            const uint4 d = *reinterpret_cast<const uint4*>(p.desc + f0 + lane);
            d_lo = d.x; d_hi = d.y; d_len = d.z; d_seed = d.w;
        }
    }
    raw_wave<G, CPL, U, UNIFORM, NT>(p, f0, cnt, d_lo, d_hi, d_len, d_seed);
}

// Descriptor batch, launch shape chosen PER WAVE: the wave reads its (up to 16)
// descriptors, takes the mean chunk count of its frames and runs the lane-group
// body with the smallest G in 4..64 with G*8 >= mean chunks (CPL 8, 16 frames per
// wave = a multiple of every 64/G).  Mixed-size batches (IMIX) then get small
// groups where frames are small and wide groups where they are large, without the
// host knowing the sizes.  Frames > 1 MiB are summed with G = 64.
// Non-temporal loads for waves of frames >= 1 KiB (G >= 16), as for uniform batches.
__global__ __launch_bounds__(256) void csum_desc_adaptive_kernel(RawArgs p) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t wave = (uint64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    const uint64_t f0 = wave * p.fpw;
    if (f0 >= p.n) return;
    const uint32_t cnt = (uint32_t)min((uint64_t)p.fpw, (uint64_t)p.n - f0);
    uint32_t d_lo = 0, d_hi = 0, d_len = 0, d_seed = 0;
    if (lane < cnt) {
        const uint4 d = *reinterpret_cast<const uint4*>(p.desc + f0 + lane);
        d_lo = d.x; d_hi = d.y; d_len = d.z; d_seed = d.w;
    }
    // mean chunks per frame (lengths capped at 1 MiB so the 32-bit sum cannot wrap)
    uint32_t ch = lane < cnt ? (min(d_len, 1u << 20) >> 4) + 1u : 0u;
    ch = group_sum<64>(ch);
    const uint32_t mean = (uint32_t)__builtin_amdgcn_readlane((int)ch, 63) / max(cnt, 1u);
    if (mean <= 32u)       raw_wave<4, 8, 1, false, false>(p, f0, cnt, d_lo, d_hi, d_len, d_seed);
    else if (mean <= 64u)  raw_wave<8, 8, 1, false, false>(p, f0, cnt, d_lo, d_hi, d_len, d_seed);
    else if (mean <= 128u) raw_wave<16, 8, 1, false, true>(p, f0, cnt, d_lo, d_hi, d_len, d_seed);
    else if (mean <= 256u) raw_wave<32, 8, 1, false, true>(p, f0, cnt, d_lo, d_hi, d_len, d_seed);
    else                   raw_wave<64, 8, 1, false, true>(p, f0, cnt, d_lo, d_hi, d_len, d_seed);
}

// Uniform batch, software-pipelined: when a frame fits in one pass (G*CPL chunks),
// a lane group holds two frame sets in registers -- the loads of set i+1 are
// issued before set i is consumed, so a wave never waits on the HBM round trip
// of the frame it is about to reduce.  Frame pairing, masks and results are
// exactly those of csum_raw_kernel (same helpers).
// NTM: 0 plain loads, 1 non-temporal, 2 non-temporal except the slots that hold a
// frame's head or tail chunk (the 128-byte line two neighbouring frames share
// stays in L2 for the second reader).
// BUF (NTM 0/1): loads through a buffer window over the wave's frames (see
// make_window), so the two frame sets really overlap; the host guarantees the
// window, (fpw - 1) * stride + len + 32 bytes, is below 2 GiB.
template <int G, int CPL, int NTM, bool BUF = false>
__global__ __launch_bounds__(256) void csum_uniform_pf_kernel(RawArgs p) {
    static_assert(!BUF || NTM < 2, "windowed loads: NTM 0 or 1");
    constexpr uint32_t NG = 64 / G;
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t g = lane / G, l = lane % G;
    const uint64_t wave = (uint64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    const uint64_t f0 = wave * p.fpw;
    if (f0 >= p.n) return;
    const uint32_t cnt = (uint32_t)min((uint64_t)p.fpw, (uint64_t)p.n - f0);
    Window win{};
    if constexpr (BUF)
        win = make_window(reinterpret_cast<uint64_t>(p.base + f0 * p.stride) & ~15ull,
                          (uint32_t)((uint64_t)(cnt - 1u) * p.stride + p.len + 32u));

    struct Frame {
        const uint8_t* a0;
        uint32_t r, nch, sel;
        uint64_t span;
    };
    auto frame = [&](uint32_t i) {
        Frame f;
        const uint32_t j = i + g;
        const uint32_t len = j < cnt ? p.len : 0u;
        const uint8_t* fp = p.base + (f0 + j) * p.stride;
        f.r = (uint32_t)(reinterpret_cast<uintptr_t>(fp) & 15u);
        f.a0 = fp - f.r;
        f.span = (uint64_t)f.r + len;
        f.nch = len ? (uint32_t)((f.span + 15u) >> 4) : 0u;
        f.sel = (f.r & 1u) ? SEL_ODD : SEL_EVEN;
        return f;
    };
    auto issue = [&](const Frame& f, uint4 (&v)[CPL]) {
#pragma unroll
        for (int c = 0; c < CPL; ++c) {
            const uint32_t k = l + G * c;
            if constexpr (NTM == 2) {
                const bool edge_slot = __builtin_amdgcn_ballot_w64(k < f.nch && (k == 0 || k + 1 == f.nch)) != 0;
                if (edge_slot) v[c] = k < f.nch ? load_chunk_t<false>(f.a0, k) : make_uint4(0, 0, 0, 0);
                else v[c] = k < f.nch ? load_chunk_t<true>(f.a0, k) : make_uint4(0, 0, 0, 0);
            } else if constexpr (BUF) {
                const uint32_t rel = (uint32_t)(reinterpret_cast<uint64_t>(f.a0) - win.base);
                v[c] = load_win<NTM == 1>(win, k < f.nch ? rel + (k << 4) : WIN_OOB);
            } else {
                v[c] = k < f.nch ? load_chunk_t<NTM == 1>(f.a0, k) : make_uint4(0, 0, 0, 0);
            }
        }
    };
    auto consume = [&](const Frame& f, const uint4 (&v)[CPL]) {
        uint32_t acc = 0;
#pragma unroll
        for (int c = 0; c < CPL; ++c) {
            const uint32_t k = l + G * c;
            acc = add_full<true>(v[c], f.sel, acc);
            if (k < f.nch && (k == 0 || k + 1 == f.nch))
                acc -= add_chunk(v[c], ~chunk_range_mask(k, f.r, f.span) & 0xFFFFu, f.sel, 0u);
        }
        return finalize(group_sum<G>(acc) + p.seed);
    };

    uint32_t res = 0;
    uint4 va[CPL], vb[CPL];
    Frame fa = frame(0), fb;
    issue(fa, va);
    for (uint32_t i = 0; i < cnt; i += 2 * NG) {
        fb = frame(i + NG);
        issue(fb, vb);                                   // set i+NG in flight
        res = collect<G>(res, consume(fa, va), lane, i);
        fa = frame(i + 2 * NG);
        issue(fa, va);                                   // set i+2NG in flight
        if (i + NG < cnt) res = collect<G>(res, consume(fb, vb), lane, i + NG);
    }
    if (lane < cnt) p.out[f0 + lane] = (uint16_t)res;
}


// Fused IPv4 header + TCP/UDP/ICMP checksums, RX verify or TX compute.
// Semantics: include/pico_csum.h pico_ipv4_checksum_batch_dev; reference
// modules/pico_ipv4.c:231-257,381-420, stack/pico_socket.c:1916-1968,
// modules/pico_tcp.c:422-446, pico_udp.c:36-60,123, pico_icmp4.c:30-41.
template <int G, int CPL>
__global__ __launch_bounds__(256) void csum_ipv4_kernel(Ipv4Args p) {
    constexpr uint32_t NG = 64 / G;
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t g = lane / G, l = lane % G;
    const uint64_t wave = (uint64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    const uint64_t f0 = wave * p.fpw;
    if (f0 >= p.n) return;
    const uint32_t cnt = (uint32_t)min((uint64_t)p.fpw, (uint64_t)p.n - f0);
    const bool tx = (p.flags & 2u) != 0;

    uint32_t d_lo = 0, d_hi = 0, d_len = 0;
    if (lane < cnt) {
        const uint4 d = *reinterpret_cast<const uint4*>(p.desc + f0 + lane);
        d_lo = d.x; d_hi = d.y; d_len = d.z;
    }

    uint32_t res_net = 0, res_l4 = 0, res_v = 0;
    for (uint32_t i = 0; i < cnt; i += NG) {
        const uint32_t j = i + g;
        const uint32_t lo = (uint32_t)__shfl((int)d_lo, (int)j);
        const uint32_t hi = (uint32_t)__shfl((int)d_hi, (int)j);
        uint32_t avail = (uint32_t)__shfl((int)d_len, (int)j);
        const uint64_t off = ((uint64_t)hi << 32) | lo;
        if (j >= cnt || off > p.base_len || avail > p.base_len - off) avail = 0;   // unread -> MALFORMED
        uint8_t* fp = p.base + off;
        const uintptr_t a = reinterpret_cast<uintptr_t>(fp);
        const uint32_t r = (uint32_t)(a & 15u);
        const uint8_t* a0 = fp - r;
        const uint32_t sel = (a & 1u) ? SEL_ODD : SEL_EVEN;

        // ---- header parse: chunks 0..2 cover header bytes [0, 20); every lane
        // of the group loads the same lines (one request per line).
        uint32_t verdict = V_MALFORMED;
        bool parsed = false;
        uint32_t hl = 0, tl = 0, proto = 0, ipcrc = 0, pseudo = 0;
        uint32_t span = 0, load_len = 0;
        int64_t xoff = (int64_t)1 << 40;
        bool l4_needed = false;
        if (avail >= 20) {
            const uint4 c0 = load_chunk(a0, 0);
            const uint4 c1 = (r + 20 > 16) ? load_chunk(a0, 1) : make_uint4(0, 0, 0, 0);
            const uint4 c2 = (r + 20 > 32) ? load_chunk(a0, 2) : make_uint4(0, 0, 0, 0);
            const uint32_t D[12] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w, c2.x, c2.y, c2.z, c2.w};
            const uint32_t q = r >> 2, s = r & 3u;
            uint32_t E[6];
#pragma unroll
            for (int m = 0; m < 6; ++m) E[m] = sel4(q, D[m], D[m + 1], D[m + 2], D[m + 3]);
            uint32_t H[5];
#pragma unroll
            for (int m = 0; m < 5; ++m) H[m] = __builtin_amdgcn_alignbyte(E[m + 1], E[m], s);
            const uint32_t ihl = H[0] & 0x0Fu;
            hl = 20u + (ihl > 5u ? 4u * (ihl - 5u) : 0u);
            const uint32_t tot = (((H[0] >> 16) & 0xFFu) << 8) | (H[0] >> 24);
            proto = (H[2] >> 8) & 0xFFu;
            ipcrc = H[2] >> 16;
            tl = (tot - hl) & 0xFFFFu;                       // uint16 wrap, pico_ipv4.c:395
            const uint32_t max_allowed = (avail - 20u) & 0xFFFFu;  // pico_ipv4.c:386
            const bool bad = hl > avail || (!tx && tl > max_allowed) || hl + tl > avail;
            if (!bad) {
                parsed = true;
                verdict = 0;
                span = hl + tl;
                load_len = span;
                pseudo = (H[3] & 0xFFFFu) + (H[3] >> 16) + (H[4] & 0xFFFFu) + (H[4] >> 16) +
                         (proto << 8) + (((tl & 0xFFu) << 8) | (tl >> 8));
                if (!tx) {
                    if (proto == 6u) {
                        l4_needed = true;
                    } else if (proto == 17u) {
                        if (hl + 8u > avail) {
                            verdict |= V_MALFORMED;
                        } else {
                            l4_needed = true;   // decided after the crc field is read
                            xoff = hl + 6u;
                            load_len = max(span, hl + 8u);
                        }
                    }
                } else {
                    if (proto == 6u) {
                        if (tl < 20u) verdict |= V_MALFORMED;
                        else { l4_needed = true; xoff = hl + 16u; }
                    } else if (proto == 1u) {
                        if (tl < 8u) verdict |= V_MALFORMED;
                        else { l4_needed = true; xoff = hl + 2u; }
                    }
                }
            }
        }

        // ---- one pass over the datagram: all bytes, header bytes, crc field
        const uint32_t nchunks = load_len ? (r + load_len + 15u) >> 4 : 0u;
        const uint64_t xr = (uint64_t)((int64_t)r + xoff);
        uint32_t acc_all = 0, acc_hdr = 0, acc_x = 0;
        for (uint32_t kb = 0; kb < nchunks; kb += G * CPL) {
            uint4 v[CPL];
#pragma unroll
            for (int c = 0; c < CPL; ++c) {
                const uint32_t k = kb + l + G * c;
                v[c] = k < nchunks ? load_chunk(a0, k) : make_uint4(0, 0, 0, 0);
            }
#pragma unroll
            for (int c = 0; c < CPL; ++c) {
                const uint32_t k = kb + l + G * c;
                if (k < nchunks) {
                    acc_all = add_chunk(v[c], chunk_range_mask(k, r, (uint64_t)r + span), sel, acc_all);
                    if (k < ((r + hl + 15u) >> 4))
                        acc_hdr = add_chunk(v[c], chunk_range_mask(k, r, (uint64_t)r + hl), sel, acc_hdr);
                    acc_x = add_chunk(v[c], chunk_range_mask(k, xr, xr + 2u), sel, acc_x);
                }
            }
        }
        acc_all = group_sum<G>(acc_all);
        acc_hdr = group_sum<G>(acc_hdr);
        acc_x = group_sum<G>(acc_x);

        uint32_t net = 0, l4 = 0;
        if (parsed) {
            net = finalize(acc_hdr - (tx ? ipcrc : 0u));
            if (!tx && net != 0) verdict |= V_NET_BAD;
            const uint32_t tsum = acc_all - acc_hdr;
            if (l4_needed) {
                if (!tx) {
                    if (proto == 6u || acc_x != 0u) {       // UDP: only a non-zero stored crc (pico_socket.c:1941)
                        l4 = finalize(pseudo + tsum);
                        if (l4 != 0) verdict |= V_L4_BAD;
                    }
                } else if (proto == 6u) {
                    l4 = finalize(pseudo + tsum - acc_x);
                } else {
                    l4 = finalize(tsum - acc_x);          // ICMPv4: no pseudo header
                }
            }
            if (verdict == 0) verdict = V_ACCEPT;
        }

        if (tx && (p.flags & 1u) && verdict == V_ACCEPT && l == G - 1 && j < cnt) {
            store_crc(fp + 10, net);
            if ((proto == 6u || proto == 1u) && l4_needed) store_crc(fp + xoff, l4);
            else if (proto == 17u && tl >= 8u) store_crc(fp + hl + 6u, 0u);
        }
        res_net = collect<G>(res_net, net, lane, i);
        res_l4 = collect<G>(res_l4, l4, lane, i);
        res_v = collect<G>(res_v, verdict, lane, i);
    }
    if (lane < cnt) {
        if (p.out_net) p.out_net[f0 + lane] = (uint16_t)res_net;
        if (p.out_l4) p.out_l4[f0 + lane] = (uint16_t)res_l4;
        if (p.verdict) p.verdict[f0 + lane] = (uint8_t)res_v;
    }
}


}  // namespace

extern "C" {

// Per-wave adaptive descriptor kernel (16 frames per wave).
int pico_csum_launch_desc_adaptive(void* base, uint64_t base_len, const void* desc, uint32_t n, int32_t crc_off,
                                   uint32_t flags, uint16_t* out, uint32_t* bad, uint32_t nt, void* stream) {
    if (n == 0) return (int)hipSuccess;
    RawArgs a{static_cast<uint8_t*>(base), base_len, static_cast<const pico_csum_desc_dev*>(desc), 0, 0, n, 0,
              crc_off, flags, 16u, out, bad};
    const dim3 grid = grid_for(n, 16u), block(256);
    hipStream_t s = static_cast<hipStream_t>(stream);
    (void)nt;
    hipLaunchKernelGGL(csum_desc_adaptive_kernel, grid, block, 0, s, a);
    return (int)hipGetLastError();
}

// Software-pipelined uniform kernel (one pass per frame: G*CPL*16 >= len + 15).
int pico_csum_launch_uniform_pf(const void* base, uint64_t base_len, uint64_t stride, uint32_t len, uint32_t n,
                                uint32_t seed, uint16_t* out, uint32_t G, uint32_t CPL, uint32_t nt, uint32_t fpw,
                                uint32_t win, void* stream) {
    if (!shape_ok(G, CPL, fpw) || (uint64_t)G * CPL * 16u < (uint64_t)len + 15u) return (int)hipErrorInvalidValue;
    if (n == 0) return (int)hipSuccess;
    RawArgs a{static_cast<uint8_t*>(const_cast<void*>(base)), base_len, nullptr, stride, len, n, seed, -1, 0u, fpw,
              out, nullptr};
    const dim3 grid = grid_for(n, fpw), block(256);
    hipStream_t s = static_cast<hipStream_t>(stream);
    // windowed loads unless the override asks for the global-load form (A/B) or the
    // wave's window would reach 2 GiB
    const bool buf = win && nt < 2 && (uint64_t)(fpw - 1) * stride + len + 32u < (1ull << 31);
#define X(g, c)                                                                                          \
    if (G == g && CPL == c) {                                                                            \
        if (nt == 2) hipLaunchKernelGGL((csum_uniform_pf_kernel<g, c, 2>), grid, block, 0, s, a);        \
        else if (buf && nt) hipLaunchKernelGGL((csum_uniform_pf_kernel<g, c, 1, true>), grid, block, 0, s, a); \
        else if (buf) hipLaunchKernelGGL((csum_uniform_pf_kernel<g, c, 0, true>), grid, block, 0, s, a); \
        else if (nt) hipLaunchKernelGGL((csum_uniform_pf_kernel<g, c, 1>), grid, block, 0, s, a);        \
        else hipLaunchKernelGGL((csum_uniform_pf_kernel<g, c, 0>), grid, block, 0, s, a);               \
        return (int)hipGetLastError();                                                                   \
    }
    PICO_FOR_SHAPES(X)
#undef X
    return (int)hipErrorInvalidValue;
}

int pico_csum_launch_raw(void* base, uint64_t base_len, const void* desc, uint64_t stride, uint32_t len,
                         uint32_t n, uint32_t seed, int32_t crc_off, uint32_t flags, uint16_t* out,
                         uint32_t* bad, uint32_t G, uint32_t CPL, uint32_t U, uint32_t nt, uint32_t fpw,
                         int uniform, void* stream) {
    if (!shape_ok(G, CPL, fpw) || !(U == 1 || U == 2 || U == 4) || CPL * U > 8) return (int)hipErrorInvalidValue;
    if (n == 0) return (int)hipSuccess;
    RawArgs a{static_cast<uint8_t*>(base), base_len, static_cast<const pico_csum_desc_dev*>(desc), stride, len, n,
              seed, crc_off, flags, fpw, out, bad};
    const dim3 grid = grid_for(n, fpw), block(256);
    hipStream_t s = static_cast<hipStream_t>(stream);
#define Y(g, c, u)                                                                                          \
    if (G == g && CPL == c && U == u) {                                                                     \
        if (uniform) {                                                                                      \
            if (nt) hipLaunchKernelGGL((csum_raw_kernel<g, c, u, true, true>), grid, block, 0, s, a);       \
            else hipLaunchKernelGGL((csum_raw_kernel<g, c, u, true, false>), grid, block, 0, s, a);         \
        } else {                                                                                            \
            if (nt) hipLaunchKernelGGL((csum_raw_kernel<g, c, u, false, true>), grid, block, 0, s, a);      \
            else hipLaunchKernelGGL((csum_raw_kernel<g, c, u, false, false>), grid, block, 0, s, a);        \
        }                                                                                                   \
        return (int)hipGetLastError();                                                                      \
    }
    PICO_FOR_RAW(Y)
#undef Y
    return (int)hipErrorInvalidValue;
}

int pico_csum_launch_ipv4(void* base, uint64_t base_len, const void* desc, uint32_t n, uint32_t flags,
                          uint16_t* out_net, uint16_t* out_l4, uint8_t* verdict, uint32_t G, uint32_t CPL,
                          uint32_t fpw, void* stream) {
    if (!shape_ok(G, CPL, fpw)) return (int)hipErrorInvalidValue;
    if (n == 0) return (int)hipSuccess;
    Ipv4Args a{static_cast<uint8_t*>(base), base_len, static_cast<const pico_csum_desc_dev*>(desc), n, flags, fpw,
               out_net, out_l4, verdict};
    const dim3 grid = grid_for(n, fpw), block(256);
    hipStream_t s = static_cast<hipStream_t>(stream);
#define X(g, c)                                                                      \
    if (G == g && CPL == c) {                                                        \
        hipLaunchKernelGGL((csum_ipv4_kernel<g, c>), grid, block, 0, s, a);          \
        return (int)hipGetLastError();                                               \
    }
    PICO_FOR_SHAPES(X)
#undef X
    return (int)hipErrorInvalidValue;
}

}  // extern "C"

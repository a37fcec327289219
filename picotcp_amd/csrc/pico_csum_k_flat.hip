// pico_csum_k_flat.hip -- the flat work-list descriptor kernel (K2) and its launcher.
// Helpers, argument structs and the arithmetic contract: pico_csum_dev.h.
#include "pico_csum_dev.h"

namespace {

// ---------------------------------------------------------------- flat work-list kernel
//
// Descriptor batches of mixed lengths (C2 simple-IMIX, 64..1500 B).  A lane group
// per frame leaves most lanes idle when a wave's frames differ in size, so here
// a wave takes up to 64 frames and streams them as ONE list of 16-byte chunks:
//   1. lane j owns frame j: reads its descriptor (and, IPv4, parses its header)
//      and counts the chunks it spans, padded to a multiple of 8; a DPP prefix
//      scan of the padded counts gives each frame's start S[j] (per-wave LDS);
//   2. every lane walks consecutive virtual chunks t = t0 + 64c + lane: each load
//      instruction covers 1 KiB that is contiguous wherever the frames are packed,
//      whatever their sizes.  The frame of t is a 6-step binary search in S.  Each
//      chunk is added through a branch-free 128-bit byte mask (two 64-bit shifts)
//      that drops the bytes outside the frame;
//   3. because frames start on 8-lane boundaries, every aligned 8-lane group holds
//      chunks of one frame: 3 DPP adds fold it (a 4th joins the two halves of a row
//      when they share the frame; a whole-wave frame folds in 6) and one lane per
//      run adds into the frame's LDS accumulator (ds_add_u32);
//   4. lane j finalizes frame j: one coalesced store per output per wave.
// Frames of more than 64K chunks (> 1 MiB) are streamed afterwards by the whole
// wave, one at a time, so the 32-bit chunk counts cannot overflow.

constexpr uint32_t FLAT_MAP_BLOCKS = 1024;   // 8-chunk blocks mapped per wave (8K chunks, 128 KiB)

struct FlatWaveLds {
    uint8_t map[FLAT_MAP_BLOCKS];  // 8-chunk block -> frame index (when the batch fits)
    uint32_t S[64];        // exclusive prefix of the padded chunk counts
    uint32_t acc_all[64];  // bytes [0, span) of the frame
    uint32_t acc_x[64];    // the isolated 2-byte field (RAW crc / UDP crc / TX crc)
    uint32_t acc_opt[64];  // IPv4 option bytes [20, hl)
    uint4 info[64];        // {a0 offset lo, hi, span_end = r + span, r | odd << 4 | nch << 5}
    uint2 xo[64];          // {field position r + xoff (NONE), option end r + hl (0)}
};

// Persistent: each wave loops over batches b = wave, wave + W, ... of fpw frames.
// The next batch's descriptors (two batches ahead) and IPv4 header chunks (one
// ahead) are loaded before the current batch streams, so their HBM round trips
// overlap the stream instead of preceding it.
// MODE: 0 RAW, 1 fused IPv4, 2 fused IPv6 transport (TCP / UDP / ICMPv6).
template <int MODE, int CPL, bool NT>
__global__ __launch_bounds__(256) void csum_flat_kernel(FlatArgs p) {
    constexpr bool IPV4 = MODE == 1, IPV6 = MODE == 2;
    __shared__ FlatWaveLds lds_all[4];
    const uint32_t lane = threadIdx.x & 63u;
    FlatWaveLds& L = lds_all[threadIdx.x >> 6];
    const uint64_t W = (uint64_t)gridDim.x * (blockDim.x >> 6);
    const uint64_t nb = ((uint64_t)p.n + p.fpw - 1) / p.fpw;
    uint64_t b = (uint64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    if (b >= nb) return;
    const bool tx = MODE != 0 && (p.flags & 2u) != 0;
    constexpr uint32_t HDR = IPV6 ? 40u : 20u;      // fixed header bytes parsed in phase 1

    auto load_desc = [&](uint64_t bb) {
        uint4 d = make_uint4(0, 0, 0, 0);
        if (bb < nb) {
            const uint64_t f = bb * p.fpw + lane;
            if (lane < p.fpw && f < p.n) d = *reinterpret_cast<const uint4*>(p.desc + f);
        }
        return d;
    };
    // header window: the chunks covering the fixed header of the lane's datagram
    struct Hdr { uint4 c0, c1, c2, c3; };
    auto load_hdr = [&](const uint4 d) {
        const uint4 z = make_uint4(0, 0, 0, 0);
        Hdr h{z, z, z, z};
        if constexpr (MODE != 0) {
            const uint64_t off = ((uint64_t)d.y << 32) | d.x;
            const uint32_t len = d.z;
            if (len >= HDR && off <= p.base_len && len <= p.base_len - off) {
                uint8_t* fp = p.base + off;
                const uint32_t r = (uint32_t)(reinterpret_cast<uintptr_t>(fp) & 15u);
                const uint8_t* a0 = fp - r;
                h.c0 = load_chunk(a0, 0);
                if (r + HDR > 16) h.c1 = load_chunk(a0, 1);
                if (r + HDR > 32) h.c2 = load_chunk(a0, 2);
                if (IPV6 && r + HDR > 48) h.c3 = load_chunk(a0, 3);
            }
        }
        return h;
    };

    uint4 dcur = load_desc(b);
    Hdr hcur = load_hdr(dcur);
    uint4 dnext = load_desc(b + W);

    for (; b < nb; b += W) {
        const uint64_t f0 = b * p.fpw;
        const uint32_t cnt = (uint32_t)min((uint64_t)p.fpw, (uint64_t)p.n - f0);

        // ---- 1. lane j = frame j of this batch
        uint64_t off = ((uint64_t)dcur.y << 32) | dcur.x;
        uint32_t len = lane < cnt ? dcur.z : 0u;
        const uint32_t seed = dcur.w;
        const bool oob = lane < cnt && (off > p.base_len || len > p.base_len - off);
        if (oob || lane >= cnt) { len = 0; off = 0; }
        uint8_t* fp = p.base + off;
        uint32_t r = (uint32_t)(reinterpret_cast<uintptr_t>(fp) & 15u);
        uint64_t a0off = off - r;
        uint32_t odd = r & 1u;

        uint32_t span = 0, ext = 0, xpos = NONE, optend = 0;
        uint32_t verdict = V_MALFORMED, hl = 0, tl = 0, proto = 0, ipcrc = 0, pseudo = 0, hdr20 = 0;
        bool parsed = false, l4_needed = false;
        if constexpr (MODE == 0) {
            span = ext = len;
            if (p.crc_off >= 0 && (uint64_t)p.crc_off + 2u <= len) xpos = r + (uint32_t)p.crc_off;
        } else if constexpr (IPV4) {
            const uint32_t avail = len;
            if (avail >= 20) {
                const uint32_t D[12] = {hcur.c0.x, hcur.c0.y, hcur.c0.z, hcur.c0.w, hcur.c1.x, hcur.c1.y,
                                        hcur.c1.z, hcur.c1.w, hcur.c2.x, hcur.c2.y, hcur.c2.z, hcur.c2.w};
                const uint32_t q = r >> 2, sh = r & 3u;
                uint32_t E[6];
#pragma unroll
                for (int m = 0; m < 6; ++m) E[m] = sel4(q, D[m], D[m + 1], D[m + 2], D[m + 3]);
                uint32_t H[5];
#pragma unroll
                for (int m = 0; m < 5; ++m) H[m] = __builtin_amdgcn_alignbyte(E[m + 1], E[m], sh);
                const uint32_t ihl = H[0] & 0x0Fu;
                hl = 20u + (ihl > 5u ? 4u * (ihl - 5u) : 0u);
                const uint32_t tot = (((H[0] >> 16) & 0xFFu) << 8) | (H[0] >> 24);
                proto = (H[2] >> 8) & 0xFFu;
                ipcrc = H[2] >> 16;
                tl = (tot - hl) & 0xFFFFu;                              // uint16 wrap, pico_ipv4.c:395
                const uint32_t max_allowed = (avail - 20u) & 0xFFFFu;   // pico_ipv4.c:386
                if (!(hl > avail || (!tx && tl > max_allowed) || hl + tl > avail)) {
                    parsed = true;
                    verdict = 0;
                    span = ext = hl + tl;
#pragma unroll
                    for (int m = 0; m < 5; ++m) hdr20 = dot2_add(H[m], hdr20);
                    pseudo = (H[3] & 0xFFFFu) + (H[3] >> 16) + (H[4] & 0xFFFFu) + (H[4] >> 16) +
                             (proto << 8) + (((tl & 0xFFu) << 8) | (tl >> 8));
                    if (hl > 20u) optend = r + hl;
                    if (!tx) {
                        if (proto == 6u) {
                            l4_needed = true;
                        } else if (proto == 17u) {
                            if (hl + 8u > avail) verdict |= V_MALFORMED;
                            else { l4_needed = true; xpos = r + hl + 6u; ext = max(span, hl + 8u); }
                        }
                    } else {
                        if (proto == 6u) {
                            if (tl < 20u) verdict |= V_MALFORMED;
                            else { l4_needed = true; xpos = r + hl + 16u; }
                        } else if (proto == 1u) {
                            if (tl < 8u) verdict |= V_MALFORMED;
                            else { l4_needed = true; xpos = r + hl + 2u; }
                        }
                    }
                }
            }
        } else {
            // IPv6: pico_ipv6.c:707-800 lengths, pico_ipv6.h:46-53 pseudo header.  The
            // streamed region is the transport [net_len, net_len + tl) alone.
            const uint32_t avail = len;
            if (avail >= 40) {
                const uint32_t D[16] = {hcur.c0.x, hcur.c0.y, hcur.c0.z, hcur.c0.w, hcur.c1.x, hcur.c1.y,
                                        hcur.c1.z, hcur.c1.w, hcur.c2.x, hcur.c2.y, hcur.c2.z, hcur.c2.w,
                                        hcur.c3.x, hcur.c3.y, hcur.c3.z, hcur.c3.w};
                const uint32_t q = r >> 2, sh = r & 3u;
                uint32_t E[11];
#pragma unroll
                for (int m = 0; m < 11; ++m) E[m] = sel4(q, D[m], D[m + 1], D[m + 2], D[m + 3]);
                uint32_t H[10];
#pragma unroll
                for (int m = 0; m < 10; ++m) H[m] = __builtin_amdgcn_alignbyte(E[m + 1], E[m], sh);
                const uint32_t plen = ((H[1] & 0xFFu) << 8) | ((H[1] >> 8) & 0xFFu);
                uint32_t net_len = seed & 0xFFFFu;
                proto = (seed >> 16) & 0xFFu;
                if (seed == 0) { net_len = 40u; proto = (H[1] >> 16) & 0xFFu; }
                tl = (plen - (net_len - 40u)) & 0xFFFFu;                // pico_ipv6.c:790
                if (net_len >= 40u && net_len <= avail && net_len + tl <= avail) {
                    uint32_t addr = 0, xrel = NONE;
#pragma unroll
                    for (int m = 2; m < 10; ++m) addr = dot2_add(H[m], addr);
                    pseudo = addr + (((tl & 0xFFu) << 8) | (tl >> 8)) + (proto << 8);
                    parsed = true;
                    verdict = 0;
                    ext = tl;
                    if (!tx) {
                        if (proto == 6u) {
                            l4_needed = true;
                        } else if (proto == 17u) {
                            if (net_len + 8u > avail) { parsed = false; verdict = V_MALFORMED; }
                            else { l4_needed = true; xrel = 6u; ext = max(tl, 8u); }
                        } else if (proto == 58u) {
                            if (net_len + 1u > avail) { parsed = false; verdict = V_MALFORMED; }
                            else { l4_needed = true; xrel = 0u; ext = max(tl, 1u); }
                        }
                    } else {
                        const uint32_t need = proto == 6u ? 20u : proto == 17u ? 8u : 4u;
                        if (proto == 6u || proto == 17u || proto == 58u) {
                            if (tl < need) { parsed = false; verdict = V_MALFORMED; }
                            else { l4_needed = true; xrel = proto == 6u ? 16u : proto == 17u ? 6u : 2u; }
                        }
                    }
                    if (parsed) {
                        off += net_len;                             // the region: the transport
                        fp = p.base + off;
                        r = (uint32_t)(reinterpret_cast<uintptr_t>(fp) & 15u);
                        a0off = off - r;
                        odd = r & 1u;
                        span = tl;
                        if (xrel != NONE) xpos = r + xrel;
                    } else {
                        ext = 0;
                    }
                }
            }
        }
        const uint64_t nch64 = ext ? ((uint64_t)r + ext + 15u) >> 4 : 0u;
        const bool big = nch64 > BIG_CHUNKS;
        const uint32_t nch = big ? 0u : (uint32_t)nch64;
        const uint32_t pch = (nch + 7u) & ~7u;
        const uint32_t incl = wave_scan_add(pch);
        const uint32_t T = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
        const uint32_t S = incl - pch;
        const bool any_odd = __builtin_amdgcn_ballot_w64(nch64 != 0 && odd) != 0;
        const bool any_x = __builtin_amdgcn_ballot_w64(nch64 != 0 && xpos != NONE) != 0;
        const bool any_opt = IPV4 && __builtin_amdgcn_ballot_w64(nch != 0 && optend != 0) != 0;
        uint64_t bigmask = __builtin_amdgcn_ballot_w64(big);
        L.S[lane] = lane < cnt ? S : T;
        L.acc_all[lane] = 0;
        L.acc_x[lane] = 0;
        L.acc_opt[lane] = 0;
        L.info[lane] = make_uint4((uint32_t)a0off, (uint32_t)(a0off >> 32), r + span, r | (odd << 4) | (nch << 5));
        L.xo[lane] = make_uint2(xpos, optend);
        // block -> frame map: a frame's blocks are written by its own lane
        const bool use_map = T <= 8u * FLAT_MAP_BLOCKS;
        if (use_map && lane < cnt)
            for (uint32_t i = 0; i < (pch >> 3); ++i) L.map[(S >> 3) + i] = (uint8_t)lane;
        __builtin_amdgcn_wave_barrier();

        // ---- prefetch: headers of the next batch, descriptors of the one after
        if constexpr (MODE != 0) hcur = load_hdr(dnext);
        dcur = dnext;
        dnext = load_desc(b + 2 * W);

        // ---- 2. stream this batch's chunk list
        auto stream = [&](auto perm_tag) {
            constexpr bool PERM = decltype(perm_tag)::value;
            for (uint32_t t0 = 0; t0 < T; t0 += 64u * CPL) {
                uint4 v[CPL];
                uint32_t jj[CPL], kk[CPL];
                uint4 fi[CPL];
                bool ok[CPL];
#pragma unroll
                for (int c = 0; c < CPL; ++c) {
                    const uint32_t t = t0 + 64u * c + lane;
                    uint32_t j = 0, sj = 0;
                    if (use_map) {
                        j = t < T ? L.map[t >> 3] : 63u;
                        sj = L.S[j];
                    } else {
#pragma unroll
                        for (uint32_t step = 32; step; step >>= 1) {
                            const uint32_t s2 = L.S[j + step];
                            if (s2 <= t) { j += step; sj = s2; }
                        }
                    }
                    jj[c] = j;
                    kk[c] = t - sj;
                    fi[c] = L.info[j];
                    ok[c] = t < T && kk[c] < (fi[c].w >> 5);
                    const uint8_t* a0 = p.base + ((((uint64_t)fi[c].y) << 32) | fi[c].x);
                    v[c] = ok[c] ? load_chunk_t<NT>(a0, kk[c]) : make_uint4(0, 0, 0, 0);
                }
#pragma unroll
                for (int c = 0; c < CPL; ++c) {
                    const uint32_t k = kk[c], j = jj[c];
                    const uint32_t rr = fi[c].w & 15u;
                    const uint32_t sl = (fi[c].w & 16u) ? SEL_ODD : SEL_EVEN;
                    const uint32_t ch = k << 4;
                    uint32_t x = ok[c] ? masked_chunk_sum<PERM>(v[c], ch, rr, fi[c].z, sl) : 0u;
                    if (any_x || any_opt) {
                        const uint2 xo = L.xo[j];
                        if (any_x && ok[c] && xo.x != NONE && (k == (xo.x >> 4) || k == ((xo.x + 1u) >> 4))) {
                            const uint32_t xv = masked_chunk_sum<PERM>(v[c], ch, xo.x, xo.x + 2u, sl);
                            if (xv) atomicAdd(&L.acc_x[j], xv);
                        }
                        if (IPV4 && any_opt && ok[c] && xo.y != 0u && ch < xo.y) {
                            const uint32_t ov = masked_chunk_sum<PERM>(v[c], ch, rr + 20u, xo.y, sl);
                            if (ov) atomicAdd(&L.acc_opt[j], ov);
                        }
                    }
                    const bool blk_ok = (t0 + 64u * c + lane) < T;      // the lane's 8-block is in the list
                    const uint32_t k0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)j);
                    const uint32_t k63 = (uint32_t)__builtin_amdgcn_readlane((int)j, 63);
                    const bool whole = k0 == k63 && __builtin_amdgcn_readlane((int)blk_ok, 63);
                    if (whole) {                                     // the slot is one frame
                        const uint32_t tot = group_sum<64>(x);
                        if (lane == 63) atomicAdd(&L.acc_all[j], tot);
                    } else {                                         // 8-lane runs, halves joined
                        x = group_sum<8>(x);
                        const uint32_t xm = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x140, 0xF, 0xF, false);
                        const uint32_t jm = (uint32_t)__builtin_amdgcn_update_dpp(-1, (int)j, 0x140, 0xF, 0xF, false);
                        const bool same = jm == j;
                        const uint32_t q = lane & 15u;
                        const bool hi_ok = (t0 + 64u * c + (lane | 15u)) < T;
                        const bool adder = blk_ok && (q == 15u || (q == 7u && (!same || !hi_ok)));
                        const uint32_t val = (q == 15u && same) ? x + xm : x;
                        if (adder) atomicAdd(&L.acc_all[j], val);
                    }
                }
            }
        };
        if (T) {
            if (any_odd) stream(std::integral_constant<bool, true>{});
            else stream(std::integral_constant<bool, false>{});
        }

        // ---- 2b. frames over BIG_CHUNKS, one at a time by the whole wave
        while (bigmask) {
            const uint32_t j = (uint32_t)__builtin_ctzll(bigmask);
            bigmask &= bigmask - 1;
            const uint32_t blo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)a0off, (int)j);
            const uint32_t bhi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(a0off >> 32), (int)j);
            const uint32_t br = (uint32_t)__builtin_amdgcn_readlane((int)r, (int)j);
            const uint32_t bspan = (uint32_t)__builtin_amdgcn_readlane((int)span, (int)j);
            const uint32_t bx = (uint32_t)__builtin_amdgcn_readlane((int)xpos, (int)j);
            const uint64_t bend = (uint64_t)br + bspan;
            const uint32_t bn = (uint32_t)((bend + 15u) >> 4);
            const uint32_t bsel = (br & 1u) ? SEL_ODD : SEL_EVEN;
            const uint8_t* a0 = p.base + (((uint64_t)bhi << 32) | blo);
            uint32_t acc = 0, accx = 0;
            for (uint32_t kb = 0; kb < bn; kb += 64u * CPL) {
                uint4 v[CPL];
#pragma unroll
                for (int c = 0; c < CPL; ++c) {
                    const uint32_t k = kb + 64u * c + lane;
                    v[c] = k < bn ? load_chunk_t<NT>(a0, k) : make_uint4(0, 0, 0, 0);
                }
#pragma unroll
                for (int c = 0; c < CPL; ++c) {
                    const uint32_t k = kb + 64u * c + lane;
                    const bool edge = k < bn && (k == 0 || k + 1 == bn);
                    acc = add_full<true>(v[c], bsel, acc);
                    if (edge) acc -= add_chunk(v[c], ~chunk_range_mask(k, br, bend) & 0xFFFFu, bsel, 0u);
                    if (bx != NONE && (k == (bx >> 4) || k == ((bx + 1u) >> 4)))
                        accx += add_chunk(v[c], chunk_range_mask(k, bx, (uint64_t)bx + 2u), bsel, 0u);
                }
            }
            acc = group_sum<64>(acc);
            accx = group_sum<64>(accx);
            if (lane == 63) { L.acc_all[j] = acc; L.acc_x[j] = accx; }
        }
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0): this wave's LDS updates are done

        // ---- 3. lane j finalizes frame j
        if (lane < cnt) {
            const uint32_t acc_all = L.acc_all[lane], acc_x = L.acc_x[lane], acc_opt = L.acc_opt[lane];
            if constexpr (MODE == 0) {
                uint32_t ret = 0;
                if (oob) {
                    if (p.bad) atomicAdd(p.bad, 1u);
                } else {
                    ret = finalize(seed + acc_all - acc_x);
                    if ((p.flags & 1u) && xpos != NONE) store_crc(fp + p.crc_off, ret);
                }
                p.out[f0 + lane] = (uint16_t)ret;
            } else if constexpr (IPV6) {
                uint32_t l4 = 0;
                if (parsed) {
                    if (l4_needed) {
                        if (!tx) {
                            if (proto == 6u || (proto == 17u && acc_x != 0u) || proto == 58u) {
                                l4 = finalize(pseudo + acc_all);
                                const uint32_t type = acc_x & 0xFFu;   // ICMPv6 type (x field = [0, 2))
                                const bool checked = proto != 58u || (type >= 130u && type <= 137u) || type == 143u;
                                if (l4 != 0 && checked) verdict |= V_L4_BAD;
                            }
                        } else {
                            l4 = finalize(pseudo + acc_all - acc_x);
                        }
                    }
                    if (verdict == 0) verdict = V_ACCEPT;
                }
                if (tx && (p.flags & 1u) && verdict == V_ACCEPT && l4_needed)
                    store_crc(fp + (xpos - r), l4);
                if (p.out_l4) p.out_l4[f0 + lane] = (uint16_t)l4;
                if (p.verdict) p.verdict[f0 + lane] = (uint8_t)verdict;
            } else {
                uint32_t net = 0, l4 = 0;
                if (parsed) {
                    const uint32_t acc_hdr = hdr20 + acc_opt;
                    net = finalize(acc_hdr - (tx ? ipcrc : 0u));
                    if (!tx && net != 0) verdict |= V_NET_BAD;
                    const uint32_t tsum = acc_all - acc_hdr;
                    if (l4_needed) {
                        if (!tx) {
                            if (proto == 6u || acc_x != 0u) {
                                l4 = finalize(pseudo + tsum);
                                if (l4 != 0) verdict |= V_L4_BAD;
                            }
                        } else if (proto == 6u) {
                            l4 = finalize(pseudo + tsum - acc_x);
                        } else {
                            l4 = finalize(tsum - acc_x);
                        }
                    }
                    if (verdict == 0) verdict = V_ACCEPT;
                }
                if (tx && (p.flags & 1u) && verdict == V_ACCEPT) {
                    store_crc(fp + 10, net);
                    if ((proto == 6u || proto == 1u) && l4_needed) store_crc(fp + hl + (proto == 6u ? 16u : 2u), l4);
                    else if (proto == 17u && tl >= 8u) store_crc(fp + hl + 6u, 0u);
                }
                if (p.out_net) p.out_net[f0 + lane] = (uint16_t)net;
                if (p.out_l4) p.out_l4[f0 + lane] = (uint16_t)l4;
                if (p.verdict) p.verdict[f0 + lane] = (uint8_t)verdict;
            }
        }
        __builtin_amdgcn_wave_barrier();
    }
}


}  // namespace

extern "C" {

// Flat work-list kernel for descriptor batches: mode 0 RAW, 1 fused IPv4, 2 fused IPv6.
int pico_csum_launch_flat(void* base, uint64_t base_len, const void* desc, uint32_t n, int mode,
                          int32_t crc_off, uint32_t flags, uint16_t* out, uint32_t* bad, uint16_t* out_net,
                          uint16_t* out_l4, uint8_t* verdict, uint32_t CPL, uint32_t nt, uint32_t fpw,
                          uint32_t max_blocks, void* stream) {
    if (!(CPL == 1 || CPL == 2 || CPL == 4 || CPL == 8) || fpw < 1 || fpw > 64 || max_blocks == 0)
        return (int)hipErrorInvalidValue;
    if (n == 0) return (int)hipSuccess;
    FlatArgs a{static_cast<uint8_t*>(base), base_len, static_cast<const pico_csum_desc_dev*>(desc), n, fpw,
               crc_off, flags, out, bad, out_net, out_l4, verdict};
    dim3 grid = grid_for(n, fpw), block(256);
    if (grid.x > max_blocks) grid.x = max_blocks;             // persistent: waves loop over batches
    hipStream_t s = static_cast<hipStream_t>(stream);
#define Z(c)                                                                                        \
    if (CPL == c) {                                                                                 \
        if (mode == 2) {                                                                            \
            if (nt) hipLaunchKernelGGL((csum_flat_kernel<2, c, true>), grid, block, 0, s, a);       \
            else hipLaunchKernelGGL((csum_flat_kernel<2, c, false>), grid, block, 0, s, a);         \
        } else if (mode == 1) {                                                                     \
            if (nt) hipLaunchKernelGGL((csum_flat_kernel<1, c, true>), grid, block, 0, s, a);       \
            else hipLaunchKernelGGL((csum_flat_kernel<1, c, false>), grid, block, 0, s, a);         \
        } else {                                                                                    \
            if (nt) hipLaunchKernelGGL((csum_flat_kernel<0, c, true>), grid, block, 0, s, a);       \
            else hipLaunchKernelGGL((csum_flat_kernel<0, c, false>), grid, block, 0, s, a);         \
        }                                                                                           \
        return (int)hipGetLastError();                                                              \
    }
    Z(1) Z(2) Z(4) Z(8)
#undef Z
    return (int)hipErrorInvalidValue;
}

}  // extern "C"

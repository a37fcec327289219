// pico_csum_k_sorted.hip -- the sorted-rounds descriptor kernel (K4: RAW / fused IPv4 / IPv6 /
// Ethernet front end), the IPv4 forwarding step (K5), and their launchers.
// Helpers, argument structs and the arithmetic contract: pico_csum_dev.h.
#include "pico_csum_dev.h"

#ifndef SORTED_MODE
#define SORTED_MODE 0
#endif

namespace {

#ifdef PICO_CSUM_STAMPS
// Diagnostic build only (tools/stamps.py; never the product library): per wave, s_memrealtime
// (100 MHz, comparable across XCDs) at entry, after phase 1, after the rounds and at the end,
// into a buffer no other code reads.
__device__ uint64_t* g_stamps;
__device__ uint32_t g_stamps_n;
#define STAMP(k)                                                                                   \
    do {                                                                                           \
        const uint64_t wv_ = (uint64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);        \
        const uint64_t t_ = __builtin_amdgcn_s_memrealtime();                                      \
        if ((threadIdx.x & 63u) == 0 && g_stamps && wv_ < g_stamps_n) g_stamps[4 * wv_ + (k)] = t_; \
    } while (0)
#else
#define STAMP(k) do {} while (0)
#endif

// ---------------------------------------------------------------- sorted-rounds kernel
//
// Descriptor batches of any size mix, all modes (RAW / fused IPv4 / fused IPv6).
// The lane-group body is the cheapest per chunk (an unmasked v_dot2 chain, edge
// corrections only at frame edges) but a fixed group width G fits no size mix:
// a wave waits for its largest frame.  Here a wave
//   1. parses its (up to 64) frames, lane j = frame j (as the flat kernel);
//   2. orders them by size class -- the narrowest width G in {4..64} whose one pass
//      (G lanes x CPL chunks) covers the frame -- with 5 ballots and mbcnt (a
//      64-lane bitonic sort by length measured the same round times at ~1K more
//      cycles of shuffle latency per batch);
//   3. walks that order in rounds: each round takes the next 64/G frames with G the
//      class of the last of them, so every round holds frames of similar size and
//      keeps its lanes busy; per-frame sums go to LDS;
//   4. lane j finalizes frame j (one coalesced store per output).

constexpr uint32_t HW = 8;   // head-window chunks the fused modes load in phase 1
#ifndef PICO_HW_NT
#define PICO_HW_NT 0         // non-temporal head-window loads: A/B builds only (5 % slower, profiles/r02nt)
#endif

struct SortedWaveLds {
    uint32_t acc_all[64];
    uint32_t acc_x[64];
    uint32_t acc_opt[64];
    uint32_t nch[64];
    uint4 info[64];        // {a0 offset lo, hi, span_end = r + span, r | odd << 4 | k0 << 5}
    uint2 xo[64];          // {field position (NONE), option end (0)}, relative to a0 + 16 k0
    uint32_t order[64];    // frames by size class: order[position] = frame (lane)
    uint4 fin[64];         // parse state for phase 4 (kept in LDS, not VGPRs, across the rounds):
                           // {verdict | parsed << 4 | l4 << 5 | oob << 6 | proto << 8 | tl << 16,
                           //  hl | ip crc << 16, pseudo sum (RAW: seed), header sum}
};

// A wave's LDS.  Fused modes: the phase-1 head-window staging (64 frames x HW chunks,
// chunk slots XOR-swizzled) shares the space with the state it is parsed into -- 8 KiB a
// wave, 4 workgroups of 4 waves per CU.  RAW mode: the state alone (3.75 KiB).
template <bool STAGE>
union SortedWaveSmem {
    SortedWaveLds s;
    uint4 stage[64 * HW];
};
template <>
union SortedWaveSmem<false> {
    SortedWaveLds s;
    uint4 stage[1];
};

// One round: group g sums the frame at position pos + g of the class order.
template <int G, int CPL, bool PERM, bool NT, bool XO>
__device__ __forceinline__ void sorted_round(const RawArgs& p, SortedWaveLds& L, uint32_t pos, uint32_t m) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t g = lane / G, l = lane % G;
    const uint32_t si = pos + g;
    const bool valid = si < m;
    const uint32_t j = L.order[min(si, 63u)] & 63u;
    const uint32_t nch = valid ? L.nch[j] : 0u;
    const uint4 fi = L.info[j];
    const uint2 xo = XO ? L.xo[j] : make_uint2(NONE, 0u);
    // the rounds start k0 chunks into the region (phase 1 summed the head window)
    const uint32_t k0 = (fi.w >> 5) & 15u;
    const uint32_t rr = k0 ? 0u : fi.w & 15u;
    const uint32_t sl = (fi.w & 16u) ? SEL_ODD : SEL_EVEN;
    const uint32_t send = fi.z > 16u * k0 ? fi.z - 16u * k0 : 0u;
    const uint8_t* a0 = p.base + ((((uint64_t)fi.y) << 32) | fi.x) + 16u * k0;
    uint32_t acc = 0, accx = 0, acco = 0;
    for (uint32_t kb = 0; kb < nch; kb += G * CPL) {
        uint4 v[CPL];
#pragma unroll
        for (int c = 0; c < CPL; ++c) {
            const uint32_t k = kb + l + G * c;
            v[c] = k < nch ? load_chunk_t<NT>(a0, k) : make_uint4(0, 0, 0, 0);
        }
        // interior chunks unmasked; masked sums only where a chunk holds a region edge
        // (a wave-uniform branch: skipped for slots no lane's edge falls in)
#pragma unroll
        for (int c = 0; c < CPL; ++c) {
            const uint32_t k = kb + l + G * c;
            const uint32_t ch = k << 4;
            if (k < nch && (ch < rr || ch + 16u > send)) acc += masked_chunk_sum<PERM>(v[c], ch, rr, send, sl);
            else acc = add_full<PERM>(v[c], sl, acc);
            if constexpr (XO) {
                if (k < nch && xo.x != NONE && (k == (xo.x >> 4) || k == ((xo.x + 1u) >> 4)))
                    accx += masked_chunk_sum<PERM>(v[c], ch, xo.x, xo.x + 2u, sl);
                if (k < nch && xo.y != 0u && ch < xo.y)
                    acco += masked_chunk_sum<PERM>(v[c], ch, rr + 20u, xo.y, sl);
            }
        }
    }
    acc = group_sum<G>(acc);
    if constexpr (XO) {
        accx = group_sum<G>(accx);
        acco = group_sum<G>(acco);
    }
    if (valid && l == G - 1) {           // added to phase 1's head-window sums
        L.acc_all[j] += acc;
        if constexpr (XO) {
            if (xo.x != NONE) L.acc_x[j] += accx;
            if (xo.y != 0u) L.acc_opt[j] += acco;
        }
    }
}

// Round width: the smallest G whose one pass (G lanes x CPL chunks) covers the
// round's largest frame; 64 lanes per frame beyond that.  NT: non-temporal loads
// in the rounds of G >= 16 (frames over ~1 KiB; measured: they cost on small ones).
// SMALL adds a 1-lane class below the 4-lane one: frames of <= CPL chunks (<= 8 x 16 B,
// e.g. 64-byte IMIX frames) are summed one frame per lane, 64 per round, so a wave
// pays one dependent HBM round trip for all its small frames instead of one per 16.
template <int CPL, bool PERM, bool NT, bool XO, bool SMALL>
__device__ __forceinline__ void sorted_rounds(const RawArgs& p, SortedWaveLds& L, const uint32_t (&e)[5], uint32_t m) {
    // position s holds a frame of class <= c iff s < e[c]; a round of width G may
    // take the next 64/G positions when the last of them is of class <= G's class
    constexpr int o = SMALL ? 1 : 0;
    uint32_t pos = 0;
    if constexpr (SMALL) {
        if (e[0]) { sorted_round<1, CPL, PERM, false, XO>(p, L, 0u, min(m, e[0])); pos = min(e[0], 64u); }
    }
    while (pos < m) {
        if (min(pos + 15u, m - 1u) < e[o])            { sorted_round<4, CPL, PERM, false, XO>(p, L, pos, m);  pos += 16u; }
        else if (min(pos + 7u, m - 1u) < e[o + 1])    { sorted_round<8, CPL, PERM, false, XO>(p, L, pos, m);  pos += 8u; }
        else if (min(pos + 3u, m - 1u) < e[o + 2])   { sorted_round<16, CPL, PERM, NT, XO>(p, L, pos, m); pos += 4u; }
        else if (min(pos + 1u, m - 1u) < e[o + 3])   { sorted_round<32, CPL, PERM, NT, XO>(p, L, pos, m); pos += 2u; }
        else                                          { sorted_round<64, CPL, PERM, NT, XO>(p, L, pos, m); pos += 1u; }
    }
}

// ---------------------------------------------------------------- span stream (dense waves)
//
// Most descriptor batches are bursts laid out back to back (a TAP / pico_device ring, the
// C2 layout: datagrams behind 14-byte Ethernet headers).  For such a wave -- frames in
// ascending order, each >= 16 bytes and < 64 KiB, gaps < 16 bytes -- the rounds are replaced
// by ONE coalesced stream over the wave's span: step t reads chunks 64t .. 64t+63 (1 KiB, lane
// l = chunk 64t + l; 8 steps in flight), so every line is fetched once and whole.  Per step,
// no masks: each chunk gives two unmasked sums in the batch's own (absolute) pairing,
// a = E + 256 O (v_dot2) and b = E + O (v_sad_u8); a frame owns the whole chunks from the one
// holding its first byte up to the next frame's, and lane j (= frame j) adds its owned
// chunks' a and b through two wave prefix sums (differences: exact, the reference's
// wrapping uint32 arithmetic).  Once per frame: the bytes before its start in the first chunk
// and past its end in the last (or its tail in the next frame's first chunk) are corrected
// from those two chunks (kept in LDS), and an odd start swaps the pairing:
// O = (a - b) / 255, E = b - O, sum = O + 256 E (exact: a frame < 64 KiB never wraps a).
// Fused modes: a chunk inside a frame's first HW chunks is also written to its LDS
// head-window row (the owner frame: a ballot of the chunks holding a frame's first byte +
// mbcnt), so the header is parsed from LDS as before; the region (transport) sum is the total
// minus the bytes before the region (Ethernet / IPv6 headers) and after it (padding).
template <bool RAWM>
struct StreamLds {
    uint16_t mk[512];      // batch markers, chunk c: low byte = frame + 1 whose first byte, high = last byte is in c
    uint4 tbuf[64];        // frame j's last chunk
    uint4 hbuf[64];        // frame j's first chunk (RAW; the fused modes have it in the head-window row)
};
template <>
struct StreamLds<false> {
    uint16_t mk[512];
    uint4 tbuf[64];
};
template <bool STREAM, bool RAWM>
struct StreamSmem {
    StreamLds<RAWM> s;
};
template <bool RAWM>
struct StreamSmem<false, RAWM> {
    uint32_t s;
};

// Dense: every frame of the wave in bounds, >= 16 bytes and < 64 KiB, each starting at or after
// the previous one's end and less than 16 bytes behind it, and an even IPv6 network-header
// length in the seed (MODE 2 / 3: the transport pairing is the frame's).  Wave-uniform.
template <int MODE>
__device__ __forceinline__ bool wave_dense(const FlatArgs& p, uint32_t lane, uint32_t cnt, bool oob, uint64_t off,
                                           uint32_t len, uint32_t seed) {
    const int prev = (int)(lane ? lane - 1u : 0u);
    const uint64_t poff = ((uint64_t)(uint32_t)__shfl((int)(uint32_t)(off >> 32), prev) << 32) |
                          (uint32_t)__shfl((int)(uint32_t)off, prev);
    const uint32_t plen = (uint32_t)__shfl((int)len, prev);
    bool ok = lane >= cnt || (!oob && len >= 16u && len < 65536u &&
                              (lane == 0 || (off >= poff + plen && off < poff + plen + 16u)));
    if (MODE == 2 || MODE == 3) ok = ok && (lane >= cnt || (seed & 1u) == 0u);
    return __builtin_amdgcn_ballot_w64(!ok) == 0;
}

// Masked sums of chunk v's bytes in [x0, x1) (positions from the batch's 16-byte line, absolute
// pairing): a = E + 256 O, b = E + O.
__device__ __forceinline__ void masked_ab(const uint4 v, uint32_t ch, uint32_t x0, uint32_t x1, uint32_t& a,
                                          uint32_t& b) {
    const uint32_t lo = x0 <= ch ? 0u : min(x0 - ch, 16u);
    const uint32_t hi = x1 <= ch ? 0u : min(x1 - ch, 16u);
    const uint64_t ALL = ~0ull;
    uint64_t m0 = lo >= 8u ? 0ull : (ALL << (8u * lo));
    m0 &= hi >= 8u ? ALL : ~(ALL << (8u * hi));
    uint64_t m1 = lo >= 16u ? 0ull : (lo <= 8u ? ALL : (ALL << (8u * (lo - 8u))));
    m1 &= hi >= 16u ? ALL : (hi <= 8u ? 0ull : ~(ALL << (8u * (hi - 8u))));
    const uint32_t x = v.x & (uint32_t)m0, y = v.y & (uint32_t)(m0 >> 32);
    const uint32_t z = v.z & (uint32_t)m1, w = v.w & (uint32_t)(m1 >> 32);
    a = dot2_add(w, dot2_add(z, dot2_add(y, dot2_add(x, 0u))));
    b = __builtin_amdgcn_sad_u8(w, 0u, __builtin_amdgcn_sad_u8(z, 0u, __builtin_amdgcn_sad_u8(y, 0u, __builtin_amdgcn_sad_u8(x, 0u, 0u))));
}

// The stream over a dense wave's span; returns lane j's frame total (pairing from the
// frame's start), fills the head-window rows (fused modes).
template <int MODE>
__device__ __forceinline__ uint32_t span_stream(const FlatArgs& p, StreamLds<MODE == 0>& T, uint4* stage,
                                                uint32_t lane, uint32_t cnt, uint64_t off, uint32_t len) {
    const uint64_t a0 = reinterpret_cast<uintptr_t>(p.base) + off;
    const uint64_t B = (((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(a0 >> 32)) << 32) |
                        (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)a0)) & ~(uint64_t)15;
    const bool fr = lane < cnt;
    const uint32_t s = fr ? (uint32_t)(a0 - B) : 0u, e = fr ? s + len : 16u;
    const uint32_t E = (uint32_t)__builtin_amdgcn_readlane((int)e, (int)cnt - 1);
    const uint32_t fc = s >> 4, tc = (e - 1u) >> 4;                  // first / last chunk
    const uint32_t nfc = (uint32_t)__shfl((int)fc, (int)min(lane + 1u, 63u));
    const uint32_t oe = lane + 1u < cnt ? nfc : tc + 1u;               // owned chunks [fc, oe)
    reinterpret_cast<uint4*>(T.mk)[lane] = make_uint4(0, 0, 0, 0);
    uint8_t* mk8 = reinterpret_cast<uint8_t*>(T.mk);
    const uint32_t nsteps = (E + 1023u) >> 10;
    const Window w = make_window(B, (E + 15u) & ~15u);
    uint32_t accA = 0u, accB = 0u, carry = 0u;
    asm volatile("" ::: "memory");
    // one batch = 8 steps (8 KiB) of loads in flight (loads past the span read zeros without a
    // memory access)
    auto load_batch = [&](uint4 (&v)[8], uint32_t tb) {
#pragma unroll
        for (uint32_t k = 0; k < 8u; ++k) v[k] = load_win<false>(w, ((tb << 6) + 64u * k + lane) << 4);
    };
    auto sum_batch = [&](const uint4 (&v)[8], uint32_t tb) {
        const uint32_t cb = tb << 6;                              // the batch's first chunk
        if (fr && fc >= cb && fc < cb + 512u) mk8[2u * (fc - cb)] = (uint8_t)(lane + 1u);
        if (fr && tc >= cb && tc < cb + 512u) mk8[2u * (tc - cb) + 1u] = (uint8_t)(lane + 1u);
        asm volatile("" ::: "memory");
#pragma unroll
        for (uint32_t k = 0; k < 8u; ++k) {
            const uint32_t ci = cb + 64u * k + lane;
            const uint32_t m = T.mk[64u * k + lane];
            T.mk[64u * k + lane] = 0;
            const uint32_t hd = m & 0xFFu, tl = m >> 8;
            const uint64_t M = __builtin_amdgcn_ballot_w64(hd != 0u);
            const uint32_t below = __builtin_amdgcn_mbcnt_hi((uint32_t)(M >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)M, 0u));
            const uint32_t f = min(carry + below + (hd ? 1u : 0u), 64u) - 1u;   // the owner (last frame started)
            carry += (uint32_t)__builtin_popcountll(M);
            const uint4 x = v[k];
            const uint32_t a = dot2_add(x.w, dot2_add(x.z, dot2_add(x.y, dot2_add(x.x, 0u))));
            const uint32_t b = __builtin_amdgcn_sad_u8(x.w, 0u, __builtin_amdgcn_sad_u8(x.z, 0u,
                               __builtin_amdgcn_sad_u8(x.y, 0u, __builtin_amdgcn_sad_u8(x.x, 0u, 0u))));
            if constexpr (MODE != 0) {
                const uint32_t t = tl ? tl - 1u : f;
                const uint32_t ffc = (uint32_t)__shfl((int)fc, (int)f), ftc = (uint32_t)__shfl((int)tc, (int)f);
                const uint32_t tfc = (uint32_t)__shfl((int)fc, (int)t);
                const uint32_t wi = ci - ffc, wt = ci - tfc;
                if (wi < HW && ci <= ftc) stage[f * HW + (wi ^ (f & (HW - 1u)))] = x;
                if (tl && t != f && wt < HW) stage[t * HW + (wt ^ (t & (HW - 1u)))] = x;
            } else {
                if (hd) T.hbuf[hd - 1u] = x;
            }
            if (tl) T.tbuf[tl - 1u] = x;
            const uint32_t PA = wave_scan_add(a), PB = wave_scan_add(b);
            const uint32_t bc = cb + 64u * k;
            const bool in = fr && fc < bc + 64u && oe > bc;
            const uint32_t lo = fc > bc ? fc - bc : 0u, hi = in ? min(oe - bc, 64u) : 1u;
            const int ih = (int)hi - 1, il = lo ? (int)lo - 1 : 0;
            const uint32_t PAh = (uint32_t)__shfl((int)PA, ih), PAl = (uint32_t)__shfl((int)PA, il);
            const uint32_t PBh = (uint32_t)__shfl((int)PB, ih), PBl = (uint32_t)__shfl((int)PB, il);
            if (in) {
                accA += PAh - (lo ? PAl : 0u);
                accB += PBh - (lo ? PBl : 0u);
            }
        }
        asm volatile("" ::: "memory");
    };
    // (two batches in flight -- the next one's loads issued before the current one is summed --
    // measured slower: C2 35.4 vs 32.6 us, the 1500-byte batch unchanged; profiles/r02u)
    for (uint32_t tb = 0; tb < nsteps; tb += 8u) {
        uint4 v[8];
        load_batch(v, tb);
        sum_batch(v, tb);
    }
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
    // the first chunk's bytes before the frame; the last chunk's bytes past it (owned) or the
    // frame's tail in the next frame's first chunk (not owned)
    uint4 H;
    if constexpr (MODE != 0) H = stage[lane * HW + (lane & (HW - 1u))];
    else H = T.hbuf[lane];
    const uint4 L = T.tbuf[lane];
    uint32_t ca, cbs;
    masked_ab(H, 16u * fc, 16u * fc, s, ca, cbs);
    accA -= ca;
    accB -= cbs;
    if (tc < oe) {
        masked_ab(L, 16u * tc, e, 16u * tc + 16u, ca, cbs);
        accA -= ca;
        accB -= cbs;
    } else {
        masked_ab(L, 16u * tc, 16u * tc, e, ca, cbs);
        accA += ca;
        accB += cbs;
    }
    if (s & 1u) {                                                 // odd start: the swapped pairing
        const uint32_t o = (uint32_t)(((uint64_t)(accA - accB) * 0x80808081ull) >> 39);
        return o + 256u * (accB - o);
    }
    return accA;
}

// MODE: 0 RAW (p.crc_off / p.flags / p.out / p.bad), 1 fused IPv4, 2 fused IPv6,
// 3 Ethernet front end (per frame: destination filter, ethertype -> IPv4 / IPv6 / ARP / drop;
// pico_ethernet.c:180-235) -- IPv4 / IPv6 outputs in Ipv4Args-compatible fields of FlatArgs.
// Phase 4: lane `lane` finalizes its frame (output index idx) from the LDS state.
template <int MODE>
__device__ __forceinline__ void sorted_finish(const FlatArgs& p, SortedWaveLds& L, uint32_t lane, uint64_t idx,
                                              bool tx) {
    asm volatile("" ::: "memory");
    const uint32_t acc_all = L.acc_all[lane], acc_x = L.acc_x[lane], acc_opt = L.acc_opt[lane];
    const uint4 info = L.info[lane], fin = L.fin[lane];
    const uint32_t xpos = L.xo[lane].x;
    const uint32_t r = info.w & 15u;
    uint8_t* fp = p.base + (((((uint64_t)info.y) << 32) | info.x) + r);
    uint32_t verdict = fin.x & 15u;
    const bool parsed = fin.x & 16u, l4_needed = fin.x & 32u, oob = fin.x & 64u;
    const bool fam6 = MODE == 2 || (MODE == 3 && (fin.x & 128u));
    const uint32_t proto = (fin.x >> 8) & 0xFFu, tl = fin.x >> 16;
    const uint32_t hl = fin.y & 0xFFu, l2v = (fin.y >> 8) & 0xFFu, ipcrc = fin.y >> 16;
    const uint32_t pseudo = fin.z, seed = fin.z, hdr20 = fin.w;
    if constexpr (MODE == 0) {
        uint32_t ret = 0;
        if (oob) {
            if (p.bad) atomicAdd(p.bad, 1u);
        } else {
            ret = finalize(seed + acc_all - acc_x);
            if ((p.flags & 1u) && xpos != NONE) store_crc(fp + p.crc_off, ret);
        }
        p.out[idx] = (uint16_t)ret;
    } else {
        uint32_t net = 0, l4 = 0;
        if (MODE == 3 && l2v) {
            verdict = l2v;                   // dropped by the Ethernet layer, or ARP: no checksum
        } else if (fam6) {
            if (parsed) {
                if (l4_needed) {
                    if (!tx && (p.flags & F_REFD) && (proto == 6u || proto == 17u)) {
                        // pico_socket.c:1919-1958 with net_hdr->proto = byte 9 of the IPv6 header
                        if (ipcrc == 6u || (ipcrc == 17u && acc_x != 0u)) {
                            l4 = finalize(pseudo - (proto << 8) + (ipcrc << 8) + acc_all);
                            if (l4 != 0) verdict |= V_L4_BAD;
                        }
                    } else if (!tx) {
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
                store_crc(fp + (proto == 6u ? 16u : proto == 17u ? 6u : 2u), l4);
            if (MODE == 3) verdict |= V_IPV6;
        } else {
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
            if (tx && (p.flags & 0x401u) == 1u && verdict == V_ACCEPT) {   // 0x400: ablation
                store_crc(fp + 10, net);
                if ((proto == 6u || proto == 1u) && l4_needed) store_crc(fp + hl + (proto == 6u ? 16u : 2u), l4);
                else if (proto == 17u && tl >= 8u) store_crc(fp + hl + 6u, 0u);
            }
        }
        if (MODE != 2 && p.out_net) p.out_net[idx] = (uint16_t)net;
        if (p.out_l4) p.out_l4[idx] = (uint16_t)l4;
        if (p.verdict) p.verdict[idx] = (uint8_t)verdict;
    }
}

// The NW little-endian dwords at byte position pos of a frame's head window (pos < 16, or
// pos < 32 with SHIFT): whole-chunk shift, then a 4-way dword select and alignbyte.
template <int NW, bool SHIFT>
__device__ __forceinline__ void window_words(const uint4 (&hw)[HW], uint32_t pos, uint32_t (&H)[NW]) {
    constexpr int NC = (4 * (NW + 4) + 15) / 16;      // chunks the selects below may touch
    static_assert(NC + (SHIFT ? 1 : 0) <= (int)HW, "head window too small");
    // a bit-mask blend, not `s1 ? hw[c + 1] : hw[c]` (which LLVM turns into a dynamic index
    // into hw -- the array then lives in scratch memory)
    const uint32_t s1 = SHIFT && pos >= 16u ? 0xFFFFFFFFu : 0u;
    uint32_t D[4 * NC];
#pragma unroll
    for (int c = 0; c < NC; ++c) {
        const uint4 a = hw[c], b = hw[SHIFT ? c + 1 : c];
        D[4 * c] = (a.x & ~s1) | (b.x & s1);
        D[4 * c + 1] = (a.y & ~s1) | (b.y & s1);
        D[4 * c + 2] = (a.z & ~s1) | (b.z & s1);
        D[4 * c + 3] = (a.w & ~s1) | (b.w & s1);
    }
    const uint32_t q = (pos >> 2) & 3u, sh = pos & 3u;
    uint32_t E[NW + 1];
#pragma unroll
    for (int m = 0; m <= NW; ++m) E[m] = sel4(q, D[m], D[m + 1], D[m + 2], D[m + 3]);
#pragma unroll
    for (int m = 0; m < NW; ++m) H[m] = __builtin_amdgcn_alignbyte(E[m + 1], E[m], sh);
}

// CPL 8 keeps 8 KiB of loads in flight per wave within 128 VGPRs (4 waves per
// SIMD: a 256K-frame batch at 64 frames per wave is one residency round); CPL 4
// fits 64 VGPRs (8 waves per SIMD).
template <int MODE, bool NT, int CPL, bool SMALL, bool STREAM>
__device__ __forceinline__ void sorted_batch(const FlatArgs& p, SortedWaveLds& L, uint4* stage, StreamSmem<STREAM, MODE == 0>& SS,
                                             uint32_t lane, uint64_t f0) {
    constexpr bool IPV4 = MODE == 1, IPV6 = MODE == 2, ETH = MODE == 3;
    const uint32_t cnt = (uint32_t)min((uint64_t)p.fpw, (uint64_t)p.n - f0);
    const bool tx = MODE != 0 && (p.flags & 2u) != 0;

    // ---- 1. lane j = frame j
    uint4 dcur = make_uint4(0, 0, 0, 0);
    if (lane < cnt) dcur = *reinterpret_cast<const uint4*>(p.desc + f0 + lane);
    uint64_t off = ((uint64_t)dcur.y << 32) | dcur.x;
    uint32_t len = lane < cnt ? dcur.z : 0u;
    const uint32_t seed = dcur.w;
    const bool oob = lane < cnt && (off > p.base_len || len > p.base_len - off);
    if (oob || lane >= cnt) { len = 0; off = 0; }
    uint8_t* fp = p.base + off;
    uint32_t r = (uint32_t)(reinterpret_cast<uintptr_t>(fp) & 15u);
    uint64_t a0off = off - r;
    uint32_t odd = r & 1u;
    const uint32_t r_desc = r;                   // the descriptor's start in its head window

    // dense waves: the span stream (phase 1 then parses from the rows it filled; no rounds)
    bool dense = false;
    uint32_t total = 0;
    if constexpr (STREAM) {
        dense = wave_dense<MODE>(p, lane, cnt, oob, off, len, seed);
        if (dense) total = span_stream<MODE>(p, SS.s, stage, lane, cnt, off, len);
    }

    uint32_t span = 0, ext = 0, xpos = NONE, optend = 0;
    uint32_t verdict = V_MALFORMED, hl = 0, tl = 0, proto = 0, ipcrc = 0, pseudo = 0, hdr20 = 0, l2v = 0;
    bool parsed = false, l4_needed = false, is6 = false;
    const uint64_t a0h = a0off;                  // the head window's first chunk (fused modes)
    uint4 hw[HW];
    uint32_t nlh = 0;                            // head-window chunks loaded
    bool staged = false;                         // the window also sits in this lane's LDS row
    uint32_t k0 = 0, p_all = 0, p_x = 0, p_opt = 0;
    if constexpr (MODE == 0) {
        span = ext = len;
        if (p.crc_off >= 0 && (uint64_t)p.crc_off + 2u <= len) xpos = r + (uint32_t)p.crc_off;
    } else {
        // the head window: the frame's first HW chunks (128 bytes from the header's
        // 16-byte line), loaded once here.  They hold the header (parsed below), the
        // usual isolated 2-byte field and the IPv4 options, and, for small datagrams
        // (64-byte IMIX frames), the whole datagram: their sums are taken here and the
        // rounds start behind the window (or are skipped).
        constexpr uint32_t HDR = IPV6 ? 40u : IPV4 ? 20u : 14u;
        nlh = len >= HDR && !(p.flags & 0x200u) ? min(HW, (r + len + 15u) >> 4) : 0u;   // 0x200: ablation
        if (STREAM && dense) {
#pragma unroll
            for (uint32_t i = 0; i < HW; ++i) hw[i] = stage[lane * HW + (i ^ (lane & (HW - 1)))];
            staged = true;
            asm volatile("" ::: "memory");
        } else {
            // Buffer loads through a window over the batch (from base's 16-byte line to
            // base_len rounded up -- the bytes load_chunk may touch -- at most 2 GiB, from
            // 1 GiB below the wave's first frame): all HW slots issue back to back and
            // slots past the frame read zeros.  (`i < nlh ? load : 0` compiled to branched
            // flat loads with a vmcnt(0) behind the second: two dependent HBM round trips
            // per wave.)  A frame outside the window (a wave spanning > 1 GiB of a batch
            // over 2 GiB) is loaded in a second, branched pass.
            const uint8_t* a0 = p.base + a0off;
            const uint64_t a0a = reinterpret_cast<uintptr_t>(a0);
            const uint64_t wb = reinterpret_cast<uintptr_t>(p.base) & ~(uint64_t)15;
            const uint64_t wn = (reinterpret_cast<uintptr_t>(p.base) + p.base_len + 15u - wb) & ~(uint64_t)15;
            const uint64_t act = __builtin_amdgcn_ballot_w64(nlh != 0);
            const int first = act ? __builtin_ffsll((long long)act) - 1 : 0;
            const uint64_t anchor = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(a0a >> 32), first) << 32) |
                                    (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)a0a, first);
            const uint64_t lo = anchor >= wb + (1ull << 30) ? anchor - (1ull << 30) : wb;
            const uint64_t wsz = min(wn - min(lo - wb, wn), (uint64_t)0x7FFFFFF0u);
            const bool inside = a0a >= lo && a0a - lo + 16u * nlh <= wsz;
            staged = inside;
            const Window w = make_window(lo, (uint32_t)wsz);
            const uint32_t v0 = (uint32_t)(a0a - lo);
            const uint32_t nin = inside ? nlh : 0u;
            // Transposed: load k covers frames FPL*k .. FPL*k+FPL-1 with HW lanes each, so one
            // instruction reads FPL whole 128-byte windows (a lane per frame touched 64
            // lines per instruction and re-fetched each line for every chunk: L1 thrash).
            // The chunks meet their frame's lane through LDS (row g holds chunk c in slot
            // c ^ (g & 7): 8 lanes reading chunk i of 8 rows hit 8 different bank groups).
            constexpr uint32_t FPL = 64u / HW;
            const uint32_t gi = lane / HW, ci = lane % HW;
            uint4 t[HW];
#pragma unroll
            for (uint32_t k = 0; k < HW; ++k) {
                const uint32_t g = FPL * k + gi;
                const uint32_t gv0 = (uint32_t)__shfl((int)v0, (int)g);
                const uint32_t gn = (uint32_t)__shfl((int)nin, (int)g);
                t[k] = load_win<PICO_HW_NT != 0>(w, ci < gn ? gv0 + 16u * ci : WIN_OOB);
            }
#pragma unroll
            for (uint32_t k = 0; k < HW; ++k) {
                const uint32_t g = FPL * k + gi;
                stage[g * HW + (ci ^ (g & (HW - 1)))] = t[k];
            }
            __builtin_amdgcn_wave_barrier();
#pragma unroll
            for (uint32_t i = 0; i < HW; ++i) hw[i] = stage[lane * HW + (i ^ (lane & (HW - 1)))];
            // the staging rows alias the wave's SortedWaveLds (written at the end of phase 1)
            asm volatile("" ::: "memory");
            if (__builtin_amdgcn_ballot_w64(!inside && nlh != 0)) {
#pragma unroll
                for (uint32_t i = 0; i < HW; ++i)
                    if (!inside && i < nlh) hw[i] = load_chunk(a0, i);
            }
        }
        // MODE 3: the Ethernet header first (pico_ethernet_receive / pico_eth_receive,
        // pico_ethernet.c:180-235), then the IP header at +14 (the region moves there).
        uint32_t fam = IPV6 ? 6u : 4u, pos = r, avail = len;
        if constexpr (ETH) {
            fam = 0;
            if (len >= 14u) {
                uint32_t M[2], T[1];
                window_words<2, true>(hw, r, M);
                window_words<1, true>(hw, r + 12u, T);
                const uint32_t m0 = M[0], m1 = M[1] & 0xFFFFu, et = T[0] & 0xFFFFu;   // ethertype, LE word
                const bool mine = !(p.flags & F_MACF) || tx || (m0 == p.mac_lo && m1 == p.mac_hi) ||
                                  (m0 & 0xFFFFFFu) == 0x5E0001u || (m0 & 0xFFFFu) == 0x3333u ||
                                  (m0 == 0xFFFFFFFFu && m1 == 0xFFFFu);
                if (!mine) l2v = V_DROP_L2;
                else if (et == 0x0608u) l2v = V_ARP;          // 0x0806 -> pico_arp_receive
                else if (et == 0x0008u) fam = 4u;             // 0x0800
                else if (et == 0xDD86u) fam = 6u;             // 0x86DD
                else l2v = V_DROP_L2;
                if (fam) {
                    pos = r + 14u;
                    off += 14u;
                    avail = len - 14u;
                    fp = p.base + off;
                    r = (uint32_t)(reinterpret_cast<uintptr_t>(fp) & 15u);
                    a0off = off - r;
                    odd = r & 1u;
                    uint32_t V[1];
                    window_words<1, true>(hw, pos, V);
                    // IS_IPV4 / IS_IPV6 (pico_ethernet.c:145,164); no byte to read: MALFORMED
                    if (avail == 0u) fam = 0;
                    else if ((V[0] & 0xF0u) != (fam << 4)) { fam = 0; l2v = V_DROP_L2; }
                }
            }
        }
        if (IPV4 || (ETH && fam == 4u)) {
            if (avail >= 20) {
                uint32_t H[5];
                window_words<5, ETH>(hw, pos, H);
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
        } else if (IPV6 || (ETH && fam == 6u)) {
            if (avail >= 40) {
                uint32_t H[10];
                window_words<10, ETH>(hw, pos, H);
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
                        // F_REF_DISPATCH: pico_transport_crc_check's proto is byte 9 (kept in ipcrc)
                        ipcrc = (H[2] >> 8) & 0xFFu;
                        const bool ref17 = (p.flags & F_REFD) && ipcrc == 17u;
                        if (proto == 6u && !ref17) {
                            l4_needed = true;
                        } else if (proto == 17u || proto == 6u) {   // the UDP crc field is read
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
                        off += net_len;
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
        is6 = fam == 6u;
    }
    const uint64_t nch64 = ext ? ((uint64_t)r + ext + 15u) >> 4 : 0u;
    uint32_t nch = (uint32_t)min(nch64, (uint64_t)0xFFFFFFFFu);
    if constexpr (STREAM && MODE == 0) {
        if (dense) {
            p_all = total;
            if (xpos != NONE) {                  // the crc field's word (crc_off even: frame pairing)
                const uint8_t* q = p.base + a0off + xpos;
                p_x = (uint32_t)q[0] | ((uint32_t)q[1] << 8);
            }
            nch = 0;
        }
    }
    if constexpr (STREAM && MODE != 0) {
        if (dense) {
            // window coordinates (origin a0h): the descriptor's bytes [r_desc, r_desc + len), the
            // region [rs, rs + span); region = total - the bytes before it - the bytes after it
            // (even offsets apart: one pairing throughout)
            const uint32_t d = (uint32_t)((a0off - a0h) >> 4);
            const uint32_t rs = 16u * d + r, sl = odd ? SEL_ODD : SEL_EVEN;
            const uint32_t e0 = r_desc + len;
            auto range_sum = [&](uint32_t x0, uint32_t x1) {
                uint32_t acc = 0;
#pragma unroll
                for (uint32_t i = 0; i < HW; ++i)
                    if (x1 > x0 && 16u * i < x1 && 16u * i + 16u > x0) acc += masked_chunk_sum<true>(hw[i], 16u * i, x0, x1, sl);
                if (x1 > x0 && x1 > 16u * HW)
                    for (uint32_t k = max(HW, x0 >> 4); 16u * k < x1; ++k)
                        acc += masked_chunk_sum<true>(load_chunk(p.base + a0h, k), 16u * k, x0, x1, sl);
                return acc;
            };
            const bool cut = parsed && (rs > r_desc || rs + span < e0);
            uint32_t c = 0;
            if (__builtin_amdgcn_ballot_w64(cut)) {
                if (cut) c = range_sum(r_desc, rs) + range_sum(rs + span, e0);
            }
            p_all = total - c;
            if (xpos != NONE) {
                const uint32_t xs = 16u * d + xpos;
                if (xs + 2u <= 16u * HW) {
                    const uint8_t* row = reinterpret_cast<const uint8_t*>(stage + lane * HW);
                    const uint32_t sw = (lane & (HW - 1)) << 4;
                    p_x = (uint32_t)row[xs ^ sw] | ((uint32_t)row[(xs + 1u) ^ sw] << 8);
                } else {
                    const uint8_t* q = p.base + a0h + xs;
                    p_x = (uint32_t)q[0] | ((uint32_t)q[1] << 8);
                }
            }
            if (__builtin_amdgcn_ballot_w64(optend != 0u)) {      // IPv4 options (always inside the window)
                if (optend != 0u) p_opt = range_sum(rs + 20u, 16u * d + optend);
            }
            asm volatile("" ::: "memory");
            xpos = NONE;
            optend = 0;
            nch = 0;
        }
    }
    if (MODE != 0 && !(STREAM && dense)) {
        // sums over the head window: the region's chunks [0, k0) = window chunks
        // [d, d + k0) (d: where the region's chunk grid starts in the window -- IPv6:
        // behind the header); the rounds take region chunks [k0, nch).  A field
        // straddling the cut moves the cut down a chunk (a field is summed whole on one
        // side); options not inside the window (never, for IPv4) leave it all to the rounds.
        const uint32_t d = (uint32_t)min((a0off - a0h) >> 4, (uint64_t)HW);
        k0 = nlh > d ? min(nlh - d, nch) : 0u;
        if (xpos != NONE && xpos < 16u * k0 && xpos + 2u > 16u * k0) k0 = xpos >> 4;
        if (optend != 0u && optend > 16u * k0) k0 = 0;     // options: all in the window part, or all in the rounds
        // window coordinates: the region's window part is [rs, re), chunks [d, d + k0)
        const uint32_t P = 16u * (d + k0), rs = 16u * d + r;
        const uint32_t re = min(rs + span, P);
        const bool xin = xpos != NONE && xpos + 2u <= 16u * k0;
        const uint32_t xs = 16u * d + xpos;
        const bool oin = optend != 0u && k0 != 0u;
        const uint32_t sl = odd ? SEL_ODD : SEL_EVEN;
        // p_all: whole-chunk sums of chunks [d, d + k0), minus the bytes of the first chunk
        // before rs and of the last chunk from re on.  The two edge chunks come from the LDS
        // stage (one ds_read each).  Against one masked sum per window chunk: -14 % VALU
        // instructions per wave, C2 -1.5 % (r02d, profiles/r02d).
        auto edge_chunk = [&](uint32_t idx) {      // bit-mask blends (a select chain becomes a scratch array)
            uint4 v = make_uint4(0, 0, 0, 0);
#pragma unroll
            for (uint32_t i = 0; i < HW; ++i) {
                const uint32_t m = idx == i ? 0xFFFFFFFFu : 0u;
                v.x |= hw[i].x & m; v.y |= hw[i].y & m; v.z |= hw[i].z & m; v.w |= hw[i].w & m;
            }
            return v;
        };
        auto window_sums = [&](auto perm_tag) {
            constexpr bool PERM = decltype(perm_tag)::value;
#pragma unroll
            for (uint32_t i = 0; i < HW; ++i) {
                const uint32_t c = add_full<PERM>(hw[i], sl, 0u);
                p_all += (i >= d && i < d + k0) ? c : 0u;
            }
            if (__builtin_amdgcn_ballot_w64(k0 != 0u)) {
                const uint32_t e0 = k0 ? d : 0u, e1 = k0 ? d + k0 - 1u : 0u;
                uint4 h0, h1;
                if (__builtin_amdgcn_ballot_w64(k0 != 0u && !staged) == 0) {
                    h0 = stage[lane * HW + (e0 ^ (lane & (HW - 1)))];
                    h1 = stage[lane * HW + (e1 ^ (lane & (HW - 1)))];
                } else {
                    h0 = edge_chunk(e0);
                    h1 = edge_chunk(e1);
                }
                if (k0) {
                    p_all -= masked_chunk_sum<PERM>(h0, 16u * e0, 16u * e0, rs, sl);
                    p_all -= masked_chunk_sum<PERM>(h1, 16u * e1, re, P, sl);
                }
            }
        };
        if (__builtin_amdgcn_ballot_w64(k0 != 0u && odd)) window_sums(std::integral_constant<bool, true>{});
        else window_sums(std::integral_constant<bool, false>{});
        if (__builtin_amdgcn_ballot_w64(oin || (xin && !staged))) {     // IPv4 options / > 2 GiB batches
#pragma unroll
            for (uint32_t i = 0; i < HW; ++i) {
                if (i >= d && i < d + k0) {
                    if (xin && !staged) p_x += masked_chunk_sum<true>(hw[i], 16u * i, xs, xs + 2u, sl);
                    if (oin) p_opt += masked_chunk_sum<true>(hw[i], 16u * i, rs + 20u, 16u * d + optend, sl);
                }
            }
        }
        // The isolated field is one word of the region's pairing: whatever the start's
        // parity, its share is byte[xs] | byte[xs+1] << 8 in the accumulators' (byte-
        // swapped) domain -- two LDS byte reads instead of HW masked sums.
        if (xin && staged) {
            const uint8_t* row = reinterpret_cast<const uint8_t*>(stage + lane * HW);
            const uint32_t sw = (lane & (HW - 1)) << 4, x1 = xs + 1u;   // chunk slots are XOR-swizzled
            p_x = (uint32_t)row[xs ^ sw] | ((uint32_t)row[x1 ^ sw] << 8);
        }
        asm volatile("" ::: "memory");   // stage rows are read before the state below overwrites them
        if (xin) xpos = NONE;
        else if (xpos != NONE) xpos -= 16u * k0;
        if (oin) optend = 0;
        nch -= k0;
    }
    L.acc_all[lane] = p_all;
    L.acc_x[lane] = p_x;
    L.acc_opt[lane] = p_opt;
    L.nch[lane] = nch;
    L.info[lane] = make_uint4((uint32_t)a0off, (uint32_t)(a0off >> 32), r + span, r | (odd << 4) | (k0 << 5));
    L.xo[lane] = make_uint2(xpos, optend);
    L.fin[lane] = make_uint4(verdict | (parsed ? 16u : 0u) | (l4_needed ? 32u : 0u) | (oob ? 64u : 0u) |
                                 (is6 ? 128u : 0u) | (proto << 8) | (tl << 16),
                             hl | (l2v << 8) | (ipcrc << 16), MODE == 0 ? seed : pseudo, hdr20);
    const bool any_odd = __builtin_amdgcn_ballot_w64(nch != 0 && odd) != 0;
    const bool any_xo = __builtin_amdgcn_ballot_w64(nch != 0 && (xpos != NONE || optend != 0)) != 0;

    STAMP(1);
    // ---- 2. order the frames by size class (the narrowest round width that covers
    //         them in one pass): ballots and bit counts, no data movement but one
    //         LDS store per frame
    // classes by round width: (SMALL: 1,) 4, 8, 16, 32, 64 lanes; NC = no data
    constexpr uint32_t NC = SMALL ? 6u : 5u;
    const uint32_t cw = nch <= 4u * CPL ? 0u : nch <= 8u * CPL ? 1u : nch <= 16u * CPL ? 2u : nch <= 32u * CPL ? 3u : 4u;
    const uint32_t cls = nch == 0 ? NC : SMALL ? (nch <= (uint32_t)CPL ? 0u : cw + 1u) : cw;
    uint64_t bal[NC];
#pragma unroll
    for (uint32_t c = 0; c < NC; ++c) bal[c] = __builtin_amdgcn_ballot_w64(cls == c);
    uint32_t e[5] = {0, 0, 0, 0, 0};     // e[c] = frames of class <= c
    e[0] = (uint32_t)__builtin_popcountll(bal[0]);
#pragma unroll
    for (uint32_t c = 1; c + 1 < NC; ++c) e[c] = e[c - 1] + (uint32_t)__builtin_popcountll(bal[c]);
    const uint32_t m = e[NC - 2] + (uint32_t)__builtin_popcountll(bal[NC - 1]);
    if (cls < NC) {
        uint64_t mine = bal[0];
        uint32_t start = 0;
#pragma unroll
        for (uint32_t c = 1; c < NC; ++c) {
            mine = cls == c ? bal[c] : mine;
            start = cls == c ? e[c - 1] : start;
        }
        const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(mine >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mine, 0u));
        L.order[start + rank] = lane;
    }
    __builtin_amdgcn_wave_barrier();

    // ---- 3. rounds over the sorted frames
    RawArgs ra{p.base, p.base_len, nullptr, 0, 0, 0, 0, -1, 0u, 0u, nullptr, nullptr};
    // ablation only (PICO_CSUM_ABLATE): flags bit 8 skips the rounds (times phases 1, 2, 4);
    // bit 9 skips the head-window loads (then nothing parses: descriptors + stores alone);
    // bit 10 skips the IPv4 TX in-place crc writes
    if (m && !(p.flags & 0x100u)) {
        if (any_odd) {
            if (any_xo) sorted_rounds<CPL, true, NT, true, SMALL>(ra, L, e, m);
            else sorted_rounds<CPL, true, NT, false, SMALL>(ra, L, e, m);
        } else {
            if (any_xo) sorted_rounds<CPL, false, NT, true, SMALL>(ra, L, e, m);
            else sorted_rounds<CPL, false, NT, false, SMALL>(ra, L, e, m);
        }
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0)

    STAMP(2);
    // ---- 4. lane j finalizes frame j (state reloaded from LDS)
    if (lane < cnt) sorted_finish<MODE>(p, L, lane, f0 + lane, tx);
    __builtin_amdgcn_wave_barrier();
}

// One wave per batch of up to 64 frames.  (A persistent grid looping over batches
// measured slower: every wave repeats the same serial descriptor -> rounds chain.)
#ifndef PICO_SORTED_WPB
#define PICO_SORTED_WPB 4    // waves per workgroup (A/B builds: 8)
#endif
template <int MODE, bool NT, int CPL, bool SMALL = false, bool STREAM = false>
__global__ __launch_bounds__(64 * PICO_SORTED_WPB, CPL >= 8 || MODE != 0 ? 4 : 5) void csum_sorted_kernel(FlatArgs p) {
    __shared__ SortedWaveSmem<MODE != 0> lds_all[PICO_SORTED_WPB];
    __shared__ StreamSmem<STREAM, MODE == 0> lds_stream[PICO_SORTED_WPB];
    const uint32_t lane = threadIdx.x & 63u;
    SortedWaveSmem<MODE != 0>& S = lds_all[threadIdx.x >> 6];
    const uint64_t f0 = ((uint64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) * p.fpw;
    STAMP(0);
    if (f0 < p.n) sorted_batch<MODE, NT, CPL, SMALL, STREAM>(p, S.s, S.stage, lds_stream[threadIdx.x >> 6], lane, f0);
    STAMP(3);
}

#if SORTED_MODE == 0
// ---------------------------------------------------------------- IPv4 forwarding step
//
// pico_ipv4_forward (modules/pico_ipv4.c:1547-1556) on a batch of datagrams that are
// routed through this host: hdr->ttl = ttl - 1 (written back whatever follows);
// ttl < 1 -> expired (pico_notify_ttl_expired, the frame is dropped, crc untouched);
// else hdr->crc++ -- the reference's "HACK: increase crc to compensate decreased
// TTL": a native (little-endian) uint16 increment of the stored big-endian field.
// That is the incremental update of RFC 1141 (+0x0100 on the checksum for -1 on the
// TTL byte) except where it carries out of the first byte, and it is kept exactly
// so, bit-compatible with the reference.  One lane per datagram; the 4 bytes at
// header offset 8..11 (ttl, proto, crc) are read and written, nothing else.
struct FwdArgs {
    uint8_t* base;
    uint64_t base_len;
    const pico_csum_desc_dev* desc;
    uint32_t n;
    uint8_t* verdict;
};

__global__ __launch_bounds__(256) void ipv4_forward_kernel(FwdArgs p) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= p.n) return;
    const uint4 d = *reinterpret_cast<const uint4*>(p.desc + i);
    const uint64_t off = ((uint64_t)d.y << 32) | d.x;
    uint32_t v = V_MALFORMED;
    if (off <= p.base_len && d.z <= p.base_len - off && d.z >= 20u) {
        uint8_t* h = p.base + off;
        const uint8_t ttl = (uint8_t)(h[8] - 1u);
        h[8] = ttl;
        if (ttl < 1u) {
            v = V_EXPIRED;
        } else {
            const uint32_t crc = (uint32_t)h[10] | ((uint32_t)h[11] << 8);
            const uint32_t inc = (crc + 1u) & 0xFFFFu;
            h[10] = (uint8_t)inc;
            h[11] = (uint8_t)(inc >> 8);
            v = V_ACCEPT;
        }
    }
    if (p.verdict) p.verdict[i] = (uint8_t)v;
}


#endif

}  // namespace

#define SORTED_CAT2(a, b) a##b
#define SORTED_CAT(a, b) SORTED_CAT2(a, b)

extern "C" {

#ifdef PICO_CSUM_STAMPS
int SORTED_CAT(pico_csum_diag_stamps_mode, SORTED_MODE)(void* d_buf, uint32_t waves);
int SORTED_CAT(pico_csum_diag_stamps_mode, SORTED_MODE)(void* d_buf, uint32_t waves) {
    uint64_t* b = static_cast<uint64_t*>(d_buf);
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), &b, sizeof(b)) != hipSuccess) return -1;
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_stamps_n), &waves, sizeof(waves)) != hipSuccess) return -1;
    return 0;
}
#if SORTED_MODE == 0
int pico_csum_diag_stamps_mode1(void*, uint32_t);
int pico_csum_diag_stamps_mode2(void*, uint32_t);
int pico_csum_diag_stamps_mode3(void*, uint32_t);
int pico_csum_diag_set_stamps(void* d_buf, uint32_t waves) {
    return pico_csum_diag_stamps_mode0(d_buf, waves) | pico_csum_diag_stamps_mode1(d_buf, waves) |
           pico_csum_diag_stamps_mode2(d_buf, waves) | pico_csum_diag_stamps_mode3(d_buf, waves);
}
#endif
#endif

// One kernel table per mode: this TU is compiled once per SORTED_MODE (parallel build).
#define SORTED_LAUNCH SORTED_CAT(pico_csum_sorted_launch_mode, SORTED_MODE)
int SORTED_LAUNCH(const void* args, uint32_t nt, int v, void* stream);
int SORTED_LAUNCH(const void* args, uint32_t nt, int v, void* stream) {
    const FlatArgs& a = *static_cast<const FlatArgs*>(args);
    using K = void (*)(FlatArgs);
    constexpr int M = SORTED_MODE;
    // [nt][cpl 4 | cpl 8 | cpl 8 + 1-lane | cpl 8 + 1-lane + span stream]
#define SK(t) {csum_sorted_kernel<M, t, 4>, csum_sorted_kernel<M, t, 8>, csum_sorted_kernel<M, t, 8, true>,       \
               csum_sorted_kernel<M, t, 8, true, true>}
    static const K table[2][4] = {SK(false), SK(true)};
#undef SK
    const uint64_t waves = ((uint64_t)a.n + a.fpw - 1) / a.fpw;
    hipLaunchKernelGGL(table[nt ? 1 : 0][v], dim3((unsigned)((waves + PICO_SORTED_WPB - 1) / PICO_SORTED_WPB)),
                       dim3(64 * PICO_SORTED_WPB), 0, static_cast<hipStream_t>(stream), a);
    return (int)hipGetLastError();
}

#if SORTED_MODE == 0
int pico_csum_sorted_launch_mode1(const void* args, uint32_t nt, int v, void* stream);
int pico_csum_sorted_launch_mode2(const void* args, uint32_t nt, int v, void* stream);
int pico_csum_sorted_launch_mode3(const void* args, uint32_t nt, int v, void* stream);

// Sorted-rounds descriptor kernel: mode 0 RAW, 1 fused IPv4, 2 fused IPv6, 3 Ethernet front end;
// small (cpl 8 only): 0 none, 1 the 1-lane class, 2 the 1-lane class + the span stream for dense waves.
// mac48 = the device MAC's 6 bytes (little-endian in a uint64), used when flags carry F_MACF
// (set by the host layer).
int pico_csum_launch_sorted(void* base, uint64_t base_len, const void* desc, uint32_t n, int mode, int32_t crc_off,
                            uint32_t flags, uint16_t* out, uint32_t* bad, uint16_t* out_net, uint16_t* out_l4,
                            uint8_t* verdict, uint32_t cpl, uint32_t nt, uint32_t fpw, uint32_t small,
                            uint64_t mac48, void* stream) {
    if (fpw < 1 || fpw > 64 || !(cpl == 4 || cpl == 8) || mode < 0 || mode > 3 || small > 2 || (small && cpl != 8))
        return (int)hipErrorInvalidValue;
    if (n == 0) return (int)hipSuccess;
    FlatArgs a{static_cast<uint8_t*>(base), base_len, static_cast<const pico_csum_desc_dev*>(desc), n, fpw,
               crc_off, flags, out, bad, out_net, out_l4, verdict, (uint32_t)mac48, (uint32_t)(mac48 >> 32)};
    const int v = cpl == 4 ? 0 : (int)small + 1;
    switch (mode) {
        case 0: return pico_csum_sorted_launch_mode0(&a, nt, v, stream);
        case 1: return pico_csum_sorted_launch_mode1(&a, nt, v, stream);
        case 2: return pico_csum_sorted_launch_mode2(&a, nt, v, stream);
        default: return pico_csum_sorted_launch_mode3(&a, nt, v, stream);
    }
}

int pico_csum_launch_ipv4_forward(void* base, uint64_t base_len, const void* desc, uint32_t n, uint8_t* verdict,
                                  void* stream) {
    if (n == 0) return (int)hipSuccess;
    FwdArgs a{static_cast<uint8_t*>(base), base_len, static_cast<const pico_csum_desc_dev*>(desc), n, verdict};
    const dim3 grid((unsigned)(((uint64_t)n + 255u) / 256u)), block(256);
    hipLaunchKernelGGL(ipv4_forward_kernel, grid, block, 0, static_cast<hipStream_t>(stream), a);
    return (int)hipGetLastError();
}
#endif  // SORTED_MODE == 0

}  // extern "C"

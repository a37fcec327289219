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
// Descriptor batches of any size mix, all modes (RAW / fused IPv4 / fused IPv6 / Ethernet).
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

// waves per workgroup: 8 measured the same on the sorted rounds (profiles/r02wpb); 1 the same and
// 2 slower on the stream (profiles/r04/ab_*_wave_workgroups.txt)
constexpr uint32_t WPB = 4;
constexpr uint32_t HW = 8;   // head-window chunks the fused modes load in phase 1 (temporal loads:
                             // non-temporal ones measured 5 % slower, profiles/r02nt)

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
// Stream-order waves for dense fused batches (stream_batch).  Product shape, measured
// (profiles/r03s3/README.md): 8 chunks per lane per step (8 KiB; StreamLds 10 KiB a wave, 4
// workgroups of 4 waves per CU), two steps in flight, non-temporal loads.
constexpr uint32_t SCPL = 8;                 // chunks per lane per step
#ifndef STREAM_LAST_NOPF
#define STREAM_LAST_NOPF 1
#endif
constexpr uint32_t SQ = 64u * SCPL;          // chunks per step
struct StreamLds {
    uint4 raw[SQ];           // the step's bytes, chunk slots swizzled (sslot)
    uint32_t pxc[SQ];        // exclusive prefix sum before each chunk, chunk order
};

template <bool STAGE>
union SortedWaveSmem {
    SortedWaveLds s;
    uint4 stage[64 * HW];
    StreamLds st;
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

// MODE: 0 RAW (p.crc_off / p.flags / p.out / p.bad), 1 fused IPv4, 2 fused IPv6,
// 3 Ethernet front end (per frame: destination filter, ethertype -> IPv4 / IPv6 / ARP / drop;
// pico_ethernet.c:180-235) -- IPv4 / IPv6 outputs in the out_net / out_l4 / verdict fields of FlatArgs.
// Phase 4: lane `lane` finalizes its frame (output index idx) from the LDS state.
template <int MODE>
__device__ __forceinline__ void finish_frame(const FlatArgs& p, uint64_t idx, bool tx, uint32_t acc_all,
                                             uint32_t acc_x, uint32_t acc_opt, uint4 info, uint4 fin, uint32_t xpos) {
    const uint32_t r = info.w & 15u;
    uint8_t* fp = p.base + (((((uint64_t)info.y) << 32) | info.x) + r);
    uint32_t verdict = fin.x & 8u;               // V_MALFORMED from phase 1, or 0
    const uint32_t post = fin.x & 3u;            // PV_DROP / PV_FRAG: decided after the header check
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
                if (post == PV_FRAG) {
                    verdict = V_FRAG;                // pico_ipv6_process_frag (pico_ipv6.c:791-795)
                } else if (l4_needed) {
                    if (!tx && !(p.flags & F_NXD) && (proto == 6u || proto == 17u)) {
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
                // pico_ipv4_process_in's order (pico_ipv4.c:420-455): the header check, then the
                // discards decided in phase 1 (source, evil bit, IHL < 5), then the fragment
                // hand-off; TX: a fragment gets its header checksum only
                const uint32_t acc_hdr = hdr20 + acc_opt;
                net = finalize(acc_hdr - (tx ? ipcrc : 0u));
                const uint32_t tsum = acc_all - acc_hdr;
                if (!tx && net != 0) {
                    verdict = V_NET_BAD;
                } else if (post == PV_DROP) {
                    verdict = V_MALFORMED;
                } else if (post == PV_FRAG) {
                    verdict = V_FRAG;
                } else if (l4_needed) {
                    if (!tx) {
                        if (proto == 6u || acc_x != 0u) {
                            l4 = finalize(pseudo + tsum);
                            if (l4 != 0) verdict |= V_L4_BAD;
                        }
                    } else if (proto != 1u) {         // TCP (and, NAT, UDP): pseudo header
                        l4 = finalize(pseudo + tsum - acc_x);
                    } else {
                        l4 = finalize(tsum - acc_x);
                    }
                }
                if (verdict == 0) verdict = V_ACCEPT;
            }
            const bool nat = MODE == 1 && (p.flags & F_NAT);
            if (nat) {
                // pico_ipv4_nat_outbound / _inbound's stores (pico_nat.c:443-449, :461-465,
                // :478-481, :511-517, :527-532, :543-546): address, port, transport crc, header crc
                const uint32_t ns = l2v & 15u, ndir = l2v >> 4;
                if (parsed && post != PV_FRAG)
                    verdict = ns == NS_SKIP ? V_UNTOUCHED : ns == NS_BAD ? V_MALFORMED : V_ACCEPT;
                if (verdict != V_ACCEPT) net = 0;
                if (ns != NS_XLATE || verdict != V_ACCEPT) l4 = 0;
                if (verdict == V_ACCEPT && (p.flags & 1u)) {
                    store_crc(fp + 10, net);
                    if (ns == NS_XLATE) {
                        const uint8_t* rec = reinterpret_cast<const uint8_t*>(((uint64_t)p.mac_hi << 32) | p.mac_lo);
                        const uint2 rw = *reinterpret_cast<const uint2*>(rec + 8ull * idx);
                        store_crc(fp + hl + (proto == 6u ? 16u : 6u), l4);
                        store_le(fp + (ndir == 1u ? 12u : 16u), rw.x, 4);
                        store_le(fp + hl + (ndir == 1u ? 0u : 2u), rw.y, 2);
                    }
                }
            } else if (tx && (p.flags & 1u)) {
                if (verdict == V_ACCEPT) {
                    store_crc(fp + 10, net);
                    if ((proto == 6u || proto == 1u) && l4_needed) store_crc(fp + hl + (proto == 6u ? 16u : 2u), l4);
                    else if (proto == 17u && tl >= 8u) store_crc(fp + hl + 6u, 0u);
                } else if (verdict == V_FRAG) {
                    store_crc(fp + 10, net);
                }
            }
        }
        if (MODE != 2 && p.out_net) p.out_net[idx] = (uint16_t)net;
        if (p.out_l4) p.out_l4[idx] = (uint16_t)l4;
        if (p.verdict) p.verdict[idx] = (uint8_t)verdict;
    }
}

template <int MODE>
__device__ __forceinline__ void sorted_finish(const FlatArgs& p, SortedWaveLds& L, uint32_t lane, uint64_t idx,
                                              bool tx) {
    asm volatile("" ::: "memory");
    finish_frame<MODE>(p, idx, tx, L.acc_all[lane], L.acc_x[lane], L.acc_opt[lane], L.info[lane], L.fin[lane],
                       L.xo[lane].x);
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
template <int MODE, bool NT, int CPL, bool SMALL>
__device__ __forceinline__ void sorted_batch(const FlatArgs& p, SortedWaveLds& L, uint4* stage, uint32_t lane,
                                             uint64_t f0) {
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

    uint32_t span = 0, ext = 0, xpos = NONE, optend = 0;
    uint32_t verdict = V_MALFORMED, hl = 0, tl = 0, proto = 0, ipcrc = 0, pseudo = 0, hdr20 = 0, l2v = 0;
    uint32_t post = 0;                           // PV_DROP / PV_FRAG (sorted_finish applies them)
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
        nlh = len >= HDR ? min(HW, (r + len + 15u) >> 4) : 0u;
        {
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
                t[k] = load_win<false>(w, ci < gn ? gv0 + 16u * ci : WIN_OOB);
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
                    // after the header check (sorted_finish): pico_ipv4_is_valid_src (:425-428,
                    // :187-229 -- 255.255.255.255, 224-254.x.x.x, 127/8 from a device that is not
                    // "loop"), the evil bit (:431-435), IHL < 5 (:438-443): discarded; MF or an
                    // offset (:446-455): handed to reassembly.  Then only the header is summed.
                    const uint32_t frag = ((H[1] >> 8) & 0xFF00u) | (H[1] >> 24);
                    const uint32_t s0 = H[3] & 0xFFu;
                    const bool bad_src = H[3] == 0xFFFFFFFFu || (s0 != 0xFFu && (s0 & 0xE0u) == 0xE0u) || s0 == 0x7Fu;
                    if (!tx && (bad_src || (frag & 0x8000u) || ihl < 5u)) post = PV_DROP;
                    else if (frag & 0x3FFFu) post = PV_FRAG;
                    if (post) {
                        span = ext = hl;
                    } else if (!tx) {
                        if (proto == 6u) {
                            l4_needed = true;
                        } else if (proto == 17u) {     // the UDP crc field lies past the frame: MALFORMED
                            if (hl + 8u > avail) { post = PV_DROP; span = ext = hl; }
                            else { l4_needed = true; xpos = r + hl + 6u; ext = max(span, hl + 8u); }
                        }
                    } else {
                        // NAT (F_NAT): TCP and UDP are recomputed in full (pico_nat.c:443-449,
                        // :461-465, :511-517, :527-532), ICMP only gets its header checksum
                        const bool nat = IPV4 && (p.flags & F_NAT);
                        if (proto == 6u) {
                            if (tl < 20u) verdict |= V_MALFORMED;
                            else { l4_needed = true; xpos = r + hl + 16u; }
                        } else if (proto == 17u && nat) {
                            if (tl < 8u) verdict |= V_MALFORMED;
                            else { l4_needed = true; xpos = r + hl + 6u; }
                        } else if (proto == 1u && !nat) {
                            if (tl < 8u) verdict |= V_MALFORMED;
                            else { l4_needed = true; xpos = r + hl + 2u; }
                        }
                    }
                }
            }
            if constexpr (IPV4) {
                // pico_ipv4_nat_outbound / _inbound (modules/pico_nat.c:424-545) after the host's
                // tuple lookup: record {addr, port, dir} per frame (dir 1 outbound: src + sport,
                // 2 inbound: dst + dport, 0 none).  The rewritten words enter the sums as deltas
                // (header, pseudo header, region), so the one pass over the old bytes gives the
                // checksums of the new ones (RFC 1624's incremental update, applied to full sums).
                if (p.flags & F_NAT) {
                    const uint8_t* nat = reinterpret_cast<const uint8_t*>(((uint64_t)p.mac_hi << 32) | p.mac_lo);
                    uint2 rw = make_uint2(0u, 0u);
                    if (lane < cnt) rw = *reinterpret_cast<const uint2*>(nat + 8ull * (f0 + lane));
                    const uint32_t dir = (rw.y >> 16) & 0xFFu;
                    l2v = NS_SKIP;
                    if (parsed && post == 0u && (dir == 1u || dir == 2u)) {
                        if ((proto == 6u || proto == 17u) && !l4_needed) {
                            l2v = NS_BAD;                            // transport shorter than its header
                        } else if (proto == 6u || proto == 17u) {
                            uint32_t H[5];
                            window_words<5, false>(hw, r, H);
                            const uint32_t old = dir == 1u ? H[3] : H[4];
                            const uint32_t da = (rw.x & 0xFFFFu) + (rw.x >> 16) - (old & 0xFFFFu) - (old >> 16);
                            // the old port: from the LDS stage, or -- a frame outside the wave's window
                            // (staged false: outside the wave's <= 2 GiB window around its first frame) -- from memory
                            const uint32_t pb = r + hl + (dir == 1u ? 0u : 2u);
                            uint32_t op;
                            if (staged) {
                                const uint8_t* row = reinterpret_cast<const uint8_t*>(stage + lane * HW);
                                const uint32_t sw = (lane & (HW - 1)) << 4;
                                op = (uint32_t)row[pb ^ sw] | ((uint32_t)row[(pb + 1u) ^ sw] << 8);
                            } else {
                                const uint8_t* q = fp + (pb - r);
                                op = (uint32_t)q[0] | ((uint32_t)q[1] << 8);
                            }
                            hdr20 += da;
                            pseudo += da;
                            p_all = da + (rw.y & 0xFFFFu) - op;     // the region's share of both words
                            l2v = NS_XLATE | (dir << 4);
                        } else if (proto == 1u) {
                            l2v = NS_HDR;
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
                bool walked = true;
                if (seed == 0) {
                    net_len = 40u;
                    proto = (H[1] >> 16) & 0xFFu;
                    // RX with extension headers and no seed: walk them here, as
                    // pico_ipv6_extension_headers does (ipv6_walk)
                    if (!tx && proto != 6u && proto != 17u && proto != 58u) {
                        const uint32_t w = (uint32_t)ipv6_walk_packed(p.base + off, avail);
                        const int k = (int)(w & 0xFFu) - 1;
                        if (k == WALK_FRAG) post = PV_FRAG;
                        walked = k == WALK_PROTO;
                        net_len = (w >> 8) & 0xFFFFu;
                        proto = w >> 24;
                    }
                }
                tl = (plen - (net_len - 40u)) & 0xFFFFu;                // pico_ipv6.c:790
                if (post == PV_FRAG) {
                    parsed = true;                   // handed to reassembly: nothing to sum
                    verdict = 0;
                } else if (walked && net_len >= 40u && net_len <= avail && net_len + tl <= avail) {
                    uint32_t addr = 0, xrel = NONE;
#pragma unroll
                    for (int m = 2; m < 10; ++m) addr = dot2_add(H[m], addr);
                    pseudo = addr + (((tl & 0xFFu) << 8) | (tl >> 8)) + (proto << 8);
                    parsed = true;
                    verdict = 0;
                    ext = tl;
                    if (!tx) {
                        // pico_transport_crc_check's proto is byte 9 (kept in ipcrc) unless F_NXD
                        ipcrc = (H[2] >> 8) & 0xFFu;
                        const bool ref17 = !(p.flags & F_NXD) && ipcrc == 17u;
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
    if (MODE != 0) {
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
        // Only the chunks that hold region bytes count: a region can end well before the window
        // part does (a UDP / ICMPv6 transport shorter than the field the reference reads: ext >
        // span), so the last counted chunk is the one holding the region's last byte.
        const bool wreg = k0 != 0u && re > rs;
        const uint32_t we1 = wreg ? (re - 1u) >> 4 : 0u;
        auto window_sums = [&](auto perm_tag) {
            constexpr bool PERM = decltype(perm_tag)::value;
#pragma unroll
            for (uint32_t i = 0; i < HW; ++i) {
                const uint32_t c = add_full<PERM>(hw[i], sl, 0u);
                p_all += (wreg && i >= d && i <= we1) ? c : 0u;
            }
            if (__builtin_amdgcn_ballot_w64(wreg)) {
                const uint32_t e0 = wreg ? d : 0u, e1 = we1;
                uint4 h0, h1;
                if (__builtin_amdgcn_ballot_w64(wreg && !staged) == 0) {
                    h0 = stage[lane * HW + (e0 ^ (lane & (HW - 1)))];
                    h1 = stage[lane * HW + (e1 ^ (lane & (HW - 1)))];
                } else {
                    h0 = edge_chunk(e0);
                    h1 = edge_chunk(e1);
                }
                if (wreg) {
                    p_all -= masked_chunk_sum<PERM>(h0, 16u * e0, 16u * e0, rs, sl);
                    p_all -= masked_chunk_sum<PERM>(h1, 16u * e1, re, 16u * (e1 + 1u), sl);
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
    L.fin[lane] = make_uint4(verdict | post | (parsed ? 16u : 0u) | (l4_needed ? 32u : 0u) | (oob ? 64u : 0u) |
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
    if (m) {
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

// ---------------------------------------------------------------- stream-order waves (fused modes)
//
// A wave whose 64 datagrams lie densely in one span of the batch (a TAP / ring burst: back to
// back behind their link headers) reads that span in address order -- 64 lanes x SCPL
// coalesced 16-byte loads a step, every line fetched once -- instead of sorting the frames
// into size-class rounds.  Each step is staged in LDS and turned into exclusive prefix sums
// per dword (in the memory-even little-endian word domain, plain 32-bit sums: a region's sum
// is the difference of two prefixes, exact below 128 KiB).  Lane j meanwhile collects frame
// j's head window from the stage, parses it as soon as its first two chunks are in, and
// reads the prefixes at its region boundaries (options start, transport start / end, the
// isolated crc field) when they pass.  Frames of odd start byte take the byte-swapped fold.

// Chunk q's slot: lane-major readers (lane L, chunks SCPL L + c) and column-major writers
// (lane l, chunks 64 c + l) both land on distinct banks within their ds_read/write_b128 groups.
__device__ __forceinline__ uint32_t sslot(uint32_t q) { return q ^ ((q >> 4) & (SCPL - 1u)); }

// The prefix at byte position b of the span (the sum of the span's bytes before b), taken when
// b's last byte before it lies in the step starting at byte byte0.
__device__ __forceinline__ bool stream_point(const StreamLds& S, uint32_t b, uint32_t byte0, uint32_t& P) {
    const uint32_t t = b - 1u - byte0;
    const bool in = b != 0u && t < 16u * SQ;
    if (in) {
        const uint32_t q = t >> 4, sh = 8u * (t & 15u) + 8u;  // bits of chunk q before b: 8..128
        const uint4 u = S.raw[sslot(q)];
        uint32_t a = S.pxc[q];
        // the chunk's first sh bits as two 64-bit masks (v_lshlrev_b64 takes the shift mod 64)
        const uint64_t ml = sh >= 64u ? ~0ull : (1ull << (sh & 63u)) - 1ull;
        const uint64_t mh = sh <= 64u ? 0ull : sh >= 128u ? ~0ull : (1ull << (sh & 63u)) - 1ull;
        a = dot2_add(u.x & (uint32_t)ml, a);
        a = dot2_add(u.y & (uint32_t)(ml >> 32), a);
        a = dot2_add(u.z & (uint32_t)mh, a);
        a = dot2_add(u.w & (uint32_t)(mh >> 32), a);
        P = a;
    }
    return in;
}

template <int OP, int CTRL, int RM>
__device__ __forceinline__ int scan_step(int x) {
    const int o = __builtin_amdgcn_update_dpp(OP == 0 ? 0 : x, x, CTRL, RM, 0xF, false);
    return OP == 0 ? x + o : OP == 1 ? min(x, o) : max(x, o);
}
template <int OP>
__device__ __forceinline__ int wave_incl(int v) {
    v = scan_step<OP, 0x111, 0xF>(v);
    v = scan_step<OP, 0x112, 0xF>(v);
    v = scan_step<OP, 0x114, 0xF>(v);
    v = scan_step<OP, 0x118, 0xF>(v);
    v = scan_step<OP, 0x142, 0xA>(v);
    v = scan_step<OP, 0x143, 0xC>(v);
    return v;
}

// The two bytes at head-window position pos (pos + 1 < 16 * n), low byte first.
template <uint32_t N>
__device__ __forceinline__ uint32_t hw_pair(const uint4 (&hw)[HW], uint32_t pos) {
    const uint32_t q = pos >> 2;
    uint32_t d0 = 0, d1 = 0;
#pragma unroll
    for (uint32_t k = 0; k < 4 * N; ++k) {
        const uint4 c = hw[k >> 2];
        const uint32_t d = (k & 3u) == 0 ? c.x : (k & 3u) == 1 ? c.y : (k & 3u) == 2 ? c.z : c.w;
        d0 = q == k ? d : d0;
        d1 = q + 1u == k ? d : d1;
    }
    return __builtin_amdgcn_alignbyte(d1, d0, pos & 3u) & 0xFFFFu;
}

// An even-domain sum as the frame's own word pairing sees it: unchanged for an even start,
// folded (zero stays zero, anything else stays in [1, 0xFFFF]) and byte-swapped for an odd one.
__device__ __forceinline__ uint32_t pairing(uint32_t v, bool odd) {
    if (!odd) return v;
    v = (v & 0xFFFFu) + (v >> 16);
    v = (v & 0xFFFFu) + (v >> 16);
    return ((v >> 8) | (v << 8)) & 0xFFFFu;
}

// A wave streams its frames' span when they lie back to back (a TAP / ring burst: the span at
// most 2 x their bytes + 4 KiB); anything else takes the sorted rounds, which read only the frames'
// own lines. (Round 4 measured two alternatives, both slower and removed -- DESIGN.md 4: the 4 waves
// of a workgroup splitting its 256 frames into equal-byte ranges, two barriers a step; and a
// COMPACT stream over the frames' own lines in frame order for slot rings and scattered frames, its
// chunk -> line map a binary search per chunk.)

// Returns false (nothing written) for a wave whose frames are not streamed: they are not back to
// back, or after the loop, the wave holds a frame the stream does not finish (below).  NATM: the NAT batch (F_NAT), its own instantiation so the RX / TX waves
// carry none of its registers or instructions.  V6: the IPv6 batch (MODE 2) for datagrams whose
// transport follows the 40-byte header (descriptor seed 0; RX next header TCP / UDP / ICMPv6 --
// anything else needs the extension-header walk: the sorted rounds).  ETH: the Ethernet batch
// (MODE 3): IPv4 and IPv6 behind the 14-byte header (ARP / dropped frames need no sums; a wave
// holding an IPv6 datagram that needs the extension-header walk falls back after the loop).
// (eth6_field, uniform64, lds_pair: used by the fused modes' stream waves only -- the RAW-mode
// translation unit, SORTED_MODE 0, instantiates none of them.)
// MODE 3 stream, an IPv6 frame: where the transport field the finish reads lies (relative to the
// transport start; NONE = none) -- RX: the UDP crc (present?) when byte 9 (the reference's dispatch,
// or with F_NXD the next header) says UDP, the ICMPv6 type; TX: the crc field to compute
// (sorted_batch's MODE 2 rules)
[[maybe_unused]] __device__ __forceinline__ uint32_t eth6_field(bool tx, uint32_t nh, uint32_t b9, bool nxd) {
    if (!tx) {
        const bool ref17 = !nxd && b9 == 17u;
        if (nh == 6u && !ref17) return NONE;
        if (nh == 17u || nh == 6u) return 6u;
        return nh == 58u ? 0u : NONE;
    }
    return nh == 6u ? 16u : nh == 17u ? 6u : nh == 58u ? 2u : NONE;
}

// The even-domain sum of the head window's bytes [a, b) (window positions, b <= 16 * N): the
// window starts on a 16-byte line of the span, so a byte's parity in the window is its parity there.
template <uint32_t N>
__device__ __forceinline__ uint32_t hw_range_sum(const uint4 (&hw)[HW], uint32_t a, uint32_t b) {
    uint32_t s = 0u;
#pragma unroll
    for (uint32_t k = 0; k < 4u * N; ++k) {
        const uint4 c = hw[k >> 2];
        const uint32_t d = (k & 3u) == 0 ? c.x : (k & 3u) == 1 ? c.y : (k & 3u) == 2 ? c.z : c.w;
        const uint32_t lo = (uint32_t)min(max((int)a - (int)(4u * k), 0), 4);
        const uint32_t hi = (uint32_t)min(max((int)b - (int)(4u * k), 0), 4);
        const uint32_t mh = (uint32_t)((1ull << (8u * hi)) - 1ull), ml = (uint32_t)((1ull << (8u * lo)) - 1ull);
        s = dot2_add(d & (mh & ~ml), s);
    }
    return s;
}

[[maybe_unused]] __device__ __forceinline__ uint64_t uniform64(uint64_t x) {
    return ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(x >> 32)) << 32) |
           (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)x);
}

// The head window as the stream's finish keeps it in LDS (wl: the lane's copy, dword-aligned, one
// zero dword past it): NW words starting at byte pos, and the two bytes at pos, low byte first.
template <int NW>
__device__ __forceinline__ void lds_words(const uint32_t* wl, uint32_t pos, uint32_t (&H)[NW]) {
    const uint32_t q = pos >> 2, sh = pos & 3u;
    uint32_t E[NW + 1];
#pragma unroll
    for (int m = 0; m <= NW; ++m) E[m] = wl[q + m];
#pragma unroll
    for (int m = 0; m < NW; ++m) H[m] = __builtin_amdgcn_alignbyte(E[m + 1], E[m], sh);
}
[[maybe_unused]] __device__ __forceinline__ uint32_t lds_pair(const uint32_t* wl, uint32_t pos) {
    const uint32_t q = pos >> 2;
    return __builtin_amdgcn_alignbyte(wl[q + 1], wl[q], pos & 3u) & 0xFFFFu;
}

// The finish of a streamed group (stream_batch, the persistent waves): lane j's frame from its head
// window and the prefixes taken at its points -- the verdict, the sums, the stores (finish_frame).
// Returns false, with nothing written, for a group the stream does not finish (the sorted rounds
// take it): options, a field or trailing bytes past the head window, an IPv6 walk, NAT with options.
template <bool NATM, bool V6, bool ETH>
__device__ __forceinline__ bool stream_finish(const FlatArgs& p, StreamLds& S, uint32_t lane, uint64_t f0,
                                              uint32_t cnt, bool tx, uint2 rw, bool valid, bool oob, uint32_t len,
                                              bool seeded, uint32_t rel, uint64_t lo, const uint4 (&hw)[HW],
                                              uint32_t P0, uint32_t P1, uint32_t P2, uint32_t P3, uint32_t P4) {
    constexpr uint32_t L2 = ETH ? 14u : 0u;
    constexpr bool natm = NATM;
    constexpr uint32_t HS = 4u;
    const uint32_t r = rel & 15u;
    // the head window into the stage (free now), 144 bytes a lane: the finish takes its header
    // words and fields with aligned LDS reads and one alignbyte each, not select chains over hw
    static_assert(64u * 36u * sizeof(uint32_t) <= sizeof(StreamLds), "head windows must fit the stage");
    uint32_t* const wl = reinterpret_cast<uint32_t*>(&S) + 36u * lane;
#pragma unroll
    for (uint32_t i = 0; i < HS; ++i) *reinterpret_cast<uint4*>(wl + 4u * i) = hw[i];
    wl[4u * HS] = 0u;
    __builtin_amdgcn_wave_barrier();
    // the frame's offset again, from the span (a 64-bit value less to keep across the loop)
    const uint64_t off = valid ? lo + rel - reinterpret_cast<uintptr_t>(p.base) : 0u;
    if constexpr (V6) {
        // pico_ipv6_process_in / pico_transport_crc_check as sorted_batch's MODE 2 (seed 0, no
        // extension header): lengths, byte-9 dispatch (ipcrc), the field, the pseudo header
        uint32_t verdict = V_MALFORMED, tl = 0, proto = 0, ipcrc = 0, pseudo = 0, xo = NONE;
        bool parsed = false, l4_needed = false, walk = false;
        if (valid) {
            uint32_t H[10];
            lds_words<10>(wl, r, H);
            tl = ((H[1] & 0xFFu) << 8) | ((H[1] >> 8) & 0xFFu);
            proto = (H[1] >> 16) & 0xFFu;
            if (!tx && proto != 6u && proto != 17u && proto != 58u) {
                walk = true;
            } else if (40u + tl <= len) {
                uint32_t addr = 0;
#pragma unroll
                for (int m = 2; m < 10; ++m) addr = dot2_add(H[m], addr);
                pseudo = addr + (((tl & 0xFFu) << 8) | (tl >> 8)) + (proto << 8);
                parsed = true;
                verdict = 0;
                if (!tx) {
                    ipcrc = (H[2] >> 8) & 0xFFu;
                    const bool ref17 = !(p.flags & F_NXD) && ipcrc == 17u;
                    if (proto == 6u && !ref17) {
                        l4_needed = true;
                    } else if (proto == 17u || proto == 6u) {
                        if (48u > len) { parsed = false; verdict = V_MALFORMED; }
                        else { l4_needed = true; xo = 6u; }
                    } else if (proto == 58u) {
                        if (41u > len) { parsed = false; verdict = V_MALFORMED; }
                        else { l4_needed = true; xo = 0u; }
                    }
                } else if (proto == 6u || proto == 17u || proto == 58u) {
                    if (tl < (proto == 6u ? 20u : proto == 17u ? 8u : 4u)) { parsed = false; verdict = V_MALFORMED; }
                    else { l4_needed = true; xo = proto == 6u ? 16u : proto == 17u ? 6u : 2u; }
                }
            }
        }
        // bytes past the datagram (P2 was taken at the frame's end): from the head window
        const bool tail = parsed && 40u + tl < len;
        if (__builtin_amdgcn_ballot_w64(walk || (tail && r + len > 16u * HS))) return false;
        uint32_t P2d = P2;
        if (__builtin_amdgcn_ballot_w64(tail) && tail) P2d = P2 - hw_range_sum<HS>(hw, r + 40u + tl, r + len);
        const bool odd = r & 1u;
        uint32_t xe = 0, xp = 0;
        if (xo == 16u) {                       // TX TCP: by prefixes
            xe = P4 - P3;
            xp = odd ? ((xe >> 8) | (xe << 8)) & 0xFFFFu : xe;
        } else if (xo != NONE) {
            xp = lds_pair(wl, r + 40u + xo);
            xe = odd ? ((xp >> 8) | (xp << 8)) & 0xFFFFu : xp;
        }
        const uint32_t tsum = tx ? pairing(P2d - P1 - xe, odd) + xp : pairing(P2d - P1, odd);
        // the transport's line and offset (finish stores the field relative to it)
        const uint32_t rt = (r + 40u) & 15u;
        const uint64_t a0t = valid ? off + 40u - rt : 0u;
        if (lane < cnt)
            finish_frame<2>(p, f0 + lane, tx, tsum, xp, 0u, make_uint4((uint32_t)a0t, (uint32_t)(a0t >> 32), 0u, rt),
                            make_uint4(verdict | (parsed ? 16u : 0u) | (l4_needed ? 32u : 0u) | (oob ? 64u : 0u) |
                                           (proto << 8) | (tl << 16),
                                       ipcrc << 16, pseudo, 0u),
                            NONE);
        STAMP(3);
        return true;
    }
    // the header (pico_ipv4_process_in's checks and dispatch, as sorted_batch)
    uint32_t verdict = V_MALFORMED, hl = 0, tl = 0, proto = 0, ipcrc = 0, pseudo = 0, hdr20 = 0, post = 0;
    uint32_t l2v = natm ? NS_SKIP : 0u, nop = 0, nnw = 0;   // NAT: state, old / new port (frame pairing)
    bool parsed = false, l4_needed = false, hasx = false, nat_opt = false, ip4 = valid, eth6 = false;
    bool walk6 = false;
    const uint32_t ilen = len - L2;
    // MODE 3 IPv6 frames (as sorted_batch's MODE 3 -> MODE 2 path, seed 0, no extension header):
    // transport sum, field, pseudo header from the prefixes
    uint32_t v6sum = 0u, v6x = 0u;
    if constexpr (ETH) {
        // pico_ethernet_receive (pico_ethernet.c:180-235): destination filter, ethertype, version
        ip4 = false;
        if (valid) {
            uint32_t M[2], T[1];
            lds_words<2>(wl, r, M);
            lds_words<1>(wl, r + 12u, T);
            const uint32_t m0 = M[0], m1 = M[1] & 0xFFFFu, et = T[0] & 0xFFFFu;
            const bool mine = !(p.flags & F_MACF) || tx || (m0 == p.mac_lo && m1 == p.mac_hi) ||
                              (m0 & 0xFFFFFFu) == 0x5E0001u || (m0 & 0xFFFFu) == 0x3333u ||
                              (m0 == 0xFFFFFFFFu && m1 == 0xFFFFu);
            if (!mine) l2v = V_DROP_L2;
            else if (et == 0x0608u) l2v = V_ARP;
            else if (et == 0xDD86u) {                    // IPv6 (pico_ethernet.c:162-176)
                if (ilen != 0u) {
                    uint32_t V[1];
                    lds_words<1>(wl, r + 14u, V);
                    if ((V[0] & 0xF0u) != 0x60u) l2v = V_DROP_L2;
                    else eth6 = true;
                }
            }
            else if (et != 0x0008u) l2v = V_DROP_L2;
            else if (ilen != 0u) {
                uint32_t V[1];
                lds_words<1>(wl, r + 14u, V);
                if ((V[0] & 0xF0u) != 0x40u) l2v = V_DROP_L2;
                else ip4 = true;
            }
        }
    }
    walk6 = eth6 && seeded;
    if (ETH && eth6 && ilen >= 40u && !seeded) {
        uint32_t H[3];
        lds_words<3>(wl, r + 14u, H);
        tl = ((H[1] & 0xFFu) << 8) | ((H[1] >> 8) & 0xFFu);
        proto = (H[1] >> 16) & 0xFFu;
        const uint32_t b9 = (H[2] >> 8) & 0xFFu;
        if (!tx && proto != 6u && proto != 17u && proto != 58u) {
            walk6 = true;                                // extension headers: the sorted rounds
        } else if (40u + tl <= ilen) {
            const bool odd6 = r & 1u;
            pseudo = pairing(P1 - P0, odd6) + (((tl & 0xFFu) << 8) | (tl >> 8)) + (proto << 8);
            parsed = true;
            verdict = 0;
            const uint32_t xo = eth6_field(tx, proto, b9, (p.flags & F_NXD) != 0u);
            if (!tx) {
                ipcrc = b9;
                if (xo == 6u && 48u > ilen) { parsed = false; verdict = V_MALFORMED; }
                else if (xo == 0u && 41u > ilen) { parsed = false; verdict = V_MALFORMED; }
                else l4_needed = proto == 6u || proto == 17u || proto == 58u;
            } else if (xo != NONE) {
                if (tl < (proto == 6u ? 20u : proto == 17u ? 8u : 4u)) { parsed = false; verdict = V_MALFORMED; }
                else l4_needed = true;
            }
            if (xo != NONE) {
                const uint32_t xe6 = P4 - P3;
                v6x = odd6 ? ((xe6 >> 8) | (xe6 << 8)) & 0xFFFFu : xe6;
                v6sum = tx ? pairing(P2 - P1 - xe6, odd6) + v6x : pairing(P2 - P1, odd6);
            } else {
                v6sum = pairing(P2 - P1, odd6);
            }
        }
    }
    if (ETH ? ip4 && ilen >= 20u : valid) {
        uint32_t H[5];
        lds_words<5>(wl, r + L2, H);
        const uint32_t ihl = H[0] & 0x0Fu;
        hl = 20u + (ihl > 5u ? 4u * (ihl - 5u) : 0u);
        const uint32_t tot = (((H[0] >> 16) & 0xFFu) << 8) | (H[0] >> 24);
        proto = (H[2] >> 8) & 0xFFu;
        ipcrc = H[2] >> 16;
        tl = (tot - hl) & 0xFFFFu;
        const uint32_t max_allowed = (ilen - 20u) & 0xFFFFu;
        if (!(hl > ilen || (!tx && tl > max_allowed) || hl + tl > ilen)) {
            parsed = true;
            verdict = 0;
#pragma unroll
            for (int m = 0; m < 5; ++m) hdr20 = dot2_add(H[m], hdr20);
            pseudo = (H[3] & 0xFFFFu) + (H[3] >> 16) + (H[4] & 0xFFFFu) + (H[4] >> 16) + (proto << 8) +
                     (((tl & 0xFFu) << 8) | (tl >> 8));
            const uint32_t frag = ((H[1] >> 8) & 0xFF00u) | (H[1] >> 24);
            const uint32_t s0 = H[3] & 0xFFu;
            const bool bad_src = H[3] == 0xFFFFFFFFu || (s0 != 0xFFu && (s0 & 0xE0u) == 0xE0u) || s0 == 0x7Fu;
            if (!tx && (bad_src || (frag & 0x8000u) || ihl < 5u)) post = PV_DROP;
            else if (frag & 0x3FFFu) post = PV_FRAG;
            if (!post && !tx) {
                if (proto == 6u) {
                    l4_needed = true;
                } else if (proto == 17u) {
                    if (hl + 8u > ilen) post = PV_DROP;
                    else { l4_needed = true; hasx = true; }
                }
            } else if (!post) {
                // NAT: TCP and UDP recomputed in full, ICMP only its header checksum (as sorted_batch)
                if (proto == 6u) {
                    if (tl < 20u) verdict |= V_MALFORMED;
                    else { l4_needed = true; hasx = true; }
                } else if (proto == (natm ? 17u : 1u)) {
                    if (tl < 8u) verdict |= V_MALFORMED;
                    else { l4_needed = true; hasx = true; }
                }
            }
            // NAT (pico_nat.c:424-545): the rewritten address enters the header and pseudo sums as
            // a delta, the port the region's (below) -- sorted_batch's NAT stage, with the old port
            // from the head window (a datagram with options falls back to the sorted rounds)
            if constexpr (NATM) {
                const uint32_t dir = (rw.y >> 16) & 0xFFu;
                l2v = NS_SKIP;
                if (post == 0u && (dir == 1u || dir == 2u)) {
                    if ((proto == 6u || proto == 17u) && !l4_needed) {
                        l2v = NS_BAD;
                    } else if (proto == 6u || proto == 17u) {
                        const uint32_t old = dir == 1u ? H[3] : H[4];
                        const uint32_t da = (rw.x & 0xFFFFu) + (rw.x >> 16) - (old & 0xFFFFu) - (old >> 16);
                        hdr20 += da;
                        pseudo += da;
                        if (hl == 20u) nop = lds_pair(wl, r + 20u + (dir == 1u ? 0u : 2u));
                        else nat_opt = true;
                        nnw = rw.y & 0xFFFFu;
                        l2v = NS_XLATE | (dir << 4);
                    } else if (proto == 1u) {
                        l2v = NS_HDR;
                    }
                }
            }
        }
    }
    // MODE 1 (no parse in the loop: P1 at the options start, P2 at the frame's end): the options,
    // the field and any bytes past the datagram from the head window, else the sorted rounds
    const uint32_t xo4 = (!tx || proto == 17u) ? 6u : proto == 6u ? 16u : 2u;
    const bool v4 = parsed && !eth6;                   // an IPv4 datagram with sums to take
    const bool fx = ETH && tx && proto == 6u && hl == 20u;   // MODE 3 TX TCP crc: by prefixes (50)
    const bool tail = v4 && hl + tl < ilen;
    const bool fb = (v4 && r + L2 + hl > 16u * HS) || (tail && r + len > 16u * HS) ||
                    (v4 && hasx && !fx && r + L2 + hl + xo4 + 2u > 16u * HS);
    if (__builtin_amdgcn_ballot_w64((ETH && walk6) || nat_opt || fb)) return false;
    uint32_t optd = 0u, P2d = P2;
    if (__builtin_amdgcn_ballot_w64(v4 && (hl > 20u || tail))) {
        if (v4 && hl > 20u) optd = hw_range_sum<HS>(hw, r + L2 + 20u, r + L2 + hl);
        if (tail) P2d = P2 - hw_range_sum<HS>(hw, r + L2 + hl + tl, r + len);
    }
    const uint32_t P1d = P1 + optd;
    const bool odd = r & 1u;
    // the field (frame pairing xp, even domain xe): from the head window, or (MODE 3 TX TCP without
    // options: frame + 50, past the head chunks at some starts) by prefixes
    uint32_t xe = 0, xp = 0;
    if (hasx) {
        if (!fx) {
            xp = lds_pair(wl, r + L2 + hl + xo4);
            xe = odd ? ((xp >> 8) | (xp << 8)) & 0xFFFFu : xp;
        } else {
            xe = P4 - P3;
            xp = odd ? ((xe >> 8) | (xe << 8)) & 0xFFFFu : xe;
        }
    }
    // transport; TX: the field's share kept apart (finish subtracts it; TX fields lie inside the
    // region), RX: the field only says "present" (a UDP crc may lie past a short region)
    // NAT: the old port leaves the region in the even domain (no wrap below zero), the new enters
    const uint32_t noe = odd ? ((nop >> 8) | (nop << 8)) & 0xFFFFu : nop;
    const uint32_t tsum = tx ? pairing(P2d - P1d - xe - noe, odd) + xp + nnw : pairing(P2d - P1d, odd);
    const uint32_t opt = hl > 20u ? pairing(optd, odd) : 0u;
    // the IPv4 header's line and offset (finish stores relative to it)
    // (MODE 3 IPv6: the transport's line and offset; finish stores the field relative to it)
    const uint32_t ri = (r + (eth6 ? 54u : L2)) & 15u;
    const uint64_t a0off = valid ? off + (eth6 ? 54u : L2) - ri : 0u;
    if (lane < cnt)
        finish_frame<ETH ? 3 : 1>(p, f0 + lane, tx, eth6 ? v6sum : hdr20 + opt + tsum, eth6 ? v6x : xp, opt,
                        make_uint4((uint32_t)a0off, (uint32_t)(a0off >> 32), 0u, ri),
                        make_uint4(verdict | post | (parsed ? 16u : 0u) | (l4_needed ? 32u : 0u) | (oob ? 64u : 0u) |
                                       (eth6 ? 128u : 0u) | (proto << 8) | (tl << 16),
                                   hl | (l2v << 8) | (ipcrc << 16), pseudo, hdr20),
                        NONE);
    STAMP(3);
    return true;
}

template <bool NATM, bool V6 = false, bool ETH = false>
__device__ __forceinline__ bool stream_batch(const FlatArgs& p, StreamLds& S, uint32_t lane, uint64_t f0) {
    constexpr uint32_t L2 = ETH ? 14u : 0u;   // the IPv4 header's offset in the frame
    if (!ETH && (p.flags & F_MACF)) return false;
    const uint32_t cnt = f0 < p.n ? (uint32_t)min((uint64_t)p.fpw, (uint64_t)p.n - f0) : 0u;
    const bool tx = (p.flags & 2u) != 0;
    uint4 dcur = make_uint4(0, 0, 0, 0);
    if (lane < cnt) dcur = *reinterpret_cast<const uint4*>(p.desc + f0 + lane);
    // NAT: the frame's record {addr, port | dir << 16} (sorted_batch's NAT stage)
    uint2 rw = make_uint2(0u, 0u);
    if (NATM && lane < cnt)
        rw = *reinterpret_cast<const uint2*>(reinterpret_cast<const uint8_t*>(((uint64_t)p.mac_hi << 32) | p.mac_lo) +
                                             8ull * (f0 + lane));
    uint64_t off0 = ((uint64_t)dcur.y << 32) | dcur.x;
    uint32_t len = lane < cnt ? dcur.z : 0u;
    const bool oob = lane < cnt && (off0 > p.base_len || len > p.base_len - off0);
    if (oob || lane >= cnt) { len = 0; off0 = 0; }
    const bool valid = len >= (V6 ? 40u : ETH ? 14u : 20u);  // shorter: MALFORMED, nothing to sum
    const bool seeded = ETH && dcur.w != 0u;     // MODE 3 IPv6 with a stack-walked net_len: sorted rounds
    const uint32_t blen = valid ? len : 0u;
    const uint64_t addr = reinterpret_cast<uintptr_t>(p.base) + off0;
    const uint64_t la = addr & ~(uint64_t)15;
    // MODE 3: the first step's loads go out before the span is worked out: 8 KiB from lane 0's
    // frame's line (where a burst's span starts) through a window clamped to the batch buffer. They
    // are kept when the span does start there -- bytes past the span's end only ever enter prefixes
    // past every frame (a span longer than one step fills its first step) -- else the step is
    // loaded again. (Measured: c2eth 23.3-23.5 against 24.5-24.7 us; C2 / C2-IPv6 no better, C2
    // 21.5-21.8 against 21.2, so MODE 1 / MODE 2 load after the setup: profiles/r04/ab_spec_first_step.txt)
    // (whole lines, as the span's own window: a buffer load partly past its window's end returns
    // zeros for all of it, and a frame's last line can run past the batch buffer's end)
    const uint64_t lo0 = uniform64(la);
    const uint64_t bend = (reinterpret_cast<uintptr_t>(p.base) + p.base_len + 15u) & ~(uint64_t)15;
    const Window w0 = make_window(lo0, (uint32_t)min((uint64_t)(16u * SQ), bend > lo0 ? bend - lo0 : 0ull));
    uint4 v[SCPL], vn[SCPL];
    if constexpr (ETH) {
#pragma unroll
        for (uint32_t c = 0; c < SCPL; ++c) v[c] = load_win<true>(w0, 16u * (64u * c + lane));
    }
    // ---- the span: anchor, extent, layout
    uint64_t anchor = ~0ull;
    int mn = 0, mx = 0;
    uint32_t q1 = 0u, nsteps = 0u;
    {
        const uint64_t vb = __builtin_amdgcn_ballot_w64(valid);
        if (!vb) return false;
        // a stack-walked IPv6 seed, or a frame over 1 MiB (the 32-bit byte sums): no stream
        if (__builtin_amdgcn_ballot_w64(valid && ((V6 && dcur.w != 0u) || len > (1u << 20)))) return false;
        const int fv = __builtin_ffsll((long long)vb) - 1;
        anchor = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(la >> 32), fv) << 32) |
                 (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)la, fv);
        const int64_t dl = (int64_t)(la - anchor), dh = (int64_t)(addr + len - anchor);
        if (__builtin_amdgcn_ballot_w64(valid && (dl < -(1ll << 29) || dh > (1ll << 29)))) return false;
        // frames in address order (a burst): the first valid frame's line (dl = 0) and the last
        // one's end bound the span; a frame outside them makes the wave scan for both
        mx = __builtin_amdgcn_readlane((int)dh, 63 - __builtin_clzll(vb));
        if (__builtin_amdgcn_ballot_w64(valid && (dl < 0 || dh > (int64_t)mx))) {
            mn = __builtin_amdgcn_readlane(wave_incl<1>(valid ? (int)dl : 0x7FFFFFFF), 63);
            mx = __builtin_amdgcn_readlane(wave_incl<2>(valid ? (int)dh : -0x7FFFFFFF), 63);
        }
        const uint32_t rs = (uint32_t)__builtin_amdgcn_readlane(wave_incl<0>((int)blen), 63);
        const uint32_t ext = (uint32_t)(((int64_t)mx + 15 - (int64_t)mn) & ~(int64_t)15);
        if (!((uint64_t)ext <= 2ull * rs + 4096u)) return false;    // not back to back
        q1 = ext >> 4;
        nsteps = (q1 + SQ - 1u) / SQ;
    }
    const uint64_t lo = uniform64(anchor + (int64_t)mn);
    const uint64_t extent = (uint64_t)(((int64_t)mx + 15 - (int64_t)mn) & ~(int64_t)15);
    const Window w = make_window(lo, (uint32_t)extent);
    const uint32_t rel = valid ? (uint32_t)(addr - lo) : 0u;   // frame start in the span
    const uint32_t r = rel & 15u, hq = rel >> 4;
    // head-window chunks: the header and, without options, the crc field (r + 38 <= 64). (MODE 3
    // with a fifth -- a padded 60-byte frame's end at any start -- spills into its loop: a padded
    // frame starting past byte 4 of its line sends the wave to the sorted rounds instead)
    constexpr uint32_t HS = 4u;
    const uint32_t nlh = valid ? min(HS, (r + len + 15u) >> 4) : 0u;
    uint4 hw[HW];
#pragma unroll
    for (uint32_t i = 0; i < HW; ++i) hw[i] = make_uint4(0, 0, 0, 0);
    // boundaries (span byte positions, 0 = none): options start, transport start / end, field
    // MODE 3: b0 = an IPv6 datagram's addresses (frame + 22), which can lie in the step before the
    // one that completes the header parse: set once the ethertype is in (chunk 1), which is never
    // later than the step holding frame + 21
    uint32_t b0 = 0, b1 = 0, b2 = 0, x0 = 0, x1 = 0;
    bool pre6 = !ETH || !valid;
    // No IPv4 parse in the loop: the options start (where the transport starts without options),
    // the frame's end and, for TX, the TCP crc field's place without options (MODE 2: the transport
    // start and the TCP crc at 56); the finish corrects them from the head window (options, bytes
    // past the datagram, the field with options) or falls back. MODE 3 moves an IPv6 frame's points
    // once its ethertype is in, and parses IPv6 headers in the loop (their field depends on them).
    if (valid) {
        b1 = rel + min(V6 ? 40u : L2 + 20u, len);
        b2 = rel + len;
        if (V6 && tx && 58u <= len) { x0 = rel + 56u; x1 = x0 + 2u; }
        if (ETH && tx && 52u <= len) { x0 = rel + 50u; x1 = x0 + 2u; }
    }
    uint32_t P0 = 0, P1 = 0, P2 = 0, P3 = 0, P4 = 0;
    bool pre = !valid;
    uint32_t base = 0;
    // two steps in flight: step k + 1's loads go out before step k is staged and summed
    // (loads issued on two paths -- a layout branch -- leave the compiler's wait counting at the
    // join with a full vmcnt(0): the next step's loads waited on before this one is staged)
    auto load_step = [&](uint32_t qs, uint4 (&dst)[SCPL]) {
        const uint32_t o = 16u * (qs + lane), oe = 16u * q1;
#pragma unroll
        for (uint32_t c = 0; c < SCPL; ++c) dst[c] = load_win<true>(w, o + 1024u * c < oe ? o + 1024u * c : WIN_OOB);
    };
    // NAT: the record is in before the loop (an older load still in flight at the loop leaves the
    // compiler's wait counting with a vmcnt(0) at every stage write)
    if constexpr (NATM) asm volatile("" ::"v"(rw.x), "v"(rw.y));
    if (!ETH || lo != lo0) load_step(0u, v);             // MODE 3: the span starts elsewhere
    STAMP(1);
    // one step: cur is staged and summed while nxt's loads (step st + 1) are in flight
    auto step = [&](auto pf, uint32_t st, uint4 (&cur)[SCPL], uint4 (&nxt)[SCPL]) {
        const uint32_t qb = st * SQ;
#if STREAM_LAST_NOPF
        if constexpr (decltype(pf)::value) load_step(qb + SQ, nxt);
#else
        (void)pf;
        load_step(qb + SQ, nxt);
#endif
        asm volatile("" ::: "memory");
#pragma unroll
        for (uint32_t c = 0; c < SCPL; ++c) S.raw[sslot(64u * c + lane)] = cur[c];
        __builtin_amdgcn_wave_barrier();
        // lane-major: lane L's SCPL chunks, chunk prefixes, one wave scan of the lane totals
        uint32_t loc[SCPL];
        uint32_t t = 0;
#pragma unroll
        for (uint32_t k = 0; k < SCPL; ++k) {
            loc[k] = t;
            t = add_full<false>(S.raw[sslot(SCPL * lane + k)], SEL_EVEN, t);
        }
        const uint32_t incs = (uint32_t)wave_incl<0>((int)t);
        const uint32_t tot = (uint32_t)__builtin_amdgcn_readlane((int)incs, 63);
        const uint32_t exs = base + incs - t;
#pragma unroll
        for (uint32_t k = 0; k < SCPL; k += 4)
            *reinterpret_cast<uint4*>(&S.pxc[SCPL * lane + k]) =
                make_uint4(exs + loc[k], exs + loc[k + 1], exs + loc[k + 2], exs + loc[k + 3]);
        __builtin_amdgcn_wave_barrier();
        // frame j's head window chunks that are in this step
#pragma unroll
        for (uint32_t i = 0; i < HS; ++i) {
            const uint32_t qi = hq + i - qb;
            if (i < nlh && qi < SQ) hw[i] = S.raw[sslot(qi)];
        }
        // once chunks 0 and 1 are in: the boundaries (clamped into the frame; a frame that
        // fails the header checks below never reads them)
        if (ETH && !pre6 && hq + 1u < qb + SQ) {
            // the ethertype: an IPv6 frame's addresses, transport start (neither taken yet: both
            // lie past chunk 1); anything else needs no parse in the loop
            pre6 = true;
            uint32_t T[1];
            window_words<1, true>(hw, r + 12u, T);
            if ((T[0] & 0xFFFFu) == 0xDD86u) {
                b0 = rel + 22u;
                b1 = rel + min(54u, len);
                x0 = x1 = 0u;
            } else {
                pre = true;
            }
        }
        if (ETH && !pre && hq + 2u < qb + SQ) {
            // MODE 3: an IPv6 frame -- its transport end and field, by prefixes (past the head chunks)
            {
                pre = true;
                uint32_t H[3];
                window_words<3, true>(hw, r + 14u, H);
                const uint32_t ilen = len - 14u;
                const uint32_t plen = ((H[1] & 0xFFu) << 8) | ((H[1] >> 8) & 0xFFu);
                const uint32_t nh = (H[1] >> 16) & 0xFFu, b9 = (H[2] >> 8) & 0xFFu;
                if (ilen >= 40u) {
                    // (b0, b1 since the ethertype)
                    b2 = rel + 14u + min(40u + plen, ilen);
                    const uint32_t xo = eth6_field(tx, nh, b9, (p.flags & F_NXD) != 0u);
                    if (xo != NONE && 40u + xo < ilen) {
                        x0 = rel + 54u + xo;
                        x1 = x0 + min(2u, ilen - 40u - xo);
                    }
                }
            }
        }
        const uint32_t byte0 = 16u * qb;
        stream_point(S, b1, byte0, P1);
        stream_point(S, b2, byte0, P2);
        // the optional points, each cleared once taken (the group is skipped once none is left)
        if ((ETH || V6) && __builtin_amdgcn_ballot_w64((b0 | x0 | x1) != 0u)) {
            b0 = stream_point(S, b0, byte0, P0) ? 0u : b0;
            x0 = stream_point(S, x0, byte0, P3) ? 0u : x0;
            x1 = stream_point(S, x1, byte0, P4) ? 0u : x1;
        }
        base += tot;
        asm volatile("" ::: "memory");
        __builtin_amdgcn_wave_barrier();               // every stage read before the next is written
    };
    if constexpr (!ETH) {
        // two steps a trip, the register sets swapping roles: each step's wait covers only its own
        // loads (a copy of the next set into this one at the end of a trip would wait on them too,
        // leaving one step in flight across the wait)
#if STREAM_LAST_NOPF
        // the last step loads nothing ahead (its next step would be past the span: 8 void loads):
        // c2v6 22.3-22.7 vs 22.9-23.5 us, c2nat 30.9-31.4 vs 31.2-31.7, c2 and c2tx the same
        // (profiles/r06/ab_stream_last_nopf.txt)
        uint32_t st = 0;
        for (; st + 2u < nsteps; st += 2) {
            step(std::true_type{}, st, v, vn);
            step(std::true_type{}, st + 1u, vn, v);
        }
        if (st + 1u < nsteps) {
            step(std::true_type{}, st, v, vn);
            step(std::false_type{}, st + 1u, vn, v);
        } else if (st < nsteps) {
            step(std::false_type{}, st, v, vn);
        }
#else
        for (uint32_t st = 0; st < nsteps; st += 2) {
            step(std::true_type{}, st, v, vn);
            if (st + 1u >= nsteps) break;
            step(std::true_type{}, st + 1u, vn, v);
        }
#endif
    } else {
        // MODE 3 (both families' parse in the loop): one step a trip, the sets copied -- the
        // two-step trip spills there
        // (every step loads ahead here: the last step without its void loads measured slower on
        // MODE 3, c2eth 25.5-25.8 vs 23.5-23.8 us, c2ethmix 28.2-29.0 vs 26.4-27.3;
        // profiles/r06/ab_stream_last_nopf.txt)
        for (uint32_t st = 0; st < nsteps; ++st) {
            step(std::true_type{}, st, v, vn);
#pragma unroll
            for (uint32_t c = 0; c < SCPL; ++c) v[c] = vn[c];
        }
    }

    STAMP(2);
    return stream_finish<NATM, V6, ETH>(p, S, lane, f0, cnt, tx, rw, valid, oob, len, seeded, rel, lo, hw, P0, P1,
                                        P2, P3, P4);
}

// One wave per batch of up to 64 frames.  (A persistent grid looping over batches
// measured slower: every wave repeats the same serial descriptor -> rounds chain.)
// The product shape (measured): 8 chunks per lane per round, the 1-lane class for
// frames of <= 8 chunks, non-temporal loads in the >= 16-lane rounds; 4 waves per SIMD.
template <int MODE, bool NT = true, int CPL = 8, bool SMALL = true>
__global__ __launch_bounds__(64 * WPB, 16 / WPB) void csum_sorted_kernel(FlatArgs p) {
    __shared__ SortedWaveSmem<MODE != 0> lds_all[WPB];
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    SortedWaveSmem<MODE != 0>& S = lds_all[wv];
    const uint64_t f0 = ((uint64_t)blockIdx.x * (blockDim.x >> 6) + wv) * p.fpw;
    STAMP(0);
    if ((uint64_t)blockIdx.x * (blockDim.x >> 6) * p.fpw < p.n) {     // workgroup-uniform
        if constexpr (MODE != 0) {
            bool done;
            if constexpr (MODE == 2) done = stream_batch<false, true>(p, S.st, lane, f0);
            else if constexpr (MODE == 3) done = stream_batch<false, false, true>(p, S.st, lane, f0);
            else done = (p.flags & F_NAT) ? stream_batch<true>(p, S.st, lane, f0) : stream_batch<false>(p, S.st, lane, f0);
            if (done) return;
        }
        if (f0 < p.n) sorted_batch<MODE, NT, CPL, SMALL>(p, S.s, S.stage, lane, f0);
    }
    STAMP(3);
}


#if SORTED_MODE == 0
// ---------------------------------------------------------------- uniform rings: stream waves
//
// C1 / C3 / C4: frame i at base + i * stride, len bytes, densely packed (stride close to len).  Wave
// w takes frames [w R, w R + R) and reads their span in address order, one continuous stream (64
// lanes x SCPL coalesced 16-byte non-temporal buffer loads a step, the next step's loads in flight
// while this one is summed -- stream_batch's loop, nothing parsed).  Lane j owns frames j, j + 64,
// j + 128, ... of the range: it takes its frame's two prefixes (start, end) as their steps pass,
// stores the frame's checksum and moves on to its next frame, so results leave during the stream
// and no lane waits for the wave.  sum = end - start is exact mod 2^32 for an even start (the
// reference's uint32 accumulator); an odd start is folded and byte-swapped, which the host allows
// only where no carry can leave 32 bits (len <= 65535, seed < 2^31).  The host requires 64 frames
// to span more than two steps, so a lane's next frame never starts in the step its last one ended.
struct UniArgs {
    uint8_t* base;
    uint64_t stride;
    uint32_t len;
    uint32_t n;
    uint32_t seed;
    uint32_t fpw;          // frames per wave (R)
    uint16_t* out;
};

__device__ __forceinline__ void uniform_stream_range(const UniArgs& p, StreamLds& S, uint32_t lane, uint64_t f0) {
    const uint32_t cnt = (uint32_t)min((uint64_t)p.fpw, (uint64_t)p.n - f0);
    const uint64_t first = reinterpret_cast<uintptr_t>(p.base) + f0 * p.stride;
    const uint64_t lo = first & ~(uint64_t)15;
    const uint64_t end = first + (uint64_t)(cnt - 1u) * p.stride + p.len;
    const uint32_t extent = (uint32_t)(((end + 15u) & ~(uint64_t)15) - lo);     // < 2^31 (host)
    const Window w = make_window(lo, extent);
    const uint32_t q1 = extent >> 4, nsteps = (q1 + SQ - 1u) / SQ;
    const uint32_t r0 = (uint32_t)(first - lo);
    const uint32_t nmine = lane < cnt ? (cnt - lane + 63u) >> 6 : 0u;   // this lane's frames
    uint32_t m = 0;                                                   // its current one: lane + 64 m
    uint32_t b1 = 0, b2 = 0, P1 = 0, P2 = 0;
    bool t1 = false;                                                  // start prefix taken
    auto frame_points = [&]() {
        const uint32_t rel = r0 + (uint32_t)((uint64_t)(lane + 64u * m) * p.stride);
        b1 = rel;
        b2 = rel + p.len;
        P1 = 0u;
        t1 = rel == 0u;                                               // the span's first byte: prefix 0
    };
    if (nmine) frame_points();
    uint32_t base = 0;
    uint4 v[SCPL], vn[SCPL];
    auto load_step = [&](uint32_t qs, uint4 (&dst)[SCPL]) {
        const uint32_t o = 16u * (qs + lane), oe = 16u * q1;
#pragma unroll
        for (uint32_t c = 0; c < SCPL; ++c) dst[c] = load_win<true>(w, o + 1024u * c < oe ? o + 1024u * c : WIN_OOB);
    };
    load_step(0u, v);
    auto step = [&](uint32_t st, uint4 (&cur)[SCPL], uint4 (&nxt)[SCPL]) {
        const uint32_t qb = st * SQ;
        load_step(qb + SQ, nxt);
        asm volatile("" ::: "memory");
#pragma unroll
        for (uint32_t c = 0; c < SCPL; ++c) S.raw[sslot(64u * c + lane)] = cur[c];
        __builtin_amdgcn_wave_barrier();
        if (st == 0u) STAMP(1);                        // (diagnostic build: the first step's data in)
        uint32_t loc[SCPL];
        uint32_t t = 0;
#pragma unroll
        for (uint32_t k = 0; k < SCPL; ++k) {
            loc[k] = t;
            t = add_full<false>(S.raw[sslot(SCPL * lane + k)], SEL_EVEN, t);
        }
        const uint32_t incs = (uint32_t)wave_incl<0>((int)t);
        const uint32_t tot = (uint32_t)__builtin_amdgcn_readlane((int)incs, 63);
        const uint32_t exs = base + incs - t;
#pragma unroll
        for (uint32_t k = 0; k < SCPL; k += 4)
            *reinterpret_cast<uint4*>(&S.pxc[SCPL * lane + k]) =
                make_uint4(exs + loc[k], exs + loc[k + 1], exs + loc[k + 2], exs + loc[k + 3]);
        __builtin_amdgcn_wave_barrier();
        const uint32_t byte0 = 16u * qb;
        if (m < nmine) {
            if (!t1) t1 = stream_point(S, b1, byte0, P1);
            if (t1 && stream_point(S, b2, byte0, P2)) {
                p.out[f0 + lane + 64u * m] = (uint16_t)finalize(p.seed + pairing(P2 - P1, (b1 & 1u) != 0u));
                ++m;
                if (m < nmine) frame_points();
            }
        }
        base += tot;
        asm volatile("" ::: "memory");
        __builtin_amdgcn_wave_barrier();               // every stage read before the next is written
    };
    for (uint32_t st = 0; st < nsteps; st += 2) {
        step(st, v, vn);
        if (st + 1u >= nsteps) break;
        step(st + 1u, vn, v);
    }
}

template <int WPS>
__global__ __launch_bounds__(64 * WPB, WPS) void csum_uniform_stream_kernel(UniArgs p) {
    __shared__ StreamLds lds_all[WPB];
    const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
    const uint64_t f0 = ((uint64_t)blockIdx.x * WPB + wv) * p.fpw;
    STAMP(0);
    if (f0 < p.n) uniform_stream_range(p, lds_all[wv], lane, f0);
    STAMP(2);
    STAMP(3);
}
#endif

#if SORTED_MODE == 0
// ---------------------------------------------------------------- IPv4 forwarding step
//
// pico_ipv4_pre_forward_checks (modules/pico_ipv4.c:1535-1574, called by pico_ipv4_forward :1600)
// on a batch of datagrams routed through this host, in batch order:
//   hdr->ttl = ttl - 1 (written back whatever follows); ttl < 1 -> expired (dropped, crc untouched);
//   else hdr->crc++ -- the reference's "HACK: increase crc to compensate decreased TTL": a native
//   (little-endian) uint16 increment of the stored big-endian field (RFC 1141's +0x0100 except where
//   it carries out of the first byte; kept exactly so, bit-compatible);
//   a source that is one of the host's link addresses -> dropped;
//   (src, id, dst, proto) equal to the last datagram that got this far -> dropped as a duplicate,
//   else it becomes the last one (static state in the reference; here a device struct carried from
//   one batch to the next).
// "The last datagram that got this far" is the nearest earlier datagram of the batch that passed the
// TTL and source checks (a duplicate leaves the state as it was: it equals it), or the carried state.
// Three launches on one stream:
//   K5a  one lane per datagram: TTL, crc++, local source -> verdict ACCEPT / EXPIRED / LOCAL_SRC.
//   K5b  one lane per datagram: the nearest earlier ACCEPT datagram (a wave ballot, then the
//        workgroup's wave maxima in LDS, then -- for the workgroup's first one only -- a backward
//        scan over the earlier verdict bytes, 256 a step), its tuple compared with this one's:
//        DUPLICATE.  Bytes another workgroup turns from ACCEPT to DUPLICATE meanwhile count the
//        same (both reached the check).
//   K5c  one workgroup: the batch's last such datagram's tuple -> the carried state.
struct FwdArgs {
    uint8_t* base;
    uint64_t base_len;
    const pico_csum_desc_dev* desc;
    uint32_t n;
    uint32_t n_local;
    uint8_t* verdict;
    uint32_t* state;          // {src, dst, id | proto << 16, reserved} as stored; NULL: zeros, not kept
    uint32_t local[32];       // the host's link addresses as stored (pico_ipv4_link_get's table)
};
constexpr uint32_t V_LOCAL_SRC = 32u, V_DUPLICATE = 64u;   // forwarding batch (include/pico_csum.h)

__device__ __forceinline__ uint32_t ld_le32(const uint8_t* p) {
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

// (src, dst, id | proto << 16) of datagram j, as stored
__device__ __forceinline__ uint3 fwd_tuple(const FwdArgs& p, uint32_t j) {
    const uint4 d = *reinterpret_cast<const uint4*>(p.desc + j);
    const uint8_t* h = p.base + (((uint64_t)d.y << 32) | d.x);
    return make_uint3(ld_le32(h + 12), ld_le32(h + 16),
                      ((uint32_t)h[4] | ((uint32_t)h[5] << 8)) | ((uint32_t)h[9] << 16));
}

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
            const uint32_t src = ld_le32(h + 12);
            bool local = false;
            for (uint32_t k = 0; k < p.n_local; ++k) local |= p.local[k] == src;
            v = local ? V_LOCAL_SRC : V_ACCEPT;
        }
    }
    p.verdict[i] = (uint8_t)v;
}

__device__ __forceinline__ bool fwd_reached(uint32_t v) { return v == V_ACCEPT || v == V_DUPLICATE; }

// The highest index < below (a multiple of 256) whose verdict byte says "reached the duplicate
// check", or -1: the whole workgroup scans backwards 256 bytes a step.
__device__ __forceinline__ int64_t fwd_scan_back(const FwdArgs& p, uint64_t below, int* wmax) {
    const uint32_t t = threadIdx.x, w = t >> 6;
    for (uint64_t top = below; top != 0; top -= 256u) {
        const uint64_t j = top - 256u + t;
        const bool e = fwd_reached(p.verdict[j]);
        const uint64_t b = __builtin_amdgcn_ballot_w64(e);
        __syncthreads();
        if ((t & 63u) == 0) wmax[w] = b ? 63 - __builtin_clzll(b) + 64 * (int)w : -1;
        __syncthreads();
        const int m = max(max(wmax[0], wmax[1]), max(wmax[2], wmax[3]));
        if (m >= 0) return (int64_t)(top - 256u) + m;
    }
    return -1;
}

__global__ __launch_bounds__(256) void ipv4_forward_dup_kernel(FwdArgs p) {
    __shared__ int wlast[4], wmax[4];
    const uint32_t t = threadIdx.x, lane = t & 63u, w = t >> 6;
    const uint64_t blk0 = (uint64_t)blockIdx.x * 256u, i = blk0 + t;
    const bool elig = i < p.n && p.verdict[i] == V_ACCEPT;   // this launch writes DUPLICATE only after the reads below
    const uint64_t b = __builtin_amdgcn_ballot_w64(elig);
    if (lane == 0) wlast[w] = b ? 63 - __builtin_clzll(b) : -1;
    __syncthreads();
    // nearest earlier eligible in the workgroup
    int64_t prev = -1;
    const uint64_t below = b & ((1ull << lane) - 1ull);
    if (below) {
        prev = (int64_t)(blk0 + 64u * w + 63u - __builtin_clzll(below));
    } else {
        for (int k = (int)w - 1; k >= 0; --k)
            if (wlast[k] >= 0) { prev = (int64_t)(blk0 + 64u * k + wlast[k]); break; }
    }
    // the workgroup's first eligible datagram looks further back (workgroup-uniform condition)
    const bool any = wlast[0] >= 0 || wlast[1] >= 0 || wlast[2] >= 0 || wlast[3] >= 0;
    int64_t back = -1;
    if (any && blk0 != 0) back = fwd_scan_back(p, blk0, wmax);
    if (!elig) return;
    if (prev < 0) prev = back;
    uint3 last;
    if (prev >= 0) {
        last = fwd_tuple(p, (uint32_t)prev);
    } else if (p.state) {
        last = make_uint3(p.state[0], p.state[1], p.state[2] & 0x00FFFFFFu);
    } else {
        last = make_uint3(0u, 0u, 0u);
    }
    const uint3 mine = fwd_tuple(p, (uint32_t)i);
    if (mine.x == last.x && mine.y == last.y && mine.z == last.z) p.verdict[i] = (uint8_t)V_DUPLICATE;
}

__global__ __launch_bounds__(256) void ipv4_forward_state_kernel(FwdArgs p) {
    __shared__ int wmax[4];
    const uint64_t top = ((uint64_t)p.n + 255u) & ~(uint64_t)255u;
    // verdict bytes past n are not ours: scan [top - 256, n) first with them masked
    const uint32_t t = threadIdx.x, w = t >> 6;
    int64_t last = -1;
    {
        const uint64_t j = top - 256u + t;
        const bool e = j < p.n && fwd_reached(p.verdict[j]);
        const uint64_t b = __builtin_amdgcn_ballot_w64(e);
        if ((t & 63u) == 0) wmax[w] = b ? 63 - __builtin_clzll(b) + 64 * (int)w : -1;
        __syncthreads();
        const int m = max(max(wmax[0], wmax[1]), max(wmax[2], wmax[3]));
        if (m >= 0) last = (int64_t)(top - 256u) + m;
    }
    if (last < 0 && top > 256u) last = fwd_scan_back(p, top - 256u, wmax);
    if (last >= 0 && t == 0) {
        const uint3 tu = fwd_tuple(p, (uint32_t)last);
        p.state[0] = tu.x;
        p.state[1] = tu.y;
        p.state[2] = tu.z;
    }
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

// One kernel per mode: this TU is compiled once per SORTED_MODE (parallel build).
#define SORTED_LAUNCH SORTED_CAT(pico_csum_sorted_launch_mode, SORTED_MODE)
int SORTED_LAUNCH(const void* args, void* stream);
int SORTED_LAUNCH(const void* args, void* stream) {
    const FlatArgs& a = *static_cast<const FlatArgs*>(args);
    const uint64_t waves = ((uint64_t)a.n + a.fpw - 1) / a.fpw;
    hipLaunchKernelGGL(csum_sorted_kernel<SORTED_MODE>, dim3((unsigned)((waves + WPB - 1) / WPB)),
                       dim3(64 * WPB), 0, static_cast<hipStream_t>(stream), a);
    return (int)hipGetLastError();
}

#if SORTED_MODE == 0
int pico_csum_sorted_launch_mode1(const void* args, void* stream);
int pico_csum_sorted_launch_mode2(const void* args, void* stream);
int pico_csum_sorted_launch_mode3(const void* args, void* stream);

// Sorted-rounds descriptor kernel: mode 0 RAW, 1 fused IPv4, 2 fused IPv6, 3 Ethernet front end;
// fpw frames per wave (1..64).  mac48 = the device MAC's 6 bytes (little-endian in a uint64),
// used when flags carry F_MACF (set by the host layer).
int pico_csum_launch_sorted(void* base, uint64_t base_len, const void* desc, uint32_t n, int mode, int32_t crc_off,
                            uint32_t flags, uint16_t* out, uint32_t* bad, uint16_t* out_net, uint16_t* out_l4,
                            uint8_t* verdict, uint32_t fpw, uint64_t mac48, void* stream) {
    if (fpw < 1 || fpw > 64 || mode < 0 || mode > 3) return (int)hipErrorInvalidValue;
    if (n == 0) return (int)hipSuccess;
    FlatArgs a{static_cast<uint8_t*>(base), base_len, static_cast<const pico_csum_desc_dev*>(desc), n, fpw,
               crc_off, flags, out, bad, out_net, out_l4, verdict, (uint32_t)mac48, (uint32_t)(mac48 >> 32)};
    switch (mode) {
        case 0: return pico_csum_sorted_launch_mode0(&a, stream);
        case 1: return pico_csum_sorted_launch_mode1(&a, stream);
        case 2: return pico_csum_sorted_launch_mode2(&a, stream);
        default: return pico_csum_sorted_launch_mode3(&a, stream);
    }
}

// Uniform rings on the stream waves (pico_csum.c decides when: dense rings): fpw frames per wave.
int pico_csum_launch_uniform_stream(const void* base, uint64_t stride, uint32_t len, uint32_t n, uint32_t seed,
                                    uint16_t* out, uint32_t fpw, void* stream) {
    if (n == 0) return (int)hipSuccess;
    if (fpw < 1) return (int)hipErrorInvalidValue;
    UniArgs a{static_cast<uint8_t*>(const_cast<void*>(base)), stride, len, n, seed, fpw, out};
    const uint64_t waves = ((uint64_t)n + fpw - 1u) / fpw;
    hipLaunchKernelGGL(csum_uniform_stream_kernel<4>, dim3((unsigned)((waves + WPB - 1u) / WPB)), dim3(64 * WPB), 0,
                       static_cast<hipStream_t>(stream), a);
    return (int)hipGetLastError();
}

int pico_csum_launch_ipv4_forward(void* base, uint64_t base_len, const void* desc, uint32_t n, const uint32_t* local,
                                  uint32_t n_local, uint32_t* state, uint8_t* verdict, void* stream) {
    if (n == 0) return (int)hipSuccess;
    if (n_local > 32 || !verdict) return (int)hipErrorInvalidValue;
    FwdArgs a{static_cast<uint8_t*>(base), base_len, static_cast<const pico_csum_desc_dev*>(desc), n, n_local, verdict,
              state, {}};
    for (uint32_t k = 0; k < n_local; ++k) a.local[k] = local[k];
    const hipStream_t s = static_cast<hipStream_t>(stream);
    const dim3 grid((unsigned)(((uint64_t)n + 255u) / 256u)), block(256);
    hipLaunchKernelGGL(ipv4_forward_kernel, grid, block, 0, s, a);
    hipLaunchKernelGGL(ipv4_forward_dup_kernel, grid, block, 0, s, a);
    if (state) hipLaunchKernelGGL(ipv4_forward_state_kernel, dim3(1), block, 0, s, a);
    return (int)hipGetLastError();
}
#endif  // SORTED_MODE == 0

}  // extern "C"

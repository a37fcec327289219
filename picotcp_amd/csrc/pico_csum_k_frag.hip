// pico_csum_k_frag.hip -- IPv4 and IPv6 fragment reassembly gather fused with the transport
// check of the reassembled datagram, and its launcher.
// Helpers, argument conventions and the arithmetic contract: pico_csum_dev.h.
//
// Reference: pico_ipv4_process_frag / pico_ipv6_process_frag / pico_fragments_check_complete /
// pico_fragments_reassemble (modules/pico_fragments.c:73-139, 216-239, 304-358, 432-568), then
// pico_transport_crc_check (stack/pico_socket.c:1916-1968) -- or, for ICMPv6,
// pico_icmp6_checksum -- on the reassembled frame.  IPv6 fragments are walked on device
// (ipv6_walk_packed, pico_csum_dev.h: pico_ipv6_extension_headers) for net_len, the fragment
// field and the transport protocol.
// The reference copies every fragment into a fresh frame (memcpy, :334-345) and then sums
// the whole transport again; here one pass reads each fragment's payload once, writes it to
// its place in the reassembled datagram and adds it to the checksum on the way.
//
// Batches of >= 512 datagrams take the flat grid (reasm_flat_kernel + the finish, below:
// the gather spread over ~one wave per four fragments, the plan and the sums brought together
// after it).  Otherwise -- and for a flat-grid datagram the plan could not settle -- one workgroup
// (4 waves; 1 wave in batches of >= 3072 datagrams) per datagram (its fragments are a contiguous
// descriptor range, in arrival order):
//   1. all threads parse the fragment headers (IPv4: IHL, total length, MF, offset; IPv6: the
//      extension-header walk, payload length, M, offset, protocol) into LDS and
//      mark repeated offsets (pico_tree_insert rejects a repeated key: the earliest arrival
//      of each offset is kept);
//   2. the gather starts at once: a kept fragment's place in the transport is its own offset
//      (completeness, checked beside it, requires offset == bookmark), so no wave waits for the
//      ordering.  Waves 1-3 gather fragments 1, 2, 3 mod 4 while wave 0 checks completeness
//      (rank by offset among the kept fragments, LDS broadcast reads; a wave prefix scan of
//      the sorted transport lengths against the offsets, up to the first fragment without MF,
//      which must be the last in tree order), copies the first fragment's 20 (IPv6: 40) header bytes,
//      then gathers fragments 0 mod 4 (one wave per datagram: the same, in order);
//   3. gather: two fragments' payloads per step (a wave's fragments w, w + 4, ... in pairs), in
//      16-byte units on the output's 16-byte lines, 3 x 64 units per wave per step (two 1480-byte
//      payloads): one byte-unaligned 16-byte load per unit through one buffer window over both
//      payloads (out-of-range slots read zeros, no branches; cached loads -- neighbouring units
//      share lines: non-temporal ones measured 123.4 / 132.2 us against 119.0 / 127.2 one
//      workgroup per datagram, profiles/r05/ab_reasm_flat.txt); v_dot2 sums on the
//      fly (every unit is a whole number of checksum words); a
//      workgroup reduction at the end.  Software-pipelined over two register sets: the next
//      step's loads are issued before this step's stores, and the stores are a fixed sequence
//      per unit (one 16-byte store if the unit is whole, else its whole dwords as a b64 and / or a
//      b32, then a last partial dword's bytes; the others at an out-of-range offset), so
//      the loads are waited on with the stores still in flight.  The fragments' metadata is
//      held in registers across two lanes' worth of indices (no LDS reads in the loop).
//      Measured (profiles/r03): one fragment per step 154.6 / 171.9 us (c3_reasm / c3_reasm6),
//      pairs 148.9 / 162.0 us (ab_frag2.txt), pipelined 144.8 / 153.4 us (ab_frag_pipe.txt);
//      without the stores 89.5 / 97.6 us, without the gather 18.2 / 26.2 us (ab_frag_ablate.txt,
//      measurement builds of round 3); one wave per datagram at 4096 datagrams 145.6 / 154.8 us vs
//      149.0 / 157.9 at four (ab_frag_wpd.txt).  Stores keep the default cache policy: nt 194 /
//      201 us, sc1 244 / 255 us (ab_frag_saux.txt).  Units on the output's 16-byte lines (every
//      interior unit one aligned b128 store, 5 store instructions per slot instead of 8): 130.6 /
//      140.2 us vs 145.5 / 154.7 (profiles/r03s2/ab_frag_grid.txt); the second line by DPP 128.5 /
//      138.3 us; one unaligned load 124.0 / 133.8 us (ab_frag_una.txt).  Tried, not kept (r03s2):
//      larger-occupancy LDS tables, three register sets, the completeness check or the header
//      copy after the gather, a lean whole-unit slot path with the edge units in 4 lanes, the
//      gather in tree order.
// The bytes of an output region are unspecified when its datagram is not reassembled, and past
// the reassembled datagram's end.
#include "pico_csum_dev.h"

#include <mutex>
#include <vector>

namespace {

// min / max of two device addresses (< 2^63) from the sign of their difference: scalar ALU only
// (a 64-bit compare is a vector instruction, whose temporaries inside the pipelined gather get
// waited on)
__device__ __forceinline__ uint64_t min64s(uint64_t a, uint64_t b) {
    return ((a - b) >> 63) ? a : b;
}
__device__ __forceinline__ uint64_t max64s(uint64_t a, uint64_t b) {
    return ((a - b) >> 63) ? b : a;
}

// sel4 as three selects (the nested form compiles to branches inside the pipelined gather)
__device__ __forceinline__ uint32_t sel4s(uint32_t q, uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
    const uint32_t lo = (q & 1u) ? b : a, hi = (q & 1u) ? d : c;
    return (q & 2u) ? hi : lo;
}

#ifndef FRAG_MAX_N
#define FRAG_MAX_N 512
#endif
constexpr uint32_t FRAG_MAX = FRAG_MAX_N;   // fragments per datagram handled on device

struct FragArgs {
    const uint8_t* base;
    uint32_t flags;                     // IPv6: F_NXD
    uint64_t base_len;
    const pico_csum_desc_dev* frag;
    const uint32_t* grp;                // 2 per datagram: first descriptor, count
    uint32_t n_dgram;
    uint32_t n_frag;
    uint8_t* out;
    uint64_t out_len;
    const pico_csum_desc_dev* odesc;    // per datagram: output region (off, capacity)
    uint32_t* o_len;
    uint16_t* o_l4;
    uint8_t* verdict;
    // flat grid (reasm_flat_kernel, then reasm_finish_kernel): S waves per datagram,
    // one plan per datagram, one partial sum per wave
    struct ReasmPlan* plan;
    uint32_t* slot;
    uint32_t S;
};

// A datagram's plan, written by its planner: GOOD (complete: the finish adds the waves' partial
// sums, less corr -- the sums of retransmitted fragments the gather waves gathered a second time),
// BAD (not reassembled) or SLOW (a repeated offset whose later arrival differs from the kept one,
// or more than FLAT_MAXF fragments: the finish runs the one-workgroup path over the datagram again).
struct ReasmPlan {
    uint32_t state, len, proto, pseudo, w0, w1, corr, pad;
};
constexpr uint32_t PLAN_GOOD = 0u, PLAN_BAD = 1u, PLAN_SLOW = 2u;
constexpr uint32_t FLAT_MAXF = 128u;         // fragments a plan holds (two a lane)
#ifndef REASM_NP4
#define REASM_NP4 2u
#endif
#ifndef REASM_NP6
#define REASM_NP6 3u
#endif
// The gathers' whole 16-byte unit stores are non-temporal (aux 2, `nt`): c3_reasm 105.5-107.4 us
// against 110.0-110.8 cached, c3_reasm6 111.2-112.1 against 117.9-118.8; the edge units' partial
// stores the same either way (profiles/r06/ab_reasm_nts.txt).  Write-through `sc1` (16), `sc1 nt`
// (18) or `sc0 sc1` (17) whole-unit stores: c3_reasm 116.4-117.2 / 112.9-114.3 / 116.5-116.8 us,
// c3_reasm6 125.6-125.9 / 123.2-123.7 / 125.7-125.9 (ab_reasm_sc1.txt).  The payload loads stay
// cached (reasm_flat_kernel).
#ifndef REASM_FLAT_LDS
// LDS a flat-grid wave reserves when its datagrams average <= 64 fragments: 8 KiB holds the grid
// at 5 waves a SIMD (20 a CU; the IPv4 kernel's 62 VGPRs would allow 8).  c3_reasm_retx 111.9-112.0
// against 119.0-119.3 us, c3_reasm and c3_reasm6 the same (99.3-99.5 / 105.8-106.4); smaller
// fragments want every wave: c3_reasm_576 186.4-186.7 capped against 159.0-159.3
// (profiles/r06/ab_reasm_flat_occupancy.txt).
#define REASM_FLAT_LDS 8192u
#endif
#ifndef REASM_STORE_AUX
#define REASM_STORE_AUX 2
#endif
#ifndef REASM_EDGE_AUX
#define REASM_EDGE_AUX 0
#endif
// fragment pairs a flat-grid wave gathers at once (their loads in flight together): IPv4 2
// (3: 113.2 vs 113.4 us, no gain), IPv6 3 (120.9 us; 2: 128.0, 4: 122.2 at 118 VGPRs); again
// with the nt stores (profiles/r06/ab_reasm_np.txt): IPv4 3 pairs 106.5-107.7 against 103.2-103.8,
// IPv6 2 / 4 pairs 114.7-115.4 / 114.2-114.6 against 110.7-111.1; on c3_reasm_576 (552 B fragments) IPv4
// 3 / 4 pairs 155.3-155.6 / 154.4-155.2 against 158.9-159.3, c3_reasm 102.8-102.9 / 111.1 against
// 98.4-99.7 (ab_reasm576_np.txt: not worth a second instantiation)
__host__ __device__ constexpr uint32_t flat_np(bool v6) { return v6 ? REASM_NP6 : REASM_NP4; }
// Datagrams a planner workgroup plans in turn: 512 planners, at most 8 datagrams each (c3_reasm /
// c3_reasm6, 4096 datagrams: 8 a planner 113.7 / 127.3 us, 4 127.4 (IPv6), 1 118.0 / 130.0, 16
// 130.5 / 143.6 -- the planners then end in the launch's tail).  Again on the final gather
// (profiles/r06/ab_reasm_plan_per_final.txt): 4 a planner c3_reasm 98.6-99.3 vs 97.7-98.1 us,
// c3_reasm6 104.8-106.1 vs 104.6, c3_reasm_retx 105.9-106.8 vs 110.1-110.3; 16: 114.5 / 130.2 / 169
// A planner that loads the next datagram's descriptors before planning this one and its headers
// before this one's header copy measured no better: c3_reasm 102.7-104.1 against 104.4-105.1 us,
// c3_reasm6 112.6-113.7 against 110.2-111.2, c3_reasm_retx 119.3-119.8 against 111.6-113.4; with
// the gather's occupancy held at 4 / 5 / 5.5 waves a SIMD (LDS) slower still
// (profiles/r06/ab_reasm_plan_pipelined.txt, ab_reasm_plan_occupancy.txt).
__host__ __device__ __forceinline__ uint32_t plan_per(uint32_t n_dgram) {
#ifdef REASM_PLAN_PER
    return REASM_PLAN_PER;
#endif
    const uint32_t q = n_dgram / 512u;
    return q < 1u ? 1u : (q > 8u ? 8u : q);
}             // fragment pairs a flat-grid wave gathers at once

struct FragLds {
    uint32_t key[FRAG_MAX];   // offset | MF << 16 | dup << 24
    uint32_t tl[FRAG_MAX];    // transport length
    uint16_t sidx[FRAG_MAX];  // tree position -> fragment
    uint64_t src[FRAG_MAX];   // fragment -> payload address (no descriptor re-read in the gather)
    uint8_t pr[FRAG_MAX];     // IPv6: the walk's transport protocol (the module it is handed to)
    uint32_t len, bad, proto, pseudo, first0;
    uint32_t acc[4], w0[4], w1[4];
};

__device__ __forceinline__ uint32_t ld_u8(const uint8_t* p) { return (uint32_t)*p; }

// One masked unit's stores into the output window at so (16-byte aligned): the whole unit as one
// aligned 16-byte store; else, by the edge lanes alone (exec-masked), its whole dwords [a, a + c)
// as a b64 and / or a b32, then its last partial dword's bytes as a b16 and / or a b8.  The whole
// units' stores are non-temporal (REASM_STORE_AUX).
__device__ __forceinline__ void edge_store(const Window& ow, const uint32_t (&xw)[4], uint32_t lo, uint32_t hi, uint32_t so) {
    const bool whole = lo == 0u && hi == 16u;
    __builtin_amdgcn_raw_buffer_store_b128((u32x4){xw[0], xw[1], xw[2], xw[3]}, ow.rsrc, (int)(whole ? so : WIN_OOB), 0,
                                           REASM_STORE_AUX);
    if (!whole && hi > lo) {
        const uint32_t a = lo >> 2, bq = hi >> 2, c = bq <= a ? 0u : bq - a, nr = hi & 3u;
        const uint32_t a1 = min(a + 1u, 3u), a2 = c >= 2u ? a + 2u : a;
        const uint32_t tw = sel4s(bq & 3u, xw[0], xw[1], xw[2], xw[3]);
        if (c >= 2u)
            __builtin_amdgcn_raw_buffer_store_b64(
                (u32x2){sel4s(a & 3u, xw[0], xw[1], xw[2], xw[3]), sel4s(a1, xw[0], xw[1], xw[2], xw[3])}, ow.rsrc,
                (int)(so + 4u * a), 0, REASM_EDGE_AUX);
        if (c & 1u)
            __builtin_amdgcn_raw_buffer_store_b32(sel4s(a2 & 3u, xw[0], xw[1], xw[2], xw[3]), ow.rsrc, (int)(so + 4u * a2),
                                                  0, REASM_EDGE_AUX);
        if (nr >= 2u) __builtin_amdgcn_raw_buffer_store_b16((unsigned short)tw, ow.rsrc, (int)(so + 4u * bq), 0, REASM_EDGE_AUX);
        if (nr & 1u)
            __builtin_amdgcn_raw_buffer_store_b8((unsigned char)(tw >> (8u * (nr & 2u))), ow.rsrc,
                                                 (int)(so + 4u * bq + (nr & 2u)), 0, REASM_EDGE_AUX);
    }
}

// One fragment's header.  IPv4 as pico_ipv4_process_in hands a fragment on (net_len,
// transport_len = tot - net_len, frag); IPv6 as pico_ipv6_extension_headers does (the walk must
// reach the transport behind a fragment header; transport_len = payload_len - (net_len - 40)).
// key = offset | MF << 16; pr: IPv6, the walk's transport protocol.  False: the fragment is
// malformed (its datagram is not reassembled).
template <bool V6>
__device__ __forceinline__ bool frag_parse(const FragArgs& p, const pico_csum_desc_dev& d, uint32_t& key, uint32_t& tl,
                                           uint32_t& hl, uint32_t& pr) {
    constexpr uint32_t HDR = V6 ? 40u : 20u;
    key = tl = hl = pr = 0;
    if (d.len < HDR || d.off > p.base_len || d.len > p.base_len - d.off) return false;
    const uint8_t* h = p.base + d.off;
    if constexpr (!V6) {
        const uint32_t ihl = ld_u8(h) & 0x0Fu;
        hl = 20u + (ihl > 5u ? 4u * (ihl - 5u) : 0u);
        tl = (((ld_u8(h + 2) << 8) | ld_u8(h + 3)) - hl) & 0xFFFFu;
        const uint32_t frag = (ld_u8(h + 6) << 8) | ld_u8(h + 7);
        key = ((frag & 0x1FFFu) << 3) | ((frag & 0x2000u) ? 1u << 16 : 0u);
        return hl + tl <= d.len;
    } else {
        // the common chain -- the fixed header, a fragment header, the transport -- from loads
        // issued together (the walk's are a dependent chain); it is exactly what the walk returns
        // for that chain (net_len 48, M with a payload length not a multiple of 8 dropped)
        uint64_t w;
        const uint32_t h6 = ld_u8(h + 6);
        if (d.len > 43u) {
            const uint32_t h40 = ld_u8(h + 40), om = (ld_u8(h + 42) << 8) | ld_u8(h + 43);
            const uint32_t plen = (ld_u8(h + 4) << 8) | ld_u8(h + 5);
            if (h6 == 44u && (h40 == 6u || h40 == 17u || h40 == 58u))
                w = ((om & 1u) && (plen & 7u)) ? (uint64_t)(WALK_DROP + 1)
                                               : ((uint64_t)om << 32) | (uint32_t)(WALK_FRAG + 1) | (48u << 8) | (h40 << 24);
            else
                w = ipv6_walk_packed(h, d.len);
        } else {
            w = ipv6_walk_packed(h, d.len);
        }
        const uint32_t om = (uint32_t)(w >> 32);
        hl = ((uint32_t)w >> 8) & 0xFFFFu;
        tl = ((((ld_u8(h + 4) << 8) | ld_u8(h + 5))) - (hl - 40u)) & 0xFFFFu;
        key = (om & 0xFFF8u) | ((om & 1u) << 16);
        pr = ((uint32_t)w >> 24) & 0xFFu;
        return (int)(w & 0xFFu) - 1 == WALK_FRAG && hl + tl <= d.len;
    }
}

// frag_parse from the header's bytes 0..15 (v0) and, IPv6, 40..55 (v40) already in registers (the
// flat grid reads every fragment's header in every wave: one 16-byte load per lane instead of a
// byte load per field).  pre = false (the header outside the wave's load window): frag_parse.
template <bool V6>
__device__ __forceinline__ bool frag_parse_pre(const FragArgs& p, const pico_csum_desc_dev& d, bool pre, uint4 v0,
                                               uint4 v40, uint32_t& key, uint32_t& tl, uint32_t& hl, uint32_t& pr) {
    constexpr uint32_t HDR = V6 ? 40u : 20u;
    if (!pre) return frag_parse<V6>(p, d, key, tl, hl, pr);
    key = tl = hl = pr = 0;
    if (d.len < HDR || d.off > p.base_len || d.len > p.base_len - d.off) return false;
    if constexpr (!V6) {
        const uint32_t ihl = v0.x & 0x0Fu;
        hl = 20u + (ihl > 5u ? 4u * (ihl - 5u) : 0u);
        tl = (((((v0.x >> 16) & 0xFFu) << 8) | (v0.x >> 24)) - hl) & 0xFFFFu;
        const uint32_t frag = (((v0.y >> 16) & 0xFFu) << 8) | (v0.y >> 24);
        key = ((frag & 0x1FFFu) << 3) | ((frag & 0x2000u) ? 1u << 16 : 0u);
        return hl + tl <= d.len;
    } else {
        const uint32_t h6 = (v0.y >> 16) & 0xFFu, plen = ((v0.y & 0xFFu) << 8) | ((v0.y >> 8) & 0xFFu);
        const uint32_t h40 = v40.x & 0xFFu, om = (((v40.x >> 16) & 0xFFu) << 8) | (v40.x >> 24);
        uint64_t w;
        // (v40 is zero when its 16 bytes run past the buffer: h40 = 0, the walk)
        if (d.len > 43u && h6 == 44u && (h40 == 6u || h40 == 17u || h40 == 58u))
            w = ((om & 1u) && (plen & 7u)) ? (uint64_t)(WALK_DROP + 1)
                                           : ((uint64_t)om << 32) | (uint32_t)(WALK_FRAG + 1) | (48u << 8) | (h40 << 24);
        else
            w = ipv6_walk_packed(p.base + d.off, d.len);
        const uint32_t omw = (uint32_t)(w >> 32);
        hl = ((uint32_t)w >> 8) & 0xFFFFu;
        tl = (plen - (hl - 40u)) & 0xFFFFu;
        key = (omw & 0xFFF8u) | ((omw & 1u) << 16);
        pr = ((uint32_t)w >> 24) & 0xFFu;
        return (int)(w & 0xFFu) - 1 == WALK_FRAG && hl + tl <= d.len;
    }
}

// The flat grid's header reads: lane's fragment descriptor p.frag[idx] (in: the lane has one), then
// its header's first 16 bytes (IPv6: also bytes 40..55) in one load each through a window over
// the batch from 1 GiB below the wave's first fragment, parsed by frag_parse_pre (a header
// outside the window: frag_parse's byte loads).  Returns frag_parse's verdict (true without one).
template <bool V6>
__device__ __forceinline__ bool parse_lane(const FragArgs& p, bool in, uint32_t idx, uint64_t& off, uint32_t& key,
                                           uint32_t& tl, uint32_t& hl, uint32_t& pr) {
    pico_csum_desc_dev d{0, 0, 0};
    if (in) d = p.frag[idx];
    off = d.off;
    key = tl = hl = pr = 0;
#ifdef REASM_BYTE_PARSE
    return in ? frag_parse<V6>(p, d, key, tl, hl, pr) : true;
#else
    const uint64_t act = __builtin_amdgcn_ballot_w64(in);
    const int f = act ? __builtin_ffsll((long long)act) - 1 : 0;
    const uint64_t a0 = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)off, f) |
                        ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(off >> 32), f) << 32);
    const uint64_t lo = a0 > (1ull << 30) ? (a0 - (1ull << 30)) & ~(uint64_t)15 : 0ull;
    const uint64_t wsz = p.base_len > lo ? min(p.base_len - lo, (uint64_t)0x7FFFFFF0u) : 0ull;
    const Window hw = make_window(reinterpret_cast<uint64_t>(p.base) + lo, (uint32_t)wsz);
    const bool pre = in && off >= lo && off - lo + (V6 ? 56u : 16u) <= wsz;
    const uint32_t v = pre ? (uint32_t)(off - lo) : WIN_OOB;
    const uint4 v0 = load_win<false>(hw, v);
    const uint4 v40 = V6 ? load_win<false>(hw, pre ? v + 40u : WIN_OOB) : make_uint4(0, 0, 0, 0);
    return in ? frag_parse_pre<V6>(p, d, pre, v0, v40, key, tl, hl, pr) : true;
#endif
}

// pico_transport_crc_check on the reassembled frame (ICMPv6: pico_icmp6_process_in): s = the
// transport's word sum, word0 / word1 = its bytes 0..3 / 4..7 (little-endian)
template <bool V6>
__device__ __forceinline__ uint32_t reasm_verdict(uint32_t flags, uint32_t len, uint32_t proto, uint32_t pseudo,
                                                  uint32_t s, uint32_t word0, uint32_t word1, uint32_t& l4) {
    uint32_t v = V_ACCEPT;
    l4 = 0;
    if constexpr (!V6) {
        if (proto == 6u || (proto == 17u && len >= 8u && (word1 >> 16) != 0u)) {
            l4 = finalize(pseudo + s);
            if (l4) v = V_L4_BAD;
        }
    } else {
        const uint32_t module = proto & 0xFFu, b9 = proto >> 8;
        uint32_t cp = module;
        bool check = false;
        if (module == 6u || module == 17u) {
            if (!(flags & F_NXD)) cp = b9;                // pico_socket.c:1923 through the IPv4 cast
            check = cp == 6u || (cp == 17u && len >= 8u && (word1 >> 16) != 0u);
        } else if (module == 58u && len >= 1u) {
            check = true;
        }
        if (check) {
            l4 = finalize(pseudo + (cp << 8) + s);
            const uint32_t type = word0 & 0xFFu;
            const bool checked = module != 58u || (type >= 130u && type <= 137u) || type == 143u;
            if (l4 && checked) v = V_L4_BAD;
        }
    }
    return v;
}

// Datagram g on the workgroup (WPD waves: 1 or 4; the launcher picks it from the batch size),
// L its LDS tables; g < n_dgram
template <bool V6, int WPD>
__device__ __forceinline__ void reassemble_one(const FragArgs& p, uint32_t g, FragLds& L) {
    constexpr uint32_t HDR = V6 ? 40u : 20u;          // PICO_SIZE_IP6HDR / PICO_SIZE_IP4HDR
    constexpr uint32_t NT = 64u * WPD;
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wv = tid >> 6;
    const uint32_t first = p.grp[2 * g], cnt = p.grp[2 * g + 1];
    const pico_csum_desc_dev od = p.odesc[g];
    const bool bad0 = cnt == 0 || cnt > FRAG_MAX || first > p.n_frag || cnt > p.n_frag - first ||
                      (od.off & 3u) != 0 || od.off > p.out_len || od.len > p.out_len - od.off || od.len < HDR;
    if (tid == 0) {
        L.bad = bad0 ? 1u : 0u;
        L.first0 = NONE;
    }
    __syncthreads();

    // ---- 1. parse (frag_parse)
    if (!bad0) {
        for (uint32_t j = tid; j < cnt; j += NT) {
            const pico_csum_desc_dev d = p.frag[first + j];
            uint32_t key, tl, hl, pr;
            if (!frag_parse<V6>(p, d, key, tl, hl, pr)) L.bad = 1u;
            if constexpr (V6) L.pr[j] = (uint8_t)pr;
            L.key[j] = key;
            L.tl[j] = tl;
            L.src[j] = reinterpret_cast<uint64_t>(p.base + d.off) + hl;
        }
    }
    __syncthreads();
    bool bad = L.bad != 0;                              // workgroup-uniform
    if (!bad) {                                         // repeated offsets: the earliest arrival stays
        for (uint32_t j = tid; j < cnt; j += NT) {
            const uint32_t fj = L.key[j] & 0xFFFFu;
            bool dup = false;
            for (uint32_t k = 0; k < j; ++k) dup |= (L.key[k] & 0xFFFFu) == fj;
            if (dup) L.key[j] |= 1u << 24;
            else if (fj == 0u) L.first0 = j;            // the tree's first fragment (offset 0)
        }
    }
    __syncthreads();
    uint8_t* t = p.out + od.off + HDR;
    const uint32_t cap = od.len - HDR;                  // transport bytes the output region holds

    // ---- 2. wave 0: completeness (pico_fragments_check_complete) and the header
    if (wv == 0 && !bad) {
        uint32_t kept = 0;
        for (uint32_t j = lane; j < cnt; j += 64u) {
            const uint32_t kj = L.key[j];
            if (kj >> 24) continue;
            uint32_t r = 0;
            for (uint32_t k = 0; k < cnt; ++k) {
                const uint32_t kk = L.key[k];
                r += ((kk >> 24) == 0 && (kk & 0xFFFFu) < (kj & 0xFFFFu)) ? 1u : 0u;
            }
            L.sidx[r] = (uint16_t)j;
            ++kept;
        }
        const uint32_t m = (uint32_t)__builtin_amdgcn_readlane((int)group_sum<64>(kept), 63);
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_s_waitcnt(0xC07F);
        uint32_t carry = 0, e = NONE, len = 0;
        bool gap = false;
        for (uint32_t i0 = 0; i0 < m && e == NONE; i0 += 64u) {
            const uint32_t i = i0 + lane;
            const bool in = i < m;
            const uint32_t j = in ? L.sidx[i] : 0u;
            const uint32_t kj = in ? L.key[j] : 0u, tl = in ? L.tl[j] : 0u;
            const uint32_t incl = wave_scan_add(tl);
            const uint32_t P = carry + incl - tl;
            const uint64_t last = __builtin_amdgcn_ballot_w64(in && !(kj & (1u << 16)));
            const uint32_t le = last ? (uint32_t)__builtin_ctzll(last) : 64u;     // first MF-clear lane
            gap |= __builtin_amdgcn_ballot_w64(in && lane <= le && (kj & 0xFFFFu) != P) != 0;
            if (last) {
                e = i0 + le;
                len = (uint32_t)__builtin_amdgcn_readlane((int)(P + tl), (int)le);
            }
            carry += (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
        }
        const bool b = gap || e == NONE || e + 1u != m || HDR + len > 0xFFFFu || len > cap;
        // the first fragment's PICO_SIZE_IP4HDR / PICO_SIZE_IP6HDR bytes (pico_fragments.c:332-338)
        // and the pseudo header's address part: IPv4 struct pico_ipv4_pseudo_hdr as LE words (src,
        // dst, proto << 8, bswap16(len)); IPv6 struct pico_ipv6_pseudo_hdr (src, dst, long_be(len);
        // the next-header word is added in phase 4, once the checked protocol is known)
        uint32_t proto = 0, pseudo = 0;
        if (!b) {
            const uint8_t* h0 = p.base + p.frag[first + L.first0].off;
            const uint32_t hb = lane < HDR ? ld_u8(h0 + lane) : 0u;
            if (lane < HDR) t[(int)lane - (int)HDR] = (uint8_t)hb;
            if constexpr (!V6) {
                proto = (uint32_t)__shfl((int)hb, 9);
                const uint32_t pw = lane >= 12u && lane < 20u ? (lane & 1u ? hb << 8 : hb) : 0u;
                pseudo = (uint32_t)__builtin_amdgcn_readlane((int)group_sum<64>(pw), 63) + (proto << 8) +
                         (((len & 0xFFu) << 8) | ((len >> 8) & 0xFFu));
            } else {
                // the module: the walk's protocol of the chain fragment that arrived last (the
                // arrival that completes the set hands its protocol on, pico_fragments.c:492);
                // byte 9 of the copied header rides in bits 8-15 (the reference's TCP / UDP dispatch)
                uint32_t last = 0;
                for (uint32_t i = lane; i <= e; i += 64u) last = max(last, (uint32_t)L.sidx[i] + 1u);
                last = (uint32_t)__builtin_amdgcn_readlane((int)wave_scan_max(last), 63) - 1u;
                proto = (uint32_t)L.pr[last] | ((uint32_t)__shfl((int)hb, 9) << 8);
                const uint32_t pw = lane >= 8u && lane < 40u ? (lane & 1u ? hb << 8 : hb) : 0u;
                pseudo = (uint32_t)__builtin_amdgcn_readlane((int)group_sum<64>(pw), 63) +
                         (((len >> 24) & 0xFFu) | ((len >> 8) & 0xFF00u)) + (((len & 0xFFu) << 8) | ((len >> 8) & 0xFFu));
            }
        }
        if (lane == 0) {
            L.len = b ? 0u : len;
            L.proto = proto;
            L.pseudo = pseudo;
            if (b) L.bad = 1u;
        }
    }

    // ---- 3. gather + checksum, all waves (wave w: fragments w, w + WPD, ... in arrival order, two
    //         at a time), each kept fragment at its own offset.  Software-pipelined: a step's
    //         loads are issued before the previous step is stored, and every load and store of a
    //         step is issued unconditionally (buffer operations, out-of-range offsets do nothing),
    //         so the in-order vmcnt the loads are waited on never includes the stores before them.
    uint32_t acc = 0, w0 = 0, w1 = 0;
    if (!bad) {
        const uint64_t tb = reinterpret_cast<uintptr_t>(t);
        const Window ow = make_window(tb, cap);           // the transport part of the output region
        // a kept fragment the output region can hold (else its datagram is not reassembled:
        // past the region's end, or larger than it); wave-uniform
        auto uni = [](uint32_t x) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)x); };
        // this wave's fragments j = w + WPD i, held 64 at a time in one register per field (lane
        // i - cb: fragment i), read when the walk enters the block: the loop below reads no LDS
        // inside a block (an LDS read there waits on the loads issued ahead of it)
        const uint32_t w = uni(wv);
        const uint32_t nidx = cnt > w ? (cnt - w + WPD - 1u) / WPD : 0u;   // this wave's fragments
        constexpr uint32_t NONE_I = 0xFFFFFFFFu;
        uint32_t cb = 0, ck, ct, cl, ch;
        uint64_t gm;                          // bit i - cb: fragment i is gathered
        auto load_block = [&](uint32_t b) {
            cb = b;
            const uint32_t j = w + WPD * (b + lane);
            const bool in = j < cnt;
            ck = in ? L.key[j] : 0u;
            ct = in ? L.tl[j] : 0u;
            const uint64_t x = in ? L.src[j] : 0ull;
            cl = (uint32_t)x;
            ch = (uint32_t)(x >> 32);
            // kept, and inside the output region (else the datagram is not reassembled: past the
            // region's end, or larger than it)
            gm = __builtin_amdgcn_ballot_w64(in && (ck >> 24) == 0 && (ck & 0xFFFFu) + ct <= cap);
        };
        load_block(0);
        auto field = [&](uint32_t c, uint32_t i) { return (uint32_t)__builtin_amdgcn_readlane((int)c, (int)(i - cb)); };
        auto next_gathered = [&](uint32_t i) {        // first gathered i' >= i (its block loaded), else NONE_I
            for (;;) {
                if (i >= nidx) return NONE_I;
                if (i >= cb + 64u) load_block(i & ~63u);
                const uint64_t m = gm & (~0ull << (i - cb));
                if (m) return cb + (uint32_t)__builtin_ctzll(m);
                i = cb + 64u;
            }
        };
        auto src_of = [&](uint32_t i) { return ((uint64_t)field(ch, i) << 32) | field(cl, i); };
        constexpr int U = 3;                   // 64-unit slots per step: two 1480 B payloads
        struct Step {                          // plain scalars (a buffer resource inside a copied
            uint64_t wlo;                      // struct ends up in an LDS-promoted alloca)
            uint32_t wsz, i, i2, va, vb, na, nt, ta, tb, ata, atb, oa, ob, u0, valid;
        };
        // Units follow the OUTPUT's 16-byte lines: a fragment whose place starts o = (t + offset) & 15
        // bytes into a line has units [0, (o + tl + 15) / 16), unit u = its bytes [16 u - o, 16 u - o + 16),
        // so every unit but its first and last is one aligned 16-byte store (units on the payload's own
        // grid gave dword stores for every unit of a fragment at 8 mod 16).  The loads take the shift:
        // one byte-unaligned 16-byte load per unit.
        // fragment A = i and (if any) B = i2: units [0, na) are A's, [na, nt) B's, read through
        // one buffer window over both payloads' 16-byte lines when they lie within 1 GiB of each
        // other (else B waits for the next step)
        auto make_pair = [&](uint32_t i0) {
            Step st;
            const uint32_t i = next_gathered(i0);
            st.valid = i != NONE_I;
            st.u0 = 0;
            st.i = st.i2 = i;
            st.wlo = tb;
            st.wsz = 0;
            st.va = st.vb = st.na = st.nt = st.ta = st.tb = st.ata = st.atb = st.oa = st.ob = 0;
            if (!st.valid) return st;
            st.ata = field(ck, i) & 0xFFFFu;
            st.oa = (uint32_t)((tb + st.ata) & 15u);
            const uint64_t sa = src_of(i) - st.oa;        // where unit 0 starts (o bytes before the payload)
            st.ta = field(ct, i);
            st.na = (st.oa + st.ta + 15u) >> 4;
            const uint32_t i2 = next_gathered(i + 1u);   // (may move the block past i)
            uint64_t sb = sa;
            st.tb = st.atb = 0;
            uint32_t nb = 0;
            if (i2 != NONE_I) {
                const uint32_t atb = field(ck, i2) & 0xFFFFu, ob = (uint32_t)((tb + atb) & 15u);
                const uint64_t sb2 = src_of(i2) - ob;
                const uint32_t tb2 = field(ct, i2);
                const uint64_t lo = min64s(sa, sb2) & ~15ull, hi = max64s(sa + st.oa + st.ta, sb2 + ob + tb2) + 16u;
                if (hi - lo < (1ull << 30)) {
                    sb = sb2;
                    nb = (ob + tb2 + 15u) >> 4;
                    st.tb = tb2;
                    st.atb = atb;
                    st.ob = ob;
                    st.i2 = i2;
                }
            }
            const uint64_t wlo = (nb ? min64s(sa, sb) : sa) & ~15ull;
            const uint64_t whi = nb ? max64s(sa + st.oa + st.ta, sb + st.ob + st.tb) : sa + st.oa + st.ta;
            st.wlo = wlo;
            st.wsz = (uint32_t)(((whi + 15u) & ~15ull) - wlo + 16u);
            st.va = (uint32_t)(sa - wlo);
            st.vb = (uint32_t)(sb - wlo);
            st.nt = st.na + nb;
            return st;
        };
        auto next_step = [&](const Step& c) {
            Step n = c;
            if (c.u0 + 64u * U < c.nt) n.u0 += 64u * U;
            else n = make_pair((c.i2 == c.i ? c.i : c.i2) + 1u);
            return n;
        };
        // (rows past a pair's units load through the void offset: skipping them by a uniform
        // branch, as the flat grid's pair_issue does, measured slower here -- c3_reasm_576 on this
        // path 190.8 vs 180.0 us, c3_reasm 128.4-129.5 vs 124.3-125.1; ab_reasm_wg_void_rows.txt)
        auto issue = [&](const Step& st, uint4 (&c0)[U]) {
            const Window win = make_window(st.wlo, st.wsz);   // empty for an invalid step
#pragma unroll
            for (int k = 0; k < U; ++k) {
                const uint32_t x = st.u0 + 64u * k + lane;
                const bool inb = x >= st.na;
                const uint32_t u = inb ? x - st.na : x, v = inb ? st.vb : st.va;
                const bool ok = st.valid && x < st.nt;
                c0[k] = load_win<false>(win, ok ? v + 16u * u : WIN_OOB);   // byte-unaligned: the unit's 16 bytes
            }
        };
        auto process = [&](const Step& st, const uint4 (&c0)[U]) {
#pragma unroll
            for (int k = 0; k < U; ++k) {
                const uint32_t x = st.u0 + 64u * k + lane;
                const bool ok = x < st.nt;
                const bool inb = x >= st.na;
                const uint32_t u = inb ? x - st.na : x;
                const uint32_t tl = inb ? st.tb : st.ta, at = inb ? st.atb : st.ata, o = inb ? st.ob : st.oa;
                uint32_t xw[4] = {c0[k].x, c0[k].y, c0[k].z, c0[k].w};
                // the unit's fragment bytes are [lo, hi) of its 16 (lo = o in unit 0, a multiple of 4;
                // hi < 16 only in the last unit); the rest is the neighbours' and reads as zero
                const uint32_t lo = ok && u == 0u ? o : 0u, hi = ok ? min(16u, o + tl - 16u * u) : 0u;
#pragma unroll
                for (int w = 0; w < 4; ++w) {
                    const uint32_t kb = 4u * w < lo ? 0u : min((uint32_t)max((int)hi - 4 * w, 0), 4u);
                    xw[w] &= (uint32_t)(0xFFFFFFFFull >> (32u - 8u * kb));
                }
                // stores: edge_store (the whole unit, or an edge unit's bytes by its lane alone)
                const uint32_t so = at + 16u * u - o;       // the unit's place (16-byte aligned in t)
                edge_store(ow, xw, lo, hi, so);
                acc = dot2_add(xw[3], dot2_add(xw[2], dot2_add(xw[1], dot2_add(xw[0], acc))));   // even offset
                if (ok && at + 16u * u <= o + 4u) {         // transport bytes 0..3 (ICMPv6 type), 4..7 (UDP crc)
#pragma unroll
                    for (int w = 0; w < 4; ++w) {
                        const uint32_t tp = at + 16u * u + 4u * w - o;   // (wraps below the transport: no match)
                        w0 |= tp == 0u ? xw[w] : 0u;
                        w1 |= tp == 4u ? xw[w] : 0u;
                    }
                }
            }
        };
        uint4 a0[U], b0[U];
        Step cur = make_pair(0u);
        if (cur.valid) {
            issue(cur, a0);
            for (;;) {                         // two steps per trip, alternating register sets
                const Step n1 = next_step(cur);
                issue(n1, b0);
                __builtin_amdgcn_sched_barrier(0);   // the next step's loads stay ahead of these stores
                process(cur, a0);
                if (!n1.valid) break;
                const Step n2 = next_step(n1);
                issue(n2, a0);
                __builtin_amdgcn_sched_barrier(0);
                process(n1, b0);
                if (!n2.valid) break;
                cur = n2;
            }
        }
        acc = (uint32_t)__builtin_amdgcn_readlane((int)group_sum<64>(acc), 63);
        w0 = (uint32_t)__builtin_amdgcn_readlane((int)group_sum<64>(w0), 63);
        w1 = (uint32_t)__builtin_amdgcn_readlane((int)group_sum<64>(w1), 63);
        if (lane == 0) {
            L.acc[wv] = acc;
            L.w0[wv] = w0;
            L.w1[wv] = w1;
        }
    }
    __syncthreads();
    bad = L.bad != 0;

    // ---- 4. pico_transport_crc_check on the reassembled frame (ICMPv6: pico_icmp6_process_in)
    if (tid == 0) {
        uint32_t l4 = 0, v = V_MALFORMED;
        const uint32_t len = L.len, proto = L.proto;
        if (!bad) {
            uint32_t s = 0, word0 = 0, word1 = 0;
#pragma unroll
            for (int k = 0; k < WPD; ++k) {
                s += L.acc[k];
                word0 |= L.w0[k];
                word1 |= L.w1[k];
            }
            v = reasm_verdict<V6>(p.flags, len, proto, L.pseudo, s, word0, word1, l4);
        }
        if (p.o_len) p.o_len[g] = bad ? 0u : len;
        if (p.o_l4) p.o_l4[g] = (uint16_t)l4;
        if (p.verdict) p.verdict[g] = (uint8_t)v;
    }
}

template <bool V6, int WPD>
__global__ __launch_bounds__(64 * WPD) void reassemble_kernel(FragArgs p) {
    __shared__ FragLds L;
    if (blockIdx.x < p.n_dgram) reassemble_one<V6, WPD>(p, blockIdx.x, L);
}

// The flat grid's finish: a workgroup of 4 waves per 64 datagrams.  Wave 0, one lane per datagram,
// gives a GOOD or BAD plan its results from the plan and the S partial sums; then all 4 waves run
// the workgroup path (reassemble_one, 4 waves) over each SLOW datagram of the 64 in turn.  (Round 5:
// one wave per 64 datagrams, its SLOW datagrams on the one-wave path: a batch whose every datagram
// held a retransmitted fragment took 2556 us against 228 us for a workgroup per datagram, and that
// costs c3_reasm ~3 us; profiles/r06/README_reasm.md.)
#ifndef REASM_FINISH_WAVES
#define REASM_FINISH_WAVES 4
#endif
template <bool V6>
__global__ __launch_bounds__(64 * REASM_FINISH_WAVES) void reasm_finish_kernel(FragArgs p) {
    __shared__ FragLds L;
    __shared__ uint64_t slow_s;
    const uint32_t tid = threadIdx.x, lane = tid & 63u, g0 = blockIdx.x * 64u, g = g0 + lane;
    if (tid < 64u) {
        const bool in = g < p.n_dgram;
        uint32_t state = PLAN_SLOW;
        if (in) {
            // the plan and the S slots in one round trip (the slots are read whatever the plan says):
            // 8 slot loads in flight before the adds
            const ReasmPlan r = p.plan[g];
            const uint32_t* sl = p.slot + (uint64_t)g * p.S;
            uint32_t sum = 0u, k = 0;
            for (; k + 8u <= p.S; k += 8u) {
                uint32_t v[8];
#pragma unroll
                for (uint32_t i = 0; i < 8u; ++i) v[i] = sl[k + i];
#pragma unroll
                for (uint32_t i = 0; i < 8u; ++i) sum += v[i];
            }
            for (; k < p.S; ++k) sum += sl[k];
            state = r.state;
            if (state != PLAN_SLOW) {
                sum -= r.corr;
                uint32_t l4 = 0, v = V_MALFORMED;
                if (state == PLAN_GOOD) v = reasm_verdict<V6>(p.flags, r.len, r.proto, r.pseudo, sum, r.w0, r.w1, l4);
                if (p.o_len) p.o_len[g] = state == PLAN_GOOD ? r.len : 0u;
                if (p.o_l4) p.o_l4[g] = (uint16_t)l4;
                if (p.verdict) p.verdict[g] = (uint8_t)v;
            }
        }
        const uint64_t slow = __builtin_amdgcn_ballot_w64(in && state == PLAN_SLOW);
        if (lane == 0) slow_s = slow;
    }
    __syncthreads();
    uint64_t slow = slow_s;
    while (slow) {
        const uint32_t j = (uint32_t)__builtin_ctzll(slow);
        slow &= slow - 1u;
        reassemble_one<V6, REASM_FINISH_WAVES>(p, g0 + j, L);
        __syncthreads();                              // L is the next one's
    }
}

// ---------------------------------------------------------------- flat grid
//
// Large batches: S one-wave workgroups per datagram (S ~ its fragments / 4), each gathering
// fragments 4 s, ... of its datagram at their own offsets straight from their own headers, so the
// dispatcher balances the gather over the whole batch instead of one wave walking a whole
// datagram; planner workgroups dispatched ahead of them plan the datagrams (a datagram's fragments
// one per lane: dedup, completeness, header copy).  Every wave leaves its partial sum in its slot; the finish
// (reasm_finish_kernel) adds them, less the sums of retransmitted fragments (a repeated offset whose
// later arrival carries the same bytes).  A datagram with a repeated offset of different bytes, or
// more than FLAT_MAXF fragments, is gathered again there by the workgroup path (its flat-grid bytes
// may hold a later arrival's copy); the region past the reassembled datagram is unspecified.

// A retransmitted fragment's payload against the kept arrival's (n bytes each from sa / sb, wave-uniform
// addresses): true when equal; sum = the retransmission's word sum (its payload starts at an even
// transport offset), which its gather wave added to its slot a second time.  16-byte units through
// windows over the batch (byte-unaligned loads), the last partial unit by bytes.
__device__ __forceinline__ bool payload_same(const FragArgs& p, uint64_t sa, uint64_t sb, uint32_t n, uint32_t lane,
                                             uint32_t& sum) {
    const uint64_t b0 = reinterpret_cast<uint64_t>(p.base), bend = b0 + p.base_len;
    const uint64_t wa = sa & ~(uint64_t)15, wb = sb & ~(uint64_t)15;
    const Window A = make_window(wa, (uint32_t)min(bend - wa, (uint64_t)0x7FFFFFF0u));
    const Window B = make_window(wb, (uint32_t)min(bend - wb, (uint64_t)0x7FFFFFF0u));
    const uint32_t full = n >> 4;
    uint32_t acc = 0;
    bool diff = false;
    for (uint32_t u = lane; u < full; u += 64u) {
        const uint4 x = load_win<false>(A, (uint32_t)(sa - wa) + 16u * u);
        const uint4 y = load_win<false>(B, (uint32_t)(sb - wb) + 16u * u);
        diff |= x.x != y.x || x.y != y.y || x.z != y.z || x.w != y.w;
        acc = dot2_add(x.w, dot2_add(x.z, dot2_add(x.y, dot2_add(x.x, acc))));
    }
    const uint32_t i = 16u * full + lane;
    if (lane < (n & 15u)) {
        const uint32_t x = ld_u8(reinterpret_cast<const uint8_t*>(sa) + i), y = ld_u8(reinterpret_cast<const uint8_t*>(sb) + i);
        diff |= x != y;
        acc += x << (8u * (i & 1u));
    }
    sum = (uint32_t)__builtin_amdgcn_readlane((int)group_sum<64>(acc), 63);
    return __builtin_amdgcn_ballot_w64(diff) == 0;
}

// a planner: pico_fragments_check_complete on registers, NS fragments a lane (lane j: fragments j,
// j + 64).  A repeated offset's later arrival is not kept (pico_tree_insert rejects a repeated key);
// the gather waves gathered it too, so it is harmless only when it carries the kept arrival's bytes --
// a retransmission: the plan then subtracts its sum (corr) -- else the plan is SLOW.
template <bool V6, int NS>
__device__ __forceinline__ void plan_sets(const FragArgs& p, uint32_t g, uint32_t first, uint32_t cnt, uint8_t* t,
                                          uint32_t cap, uint32_t lane) {
    constexpr uint32_t HDR = V6 ? 40u : 20u;
    constexpr uint32_t W = 64u * NS;                  // fragments the planner holds
    auto rl = [](uint32_t v, uint32_t l) { return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)l); };
    // fragment k's field from set k / 64 (k wave-uniform)
    auto rk = [&](const uint32_t (&v)[NS], uint32_t k) {
        uint32_t x = rl(v[0], k & 63u);
        if constexpr (NS > 1) x = (k >> 6) ? rl(v[1], k & 63u) : x;
        return x;
    };
    uint32_t state = PLAN_BAD, len = 0, proto = 0, pseudo = 0, w0 = 0, w1 = 0, corr = 0;
    bool in[NS], ok = true;
    uint32_t key[NS], tl[NS], hl[NS], pr[NS], o[NS], offl[NS], offh[NS], srcl[NS], srch[NS];
#pragma unroll
    for (int s = 0; s < NS; ++s) {
        in[s] = lane + 64u * s < cnt;
        uint64_t off;
        ok = parse_lane<V6>(p, in[s], first + lane + 64u * s, off, key[s], tl[s], hl[s], pr[s]) && ok;
        o[s] = key[s] & 0xFFFFu;
        offl[s] = (uint32_t)off;
        offh[s] = (uint32_t)(off >> 32);
        const uint64_t src = reinterpret_cast<uint64_t>(p.base) + off + hl[s];
        srcl[s] = (uint32_t)src;
        srch[s] = (uint32_t)(src >> 32);
    }
    if (__builtin_amdgcn_ballot_w64(!ok) == 0) {
        uint32_t P[NS], rank[NS], orig[NS];           // transport bytes / kept fragments below; earliest same offset
#pragma unroll
        for (int s = 0; s < NS; ++s) { P[s] = rank[s] = 0; orig[s] = lane + 64u * s; }
        for (uint32_t k = 0; k < cnt; ++k) {
            const uint32_t kk = rk(key, k) & 0xFFFFu, tk = rk(tl, k);
#pragma unroll
            for (int s = 0; s < NS; ++s) {
                orig[s] = k < orig[s] && kk == o[s] ? k : orig[s];
                P[s] += kk < o[s] ? tk : 0u;
                rank[s] += kk < o[s] ? 1u : 0u;
            }
        }
        bool kept[NS];
        uint64_t km[NS], dups[NS];
        bool anydup = false;
#pragma unroll
        for (int s = 0; s < NS; ++s) {
            kept[s] = in[s] && orig[s] == lane + 64u * s;
            km[s] = __builtin_amdgcn_ballot_w64(kept[s]);
            dups[s] = __builtin_amdgcn_ballot_w64(in[s] && !kept[s]);
            anydup |= dups[s] != 0;
        }
        if (anydup) {                                 // (rare) P and rank over the kept arrivals only
#pragma unroll
            for (int s = 0; s < NS; ++s) P[s] = rank[s] = 0;
            for (uint32_t k = 0; k < cnt; ++k) {
                const uint32_t kk = rk(key, k) & 0xFFFFu, tk = rk(tl, k);
                const uint64_t kmk = NS > 1 && (k >> 6) ? km[NS - 1] : km[0];
                const bool kk_kept = (kmk >> (k & 63u)) & 1u;
#pragma unroll
                for (int s = 0; s < NS; ++s) {
                    const bool below = kk_kept && kk < o[s];
                    P[s] += below ? tk : 0u;
                    rank[s] += below ? 1u : 0u;
                }
            }
        }
        // retransmissions: the same length and bytes as the kept arrival, else SLOW
        bool slow = false;
#pragma unroll
        for (int s = 0; s < NS; ++s) {
            for (uint64_t dm = dups[s]; dm && !slow; dm &= dm - 1u) {
                const uint32_t k = 64u * s + (uint32_t)__builtin_ctzll(dm), j = rk(orig, k), n = rk(tl, k);
                uint32_t sk = 0;
                slow = n != rk(tl, j) ||
                       !payload_same(p, ((uint64_t)rk(srch, k) << 32) | rk(srcl, k), ((uint64_t)rk(srch, j) << 32) | rk(srcl, j),
                                     n, lane, sk);
                corr += sk;
            }
        }
        uint32_t m = 0;
#pragma unroll
        for (int s = 0; s < NS; ++s) m += (uint32_t)__builtin_popcountll(km[s]);
        if (slow) {
            state = PLAN_SLOW;
        } else {
            // rank = tree position.  Complete: offset == the transport bytes below it up to the
            // first MF-clear fragment in tree order, which is the last
            bool mfc[NS];
            uint32_t top = 0;
#pragma unroll
            for (int s = 0; s < NS; ++s) {
                mfc[s] = kept[s] && !(key[s] & (1u << 16));
                top = max(top, rl(wave_scan_max(mfc[s] ? W - rank[s] : 0u), 63));
            }
            const uint32_t re = W - top;
            bool b = re >= m || re + 1u != m;
#pragma unroll
            for (int s = 0; s < NS; ++s) b = b || __builtin_amdgcn_ballot_w64(kept[s] && rank[s] <= re && o[s] != P[s]) != 0;
            if (!b) {
#pragma unroll
                for (int s = NS - 1; s >= 0; --s) {
                    const uint64_t e = __builtin_amdgcn_ballot_w64(mfc[s] && rank[s] == re);
                    if (e) len = rl(P[s] + tl[s], (uint32_t)__builtin_ctzll(e));
                }
                b = HDR + len > 0xFFFFu || len > cap;
            }
            if (!b) {
                // the first fragment's header (pico_fragments.c:332-338), its transport bytes
                // 0..7 and the pseudo header's address part (as in reassemble_kernel)
                uint32_t f0 = 0;
#pragma unroll
                for (int s = NS - 1; s >= 0; --s) {
                    const uint64_t z = __builtin_amdgcn_ballot_w64(kept[s] && o[s] == 0u);
                    if (z) f0 = 64u * s + (uint32_t)__builtin_ctzll(z);
                }
                const uint8_t* h0 = p.base + (((uint64_t)rk(offh, f0) << 32) | rk(offl, f0));
                const uint32_t hl0 = rk(hl, f0), tl0 = rk(tl, f0);
                const uint32_t hb = lane < HDR ? ld_u8(h0 + lane) : 0u;
                if (lane < HDR) t[(int)lane - (int)HDR] = (uint8_t)hb;
                const uint32_t tb8 = lane < 8u && lane < tl0 ? ld_u8(h0 + hl0 + lane) : 0u;
                w0 = rl(tb8, 0) | (rl(tb8, 1) << 8) | (rl(tb8, 2) << 16) | (rl(tb8, 3) << 24);
                w1 = rl(tb8, 4) | (rl(tb8, 5) << 8) | (rl(tb8, 6) << 16) | (rl(tb8, 7) << 24);
                if constexpr (!V6) {
                    proto = (uint32_t)__shfl((int)hb, 9);
                    const uint32_t pw = lane >= 12u && lane < 20u ? (lane & 1u ? hb << 8 : hb) : 0u;
                    pseudo = rl(group_sum<64>(pw), 63) + (proto << 8) + (((len & 0xFFu) << 8) | ((len >> 8) & 0xFFu));
                } else {
                    // the module: the walk's protocol of the latest kept arrival (it completes the
                    // set, pico_fragments.c:492; reassemble_one's rule)
                    uint32_t last = 0;
#pragma unroll
                    for (int s = 0; s < NS; ++s)
                        if (km[s]) last = 64u * s + 63u - (uint32_t)__builtin_clzll(km[s]);
                    proto = rk(pr, last) | ((uint32_t)__shfl((int)hb, 9) << 8);
                    const uint32_t pw = lane >= 8u && lane < 40u ? (lane & 1u ? hb << 8 : hb) : 0u;
                    pseudo = rl(group_sum<64>(pw), 63) + (((len >> 24) & 0xFFu) | ((len >> 8) & 0xFF00u)) +
                             (((len & 0xFFu) << 8) | ((len >> 8) & 0xFFu));
                }
                state = PLAN_GOOD;
            }
        }
    }
    if (lane == 0) p.plan[g] = ReasmPlan{state, len, proto, pseudo, w0, w1, corr, 0u};
}

template <bool V6>
__device__ __forceinline__ void plan_datagram(const FragArgs& p, uint32_t g, uint32_t first, uint32_t cnt, bool bad0,
                                              uint8_t* t, uint32_t cap, uint32_t lane) {
    if (bad0) {
        if (lane == 0) p.plan[g] = ReasmPlan{PLAN_BAD, 0u, 0u, 0u, 0u, 0u, 0u, 0u};
    } else if (cnt <= 64u) {
        plan_sets<V6, 1>(p, g, first, cnt, t, cap, lane);
    } else if (cnt <= FLAT_MAXF) {
        plan_sets<V6, 2>(p, g, first, cnt, t, cap, lane);
    } else if (lane == 0) {
        p.plan[g] = ReasmPlan{PLAN_SLOW, 0u, 0u, 0u, 0u, 0u, 0u, 0u};
    }
}

// One or two fragments' payloads gathered into the transport at tb (fragment A: transport bytes
// [ata, ata + ta) from address srcA; B likewise when nb_on), in 16-byte units on the output's lines
// as reassemble_kernel phase 3 (its unit arithmetic and store sequence), split into prep / issue /
// process so that two pairs' loads are in flight together.  Both payloads within 1 GiB of each
// other (the window; the caller splits a pair otherwise).
struct PairStep {
    uint64_t wlo;
    uint32_t wsz, va, vb, na, nt, oa, ob, ata, atb, ta, tbb;
    bool nb_on;
};

__device__ __forceinline__ PairStep pair_prep(uint64_t tb, uint64_t srcA, uint32_t ata, uint32_t ta, bool nb_on,
                                              uint64_t srcB, uint32_t atb, uint32_t tbl) {
    PairStep q;
    q.nb_on = nb_on;
    q.oa = (uint32_t)((tb + ata) & 15u);
    q.ob = nb_on ? (uint32_t)((tb + atb) & 15u) : 0u;
    const uint64_t sa = srcA - q.oa, sb = nb_on ? srcB - q.ob : sa;
    q.na = (q.oa + ta + 15u) >> 4;
    q.nt = q.na + (nb_on ? (q.ob + tbl + 15u) >> 4 : 0u);
    q.wlo = (nb_on ? min64s(sa, sb) : sa) & ~15ull;
    const uint64_t whi = nb_on ? max64s(sa + q.oa + ta, sb + q.ob + tbl) : sa + q.oa + ta;
    q.wsz = (uint32_t)(((whi + 15u) & ~15ull) - q.wlo + 16u);
    q.va = (uint32_t)(sa - q.wlo);
    q.vb = (uint32_t)(sb - q.wlo);
    q.ata = ata;
    q.atb = atb;
    q.ta = ta;
    q.tbb = nb_on ? tbl : 0u;
    return q;
}

template <int U>
__device__ __forceinline__ void pair_issue(const PairStep& q, uint32_t lane, uint32_t u0, uint4 (&c0)[U]) {
    const Window win = make_window(q.wlo, q.wsz);
#pragma unroll
    for (int k = 0; k < U; ++k) {
        const uint32_t x = u0 + 64u * k + lane;
        const bool inb = x >= q.na;
        const uint32_t u = inb ? x - q.na : x, v = inb ? q.vb : q.va;
        if (u0 + 64u * k >= q.nt) {                     // (wave-uniform) a row past the pair's units:
            c0[k] = make_uint4(0, 0, 0, 0);             // no load (c3_reasm 98.6-98.7 vs 102.3-103.1 us,
            continue;                                   // c3_reasm6 105.8-106.3 vs 109.2-109.5,
        }                                               // c3_reasm_576 158.8-159.4 vs 165.5-166.3)
        c0[k] = load_win<false>(win, x < q.nt ? v + 16u * u : WIN_OOB);   // (cached: see reasm_flat_kernel)
    }
}

// A unit's fragment bytes: [lo, hi) of its 16 (lo = o in unit 0, a multiple of 4; hi < 16 only in the
// last unit); the rest is the neighbours' and reads as zero.
struct UnitSpan {
    uint32_t lo, hi, so;
};
__device__ __forceinline__ UnitSpan unit_span(const PairStep& q, uint32_t x) {
    const bool ok = x < q.nt;
    const bool inb = x >= q.na;
    const uint32_t u = inb ? x - q.na : x;
    const uint32_t tl = inb ? q.tbb : q.ta, at = inb ? q.atb : q.ata, o = inb ? q.ob : q.oa;
    return UnitSpan{ok && u == 0u ? o : 0u, ok ? min(16u, o + tl - 16u * u) : 0u, at + 16u * u - o};
}

// The units' bytes masked to their fragment's and added to acc (c0 keeps the masked bytes).
template <int U>
__device__ __forceinline__ uint32_t pair_sum(const PairStep& q, uint32_t lane, uint32_t u0, uint4 (&c0)[U], uint32_t acc) {
#pragma unroll
    for (int k = 0; k < U; ++k) {
        const UnitSpan us = unit_span(q, u0 + 64u * k + lane);
        uint32_t xw[4] = {c0[k].x, c0[k].y, c0[k].z, c0[k].w};
#pragma unroll
        for (int w = 0; w < 4; ++w) {
            const uint32_t kb = 4u * w < us.lo ? 0u : min((uint32_t)max((int)us.hi - 4 * w, 0), 4u);
            xw[w] &= (uint32_t)(0xFFFFFFFFull >> (32u - 8u * kb));
        }
        c0[k] = make_uint4(xw[0], xw[1], xw[2], xw[3]);
        acc = dot2_add(xw[3], dot2_add(xw[2], dot2_add(xw[1], dot2_add(xw[0], acc))));
    }
    return acc;
}

// The masked units' stores: the whole units as one aligned 16-byte store (the other lanes void);
// an edge unit's whole dwords [a, a + c) as a b64 and / or a b32, then its last partial dword's
// bytes as a b16 and / or a b8, by the edge lanes alone (exec-masked), and nothing for a row past
// the pair's units.  Against a fixed sequence of 5 stores a row, the edge ones void by offset
// (profiles/r06/ab_reasm_edge_exec.txt): c3_reasm 102.6-103.4 vs 103.4-104.3 us, c3_reasm6
// 109.3 vs 110.3-111.0, c3_reasm_576 on the flat grid 169.8-170.1 vs 217.9-219.2 (the edge stores
// issued only when a lane needs them by a wave ballot: 173.7-173.9; no edge stores at all, a
// timing-only build: c3_reasm 98.0, c3_reasm_576 161.3-161.8, ab_reasm*_edge_stores.txt).
template <int U>
__device__ __forceinline__ void pair_store(const PairStep& q, const Window& ow, uint32_t lane, uint32_t u0,
                                           const uint4 (&c0)[U]) {
#pragma unroll
    for (int k = 0; k < U; ++k) {
        if (u0 + 64u * k >= q.nt) continue;             // (wave-uniform) a row past the pair's units
        const UnitSpan us = unit_span(q, u0 + 64u * k + lane);
        const uint32_t xw[4] = {c0[k].x, c0[k].y, c0[k].z, c0[k].w};
        edge_store(ow, xw, us.lo, us.hi, us.so);
    }
}

template <int U>
__device__ __forceinline__ uint32_t pair_process(const PairStep& q, const Window& ow, uint32_t lane, uint32_t u0,
                                                 uint4 (&c0)[U], uint32_t acc) {
    acc = pair_sum<U>(q, lane, u0, c0, acc);
    pair_store<U>(q, ow, lane, u0, c0);
    return acc;
}

__device__ __forceinline__ uint32_t pair_gather(const PairStep& q, const Window& ow, uint32_t lane, uint32_t acc) {
    for (uint32_t u0 = 0; u0 < q.nt; u0 += 192u) {
        uint4 c0[3];
        pair_issue<3>(q, lane, u0, c0);
        acc = pair_process<3>(q, ow, lane, u0, c0, acc);
    }
    return acc;
}

// The flat grid: planner workgroups, then S one-wave workgroups per datagram; wave s takes
// fragments FPI s, ... in groups
// of FPI = 2 flat_np (its pairs' loads in flight together).  c3_reasm (profiles/r05/ab_reasm_flat.txt):
// 115.4 us against 124.0 us for one workgroup per datagram; one pair a wave 124.7 us (per wave the
// descriptor and header round trips come before its loads), four pairs 127 us (124 VGPRs); 5, 6
// or 8 waves per SIMD forced (96 / 75 / 60 VGPRs, no spills) 116.1 / 116.1 / 117.8 us against
// 115.7 at 4 (105 VGPRs).  The payload loads are cached, not non-temporal: the byte-unaligned
// 16-byte loads of neighbouring units share lines (113.8 -> 108.9 us, IPv6 121.3 -> 118.3).
// Fewer, longer waves measured slower, with the next iteration's descriptor and header loads
// issued under this iteration's payload loads (2 / 3 / 4 iterations a wave: c3_reasm 115.6-115.9 /
// 119.5-119.8 / 118.1-118.4 us against 103.4-104.6, c3_reasm6 120.1-120.5 / 122.1-122.6 /
// 126.4-126.5 against 110.1-111.2; profiles/r06/ab_reasm_iters.txt).  Where the time goes
// (ab_reasm_ablate_finish_plan.txt): without the finish launch 101.6-103.1 / 109.4-109.7 us,
// without planners and finish 99.5-99.9 / 105.2-106.0.
template <bool V6>
__global__ __launch_bounds__(64) void reasm_flat_kernel(FragArgs p) {
    constexpr uint32_t HDR = V6 ? 40u : 20u;
    const uint32_t lane = threadIdx.x;
    const uint32_t S = p.S;
    // Workgroups [0, npl) plan plan_per datagrams each and gather nothing -- dispatched first, so
    // no plan lands in the launch's tail and the planners hold few of the slots (with the plan in
    // each datagram's wave 0 instead: c3_reasm6 152.9 us, c3_reasm 115.3); the rest gather, S per
    // datagram.
    const uint32_t per = plan_per(p.n_dgram), npl = (p.n_dgram + per - 1u) / per;   // planner workgroups
    if (blockIdx.x < npl) {                           // per datagrams in turn
        for (uint32_t g = blockIdx.x * per; g < min(p.n_dgram, (blockIdx.x + 1u) * per); ++g) {
            const uint32_t first = p.grp[2 * g], cnt = p.grp[2 * g + 1];
            const pico_csum_desc_dev od = p.odesc[g];
            const bool bad0 = cnt == 0 || cnt > FRAG_MAX || first > p.n_frag || cnt > p.n_frag - first ||
                              (od.off & 3u) != 0 || od.off > p.out_len || od.len > p.out_len - od.off ||
                              od.len < HDR;
            plan_datagram<V6>(p, g, first, cnt, bad0, p.out + od.off + HDR, od.len - HDR, lane);
        }
        return;
    }
    const uint32_t gb = blockIdx.x - npl;
    const uint32_t g = gb / S, s = gb - g * S;
    if (g >= p.n_dgram) return;
    const uint32_t first = p.grp[2 * g], cnt = p.grp[2 * g + 1];
    const pico_csum_desc_dev od = p.odesc[g];
    const bool bad0 = cnt == 0 || cnt > FRAG_MAX || first > p.n_frag || cnt > p.n_frag - first ||
                      (od.off & 3u) != 0 || od.off > p.out_len || od.len > p.out_len - od.off || od.len < HDR;
    uint8_t* t = p.out + od.off + HDR;
    const uint32_t cap = od.len - HDR;
    uint32_t acc = 0;
    if (!bad0 && cnt <= FLAT_MAXF) {
        const uint64_t tb = reinterpret_cast<uintptr_t>(t);
        const Window ow = make_window(tb, cap);
        auto rl = [](uint32_t v, uint32_t l) { return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)l); };
        constexpr uint32_t NP = flat_np(V6), FPI = 2u * NP;      // pairs / fragments per iteration
        for (uint32_t j0 = FPI * s; j0 < cnt; j0 += FPI * S) {
            // lanes 0..FPI-1 read fragments j0, ..., j0 + FPI - 1; a fragment is gathered when it
            // parses and the output region holds it (repeated offsets too: SLOW plans are gathered
            // again); the NP pairs' loads are in flight at once
            const uint32_t j = j0 + lane;
            uint32_t key, tl, hl, pr;
            uint64_t off;
            const bool in = lane < FPI && j < cnt;
            const bool parsed = parse_lane<V6>(p, in, first + j, off, key, tl, hl, pr);
            const bool ok = in && parsed && (key & 0xFFFFu) + tl <= cap;
            const uint64_t src = reinterpret_cast<uint64_t>(p.base + off) + hl;
            const uint64_t m = __builtin_amdgcn_ballot_w64(ok);
            PairStep ps[NP];
            bool one = true;                  // every pair in one step of 3 x 64 units
#pragma unroll
            for (uint32_t q = 0; q < NP; ++q) {
                const uint32_t la = 2u * q, lb = la + 1u;
                const uint64_t sA = ((uint64_t)rl((uint32_t)(src >> 32), la) << 32) | rl((uint32_t)src, la);
                const uint64_t sB = ((uint64_t)rl((uint32_t)(src >> 32), lb) << 32) | rl((uint32_t)src, lb);
                const uint32_t aA = rl(key, la) & 0xFFFFu, aB = rl(key, lb) & 0xFFFFu, tA = rl(tl, la), tB = rl(tl, lb);
                const bool vA = (m >> la) & 1u, vB = (m >> lb) & 1u;
                if (vA && vB && max64s(sA + tA, sB + tB) - min64s(sA, sB) < (1ull << 30)) {
                    ps[q] = pair_prep(tb, sA, aA, tA, true, sB, aB, tB);
                } else if (vA) {
                    ps[q] = pair_prep(tb, sA, aA, tA, false, 0, 0, 0);
                    if (vB) acc = pair_gather(pair_prep(tb, sB, aB, tB, false, 0, 0, 0), ow, lane, acc);   // (far apart)
                } else if (vB) {
                    ps[q] = pair_prep(tb, sB, aB, tB, false, 0, 0, 0);
                } else {
                    ps[q] = pair_prep(tb, 0, 0, 0, false, 0, 0, 0);
                    ps[q].nt = 0;
                }
                one = one && ps[q].nt <= 192u;
            }
            if (one) {
                uint4 c[NP][3];
#pragma unroll
                for (uint32_t q = 0; q < NP; ++q) pair_issue<3>(ps[q], lane, 0u, c[q]);
#pragma unroll
                for (uint32_t q = 0; q < NP; ++q) acc = pair_process<3>(ps[q], ow, lane, 0u, c[q], acc);
            } else {
#pragma unroll
                for (uint32_t q = 0; q < NP; ++q) acc = pair_gather(ps[q], ow, lane, acc);
            }
        }
    }
    acc = (uint32_t)__builtin_amdgcn_readlane((int)group_sum<64>(acc), 63);
    if (lane == 0) p.slot[(uint64_t)g * S + s] = acc;
}

// Scratch of the flat grid (plans and partial sums, n_dgram x (32 + 4 S) bytes, every byte written
// by each launch before it is read), never allocated per call (per-call hipMallocAsync /
// hipFreeAsync -- alloc / free nodes in a captured graph -- cost c3_reasm ~23 us a call, an event
// record per call ~24 us: idle device time):
//  * eager calls: one buffer per calling thread, device and stream, kept across calls and grown
//    as needed -- calls on one stream are ordered by it, so a buffer is never in use by two calls
//    at once.  Up to SCR_SLOTS streams per thread; the least recently used is freed (hipFree waits
//    for the device) when another comes.  A thread's buffers are freed when it exits (the owner's
//    destructor) or when it calls pico_csum_release_thread_scratch;
//  * calls captured into a graph: one buffer per capture and captured stream (the captured calls
//    on one stream are a chain in the graph), allocated outside the capture's rules and owned by
//    the graph (a user object; freed by the next eager call, or the next release, after the graph
//    is destroyed).  Two executable instances of one graph must not run concurrently.
struct ReasmScratch {
    void* p;
    size_t n;
    hipStream_t stream;
    int dev;
    uint64_t stamp;
};
constexpr int SCR_SLOTS = 8;

std::mutex g_garbage_mu;
std::vector<void*> g_garbage;                    // buffers of destroyed graphs, freed by eager calls

void scratch_release(void* p) {                   // graph destructor: no HIP calls allowed here
    std::lock_guard<std::mutex> lk(g_garbage_mu);
    g_garbage.push_back(p);
}

void free_garbage() {
    std::vector<void*> g;
    {
        std::lock_guard<std::mutex> lk(g_garbage_mu);
        g.swap(g_garbage);
    }
    std::vector<void*> kept;
    for (void* p : g)
        if (hipFree(p) != hipSuccess) kept.push_back(p);   // (e.g. another thread capturing globally)
    if (!kept.empty()) {
        (void)hipGetLastError();
        std::lock_guard<std::mutex> lk(g_garbage_mu);
        g_garbage.insert(g_garbage.end(), kept.begin(), kept.end());
    }
}

// The calling thread's eager buffers; freed at thread exit.
struct ThreadScratch {
    ReasmScratch slot[SCR_SLOTS] = {};
    uint64_t clock = 0;
    void release() {
        int cur = -1;
        (void)hipGetDevice(&cur);
        for (ReasmScratch& c : slot) {
            if (!c.p) continue;
            if (c.dev != cur) (void)hipSetDevice(c.dev);
            if (hipFree(c.p) != hipSuccess) {
                (void)hipGetLastError();
                scratch_release(c.p);                 // retried by the next eager call
            }
            if (c.dev != cur) (void)hipSetDevice(cur);
            c.p = nullptr;
        }
    }
    ~ThreadScratch() { release(); }
};
thread_local ThreadScratch t_scr;

struct CapScratch {
    unsigned long long id;
    hipStream_t stream;
    void* p;
    size_t n;
};
thread_local CapScratch t_cap[SCR_SLOTS];
thread_local int t_cap_next;

int capture_scratch(hipStream_t s, size_t need, void** out) {
    hipStreamCaptureStatus cs;
    unsigned long long id = 0;
    hipGraph_t graph = nullptr;
    const hipGraphNode_t* deps = nullptr;
    size_t ndeps = 0;
    hipError_t e = hipStreamGetCaptureInfo_v2(s, &cs, &id, &graph, &deps, &ndeps);
    if (e != hipSuccess) return (int)e;
    for (int i = 0; i < SCR_SLOTS; ++i)
        if (t_cap[i].p && t_cap[i].id == id && t_cap[i].stream == s && t_cap[i].n >= need) {
            *out = t_cap[i].p;
            return 0;
        }
    hipStreamCaptureMode mode = hipStreamCaptureModeRelaxed;
    if ((e = hipThreadExchangeStreamCaptureMode(&mode)) != hipSuccess) return (int)e;
    void* p = nullptr;
    e = hipMalloc(&p, need);
    hipStreamCaptureMode back = mode;
    (void)hipThreadExchangeStreamCaptureMode(&back);
    if (e != hipSuccess) return (int)e;
    hipUserObject_t obj;
    if ((e = hipUserObjectCreate(&obj, p, scratch_release, 1, hipUserObjectNoDestructorSync)) != hipSuccess) {
        scratch_release(p);
        return (int)e;
    }
    if ((e = hipGraphRetainUserObject(graph, obj, 1, hipGraphUserObjectMove)) != hipSuccess) {
        (void)hipUserObjectRelease(obj, 1);
        return (int)e;
    }
    t_cap[t_cap_next] = CapScratch{id, s, p, need};
    t_cap_next = (t_cap_next + 1) % SCR_SLOTS;
    *out = p;
    return 0;
}

int reasm_scratch(hipStream_t s, size_t need, void** out) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    hipError_t e = hipStreamIsCapturing(s, &cs);
    if (e != hipSuccess) return (int)e;
    if (cs == hipStreamCaptureStatusActive) return capture_scratch(s, need, out);
    if (cs != hipStreamCaptureStatusNone) return (int)hipErrorStreamCaptureInvalidated;
    free_garbage();
    int dev = 0;
    if ((e = hipGetDevice(&dev)) != hipSuccess) return (int)e;
    ReasmScratch* c = nullptr;
    ReasmScratch* sl = t_scr.slot;
    for (int i = 0; i < SCR_SLOTS && !c; ++i)
        if (sl[i].p && sl[i].stream == s && sl[i].dev == dev) c = &sl[i];
    if (!c) {                                        // an empty slot, else the least recently used
        c = &sl[0];
        for (int i = 0; i < SCR_SLOTS; ++i) {
            if (!sl[i].p) {
                c = &sl[i];
                break;
            }
            if (sl[i].stamp < c->stamp) c = &sl[i];
        }
    }
    if (c->p && (c->stream != s || c->dev != dev || c->n < need)) {
        if (c->dev != dev) (void)hipSetDevice(c->dev);
        (void)hipFree(c->p);
        if (c->dev != dev) (void)hipSetDevice(dev);
        c->p = nullptr;
    }
    if (!c->p) {
        const size_t n = need + need / 2u;
        if ((e = hipMalloc(&c->p, n)) != hipSuccess) {
            c->p = nullptr;
            return (int)e;
        }
        c->n = n;
        c->stream = s;
        c->dev = dev;
    }
    c->stamp = ++t_scr.clock;
    *out = c->p;
    return 0;
}

}  // namespace

extern "C" {

// pico_csum_release_thread_scratch (pico_csum.c): the calling thread's flat-grid buffers, and
// the buffers of destroyed graphs
int pico_csum_reasm_release_thread(void) {
    t_scr.release();
    free_garbage();
    return (int)hipSuccess;
}

// v6: 0 IPv4, 1 IPv6; flags: F_NXD (IPv6)
// flat_min: the flat grid from this many datagrams on (0 = REASM_FLAT_MIN, UINT32_MAX = never)
int pico_csum_launch_reassemble(int v6, const void* base, uint64_t base_len, const void* frag, uint32_t n_frag,
                                const uint32_t* groups, uint32_t n_dgram, void* out, uint64_t out_len, const void* out_desc,
                                uint32_t* o_len, uint16_t* o_l4, uint8_t* verdict, uint32_t flags, uint32_t flat_min,
                                void* stream) {
    if (n_dgram == 0) return (int)hipSuccess;
    FragArgs a{static_cast<const uint8_t*>(base), flags, base_len, static_cast<const pico_csum_desc_dev*>(frag),
               groups, n_dgram, n_frag, static_cast<uint8_t*>(out), out_len,
               static_cast<const pico_csum_desc_dev*>(out_desc), o_len, o_l4, verdict, nullptr, nullptr, 0u};
    const hipStream_t s = static_cast<hipStream_t>(stream);
#ifndef REASM_FLAT_MIN
#define REASM_FLAT_MIN 512u
#endif
    // flat grid from REASM_FLAT_MIN datagrams on (64512-byte datagrams, flat vs one workgroup per
    // datagram: 256 19.2 vs 18.7 us, 512 22.6 vs 23.9, 1024 35.4 vs 36.9;
    // profiles/r05/ab_reasm_small_batches.txt)
    const uint32_t fmin = flat_min ? flat_min : REASM_FLAT_MIN;
    // automatic: a batch of more than FLAT_MAXF = 128 fragments a datagram on average takes one
    // workgroup per datagram (the planners hold 128).  c3_reasm_576 -- 117 fragments of 552 B --
    // takes 170 us on the flat grid with the exec-masked edge stores (pair_store), against 210 us
    // here; with the edge stores void by offset the flat grid took 218-221 us and this threshold
    // was 64 (profiles/r06/ab_reasm_128*.txt, ab_reasm576_edge_exec.txt).
    if (n_dgram >= fmin && (flat_min || (uint64_t)n_frag <= (uint64_t)FLAT_MAXF * n_dgram)) {
        // S waves per datagram, FPI fragments each on average
        const uint32_t fpi = 2u * flat_np(v6 != 0);
        const uint64_t its = ((uint64_t)n_frag + fpi - 1u) / fpi;
        uint32_t S = (uint32_t)((its + n_dgram - 1u) / n_dgram);
        S = S < 1u ? 1u : (S > 32u ? 32u : S);
        const size_t plan_b = (size_t)n_dgram * sizeof(ReasmPlan), need = plan_b + (size_t)n_dgram * S * 4u;
        const uint32_t per = plan_per(n_dgram);
        const uint64_t blocks = (uint64_t)n_dgram * S + (n_dgram + per - 1u) / per;   // planners + gather
        void* scratch = nullptr;
        if (blocks <= 0x7FFFFFFFu && reasm_scratch(s, need, &scratch) == 0) {
            a.plan = static_cast<ReasmPlan*>(scratch);
            a.slot = reinterpret_cast<uint32_t*>(static_cast<uint8_t*>(scratch) + plan_b);
            a.S = S;
            const dim3 fg((unsigned)blocks), fb(64);
            const uint32_t lds = (uint64_t)n_frag <= 64ull * n_dgram ? REASM_FLAT_LDS : 0u;
            if (v6) {
                hipLaunchKernelGGL((reasm_flat_kernel<true>), fg, fb, lds, s, a);
                hipLaunchKernelGGL((reasm_finish_kernel<true>), dim3((n_dgram + 63u) / 64u), dim3(64 * REASM_FINISH_WAVES), 0, s, a);
            } else {
                hipLaunchKernelGGL((reasm_flat_kernel<false>), fg, fb, lds, s, a);
                hipLaunchKernelGGL((reasm_finish_kernel<false>), dim3((n_dgram + 63u) / 64u), dim3(64 * REASM_FINISH_WAVES), 0, s, a);
            }
            return (int)hipGetLastError();
        }
        // no scratch (out of memory, or a capture state the stream query refuses) or a grid past
        // 2^31 workgroups: the same
        // results from one workgroup per datagram, which needs none
        (void)hipGetLastError();
    }
    // waves per datagram: 4 each while the batch is small, 1 each once the batch fills the chip's
    // one-wave workgroup slots (16 per CU, LDS-bound): c3_reasm (4096 datagrams) 145.6 vs 149.0 us
    // at 4 waves, 2 waves 165.0 us (2560 slots: a partial second round), ab_frag_wpd.txt
    const int wpd = n_dgram >= 3072u ? 1 : 4;
    const dim3 grid(n_dgram), block(64 * wpd);
    if (wpd == 1) {
        if (v6) hipLaunchKernelGGL((reassemble_kernel<true, 1>), grid, block, 0, s, a);
        else hipLaunchKernelGGL((reassemble_kernel<false, 1>), grid, block, 0, s, a);
    } else {
        if (v6) hipLaunchKernelGGL((reassemble_kernel<true, 4>), grid, block, 0, s, a);
        else hipLaunchKernelGGL((reassemble_kernel<false, 4>), grid, block, 0, s, a);
    }
    return (int)hipGetLastError();
}

}  // extern "C"


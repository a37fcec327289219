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
// Batches of >= 512 datagrams take the flat grid (reasm_flat_kernel, below: the gather spread
// over ~one wave per four fragments, each datagram finished by the last of its waves to arrive; a
// datagram of more than 64 fragments is taken by one of its waves on the one-wave path).
// Otherwise one workgroup (4 waves; 1 wave in batches of >= 3072 datagrams) per datagram (its
// fragments are a contiguous descriptor range, in arrival order):
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
    // flat grid (reasm_flat_kernel): S waves per datagram, one tally per datagram
    // {waves arrived << 32 | their partial sums}, zero between launches
    uint64_t* tally;
    uint32_t S;
};

constexpr uint32_t FLAT_MAXF = 64u;          // fragments a flat-grid wave holds (one per lane)
#ifndef REASM_NP4
#define REASM_NP4 2u
#endif
#ifndef REASM_NP6
#define REASM_NP6 3u
#endif
// fragment pairs a flat-grid wave gathers at once (their loads in flight together): IPv4 2
// (3: 113.2 vs 113.4 us, no gain), IPv6 3 (120.9 us; 2: 128.0, 4: 122.2 at 118 VGPRs)
__host__ __device__ constexpr uint32_t flat_np(bool v6) { return v6 ? REASM_NP6 : REASM_NP4; }
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
                // stores, a fixed sequence of 5 per slot (out-of-range ones void): the whole unit as
                // one aligned 16-byte store; else its whole dwords [a, a + c) as a b64 and / or a b32,
                // then a last partial dword's bytes as a b16 and / or a b8
                const uint32_t ou = at + 16u * u - o;       // the unit's place (16-byte aligned in t)
                const uint32_t so = ou;
                const bool whole = lo == 0u && hi == 16u;
                const uint32_t a = lo >> 2, bq = hi >> 2, c = whole || bq <= a ? 0u : bq - a;
                const uint32_t nr = hi > lo ? hi & 3u : 0u;
                __builtin_amdgcn_raw_buffer_store_b128((u32x4){xw[0], xw[1], xw[2], xw[3]}, ow.rsrc,
                                                       (int)(whole ? so : WIN_OOB), 0, 0);
                const uint32_t a1 = min(a + 1u, 3u), a2 = c >= 2u ? a + 2u : a;
                __builtin_amdgcn_raw_buffer_store_b64(
                    (u32x2){sel4s(a & 3u, xw[0], xw[1], xw[2], xw[3]), sel4s(a1, xw[0], xw[1], xw[2], xw[3])}, ow.rsrc,
                    (int)(c >= 2u ? so + 4u * a : WIN_OOB), 0, 0);
                __builtin_amdgcn_raw_buffer_store_b32(sel4s(a2 & 3u, xw[0], xw[1], xw[2], xw[3]), ow.rsrc,
                                                      (int)(c & 1u ? so + 4u * a2 : WIN_OOB), 0, 0);
                const uint32_t tw = sel4s(bq & 3u, xw[0], xw[1], xw[2], xw[3]);
                __builtin_amdgcn_raw_buffer_store_b16((unsigned short)tw, ow.rsrc,
                                                      (int)(nr >= 2u ? so + 4u * bq : WIN_OOB), 0, 0);
                __builtin_amdgcn_raw_buffer_store_b8((unsigned char)(tw >> (8u * (nr & 2u))), ow.rsrc,
                                                     (int)(nr & 1u ? so + 4u * bq + (nr & 2u) : WIN_OOB), 0, 0);
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

// ---------------------------------------------------------------- flat grid
//
// Large batches: S one-wave workgroups per datagram (S ~ its fragments / 4 for IPv4, / 6 for IPv6),
// no planner and no second launch.  Every wave of a datagram reads all of the datagram's fragment
// headers, one per lane (one round trip; the S waves read the same lines), gathers its own
// fragments at their own offsets -- skipping a repeated offset's later arrivals, as pico_tree_insert
// does -- and adds {1 << 32 | its partial sum} to the datagram's tally with one 64-bit atomic.  The
// wave that brings the tally to S is the last arriver: it holds every header in its lanes, so it
// checks completeness (pico_fragments_check_complete), copies the first fragment's header and
// writes the results from the total the atomic returned, then zeroes the tally for the next launch.
// Nobody waits on another wave.  (The transport is < 64 KiB, so the sum of its 16-bit words never
// reaches bit 32 and cannot carry into the count.)  A datagram of more than FLAT_MAXF fragments
// takes the one-wave LDS path in its wave s = 0 (the other waves return).
//
// Round 5 ran planners dispatched ahead of the gather waves and a finish launch that added the
// partial sums and re-gathered datagrams with repeated offsets one at a time, 64 per finish wave
// (c3_reasm 110.1 / c3_reasm6 118.0 us; the finish launch alone 4.9 us of trace time).

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

// The masked units' stores, a fixed sequence of 5 per slot (out-of-range ones void): the whole unit
// as one aligned 16-byte store; else its whole dwords [a, a + c) as a b64 and / or a b32, then a
// last partial dword's bytes as a b16 and / or a b8.
template <int U>
__device__ __forceinline__ void pair_store(const PairStep& q, const Window& ow, uint32_t lane, uint32_t u0,
                                           const uint4 (&c0)[U]) {
#pragma unroll
    for (int k = 0; k < U; ++k) {
        const UnitSpan us = unit_span(q, u0 + 64u * k + lane);
        const uint32_t xw[4] = {c0[k].x, c0[k].y, c0[k].z, c0[k].w};
        const uint32_t lo = us.lo, hi = us.hi, so = us.so;
        const bool whole = lo == 0u && hi == 16u;
        const uint32_t a = lo >> 2, bq = hi >> 2, c = whole || bq <= a ? 0u : bq - a;
        const uint32_t nr = hi > lo ? hi & 3u : 0u;
        __builtin_amdgcn_raw_buffer_store_b128((u32x4){xw[0], xw[1], xw[2], xw[3]}, ow.rsrc,
                                               (int)(whole ? so : WIN_OOB), 0, 0);
        const uint32_t a1 = min(a + 1u, 3u), a2 = c >= 2u ? a + 2u : a;
        __builtin_amdgcn_raw_buffer_store_b64(
            (u32x2){sel4s(a & 3u, xw[0], xw[1], xw[2], xw[3]), sel4s(a1, xw[0], xw[1], xw[2], xw[3])}, ow.rsrc,
            (int)(c >= 2u ? so + 4u * a : WIN_OOB), 0, 0);
        __builtin_amdgcn_raw_buffer_store_b32(sel4s(a2 & 3u, xw[0], xw[1], xw[2], xw[3]), ow.rsrc,
                                              (int)(c & 1u ? so + 4u * a2 : WIN_OOB), 0, 0);
        const uint32_t tw = sel4s(bq & 3u, xw[0], xw[1], xw[2], xw[3]);
        __builtin_amdgcn_raw_buffer_store_b16((unsigned short)tw, ow.rsrc,
                                              (int)(nr >= 2u ? so + 4u * bq : WIN_OOB), 0, 0);
        __builtin_amdgcn_raw_buffer_store_b8((unsigned char)(tw >> (8u * (nr & 2u))), ow.rsrc,
                                             (int)(nr & 1u ? so + 4u * bq + (nr & 2u) : WIN_OOB), 0, 0);
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

// The flat grid's waves (gather, tally, and for the last arriver the finish).  Payload loads are
// cached, not non-temporal: the byte-unaligned 16-byte loads of neighbouring units share lines
// (round 5: 113.8 -> 108.9 us, IPv6 121.3 -> 118.3).  Pairs in flight per wave: IPv4 2, IPv6 3
// (round 5: IPv6 two 128.0, three 120.9, four 122.2 us).
template <bool V6>
__global__ __launch_bounds__(64) void reasm_flat_kernel(FragArgs p) {
    constexpr uint32_t HDR = V6 ? 40u : 20u;
    __shared__ FragLds L;                             // the > FLAT_MAXF path only
    const uint32_t lane = threadIdx.x;
    const uint32_t S = p.S;
#ifdef REASM_XCD
    // blocks b = 8 (q S + s) + x serve datagram g = 8 q + x: blocks b and b + 8 share an XCD (the
    // dispatcher deals blocks round-robin over the 8 XCDs; speed only), so a datagram's S waves share
    // one L2 for the headers every one of them reads
    const uint32_t xb = blockIdx.x & 7u, rb = blockIdx.x >> 3;
    const uint32_t qg = rb / S, s = rb - qg * S, g = 8u * qg + xb;
#else
    const uint32_t g = blockIdx.x / S, s = blockIdx.x - g * S;
#endif
    if (g >= p.n_dgram) return;
    const uint32_t first = p.grp[2 * g], cnt = p.grp[2 * g + 1];
    const pico_csum_desc_dev od = p.odesc[g];
    const bool bad0 = cnt == 0 || cnt > FRAG_MAX || first > p.n_frag || cnt > p.n_frag - first ||
                      (od.off & 3u) != 0 || od.off > p.out_len || od.len > p.out_len - od.off || od.len < HDR;
    auto put = [&](uint32_t len, uint32_t l4, uint32_t v) {
        if (p.o_len) p.o_len[g] = len;
        if (p.o_l4) p.o_l4[g] = (uint16_t)l4;
        if (p.verdict) p.verdict[g] = (uint8_t)v;
    };
    if (bad0) {
        if (s == 0 && lane == 0) put(0u, 0u, V_MALFORMED);
        return;
    }
    if (cnt > FLAT_MAXF) {
#ifndef REASM_ABL_NOLDS
        if (s == 0) reassemble_one<V6, 1>(p, g, L);
#endif
        return;
    }
    uint8_t* t = p.out + od.off + HDR;
    const uint32_t cap = od.len - HDR;
    auto rl = [](uint32_t v, uint32_t l) { return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)l); };

    // ---- every fragment's header, lane j = fragment j: its first 16 bytes (IPv6 also 40..55) in
    //      one load each through a window over the batch from 1 GiB below the first fragment
    //      (a header outside it: frag_parse's byte loads)
    const bool in = lane < cnt;
    uint32_t key = 0, tl = 0, hl = 0, pr = 0;
    uint64_t off = 0;
    bool ok = true;
    {
        pico_csum_desc_dev d{0, 0, 0};
        if (in) d = p.frag[first + lane];
        off = d.off;
        const uint64_t a0 = rl((uint32_t)off, 0) | ((uint64_t)rl((uint32_t)(off >> 32), 0) << 32);
        const uint64_t lo = a0 > (1ull << 30) ? (a0 - (1ull << 30)) & ~(uint64_t)15 : 0ull;
        const uint64_t wsz = p.base_len > lo ? min(p.base_len - lo, (uint64_t)0x7FFFFFF0u) : 0ull;
        const Window hw = make_window(reinterpret_cast<uint64_t>(p.base) + lo, (uint32_t)wsz);
        const bool pre = in && off >= lo && off - lo + (V6 ? 56u : 16u) <= wsz;
        const uint32_t v = pre ? (uint32_t)(off - lo) : WIN_OOB;
        const uint4 v0 = load_win<false>(hw, v);
        const uint4 v40 = V6 ? load_win<false>(hw, pre ? v + 40u : WIN_OOB) : make_uint4(0, 0, 0, 0);
        if (in) ok = frag_parse_pre<V6>(p, d, pre, v0, v40, key, tl, hl, pr);
    }
    if (__builtin_amdgcn_ballot_w64(!ok)) {           // a malformed fragment: not reassembled
        if (s == 0 && lane == 0) put(0u, 0u, V_MALFORMED);
        return;
    }
    const uint32_t o = key & 0xFFFFu;
    const uint64_t src = reinterpret_cast<uint64_t>(p.base) + off + hl;
    // the first fragment (offset 0; the earliest arrival if repeated): its header bytes and the
    // transport's bytes 0..7, loaded now for the last arriver (lanes [0, HDR) the header, lanes
    // [HDR, HDR + 8) the transport bytes), in flight beside the gather
    const uint64_t z = __builtin_amdgcn_ballot_w64(in && o == 0u);
    const uint32_t f0 = z ? (uint32_t)__builtin_ctzll(z) : 0u;
    uint32_t hbt = 0;
    if (z) {
        const uint8_t* h0 = p.base + (((uint64_t)rl((uint32_t)(off >> 32), f0) << 32) | rl((uint32_t)off, f0));
        const uint32_t hl0 = rl(hl, f0), tl0 = rl(tl, f0);
        if (lane < HDR) hbt = ld_u8(h0 + lane);
        else if (lane < HDR + 8u && lane - HDR < tl0) hbt = ld_u8(h0 + hl0 + (lane - HDR));
    }

    // ---- this wave's fragments FPI s, ... (FPI = 2 NP), NP pairs' loads in flight together; the
    //      tally's atomic goes out before the last step's stores, so the wave waits for its
    //      return, not for its stores (vmcnt counts both, in issue order)
    uint32_t acc = 0;
    uint64_t before = 0;
    auto tally = [&]() {
        const uint32_t tot = rl(group_sum<64>(acc), 63);
        acc = tot;
        if (lane == 0)
            before = __hip_atomic_fetch_add(p.tally + g, (1ull << 32) | tot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("" ::: "memory");
    };
    {
        const uint64_t tb = reinterpret_cast<uintptr_t>(t);
        const Window ow = make_window(tb, cap);
        constexpr uint32_t NP = flat_np(V6), FPI = 2u * NP;
        uint32_t j0 = FPI * s;
        if (j0 >= cnt) tally();
        for (; j0 < cnt; j0 += FPI * S) {
            const bool lastit = j0 + FPI * S >= cnt;
            // gathered: parsed (all are), the first arrival of its offset, held by the output region
            uint64_t m = 0;
#pragma unroll
            for (uint32_t q = 0; q < FPI; ++q) {
                const uint32_t j = j0 + q;
                if (j < cnt) {
                    const uint32_t oj = rl(o, j);
                    const bool dup = __builtin_amdgcn_ballot_w64(lane < j && o == oj) != 0;
                    if (!dup && oj + rl(tl, j) <= cap) m |= 1ull << q;
                }
            }
            PairStep ps[NP];
            bool one = true;                  // every pair in one step of 3 x 64 units
#pragma unroll
            for (uint32_t q = 0; q < NP; ++q) {
                const uint32_t la = min(j0 + 2u * q, 63u), lb = min(j0 + 2u * q + 1u, 63u);
                const uint64_t sA = ((uint64_t)rl((uint32_t)(src >> 32), la) << 32) | rl((uint32_t)src, la);
                const uint64_t sB = ((uint64_t)rl((uint32_t)(src >> 32), lb) << 32) | rl((uint32_t)src, lb);
                const uint32_t aA = rl(o, la), aB = rl(o, lb), tA = rl(tl, la), tB = rl(tl, lb);
                const bool vA = (m >> (2u * q)) & 1u, vB = (m >> (2u * q + 1u)) & 1u;
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
                for (uint32_t q = 0; q < NP; ++q) acc = pair_sum<3>(ps[q], lane, 0u, c[q], acc);
                if (lastit) tally();
#pragma unroll
                for (uint32_t q = 0; q < NP; ++q) pair_store<3>(ps[q], ow, lane, 0u, c[q]);
            } else {
#pragma unroll
                for (uint32_t q = 0; q < NP; ++q) acc = pair_gather(ps[q], ow, lane, acc);
                if (lastit) tally();
            }
        }
    }

    // ---- the tally: the wave that brings it to S finishes the datagram
#ifdef REASM_ABL_NOATOM
    if (lane == 0 && s == 0) p.o_len[g] = (uint32_t)(__builtin_amdgcn_readfirstlane(hbt));
    return;
#endif
    before = ((uint64_t)rl((uint32_t)(before >> 32), 0) << 32) | rl((uint32_t)before, 0);
    if ((uint32_t)(before >> 32) != S - 1u) return;
    const uint32_t sum = (uint32_t)before + acc;      // (acc: this wave's total, from tally())

    // ---- the last arriver: pico_fragments_check_complete over the kept fragments (earliest arrival
    //      of each offset), in tree order by rank; complete when every offset up to the first
    //      MF-clear fragment equals the transport bytes below it and that fragment is the last
    bool dup = false;
    uint32_t P = 0, rank = 0;
    for (uint32_t k = 0; k < cnt; ++k) dup |= k < lane && rl(o, k) == o;
    const bool kept = in && !dup;
    const uint64_t km = __builtin_amdgcn_ballot_w64(kept);
    for (uint32_t k = 0; k < cnt; ++k) {
        const uint32_t ok_ = rl(o, k), tk = rl(tl, k);
        const bool below = ((km >> k) & 1u) && ok_ < o;
        P += below ? tk : 0u;
        rank += below ? 1u : 0u;
    }
    const uint32_t mkept = (uint32_t)__builtin_popcountll(km);
    const bool mfc = kept && !(key & (1u << 16));
    const uint32_t re = 64u - rl(wave_scan_max(mfc ? 64u - rank : 0u), 63);
    bool b = !z || re >= mkept || re + 1u != mkept || __builtin_amdgcn_ballot_w64(kept && rank <= re && o != P) != 0;
    uint32_t len = 0;
    if (!b) {
        const uint32_t le = (uint32_t)__builtin_ctzll(__builtin_amdgcn_ballot_w64(mfc && rank == re));
        len = rl(P + tl, le);
        b = HDR + len > 0xFFFFu || len > cap;
    }
    if (b) {
        if (lane == 0) put(0u, 0u, V_MALFORMED);
    } else {
        // the first fragment's PICO_SIZE_IP4HDR / PICO_SIZE_IP6HDR bytes (pico_fragments.c:332-338),
        // the transport's bytes 0..7 and the pseudo header's address part (as reassemble_one)
        if (lane < HDR) t[(int)lane - (int)HDR] = (uint8_t)hbt;
        const uint32_t w0 = rl(hbt, HDR) | (rl(hbt, HDR + 1u) << 8) | (rl(hbt, HDR + 2u) << 16) | (rl(hbt, HDR + 3u) << 24);
        const uint32_t w1 = rl(hbt, HDR + 4u) | (rl(hbt, HDR + 5u) << 8) | (rl(hbt, HDR + 6u) << 16) | (rl(hbt, HDR + 7u) << 24);
        const uint32_t hb = lane < HDR ? hbt : 0u;
        uint32_t proto, pseudo;
        if constexpr (!V6) {
            proto = rl(hb, 9);
            const uint32_t pw = lane >= 12u && lane < 20u ? (lane & 1u ? hb << 8 : hb) : 0u;
            pseudo = rl(group_sum<64>(pw), 63) + (proto << 8) + (((len & 0xFFu) << 8) | ((len >> 8) & 0xFFu));
        } else {
            // the module: the walk's protocol of the latest kept arrival (it completes the set,
            // pico_fragments.c:492); byte 9 of the copied header rides in bits 8-15
            proto = rl(pr, 63u - (uint32_t)__builtin_clzll(km)) | (rl(hb, 9) << 8);
            const uint32_t pw = lane >= 8u && lane < 40u ? (lane & 1u ? hb << 8 : hb) : 0u;
            pseudo = rl(group_sum<64>(pw), 63) + (((len >> 24) & 0xFFu) | ((len >> 8) & 0xFF00u)) +
                     (((len & 0xFFu) << 8) | ((len >> 8) & 0xFFu));
        }
        uint32_t l4 = 0;
        const uint32_t v = reasm_verdict<V6>(p.flags, len, proto, pseudo, sum, w0, w1, l4);
        if (lane == 0) put(len, l4, v);
    }
    if (lane == 0) p.tally[g] = 0ull;                 // every wave of this launch has arrived
}

// Scratch of the flat grid (one 8-byte tally per datagram, zero between launches: the last
// arriver of each datagram zeroes its own), never allocated per call (per-call hipMallocAsync /
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
// A new buffer is zeroed on a private non-blocking stream (no implicit join with a capturing one).
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

int zero_fill(void* p, size_t n) {
    static std::mutex mu;
    static hipStream_t zs[64] = {};
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return (int)e;
    if (dev < 0 || dev >= 64) return (int)hipErrorInvalidDevice;
    hipStream_t st;
    {
        std::lock_guard<std::mutex> lk(mu);
        if (!zs[dev] && (e = hipStreamCreateWithFlags(&zs[dev], hipStreamNonBlocking)) != hipSuccess) return (int)e;
        st = zs[dev];
    }
    if ((e = hipMemsetAsync(p, 0, n, st)) != hipSuccess) return (int)e;
    return (int)hipStreamSynchronize(st);
}

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
    int z = e == hipSuccess ? zero_fill(p, need) : 0;
    hipStreamCaptureMode back = mode;
    (void)hipThreadExchangeStreamCaptureMode(&back);
    if (e != hipSuccess) return (int)e;
    if (z) {
        scratch_release(p);
        return z;
    }
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
        int z = zero_fill(c->p, n);
        if (z) {
            (void)hipFree(c->p);
            c->p = nullptr;
            return z;
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
               static_cast<const pico_csum_desc_dev*>(out_desc), o_len, o_l4, verdict, nullptr, 0u};
    const hipStream_t s = static_cast<hipStream_t>(stream);
#ifndef REASM_FLAT_MIN
#define REASM_FLAT_MIN 512u
#endif
    // flat grid from REASM_FLAT_MIN datagrams on (round 5, 64512-byte datagrams, flat vs one
    // workgroup per datagram: 256 19.2 vs 18.7 us, 512 22.6 vs 23.9, 1024 35.4 vs 36.9;
    // profiles/r05/ab_reasm_small_batches.txt)
    const uint32_t fmin = flat_min ? flat_min : REASM_FLAT_MIN;
    // automatic: a batch of more than FLAT_MAXF fragments a datagram on average (64 KiB datagrams
    // over a small MTU) takes one workgroup per datagram -- the flat grid would give most of its
    // datagrams to the one-wave path in one of their waves, the others idle
    if (n_dgram >= fmin && (flat_min || (uint64_t)n_frag <= (uint64_t)FLAT_MAXF * n_dgram)) {
        // S waves per datagram, FPI fragments each on average
        const uint32_t fpi = 2u * flat_np(v6 != 0);
        const uint64_t its = ((uint64_t)n_frag + fpi - 1u) / fpi;
        uint32_t S = (uint32_t)((its + n_dgram - 1u) / n_dgram);
        S = S < 1u ? 1u : (S > 32u ? 32u : S);
        const size_t need = (size_t)n_dgram * sizeof(uint64_t);
#ifdef REASM_XCD
        const uint64_t blocks = (uint64_t)((n_dgram + 7u) / 8u) * 8u * S;
#else
        const uint64_t blocks = (uint64_t)n_dgram * S;
#endif
        void* scratch = nullptr;
        if (blocks <= 0x7FFFFFFFu && reasm_scratch(s, need, &scratch) == 0) {
            a.tally = static_cast<uint64_t*>(scratch);
            a.S = S;
            if (v6) hipLaunchKernelGGL((reasm_flat_kernel<true>), dim3((unsigned)blocks), dim3(64), 0, s, a);
            else hipLaunchKernelGGL((reasm_flat_kernel<false>), dim3((unsigned)blocks), dim3(64), 0, s, a);
            return (int)hipGetLastError();
        }
        // no scratch (out of memory, or a capture state the stream query refuses) or a grid past
        // 2^31 workgroups: the same results from one workgroup per datagram, which needs none
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

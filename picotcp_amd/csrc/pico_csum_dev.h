// pico_csum_dev.h -- device helpers shared by the gfx950 kernel TUs of libpicocsum
// (pico_csum_k_raw.hip, pico_csum_k_sorted.hip, pico_csum_k_frag.hip).  Header-only,
// internal; everything lives in an anonymous namespace (one copy per TU).
//
// The kernels of picoTCP's Internet checksum.
//
// What is computed (bit-exact with stack/pico_frame.c:279-328):
//   S = sum_{i<n/2} (b[2i] | b[2i+1]<<8) + (n odd ? b[n-1] : 0)    word pairing relative to the frame start
//   s = (seed + S) mod 2^32;  ret = bswap16(~fold16(s))
//
// How (DESIGN.md "Kernels"):
//   * S = E + 256*O, E/O = sums of the bytes at even/odd offsets from the frame
//     start.  A 16-byte-aligned chunk is loaded with one global_load_dwordx4
//     whatever the frame's alignment; bytes outside the frame (or inside a
//     crc field) are masked to zero; for an odd frame start v_perm_b32 swaps
//     the bytes of each 16-bit half so the pairing is frame-relative again;
//     v_dot2_u32_u16 (x . {1,1}) then adds both halves into a 32-bit
//     per-lane accumulator -- exact, two VALU ops per dword.  All later
//     additions are plain 32-bit wrapping adds, which is exactly the
//     reference's uint32_t accumulator, so the 131076-byte wrap matches too.
//   * A frame is owned by a lane group of G lanes (G = 4..64): lane l reads
//     chunks l, l+G, ... (G*16 contiguous bytes per group per load), CPL
//     chunks per lane per pass are issued back to back.  The group's partial
//     sums are folded with DPP row ops (quad_perm, row_half_mirror,
//     row_mirror) and, above 16 lanes, ds_swizzle/bpermute shuffles.
//   * A wave owns FPW consecutive frames: descriptors are read with one
//     coalesced load per wave, results are collected one per lane and written
//     with one coalesced store per wave.
//   * No MFMA: this is an HBM-bound byte reduction.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <type_traits>

namespace {

typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));

constexpr uint32_t SEL_EVEN = 0x03020100u;  // v_perm: identity
constexpr uint32_t SEL_ODD  = 0x02030001u;  // v_perm: swap bytes inside each 16-bit half

__device__ __forceinline__ uint32_t dot2_add(uint32_t x, uint32_t acc) {
    return __builtin_amdgcn_udot2(__builtin_bit_cast(u16x2, x), (u16x2){1, 1}, acc, false);
}

// 4 mask bits -> 4 byte masks (0x00 / 0xFF); the shifted copies never overlap.
__device__ __forceinline__ uint32_t nib_to_bytes(uint32_t nib) {
    return ((nib * 0x00204081u) & 0x01010101u) * 0xFFu;
}

// Adds the bytes of chunk v selected by the 16-bit mask m16 (bit i = byte i).
__device__ __forceinline__ uint32_t add_chunk(const uint4 v, uint32_t m16, uint32_t sel, uint32_t acc) {
    acc = dot2_add(__builtin_amdgcn_perm(0u, v.x & nib_to_bytes(m16 & 15u), sel), acc);
    acc = dot2_add(__builtin_amdgcn_perm(0u, v.y & nib_to_bytes((m16 >> 4) & 15u), sel), acc);
    acc = dot2_add(__builtin_amdgcn_perm(0u, v.z & nib_to_bytes((m16 >> 8) & 15u), sel), acc);
    acc = dot2_add(__builtin_amdgcn_perm(0u, v.w & nib_to_bytes((m16 >> 12) & 15u), sel), acc);
    return acc;
}

// Adds all 16 bytes of chunk v (frame-relative pairing via sel when PERM).
template <bool PERM>
__device__ __forceinline__ uint32_t add_full(const uint4 v, uint32_t sel, uint32_t acc) {
    if constexpr (PERM) {
        acc = dot2_add(__builtin_amdgcn_perm(0u, v.x, sel), acc);
        acc = dot2_add(__builtin_amdgcn_perm(0u, v.y, sel), acc);
        acc = dot2_add(__builtin_amdgcn_perm(0u, v.z, sel), acc);
        acc = dot2_add(__builtin_amdgcn_perm(0u, v.w, sel), acc);
    } else {
        acc = dot2_add(v.x, acc);
        acc = dot2_add(v.y, acc);
        acc = dot2_add(v.z, acc);
        acc = dot2_add(v.w, acc);
    }
    return acc;
}

// Bits [lo, hi) of a 16-bit chunk mask; lo, hi in [0, 16].
__device__ __forceinline__ uint32_t bits16(uint32_t lo, uint32_t hi) {
    return ((1u << hi) - 1u) & ~((1u << lo) - 1u);
}

// Mask of the bytes of chunk k (chunk 0 starts at a0 = start & ~15, r = start - a0)
// that lie in [r + x0, r + x1), x0 <= x1 relative to the frame start.
__device__ __forceinline__ uint32_t chunk_range_mask(uint32_t k, uint64_t x0r, uint64_t x1r) {
    const uint64_t c = (uint64_t)k << 4;
    const uint32_t lo = x0r <= c ? 0u : (x0r - c >= 16 ? 16u : (uint32_t)(x0r - c));
    const uint32_t hi = x1r <= c ? 0u : (x1r - c >= 16 ? 16u : (uint32_t)(x1r - c));
    return hi > lo ? bits16(lo, hi) : 0u;
}

// Clears the two bits of a 2-byte field at chunk-relative position d (may be
// outside [-1, 15], then nothing is cleared).
__device__ __forceinline__ uint32_t clear_field(uint32_t m, int64_t d) {
    const uint32_t sh = (d >= -1 && d <= 15) ? (uint32_t)(d + 1) : 20u;
    return m & ~((3u << sh) >> 1);
}

// Sum over a lane group of G lanes (G | 64, groups aligned).  The total lands in
// the group's LAST lane (lane g*G + G-1); for G <= 16 every lane of the group has it.
// DPP only: quad_perm xor1/xor2, row_half_mirror, row_mirror, then row_bcast:15
// (rows 1,3 += lane 15 of the row below) and row_bcast:31 (rows 2,3 += lane 31).
template <int G>
__device__ __forceinline__ uint32_t group_sum(uint32_t v) {
    if constexpr (G >= 2)  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false);
    if constexpr (G >= 4)  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xF, 0xF, false);
    if constexpr (G >= 8)  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x141, 0xF, 0xF, false);
    if constexpr (G >= 16) v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x140, 0xF, 0xF, false);
    if constexpr (G >= 32) v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xA, 0xF, false);
    if constexpr (G >= 64) v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xC, 0xF, false);
    return v;
}

// stack/pico_frame.c:301-307: fold with end-around carry, complement, short_be.
__device__ __forceinline__ uint32_t finalize(uint32_t s) {
    s = (s & 0xFFFFu) + (s >> 16);
    s = (s & 0xFFFFu) + (s >> 16);
    const uint32_t c = (~s) & 0xFFFFu;
    return ((c >> 8) | (c << 8)) & 0xFFFFu;
}

// The 16-bit checksum word as it sits in memory: hdr->crc = short_be(ret).  One 16-bit
// store when the field is 2-byte aligned (every IPv4 / TCP / UDP crc behind a 2-aligned
// header), two byte stores otherwise.
__device__ __forceinline__ void store_crc(uint8_t* p, uint32_t ret) {
    if ((reinterpret_cast<uintptr_t>(p) & 1u) == 0) {
        *reinterpret_cast<uint16_t*>(p) = (uint16_t)(((ret >> 8) & 0xFFu) | ((ret & 0xFFu) << 8));
    } else {
        p[0] = (uint8_t)(ret >> 8);
        p[1] = (uint8_t)(ret & 0xFFu);
    }
}

// The low n bytes of v, little-endian, at p (any alignment): 16-bit stores when p is even.
__device__ __forceinline__ void store_le(uint8_t* p, uint32_t v, int n) {
    if ((reinterpret_cast<uintptr_t>(p) & 1u) == 0) {
        for (int i = 0; i < n; i += 2) *reinterpret_cast<uint16_t*>(p + i) = (uint16_t)(v >> (8 * i));
    } else {
        for (int i = 0; i < n; ++i) p[i] = (uint8_t)(v >> (8 * i));
    }
}

__device__ __forceinline__ uint4 load_chunk(const uint8_t* a0, uint32_t k) {
    return *reinterpret_cast<const uint4*>(a0 + ((uint64_t)k << 4));
}

// Hands the group results of one iteration to lanes base..base+NG-1: lane base+g
// receives the value group g holds in its last lane.  Lane j of the wave thus ends
// up with the result of the wave's frame j (one coalesced store per wave later).
template <int G>
__device__ __forceinline__ uint32_t collect(uint32_t res, uint32_t val, uint32_t lane, uint32_t base) {
    constexpr uint32_t NG = 64 / G;
    if constexpr (NG <= 4) {
#pragma unroll
        for (uint32_t g = 0; g < NG; ++g) {
            const uint32_t s = (uint32_t)__builtin_amdgcn_readlane((int)val, (int)(g * G + G - 1));
            res = (lane == base + g) ? s : res;
        }
        return res;
    } else {
        const uint32_t src = ((lane - base) & (NG - 1)) * G + (G - 1);
        const uint32_t got = (uint32_t)__shfl((int)val, (int)src);
        return (lane >= base && lane < base + NG) ? got : res;
    }
}

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

// (generic pointer: flat loads.  As global-address-space loads -- vmcnt only -- c2slot, c2eth,
// c3_frag measured the same: profiles/r06/ab_global_chunks.txt)
template <bool NT>
__device__ __forceinline__ uint4 load_chunk_t(const uint8_t* a0, uint32_t k) {
    const u32x4* q = reinterpret_cast<const u32x4*>(a0 + ((uint64_t)k << 4));
    u32x4 x;
    if constexpr (NT) x = __builtin_nontemporal_load(q);
    else x = *q;
    return make_uint4(x.x, x.y, x.z, x.w);
}

// ---- windowed buffer loads
//
// A wave's frames lie in a window of < 2 GiB.  A buffer resource over that window
// (built from wave-uniform values: SGPRs, no waterfall) lets every lane issue every
// load slot unconditionally: a slot past its frame gets voffset WIN_OOB, which the
// range check turns into zeros without a memory access.  With no branch around the
// loads the compiler can count them, so a wave consumes set i behind
// s_waitcnt vmcnt(#set i+1) with set i+1 still in flight -- a `k < nch ? load : 0`
// becomes an s_cbranch_execz around each load, after which hipcc only dares vmcnt(0).
constexpr uint32_t WIN_OOB = 0x80000000u;    // >= every window's num_records

struct Window {
    __amdgpu_buffer_rsrc_t rsrc;
    uint64_t base;                          // window start (16-byte aligned address)
};

// Window [lo, lo + bytes) over device addresses; lo and bytes must be wave-uniform
// values (they are read from the first lane), bytes < 2^31.
__device__ __forceinline__ Window make_window(uint64_t lo, uint32_t bytes) {
    const uint32_t l = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)lo);
    const uint32_t h = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(lo >> 32));
    const uint32_t nb = (uint32_t)__builtin_amdgcn_readfirstlane((int)bytes);
    Window w;
    w.base = ((uint64_t)h << 32) | l;
    w.rsrc = __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(w.base), 0, (int)nb, 0x00020000);
    return w;
}

template <bool NT>
__device__ __forceinline__ uint4 load_win(const Window& w, uint32_t voff) {
    const u32x4 x = __builtin_amdgcn_raw_buffer_load_b128(w.rsrc, (int)voff, 0, NT ? 2 : 0);   // aux 2 = nt
    return make_uint4(x.x, x.y, x.z, x.w);
}

}  // namespace

// Device view of struct pico_csum_desc (include/pico_csum.h), 16 bytes.
struct pico_csum_desc_dev {
    uint64_t off;
    uint32_t len;
    uint32_t seed;
};

namespace {

struct RawArgs {
    uint8_t* base;
    uint64_t base_len;
    const pico_csum_desc_dev* desc;
    uint64_t stride;
    uint32_t len;
    uint32_t n;
    uint32_t seed;
    int32_t crc_off;
    uint32_t flags;
    uint32_t fpw;
    uint16_t* out;
    uint32_t* bad;
};


constexpr uint32_t V_ACCEPT = 1u, V_NET_BAD = 2u, V_L4_BAD = 4u, V_MALFORMED = 8u, V_EXPIRED = 16u;
constexpr uint32_t V_FRAG = 16u;        // RX / TX batches (V_EXPIRED: the forwarding batch only)
constexpr uint32_t V_DROP_L2 = 32u, V_ARP = 64u, V_IPV6 = 128u;   // Ethernet mode (include/pico_csum.h)
constexpr uint32_t F_MACF = 0x10000u;   // kernel flag (set by the host layer): filter destination MACs
constexpr uint32_t F_NAT = 0x20000u;    // kernel flag (pico_ipv4_nat_batch_dev): IPv4 mode, NAT rewrite
constexpr uint32_t V_UNTOUCHED = 32u;   // NAT batch: left as it is (include/pico_csum.h)
// NAT state of a frame (IPv4 mode, F_NAT), in the l2v byte of the phase-4 state
constexpr uint32_t NS_XLATE = 1u, NS_HDR = 2u, NS_SKIP = 4u, NS_BAD = 8u;
constexpr uint32_t F_NXD = 0x8u;        // PICO_CSUM_F_NXTHDR_DISPATCH (IPv6 RX)
// phase-1 outcomes applied after the IPv4 header check (sorted kernel)
constexpr uint32_t PV_DROP = 1u, PV_FRAG = 2u;

__device__ __forceinline__ uint32_t sel4(uint32_t q, uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
    return q == 0 ? a : (q == 1 ? b : (q == 2 ? c : d));
}


// Inclusive prefix sum over the 64 lanes (DPP row_shr 1/2/4/8, row_bcast 15/31).
__device__ __forceinline__ uint32_t wave_scan_add(uint32_t v) {
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, false);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xF, 0xF, false);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xF, 0xF, false);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xF, 0xF, false);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xA, 0xF, false);
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xC, 0xF, false);
    return v;
}

// Inclusive prefix maximum over the 64 lanes (the same DPP steps; 0 is the identity).
__device__ __forceinline__ uint32_t wave_scan_max(uint32_t v) {
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, false));
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xF, 0xF, false));
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xF, 0xF, false));
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xF, 0xF, false));
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xA, 0xF, false));
    v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xC, 0xF, false));
    return v;
}

// Sum of the bytes of chunk v (chunk start at relative position ch) that lie in
// [x0, x1) (relative to the same origin), frame-relative pairing via sel.
// Branch-free: the 16-byte validity mask is built as two 64-bit masks.
template <bool PERM>
__device__ __forceinline__ uint32_t masked_chunk_sum(const uint4 v, uint32_t ch, uint32_t x0, uint32_t x1,
                                                     uint32_t sel) {
    const uint32_t lo = x0 <= ch ? 0u : min(x0 - ch, 16u);
    const uint32_t hi = x1 <= ch ? 0u : min(x1 - ch, 16u);
    const uint64_t ALL = ~0ull;
    uint64_t m0 = lo >= 8u ? 0ull : (ALL << (8u * lo));
    m0 &= hi >= 8u ? ALL : ~(ALL << (8u * hi));
    uint64_t m1 = lo >= 16u ? 0ull : (lo <= 8u ? ALL : (ALL << (8u * (lo - 8u))));
    m1 &= hi >= 16u ? ALL : (hi <= 8u ? 0ull : ~(ALL << (8u * (hi - 8u))));
    uint32_t a = v.x & (uint32_t)m0, b = v.y & (uint32_t)(m0 >> 32);
    uint32_t c = v.z & (uint32_t)m1, d = v.w & (uint32_t)(m1 >> 32);
    if constexpr (PERM) {
        a = __builtin_amdgcn_perm(0u, a, sel);
        b = __builtin_amdgcn_perm(0u, b, sel);
        c = __builtin_amdgcn_perm(0u, c, sel);
        d = __builtin_amdgcn_perm(0u, d, sel);
    }
    return dot2_add(d, dot2_add(c, dot2_add(b, dot2_add(a, 0u))));
}

// ---------------------------------------------------------------- IPv6 extension headers
//
// pico_ipv6_extension_headers (modules/pico_ipv6.c:707-809) with the sequence check before it
// (pico_ipv6_check_headers_sequence, :659-694), for an RX datagram whose descriptor carries no
// seed and whose next header is not TCP / UDP / ICMPv6 (sorted kernel), and for every IPv6
// fragment (reassembly kernel) -- one lane walks its own datagram with byte loads (L2 hits: the
// header was just fetched).  Reads stay inside avail; where the reference would read past its buffer, or loop
// forever (a zero-length step: (uint8)((len + 1) << 3) wraps for len >= 31, an option length
// of 254), or let its uint16 f->net_len wrap, the datagram is WALK_BAD (MALFORMED).
//   WALK_DROP   the reference discards it (invalid / misplaced header, an option or routing
//               type that discards, M with a payload length not a multiple of 8, ESP / AUTH /
//               no next header)
//   WALK_PROTO  the transport is reached: net_len, proto
//   WALK_FRAG   the transport is reached behind a fragment header: pico_ipv6_process_frag
constexpr int WALK_BAD = -1, WALK_DROP = 0, WALK_PROTO = 1, WALK_FRAG = 2;

#define WBYTE(k, dst)                          \
    do {                                       \
        if ((uint32_t)(k) >= avail) return -2; \
        (dst) = h[(uint32_t)(k)];              \
    } while (0)

// pico_ipv6_process_hopbyhop (:525-582): must_align 1 / 0, -1 discard, -2 bad
__device__ __noinline__ int walk_hbh(const uint8_t* __restrict__ h, uint32_t avail, uint32_t e) {
    uint32_t b1, type, olen;
    WBYTE(e + 1, b1);
    uint32_t len = (((b1 + 1u) << 3) - 2u) & 0xFFu, opt = e + 2u;
    int must_align = 1;
    while (len) {
        WBYTE(opt, type);
        if (type == 0u) { ++opt; --len; continue; }                 // Pad1
        WBYTE(opt + 1u, olen);
        const uint32_t optlen = (olen + 2u) & 0xFFu;
        if (type == 5u) { if (olen == 2u) must_align = 0; }         // router alert (MLD)
        else if (type != 1u && (type & 0xC0u) != 0u) return -1;     // action: discard
        if (optlen == 0u) return -2;                                // the reference loops forever
        opt += optlen;
        len = (len - optlen) & 0xFFu;
    }
    return must_align;
}

// pico_ipv6_process_destopt (:610-657): 0 pass, -1 discard, -2 bad; every option advances opt[1] + 2
__device__ __noinline__ int walk_dst(const uint8_t* __restrict__ h, uint32_t avail, uint32_t e) {
    uint32_t b1, type, olen;
    WBYTE(e + 1, b1);
    uint32_t len = (((b1 + 1u) << 3) - 2u) & 0xFFu, opt = e + 2u;
    while (len) {
        WBYTE(opt, type);
        WBYTE(opt + 1u, olen);
        const uint32_t optlen = (olen + 2u) & 0xFFu;
        if (type != 0u && type != 1u && type != 201u && (type & 0xC0u) != 0u) return -1;
        if (optlen == 0u) return -2;
        opt += optlen;
        len = (len - optlen) & 0xFFu;
    }
    return 0;
}
#undef WBYTE

#define WBYTE(k, dst)                                            \
    do {                                                         \
        if ((uint32_t)(k) >= avail) return (uint64_t)(WALK_BAD + 1); \
        (dst) = h[(uint32_t)(k)];                                \
    } while (0)

// Returns kind + 1 | net_len << 8 | proto << 24 | f->frag << 32 (the last fragment header's
// offset / M field, :754) -- registers only, no stack slots for outputs.
__device__ __forceinline__ uint64_t ipv6_walk_packed(const uint8_t* __restrict__ h,
                                                                           uint32_t avail) {
    const uint32_t plen = ((uint32_t)h[4] << 8) | h[5];
    uint32_t nx = h[6], b, ptr = 40u;
    // sequence check: steps of (uint8)((len + 1) << 3) (0 when len >= 31: the next step reads
    // the same header again), 8 for a fragment header; at most 2 steps per 8 bytes of avail
    for (uint32_t it = 0;; ++it) {
        if (it > 2u * (avail >> 3) + 8u) return (uint64_t)(WALK_BAD + 1);
        uint32_t optlen;
        if (nx == 0u || nx == 43u || nx == 60u || nx == 50u || nx == 51u) {
            WBYTE(ptr + 1u, b);
            optlen = ((b + 1u) << 3) & 0xFFu;
        } else if (nx == 44u) {
            optlen = 8u;
        } else if (nx == 59u || nx == 6u || nx == 17u || nx == 58u) {
            break;
        } else {
            return (uint64_t)(WALK_DROP + 1);
        }
        WBYTE(ptr, nx);
        ptr += optlen;
    }
    // the walk: f->net_len (uint16) moves by >= 8 bytes a step
    uint32_t net_len = 40u, cur_nexthdr = 6u;
    bool must_align = false, frag = false;
    uint32_t om = 0;
    nx = h[6];
    ptr = 40u;
    for (;;) {
        const uint32_t e = net_len;
        uint32_t cur_optlen;
        if (nx == 6u || nx == 17u || nx == 58u) {
            if (must_align && (plen & 7u) != 0u) return (uint64_t)(WALK_DROP + 1);
            return ((uint64_t)om << 32) | (uint32_t)((frag ? WALK_FRAG : WALK_PROTO) + 1) | (net_len << 8) | (nx << 24);
        } else if (nx == 0u) {                                      // hop-by-hop: only first
            if (cur_nexthdr != 6u) return (uint64_t)(WALK_DROP + 1);
            WBYTE(e + 1u, b);
            cur_optlen = (b + 1u) << 3;
            const int r = walk_hbh(h, avail, e);
            if (r == -2) return (uint64_t)(WALK_BAD + 1);
            if (r < 0) return (uint64_t)(WALK_DROP + 1);
            must_align = r != 0;
        } else if (nx == 43u) {                                     // routing
            uint32_t segleft, type;
            WBYTE(e + 1u, b);
            cur_optlen = (b + 1u) << 3;
            WBYTE(e + 3u, segleft);
            if (segleft != 0u) {
                WBYTE(e + 2u, type);
                if (type != 2u) return (uint64_t)(WALK_DROP + 1);
            }
        } else if (nx == 44u) {                                     // fragment
            uint32_t om0, om1;
            cur_optlen = 8u;
            WBYTE(e + 3u, om1);
            WBYTE(e + 2u, om0);
            om = (om0 << 8) | om1;
            frag = true;
            if ((om1 & 1u) && (plen & 7u) != 0u) return (uint64_t)(WALK_DROP + 1);
        } else if (nx == 60u) {                                     // destination options
            WBYTE(e + 1u, b);
            cur_optlen = (b + 1u) << 3;
            must_align = true;
            const int r = walk_dst(h, avail, e);
            if (r == -2) return (uint64_t)(WALK_BAD + 1);
            if (r < 0) return (uint64_t)(WALK_DROP + 1);
        } else {                                                    // ESP, AUTH, none, invalid
            return (uint64_t)(WALK_DROP + 1);
        }
        if (net_len + cur_optlen > 0xFFFFu) return (uint64_t)(WALK_BAD + 1);        // the uint16 would wrap
        net_len += cur_optlen;
        WBYTE(e, nx);                                               // exthdr->nxthdr (:805)
        cur_nexthdr = ptr;
        ptr += cur_optlen;
    }
}
#undef WBYTE

struct FlatArgs {
    uint8_t* base;
    uint64_t base_len;
    const pico_csum_desc_dev* desc;
    uint32_t n;
    uint32_t fpw;
    int32_t crc_off;      // RAW
    uint32_t flags;
    uint16_t* out;        // RAW
    uint32_t* bad;        // RAW
    uint16_t* out_net;    // fused modes
    uint16_t* out_l4;
    uint8_t* verdict;
    uint32_t mac_lo;      // ETH: the device's MAC as stored (bytes 0-3, 4-5), with F_MACF
    uint32_t mac_hi;
};

constexpr uint32_t NONE = 0xFFFFFFFFu;


// ---------------------------------------------------------------- dispatch

// (G, CPL) shapes of the pipelined uniform kernel; the multi-pass uniform kernel adds U (frames
// in flight per group) and NT (non-temporal loads), with CPL*U <= 8 (<= 32 data VGPRs).
#define PICO_FOR_SHAPES(X) \
    X(64, 1) X(64, 2) X(64, 4) X(64, 8) \
    X(32, 1) X(32, 2) X(32, 4) X(32, 8) \
    X(16, 1) X(16, 2) X(16, 4) X(16, 8) \
    X(8, 1)  X(8, 2)  X(8, 4)  X(8, 8)  \
    X(4, 1)  X(4, 2)  X(4, 4)  X(4, 8)

#define PICO_FOR_CU(Y, g) \
    Y(g, 1, 1) Y(g, 2, 1) Y(g, 4, 1) Y(g, 8, 1) Y(g, 1, 2) Y(g, 2, 2) Y(g, 4, 2) Y(g, 1, 4) Y(g, 2, 4)

#define PICO_FOR_RAW(Y) PICO_FOR_CU(Y, 64) PICO_FOR_CU(Y, 32) PICO_FOR_CU(Y, 16) PICO_FOR_CU(Y, 8) PICO_FOR_CU(Y, 4)

// The software-pipelined uniform kernel also takes 3 and 5-7 chunks a lane (G >= 8): a frame then
// fills its lane group's one pass without whole void chunk slots (1500 B at G = 16: 6 chunks a
// lane, where CPL 8 left chunk slots 96-127 void in every frame).
#define PICO_FOR_PF_SHAPES(X) \
    PICO_FOR_SHAPES(X) \
    X(64, 3) X(64, 5) X(64, 6) X(64, 7) X(32, 3) X(32, 5) X(32, 6) X(32, 7) \
    X(16, 3) X(16, 5) X(16, 6) X(16, 7) X(8, 3)  X(8, 5)  X(8, 6)  X(8, 7)

inline bool shape_ok(uint32_t G, uint32_t CPL, uint32_t fpw, bool pf = false) {
    if (!(G == 4 || G == 8 || G == 16 || G == 32 || G == 64)) return false;
    if (!(CPL == 1 || CPL == 2 || CPL == 4 || CPL == 8 || (pf && G >= 8 && (CPL == 3 || (CPL >= 5 && CPL <= 7))))) return false;
    return fpw >= 1 && fpw <= 64 && fpw % (64 / G) == 0;
}

inline dim3 grid_for(uint32_t n, uint32_t fpw) {
    const uint64_t waves = ((uint64_t)n + fpw - 1) / fpw;
    return dim3((unsigned)((waves + 3) / 4));
}


}  // namespace

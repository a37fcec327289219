// pico_csum_kernels.hip -- CDNA4 (gfx950) kernels for picoTCP's Internet checksum.
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

struct Ipv4Args {
    uint8_t* base;
    uint64_t base_len;
    const pico_csum_desc_dev* desc;
    uint32_t n;
    uint32_t flags;
    uint32_t fpw;
    uint16_t* out_net;
    uint16_t* out_l4;
    uint8_t* verdict;
};

constexpr uint32_t V_ACCEPT = 1u, V_NET_BAD = 2u, V_L4_BAD = 4u, V_MALFORMED = 8u, V_EXPIRED = 16u;

__device__ __forceinline__ uint32_t sel4(uint32_t q, uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
    return q == 0 ? a : (q == 1 ? b : (q == 2 ? c : d));
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
    uint16_t* out_net;    // IPV4
    uint16_t* out_l4;
    uint8_t* verdict;
};

constexpr uint32_t NONE = 0xFFFFFFFFu;
constexpr uint32_t BIG_CHUNKS = 1u << 16;   // frames above this stream on their own

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

// The 16-bit LE word at byte q of the register-held chunks D (q + 2 <= 4 * N).
template <int N>
__device__ __forceinline__ uint32_t word_at(const uint32_t (&D)[N], uint32_t q) {
    const uint32_t i = q >> 2;
    uint32_t lo = D[0], hi = D[1];
#pragma unroll
    for (int m = 1; m < N; ++m) {
        lo = i == (uint32_t)m ? D[m] : lo;
        hi = i == (uint32_t)m ? (m + 1 < N ? D[m + 1] : 0u) : hi;
    }
    return __builtin_amdgcn_alignbyte(hi, lo, q & 3u) & 0xFFFFu;
}

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

// MODE: 0 RAW (p.crc_off / p.flags / p.out / p.bad), 1 fused IPv4, 2 fused IPv6
// (IPv4/IPv6 outputs in Ipv4Args-compatible fields of FlatArgs).
// Phase 4: lane `lane` finalizes its frame (output index idx) from the LDS state.
template <int MODE>
__device__ __forceinline__ void sorted_finish(const FlatArgs& p, SortedWaveLds& L, uint32_t lane, uint64_t idx,
                                              bool tx) {
    constexpr bool IPV6 = MODE == 2;
    asm volatile("" ::: "memory");
    const uint32_t acc_all = L.acc_all[lane], acc_x = L.acc_x[lane], acc_opt = L.acc_opt[lane];
    const uint4 info = L.info[lane], fin = L.fin[lane];
    const uint32_t xpos = L.xo[lane].x;
    const uint32_t r = info.w & 15u;
    uint8_t* fp = p.base + (((((uint64_t)info.y) << 32) | info.x) + r);
    uint32_t verdict = fin.x & 15u;
    const bool parsed = fin.x & 16u, l4_needed = fin.x & 32u, oob = fin.x & 64u;
    const uint32_t proto = (fin.x >> 8) & 0xFFu, tl = fin.x >> 16;
    const uint32_t hl = fin.y & 0xFFFFu, ipcrc = fin.y >> 16;
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
    } else if constexpr (IPV6) {
        uint32_t l4 = 0;
        if (parsed) {
            if (l4_needed) {
                if (!tx) {
                    if (proto == 6u || (proto == 17u && acc_x != 0u) || proto == 58u) {
                        l4 = finalize(pseudo + acc_all);
                        const uint32_t type = acc_x & 0xFFu;
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
        if (p.out_l4) p.out_l4[idx] = (uint16_t)l4;
        if (p.verdict) p.verdict[idx] = (uint8_t)verdict;
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
        if (tx && (p.flags & 0x401u) == 1u && verdict == V_ACCEPT) {   // 0x400: ablation
            store_crc(fp + 10, net);
            if ((proto == 6u || proto == 1u) && l4_needed) store_crc(fp + hl + (proto == 6u ? 16u : 2u), l4);
            else if (proto == 17u && tl >= 8u) store_crc(fp + hl + 6u, 0u);
        }
        if (p.out_net) p.out_net[idx] = (uint16_t)net;
        if (p.out_l4) p.out_l4[idx] = (uint16_t)l4;
        if (p.verdict) p.verdict[idx] = (uint8_t)verdict;
    }
}

// CPL 8 keeps 8 KiB of loads in flight per wave within 128 VGPRs (4 waves per
// SIMD: a 256K-frame batch at 64 frames per wave is one residency round); CPL 4
// fits 64 VGPRs (8 waves per SIMD).
template <int MODE, bool NT, int CPL, bool SMALL>
__device__ __forceinline__ void sorted_batch(const FlatArgs& p, SortedWaveLds& L, uint4* stage, uint32_t lane,
                                             uint64_t f0) {
    constexpr bool IPV4 = MODE == 1, IPV6 = MODE == 2;
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
    uint32_t verdict = V_MALFORMED, hl = 0, tl = 0, proto = 0, ipcrc = 0, pseudo = 0, hdr20 = 0;
    bool parsed = false, l4_needed = false;
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
        constexpr uint32_t HDR = IPV6 ? 40u : 20u;
        nlh = len >= HDR && !(p.flags & 0x200u) ? min(HW, (r + len + 15u) >> 4) : 0u;   // 0x200: ablation
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
        const uint4 c0 = hw[0], c1 = hw[1], c2 = hw[2], c3 = hw[3], c4 = hw[4];
        const uint32_t avail = len;
        if constexpr (IPV4) {
            if (avail >= 20) {
                const uint32_t D[16] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w,
                                        c2.x, c2.y, c2.z, c2.w, c3.x, c3.y, c3.z, c3.w};
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
            if (avail >= 40) {
                const uint32_t D[20] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w, c2.x, c2.y,
                                        c2.z, c2.w, c3.x, c3.y, c3.z, c3.w, c4.x, c4.y, c4.z, c4.w};
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
    }
    const uint64_t nch64 = ext ? ((uint64_t)r + ext + 15u) >> 4 : 0u;
    uint32_t nch = (uint32_t)min(nch64, (uint64_t)0xFFFFFFFFu);
    if constexpr (MODE != 0) {
        // sums over the head window: the region's chunks [0, k0) = window chunks
        // [d, d + k0) (d: where the region's chunk grid starts in the window -- IPv6:
        // behind the header); the rounds take region chunks [k0, nch).  A field
        // straddling the cut moves the cut down a chunk (a field is summed whole on one
        // side); options not inside the window (never, for IPv4) leave it all to the rounds.
        const uint32_t d = (uint32_t)min((a0off - a0h) >> 4, (uint64_t)HW);
        k0 = nlh > d ? min(nlh - d, nch) : 0u;
        if (xpos != NONE && xpos < 16u * k0 && xpos + 2u > 16u * k0) k0 = xpos >> 4;
        if (optend != 0u && optend > 16u * (d + k0)) k0 = 0;
        const uint32_t P = 16u * (d + k0), rs = 16u * d + r;
        const uint32_t re = min(rs + span, P);
        const bool xin = xpos != NONE && 16u * d + xpos + 2u <= P;
        const uint32_t xs = 16u * d + xpos;
        const bool oin = optend != 0u && k0 != 0u;
        const uint32_t sl = odd ? SEL_ODD : SEL_EVEN;
#pragma unroll
        for (uint32_t i = 0; i < HW; ++i) {
            if (i >= d && i < d + k0) {
                p_all += masked_chunk_sum<true>(hw[i], 16u * i, min(rs, re), re, sl);
                if (xin && !staged) p_x += masked_chunk_sum<true>(hw[i], 16u * i, xs, xs + 2u, sl);
                if (oin) p_opt += masked_chunk_sum<true>(hw[i], 16u * i, r + 20u, optend, sl);
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
    L.fin[lane] = make_uint4(verdict | (parsed ? 16u : 0u) | (l4_needed ? 32u : 0u) | (oob ? 64u : 0u) | (proto << 8) |
                                 (tl << 16),
                             hl | (ipcrc << 16), MODE == 0 ? seed : pseudo, hdr20);
    const bool any_odd = __builtin_amdgcn_ballot_w64(nch != 0 && odd) != 0;
    const bool any_xo = __builtin_amdgcn_ballot_w64(nch != 0 && (xpos != NONE || optend != 0)) != 0;

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

    // ---- 4. lane j finalizes frame j (state reloaded from LDS)
    if (lane < cnt) sorted_finish<MODE>(p, L, lane, f0 + lane, tx);
    __builtin_amdgcn_wave_barrier();
}

// One wave per batch of up to 64 frames.  (A persistent grid looping over batches
// measured slower: every wave repeats the same serial descriptor -> rounds chain.)
template <int MODE, bool NT, int CPL, bool SMALL = false>
__global__ __launch_bounds__(256, CPL == 8 || MODE != 0 ? 4 : 5) void csum_sorted_kernel(FlatArgs p) {
    __shared__ SortedWaveSmem<MODE != 0> lds_all[4];
    const uint32_t lane = threadIdx.x & 63u;
    SortedWaveSmem<MODE != 0>& S = lds_all[threadIdx.x >> 6];
    const uint64_t f0 = ((uint64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) * p.fpw;
    if (f0 < p.n) sorted_batch<MODE, NT, CPL, SMALL>(p, S.s, S.stage, lane, f0);
}

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

// ---------------------------------------------------------------- dispatch

// (G, CPL) shapes of the IPv4 kernel; the RAW kernel adds U (frames in flight per
// group) and NT (non-temporal loads), with CPL*U <= 8 (<= 32 data VGPRs).
#define PICO_FOR_SHAPES(X) \
    X(64, 1) X(64, 2) X(64, 4) X(64, 8) \
    X(32, 1) X(32, 2) X(32, 4) X(32, 8) \
    X(16, 1) X(16, 2) X(16, 4) X(16, 8) \
    X(8, 1)  X(8, 2)  X(8, 4)  X(8, 8)  \
    X(4, 1)  X(4, 2)  X(4, 4)  X(4, 8)

#define PICO_FOR_CU(Y, g) \
    Y(g, 1, 1) Y(g, 2, 1) Y(g, 4, 1) Y(g, 8, 1) Y(g, 1, 2) Y(g, 2, 2) Y(g, 4, 2) Y(g, 1, 4) Y(g, 2, 4)

#define PICO_FOR_RAW(Y) PICO_FOR_CU(Y, 64) PICO_FOR_CU(Y, 32) PICO_FOR_CU(Y, 16) PICO_FOR_CU(Y, 8) PICO_FOR_CU(Y, 4)

inline bool shape_ok(uint32_t G, uint32_t CPL, uint32_t fpw) {
    if (!(G == 4 || G == 8 || G == 16 || G == 32 || G == 64)) return false;
    if (!(CPL == 1 || CPL == 2 || CPL == 4 || CPL == 8)) return false;
    return fpw >= 1 && fpw <= 64 && fpw % (64 / G) == 0;
}

inline dim3 grid_for(uint32_t n, uint32_t fpw) {
    const uint64_t waves = ((uint64_t)n + fpw - 1) / fpw;
    return dim3((unsigned)((waves + 3) / 4));
}

}  // namespace

extern "C" {

int pico_csum_launch_ipv4_forward(void* base, uint64_t base_len, const void* desc, uint32_t n, uint8_t* verdict,
                                  void* stream) {
    if (n == 0) return (int)hipSuccess;
    FwdArgs a{static_cast<uint8_t*>(base), base_len, static_cast<const pico_csum_desc_dev*>(desc), n, verdict};
    const dim3 grid((unsigned)(((uint64_t)n + 255u) / 256u)), block(256);
    hipLaunchKernelGGL(ipv4_forward_kernel, grid, block, 0, static_cast<hipStream_t>(stream), a);
    return (int)hipGetLastError();
}

// Launchers used by the C host layer (picotcp_amd/csrc/pico_csum.c).  They
// validate the launch shape, enqueue, and return the hipError_t as int.

// Sorted-rounds descriptor kernel: mode 0 RAW, 1 fused IPv4, 2 fused IPv6; small: 1-lane
// rounds for frames of <= 8 chunks (cpl 8 only).
int pico_csum_launch_sorted(void* base, uint64_t base_len, const void* desc, uint32_t n, int mode, int32_t crc_off,
                            uint32_t flags, uint16_t* out, uint32_t* bad, uint16_t* out_net, uint16_t* out_l4,
                            uint8_t* verdict, uint32_t cpl, uint32_t nt, uint32_t fpw, uint32_t small,
                            void* stream) {
    if (fpw < 1 || fpw > 64 || !(cpl == 4 || cpl == 8) || mode < 0 || mode > 2 || (small && cpl != 8))
        return (int)hipErrorInvalidValue;
    if (n == 0) return (int)hipSuccess;
    FlatArgs a{static_cast<uint8_t*>(base), base_len, static_cast<const pico_csum_desc_dev*>(desc), n, fpw,
               crc_off, flags, out, bad, out_net, out_l4, verdict};
    const dim3 grid = grid_for(n, fpw), block(256);
    hipStream_t s = static_cast<hipStream_t>(stream);
    using K = void (*)(FlatArgs);
    // [mode][nt][cpl 4 | cpl 8 | cpl 8 with the 1-lane class]
#define SK(m, t) {csum_sorted_kernel<m, t, 4>, csum_sorted_kernel<m, t, 8>, csum_sorted_kernel<m, t, 8, true>}
    static const K table[3][2][3] = {{SK(0, false), SK(0, true)}, {SK(1, false), SK(1, true)},
                                     {SK(2, false), SK(2, true)}};
#undef SK
    const int v = cpl == 4 ? 0 : small ? 2 : 1;
    hipLaunchKernelGGL(table[mode][nt ? 1 : 0][v], grid, block, 0, s, a);
    return (int)hipGetLastError();
}

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

// pico_csum_k_raw.hip -- the uniform-ring kernels (K1p: frames that fit one pass, software-
// pipelined; K1: larger frames) and their launchers (called by pico_csum.c).  Descriptor batches
// of every mode run the sorted-rounds kernel (pico_csum_k_sorted.hip).
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
    // (the wave's last trip issues one set past its frames, all void loads at C1's 8 frames a
    // wave; skipping it measured mixed: c1 57.2-57.3 vs 57.6-57.8 us, c1_s1536 59.5-60.0 vs
    // 58.7-58.8 -- profiles/r06/ab_c1_notail.txt; not kept)
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


}  // namespace

extern "C" {

// Software-pipelined uniform kernel (one pass per frame: G*CPL*16 >= len + 15).
int pico_csum_launch_uniform_pf(const void* base, uint64_t base_len, uint64_t stride, uint32_t len, uint32_t n,
                                uint32_t seed, uint16_t* out, uint32_t G, uint32_t CPL, uint32_t nt, uint32_t fpw,
                                uint32_t win, void* stream) {
    if (!shape_ok(G, CPL, fpw, true) || (uint64_t)G * CPL * 16u < (uint64_t)len + 15u) return (int)hipErrorInvalidValue;
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
    PICO_FOR_PF_SHAPES(X)
#undef X
    return (int)hipErrorInvalidValue;
}

// Uniform ring, frames of any length (several passes per frame).
int pico_csum_launch_raw(const void* base, uint64_t base_len, uint64_t stride, uint32_t len, uint32_t n,
                         uint32_t seed, uint16_t* out, uint32_t G, uint32_t CPL, uint32_t U, uint32_t nt,
                         uint32_t fpw, void* stream) {
    if (!shape_ok(G, CPL, fpw) || !(U == 1 || U == 2 || U == 4) || CPL * U > 8) return (int)hipErrorInvalidValue;
    if (n == 0) return (int)hipSuccess;
    RawArgs a{static_cast<uint8_t*>(const_cast<void*>(base)), base_len, nullptr, stride, len, n, seed, -1, 0u, fpw,
              out, nullptr};
    const dim3 grid = grid_for(n, fpw), block(256);
    hipStream_t s = static_cast<hipStream_t>(stream);
#define Y(g, c, u)                                                                                          \
    if (G == g && CPL == c && U == u) {                                                                     \
        if (nt) hipLaunchKernelGGL((csum_raw_kernel<g, c, u, true, true>), grid, block, 0, s, a);           \
        else hipLaunchKernelGGL((csum_raw_kernel<g, c, u, true, false>), grid, block, 0, s, a);             \
        return (int)hipGetLastError();                                                                      \
    }
    PICO_FOR_RAW(Y)
#undef Y
    return (int)hipErrorInvalidValue;
}

}  // extern "C"

// tools/gather_ceiling.hip -- measurement aid (not product code): the bare gather of a reassembly
// batch -- every fragment's payload copied to its place in its datagram's output region, nothing
// parsed, nothing summed -- to price the reassembly kernel (pico_csum_k_frag.hip) against the data
// movement its layout forces (fragments in random arrival order across the buffer).  The per-fragment
// source / destination / length tables are computed on the host from the generator's layout.
//
//   hipcc --offload-arch=gfx950 -O3 -shared -fPIC tools/gather_ceiling.hip -o tools/bin/libgather_ceiling.so
//
// One wave per datagram (as the reassembly kernel at 4K datagrams); a step copies two fragments'
// payloads in 16-byte units (3 x 64 units, two 1480-byte payloads), byte-unaligned 16-byte buffer
// loads, 16-byte stores rounded up past a fragment's end (the bytes a neighbour then overwrites --
// the copy's result is not checked; only its time is).
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

extern "C" __global__ __launch_bounds__(64) void gather_copy(const uint8_t* src, uint64_t src_len,
                                                             const uint64_t* f_src, const uint64_t* f_dst,
                                                             const uint32_t* f_len, const uint32_t* grp,
                                                             uint32_t n_dgram, uint8_t* out, uint64_t out_len) {
    const uint32_t g = blockIdx.x, lane = threadIdx.x;
    if (g >= n_dgram) return;
    const uint32_t first = grp[2 * g], cnt = grp[2 * g + 1];
    const __amdgpu_buffer_rsrc_t sr =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(src), 0, (int)min(src_len, (uint64_t)0x7FFFFFF0u), 0x00020000);
    const __amdgpu_buffer_rsrc_t dr =
        __builtin_amdgcn_make_buffer_rsrc(out, 0, (int)min(out_len, (uint64_t)0x7FFFFFF0u), 0x00020000);
    constexpr int U = 3;
    for (uint32_t f = 0; f < cnt; f += 2) {
        const uint32_t fa = first + f, fb = first + min(f + 1u, cnt - 1u);
        const uint32_t la = f_len[fa], lb = f + 1u < cnt ? f_len[fb] : 0u;
        const uint32_t na = (la + 15u) >> 4, nt = na + ((lb + 15u) >> 4);
        const uint64_t sa = f_src[fa], sb = f_src[fb], da = f_dst[fa], db = f_dst[fb];
        u32x4 v[U];
#pragma unroll
        for (int k = 0; k < U; ++k) {
            const uint32_t x = 64u * k + lane;
            const bool b = x >= na;
            const uint64_t o = (b ? sb : sa) + 16u * (b ? x - na : x);
            v[k] = __builtin_amdgcn_raw_buffer_load_b128(sr, (int)(x < nt ? (uint32_t)o : 0x80000000u), 0, 2);
        }
#pragma unroll
        for (int k = 0; k < U; ++k) {
            const uint32_t x = 64u * k + lane;
            const bool b = x >= na;
            const uint64_t o = (b ? db : da) + 16u * (b ? x - na : x);
            __builtin_amdgcn_raw_buffer_store_b128(v[k], dr, (int)(x < nt ? (uint32_t)o : 0x80000000u), 0, 0);
        }
    }
}

extern "C" int gather_ceiling_launch(const void* src, uint64_t src_len, const void* f_src, const void* f_dst,
                                     const void* f_len, const void* grp, uint32_t n_dgram, void* out, uint64_t out_len,
                                     void* stream) {
    hipLaunchKernelGGL(gather_copy, dim3(n_dgram), dim3(64), 0, static_cast<hipStream_t>(stream),
                       static_cast<const uint8_t*>(src), src_len, static_cast<const uint64_t*>(f_src),
                       static_cast<const uint64_t*>(f_dst), static_cast<const uint32_t*>(f_len),
                       static_cast<const uint32_t*>(grp), n_dgram, static_cast<uint8_t*>(out), out_len);
    return (int)hipGetLastError();
}

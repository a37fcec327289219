// ring_probe.hip -- feasibility probe (not product code): can per-CU LDS slots filled by
// LDS-DMA loader waves and drained by consumer waves stream the C2 layout (256K simple-IMIX
// frames back to back behind 14 B gaps, descriptors in batches of FPB) at the HBM roofline?
// Consumers (CONSUMER_CHEAP: touch every chunk; otherwise lane per frame, raw byte sums checked
// against the host) read the slot and release it.  Build + run:
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/ring_probe tools/ring_probe.hip && /tmp/ring_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)

#ifndef SLOT_KB
#define SLOT_KB 16
#endif
#ifndef NSLOT_
#define NSLOT_ 8
#endif
#ifndef NCONS
#define NCONS 3
#endif
#ifndef NLOAD
#define NLOAD 4
#endif
#ifndef FPB
#define FPB 32
#endif
constexpr uint32_t SLOTC = SLOT_KB * 64;     // chunks (16 B) per slot
constexpr uint32_t NSLOT = NSLOT_;
constexpr uint32_t SPIN_CAP = 1u << 22;

struct Desc { uint64_t off; uint32_t len; uint32_t seed; };
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

struct Meta { uint32_t lo_l, lo_h, n, pad; };
struct RingLds {
    uint4 slot[NSLOT][SLOTC];
    uint4 desc[NSLOT][FPB];
    Meta meta[NSLOT];
    uint32_t full[NSLOT];
    uint32_t done[NSLOT];
};

__device__ __forceinline__ void wait_vm0() { __builtin_amdgcn_s_waitcnt(0x0F70); }

// LDS access through inline asm where a DMA may be in flight (the compiler would drain it)
__device__ __forceinline__ uint32_t lds_addr(const void* p) {
    return (uint32_t)(uintptr_t)((__attribute__((address_space(3))) const char*)p);
}
__device__ __forceinline__ uint32_t asm_ld32(const void* p) {
    uint32_t v;
    asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(lds_addr(p)) : "memory");
    return v;
}
__device__ __forceinline__ void asm_st32(void* p, uint32_t v) {
    asm volatile("ds_write_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" :: "v"(lds_addr(p)), "v"(v) : "memory");
}

// wave min / max of a uint32 (DPP row shifts + row broadcasts; result from lane 63)
template <bool MAX>
__device__ __forceinline__ uint32_t wave_ext(uint32_t v) {
    const int id = MAX ? 0 : -1;
    auto op = [](uint32_t a, uint32_t b) { return MAX ? (a > b ? a : b) : (a < b ? a : b); };
    v = op(v, (uint32_t)__builtin_amdgcn_update_dpp(id, (int)v, 0x111, 0xF, 0xF, false));   // row_shr:1
    v = op(v, (uint32_t)__builtin_amdgcn_update_dpp(id, (int)v, 0x112, 0xF, 0xF, false));   // row_shr:2
    v = op(v, (uint32_t)__builtin_amdgcn_update_dpp(id, (int)v, 0x114, 0xF, 0xF, false));   // row_shr:4
    v = op(v, (uint32_t)__builtin_amdgcn_update_dpp(id, (int)v, 0x118, 0xF, 0xF, false));   // row_shr:8
    v = op(v, (uint32_t)__builtin_amdgcn_update_dpp(id, (int)v, 0x142, 0xA, 0xF, false));   // row_bcast:15
    v = op(v, (uint32_t)__builtin_amdgcn_update_dpp(id, (int)v, 0x143, 0xC, 0xF, false));   // row_bcast:31
    return (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}

__global__ __launch_bounds__(64 * (NCONS + NLOAD), 1) void ring_kernel(const uint8_t* base, const Desc* desc, uint32_t n,
                                                                       uint32_t* out, uint32_t* err) {
    __shared__ RingLds L;
    const uint32_t wv = threadIdx.x >> 6, lane = threadIdx.x & 63u;
    const uint32_t nb = (n + FPB - 1) / FPB;
    const uint32_t nk = nb > blockIdx.x ? (nb - blockIdx.x + gridDim.x - 1) / gridDim.x : 0u;   // batches of this WG
    if (threadIdx.x < NSLOT) { L.full[threadIdx.x] = 0; L.done[threadIdx.x] = 0; }
    __syncthreads();
    auto dload = [&](uint32_t k) {
        const uint32_t f = (blockIdx.x + k * gridDim.x) * FPB + lane;
        return (lane < FPB && k < nk && f < n) ? *reinterpret_cast<const uint4*>(desc + f) : make_uint4(0, 0, 0, 0);
    };
    if (wv < NLOAD) {
        // ---- loader i: batches k = i (mod NLOAD); the next one's descriptors prefetched
        uint4 dn = dload(wv);
        for (uint32_t k = wv; k < nk; k += NLOAD) {
            const uint32_t s = k % NSLOT;
            const uint4 d = dn;
            const uint32_t f = (blockIdx.x + k * gridDim.x) * FPB + lane;
            const bool v = lane < FPB && f < n;
            // span relative to lane 0's frame (the batch is taken only within +-1 GiB of it)
            const uint64_t a = reinterpret_cast<uintptr_t>(base) + (((uint64_t)d.y << 32) | d.x);
            const uint64_t a0 = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(a >> 32)) << 32) |
                                (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)a);
            const int64_t rl = (int64_t)(a & ~15ull) - (int64_t)(a0 & ~15ull);
            const int64_t rh = (int64_t)((a + d.z + 15u) & ~15ull) - (int64_t)(a0 & ~15ull);
            const uint32_t lo_b = wave_ext<false>(v ? (uint32_t)(rl + (1ll << 31)) : 0xFFFFFFFFu);
            const uint32_t hi_b = wave_ext<true>(v ? (uint32_t)(rh + (1ll << 31)) : 0u);
            const uint64_t lo = (a0 & ~15ull) + (int64_t)lo_b - (1ll << 31);
            uint32_t nc = hi_b > lo_b ? (hi_b - lo_b) >> 4 : 0u;
            if (nc > SLOTC) nc = 0;                  // (such a batch is not staged: read from HBM)
            dn = dload(k + NLOAD);
            uint32_t spins = 0;
            while (k >= NSLOT && __builtin_amdgcn_readfirstlane(asm_ld32(&L.done[s])) != k + 1u - NSLOT) {
                if (++spins > SPIN_CAP) { if (lane == 0) atomicOr(err, 1u); return; }
                __builtin_amdgcn_s_sleep(1);
            }
            if (lane < FPB) {
                const u32x4 dv = {d.x, d.y, d.z, d.w};
                asm volatile("ds_write_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" :: "v"(lds_addr(&L.desc[s][lane])),
                             "v"(dv) : "memory");
            }
            if (lane == 0) {
                asm_st32(&L.meta[s].lo_l, (uint32_t)lo);
                asm_st32(&L.meta[s].lo_h, (uint32_t)(lo >> 32));
                asm_st32(&L.meta[s].n, nc);
            }
            for (uint32_t t = 0; t * 64u < nc; ++t) {
                const uint32_t c = t * 64u + lane;
                if (c < nc)
                    __builtin_amdgcn_global_load_lds((void*)(lo + 16ull * c),
                                                     (__attribute__((address_space(3))) void*)(&L.slot[s][64u * t]),
                                                     16, 0, 0);
            }
            wait_vm0();
            if (lane == 0) asm_st32(&L.full[s], k + 1u);
        }
    } else {
        // ---- consumer j: batches k = j (mod NCONS)
        for (uint32_t k = wv - NLOAD; k < nk; k += NCONS) {
            const uint32_t b = blockIdx.x + k * gridDim.x, s = k % NSLOT;
            uint32_t spins = 0;
            while (__builtin_amdgcn_readfirstlane(asm_ld32(&L.full[s])) != k + 1u) {
                if (++spins > SPIN_CAP) { if (lane == 0) atomicOr(err, 2u); return; }
                __builtin_amdgcn_s_sleep(1);
            }
            const uint32_t nc = L.meta[s].n;
            const uint64_t lo = ((uint64_t)L.meta[s].lo_h << 32) | L.meta[s].lo_l;
            const uint32_t f = b * FPB + lane;
            uint32_t acc = 0;
#ifdef CONSUMER_CHEAP
            for (uint32_t c = lane; c < nc; c += 64u) { const uint4 x = L.slot[s][c]; acc ^= x.x ^ x.y ^ x.z ^ x.w; }
#ifdef WORK
            // compute model: WORK dependent VALU instructions per batch
            for (int i = 0; i < WORK / 4; ++i) {
                acc = __builtin_amdgcn_alignbyte(acc, acc + 1u, 1u);
                acc = acc * 3u + (uint32_t)i;
                acc ^= acc >> 7;
            }
#endif
#else
            if (lane < FPB && f < n) {
                const uint4 dv = L.desc[s][lane];
                const uint64_t a = reinterpret_cast<uintptr_t>(base) + (((uint64_t)dv.y << 32) | dv.x);
                const uint32_t len = dv.z;
                const uint32_t r = (uint32_t)(a & 15u);
                const uint32_t c0 = (uint32_t)(((a & ~15ull) - lo) >> 4);
                const uint32_t ncf = (r + len + 15u) >> 4;
                for (uint32_t c = 0; c < ncf; ++c) {
                    const uint4 x = nc ? L.slot[s][c0 + c] : *reinterpret_cast<const uint4*>((a & ~15ull) + 16ull * c);
                    const uint32_t s0 = c == 0 ? r : 0u;
                    const uint32_t e0 = c + 1 == ncf ? r + len - 16u * c : 16u;
                    uint32_t w[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
                    for (int i = 0; i < 16; ++i) {
                        const uint32_t bb = (w[i >> 2] >> (8 * (i & 3))) & 0xFFu;
                        const bool in = (uint32_t)i >= s0 && (uint32_t)i < e0;
                        const bool first_of_pair = (((uint32_t)i - r) & 1u) == 0u;
                        acc += in ? (first_of_pair ? bb << 8 : bb) : 0u;
                    }
                }
            }
#endif
            __builtin_amdgcn_s_waitcnt(0xC07F);
            if (lane == 0) L.done[s] = k + 1u;
            if (lane < FPB && f < n) out[f] = acc;
        }
    }
}

int main(int argc, char** argv) {
    const uint32_t n = argc > 1 ? atoi(argv[1]) : 262144;
    const int grid = argc > 2 ? atoi(argv[2]) : 256;
    const uint32_t imix[12] = {64, 64, 64, 64, 64, 64, 64, 576, 576, 576, 576, 1500};
    uint64_t seedv = 12345;
    auto rnd = [&]() { seedv = seedv * 6364136223846793005ull + 1442695040888963407ull; return (uint32_t)(seedv >> 33); };
    std::vector<Desc> d(n);
    uint64_t pos = 0;
    for (uint32_t i = 0; i < n; ++i) {
        const uint32_t len = imix[rnd() % 12];
        pos += 14;
        d[i] = {pos, len, 0};
        pos += len;
    }
    const uint64_t total = pos + 64;
    std::vector<uint8_t> buf(total);
    for (auto& x : buf) x = (uint8_t)rnd();
    std::vector<uint32_t> want(n);
    for (uint32_t i = 0; i < n; ++i) {
        uint32_t acc = 0;
        for (uint32_t j = 0; j < d[i].len; ++j) acc += (j & 1u) ? buf[d[i].off + j] : (uint32_t)buf[d[i].off + j] << 8;
        want[i] = acc;
    }
    uint8_t* dbuf; Desc* ddesc; uint32_t *dout, *derr;
    CHECK(hipMalloc(&dbuf, total)); CHECK(hipMalloc(&ddesc, n * sizeof(Desc)));
    CHECK(hipMalloc(&dout, n * 4)); CHECK(hipMalloc(&derr, 4));
    CHECK(hipMemcpy(dbuf, buf.data(), total, hipMemcpyHostToDevice));
    CHECK(hipMemcpy(ddesc, d.data(), n * sizeof(Desc), hipMemcpyHostToDevice));
    CHECK(hipMemset(derr, 0, 4));
    CHECK(hipMemset(dout, 0, n * 4));
    hipEvent_t e0, e1; CHECK(hipEventCreate(&e0)); CHECK(hipEventCreate(&e1));
    const double bytes = (double)pos + 16.0 * n + 4.0 * n;
    auto launch = [&]() {
        hipLaunchKernelGGL(ring_kernel, dim3(grid), dim3(64 * (NCONS + NLOAD)), 0, 0, dbuf, ddesc, n, dout, derr);
    };
    launch();
    CHECK(hipDeviceSynchronize());
    uint32_t err = 0;
    CHECK(hipMemcpy(&err, derr, 4, hipMemcpyDeviceToHost));
    std::vector<uint32_t> got(n);
    CHECK(hipMemcpy(got.data(), dout, n * 4, hipMemcpyDeviceToHost));
    uint32_t bad = 0;
    for (uint32_t i = 0; i < n; ++i) bad += got[i] != want[i];
    const int K = 50;
    CHECK(hipEventRecord(e0));
    for (int i = 0; i < K; ++i) launch();
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms; CHECK(hipEventElapsedTime(&ms, e0, e1));
    const double us = ms * 1e3 / K;
    printf("ring slot=%dKB nslot=%d fpb=%d nload=%d ncons=%d grid=%d%s: %.2f us  %.0f GB/s (%.1f %% of 8 TB/s)  "
           "mismatches %u err %u\n", SLOT_KB, NSLOT_, FPB, NLOAD, NCONS, grid,
#ifdef CONSUMER_CHEAP
           " cheap",
#else
           "",
#endif
           us, bytes / us / 1e3, bytes / us / 1e3 / 80.0, bad, err);
    return 0;
}

// Measurement aid (not the product): the device pre-pass a byte-balanced C2 partition needs
// (VERDICT r05 item 1).  For a dense burst (descriptors in address order), wave k of W should
// start at the first datagram at or after byte k * B of the span, B = ceil(span / W).  One lane per
// descriptor, no atomics: lane i owns the boundaries in (pos[i-1], pos[i]] (pos = offset - offset[0])
// and writes start[k] = i for each; the last lane also writes n for the boundaries past the burst.
//
//   hipcc --offload-arch=gfx950 -O3 -shared -fPIC tools/c2_prepass.hip -o tools/bin/libc2_prepass.so
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {

struct Desc {
    uint64_t off;
    uint32_t len;
    uint32_t seed;
};

__global__ __launch_bounds__(256) void c2_prepass_kernel(const Desc* __restrict__ d, uint32_t n, uint32_t W,
                                                         uint32_t* __restrict__ start) {
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i >= n) return;
    const uint64_t o0 = d[0].off;
    const Desc last = d[n - 1];
    const uint64_t span = last.off + last.len - o0;
    const uint64_t B = (span + W - 1) / W;
    const uint64_t pos = d[i].off - o0;
    const uint64_t prev = i ? d[i - 1].off - o0 : 0;
    // boundaries k with prev < k B <= pos (lane 0: k = 0)
    uint64_t k = i ? prev / B + 1 : 0;
    const uint64_t ke = pos / B;
    for (; k <= ke && k < W; ++k) start[k] = i;
    if (i == n - 1)
        for (k = ke + 1; k <= W; ++k) start[k] = n;
}

}  // namespace

extern "C" int c2_prepass_launch(const void* desc, uint32_t n, uint32_t W, uint32_t* start, void* stream) {
    if (!n || !W) return (int)hipErrorInvalidValue;
    hipLaunchKernelGGL(c2_prepass_kernel, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream,
                       static_cast<const Desc*>(desc), n, W, start);
    return (int)hipGetLastError();
}

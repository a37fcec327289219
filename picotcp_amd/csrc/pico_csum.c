/*
 * pico_csum.c -- host side of libpicocsum, plain C (C99).
 *
 * Layer 1: the drop-in scalar symbols pico_checksum / pico_dualbuffer_checksum
 *          (ref stack/pico_frame.c:279-328) -- synchronous host code, the
 *          reference calls them inline per frame (see include/pico_csum.h).
 * Layer 2: argument checking + launch-shape choice for the batched HIP
 *          kernels (pico_csum_k_raw.hip: uniform rings; pico_csum_k_sorted.hip:
 *          every descriptor batch and the forwarding step; pico_csum_k_frag.hip:
 *          reassembly), reached through the thin extern "C" launchers declared below.
 * Layer 3: host-resident batches: pinned staging, two streams, chunked
 *          H2D -> kernel -> D2H overlap.
 */
#define _GNU_SOURCE
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <stdarg.h>
#include <pthread.h>

#include <hip/hip_runtime_api.h>

#include "pico_csum.h"

/* kernel TUs (C++/HIP), extern "C" */
int pico_csum_launch_raw(const void *base, uint64_t base_len, uint64_t stride, uint32_t len, uint32_t n,
                         uint32_t seed, uint16_t *out, uint32_t G, uint32_t CPL, uint32_t U, uint32_t nt,
                         uint32_t fpw, void *stream);
int pico_csum_launch_uniform_pf(const void *base, uint64_t base_len, uint64_t stride, uint32_t len, uint32_t n,
                                uint32_t seed, uint16_t *out, uint32_t G, uint32_t CPL, uint32_t nt, uint32_t fpw,
                                uint32_t win, void *stream);
/* kernel-only flags (pico_csum_dev.h F_MACF / F_NAT), set by this layer */
#define KF_MACF 0x10000u
#define KF_NAT 0x20000u
int pico_csum_launch_sorted(void *base, uint64_t base_len, const void *desc, uint32_t n, int mode, int32_t crc_off,
                            uint32_t flags, uint16_t *out, uint32_t *bad, uint16_t *out_net, uint16_t *out_l4,
                            uint8_t *verdict, uint32_t fpw, uint64_t mac48, void *stream);
int pico_csum_launch_uniform_stream(const void *base, uint64_t stride, uint32_t len, uint32_t n, uint32_t seed,
                                    uint16_t *out, uint32_t fpw, void *stream);
int pico_csum_launch_ipv4_forward(void *base, uint64_t base_len, const void *desc, uint32_t n, const uint32_t *local,
                                  uint32_t n_local, uint32_t *state, uint8_t *verdict, void *stream);
int pico_csum_launch_reassemble(int v6, const void *base, uint64_t base_len, const void *frag, uint32_t n_frag,
                                const uint32_t *groups, uint32_t n_dgram, void *out, uint64_t out_len, const void *out_desc,
                                uint32_t *o_len, uint16_t *o_l4, uint8_t *verdict, uint32_t flags, uint32_t flat_min,
                                void *stream);
int pico_csum_reasm_release_thread(void);

/* ------------------------------------------------------------------ errors */

static __thread char g_err[256];

static int fail(int code, const char *fmt, ...)
{
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
    return -code;
}

const char *pico_csum_last_error(void) { return g_err; }

/* ABI 1's F_REF_DISPATCH (0x4) meant the opposite of today's F_NXTHDR_DISPATCH (0x8): refused */
static const char *retired_note(uint32_t flags)
{
    return (flags & PICO_CSUM_F_RETIRED_0x4) ? " (0x4 is the retired ABI-1 dispatch bit; ABI 3: F_NXTHDR_DISPATCH = 0x8)"
                                             : "";
}
int pico_csum_abi_version(void) { return PICO_CSUM_ABI_VERSION; }

/* ------------------------------------------------------------------ layer 1 */

/* Exact S = sum of LE 16-bit words (+ odd trailing byte as the low byte),
 * 4 words per 8-byte load into a 64-bit accumulator; the caller reduces it
 * mod 2^32 exactly as the reference's uint32_t accumulator does. */
static uint64_t word_sum(const uint8_t *p, uint32_t len)
{
    uint64_t s = 0;
    uint32_t i = 0;
    for (; i + 8 <= len; i += 8) {
        uint64_t x;
        memcpy(&x, p + i, 8);
        s += (x & 0xFFFFu) + ((x >> 16) & 0xFFFFu) + ((x >> 32) & 0xFFFFu) + (x >> 48);
    }
    for (; i + 2 <= len; i += 2) {
        uint16_t w;
        memcpy(&w, p + i, 2);
        s += w;
    }
    if (len & 1u)
        s += p[len - 1];
    return s;
}

uint32_t pico_checksum_partial(uint32_t sum, const void *buf, uint32_t len)
{
    if (len == 0)
        return sum;
    return (uint32_t)(sum + word_sum((const uint8_t *)buf, len));
}

static uint16_t finalize(uint32_t sum)
{
    uint16_t c;
    while (sum >> 16)
        sum = (sum & 0xFFFFu) + (sum >> 16);
    c = (uint16_t)~sum;
    return (uint16_t)((c >> 8) | (c << 8));
}

uint16_t pico_checksum(void *inbuf, uint32_t len)
{
    return finalize(pico_checksum_partial(0, inbuf, len));
}

uint16_t pico_dualbuffer_checksum(void *inbuf1, uint32_t len1, void *inbuf2, uint32_t len2)
{
    return finalize(pico_checksum_partial(pico_checksum_partial(0, inbuf1, len1), inbuf2, len2));
}

uint32_t pico_ipv4_pseudo_partial(uint32_t src_addr, uint32_t dst_addr, uint8_t proto, uint16_t transport_len)
{
    /* struct pico_ipv4_pseudo_hdr bytes: src(4) dst(4) 0 proto len_be(2) as LE words */
    uint32_t s = 0;
    s += (src_addr & 0xFFFFu) + (src_addr >> 16);
    s += (dst_addr & 0xFFFFu) + (dst_addr >> 16);
    s += (uint32_t)proto << 8;
    s += (uint32_t)(uint16_t)((transport_len >> 8) | (transport_len << 8));
    return s;
}

uint32_t pico_ipv6_pseudo_partial(const void *src16, const void *dst16, uint8_t nxthdr, uint32_t transport_len)
{
    /* struct pico_ipv6_pseudo_hdr bytes: src(16) dst(16) len_be(4) zero(3) nxthdr as LE words */
    uint32_t s = (uint32_t)(word_sum((const uint8_t *)src16, 16) + word_sum((const uint8_t *)dst16, 16));
    uint32_t be = ((transport_len & 0xFFu) << 24) | ((transport_len & 0xFF00u) << 8) |
                  ((transport_len >> 8) & 0xFF00u) | (transport_len >> 24);
    s += (be & 0xFFFFu) + (be >> 16);
    s += (uint32_t)nxthdr << 8;
    return s;
}

/* ------------------------------------------------------------------ layer 2 */

/* Launch-shape override: per calling thread (a test or sweep setting it cannot race a
 * launch from another thread). */
static __thread uint32_t g_ovr_group, g_ovr_cpl, g_ovr_unroll, g_ovr_fpw, g_ovr_nt, g_ovr_pipe;
static __thread uint32_t g_ovr_smode, g_ovr_sfpw;     /* uniform-ring stream: 0 = automatic */
static __thread uint32_t g_host_staged;                 /* host descriptor batches: 1 = never in place */
static __thread uint32_t g_reasm_flat;                  /* reassembly flat grid: 0 auto, 1 always, 2 never */

int pico_csum_set_reasm_flat(uint32_t mode)
{
    if (mode > 2)
        return fail(PICO_CSUM_EINVAL, "reassembly flat-grid mode must be 0 (auto), 1 (always) or 2 (never)");
    g_reasm_flat = mode;
    return 0;
}

int pico_csum_release_thread_scratch(void)
{
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) {
        (void)hipGetLastError();
        return fail(PICO_CSUM_ENODEV, "pico_csum_release_thread_scratch: no HIP device");
    }
    return pico_csum_reasm_release_thread() ? fail(PICO_CSUM_EIO, "pico_csum_release_thread_scratch failed") : 0;
}

int pico_csum_set_host_in_place(uint32_t on)
{
    if (on > 1)
        return fail(PICO_CSUM_EINVAL, "in-place mode must be 0 (always staged) or 1 (automatic)");
    g_host_staged = !on;
    return 0;
}

int pico_csum_set_uniform_stream(uint32_t mode, uint32_t frames_per_wave)
{
    if (!(mode <= 1 || mode == PICO_CSUM_STREAM_OFF))
        return fail(PICO_CSUM_EINVAL, "uniform stream mode must be 0 (auto), 1 (on) or PICO_CSUM_STREAM_OFF");
    if (frames_per_wave > 65536)
        return fail(PICO_CSUM_EINVAL, "frames per wave in [1, 65536] (0 = auto)");
    g_ovr_smode = mode;
    g_ovr_sfpw = frames_per_wave;
    return 0;
}

int pico_csum_set_launch_override(uint32_t group, uint32_t cpl, uint32_t unroll, uint32_t fpw, uint32_t nt,
                                  uint32_t pipeline)
{
    if (group == 0 && cpl == 0 && unroll == 0 && fpw == 0 && nt == 0 && pipeline == 0) {
        g_ovr_group = g_ovr_cpl = g_ovr_unroll = g_ovr_fpw = g_ovr_nt = g_ovr_pipe = 0;
        return 0;
    }
    if (group == 2) {            /* descriptor batches: the sorted-rounds kernel, fpw frames per wave */
        if (fpw == 0 || fpw > 64)
            return fail(PICO_CSUM_EINVAL, "sorted-rounds kernel: fpw in [1, 64]");
        g_ovr_group = 2; g_ovr_fpw = fpw;
        g_ovr_cpl = g_ovr_unroll = g_ovr_nt = g_ovr_pipe = 0;
        return 0;
    }
    if (pipeline > 3)
        return fail(PICO_CSUM_EINVAL, "pipeline must be 0 (auto), 1 (off), 2 (on) or 3 (on, global loads "
                                        "instead of the buffer window)");
    if (!(group == 4 || group == 8 || group == 16 || group == 32 || group == 64))
        return fail(PICO_CSUM_EINVAL, "group must be 2 (descriptor batches) or 4, 8, 16, 32, 64 (uniform rings)");
    if (!(cpl >= 1 && cpl <= 8) || ((cpl == 3 || cpl >= 5) && cpl != 8 && (group < 8 || pipeline == 1)))
        return fail(PICO_CSUM_EINVAL, "cpl must be 1, 2, 4 or 8, or 3 / 5-7 with group >= 8 on the pipelined kernel");
    if (!(unroll == 1 || unroll == 2 || unroll == 4) || cpl * unroll > 8)
        return fail(PICO_CSUM_EINVAL, "unroll must be 1, 2 or 4 with cpl*unroll <= 8");
    if (fpw == 0 || fpw > 64 || fpw % (64 / group) != 0)
        return fail(PICO_CSUM_EINVAL, "fpw must be a multiple of 64/group in [1, 64]");
    if (nt > 3)
        return fail(PICO_CSUM_EINVAL, "nt must be 0 (auto), 1 (off), 2 (on) or 3 (on except frame edges)");
    g_ovr_group = group; g_ovr_cpl = cpl; g_ovr_unroll = unroll; g_ovr_fpw = fpw; g_ovr_nt = nt;
    g_ovr_pipe = pipeline;
    return 0;
}

struct shape { uint32_t G, CPL, U, nt, fpw, pipe; };

/* Uniform rings (measured on MI355X, DESIGN.md "Launch shapes"): a lane group spans the frame in
 * about 6-8 16-byte chunks per lane, all issued in one pass (CPL = 8), so a wave keeps 8 KiB of
 * loads in flight and the per-frame head/tail corrections and group reductions are shared by
 * 64/G frames.  Frames that fit one pass take the software-pipelined kernel (two frame sets in
 * registers; C1 8 frames per wave, bursts of <= 4K frames one set per group).  Larger frames
 * (C3 9000 B): the multi-pass kernel, ~16K waves in the grid.  Non-temporal loads pay on
 * frames >= 1 KiB (C1 +3 %, C3 +10 %). */
static struct shape uniform_shape(uint32_t n, uint32_t len)
{
    struct shape s;
    uint32_t chunks = len / 16u + 1u, per, ng, f;
    s.G = 4;
    while (s.G < 64 && s.G * 8u < chunks)
        s.G *= 2;
    per = (chunks + s.G - 1) / s.G;
    s.CPL = per <= 1 ? 1 : per <= 2 ? 2 : per <= 4 ? 4 : 8;
    s.U = 1;
    s.nt = len >= 1024u;
    ng = 64u / s.G;
    s.pipe = (uint64_t)s.G * s.CPL * 16u >= (uint64_t)len + 15u;
    if (s.pipe && s.G >= 8) {
        /* the pipelined kernel takes exactly the chunks a lane needs (3, 5-7 besides the powers of
         * two), so no chunk slot is void in every frame: C1 (1500 B, G 16) 59.2-59.4 us at 6 a lane
         * against 61.3 at 8 (profiles/r06/c1_cpl_sweep.txt) */
        const uint32_t need = (uint32_t)(((uint64_t)len + 15u + 15u) / 16u);
        const uint32_t exact = (need + s.G - 1) / s.G;
        if (exact == 3 || (exact >= 5 && exact < s.CPL))
            s.CPL = exact;
    }
    if (s.pipe) {
        f = n / 32768u;
        f -= f % ng;
        s.fpw = f < 2 * ng ? 2 * ng : f > 64 ? 64 : f;
        if (n <= 4096u)          /* bursts of <= 4K frames (tools/burst_sweep.py, r02g) */
            s.fpw = ng;
    } else {
        f = n / 16384u;
        if (f > 64u) f = 64u;
        f -= f % ng;
        s.fpw = f < ng ? ng : f;
    }
    if (g_ovr_group >= 4) {
        s.G = g_ovr_group; s.CPL = g_ovr_cpl; s.U = g_ovr_unroll; s.fpw = g_ovr_fpw;
        s.nt = g_ovr_nt >= 2 ? g_ovr_nt - 1 : 0;
        if (g_ovr_pipe)
            s.pipe = g_ovr_pipe >= 2;
    }
    return s;
}

/* Descriptor batches: the sorted-rounds kernel (each wave orders its <= 64 frames by size class
 * and sums them in lane-group rounds sized per round).  n / 2048 frames per wave in [4, 64]:
 * 1K-4K bursts 4 (-20 % vs 16), 16K 8, 64K 32, 256K 64 (one residency round of 64-frame waves)
 * -- tools/burst_sweep.py, r02g. */
static int desc_fpw(uint32_t n, uint32_t *fpw)
{
    uint32_t f = n / 2048u;
    if (g_ovr_group >= 4)
        return fail(PICO_CSUM_EINVAL, "launch override group %u is for uniform rings; descriptor batches take "
                                        "group 2", g_ovr_group);
    *fpw = g_ovr_group == 2 ? g_ovr_fpw : f < 4 ? 4 : f > 64 ? 64 : f;
    return 0;
}

static uint32_t cur_cus(void);

/* Device discovery runs once per process (pthread_once); compute-unit counts are read
 * per device, for the device current on the calling thread at launch. */
#define MAX_DEVS 64
static pthread_once_t g_dev_once = PTHREAD_ONCE_INIT;
static int g_dev_count;                     /* 0: no usable HIP device */
static uint32_t g_dev_cus[MAX_DEVS];        /* compute units per device (MI355X: 256) */

static void probe_devices(void)
{
    int count = 0, d;
    if (hipGetDeviceCount(&count) != hipSuccess || count <= 0)
        return;
    if (count > MAX_DEVS)
        count = MAX_DEVS;
    for (d = 0; d < count; d++) {
        int cus = 0;
        g_dev_cus[d] = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, d) == hipSuccess &&
                       cus > 0 ? (uint32_t)cus : 256u;
    }
    g_dev_count = count;
}

/* compute units of the device current on the calling thread */
static uint32_t cur_cus(void)
{
    int d = 0;
    if (hipGetDevice(&d) != hipSuccess || d < 0 || d >= g_dev_count)
        return 256u;
    return g_dev_cus[d];
}

static int need_device(void)
{
    pthread_once(&g_dev_once, probe_devices);
    if (g_dev_count <= 0)
        return fail(PICO_CSUM_ENODEV, "no HIP device: the batched checksum path runs only on the GPU");
    return 0;
}

static int launch_status(int herr, const char *what)
{
    if (herr == (int)hipSuccess)
        return 0;
    if (herr == (int)hipErrorInvalidValue)
        return fail(PICO_CSUM_EINVAL, "%s: invalid launch shape", what);
    if (herr == (int)hipErrorNoBinaryForGpu || herr == (int)hipErrorInvalidDeviceFunction)
        return fail(PICO_CSUM_ENODEV, "%s: no gfx950 kernel image for this device (%s)", what,
                    hipGetErrorString((hipError_t)herr));
    return fail(PICO_CSUM_EIO, "%s: %s", what, hipGetErrorString((hipError_t)herr));
}

int pico_checksum_batch_dev(void *d_base, uint64_t base_len, const struct pico_csum_desc *d_desc,
                            uint32_t n, int32_t crc_off, uint32_t flags, uint16_t *d_out,
                            uint32_t *d_bad, void *stream)
{
    uint32_t fpw = 0;
    int rc;
    if (n == 0)
        return 0;
    if (!d_base || !d_desc || !d_out)
        return fail(PICO_CSUM_EINVAL, "NULL buffer");
    if (((uintptr_t)d_desc & 15u) != 0)
        return fail(PICO_CSUM_EINVAL, "descriptor array must be 16-byte aligned");
    if (crc_off >= 0 && (crc_off & 1))
        return fail(PICO_CSUM_EINVAL, "crc_off must be even");
    if (flags & ~PICO_CSUM_F_WRITE)
        return fail(PICO_CSUM_EINVAL, "unknown flags 0x%x", flags);
    if ((flags & PICO_CSUM_F_WRITE) && crc_off < 0)
        return fail(PICO_CSUM_EINVAL, "F_WRITE needs crc_off >= 0");
    if ((rc = need_device()) != 0 || (rc = desc_fpw(n, &fpw)) != 0)
        return rc;
    return launch_status(pico_csum_launch_sorted(d_base, base_len, d_desc, n, 0, crc_off, flags,
                                                 d_out, d_bad, NULL, NULL, NULL, fpw, 0, stream),
                         "pico_checksum_batch_dev");
}

/* Uniform rings on the persistent stream waves (pico_csum_k_sorted.hip, csum_uniform_stream_kernel):
 * densely packed frames (the span a wave reads is the frames' own bytes, give or take a small gap),
 * no shape override, and -- where a frame can start at an odd address -- no carry out of 32 bits in
 * the byte-swapped fold (len <= 65535, seed < 2^31).  Measured against uniform_shape's kernels:
 * DESIGN.md 4. */
/* automatic: rings of at least 1 GiB.  One long stream per SIMD beats the lane-group kernels there
 * (C3 -5 %, C3 64 KiB -6 %, C4 -3.6 %) but not on C1's 375 MiB (+6 %: the XCDs' dispatch stagger
 * is a larger share of a shorter stream), profiles/r05/ab_uniform_stream_*.txt */
#define UNIFORM_STREAM_MIN_BYTES (1ull << 30)

static int uniform_stream_ok(const void *d_base, uint64_t stride, uint32_t len, uint32_t n, uint32_t seed)
{
    const uint64_t slack = len / 8u > 64u ? len / 8u : 64u;
    if (g_ovr_group >= 4 || g_ovr_smode == PICO_CSUM_STREAM_OFF || n == 0 || len == 0)
        return 0;
    if (stride < len || stride > (uint64_t)len + slack || stride * 64u <= 2u * 8192u)
        return 0;
    if ((((uintptr_t)d_base | stride) & 1u) && (len > 65535u || seed >= 0x80000000u))
        return 0;
    return 1;
}

int pico_checksum_batch_uniform_dev(const void *d_base, uint64_t base_len, uint64_t stride, uint32_t len,
                                    uint32_t n, uint32_t seed, uint16_t *d_out, void *stream)
{
    struct shape s;
    int rc;
    if (n == 0)
        return 0;
    if (!d_base || !d_out)
        return fail(PICO_CSUM_EINVAL, "NULL buffer");
    if ((uint64_t)(n - 1) > (UINT64_MAX - len) / (stride ? stride : 1) ||
        (uint64_t)(n - 1) * stride + len > base_len)
        return fail(PICO_CSUM_EINVAL, "frames exceed base_len");
    if ((rc = need_device()) != 0)
        return rc;
    if (g_ovr_group == 2)
        return fail(PICO_CSUM_EINVAL, "launch override group 2 is for descriptor batches");
    if (uniform_stream_ok(d_base, stride, len, n, seed) &&
        (g_ovr_smode == 1 || (g_ovr_smode == 0 && (uint64_t)n * stride >= UNIFORM_STREAM_MIN_BYTES))) {
        /* frames per wave: one wave per SIMD over the whole batch (C3: 256 frames of 9000 B, C4: 4096
         * of 1500 B) */
        const uint32_t waves = 4u * cur_cus();
        const uint32_t fpw = g_ovr_sfpw ? g_ovr_sfpw : (uint32_t)(((uint64_t)n + waves - 1u) / waves);
        if ((uint64_t)(fpw - 1u) * stride + len + 32u < (1ull << 31))
            return launch_status(pico_csum_launch_uniform_stream(d_base, stride, len, n, seed, d_out, fpw, stream),
                                 "pico_checksum_batch_uniform_dev");
    }
    s = uniform_shape(n, len);
    if (s.pipe && (uint64_t)s.G * s.CPL * 16u >= (uint64_t)len + 15u)
        return launch_status(pico_csum_launch_uniform_pf(d_base, base_len, stride, len, n, seed, d_out, s.G, s.CPL,
                                                         s.nt, s.fpw, g_ovr_pipe != 3, stream),
                             "pico_checksum_batch_uniform_dev");
    if (s.CPL == 3 || (s.CPL >= 5 && s.CPL <= 7)) {   /* the multi-pass kernel: power-of-two passes */
        s.CPL = s.CPL == 3 ? 4 : 8;
        if (s.CPL * s.U > 8)
            s.U = 1;
    }
    return launch_status(pico_csum_launch_raw(d_base, base_len, stride, len, n, seed, d_out, s.G, s.CPL, s.U, s.nt,
                                              s.fpw, stream),
                         "pico_checksum_batch_uniform_dev");
}

int pico_ipv4_checksum_batch_dev(void *d_base, uint64_t base_len, const struct pico_csum_desc *d_desc,
                                 uint32_t n, uint32_t flags, uint16_t *d_out_net,
                                 uint16_t *d_out_transport, uint8_t *d_verdict, void *stream)
{
    uint32_t fpw = 0;
    int rc;
    if (n == 0)
        return 0;
    if (!d_base || !d_desc)
        return fail(PICO_CSUM_EINVAL, "NULL buffer");
    if (((uintptr_t)d_desc & 15u) != 0)
        return fail(PICO_CSUM_EINVAL, "descriptor array must be 16-byte aligned");
    if (flags & ~(PICO_CSUM_F_WRITE | PICO_CSUM_F_TX))
        return fail(PICO_CSUM_EINVAL, "unknown flags 0x%x", flags);
    if ((flags & PICO_CSUM_F_WRITE) && !(flags & PICO_CSUM_F_TX))
        return fail(PICO_CSUM_EINVAL, "F_WRITE is a TX (F_TX) operation");
    if ((rc = need_device()) != 0 || (rc = desc_fpw(n, &fpw)) != 0)
        return rc;
    return launch_status(pico_csum_launch_sorted(d_base, base_len, d_desc, n, 1, -1, flags, NULL,
                                                 NULL, d_out_net, d_out_transport, d_verdict, fpw, 0, stream),
                         "pico_ipv4_checksum_batch_dev");
}

int pico_ipv4_nat_batch_dev(void *d_base, uint64_t base_len, const struct pico_csum_desc *d_desc, uint32_t n,
                            const struct pico_csum_nat *d_nat, uint16_t *d_out_net, uint16_t *d_out_transport,
                            uint8_t *d_verdict, void *stream)
{
    uint32_t fpw = 0;
    int rc;
    if (n == 0)
        return 0;
    if (!d_base || !d_desc || !d_nat)
        return fail(PICO_CSUM_EINVAL, "NULL buffer");
    if (((uintptr_t)d_desc & 15u) != 0 || ((uintptr_t)d_nat & 7u) != 0)
        return fail(PICO_CSUM_EINVAL, "descriptor array must be 16-byte, NAT records 8-byte aligned");
    if ((rc = need_device()) != 0 || (rc = desc_fpw(n, &fpw)) != 0)
        return rc;
    /* the IPv4 kernel in TX + in-place mode with the NAT stage; the records' address rides in the
     * launcher's 64-bit MAC argument (used as a MAC by the Ethernet mode only) */
    return launch_status(pico_csum_launch_sorted(d_base, base_len, d_desc, n, 1, -1,
                                                 PICO_CSUM_F_TX | PICO_CSUM_F_WRITE | KF_NAT, NULL,
                                                 NULL, d_out_net, d_out_transport, d_verdict, fpw,
                                                 (uint64_t)(uintptr_t)d_nat, stream),
                         "pico_ipv4_nat_batch_dev");
}

int pico_ipv6_checksum_batch_dev(void *d_base, uint64_t base_len, const struct pico_csum_desc *d_desc,
                                 uint32_t n, uint32_t flags, uint16_t *d_out_transport, uint8_t *d_verdict,
                                 void *stream)
{
    uint32_t fpw = 0;
    int rc;
    if (n == 0)
        return 0;
    if (!d_base || !d_desc)
        return fail(PICO_CSUM_EINVAL, "NULL buffer");
    if (((uintptr_t)d_desc & 15u) != 0)
        return fail(PICO_CSUM_EINVAL, "descriptor array must be 16-byte aligned");
    if (flags & ~(PICO_CSUM_F_WRITE | PICO_CSUM_F_TX | PICO_CSUM_F_NXTHDR_DISPATCH))
        return fail(PICO_CSUM_EINVAL, "unknown flags 0x%x%s", flags, retired_note(flags));
    if ((flags & PICO_CSUM_F_WRITE) && !(flags & PICO_CSUM_F_TX))
        return fail(PICO_CSUM_EINVAL, "F_WRITE is a TX (F_TX) operation");
    if ((flags & PICO_CSUM_F_NXTHDR_DISPATCH) && (flags & PICO_CSUM_F_TX))
        return fail(PICO_CSUM_EINVAL, "F_NXTHDR_DISPATCH is an RX option");
    if ((rc = need_device()) != 0 || (rc = desc_fpw(n, &fpw)) != 0)
        return rc;
    return launch_status(pico_csum_launch_sorted(d_base, base_len, d_desc, n, 2, -1, flags, NULL,
                                                 NULL, NULL, d_out_transport, d_verdict, fpw, 0, stream),
                         "pico_ipv6_checksum_batch_dev");
}

int pico_eth_checksum_batch_dev(void *d_base, uint64_t base_len, const struct pico_csum_desc *d_desc, uint32_t n,
                                uint32_t flags, const uint8_t *mac, uint16_t *d_out_net, uint16_t *d_out_transport,
                                uint8_t *d_verdict, void *stream)
{
    uint64_t mac48 = 0;
    uint32_t fpw = 0;
    int rc, i;
    if (n == 0)
        return 0;
    if (!d_base || !d_desc)
        return fail(PICO_CSUM_EINVAL, "NULL buffer");
    if (((uintptr_t)d_desc & 15u) != 0)
        return fail(PICO_CSUM_EINVAL, "descriptor array must be 16-byte aligned");
    if (flags & ~(PICO_CSUM_F_WRITE | PICO_CSUM_F_TX | PICO_CSUM_F_NXTHDR_DISPATCH))
        return fail(PICO_CSUM_EINVAL, "unknown flags 0x%x%s", flags, retired_note(flags));
    if ((flags & PICO_CSUM_F_WRITE) && !(flags & PICO_CSUM_F_TX))
        return fail(PICO_CSUM_EINVAL, "F_WRITE is a TX (F_TX) operation");
    if ((flags & PICO_CSUM_F_NXTHDR_DISPATCH) && (flags & PICO_CSUM_F_TX))
        return fail(PICO_CSUM_EINVAL, "F_NXTHDR_DISPATCH is an RX option");
    if ((rc = need_device()) != 0 || (rc = desc_fpw(n, &fpw)) != 0)
        return rc;
    if (mac) {
        for (i = 0; i < 6; i++)
            mac48 |= (uint64_t)mac[i] << (8 * i);
        flags |= KF_MACF;
    }
    return launch_status(pico_csum_launch_sorted(d_base, base_len, d_desc, n, 3, -1, flags, NULL, NULL,
                                                 d_out_net, d_out_transport, d_verdict, fpw, mac48, stream),
                         "pico_eth_checksum_batch_dev");
}

int pico_ipv4_forward_batch_dev(void *d_base, uint64_t base_len, const struct pico_csum_desc *d_desc, uint32_t n,
                                const uint32_t *local_addrs, uint32_t n_local, struct pico_csum_fwd_state *d_state,
                                uint8_t *d_verdict, void *stream)
{
    int rc;
    if (n == 0)
        return 0;
    if (!d_base || !d_desc || !d_verdict)
        return fail(PICO_CSUM_EINVAL, "NULL buffer (d_verdict is required)");
    if (((uintptr_t)d_desc & 15u) != 0)
        return fail(PICO_CSUM_EINVAL, "descriptor array must be 16-byte aligned");
    if (((uintptr_t)d_state & 3u) != 0)
        return fail(PICO_CSUM_EINVAL, "d_state must be 4-byte aligned");
    if (n_local > 32 || (n_local && !local_addrs))
        return fail(PICO_CSUM_EINVAL, "local_addrs: at most 32 host addresses");
    if ((rc = need_device()) != 0)
        return rc;
    return launch_status(pico_csum_launch_ipv4_forward(d_base, base_len, d_desc, n, local_addrs, n_local,
                                                       (uint32_t *)d_state, d_verdict, stream),
                         "pico_ipv4_forward_batch_dev");
}

static int reassemble_dev(int v6, const void *d_base, uint64_t base_len, const struct pico_csum_desc *d_frag,
                          uint32_t n_frag, const uint32_t *d_groups, uint32_t n_dgram, void *d_out, uint64_t out_len,
                          const struct pico_csum_desc *d_out_desc, uint32_t *d_out_len, uint16_t *d_out_transport,
                          uint8_t *d_verdict, uint32_t flags, void *stream, const char *what)
{
    int rc;
    if (n_dgram == 0)
        return 0;
    if (!d_base || !d_frag || !d_groups || !d_out || !d_out_desc)
        return fail(PICO_CSUM_EINVAL, "NULL buffer");
    if (((uintptr_t)d_frag & 15u) != 0 || ((uintptr_t)d_out_desc & 15u) != 0)
        return fail(PICO_CSUM_EINVAL, "descriptor arrays must be 16-byte aligned");
    if (((uintptr_t)d_groups & 3u) != 0 || ((uintptr_t)d_out & 3u) != 0)
        return fail(PICO_CSUM_EINVAL, "d_groups and d_out must be 4-byte aligned");
    if (flags & ~(v6 ? PICO_CSUM_F_NXTHDR_DISPATCH : 0u))
        return fail(PICO_CSUM_EINVAL, "unknown flags 0x%x%s", flags, retired_note(flags));
    if ((rc = need_device()) != 0)
        return rc;
    return launch_status(pico_csum_launch_reassemble(v6, d_base, base_len, d_frag, n_frag, d_groups, n_dgram, d_out,
                                                     out_len, d_out_desc, d_out_len, d_out_transport, d_verdict,
                                                     flags, g_reasm_flat == 1 ? 1u : g_reasm_flat == 2 ? UINT32_MAX : 0u,
                                                     stream),
                         what);
}

int pico_ipv4_reassemble_batch_dev(const void *d_base, uint64_t base_len, const struct pico_csum_desc *d_frag,
                                   uint32_t n_frag, const uint32_t *d_groups, uint32_t n_dgram, void *d_out,
                                   uint64_t out_len, const struct pico_csum_desc *d_out_desc, uint32_t *d_out_len,
                                   uint16_t *d_out_transport, uint8_t *d_verdict, void *stream)
{
    return reassemble_dev(0, d_base, base_len, d_frag, n_frag, d_groups, n_dgram, d_out, out_len, d_out_desc,
                          d_out_len, d_out_transport, d_verdict, 0, stream, "pico_ipv4_reassemble_batch_dev");
}

int pico_ipv6_reassemble_batch_dev(const void *d_base, uint64_t base_len, const struct pico_csum_desc *d_frag,
                                   uint32_t n_frag, const uint32_t *d_groups, uint32_t n_dgram, void *d_out,
                                   uint64_t out_len, const struct pico_csum_desc *d_out_desc, uint32_t *d_out_len,
                                   uint16_t *d_out_transport, uint8_t *d_verdict, uint32_t flags, void *stream)
{
    return reassemble_dev(1, d_base, base_len, d_frag, n_frag, d_groups, n_dgram, d_out, out_len, d_out_desc,
                          d_out_len, d_out_transport, d_verdict, flags, stream, "pico_ipv6_reassemble_batch_dev");
}

/* ------------------------------------------------------------------ layer 3 */

/* results buffer of a staging slot: one uint16 per frame, up to this many frames per chunk */
#define CTX_MAX_FRAMES(staging) ((staging) / 16u + 64u)

/* descriptors per chunk of a host-resident descriptor batch (>= 64 bytes a frame on average) */
#define CTX_MAX_DESC(staging) ((staging) / 64u + 64u)

/* staging slots (a buffer, a stream, an event each): the uniform ring alternates slots 0 and 1 (its
 * chunks need no per-chunk host work); staged descriptor batches rotate over all NSLOT, so the host
 * loop waits on the chunk three back, not two (r05: C2 staged).  The third slot's
 * staging buffer is allocated when a staged descriptor batch first needs it (the uniform ring and
 * the in-place descriptor path never do). */
#define NSLOT 3

struct pico_csum_ctx {
    int device;
    uint64_t staging;          /* bytes per staging buffer */
    void *d_buf[NSLOT];
    uint16_t *d_out[NSLOT];
    hipStream_t st[NSLOT];
    hipEvent_t done[NSLOT];
    /* descriptor batches (allocated on first use): rebased descriptors (pinned host ->
     * device) and the per-frame results of a chunk */
    struct pico_csum_desc *h_desc[NSLOT], *d_desc[NSLOT];
    /* a chunk's results, packed [net: 2 cnt B | transport: 2 cnt B | verdict: cnt B], so one D2H
     * brings them all back */
    uint8_t *d_res[NSLOT];
    /* pinned result staging: the D2H stays asynchronous (into pageable memory HIP would block
     * the host loop until it completes, serialising the chunks); copied out when the slot is
     * next reused or at the end */
    uint8_t *h_res[NSLOT];
    uint32_t pend_first[NSLOT], pend_cnt[NSLOT];
    int desc_ready;
};

static void ctx_desc_free(struct pico_csum_ctx *c);

struct pico_csum_ctx *pico_csum_ctx_create(int device, uint64_t staging_bytes)
{
    struct pico_csum_ctx *c;
    int i;
    if (need_device() != 0)
        return NULL;
    if (staging_bytes < (1u << 20))
        staging_bytes = 1u << 20;
    c = (struct pico_csum_ctx *)calloc(1, sizeof(*c));
    if (!c) { fail(PICO_CSUM_ENOMEM, "ctx alloc"); return NULL; }
    c->device = device;
    c->staging = staging_bytes;
    if (hipSetDevice(device) != hipSuccess) { fail(PICO_CSUM_ENODEV, "hipSetDevice(%d)", device); free(c); return NULL; }
    for (i = 0; i < NSLOT; i++) {
        if ((i < 2 && hipMalloc(&c->d_buf[i], staging_bytes) != hipSuccess) ||
            hipMalloc((void **)&c->d_out[i], 2u * CTX_MAX_FRAMES(staging_bytes)) != hipSuccess ||
            hipStreamCreateWithFlags(&c->st[i], hipStreamNonBlocking) != hipSuccess ||
            hipEventCreateWithFlags(&c->done[i], hipEventDisableTiming) != hipSuccess) {
            fail(PICO_CSUM_ENOMEM, "ctx device allocation (%llu B staging)", (unsigned long long)staging_bytes);
            pico_csum_ctx_destroy(c);
            return NULL;
        }
    }
    return c;
}

void pico_csum_ctx_destroy(struct pico_csum_ctx *c)
{
    int i;
    if (!c)
        return;
    hipSetDevice(c->device);
    for (i = 0; i < NSLOT; i++) {
        if (c->st[i]) hipStreamSynchronize(c->st[i]);
        if (c->d_buf[i]) hipFree(c->d_buf[i]);
        if (c->d_out[i]) hipFree(c->d_out[i]);
        if (c->done[i]) hipEventDestroy(c->done[i]);
        if (c->st[i]) hipStreamDestroy(c->st[i]);
    }
    ctx_desc_free(c);
    free(c);
}

int pico_csum_host_register(void *ptr, uint64_t bytes)
{
    hipError_t e = hipHostRegister(ptr, (size_t)bytes, hipHostRegisterDefault);
    if (e != hipSuccess)
        return fail(PICO_CSUM_EIO, "hipHostRegister: %s", hipGetErrorString(e));
    return 0;
}

void *pico_csum_host_device_pointer(void *ptr)
{
    void *d = NULL;
    hipError_t e = hipHostGetDevicePointer(&d, ptr, 0);
    if (e != hipSuccess) {
        fail(PICO_CSUM_EINVAL, "hipHostGetDevicePointer: %s (register the memory first)", hipGetErrorString(e));
        return NULL;
    }
    return d;
}

int pico_csum_host_unregister(void *ptr)
{
    hipError_t e = hipHostUnregister(ptr);
    if (e != hipSuccess)
        return fail(PICO_CSUM_EIO, "hipHostUnregister: %s", hipGetErrorString(e));
    return 0;
}

/* Frames [first, first+cnt) go into staging buffer b on stream b: H2D of the
 * contiguous span they occupy, kernel, D2H of their results.  The two streams
 * alternate so chunk c+1's H2D overlaps chunk c's kernel and D2H. */
int pico_checksum_batch_uniform_host(struct pico_csum_ctx *c, const void *base, uint64_t stride,
                                     uint32_t len, uint32_t n, uint32_t seed, uint16_t *out)
{
    uint64_t per;
    uint32_t first = 0;
    int b = 0, rc = 0;
    if (!c || !base || !out)
        return fail(PICO_CSUM_EINVAL, "NULL argument");
    if (n == 0)
        return 0;
    if (stride < len)
        return fail(PICO_CSUM_EINVAL, "host batch needs stride >= len (non-overlapping frames)");
    if (stride == 0 || (uint64_t)len > c->staging)
        return fail(PICO_CSUM_EINVAL, "frame larger than the staging buffer");
    per = (c->staging - len) / stride + 1;
    if (per > CTX_MAX_FRAMES(c->staging)) per = CTX_MAX_FRAMES(c->staging);
    if (hipSetDevice(c->device) != hipSuccess)
        return fail(PICO_CSUM_ENODEV, "hipSetDevice(%d)", c->device);
    while (first < n) {
        uint32_t cnt = (uint32_t)((n - first) < per ? (n - first) : per);
        uint64_t bytes = (uint64_t)(cnt - 1) * stride + len;
        const uint8_t *src = (const uint8_t *)base + (uint64_t)first * stride;
        hipError_t e;
        /* staging buffer b is free once its previous chunk's D2H is done (same stream: ordered) */
        e = hipMemcpyAsync(c->d_buf[b], src, bytes, hipMemcpyHostToDevice, c->st[b]);
        if (e != hipSuccess) { rc = fail(PICO_CSUM_EIO, "H2D: %s", hipGetErrorString(e)); break; }
        rc = pico_checksum_batch_uniform_dev(c->d_buf[b], c->staging, stride, len, cnt, seed, c->d_out[b], c->st[b]);
        if (rc) break;
        e = hipMemcpyAsync(out + first, c->d_out[b], (size_t)cnt * 2u, hipMemcpyDeviceToHost, c->st[b]);
        if (e != hipSuccess) { rc = fail(PICO_CSUM_EIO, "D2H: %s", hipGetErrorString(e)); break; }
        first += cnt;
        b ^= 1;
    }
    if (hipStreamSynchronize(c->st[0]) != hipSuccess || hipStreamSynchronize(c->st[1]) != hipSuccess)
        if (!rc) rc = fail(PICO_CSUM_EIO, "stream synchronize failed");
    return rc;
}

/* ---- host-resident descriptor batches (raw / IPv4 / IPv6 / Ethernet) */

enum { HB_RAW = 0, HB_IPV4 = 1, HB_IPV6 = 2, HB_ETH = 3 };

static void ctx_desc_free(struct pico_csum_ctx *c)
{
    int i;
    for (i = 0; i < NSLOT; i++) {
        if (c->h_desc[i]) hipHostFree(c->h_desc[i]);
        if (c->d_desc[i]) hipFree(c->d_desc[i]);
        if (c->d_res[i]) hipFree(c->d_res[i]);
        if (c->h_res[i]) hipHostFree(c->h_res[i]);
        c->h_desc[i] = c->d_desc[i] = NULL;
        c->d_res[i] = c->h_res[i] = NULL;
    }
    c->desc_ready = 0;
}

/* on the ctx's device (the caller has made it current); on failure nothing stays allocated */
static int ctx_desc_alloc(struct pico_csum_ctx *c)
{
    uint64_t nd = CTX_MAX_DESC(c->staging);
    int i;
    if (c->desc_ready)
        return 0;
    for (i = 0; i < NSLOT; i++) {
        if (hipHostMalloc((void **)&c->h_desc[i], nd * sizeof(struct pico_csum_desc), hipHostMallocDefault) != hipSuccess ||
            hipMalloc((void **)&c->d_desc[i], nd * sizeof(struct pico_csum_desc)) != hipSuccess ||
            hipMalloc((void **)&c->d_res[i], nd * 5u) != hipSuccess ||
            hipHostMalloc((void **)&c->h_res[i], nd * 5u, hipHostMallocDefault) != hipSuccess) {
            ctx_desc_free(c);
            return fail(PICO_CSUM_ENOMEM, "ctx descriptor staging (%llu descriptors)", (unsigned long long)nd);
        }
    }
    c->desc_ready = 1;
    return 0;
}

static int in_bounds(const struct pico_csum_desc *d, uint64_t base_len)
{
    return d->off <= base_len && d->len <= base_len - d->off;
}

/* a frame the staged path cannot stage (its 16-byte-aligned span exceeds the staging buffer) */
static int too_big(const struct pico_csum_ctx *c, const struct pico_csum_desc *d, uint64_t base_len)
{
    return in_bounds(d, base_len) && (d->len > c->staging || (d->off & 15u) + d->len > c->staging);
}

/* results of slot bb's last chunk, from pinned staging to the caller's arrays */
static void flush_results(struct pico_csum_ctx *c, int bb, uint16_t *out, uint16_t *out_net, uint16_t *out_l4,
                          uint8_t *verdict)
{
    const uint32_t f0 = c->pend_first[bb], fc = c->pend_cnt[bb];
    const uint8_t *r = c->h_res[bb];
    if (!fc)
        return;
    if (out) memcpy(out + f0, r + 2u * (size_t)fc, (size_t)fc * 2u);
    if (out_net) memcpy(out_net + f0, r, (size_t)fc * 2u);
    if (out_l4) memcpy(out_l4 + f0, r + 2u * (size_t)fc, (size_t)fc * 2u);
    if (verdict) memcpy(verdict + f0, r + 4u * (size_t)fc, fc);
    c->pend_cnt[bb] = 0;
}

/* the device batch of a host batch's mode (raw: its results in r_l4) */
static int run_desc_batch(int mode, void *kbase, uint64_t klen, const struct pico_csum_desc *d_desc, uint32_t cnt,
                          int32_t crc_off, uint32_t flags, const uint8_t *mac, uint16_t *r_net, uint16_t *r_l4,
                          uint8_t *r_ver, void *stream)
{
    switch (mode) {
    case HB_RAW:
        return pico_checksum_batch_dev(kbase, klen, d_desc, cnt, crc_off, flags, r_l4, NULL, stream);
    case HB_IPV4:
        return pico_ipv4_checksum_batch_dev(kbase, klen, d_desc, cnt, flags, r_net, r_l4, r_ver, stream);
    case HB_IPV6:
        return pico_ipv6_checksum_batch_dev(kbase, klen, d_desc, cnt, flags, r_l4, r_ver, stream);
    default:
        return pico_eth_checksum_batch_dev(kbase, klen, d_desc, cnt, flags, mac, r_net, r_l4, r_ver, stream);
    }
}

/* a chunk's packed result slot [net: 2 cnt B | transport: 2 cnt B | verdict: cnt B] */
static int run_desc_batch_packed(int mode, void *kbase, uint64_t klen, const struct pico_csum_desc *d_desc,
                                 uint32_t cnt, int32_t crc_off, uint32_t flags, const uint8_t *mac, uint8_t *d_res,
                                 void *stream)
{
    return run_desc_batch(mode, kbase, klen, d_desc, cnt, crc_off, flags, mac, (uint16_t *)d_res,
                          (uint16_t *)(d_res + 2u * (size_t)cnt), d_res + 4u * (size_t)cnt, stream);
}

/* the device alias of host memory [p, p + bytes) when the device addresses all of it (page-locked
 * by hipHostMalloc or registered), else NULL */
static void *host_alias(const void *p, uint64_t bytes)
{
    void *d0 = NULL, *d1 = NULL;
    if (!p || bytes == 0)
        return NULL;
    if (hipHostGetDevicePointer(&d0, (void *)p, 0) != hipSuccess || !d0 ||
        hipHostGetDevicePointer(&d1, (void *)((const uint8_t *)p + bytes - 1u), 0) != hipSuccess ||
        (uintptr_t)d1 - (uintptr_t)d0 != bytes - 1u) {
        (void)hipGetLastError();
        return NULL;
    }
    return d0;
}

/* the requested results of a chunk as one D2H range of its packed slot [net | transport | verdict] */
static void result_range(uint32_t cnt, const void *out, const void *out_net, const void *out_l4, const void *verdict,
                         size_t *r0, size_t *r1)
{
    *r0 = out_net ? 0u : (out || out_l4) ? 2u * (size_t)cnt : 4u * (size_t)cnt;
    *r1 = verdict ? 5u * (size_t)cnt : (out || out_l4) ? 4u * (size_t)cnt : 2u * (size_t)cnt;
}

/* descriptors a chunk of the in-place path (r05: 32K chunks 31.6 GiB/s, 128K 41.2, one chunk 40.4
 * on the C2 burst; profiles/r05/host_inplace_*.txt) */
#ifndef ZC_DESC
#define ZC_DESC 131072u
#endif

/* The in-place form of desc_batch_host: d_base is the burst's device alias. */
static int desc_batch_in_place(struct pico_csum_ctx *c, int mode, void *d_base, uint64_t base_len,
                               const struct pico_csum_desc *desc, uint32_t n, int32_t crc_off, uint32_t flags,
                               const uint8_t *mac, uint16_t *out, uint16_t *out_net, uint16_t *out_l4,
                               uint8_t *verdict, const char *what)
{
    const uint64_t maxd = CTX_MAX_DESC(c->staging);
    const uint32_t per = (uint32_t)(maxd < ZC_DESC ? maxd : ZC_DESC);
    const int write = (flags & PICO_CSUM_F_WRITE) != 0;
    uint32_t i = 0;
    int b = 0, prev = -1, o, rc = 0;
    hipError_t e;
    /* descriptors and every requested result array device-addressable too (a driver's pinned
     * rings): one launch over their aliases, nothing staged at all */
    {
        void *dd = ((uintptr_t)desc & 15u) == 0 ? host_alias(desc, (uint64_t)n * sizeof(struct pico_csum_desc)) : NULL;
        void *a_out = out ? host_alias(out, 2ull * n) : NULL, *a_net = out_net ? host_alias(out_net, 2ull * n) : NULL;
        void *a_l4 = out_l4 ? host_alias(out_l4, 2ull * n) : NULL, *a_ver = verdict ? host_alias(verdict, n) : NULL;
        if (dd && (!out || a_out) && (!out_net || a_net) && (!out_l4 || a_l4) && (!verdict || a_ver)) {
            rc = run_desc_batch(mode, d_base, base_len, (const struct pico_csum_desc *)dd, n, crc_off, flags, mac,
                                (uint16_t *)a_net, (uint16_t *)(mode == HB_RAW ? a_out : a_l4), (uint8_t *)a_ver,
                                c->st[0]);
            if ((e = hipStreamSynchronize(c->st[0])) != hipSuccess && !rc)
                rc = fail(PICO_CSUM_EIO, "%s: stream synchronize: %s", what, hipGetErrorString(e));
            return rc;
        }
    }
    while (i < n) {
        const uint32_t cnt = n - i < per ? n - i : per;
        size_t r0, r1;
        if ((e = hipEventSynchronize(c->done[b])) != hipSuccess) {
            rc = fail(PICO_CSUM_EIO, "%s: event synchronize: %s", what, hipGetErrorString(e));
            break;
        }
        flush_results(c, b, out, out_net, out_l4, verdict);
        memcpy(c->h_desc[b], desc + i, (size_t)cnt * sizeof(struct pico_csum_desc));
        if (write && prev >= 0 && (e = hipStreamWaitEvent(c->st[b], c->done[prev], 0)) != hipSuccess) {
            rc = fail(PICO_CSUM_EIO, "%s: stream wait: %s", what, hipGetErrorString(e));
            break;
        }
        if ((e = hipMemcpyAsync(c->d_desc[b], c->h_desc[b], (size_t)cnt * sizeof(struct pico_csum_desc),
                                hipMemcpyHostToDevice, c->st[b])) != hipSuccess) {
            rc = fail(PICO_CSUM_EIO, "%s: H2D: %s", what, hipGetErrorString(e));
            break;
        }
        if ((rc = run_desc_batch_packed(mode, d_base, base_len, c->d_desc[b], cnt, crc_off, flags, mac, c->d_res[b],
                                        c->st[b])) != 0)
            break;
        result_range(cnt, out, out_net, out_l4, verdict, &r0, &r1);
        if ((out || out_net || out_l4 || verdict) && r1 > r0 &&
            (e = hipMemcpyAsync(c->h_res[b] + r0, c->d_res[b] + r0, r1 - r0, hipMemcpyDeviceToHost, c->st[b])) !=
                hipSuccess) {
            rc = fail(PICO_CSUM_EIO, "%s: D2H: %s", what, hipGetErrorString(e));
            break;
        }
        c->pend_first[b] = i;
        c->pend_cnt[b] = cnt;
        if ((e = hipEventRecord(c->done[b], c->st[b])) != hipSuccess) {
            rc = fail(PICO_CSUM_EIO, "%s: event record: %s", what, hipGetErrorString(e));
            break;
        }
        prev = b;
        i += cnt;
        b = b + 1 == NSLOT ? 0 : b + 1;
    }
    for (o = 0; o < NSLOT; o++)                  /* drain: nothing lands after the return */
        if (hipStreamSynchronize(c->st[o]) != hipSuccess && !rc)
            rc = fail(PICO_CSUM_EIO, "%s: stream synchronize failed", what);
    if (!rc)
        for (o = 0; o < NSLOT; o++)
            flush_results(c, o, out, out_net, out_l4, verdict);
    return rc;
}

/* One burst: descriptors [i, j) whose bytes span at most the staging buffer go H2D (the span
 * and the descriptors, rebased to it) on stream b, through the device batch, and their results
 * D2H; the next chunk's H2D overlaps this one on the other stream.  A region outside base_len is
 * handed to the kernel as one (offset past the staging bound), so it gets the device API's
 * answer for it.
 * F_WRITE copies back only the hull of the chunk's own frames [first frame start, last frame
 * end) -- never the 16-byte rounding below it, which may hold the previous chunk's last frame --
 * and a chunk whose hull overlaps the hull of any chunk issued on the other stream (descriptors
 * not in ascending order) first waits for that stream, so no stale copy can land over a
 * result.  With F_WRITE every argument is checked before the first copy: an error returns with
 * nothing queued and no byte of `base` changed; without it a frame too large to stage is found
 * where its chunk would start (the results before it are unspecified, nothing is written to
 * `base`); a HIP error mid-burst drains the streams first. */
static int desc_batch_host(struct pico_csum_ctx *c, int mode, const void *base, uint64_t base_len,
                           const struct pico_csum_desc *desc, uint32_t n, int32_t crc_off, uint32_t flags,
                           const uint8_t *mac, uint16_t *out, uint16_t *out_net, uint16_t *out_l4, uint8_t *verdict,
                           const char *what)
{
    const uint64_t maxd = CTX_MAX_DESC(c ? c->staging : 0);
    const int write = (flags & PICO_CSUM_F_WRITE) != 0;
    uint32_t k;
    int o;
    uint64_t wlo[NSLOT], whi[NSLOT];            /* F_WRITE hulls issued per stream */
    uint32_t i = 0;
    int b = 0, rc = 0;
    if (!c || !base || !desc)
        return fail(PICO_CSUM_EINVAL, "%s: NULL argument", what);
    if (n == 0)
        return 0;
    if (hipSetDevice(c->device) != hipSuccess)
        return fail(PICO_CSUM_ENODEV, "hipSetDevice(%d)", c->device);
    if ((rc = ctx_desc_alloc(c)) != 0)
        return rc;
    for (k = 0; k < NSLOT; k++) {
        c->pend_cnt[k] = 0;
        wlo[k] = UINT64_MAX;
        whi[k] = 0;
    }
    /* A burst in page-locked memory the device addresses directly (hipHostMalloc'd, or registered
     * with pico_csum_host_register) is read in place -- and with F_WRITE written in place -- by the
     * kernel through its device alias: only descriptors and results go through the staging slots,
     * or nothing at all when they are device-addressable too (DESIGN.md 4 "PCIe-inclusive rate").
     * Chunks of ZC_DESC descriptors let one chunk's descriptor copy overlap the previous chunk's
     * kernel; with F_WRITE the kernels run in order (a chunk may read bytes an earlier one writes).
     * No frame is staged there, so no frame is too large for the staging buffer. */
    if (!g_host_staged) {
        void *d0 = host_alias(base, base_len);   /* (a pageable burst: the staged path below) */
        if (d0)
            return desc_batch_in_place(c, mode, d0, base_len, desc, n, crc_off, flags, mac, out, out_net, out_l4,
                                       verdict, what);
    }
    /* a frame larger than the staging buffer: with F_WRITE found before anything is queued (no byte
     * of base changes); else where the chunk loop meets it (the streams drained first) -- a pass
     * over every descriptor up front costs an RX burst ~0.2 ms of host time (C2, r05) */
    if (write)
        for (i = 0; i < n; i++)
            if (too_big(c, &desc[i], base_len))
                return fail(PICO_CSUM_EINVAL, "%s: frame %u of %u bytes exceeds the staging buffer", what, i,
                            desc[i].len);
    if (!c->d_buf[NSLOT - 1] && hipMalloc(&c->d_buf[NSLOT - 1], c->staging) != hipSuccess) {
        c->d_buf[NSLOT - 1] = NULL;
        return fail(PICO_CSUM_ENOMEM, "%s: third staging buffer (%llu B)", what, (unsigned long long)c->staging);
    }
    i = 0;
#define FLUSH(bb) flush_results(c, bb, out, out_net, out_l4, verdict)
#define TRY(call, msg)                                                                             \
    if ((e = (call)) != hipSuccess) {                                                              \
        rc = fail(PICO_CSUM_EIO, "%s: %s: %s", what, msg, hipGetErrorString(e));                   \
        break;                                                                                     \
    }
    while (i < n) {
        uint64_t lo = UINT64_MAX, hi = 0, hlo = UINT64_MAX;
        uint32_t j = i, cnt;
        hipError_t e;
        int vbase;
        uint8_t *kbase;
        uint64_t klen;
        /* grow the chunk while the span fits the staging buffer */
        while (j < n && (uint64_t)(j - i) < maxd) {
            uint64_t o = desc[j].off, oa, end;
            if (!in_bounds(&desc[j], base_len)) {      /* out of bounds: no bytes */
                j++;
                continue;
            }
            if (too_big(c, &desc[j], base_len)) {
                rc = fail(PICO_CSUM_EINVAL, "%s: frame %u of %u bytes exceeds the staging buffer", what, j,
                          desc[j].len);
                break;
            }
            oa = o & ~(uint64_t)15;   /* the span starts on a 16-byte line: frames keep their alignment */
            end = o + desc[j].len;
            if ((end > hi ? end : hi) - (oa < lo ? oa : lo) > c->staging)
                break;                /* (j > i: a single frame fits, checked above) */
            if (oa < lo) lo = oa;
            if (o < hlo) hlo = o;
            if (end > hi) hi = end;
            j++;
        }
        if (rc)
            break;
        cnt = j - i;
        if (lo == UINT64_MAX) lo = hi = hlo = 0;
        /* the pinned descriptor and result slots are reused: the previous chunk on them must be
         * done, and its results copied out */
        TRY(hipEventSynchronize(c->done[b]), "event synchronize")
        FLUSH(b);
        /* The kernel sees the staged span through a base pointer lo bytes below the staging
         * buffer, with base_len = hi: the caller's descriptors go over unchanged (one memcpy, no
         * rebase), a descriptor outside base_len stays outside [0, hi).  A staging buffer at a
         * device address below lo (never, in practice) and a chunk that ends more than 1 GiB into
         * the caller's buffer get rebased descriptors instead: the kernels' buffer windows (at
         * most 2 GiB, from 1 GiB below a wave's first frame) then always cover a whole chunk, so
         * no chunk takes their out-of-window paths. */
        vbase = (uintptr_t)c->d_buf[b] >= lo && hi <= (1ull << 30);
        if (vbase) {
            memcpy(c->h_desc[b], desc + i, (size_t)cnt * sizeof(struct pico_csum_desc));
        } else {
            for (k = 0; k < cnt; k++) {
                const struct pico_csum_desc *s = &desc[i + k];
                struct pico_csum_desc *t = &c->h_desc[b][k];
                t->off = in_bounds(s, base_len) ? s->off - lo : UINT64_MAX;
                t->len = s->len;
                t->seed = s->seed;
            }
        }
        kbase = vbase ? (uint8_t *)c->d_buf[b] - lo : (uint8_t *)c->d_buf[b];
        klen = vbase ? hi : hi - lo;
        for (o = 0; o < NSLOT && rc == 0; o++)      /* F_WRITE hulls of the other streams' chunks */
            if (o != b && write && hi > hlo && hlo < whi[o] && wlo[o] < hi)
                if ((e = hipStreamWaitEvent(c->st[b], c->done[o], 0)) != hipSuccess)
                    rc = fail(PICO_CSUM_EIO, "%s: stream wait: %s", what, hipGetErrorString(e));
        if (rc)
            break;
        if (hi > lo)
            TRY(hipMemcpyAsync(c->d_buf[b], (const uint8_t *)base + lo, hi - lo, hipMemcpyHostToDevice, c->st[b]), "H2D")
        TRY(hipMemcpyAsync(c->d_desc[b], c->h_desc[b], (size_t)cnt * sizeof(struct pico_csum_desc),
                           hipMemcpyHostToDevice, c->st[b]), "H2D")
        if ((rc = run_desc_batch_packed(mode, kbase, klen, c->d_desc[b], cnt, crc_off, flags, mac, c->d_res[b],
                                        c->st[b])) != 0)
            break;
        /* every requested result in one D2H (from the first requested array to the last) */
        {
            size_t r0, r1;
            result_range(cnt, out, out_net, out_l4, verdict, &r0, &r1);
            if ((out || out_net || out_l4 || verdict) && r1 > r0)
                TRY(hipMemcpyAsync(c->h_res[b] + r0, c->d_res[b] + r0, r1 - r0, hipMemcpyDeviceToHost, c->st[b]), "D2H")
        }
        c->pend_first[b] = i;
        c->pend_cnt[b] = cnt;
        if (write && hi > hlo) {
            TRY(hipMemcpyAsync((uint8_t *)base + hlo, (const uint8_t *)c->d_buf[b] + (hlo - lo), hi - hlo,
                               hipMemcpyDeviceToHost, c->st[b]), "D2H")
            if (hlo < wlo[b]) wlo[b] = hlo;
            if (hi > whi[b]) whi[b] = hi;
        }
        TRY(hipEventRecord(c->done[b], c->st[b]), "event record")
        i = j;
        b = b + 1 == NSLOT ? 0 : b + 1;
    }
#undef TRY
    /* drain every stream whatever happened: no copy may land after the return */
    for (o = 0; o < NSLOT; o++)
        if (hipStreamSynchronize(c->st[o]) != hipSuccess && !rc)
            rc = fail(PICO_CSUM_EIO, "%s: stream synchronize failed", what);
    if (!rc)
        for (o = 0; o < NSLOT; o++)
            FLUSH(o);
#undef FLUSH
    return rc;
}

int pico_checksum_batch_host(struct pico_csum_ctx *ctx, const void *base, uint64_t base_len,
                             const struct pico_csum_desc *desc, uint32_t n, int32_t crc_off, uint32_t flags,
                             uint16_t *out)
{
    if (!out)
        return fail(PICO_CSUM_EINVAL, "NULL argument");
    return desc_batch_host(ctx, HB_RAW, base, base_len, desc, n, crc_off, flags, NULL, out, NULL, NULL, NULL,
                           "pico_checksum_batch_host");
}

int pico_ipv4_checksum_batch_host(struct pico_csum_ctx *ctx, const void *base, uint64_t base_len,
                                  const struct pico_csum_desc *desc, uint32_t n, uint32_t flags, uint16_t *out_net,
                                  uint16_t *out_transport, uint8_t *verdict)
{
    return desc_batch_host(ctx, HB_IPV4, base, base_len, desc, n, -1, flags, NULL, NULL, out_net, out_transport,
                           verdict, "pico_ipv4_checksum_batch_host");
}

int pico_ipv6_checksum_batch_host(struct pico_csum_ctx *ctx, const void *base, uint64_t base_len,
                                  const struct pico_csum_desc *desc, uint32_t n, uint32_t flags,
                                  uint16_t *out_transport, uint8_t *verdict)
{
    return desc_batch_host(ctx, HB_IPV6, base, base_len, desc, n, -1, flags, NULL, NULL, NULL, out_transport, verdict,
                           "pico_ipv6_checksum_batch_host");
}

int pico_eth_checksum_batch_host(struct pico_csum_ctx *ctx, const void *base, uint64_t base_len,
                                 const struct pico_csum_desc *desc, uint32_t n, uint32_t flags, const uint8_t *mac,
                                 uint16_t *out_net, uint16_t *out_transport, uint8_t *verdict)
{
    return desc_batch_host(ctx, HB_ETH, base, base_len, desc, n, -1, flags, mac, NULL, out_net, out_transport,
                           verdict, "pico_eth_checksum_batch_host");
}

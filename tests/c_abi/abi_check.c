/*
 * abi_check.c -- the C host boundary of libpicocsum, exercised from plain C (no Python):
 * a C99 program compiled with gcc against include/pico_csum.h only, the way a picoTCP
 * host build would bind it.  Test infrastructure (tests/test_c_abi.py).
 *
 *   abi_check <fixture>          fixture: tests/golden/c_abi_burst.bin
 *
 * 1. pico_ipv4_checksum_batch_dev over a mixed IPv4 burst in device memory: TX compute
 *    with the in-place write (F_TX | F_WRITE), then RX verify of a corrupted copy;
 *    outputs and verdicts against the fixture's expected values.
 * 2. pico_checksum_batch_uniform_host over 1024 x 1500 B host frames (pinned with
 *    pico_csum_host_register), results against the fixture.
 * 3. The scalar drop-in pico_checksum on the same frames.
 * Exit status 0 only if every value matches; 2 when no HIP device is usable.
 * HIP is used only for device memory (hipMalloc / hipMemcpy): plain C API.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <hip/hip_runtime_api.h>

#include "pico_csum.h"

static uint8_t *g_fix;
static size_t g_fix_len, g_pos;

static const void *take(size_t n)
{
    const void *p;
    if (g_pos + n > g_fix_len) {
        fprintf(stderr, "fixture truncated at %zu (+%zu)\n", g_pos, n);
        exit(1);
    }
    p = g_fix + g_pos;
    g_pos += n;
    return p;
}

static uint32_t take_u32(void)
{
    uint32_t v;
    memcpy(&v, take(4), 4);
    return v;
}

static uint64_t splitmix64(uint64_t seed, uint64_t i)
{
    uint64_t z = seed + (i + 1) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

#define HIPCHECK(x)                                                                  \
    do {                                                                             \
        hipError_t e_ = (x);                                                         \
        if (e_ != hipSuccess) {                                                      \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                 \
        }                                                                            \
    } while (0)

static int cmp16(const char *what, const uint16_t *got, const void *want_raw, uint32_t n)
{
    uint32_t i, bad = 0;
    const uint8_t *w = (const uint8_t *)want_raw;
    for (i = 0; i < n; i++) {
        uint16_t want;
        memcpy(&want, w + 2u * i, 2);
        if (got[i] != want) {
            if (bad < 5)
                fprintf(stderr, "%s[%u]: got 0x%04x want 0x%04x\n", what, i, got[i], want);
            bad++;
        }
    }
    return bad ? 1 : 0;
}

static int cmp8(const char *what, const uint8_t *got, const uint8_t *want, uint32_t n)
{
    uint32_t i, bad = 0;
    for (i = 0; i < n; i++)
        if (got[i] != want[i]) {
            if (bad < 5)
                fprintf(stderr, "%s[%u]: got %u want %u\n", what, i, got[i], want[i]);
            bad++;
        }
    return bad ? 1 : 0;
}

int main(int argc, char **argv)
{
    FILE *f;
    uint32_t n, buf_len, i, u_n, u_len;
    uint64_t u_seed;
    const uint8_t *buf;
    const struct pico_csum_desc *desc;
    const void *tx_net, *tx_l4, *rx_net, *rx_l4;
    const uint8_t *tx_v, *rx_v;
    const void *u_want;
    void *d_buf, *d_desc, *d_net, *d_l4, *d_v;
    uint16_t *h_net, *h_l4, *u_out;
    uint8_t *h_v, *host, *frames;
    int fails = 0, rc, count = 0;
    struct pico_csum_ctx *ctx;

    if (argc != 2) {
        fprintf(stderr, "usage: %s <c_abi_burst.bin>\n", argv[0]);
        return 1;
    }
    f = fopen(argv[1], "rb");
    if (!f) { perror(argv[1]); return 1; }
    fseek(f, 0, SEEK_END);
    g_fix_len = (size_t)ftell(f);
    fseek(f, 0, SEEK_SET);
    g_fix = (uint8_t *)malloc(g_fix_len);
    if (!g_fix || fread(g_fix, 1, g_fix_len, f) != g_fix_len) { fprintf(stderr, "read failed\n"); return 1; }
    fclose(f);
    if (memcmp(take(4), "PCSA", 4) != 0 || take_u32() != 1) { fprintf(stderr, "bad fixture\n"); return 1; }
    n = take_u32();
    buf_len = take_u32();
    buf = (const uint8_t *)take(buf_len);
    desc = (const struct pico_csum_desc *)take((size_t)n * sizeof(struct pico_csum_desc));
    tx_net = take(2u * n); tx_l4 = take(2u * n); tx_v = (const uint8_t *)take(n);
    rx_net = take(2u * n); rx_l4 = take(2u * n); rx_v = (const uint8_t *)take(n);
    u_n = take_u32(); u_len = take_u32();
    memcpy(&u_seed, take(8), 8);
    u_want = take(2u * u_n);

    if (pico_csum_abi_version() != PICO_CSUM_ABI_VERSION) { fprintf(stderr, "ABI version mismatch\n"); return 1; }
    if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) {
        fprintf(stderr, "no HIP device\n");
        return 2;
    }

    /* ---- 1. fused IPv4 batch in device memory */
    HIPCHECK(hipMalloc(&d_buf, buf_len));
    HIPCHECK(hipMalloc(&d_desc, (size_t)n * sizeof(struct pico_csum_desc)));
    HIPCHECK(hipMalloc(&d_net, 2u * n));
    HIPCHECK(hipMalloc(&d_l4, 2u * n));
    HIPCHECK(hipMalloc(&d_v, n));
    HIPCHECK(hipMemcpy(d_buf, buf, buf_len, hipMemcpyHostToDevice));
    HIPCHECK(hipMemcpy(d_desc, desc, (size_t)n * sizeof(struct pico_csum_desc), hipMemcpyHostToDevice));
    h_net = (uint16_t *)malloc(2u * n); h_l4 = (uint16_t *)malloc(2u * n); h_v = (uint8_t *)malloc(n);
    host = (uint8_t *)malloc(buf_len);

    rc = pico_ipv4_checksum_batch_dev(d_buf, buf_len, (const struct pico_csum_desc *)d_desc, n,
                                      PICO_CSUM_F_TX | PICO_CSUM_F_WRITE, (uint16_t *)d_net, (uint16_t *)d_l4,
                                      (uint8_t *)d_v, NULL);
    if (rc) { fprintf(stderr, "TX batch: %d %s\n", rc, pico_csum_last_error()); return 1; }
    HIPCHECK(hipDeviceSynchronize());
    HIPCHECK(hipMemcpy(h_net, d_net, 2u * n, hipMemcpyDeviceToHost));
    HIPCHECK(hipMemcpy(h_l4, d_l4, 2u * n, hipMemcpyDeviceToHost));
    HIPCHECK(hipMemcpy(h_v, d_v, n, hipMemcpyDeviceToHost));
    fails += cmp16("tx_net", h_net, tx_net, n);
    fails += cmp16("tx_l4", h_l4, tx_l4, n);
    fails += cmp8("tx_verdict", h_v, tx_v, n);

    /* corrupt every 7th datagram's last byte (as the fixture's RX expectation does) */
    HIPCHECK(hipMemcpy(host, d_buf, buf_len, hipMemcpyDeviceToHost));
    for (i = 0; i < n; i += 7) {
        uint64_t last = desc[i].off + desc[i].len - 1;
        host[last] = (uint8_t)(host[last] + 1);
    }
    HIPCHECK(hipMemcpy(d_buf, host, buf_len, hipMemcpyHostToDevice));
    rc = pico_ipv4_checksum_batch_dev(d_buf, buf_len, (const struct pico_csum_desc *)d_desc, n, 0,
                                      (uint16_t *)d_net, (uint16_t *)d_l4, (uint8_t *)d_v, NULL);
    if (rc) { fprintf(stderr, "RX batch: %d %s\n", rc, pico_csum_last_error()); return 1; }
    HIPCHECK(hipDeviceSynchronize());
    HIPCHECK(hipMemcpy(h_net, d_net, 2u * n, hipMemcpyDeviceToHost));
    HIPCHECK(hipMemcpy(h_l4, d_l4, 2u * n, hipMemcpyDeviceToHost));
    HIPCHECK(hipMemcpy(h_v, d_v, n, hipMemcpyDeviceToHost));
    fails += cmp16("rx_net", h_net, rx_net, n);
    fails += cmp16("rx_l4", h_l4, rx_l4, n);
    fails += cmp8("rx_verdict", h_v, rx_v, n);

    /* ---- 2. host-resident uniform batch */
    frames = (uint8_t *)malloc((size_t)u_n * u_len + 8);
    for (i = 0; i < ((size_t)u_n * u_len + 7) / 8; i++) {
        uint64_t w = splitmix64(u_seed, i);
        memcpy(frames + 8u * i, &w, 8);
    }
    u_out = (uint16_t *)malloc(2u * u_n);
    if (pico_csum_host_register(frames, (uint64_t)u_n * u_len) != 0)
        fprintf(stderr, "note: host_register: %s (continuing pageable)\n", pico_csum_last_error());
    ctx = pico_csum_ctx_create(0, 1u << 20);
    if (!ctx) { fprintf(stderr, "ctx: %s\n", pico_csum_last_error()); return 1; }
    rc = pico_checksum_batch_uniform_host(ctx, frames, u_len, u_len, u_n, 0, u_out);
    if (rc) { fprintf(stderr, "uniform host: %d %s\n", rc, pico_csum_last_error()); return 1; }
    fails += cmp16("uniform_host", u_out, u_want, u_n);
    pico_csum_ctx_destroy(ctx);

    /* ---- 3. scalar drop-in on the same frames */
    for (i = 0; i < u_n; i++)
        u_out[i] = pico_checksum(frames + (size_t)i * u_len, u_len);
    fails += cmp16("scalar", u_out, u_want, u_n);
    pico_csum_host_unregister(frames);

    /* ---- 4. (ABI 4) this thread has run no reassembly: the release has nothing to free */
    if ((rc = pico_csum_release_thread_scratch()) != 0) {
        fprintf(stderr, "release_thread_scratch: %d %s\n", rc, pico_csum_last_error());
        fails++;
    }

    hipFree(d_buf); hipFree(d_desc); hipFree(d_net); hipFree(d_l4); hipFree(d_v);
    printf("abi_check: %u datagrams TX+RX, %u host frames, scalar: %s\n", n, u_n, fails ? "MISMATCH" : "ok");
    return fails ? 1 : 0;
}

/*
 * burst_main.c -- TEST INFRASTRUCTURE (tests/test_burst_driver.py): the batched RX driver of
 * integration/pico_dev_burst.c on an Ethernet burst, in front of the unmodified reference stack
 * built with CRC=0 (oracle/_ref/libref_rx_crc0.so, oracle/Makefile `burst`).
 *
 *   burst_main <burst.bin> <out.bin> [--no-gpu]
 *
 * burst.bin (little-endian): u32 n, u32 n4, u32 n6, u8 mac[6], u16 0, u64 ring_len,
 *   u32 ipv4_link[n4], u8 ipv6_link[n6][16], struct pico_csum_desc desc[n], u8 ring[ring_len].
 * out.bin: i32 used_gpu, u8 verdict[n], i32 delivered[n] (the protocol handed to the transport
 *   layer, -1 none), i32 check[n] (pico_transport_crc_check on it: the CRC=0 no-op, 1; -1 none),
 *   i32 routed[n] (1: the stack routed the frame on instead, rr_take_forwarded).
 *
 * The frames go on one by one as pico_burst_rx hands them on (pico_burst_hand_on), each through
 * rr_stack_rx (pico_stack_recv + the receive loops) so every transport hand-off is attributed to
 * its frame.  --no-gpu: no libpicocsum context, so the driver's host fallback makes the verdicts.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "pico_csum.h"
#include "pico_dev_burst.h"

int rr_init(void);
int rr_eth_init(const uint8_t *mac);
int rr_ipv4_link(uint32_t addr);
int rr_ipv6_link(const uint8_t *addr16);
int rr_stack_rx(const uint8_t *frame, uint32_t len);
int rr_take_delivered(int *check);
int rr_take_forwarded(void);

static void *slurp(const char *path, size_t *size)
{
    FILE *f = fopen(path, "rb");
    void *p;
    long sz;
    if (!f)
        return NULL;
    fseek(f, 0, SEEK_END);
    sz = ftell(f);
    fseek(f, 0, SEEK_SET);
    p = malloc((size_t)sz);
    if (p && fread(p, 1, (size_t)sz, f) != (size_t)sz) {
        free(p);
        p = NULL;
    }
    fclose(f);
    *size = (size_t)sz;
    return p;
}

int main(int argc, char **argv)
{
    size_t size, pos = 0;
    uint8_t *in, *ring, *verdict, mac[6];
    uint32_t n, n4, n6, i;
    uint64_t ring_len;
    struct pico_csum_desc *desc;
    int32_t *deliv, *check, *routed, used;
    struct pico_csum_ctx *ctx = NULL;
    FILE *out;
    if (argc < 3 || !(in = slurp(argv[1], &size)) || size < 24)
        return 2;
    memcpy(&n, in, 4);
    memcpy(&n4, in + 4, 4);
    memcpy(&n6, in + 8, 4);
    memcpy(mac, in + 12, 6);
    memcpy(&ring_len, in + 20, 8);
    pos = 28;
    if (rr_init() != 0 || rr_eth_init(mac) != 0)
        return 3;
    for (i = 0; i < n4; i++, pos += 4) {
        uint32_t a;
        memcpy(&a, in + pos, 4);
        rr_ipv4_link(a);
    }
    for (i = 0; i < n6; i++, pos += 16)
        rr_ipv6_link(in + pos);
    desc = malloc((size_t)n * sizeof(*desc) + 1);
    memcpy(desc, in + pos, (size_t)n * sizeof(*desc));
    pos += (size_t)n * sizeof(*desc);
    ring = in + pos;
    if (pos + ring_len > size)
        return 4;
    verdict = malloc(n + 1u);
    deliv = malloc(4u * n + 4u);
    check = malloc(4u * n + 4u);
    routed = malloc(4u * n + 4u);
    if (!(argc > 3 && strcmp(argv[3], "--no-gpu") == 0))
        ctx = pico_csum_ctx_create(0, 16u << 20);
    used = pico_burst_verdicts(ctx, mac, ring, ring_len, desc, n, verdict);
    if (ctx == NULL && argc <= 3)
        fprintf(stderr, "no context: %s\n", pico_csum_last_error());
    for (i = 0; i < n; i++) {
        deliv[i] = -1;
        check[i] = -1;
        routed[i] = 0;
        if (!pico_burst_hand_on(verdict[i], ring + desc[i].off, desc[i].len))
            continue;
        rr_stack_rx(ring + desc[i].off, desc[i].len);
        deliv[i] = rr_take_delivered(&check[i]);
        routed[i] = rr_take_forwarded();
    }
    if (ctx)
        pico_csum_ctx_destroy(ctx);
    out = fopen(argv[2], "wb");
    if (!out)
        return 5;
    fwrite(&used, 4, 1, out);
    fwrite(verdict, 1, n, out);
    fwrite(deliv, 4, n, out);
    fwrite(check, 4, n, out);
    fwrite(routed, 4, n, out);
    fclose(out);
    return 0;
}

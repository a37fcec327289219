/*
 * dropin_check.c -- TEST INFRASTRUCTURE ONLY: the drop-in proof.
 *
 * The reference's own caller code, compiled unmodified from /root/reference by
 * oracle/Makefile, is linked twice:
 *   argv[1]  libref_udp_dropin.so = modules/pico_udp.o + stack/pico_frame.o with
 *            its two checksum symbols renamed away (objcopy --redefine-sym), linked
 *            against libpicocsum.so -- the recipe of INTEGRATION.md section 1;
 *   argv[2]  libref_udp_native.so = the same two objects, unmodified.
 * pico_udp_checksum_ipv4 (modules/pico_udp.c:36-60, RX: pseudo header from the IPv4
 * header) then runs over the same frames through both; the drop-in build reaches
 * libpicocsum's pico_dualbuffer_checksum, the native one the reference's.  Frames
 * are allocated with the reference's pico_frame_alloc (stack/pico_frame.c).
 * Also checks pico_checksum (RFC 1071 section 3 vector, random regions) the same way.
 *
 * Output: one line "bound <path of the pico_dualbuffer_checksum the drop-in build
 * calls> frames <n> mismatches <m>"; exit 0 iff m == 0.
 * The libraries are opened RTLD_LAZY: pico_udp.o's other imports (pico_network_send,
 * ...) belong to the rest of the stack and are never called here.
 */
#define _GNU_SOURCE
#include <dlfcn.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include "pico_frame.h"

typedef uint16_t (*udp_fn)(struct pico_frame *);
typedef uint16_t (*csum_fn)(void *, uint32_t);
typedef uint16_t (*dual_fn)(void *, uint32_t, void *, uint32_t);
typedef struct pico_frame *(*alloc_fn)(uint32_t);
typedef void (*discard_fn)(struct pico_frame *);

static uint64_t rng_state = 0x5eedf00dULL;
static uint64_t splitmix64(void)
{
    uint64_t z = (rng_state += 0x9E3779B97F4A7C15ULL);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

static void *sym(void *h, const char *name)
{
    void *p = dlsym(h, name);
    if (!p) {
        fprintf(stderr, "dlsym %s: %s\n", name, dlerror());
        _exit(2);
    }
    return p;
}

int main(int argc, char **argv)
{
    void *hd, *hn;
    udp_fn udp_d, udp_n;
    csum_fn cs_d, cs_n;
    alloc_fn alloc;
    discard_fn discard;
    Dl_info di;
    unsigned frames = 0, bad = 0;
    static uint8_t rfc[8] = {0x00, 0x01, 0xf2, 0x03, 0xf4, 0xf5, 0xf6, 0xf7};

    if (argc < 3) {
        fprintf(stderr, "usage: %s libref_udp_dropin.so libref_udp_native.so\n", argv[0]);
        return 2;
    }
    hd = dlopen(argv[1], RTLD_LAZY | RTLD_LOCAL);
    hn = dlopen(argv[2], RTLD_LAZY | RTLD_LOCAL);
    if (!hd || !hn) {
        fprintf(stderr, "dlopen: %s\n", dlerror());
        return 2;
    }
    udp_d = (udp_fn)sym(hd, "pico_udp_checksum_ipv4");
    udp_n = (udp_fn)sym(hn, "pico_udp_checksum_ipv4");
    cs_d = (csum_fn)sym(hd, "pico_checksum");
    cs_n = (csum_fn)sym(hn, "pico_checksum");
    alloc = (alloc_fn)sym(hn, "pico_frame_alloc");
    discard = (discard_fn)sym(hn, "pico_frame_discard");
    if (!dladdr(sym(hd, "pico_dualbuffer_checksum"), &di) || !di.dli_fname)
        return 2;

    if (cs_d(rfc, 8) != 0x220D || cs_n(rfc, 8) != 0x220D)
        bad++;
    frames++;

    for (unsigned i = 0; i < 20000; i++) {
        uint32_t tl = 8u + (uint32_t)(splitmix64() % (i % 7 == 0 ? 65000u : 1493u));
        uint32_t lead = (uint32_t)(splitmix64() % 3u);           /* 0..2 bytes before the IPv4 header */
        uint32_t size = lead + 20u + tl;
        struct pico_frame *f = alloc(size);
        if (!f)
            return 2;
        for (uint32_t k = 0; k < size; k++)
            f->buffer[k] = (uint8_t)splitmix64();
        f->net_hdr = f->buffer + lead;
        f->net_hdr[0] = 0x45;
        f->net_hdr[9] = 17;
        f->net_len = 20;
        f->transport_hdr = f->net_hdr + 20;
        f->transport_len = (uint16_t)tl;
        f->sock = NULL;                                          /* RX: addresses from the header */
        if (udp_d(f) != udp_n(f))
            bad++;
        if (cs_d(f->net_hdr, 20u + tl) != cs_n(f->net_hdr, 20u + tl))
            bad++;
        frames++;
        discard(f);
    }
    printf("bound %s frames %u mismatches %u\n", di.dli_fname, frames, bad);
    return bad ? 1 : 0;
}

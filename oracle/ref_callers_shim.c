/*
 * ref_callers_shim.c -- TEST INFRASTRUCTURE ONLY (VERDICT r01 "next" item 2).
 *
 * Drives the reference's own compiled checksum CALLERS, so the fused IPv4 / IPv6
 * kernels are pinned to the reference and not only to restatements:
 *   pico_tcp_checksum_ipv4   modules/pico_tcp.c:422-446
 *   pico_tcp_checksum_ipv6   modules/pico_tcp.c:449-475
 *   pico_udp_checksum_ipv4   modules/pico_udp.c:36-60
 *   pico_udp_checksum_ipv6   modules/pico_udp.c:63-92
 *   pico_icmp6_checksum      modules/pico_icmp6.c:38-55
 *   pico_mld_checksum        modules/pico_mld.c:421-437
 * oracle/Makefile (`make refcallers`) compiles those files, unmodified, from
 * /root/reference together with stack/pico_frame.c and links them with this shim
 * into oracle/_ref/libref_callers.so (--gc-sections + a version script exporting
 * rc_checksum only, so nothing else of the stack is needed).
 *
 * rc_checksum builds the struct pico_frame the way the stack hands it to these
 * functions -- allocated with the reference's pico_frame_alloc, net_hdr at the
 * buffer start, transport_hdr = net_hdr + net_len, transport_len as the IPv4 /
 * IPv6 layer derived it -- and returns the caller's value:
 *   tx == 0  RX: f->sock = NULL, pseudo header from the IP header
 *   tx != 0  TX: the crc field is zeroed first (pico_tcp.c:980, pico_udp.c:121-123,
 *            pico_ipv6.c:1337,1345, pico_mld.c MLD report) and, for TCP / UDP, f->sock is
 *            a socket whose local / remote addresses are the header's source /
 *            destination (pico_tcp.c:429-433); ICMPv6 / MLD always use the header's.
 * tests/golden/make_ref_callers.py calls it through ctypes to write
 * tests/golden/ref_callers.npz.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "pico_frame.h"
#include "pico_socket.h"
#include "pico_tcp.h"
#include "pico_udp.h"
#include "pico_icmp6.h"
#include "pico_mld.h"

enum { RC_TCP4 = 0, RC_UDP4 = 1, RC_TCP6 = 2, RC_UDP6 = 3, RC_ICMP6 = 4, RC_MLD = 5 };

/* returns the caller's checksum (0..0xFFFF) or -1 on a bad argument */
int rc_checksum(int which, const uint8_t *datagram, uint32_t size, uint32_t net_len, uint32_t transport_len, int tx)
{
    struct pico_frame *f;
    struct pico_socket *s = NULL;
    int v6 = which >= RC_TCP6;
    /* crc field in the transport: TCP 16, UDP 6, ICMPv6 2, MLD 2 behind the 8-byte router alert */
    uint32_t xoff = which == RC_TCP4 || which == RC_TCP6 ? 16u : which == RC_UDP4 || which == RC_UDP6 ? 6u
                    : which == RC_MLD ? 10u : 2u;
    uint16_t ret;

    if (which < RC_TCP4 || which > RC_MLD || net_len + transport_len > size || net_len < (v6 ? 40u : 20u))
        return -1;
    f = pico_frame_alloc(size ? size : 1u);
    if (!f)
        return -1;
    memcpy(f->buffer, datagram, size);
    f->net_hdr = f->buffer;
    f->net_len = (uint16_t)net_len;
    f->transport_hdr = f->net_hdr + net_len;
    f->transport_len = (uint16_t)transport_len;
    f->sock = NULL;
    f->info = NULL;
    if (tx) {
        if (transport_len < xoff + 2u) {
            pico_frame_discard(f);
            return -1;
        }
        f->transport_hdr[xoff] = 0;
        f->transport_hdr[xoff + 1] = 0;
    }
    if (tx && which != RC_ICMP6 && which != RC_MLD) {   /* those two take the header's addresses */
        s = (struct pico_socket *)calloc(1, sizeof(*s));
        if (!s) {
            pico_frame_discard(f);
            return -1;
        }
        if (v6) {
            memcpy(s->local_addr.ip6.addr, f->net_hdr + 8, 16);
            memcpy(s->remote_addr.ip6.addr, f->net_hdr + 24, 16);
        } else {
            memcpy(&s->local_addr.ip4.addr, f->net_hdr + 12, 4);
            memcpy(&s->remote_addr.ip4.addr, f->net_hdr + 16, 4);
        }
        f->sock = s;
    }
    switch (which) {
    case RC_TCP4: ret = pico_tcp_checksum_ipv4(f); break;
    case RC_UDP4: ret = pico_udp_checksum_ipv4(f); break;
    case RC_TCP6: ret = pico_tcp_checksum_ipv6(f); break;
    case RC_UDP6: ret = pico_udp_checksum_ipv6(f); break;
    case RC_ICMP6: ret = pico_icmp6_checksum(f); break;
    default: ret = pico_mld_checksum(f); break;
    }
    f->sock = NULL;
    free(s);
    pico_frame_discard(f);
    return (int)ret;
}

/*
 * rc_batch_mt -- the reference's own per-datagram work of the C2 configurations, timed as the CPU
 * baseline of bench.py's fused lines: for each datagram of a batch (the
 * 16-byte descriptors of include/pico_csum.h), on `threads` pthreads over contiguous index ranges,
 * with a struct pico_frame per thread pointing at the datagram in place (the stack's frame after
 * pico_stack_recv; no allocation or copy is timed):
 *   mode 0  IPv4 RX: pico_checksum(hdr, net_len) (pico_ipv4_crc_check, modules/pico_ipv4.c:244-257)
 *           + pico_tcp_checksum_ipv4 / pico_udp_checksum_ipv4 with f->sock NULL (the RX check
 *           pico_transport_crc_check makes, stack/pico_socket.c:1916-1968)
 *   mode 1  IPv6 RX: pico_tcp_checksum_ipv6 / pico_udp_checksum_ipv6 of the transport behind
 *           the 40-byte header
 *   mode 2  IPv4 TX: the crc fields zeroed, pico_tcp_checksum_ipv4 with a socket carrying the
 *           header's addresses (tcp_send, modules/pico_tcp.c:968-985) and pico_checksum of the
 *           header (pico_ipv4_frame_push, modules/pico_ipv4.c:1079), both stored big-endian --
 *           in place, so `base` must be the caller's copy
 *   mode 3  Ethernet: the ethertype, then mode 0 or mode 1 at +14
 * out_net / out_l4 get the values (0 where none), for a parity check of the sample.
 */
#include <pthread.h>

struct rc_desc {
    uint64_t off;
    uint32_t len;
    uint32_t seed;
};

struct rc_job {
    uint8_t *base;
    const struct rc_desc *d;
    uint32_t lo, hi;
    int mode;
    uint16_t *out_net, *out_l4;
};

static uint32_t rc_be16(const uint8_t *p) { return ((uint32_t)p[0] << 8) | p[1]; }

static void rc_one(struct pico_frame *f, struct pico_socket *s, uint8_t *ip, uint32_t avail, int mode, int fam6,
                   uint16_t *net, uint16_t *l4)
{
    uint32_t hl, tot, proto;
    *net = *l4 = 0;
    if (fam6) {
        if (avail < 40u)
            return;
        proto = ip[6];
        f->net_hdr = ip;
        f->net_len = 40;
        f->transport_hdr = ip + 40;
        f->transport_len = (uint16_t)rc_be16(ip + 4);
        if (40u + f->transport_len > avail)
            return;
        f->sock = NULL;
        *l4 = proto == 6u ? pico_tcp_checksum_ipv6(f) : proto == 17u ? pico_udp_checksum_ipv6(f) : 0;
        return;
    }
    if (avail < 20u)
        return;
    hl = 4u * (ip[0] & 15u);
    tot = rc_be16(ip + 2);
    proto = ip[9];
    if (hl < 20u || hl > avail || tot < hl || tot > avail)
        return;
    f->net_hdr = ip;
    f->net_len = (uint16_t)hl;
    f->transport_hdr = ip + hl;
    f->transport_len = (uint16_t)(tot - hl);
    if (mode == 2) {                                   /* TX */
        ip[10] = ip[11] = 0;
        if (proto == 6u && tot - hl >= 20u) {
            f->transport_hdr[16] = f->transport_hdr[17] = 0;
            memcpy(&s->local_addr.ip4.addr, ip + 12, 4);
            memcpy(&s->remote_addr.ip4.addr, ip + 16, 4);
            f->sock = s;
            *l4 = pico_tcp_checksum_ipv4(f);
            f->transport_hdr[16] = (uint8_t)(*l4 >> 8);
            f->transport_hdr[17] = (uint8_t)*l4;
        }
        *net = pico_checksum(ip, hl);
        ip[10] = (uint8_t)(*net >> 8);
        ip[11] = (uint8_t)*net;
        return;
    }
    *net = pico_checksum(ip, hl);
    f->sock = NULL;
    if (proto == 6u)
        *l4 = pico_tcp_checksum_ipv4(f);
    else if (proto == 17u && tot - hl >= 8u && rc_be16(f->transport_hdr + 6))
        *l4 = pico_udp_checksum_ipv4(f);
}

static void *rc_worker(void *arg)
{
    struct rc_job *j = (struct rc_job *)arg;
    struct pico_frame f;
    struct pico_socket *s = (struct pico_socket *)calloc(1, sizeof(*s));
    uint32_t i;
    memset(&f, 0, sizeof(f));
    for (i = j->lo; i < j->hi; i++) {
        uint8_t *p = j->base + j->d[i].off;
        uint32_t len = j->d[i].len;
        int fam6 = j->mode == 1;
        if (j->mode == 3) {
            uint32_t et = len >= 14u ? rc_be16(p + 12) : 0u;
            if (et != 0x0800u && et != 0x86DDu) {
                j->out_net[i] = j->out_l4[i] = 0;
                continue;
            }
            fam6 = et == 0x86DDu;
            p += 14;
            len -= 14u;
        }
        rc_one(&f, s, p, len, j->mode, fam6, &j->out_net[i], &j->out_l4[i]);
    }
    free(s);
    return NULL;
}

int rc_batch_mt(uint8_t *base, const void *desc, uint32_t n, int mode, int threads, uint16_t *out_net,
                uint16_t *out_l4)
{
    struct rc_job job[64];
    pthread_t tid[64];
    int t;
    if (threads < 1 || threads > 64 || mode < 0 || mode > 3)
        return -1;
    for (t = 0; t < threads; t++) {
        job[t].base = base;
        job[t].d = (const struct rc_desc *)desc;
        job[t].lo = (uint32_t)((uint64_t)n * t / threads);
        job[t].hi = (uint32_t)((uint64_t)n * (t + 1) / threads);
        job[t].mode = mode;
        job[t].out_net = out_net;
        job[t].out_l4 = out_l4;
    }
    for (t = 1; t < threads; t++)
        if (pthread_create(&tid[t], NULL, rc_worker, &job[t]) != 0)
            return -1;
    rc_worker(&job[0]);
    for (t = 1; t < threads; t++)
        pthread_join(tid[t], NULL);
    return 0;
}

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

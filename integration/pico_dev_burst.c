/*
 * pico_dev_burst.c -- the reference-side binding of libpicocsum's batched RX verify
 * (pico_dev_burst.h).  A batching picoTCP device driver's poll step: read a
 * burst (a TAP driver reads one frame per read(), modules/pico_dev_tap.c:63-75; this one keeps a
 * ring of them), get every frame's verdict in one call, hand on what the reference would accept.
 * Built inside a picoTCP build with CRC=0; compiled and run against the unmodified reference
 * stack by oracle/Makefile `burst` (tests/test_burst_driver.py).
 *
 * The host fallback (burst_host_verdict) is driver code, not libpicocsum: when the GPU call fails
 * the burst is verified on the host with the scalar drop-in, frame by frame, instead of being
 * dropped or handed on unchecked.  It makes only the decisions a CRC=1 stack's two checks make --
 * pico_ipv4_crc_check (modules/pico_ipv4.c:243-257) and pico_transport_crc_check
 * (stack/pico_socket.c:1916-1968, TCP always, UDP when its crc != 0, dispatched on byte 9 of the
 * network header, which for IPv6 is the source address's second byte) -- and hands everything
 * else to the stack, which still makes all its other decisions.
 */
#include <stdint.h>
#include <string.h>

#include "pico_stack.h"
#include "pico_device.h"
#include "pico_ipv4.h"
#include "pico_ipv6.h"
#include "pico_dev_burst.h"

#define V_HAND_ON 1u     /* fallback verdict: the stack decides the rest (== PICO_CSUM_V_ACCEPT);
                          * | V_IPV6 on IPv6 frames, as the batch sets it */

static uint32_t be16(const uint8_t *p) { return ((uint32_t)p[0] << 8) | p[1]; }

/* A datagram the stack would route on (pico_ipv4_process_finally_try_forward, pico_ipv4.c:467;
 * pico_ipv6_process_in's forward, pico_ipv6.c:845-853): its transport checksum is never checked.
 * IPv4: not a local address, broadcast or multicast (pico_ipv4.c:458-467) -- and no 0.0.0.0 link
 * on the stack, which takes every such datagram into UDP's queue instead (:353-361, checked there).
 * IPv6: unicast and not local; when the first header is hop-by-hop (nxthdr 0) the reference
 * forwards only if `hbh->ext.routing.routtype` is 0 -- read through f->transport_hdr, which on RX
 * still points at the frame buffer's start there (pico_frame.c:112; nothing on the path from
 * pico_stack_recv sets it before pico_ipv6.c:789), so the byte is the Ethernet frame's byte 2,
 * the destination MAC's third byte (0 for a 33:33:00:.. multicast MAC, not for the device's own
 * 02:00:5e:..).  tests/test_burst_driver.py holds frames of both kinds. */
static int forwarded4(const uint8_t *ip)
{
    struct pico_ip4 dst, any;
    memcpy(&dst.addr, ip + 16, 4);
    any.addr = 0u;
    return !pico_ipv4_link_find(&dst) && !pico_ipv4_is_broadcast(dst.addr) && !pico_ipv4_is_multicast(dst.addr)
           && !pico_ipv4_link_find(&any);
}

static int forwarded6(const uint8_t *frame)
{
    const uint8_t *ip = frame + 14;
    struct pico_ip6 dst;
    memcpy(dst.addr, ip + 24, 16);
    if (!pico_ipv6_is_unicast(&dst) || pico_ipv6_link_get(&dst))
        return 0;
    return ip[6] != 0u || frame[2] == 0u;
}

/* The transport check of pico_transport_crc_check on `proto` (the network header's byte 9). */
static uint32_t l4_check(const uint8_t *pseudo, uint32_t plen, const uint8_t *t, uint32_t tl, uint32_t proto)
{
    if (proto == 6u)
        return pico_dualbuffer_checksum((void *)pseudo, plen, (void *)t, tl) ? PICO_CSUM_V_L4_BAD : V_HAND_ON;
    if (proto == 17u && tl >= 8u && be16(t + 6))
        return pico_dualbuffer_checksum((void *)pseudo, plen, (void *)t, tl) ? PICO_CSUM_V_L4_BAD : V_HAND_ON;
    return V_HAND_ON;
}

static uint8_t burst_host_verdict(const uint8_t *f, uint32_t len)
{
    uint32_t et;
    if (len < 14u)
        return V_HAND_ON;
    et = be16(f + 12);
    if (et == 0x0800u) {
        const uint8_t *ip = f + 14;
        const uint32_t avail = len - 14u, ihl = avail ? ip[0] & 15u : 0u;
        const uint32_t hl = 20u + (ihl > 5u ? 4u * (ihl - 5u) : 0u);
        uint32_t tot, tl, frag;
        uint8_t pseudo[12];
        if (avail < 20u || (ip[0] >> 4) != 4u)
            return V_HAND_ON;                            /* the Ethernet / IPv4 layer drops it */
        tot = be16(ip + 2);
        tl = (tot - hl) & 0xFFFFu;                       /* uint16 (pico_ipv4.c:395) */
        if (tl > ((avail - 20u) & 0xFFFFu))
            return V_HAND_ON;                            /* infeasible length: discarded first (:402-405) */
        if (hl > avail)
            return PICO_CSUM_V_MALFORMED;                /* the header check would read past the frame */
        if (pico_checksum((void *)ip, hl))
            return PICO_CSUM_V_NET_BAD;
        frag = be16(ip + 6);
        if (frag & 0x3FFFu || hl + tl > avail || (ip[9] != 6u && ip[9] != 17u) || forwarded4(ip))
            return V_HAND_ON;                            /* fragment / no local transport check */
        memcpy(pseudo, ip + 12, 8);
        pseudo[8] = 0;
        pseudo[9] = ip[9];
        pseudo[10] = (uint8_t)(tl >> 8);
        pseudo[11] = (uint8_t)tl;
        return (uint8_t)l4_check(pseudo, 12u, ip + hl, tl, ip[9]);
    }
    if (et == 0x86DDu) {
        const uint8_t *ip = f + 14;
        const uint32_t avail = len - 14u;
        uint32_t nh, off = 40u, plen, tl;
        uint8_t pseudo[40];
        if (avail < 40u || (ip[0] >> 4) != 6u)
            return V_HAND_ON | PICO_CSUM_V_IPV6;
        /* the transport behind hop-by-hop / routing / destination-option headers (a chain the
         * reference discards, or a fragment, is the stack's: handed on) */
        nh = ip[6];
        while (nh == 0u || nh == 43u || nh == 60u) {
            if (off + 2u > avail)
                return V_HAND_ON | PICO_CSUM_V_IPV6;
            nh = ip[off];
            off += ((uint32_t)ip[off + 1] + 1u) * 8u;
        }
        plen = be16(ip + 4);
        tl = (plen - (off - 40u)) & 0xFFFFu;             /* pico_ipv6.c:790 */
        if ((nh != 6u && nh != 17u) || off + tl > avail || forwarded6(f))
            return V_HAND_ON | PICO_CSUM_V_IPV6;
        memcpy(pseudo, ip + 8, 32);
        pseudo[32] = (uint8_t)(tl >> 24);
        pseudo[33] = (uint8_t)(tl >> 16);
        pseudo[34] = (uint8_t)(tl >> 8);
        pseudo[35] = (uint8_t)tl;
        pseudo[36] = pseudo[37] = pseudo[38] = 0;
        pseudo[39] = ip[9];                              /* pico_tcp/udp_checksum_ipv6's nxthdr: TCP / UDP */
        return (uint8_t)(l4_check(pseudo, 40u, ip + off, tl, ip[9]) | PICO_CSUM_V_IPV6);
    }
    return V_HAND_ON;
}

int pico_burst_verdicts(struct pico_csum_ctx *ctx, const uint8_t mac[6], const uint8_t *ring, uint64_t ring_len,
                        const struct pico_csum_desc *desc, uint32_t n, uint8_t *verdict)
{
    uint32_t i;
    if (ctx && pico_eth_checksum_batch_host(ctx, ring, ring_len, desc, n, 0, mac, NULL, NULL, verdict) == 0)
        return 1;
    /* no GPU verdicts (pico_csum_last_error() says why): the same checks on the host */
    for (i = 0; i < n; i++)
        verdict[i] = desc[i].off <= ring_len && desc[i].len <= ring_len - desc[i].off
                         ? burst_host_verdict(ring + desc[i].off, desc[i].len)
                         : (uint8_t)PICO_CSUM_V_MALFORMED;
    return 0;
}

int pico_burst_hand_on(uint8_t verdict, const uint8_t *frame, uint32_t len)
{
    const uint8_t v = verdict & (uint8_t)~PICO_CSUM_V_IPV6;
    if (v == PICO_CSUM_V_ACCEPT || v == PICO_CSUM_V_ARP || v == PICO_CSUM_V_FRAG)
        return 1;
    /* a transport checksum only matters to a datagram delivered here: one the stack routes on
     * goes on (a CRC=1 stack never checks it) */
    if (v == PICO_CSUM_V_L4_BAD)                   /* (an L4 verdict implies a whole IP header) */
        return (verdict & PICO_CSUM_V_IPV6) ? len >= 54u && forwarded6(frame)
                                            : len >= 34u && forwarded4(frame + 14);
    return 0;
}

int pico_burst_rx(struct pico_device *dev, struct pico_csum_ctx *ctx, const uint8_t mac[6], uint8_t *ring,
                  uint64_t ring_len, const struct pico_csum_desc *desc, uint32_t n, uint8_t *verdict)
{
    uint32_t i;
    int handed = 0;
    pico_burst_verdicts(ctx, mac, ring, ring_len, desc, n, verdict);
    for (i = 0; i < n; i++) {
        if (!pico_burst_hand_on(verdict[i], ring + desc[i].off, desc[i].len))
            continue;
        if (pico_stack_recv(dev, ring + desc[i].off, desc[i].len) < 0)
            return -1;
        handed++;
    }
    return handed;
}

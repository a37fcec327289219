/*
 * pico_csum_oracle.c -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of picoTCP's Internet-checksum path, used as the parity
 * checker (tests/, __graft_entry__.smoke()) and as the CPU baseline leg of
 * bench.py.  Nothing in the product library (picotcp_amd/) links, loads or
 * calls this file; the product's batched path is the HIP kernel and it fails
 * loudly when that is unavailable.
 *
 * Parity is PINNED: every function below is checked bit-for-bit against
 * (1) oracle/_ref/libpicoref.so, built by oracle/Makefile from the unmodified
 *     reference source /root/reference/stack/pico_frame.c, and
 * (2) the golden vectors in tests/golden/ (reference KATs from
 *     test/unit/unit_socket.c:418-435, test/unit/unit_icmp4.c:225-230 and
 *     RFC/rfc1071.txt:246-268, plus seeded random frames whose expected
 *     outputs were produced by oracle/_ref).
 *
 * Semantics restated (little-endian host, the reference's default build):
 *   S   = sum over i < floor(n/2) of (b[2i] | b[2i+1] << 8)  + (n odd ? b[n-1] : 0)
 *   s   = S mod 2^32            (uint32_t accumulator, no carry fold in the loop)
 *   fold s to 16 bits with end-around carry, complement, byte-swap.
 */
#include <stdint.h>
#include <stddef.h>
#include <string.h>
#include <stdlib.h>
#include <pthread.h>
#include <time.h>

#include "pico_csum_oracle.h"

/* stack/pico_frame.c:279-299 pico_checksum_adder (LE branch at :289). */
uint32_t oracle_checksum_adder(uint32_t sum, const void *data, uint32_t len)
{
    const uint8_t *p = (const uint8_t *)data;
    uint32_t i;

    if (len & 1u) {
        --len;
        sum += p[len];                      /* odd trailing byte is the LOW byte */
    }
    for (i = 0; i < len; i += 2) {
        uint16_t w;
        memcpy(&w, p + i, 2);               /* native (LE) 16-bit word, any alignment */
        sum += w;                           /* uint32 wrap, as the reference */
    }
    return sum;
}

/* stack/pico_frame.c:301-307 pico_checksum_finalize; short_be = bswap16
 * (include/pico_config.h:156-159). */
uint16_t oracle_checksum_finalize(uint32_t sum)
{
    uint16_t r;
    while (sum >> 16)
        sum = (sum & 0xFFFFu) + (sum >> 16);
    r = (uint16_t)~sum;
    return (uint16_t)((r >> 8) | (r << 8));
}

/* stack/pico_frame.c:312-318 */
uint16_t oracle_checksum(const void *buf, uint32_t len)
{
    return oracle_checksum_finalize(oracle_checksum_adder(0, buf, len));
}

/* stack/pico_frame.c:320-328 */
uint16_t oracle_dualbuffer_checksum(const void *b1, uint32_t len1, const void *b2, uint32_t len2)
{
    uint32_t sum = oracle_checksum_adder(0, b1, len1);
    sum = oracle_checksum_adder(sum, b2, len2);
    return oracle_checksum_finalize(sum);
}

/* modules/pico_ipv4.h:46-53 pseudo header {src, dst, zeros, proto, len_be}
 * summed by pico_checksum_adder, i.e. as it would be in
 * pico_tcp.c:422-446 / pico_udp.c:36-60 (the 12-byte buffer 1 of
 * pico_dualbuffer_checksum). src/dst are in network byte order as stored. */
uint32_t oracle_ipv4_pseudo_sum(const uint8_t src[4], const uint8_t dst[4], uint8_t proto, uint16_t transport_len)
{
    uint8_t ph[12];
    memcpy(ph, src, 4);
    memcpy(ph + 4, dst, 4);
    ph[8] = 0;
    ph[9] = proto;
    ph[10] = (uint8_t)(transport_len >> 8);   /* short_be(transport_len) stored LE */
    ph[11] = (uint8_t)(transport_len & 0xFF);
    return oracle_checksum_adder(0, ph, 12);
}

/* Batched restatement of the RAW path: out[i] = finalize(adder(seed_i, base+off_i, len_i)).
 * crc_off >= 0: the two bytes at off_i+crc_off are read as zero (the
 * "hdr->crc = 0" the callers do before computing: pico_ipv4.c:237,
 * pico_icmp4.c:38, pico_tcp.c:980). */
void oracle_batch_raw(const uint8_t *base, const struct pico_csum_desc *d, uint32_t n,
                      uint16_t *out, int32_t crc_off)
{
    uint32_t i;
    for (i = 0; i < n; i++) {
        const uint8_t *p = base + d[i].off;
        uint32_t len = d[i].len;
        uint32_t sum = oracle_checksum_adder(d[i].seed, p, len);
        if (crc_off >= 0 && (uint32_t)crc_off + 2u <= len) {
            uint16_t w;                     /* crc_off is even (API contract) */
            memcpy(&w, p + crc_off, 2);
            sum -= w;
        }
        out[i] = oracle_checksum_finalize(sum);
    }
}

void oracle_batch_uniform(const uint8_t *base, uint64_t stride, uint32_t len, uint32_t n,
                          uint32_t seed, uint16_t *out)
{
    uint32_t i;
    for (i = 0; i < n; i++)
        out[i] = oracle_checksum_finalize(oracle_checksum_adder(seed, base + (uint64_t)i * stride, len));
}

/*
 * Fused IPv4 RX/TX restatement, one frame per descriptor.  desc.off points at
 * the IPv4 header (f->net_hdr); desc.len = bytes available from net_hdr to the
 * end of the frame buffer (f->buffer_len - (f->net_hdr - f->buffer)).
 *
 * RX (flags & ORACLE_IPV4_TX == 0):
 *   lengths + feasibility bound   pico_ipv4_process_in  modules/pico_ipv4.c:381-405
 *   header check                  pico_ipv4_crc_check   modules/pico_ipv4.c:243-257
 *   transport check               pico_transport_crc_check stack/pico_socket.c:1916-1968
 *     TCP: pico_tcp_checksum_ipv4 modules/pico_tcp.c:422-446 (pseudo from IP hdr, f->sock NULL)
 *     UDP: only when the stored crc != 0 (pico_socket.c:1941), pico_udp.c:36-60
 *   out_net = pico_checksum(hdr, net_len)                        (0 when valid)
 *   out_l4  = transport checksum with the IPv4 pseudo header       (0 when valid;
 *             0 when the reference computes none)
 *   verdict = PICO_CSUM_V_ACCEPT, or the OR of the failure bits.
 *   Frames where the reference would read past desc.len (header or
 *   transport beyond the buffer: reference UB) are PICO_CSUM_V_MALFORMED.
 * TX (ORACLE_IPV4_TX): the header is complete; crc fields read as zero
 *   (hdr->crc = 0 at pico_ipv4.c:237, pico_tcp.c:980, pico_icmp4.c:38); out_*
 *   are the values the reference stores with short_be() (pico_ipv4.c:238,
 *   pico_tcp.c:981, pico_icmp4.c:39).  UDP over IPv4 sends crc 0
 *   (pico_udp.c:123); other protocols get none.  TCP needs a 20-byte and ICMP
 *   an 8-byte header inside transport_len, else MALFORMED.
 */
void oracle_batch_ipv4(const uint8_t *base, const struct pico_csum_desc *d, uint32_t n,
                       uint16_t *out_net, uint16_t *out_l4, uint8_t *verdict, uint32_t flags)
{
    uint32_t i;
    int tx = (flags & ORACLE_IPV4_TX) != 0;
    for (i = 0; i < n; i++) {
        const uint8_t *h = base + d[i].off;
        const uint8_t *t;
        uint32_t avail = d[i].len;
        uint32_t option_len = 0, net_len, s;
        uint16_t tot, transport_len, max_allowed;
        uint16_t net_cs, l4_cs = 0;
        uint8_t proto, v = 0;

        out_net[i] = 0; out_l4[i] = 0; verdict[i] = PICO_CSUM_V_MALFORMED;
        if (avail < 20)
            continue;
        if ((h[0] & 0x0F) > 5)
            option_len = 4u * ((h[0] & 0x0Fu) - 5u);
        net_len = 20u + option_len;
        proto = h[9];
        tot = (uint16_t)((h[2] << 8) | h[3]);
        transport_len = (uint16_t)(tot - 20u - option_len);    /* uint16 wrap as :395 */
        max_allowed = (uint16_t)(avail - 20u);                 /* :386 */
        if (net_len > avail)
            continue;
        if (!tx && transport_len > max_allowed)                /* :402-405 discard */
            continue;
        if (net_len + (uint32_t)transport_len > avail)         /* reference would overread */
            continue;
        t = h + net_len;

        s = oracle_checksum_adder(0, h, net_len);
        if (tx) s -= (uint32_t)(h[10] | (h[11] << 8));
        net_cs = oracle_checksum_finalize(s);
        if (!tx && net_cs != 0)
            v |= PICO_CSUM_V_NET_BAD;

        if (!tx) {
            if (proto == 6 || proto == 17) {
                int check = 1;
                if (proto == 17) {
                    if (net_len + 8u > avail) { v |= PICO_CSUM_V_MALFORMED; check = 0; }
                    else if (t[6] == 0 && t[7] == 0) check = 0;
                }
                if (check) {
                    s = oracle_ipv4_pseudo_sum(h + 12, h + 16, proto, transport_len);
                    l4_cs = oracle_checksum_finalize(oracle_checksum_adder(s, t, transport_len));
                    if (l4_cs != 0)
                        v |= PICO_CSUM_V_L4_BAD;
                }
            }
        } else {
            if (proto == 6) {
                if (transport_len < 20) { v |= PICO_CSUM_V_MALFORMED; }
                else {
                    s = oracle_ipv4_pseudo_sum(h + 12, h + 16, proto, transport_len);
                    s = oracle_checksum_adder(s, t, transport_len);
                    s -= (uint32_t)(t[16] | (t[17] << 8));
                    l4_cs = oracle_checksum_finalize(s);
                }
            } else if (proto == 1) {
                if (transport_len < 8) { v |= PICO_CSUM_V_MALFORMED; }
                else {
                    s = oracle_checksum_adder(0, t, transport_len);
                    s -= (uint32_t)(t[2] | (t[3] << 8));
                    l4_cs = oracle_checksum_finalize(s);
                }
            }
        }
        out_net[i] = net_cs;
        out_l4[i] = l4_cs;
        verdict[i] = (uint8_t)(v == 0 ? PICO_CSUM_V_ACCEPT : v);
    }
}

/* modules/pico_ipv6.h:46-53 struct pico_ipv6_pseudo_hdr {src[16], dst[16], len (32-bit BE),
 * zero[3], nxthdr}, summed by pico_checksum_adder as pico_tcp_checksum_ipv6
 * (pico_tcp.c:449-475), pico_udp_checksum_ipv6 (pico_udp.c:63-92) and
 * pico_icmp6_checksum (pico_icmp6.c:38-55) pass it as buffer 1. */
uint32_t oracle_ipv6_pseudo_sum(const uint8_t src[16], const uint8_t dst[16], uint8_t nxthdr, uint32_t transport_len)
{
    uint8_t ph[40];
    memcpy(ph, src, 16);
    memcpy(ph + 16, dst, 16);
    ph[32] = (uint8_t)(transport_len >> 24);
    ph[33] = (uint8_t)(transport_len >> 16);
    ph[34] = (uint8_t)(transport_len >> 8);
    ph[35] = (uint8_t)transport_len;
    ph[36] = ph[37] = ph[38] = 0;
    ph[39] = nxthdr;
    return oracle_checksum_adder(0, ph, 40);
}

static int icmp6_checked_type(uint8_t t)
{
    /* ND: pico_ipv6_nd.c:595 (types 133-137); MLD: pico_mld.c:415 (130-132, 143) */
    return (t >= 133 && t <= 137) || (t >= 130 && t <= 132) || t == 143;
}

/*
 * Fused IPv6 transport restatement, one datagram per descriptor.  desc.off ->
 * IPv6 header; desc.len = bytes available; desc.seed = f->net_len | proto << 16
 * as pico_ipv6_extension_headers (modules/pico_ipv6.c:707-800) leaves them
 * (seed 0: net_len 40, proto = hdr->nxthdr).
 *   transport_len = (uint16)(payload_len - (net_len - 40))     pico_ipv6.c:790
 * RX: pico_transport_crc_check (stack/pico_socket.c:1916-1968): TCP always (any
 *   length), UDP when the stored crc (t[6..7], inside the buffer) != 0; ICMPv6:
 *   pico_icmp6_checksum, a verdict only for the ND / MLD types the reference
 *   checks (type byte t[0] inside the buffer).  Other protocols: none.
 *   out = the checksum (0 = valid), 0 when none is computed.
 * TX: crc field read as zero (TCP pico_tcp.c:980, ICMPv6 pico_ipv6.c:1337, UDP
 *   crc already 0 from pico_udp_push :123 when pico_ipv6.c:1345 computes it);
 *   TCP needs 20, UDP 8, ICMPv6 4 transport bytes.  Other protocols: none.
 * MALFORMED: avail < 40, net_len < 40 or past avail, transport past avail, or a
 *   field the reference reads lying past avail.
 * ORACLE_REF_DISPATCH (RX): TCP / UDP frames are checked as pico_transport_crc_check
 *   (stack/pico_socket.c:1919-1958) literally does: `switch (net_hdr->proto)` through a
 *   struct pico_ipv4_hdr cast -- for IPv6 the header's byte 9 (source address byte 1):
 *   6 -> pico_tcp_checksum -> pico_tcp_checksum_ipv6 (pico_tcp.c:492-505, TCP in the pseudo
 *   header), 17 -> when t[6..7] != 0, pico_udp_checksum_ipv6 (UDP in the pseudo header),
 *   else no check.  The transport must hold t[6..7] whenever they are read.
 */
void oracle_batch_ipv6(const uint8_t *base, const struct pico_csum_desc *d, uint32_t n,
                       uint16_t *out_l4, uint8_t *verdict, uint32_t flags)
{
    uint32_t i;
    int tx = (flags & ORACLE_IPV4_TX) != 0;
    int refd = !tx && (flags & ORACLE_REF_DISPATCH) != 0;
    for (i = 0; i < n; i++) {
        const uint8_t *h = base + d[i].off;
        const uint8_t *t;
        uint32_t avail = d[i].len, net_len, plen, s;
        uint16_t tl;
        uint8_t proto, v = 0;
        uint16_t l4 = 0;

        out_l4[i] = 0;
        verdict[i] = PICO_CSUM_V_MALFORMED;
        if (avail < 40)
            continue;
        net_len = d[i].seed & 0xFFFFu;
        proto = (uint8_t)(d[i].seed >> 16);
        if (d[i].seed == 0) {
            net_len = 40;
            proto = h[6];
        }
        plen = (uint32_t)((h[4] << 8) | h[5]);
        if (net_len < 40 || net_len > avail)
            continue;
        tl = (uint16_t)(plen - (net_len - 40u));               /* pico_ipv6.c:790 */
        if (net_len + (uint32_t)tl > avail)
            continue;
        t = h + net_len;
        s = oracle_ipv6_pseudo_sum(h + 8, h + 24, proto, tl);
        if (refd && (proto == 6 || proto == 17)) {
            uint8_t b9 = h[9];
            if (proto == 17 || b9 == 17) {
                if (net_len + 8u > avail) continue;
            }
            if (b9 == 6 || (b9 == 17 && (t[6] || t[7]))) {
                s = oracle_ipv6_pseudo_sum(h + 8, h + 24, b9, tl);
                l4 = oracle_checksum_finalize(oracle_checksum_adder(s, t, tl));
                if (l4) v |= PICO_CSUM_V_L4_BAD;
            }
        } else if (!tx) {
            if (proto == 6) {
                l4 = oracle_checksum_finalize(oracle_checksum_adder(s, t, tl));
                if (l4) v |= PICO_CSUM_V_L4_BAD;
            } else if (proto == 17) {
                if (net_len + 8u > avail) continue;
                if (t[6] || t[7]) {
                    l4 = oracle_checksum_finalize(oracle_checksum_adder(s, t, tl));
                    if (l4) v |= PICO_CSUM_V_L4_BAD;
                }
            } else if (proto == 58) {
                if (net_len + 1u > avail) continue;
                l4 = oracle_checksum_finalize(oracle_checksum_adder(s, t, tl));
                if (l4 && icmp6_checked_type(t[0])) v |= PICO_CSUM_V_L4_BAD;
            }
        } else {
            int xoff = proto == 6 ? 16 : proto == 17 ? 6 : proto == 58 ? 2 : -1;
            uint32_t need = proto == 6 ? 20u : proto == 17 ? 8u : 4u;
            if (xoff >= 0) {
                if (tl < need) continue;
                s = oracle_checksum_adder(s, t, tl);
                s -= (uint32_t)(t[xoff] | (t[xoff + 1] << 8));
                l4 = oracle_checksum_finalize(s);
            }
        }
        out_l4[i] = l4;
        verdict[i] = (uint8_t)(v == 0 ? PICO_CSUM_V_ACCEPT : v);
    }
}

/*
 * Ethernet front end of the fused RX verify (SURVEY.md 8f row 1 "Ethernet -> IPv4 ..."),
 * one frame per descriptor: desc.off -> the Ethernet header (f->datalink_hdr), desc.len =
 * frame bytes, desc.seed = the IPv6 net_len | proto << 16 (IPv6 frames only, as for
 * oracle_batch_ipv6).
 *   RX destination filter   pico_ethernet_receive  modules/pico_ethernet.c:215-235
 *     (own MAC, 01:00:5e IPv4 multicast, 33:33 IPv6 multicast, broadcast; mac == NULL:
 *     no filter; never on TX) -> PICO_CSUM_V_DROP_L2
 *   ethertype dispatch      pico_eth_receive       modules/pico_ethernet.c:180-203
 *     0x0806 ARP -> PICO_CSUM_V_ARP (pico_arp_receive: no checksum)
 *     0x0800 -> IS_IPV4 (pico_ethernet.c:143-150, else DROP_L2) -> oracle_batch_ipv4 on
 *               (off + 14, len - 14)
 *     0x86DD -> IS_IPV6 (:162-176, else DROP_L2) -> oracle_batch_ipv6, verdict | V_IPV6
 *     other  -> DROP_L2 (:201-202)
 *   A frame shorter than the 14-byte header, or with no byte behind it to read the IP
 *   version from, is MALFORMED.
 */
void oracle_batch_eth(const uint8_t *base, const struct pico_csum_desc *d, uint32_t n, const uint8_t *mac,
                      uint16_t *out_net, uint16_t *out_l4, uint8_t *verdict, uint32_t flags)
{
    static const uint8_t mc4[3] = {0x01, 0x00, 0x5e}, mc6[2] = {0x33, 0x33},
                         all[6] = {0xff, 0xff, 0xff, 0xff, 0xff, 0xff};
    uint32_t i;
    int tx = (flags & ORACLE_IPV4_TX) != 0;
    for (i = 0; i < n; i++) {
        const uint8_t *e = base + d[i].off;
        struct pico_csum_desc sub;
        uint16_t etype;
        out_net[i] = 0;
        out_l4[i] = 0;
        verdict[i] = PICO_CSUM_V_MALFORMED;
        if (d[i].len < 14)
            continue;
        if (!tx && mac && memcmp(e, mac, 6) != 0 && memcmp(e, mc4, 3) != 0 && memcmp(e, mc6, 2) != 0 &&
            memcmp(e, all, 6) != 0) {
            verdict[i] = PICO_CSUM_V_DROP_L2;
            continue;
        }
        etype = (uint16_t)((e[12] << 8) | e[13]);
        if (etype == 0x0806) {
            verdict[i] = PICO_CSUM_V_ARP;
            continue;
        }
        if (etype != 0x0800 && etype != 0x86DD) {
            verdict[i] = PICO_CSUM_V_DROP_L2;
            continue;
        }
        if (d[i].len < 15)
            continue;
        if ((e[14] & 0xF0) != (etype == 0x0800 ? 0x40 : 0x60)) {
            verdict[i] = PICO_CSUM_V_DROP_L2;
            continue;
        }
        sub.off = d[i].off + 14;
        sub.len = d[i].len - 14;
        sub.seed = d[i].seed;
        if (etype == 0x0800) {
            sub.seed = 0;
            oracle_batch_ipv4(base, &sub, 1, out_net + i, out_l4 + i, verdict + i, flags);
        } else {
            oracle_batch_ipv6(base, &sub, 1, out_l4 + i, verdict + i, flags);
            verdict[i] |= PICO_CSUM_V_IPV6;
        }
    }
}

/*
 * IPv4 fragment reassembly with the transport check of the reassembled datagram
 * (SURVEY.md 8f row 4).  Fragments arrive as pico_ipv4_process_in hands them to
 * pico_ipv4_process_frag (modules/pico_ipv4.c:381-450: f->transport_len = tot - net_len,
 * f->frag = short_be(hdr->frag)); group g = fragments grp[2g] .. grp[2g] + grp[2g+1] - 1 of
 * one datagram (src, dst, id matched by the stack, pico_fragments.c:499-568), in arrival
 * order.  Per group:
 *   tree order     pico_ipv4_frag_compare (pico_fragments.c:129-139): by offset
 *                  IP4_FRAG_OFF = (frag & 0x1FFF) << 3; pico_tree_insert rejects a second
 *                  fragment with the same offset, so the earlier arrival is kept
 *   completeness   pico_fragments_check_complete (:216-239): offsets contiguous from 0
 *                  (offset == sum of the previous transport_len), up to the first
 *                  fragment without PICO_IPV4_MOREFRAG; len = that sum
 *   gather         pico_fragments_reassemble (:304-358): PICO_SIZE_IP4HDR (20) header
 *                  bytes of the first fragment, then every fragment's transport bytes
 *   transport      pico_transport_crc_check (stack/pico_socket.c:1916-1968) with
 *                  net_hdr->proto of the copied header: TCP always, UDP when its crc != 0;
 *                  pseudo header from the copied header, transport_len = len
 * out_len[g] = len (0 when not reassembled), out_l4[g] = the checksum (0 = valid; 0 when
 * none), verdict[g] = ACCEPT / L4_BAD, or MALFORMED when not reassembled: incomplete, a
 * fragment behind the completing one (the reference's copy loop, :339-345, would write
 * past its 20 + len byte buffer), 20 + len > 65535 (its (uint16_t) allocation size wraps),
 * a fragment whose header or transport lies past desc.len, an empty group or one of more
 * than 512 fragments (the API's limit), or an output
 * region (out_desc[g].len) shorter than 20 + len or not 4-byte aligned (the API's contract).
 */
void oracle_ipv4_reassemble(const uint8_t *base, const struct pico_csum_desc *d, uint32_t nd, const uint32_t *grp,
                            uint32_t ng, uint8_t *out, const struct pico_csum_desc *od, uint32_t *out_len, uint16_t *out_l4,
                            uint8_t *verdict)
{
    uint32_t g;
    for (g = 0; g < ng; g++) {
        uint32_t first = grp[2 * g], cnt = grp[2 * g + 1], i, k, m = 0, len = 0, bad = 0, e = 0, done = 0;
        uint32_t na = cnt && cnt <= 512 ? cnt : 1;
        uint32_t *ord = (uint32_t *)malloc(sizeof(uint32_t) * na);
        uint32_t *foff = (uint32_t *)malloc(sizeof(uint32_t) * na);
        uint32_t *tl = (uint32_t *)malloc(sizeof(uint32_t) * na);
        uint32_t *hlen = (uint32_t *)malloc(sizeof(uint32_t) * na);
        uint8_t *mf = (uint8_t *)malloc(na);
        out_len[g] = 0;
        out_l4[g] = 0;
        verdict[g] = PICO_CSUM_V_MALFORMED;
        if (cnt == 0 || cnt > 512 || first > nd || cnt > nd - first)   /* 512: the device API's limit */
            bad = 1;
        for (i = 0; i < cnt && !bad; i++) {
            const struct pico_csum_desc *f = &d[first + i];
            const uint8_t *h = base + f->off;
            uint32_t ihl, frag;
            if (f->len < 20) { bad = 1; break; }
            ihl = h[0] & 0x0Fu;
            hlen[i] = 20u + (ihl > 5u ? 4u * (ihl - 5u) : 0u);
            tl[i] = (uint16_t)(((h[2] << 8) | h[3]) - hlen[i]);
            frag = (uint32_t)((h[6] << 8) | h[7]);
            foff[i] = (frag & 0x1FFFu) << 3;
            mf[i] = (frag & 0x2000u) != 0;
            if (hlen[i] + tl[i] > f->len) bad = 1;
        }
        /* tree: insertion by offset, a repeated offset keeps the earlier arrival */
        for (i = 0; i < cnt && !bad; i++) {
            uint32_t pos = 0, dup = 0;
            for (k = 0; k < m; k++) {
                if (foff[ord[k]] == foff[i]) { dup = 1; break; }
                if (foff[ord[k]] < foff[i]) pos = k + 1;
            }
            if (dup) continue;
            memmove(ord + pos + 1, ord + pos, sizeof(uint32_t) * (m - pos));
            ord[pos] = i;
            m++;
        }
        for (k = 0; k < m && !bad; k++) {
            if (foff[ord[k]] != len) break;
            len += tl[ord[k]];
            if (!mf[ord[k]]) { e = k; done = 1; break; }
        }
        if (!bad && done && e + 1 == m && 20u + len <= 0xFFFFu && od[g].len >= 20u + len && (od[g].off & 3u) == 0) {
            uint8_t *dst = out + od[g].off;
            const uint8_t *h0 = base + d[first + ord[0]].off;
            uint32_t at = 20, s;
            uint8_t proto = h0[9];
            memcpy(dst, h0, 20);
            for (k = 0; k < m; k++) {
                const uint8_t *src = base + d[first + ord[k]].off + hlen[ord[k]];
                memcpy(dst + at, src, tl[ord[k]]);
                at += tl[ord[k]];
            }
            out_len[g] = len;
            verdict[g] = PICO_CSUM_V_ACCEPT;
            if (proto == 6 || (proto == 17 && len >= 8 && (dst[20 + 6] || dst[20 + 7]))) {
                s = oracle_ipv4_pseudo_sum(dst + 12, dst + 16, proto, (uint16_t)len);
                out_l4[g] = oracle_checksum_finalize(oracle_checksum_adder(s, dst + 20, len));
                if (out_l4[g]) verdict[g] = PICO_CSUM_V_L4_BAD;
            }
        }
        free(ord); free(foff); free(tl); free(hlen); free(mf);
    }
}

/* modules/pico_ipv4.c:1547-1556 (pico_ipv4_forward): hdr->ttl = (uint8_t)(hdr->ttl - 1);
 * if (hdr->ttl < 1) -> expired, dropped; else hdr->crc++ (uint16_t field, native LE
 * increment of the stored big-endian checksum).  In place on base; verdict per
 * datagram: ACCEPT (forwarded), EXPIRED, MALFORMED (< 20 bytes: untouched). */
void oracle_batch_ipv4_forward(uint8_t *base, const struct pico_csum_desc *d, uint32_t n, uint8_t *verdict)
{
    uint32_t i;
    for (i = 0; i < n; i++) {
        uint8_t *h = base + d[i].off;
        uint16_t crc;
        if (d[i].len < 20) {
            verdict[i] = PICO_CSUM_V_MALFORMED;
            continue;
        }
        h[8] = (uint8_t)(h[8] - 1);
        if (h[8] < 1) {
            verdict[i] = PICO_CSUM_V_EXPIRED;
            continue;
        }
        memcpy(&crc, h + 10, 2);
        crc++;
        memcpy(h + 10, &crc, 2);
        verdict[i] = PICO_CSUM_V_ACCEPT;
    }
}

/* ---- multi-threaded CPU baseline driver (bench.py cpu_baseline leg) ---- */

struct mt_job {
    const uint8_t *base;
    uint64_t stride;
    uint32_t len, first, count;
    uint16_t *out;
    oracle_checksum_fn fn;
};

static void *mt_worker(void *arg)
{
    struct mt_job *j = (struct mt_job *)arg;
    uint32_t i;
    for (i = 0; i < j->count; i++) {
        uint64_t f = (uint64_t)j->first + i;
        j->out[f] = j->fn((void *)(j->base + f * j->stride), j->len);
    }
    return NULL;
}

/* Runs fn (oracle_checksum, or the reference's own pico_checksum from
 * oracle/_ref) over n uniform frames on nthreads pthreads, contiguous frame
 * ranges per thread.  Returns wall seconds. */
double oracle_uniform_mt(oracle_checksum_fn fn, const uint8_t *base, uint64_t stride, uint32_t len,
                         uint32_t n, uint16_t *out, uint32_t nthreads)
{
    struct mt_job jobs[256];
    pthread_t th[256];
    struct timespec t0, t1;
    uint32_t t, per, first = 0;

    if (fn == NULL) fn = (oracle_checksum_fn)oracle_checksum;
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    per = (n + nthreads - 1) / nthreads;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    for (t = 0; t < nthreads; t++) {
        uint32_t c = (first + per <= n) ? per : (n > first ? n - first : 0);
        jobs[t].base = base; jobs[t].stride = stride; jobs[t].len = len;
        jobs[t].first = first; jobs[t].count = c; jobs[t].out = out; jobs[t].fn = fn;
        first += c;
        if (nthreads == 1)
            mt_worker(&jobs[t]);
        else
            pthread_create(&th[t], NULL, mt_worker, &jobs[t]);
    }
    if (nthreads > 1)
        for (t = 0; t < nthreads; t++)
            pthread_join(th[t], NULL);
    clock_gettime(CLOCK_MONOTONIC, &t1);
    return (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
}

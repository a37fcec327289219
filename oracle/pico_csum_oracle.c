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
 * RX (flags & ORACLE_IPV4_TX == 0): pico_ipv4_process_in (modules/pico_ipv4.c:381-456) up to
 * the hand-off, then pico_transport_crc_check (stack/pico_socket.c:1916-1968).  The verdict is
 * the reference's FIRST discard reason, in its order:
 *   1. lengths: net_len = 20 + 4 (IHL - 5) (options only when IHL > 5, :394-396),
 *      transport_len = (uint16)(tot - net_len) (:399); transport_len > max_allowed =
 *      (uint16)(avail - 20) is discarded (:386, :405-408)                       -> MALFORMED
 *      (also MALFORMED: the header or the transport past desc.len, where the reference would
 *      read past its buffer)
 *   2. pico_ipv4_crc_check over net_len bytes (:420-422, :243-257)               -> NET_BAD
 *   3. pico_ipv4_is_valid_src (:425-428, :210-229): 255.255.255.255, a multicast source
 *      (first byte 0xE0-0xFE, :187-194), a loopback source (127/8) from a non-"loop" device
 *                                                                                 -> MALFORMED
 *      (the link-directed broadcasts of pico_ipv4_is_broadcast, :1620-1633, are the stack's
 *      link table: not decidable from the frame, left to the stack)
 *   4. the evil bit (frag & 0x8000, RFC 3514, :431-435)                           -> MALFORMED
 *   5. IHL < 5 (:438-443)                                                         -> MALFORMED
 *   6. MF or a fragment offset (frag & 0x3FFF, :446-455): handed to pico_ipv4_process_frag,
 *      no transport check on the fragment                                         -> FRAG
 *   7. transport check: TCP always (pico_tcp_checksum_ipv4, modules/pico_tcp.c:422-446, pseudo
 *      header from the IP header, f->sock NULL); UDP only when its stored crc != 0
 *      (pico_socket.c:1941, pico_udp.c:36-60; a UDP transport shorter than 8 bytes would be
 *      read past: MALFORMED)                                                      -> L4_BAD
 *   otherwise ACCEPT.
 *   out_net = pico_checksum(hdr, net_len) (0 when valid) whenever the lengths pass;
 *   out_l4  = the transport checksum (0 when valid; 0 when the reference computes none).
 * TX (ORACLE_IPV4_TX): the header is complete; crc fields read as zero
 *   (hdr->crc = 0 at pico_ipv4.c:237, pico_tcp.c:980, pico_icmp4.c:38); out_*
 *   are the values the reference stores with short_be() (pico_ipv4.c:238,
 *   pico_tcp.c:981, pico_icmp4.c:39).  UDP over IPv4 sends crc 0
 *   (pico_udp.c:123); other protocols get none.  TCP needs a 20-byte and ICMP
 *   an 8-byte header inside transport_len, else MALFORMED.  A fragment (MF or an offset) gets
 *   its own header checksum only (pico_ipv4_frame_push :1079 per fragment; the transport
 *   checksum covers the whole datagram and was set before fragmentation, :1470-1500) -> FRAG.
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
        uint16_t tot, transport_len, max_allowed, frag;
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
        frag = (uint16_t)((h[6] << 8) | h[7]);                 /* f->frag = short_be(hdr->frag), :402 */
        transport_len = (uint16_t)(tot - 20u - option_len);    /* uint16 wrap as :399 */
        max_allowed = (uint16_t)(avail - 20u);                 /* :386 */
        if (net_len > avail)
            continue;
        if (!tx && transport_len > max_allowed)                /* :405-408 discard */
            continue;
        if (net_len + (uint32_t)transport_len > avail)         /* reference would overread */
            continue;
        t = h + net_len;

        s = oracle_checksum_adder(0, h, net_len);
        if (tx) s -= (uint32_t)(h[10] | (h[11] << 8));
        net_cs = oracle_checksum_finalize(s);
        out_net[i] = net_cs;

        if (!tx) {
            if (net_cs != 0)
                v = PICO_CSUM_V_NET_BAD;                                        /* :420-422 */
            else if ((h[12] == 0xFF && h[13] == 0xFF && h[14] == 0xFF && h[15] == 0xFF) ||
                     (h[12] != 0xFF && (h[12] & 0xE0) == 0xE0) || h[12] == 0x7F)
                v = PICO_CSUM_V_MALFORMED;                                      /* :425-428 */
            else if (frag & 0x8000u)
                v = PICO_CSUM_V_MALFORMED;                                      /* :431-435 */
            else if ((h[0] & 0x0F) < 5)
                v = PICO_CSUM_V_MALFORMED;                                      /* :438-443 */
            else if (frag & 0x3FFFu)
                v = PICO_CSUM_V_FRAG;                                           /* :446-455 */
            else if (proto == 6 || proto == 17) {
                int check = 1;
                if (proto == 17) {
                    if (net_len + 8u > avail) { v = PICO_CSUM_V_MALFORMED; check = 0; }
                    else if (t[6] == 0 && t[7] == 0) check = 0;
                }
                if (check) {
                    s = oracle_ipv4_pseudo_sum(h + 12, h + 16, proto, transport_len);
                    l4_cs = oracle_checksum_finalize(oracle_checksum_adder(s, t, transport_len));
                    if (l4_cs != 0)
                        v = PICO_CSUM_V_L4_BAD;
                }
            }
        } else if (frag & 0x3FFFu) {
            v = PICO_CSUM_V_FRAG;
        } else {
            if (proto == 6) {
                if (transport_len < 20) { v = PICO_CSUM_V_MALFORMED; }
                else {
                    s = oracle_ipv4_pseudo_sum(h + 12, h + 16, proto, transport_len);
                    s = oracle_checksum_adder(s, t, transport_len);
                    s -= (uint32_t)(t[16] | (t[17] << 8));
                    l4_cs = oracle_checksum_finalize(s);
                }
            } else if (proto == 1) {
                if (transport_len < 8) { v = PICO_CSUM_V_MALFORMED; }
                else {
                    s = oracle_checksum_adder(0, t, transport_len);
                    s -= (uint32_t)(t[2] | (t[3] << 8));
                    l4_cs = oracle_checksum_finalize(s);
                }
            }
        }
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

/* The walk reads byte k of the datagram only when k < avail; a read past it is where the
 * reference would read past its buffer (reported as ORACLE_WALK_BAD). */
#define WALK_BYTE(k, dst)                          \
    do {                                           \
        if ((uint32_t)(k) >= avail)                \
            return ORACLE_WALK_BAD;                \
        (dst) = h[(uint32_t)(k)];                  \
    } while (0)

/* pico_ipv6_process_hopbyhop (modules/pico_ipv6.c:525-582) on the header at byte e:
 * 1 / 0 = must_align, -1 = discard, ORACLE_WALK_BAD (-1 is taken) -> -2.  option = e + 2,
 * len = (uint8)HBH_LEN (pico_ipv6.h:30); Pad1 advances 1 byte, PadN / router alert / an
 * unknown option with action "skip" advance (uint8)(opt[1] + 2) -- 0 when opt[1] = 254, and
 * the reference's loop then never ends; a router alert with data length 2 (MLD) clears
 * must_align; any other action (0x40 / 0x80 / 0xC0) discards. */
static int walk_hopbyhop(const uint8_t *h, uint32_t avail, uint32_t e)
{
    uint8_t b1, len, type, olen, optlen;
    uint32_t opt = e + 2;
    int must_align = 1;
    if (e + 1 >= avail) return -2;
    b1 = h[e + 1];
    len = (uint8_t)(((b1 + 1) << 3) - 2);
    while (len) {
        if (opt >= avail) return -2;
        type = h[opt];
        if (type == 0) {                        /* PICO_IPV6_EXTHDR_OPT_PAD1 */
            opt++;
            len--;
            continue;
        }
        if (opt + 1 >= avail) return -2;
        olen = h[opt + 1];
        optlen = (uint8_t)(olen + 2);
        if (type == 5) {                        /* PICO_IPV6_EXTHDR_OPT_ROUTER_ALERT */
            if (olen == 2) must_align = 0;
        } else if (type != 1 && (type & 0xC0) != 0) {
            return -1;                          /* discard (+ a parameter problem for 0x80 / 0xC0) */
        }
        if (optlen == 0) return -2;             /* the reference loops forever */
        opt += optlen;
        len = (uint8_t)(len - optlen);
    }
    return must_align;
}

/* pico_ipv6_process_destopt (modules/pico_ipv6.c:610-657): 0 = pass, -1 = discard, -2 = past
 * the frame / endless.  Every option -- Pad1 included -- advances (uint8)(opt[1] + 2). */
static int walk_destopt(const uint8_t *h, uint32_t avail, uint32_t e)
{
    uint8_t b1, len, type, optlen;
    uint32_t opt = e + 2;
    if (e + 1 >= avail) return -2;
    b1 = h[e + 1];
    len = (uint8_t)(((b1 + 1) << 3) - 2);
    while (len) {
        if (opt + 1 >= avail) return -2;
        type = h[opt];
        optlen = (uint8_t)(h[opt + 1] + 2);
        if (type != 0 && type != 1 && type != 201 && (type & 0xC0) != 0)
            return -1;
        if (optlen == 0) return -2;
        opt += optlen;
        len = (uint8_t)(len - optlen);
    }
    return 0;
}

/*
 * pico_ipv6_extension_headers (modules/pico_ipv6.c:707-809) with the sequence check before it
 * (pico_ipv6_check_headers_sequence, :659-694), on the IPv6 datagram at h (avail bytes).
 *   sequence check: from the fixed header's next header, walk DESTOPT / ROUTING / HOPBYHOP /
 *     ESP / AUTH by (uint8)IPV6_OPTLEN(len) -- wraps to 0 for len >= 31 --, FRAG by 8, stop at
 *     NONE / TCP / UDP / ICMPv6; any other value discards (parameter problem, :685-688)
 *   walk: f->net_len (uint16) from 40; HOPBYHOP only right behind the fixed header (:727-734);
 *     ROUTING with segments left and a type other than 2 discards (:585-606); FRAG sets
 *     f->frag (and with M set a payload length not a multiple of 8 discards, :750-761);
 *     DESTOPT sets must_align; ESP / AUTH / NONE end the walk with no transport (discarded by
 *     pico_ipv6_process_in, :855-859); at TCP / UDP / ICMPv6, must_align with a payload length
 *     not a multiple of 8 discards (:696-705, :783-788), else the transport is reached: behind
 *     a fragment header the datagram goes to pico_ipv6_process_frag (:791-795), otherwise it
 *     is delivered with that protocol and net_len.
 * Endless loops of the reference (a zero-length step that keeps revisiting one header), a
 * chain whose f->net_len passes 0xFFFF (the uint16 wraps and the walk starts over near the
 * fixed header) and reads past avail return ORACLE_WALK_BAD.
 */
int oracle_ipv6_walk(const uint8_t *h, uint32_t avail, uint32_t *net_len_out, uint8_t *proto_out)
{
    uint16_t om;
    return oracle_ipv6_walk_frag(h, avail, net_len_out, proto_out, &om);
}

/* oracle_ipv6_walk, also returning f->frag (the last fragment header's offset / M field, :754) */
int oracle_ipv6_walk_frag(const uint8_t *h, uint32_t avail, uint32_t *net_len_out, uint8_t *proto_out,
                          uint16_t *frag_out)
{
    uint32_t plen, ptr, iter, cur_nexthdr;
    uint16_t net_len;
    uint8_t nx, b;
    int must_align = 0, frag = 0;

    if (avail < 40) return ORACLE_WALK_BAD;
    plen = (uint32_t)((h[4] << 8) | h[5]);
    /* sequence check: each step moves >= 8 bytes, or 0 (a wrapped length) and then the next
     * step reads the same header again: at most 2 steps per 8 bytes before a read passes avail */
    ptr = 40;
    nx = h[6];
    for (iter = 0;; iter++) {
        uint8_t optlen;
        if (iter > 2u * (avail / 8u) + 8u) return ORACLE_WALK_BAD;
        if (nx == 0 || nx == 43 || nx == 60 || nx == 50 || nx == 51) {
            WALK_BYTE(ptr + 1, b);
            optlen = (uint8_t)((b + 1) << 3);
        } else if (nx == 44) {
            optlen = 8;
        } else if (nx == 59 || nx == 6 || nx == 17 || nx == 58) {
            break;
        } else {
            return ORACLE_WALK_DROP;
        }
        WALK_BYTE(ptr, nx);
        ptr += optlen;
    }
    /* the walk: each step moves f->net_len by >= 8 (uint16 arithmetic) */
    net_len = 40;
    ptr = 40;
    cur_nexthdr = 6;
    nx = h[6];
    for (iter = 0;; iter++) {
        uint32_t e = net_len;
        uint16_t cur_optlen = 0;
        int r;
        if (iter > avail / 8u + 8u) return ORACLE_WALK_BAD;   /* never: each step moves >= 8 bytes */
        switch (nx) {
        case 0:                                               /* HOPBYHOP */
            if (cur_nexthdr != 6) return ORACLE_WALK_DROP;
            WALK_BYTE(e + 1, b);
            cur_optlen = (uint16_t)((b + 1) << 3);
            if (net_len + cur_optlen > 0xFFFFu) return ORACLE_WALK_BAD;   /* uint16 net_len wraps */
            net_len = (uint16_t)(net_len + cur_optlen);
            r = walk_hopbyhop(h, avail, e);
            if (r == -2) return ORACLE_WALK_BAD;
            if (r < 0) return ORACLE_WALK_DROP;
            must_align = r;
            break;
        case 43: {                                            /* ROUTING */
            uint8_t type, segleft;
            WALK_BYTE(e + 1, b);
            cur_optlen = (uint16_t)((b + 1) << 3);
            if (net_len + cur_optlen > 0xFFFFu) return ORACLE_WALK_BAD;
            net_len = (uint16_t)(net_len + cur_optlen);
            WALK_BYTE(e + 3, segleft);
            if (segleft != 0) {
                WALK_BYTE(e + 2, type);
                if (type != 2) return ORACLE_WALK_DROP;
            }
            break;
        }
        case 44: {                                            /* FRAG */
            uint8_t om0, om1;
            cur_optlen = 8;
            if (net_len + 8u > 0xFFFFu) return ORACLE_WALK_BAD;
            net_len = (uint16_t)(net_len + 8u);
            WALK_BYTE(e + 2, om0);
            WALK_BYTE(e + 3, om1);
            *frag_out = (uint16_t)((om0 << 8) + om1);         /* f->frag, :754 (M = bit 0) */
            frag = 1;
            if ((om1 & 1u) && (plen % 8u) != 0) return ORACLE_WALK_DROP;
            break;
        }
        case 60:                                              /* DESTOPT */
            WALK_BYTE(e + 1, b);
            cur_optlen = (uint16_t)((b + 1) << 3);
            if (net_len + cur_optlen > 0xFFFFu) return ORACLE_WALK_BAD;
            net_len = (uint16_t)(net_len + cur_optlen);
            must_align = 1;
            r = walk_destopt(h, avail, e);
            if (r == -2) return ORACLE_WALK_BAD;
            if (r < 0) return ORACLE_WALK_DROP;
            break;
        case 6: case 17: case 58:
            if (must_align && (plen % 8u) != 0) return ORACLE_WALK_DROP;
            *net_len_out = net_len;
            *proto_out = nx;
            return frag ? ORACLE_WALK_FRAG : ORACLE_WALK_PROTO;
        default:                                              /* ESP, AUTH, NONE, invalid */
            return ORACLE_WALK_DROP;
        }
        WALK_BYTE(e, nx);                                     /* exthdr->nxthdr, :805 */
        cur_nexthdr = ptr;
        ptr += cur_optlen;
    }
}

/*
 * Fused IPv6 transport restatement, one datagram per descriptor.  desc.off ->
 * IPv6 header; desc.len = bytes available; desc.seed = f->net_len | proto << 16
 * when the stack already walked the extension headers (pico_ipv6_extension_headers,
 * modules/pico_ipv6.c:707-809), or 0.
 * RX, seed 0: the walk (oracle_ipv6_walk) decides: a discard (or a read past the frame) is
 *   MALFORMED; a transport behind a fragment header is FRAG (pico_ipv6_process_frag,
 *   :791-795, no transport check); otherwise net_len and proto are the walk's.
 * TX, seed 0: net_len 40, proto = hdr->nxthdr (the stack builds the header it sends).
 *   transport_len = (uint16)(payload_len - (net_len - 40))     pico_ipv6.c:790
 * RX: pico_transport_crc_check (stack/pico_socket.c:1916-1968) as the reference runs it: the
 *   `switch (net_hdr->proto)` (:1923) reads the header through a struct pico_ipv4_hdr cast --
 *   for IPv6 that is byte 9 (the source address's second byte): 6 -> pico_tcp_checksum ->
 *   pico_tcp_checksum_ipv6 (pico_tcp.c:492-505, TCP in the pseudo header), 17 -> when the
 *   transport's bytes 6-7 are != 0, pico_udp_checksum_ipv6 (pico_udp.c:63-92, UDP in the pseudo
 *   header), else no check -- for a TCP or UDP datagram (pico_transport_process_in is the TCP /
 *   UDP module's).  With ORACLE_NXTHDR_DISPATCH instead by the transport protocol: TCP always,
 *   UDP when its crc != 0.  ICMPv6 (pico_icmp6_process_in): pico_icmp6_checksum always, a
 *   verdict only for the ND / MLD types the reference checks (pico_ipv6_nd.c:595,
 *   pico_mld.c:415).  Other protocols: none.
 *   out = the checksum (0 = valid), 0 when none is computed.
 * TX: crc field read as zero (TCP pico_tcp.c:980, ICMPv6 pico_ipv6.c:1337, UDP
 *   crc already 0 from pico_udp_push :123 when pico_ipv6.c:1345 computes it);
 *   TCP needs 20, UDP 8, ICMPv6 4 transport bytes.  Other protocols: none.
 * MALFORMED: avail < 40, net_len < 40 or past avail, transport past avail, or a
 *   field the reference reads lying past avail (a UDP header: 8 bytes).
 */
void oracle_batch_ipv6(const uint8_t *base, const struct pico_csum_desc *d, uint32_t n,
                       uint16_t *out_l4, uint8_t *verdict, uint32_t flags)
{
    uint32_t i;
    int tx = (flags & ORACLE_IPV4_TX) != 0;
    int refd = !tx && (flags & ORACLE_NXTHDR_DISPATCH) == 0;
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
            if (!tx) {
                int w = oracle_ipv6_walk(h, avail, &net_len, &proto);
                if (w == ORACLE_WALK_FRAG) {
                    verdict[i] = PICO_CSUM_V_FRAG;
                    continue;
                }
                if (w != ORACLE_WALK_PROTO)
                    continue;
            }
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
 * Fragment reassembly with the transport check of the reassembled datagram,
 * IPv4 and IPv6.  Group g = fragments grp[2g] .. grp[2g] + grp[2g+1] - 1 of one datagram (src,
 * dst, id matched by the stack, pico_fragments.c:104-178, 432-568), in arrival order.
 * Per fragment:
 *   IPv4  as pico_ipv4_process_in hands it on (modules/pico_ipv4.c:381-450): net_len = 20 +
 *         4 (IHL - 5), f->transport_len = (uint16)(tot - net_len), f->frag = short_be(hdr->frag);
 *         offset IP4_FRAG_OFF = (frag & 0x1FFF) << 3, more = frag & 0x2000 (pico_fragments.c:46-49)
 *   IPv6  as pico_ipv6_extension_headers hands it on (modules/pico_ipv6.c:707-809, the walk of
 *         oracle_ipv6_walk): the transport must be reached behind a fragment header (else the
 *         reference never reassembles it: MALFORMED); net_len = the walk's, f->transport_len =
 *         (uint16)(payload_len - (net_len - 40)) (:790), f->frag = that header's offset / M
 *         field; offset IP6_FRAG_OFF = frag & 0xFFF8, more = frag & 1 (pico_fragments.c:35-36);
 *         the module it goes to (pico_ipv6_process_frag's proto) = the walk's transport protocol
 * Per group:
 *   tree order     by offset (pico_ipv4/6_frag_compare, pico_fragments.c:73-83, 129-139);
 *                  pico_tree_insert rejects a repeated offset: the earlier arrival is kept
 *   completeness   pico_fragments_check_complete (:216-239): offsets contiguous from 0
 *                  (offset == sum of the previous transport_len), up to the first fragment
 *                  without "more"; len = that sum.  The set completes at the arrival of the last
 *                  of those fragments, whose protocol pico_fragments_reassemble hands on.
 *   gather         pico_fragments_reassemble (:304-358): the first fragment's PICO_SIZE_IP4HDR
 *                  (20) / PICO_SIZE_IP6HDR (40) bytes, then every fragment's transport bytes
 *   transport      IPv4: pico_transport_crc_check (stack/pico_socket.c:1916-1968) with
 *                  net_hdr->proto of the copied header: TCP always, UDP when its crc != 0 (and
 *                  the datagram holds the 8-byte UDP header), pseudo header from the copied
 *                  header, transport_len = len.
 *                  IPv6: the module of the completing fragment -- TCP / UDP: the same check,
 *                  dispatched on byte 9 of the copied header as the reference does (with
 *                  ORACLE_NXTHDR_DISPATCH: on the module), pseudo header = struct
 *                  pico_ipv6_pseudo_hdr of the copied header; ICMPv6: pico_icmp6_checksum, a
 *                  verdict only for the ND / MLD types (pico_icmp6_process_in); others: none.
 * out_len[g] = len (0 when not reassembled), out_l4[g] = the checksum (0 = valid; 0 when none),
 * verdict[g] = ACCEPT / L4_BAD, or MALFORMED when not reassembled: incomplete, a fragment behind
 * the completing one (the reference's copy loop, :339-345, would write past its HDR + len byte
 * buffer), HDR + len > 65535 (its (uint16_t) allocation size wraps), a fragment whose header or
 * transport lies past desc.len, an empty group or one of more than 512 fragments (the API's
 * limit), or an output region (out_desc[g].len) shorter than HDR + len or not 4-byte aligned
 * (the API's contract).
 */
static void oracle_reassemble(int v6, const uint8_t *base, const struct pico_csum_desc *d, uint32_t nd,
                              const uint32_t *grp, uint32_t ng, uint8_t *out, const struct pico_csum_desc *od,
                              uint32_t *out_len, uint16_t *out_l4, uint8_t *verdict, uint32_t flags)
{
    const uint32_t HDR = v6 ? 40u : 20u;
    uint32_t g;
    for (g = 0; g < ng; g++) {
        uint32_t first = grp[2 * g], cnt = grp[2 * g + 1], i, k, m = 0, len = 0, bad = 0, e = 0, done = 0, comp = 0;
        uint32_t na = cnt && cnt <= 512 ? cnt : 1;
        uint32_t *ord = (uint32_t *)malloc(sizeof(uint32_t) * na);
        uint32_t *foff = (uint32_t *)malloc(sizeof(uint32_t) * na);
        uint32_t *tl = (uint32_t *)malloc(sizeof(uint32_t) * na);
        uint32_t *hlen = (uint32_t *)malloc(sizeof(uint32_t) * na);
        uint8_t *mf = (uint8_t *)malloc(na), *pr = (uint8_t *)malloc(na);
        out_len[g] = 0;
        out_l4[g] = 0;
        verdict[g] = PICO_CSUM_V_MALFORMED;
        if (cnt == 0 || cnt > 512 || first > nd || cnt > nd - first)   /* 512: the device API's limit */
            bad = 1;
        for (i = 0; i < cnt && !bad; i++) {
            const struct pico_csum_desc *f = &d[first + i];
            const uint8_t *h = base + f->off;
            if (!v6) {
                uint32_t ihl, frag;
                if (f->len < 20) { bad = 1; break; }
                ihl = h[0] & 0x0Fu;
                hlen[i] = 20u + (ihl > 5u ? 4u * (ihl - 5u) : 0u);
                tl[i] = (uint16_t)(((h[2] << 8) | h[3]) - hlen[i]);
                frag = (uint32_t)((h[6] << 8) | h[7]);
                foff[i] = (frag & 0x1FFFu) << 3;
                mf[i] = (frag & 0x2000u) != 0;
                pr[i] = h[9];
            } else {
                uint32_t nl = 0;
                uint8_t proto = 0;
                uint16_t om = 0;
                if (f->len < 40 || oracle_ipv6_walk_frag(h, f->len, &nl, &proto, &om) != ORACLE_WALK_FRAG) {
                    bad = 1;
                    break;
                }
                hlen[i] = nl;
                tl[i] = (uint16_t)((((uint32_t)h[4] << 8) | h[5]) - (nl - 40u));
                foff[i] = om & 0xFFF8u;
                mf[i] = om & 1u;
                pr[i] = proto;
            }
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
            if (ord[k] > comp) comp = ord[k];                /* the set completes at its last arrival */
            if (!mf[ord[k]]) { e = k; done = 1; break; }
        }
        if (!bad && done && e + 1 == m && HDR + len <= 0xFFFFu && od[g].len >= HDR + len && (od[g].off & 3u) == 0) {
            uint8_t *dst = out + od[g].off;
            const uint8_t *h0 = base + d[first + ord[0]].off;
            uint32_t at = HDR, s;
            memcpy(dst, h0, HDR);
            for (k = 0; k < m; k++) {
                const uint8_t *src = base + d[first + ord[k]].off + hlen[ord[k]];
                memcpy(dst + at, src, tl[ord[k]]);
                at += tl[ord[k]];
            }
            out_len[g] = len;
            verdict[g] = PICO_CSUM_V_ACCEPT;
            if (!v6) {
                uint8_t proto = h0[9];
                if (proto == 6 || (proto == 17 && len >= 8 && (dst[20 + 6] || dst[20 + 7]))) {
                    s = oracle_ipv4_pseudo_sum(dst + 12, dst + 16, proto, (uint16_t)len);
                    out_l4[g] = oracle_checksum_finalize(oracle_checksum_adder(s, dst + 20, len));
                    if (out_l4[g]) verdict[g] = PICO_CSUM_V_L4_BAD;
                }
            } else {
                uint8_t module = pr[comp], cp = module;
                int check = 0;
                if (module == 6 || module == 17) {
                    if (!(flags & ORACLE_NXTHDR_DISPATCH))
                        cp = dst[9];                          /* pico_socket.c:1923 through the IPv4 cast */
                    check = cp == 6 || (cp == 17 && len >= 8 && (dst[40 + 6] || dst[40 + 7]));
                } else if (module == 58 && len >= 1) {
                    check = 1;
                }
                if (check) {
                    s = oracle_ipv6_pseudo_sum(dst + 8, dst + 24, cp, len);
                    out_l4[g] = oracle_checksum_finalize(oracle_checksum_adder(s, dst + 40, len));
                    if (out_l4[g] && (module != 58 || icmp6_checked_type(dst[40])))
                        verdict[g] = PICO_CSUM_V_L4_BAD;
                }
            }
        }
        free(ord); free(foff); free(tl); free(hlen); free(mf); free(pr);
    }
}

void oracle_ipv4_reassemble(const uint8_t *base, const struct pico_csum_desc *d, uint32_t nd, const uint32_t *grp,
                            uint32_t ng, uint8_t *out, const struct pico_csum_desc *od, uint32_t *out_len, uint16_t *out_l4,
                            uint8_t *verdict)
{
    oracle_reassemble(0, base, d, nd, grp, ng, out, od, out_len, out_l4, verdict, 0);
}

void oracle_ipv6_reassemble(const uint8_t *base, const struct pico_csum_desc *d, uint32_t nd, const uint32_t *grp,
                            uint32_t ng, uint8_t *out, const struct pico_csum_desc *od, uint32_t *out_len, uint16_t *out_l4,
                            uint8_t *verdict, uint32_t flags)
{
    oracle_reassemble(1, base, d, nd, grp, ng, out, od, out_len, out_l4, verdict, flags);
}

/* modules/pico_ipv4.c:1535-1574 (pico_ipv4_pre_forward_checks, called by pico_ipv4_forward :1600
 * for a datagram whose destination has a route):
 *   hdr->ttl = (uint8_t)(hdr->ttl - 1); if (hdr->ttl < 1) -> expired, dropped (crc untouched);
 *   hdr->crc++ (uint16_t field, native LE increment of the stored big-endian checksum);
 *   pico_ipv4_link_get(&hdr->src) -> a local source, dropped (:1559-1560);
 *   (src, id, dst, proto) == the last tuple that reached this point -> dropped as a duplicate,
 *   else it becomes the last tuple (:1562-1571; static state, zero at start).
 * In place on base, in batch order; `st` carries the last tuple from one call to the next (the
 * reference's statics; zero = its initial state).  Verdict per datagram: ACCEPT (forwarded),
 * EXPIRED, LOCAL_SRC, DUPLICATE, MALFORMED (< 20 bytes: untouched, no state change). */
void oracle_batch_ipv4_forward(uint8_t *base, const struct pico_csum_desc *d, uint32_t n, const uint32_t *local,
                               uint32_t n_local, struct oracle_fwd_state *st, uint8_t *verdict)
{
    uint32_t i, k;
    for (i = 0; i < n; i++) {
        uint8_t *h = base + d[i].off;
        uint16_t crc, id;
        uint32_t src, dst;
        int is_local = 0;
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
        memcpy(&src, h + 12, 4);
        memcpy(&dst, h + 16, 4);
        memcpy(&id, h + 4, 2);
        for (k = 0; k < n_local; k++)
            is_local |= local[k] == src;
        if (is_local) {
            verdict[i] = PICO_CSUM_V_LOCAL_SRC;
        } else if (st->src == src && st->id == id && st->dst == dst && st->proto == h[9]) {
            verdict[i] = PICO_CSUM_V_DUPLICATE;
        } else {
            st->src = src;
            st->dst = dst;
            st->id = id;
            st->proto = h[9];
            verdict[i] = PICO_CSUM_V_ACCEPT;
        }
    }
}

/* modules/pico_nat.c:424-545, pico_ipv4_nat_inbound / pico_ipv4_nat_outbound after the tuple
 * lookup (the host's table decides rw[i]; dir 0 = no tuple: return -1, nothing written).  The
 * frame as pico_ipv4_process_in leaves it (:392-405): net_len = 20 + options, transport_len =
 * (uint16)(tot_len - net_len), transport_hdr = net_hdr + net_len; f->sock NULL, so the pseudo
 * header comes from the (rewritten) IP header (pico_tcp.c:428-443, pico_udp.c:42-57).  In place:
 *   TCP / UDP: addr into src (outbound, :509 / :525) or dst (inbound, :446 / :462), port into
 *     sport / dport (:510 / :526, :447 / :463); crc = 0; crc = short_be(pico_tcp_checksum_ipv4 /
 *     pico_udp_checksum_ipv4) (:448-449, :464-465, :515-516, :531-532) -- UDP included, whatever
 *     its crc was; then the header checksum (:480-481, :545-546).
 *   ICMPv4: no rewrite (:466-468, :533-535), the header checksum only.
 *   Other protocols: return -1 (:472-474, :537-539): untouched.
 * Datagrams the batch leaves alone as the stack never NATs them: a fragment (handed to
 * reassembly first, pico_ipv4.c:446-455) -> FRAG; infeasible lengths (the TX-path bounds of
 * oracle_batch_ipv4) or a TCP / UDP transport shorter than 20 / 8 bytes with a record (the
 * reference would write past it) -> MALFORMED.  out_net / out_l4: the values stored (else 0). */
void oracle_batch_ipv4_nat(uint8_t *base, const struct pico_csum_desc *d, uint32_t n, const struct oracle_nat *rw,
                           uint16_t *out_net, uint16_t *out_l4, uint8_t *verdict)
{
    uint32_t i;
    for (i = 0; i < n; i++) {
        uint8_t *h = base + d[i].off, *t;
        uint32_t avail = d[i].len, net_len, s;
        uint16_t tot, transport_len, frag, cs;
        uint8_t proto;

        out_net[i] = 0; out_l4[i] = 0; verdict[i] = PICO_CSUM_V_MALFORMED;
        if (avail < 20)
            continue;
        net_len = 20u + ((h[0] & 0x0Fu) > 5u ? 4u * ((h[0] & 0x0Fu) - 5u) : 0u);
        tot = (uint16_t)((h[2] << 8) | h[3]);
        transport_len = (uint16_t)(tot - net_len);
        frag = (uint16_t)((h[6] << 8) | h[7]);
        proto = h[9];
        if (net_len > avail || net_len + (uint32_t)transport_len > avail)
            continue;
        if (frag & 0x3FFFu) {
            verdict[i] = PICO_CSUM_V_FRAG;
            continue;
        }
        t = h + net_len;
        if (rw[i].dir != 1 && rw[i].dir != 2) {
            verdict[i] = PICO_CSUM_V_UNTOUCHED;
            continue;
        }
        if (proto == 6 || proto == 17) {
            const uint32_t crc_at = proto == 6 ? 16u : 6u;
            if (transport_len < (proto == 6 ? 20u : 8u))
                continue;                                                /* MALFORMED */
            memcpy(h + (rw[i].dir == 1 ? 12 : 16), &rw[i].addr, 4);
            memcpy(t + (rw[i].dir == 1 ? 0 : 2), &rw[i].port, 2);
            t[crc_at] = 0;
            t[crc_at + 1] = 0;
            s = oracle_ipv4_pseudo_sum(h + 12, h + 16, proto, transport_len);
            cs = oracle_checksum_finalize(oracle_checksum_adder(s, t, transport_len));
            t[crc_at] = (uint8_t)(cs >> 8);                              /* short_be */
            t[crc_at + 1] = (uint8_t)cs;
            out_l4[i] = cs;
        } else if (proto != 1) {
            verdict[i] = PICO_CSUM_V_UNTOUCHED;
            continue;
        }
        h[10] = 0;
        h[11] = 0;
        cs = oracle_checksum(h, net_len);
        h[10] = (uint8_t)(cs >> 8);
        h[11] = (uint8_t)cs;
        out_net[i] = cs;
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

/*
 * pico_csum.h -- C ABI of libpicocsum, the MI355X-native drop-in for picoTCP's
 * Internet-checksum path (RFC 1071 one's-complement sum, stack/pico_frame.c).
 *
 * Plain C: no torch, no HIP types in any signature.  Device pointers are
 * plain `void *` / `T *`; a HIP stream is passed as an opaque `void *`
 * (NULL = the device's default stream).
 *
 * Three layers:
 *
 *  1. Scalar drop-in (replaces the two strong symbols of the reference's
 *     stack/pico_frame.o; callers keep compiling against
 *     include/pico_frame.h unchanged):
 *       pico_checksum            ref: include/pico_frame.h:106, stack/pico_frame.c:312-318
 *       pico_dualbuffer_checksum ref: include/pico_frame.h:107, stack/pico_frame.c:320-328
 *     The reference calls these inline, once per frame, from a single-threaded
 *     tick loop on host pointers.  A GPU launch costs ~10 us
 *     against ~100 ns of work, so these two stay synchronous host code with
 *     bit-identical results; the accelerated path is layer 2.
 *
 *  2. Batched device API (the MI355X hot path; the reference has no batch
 *     entry -- each function below is the batch form of the per-frame calls
 *     cited on it).  Buffers are device-resident; calls are asynchronous on
 *     `stream`; they never fall back to host code: when no HIP device or
 *     kernel image is usable they return -PICO_ERR_ENODEV and set
 *     pico_csum_last_error().
 *
 *  3. Host-resident batch API: H2D -> kernel -> D2H, chunked and overlapped on
 *     two streams (the path starts and ends in host memory: a pico_device /
 *     TAP buffer, modules/pico_dev_tap.c:53-79).
 *
 * Return convention of every checksum value (device and host alike) is the
 * reference's: ret = short_be((uint16_t)~fold(sum)); a caller stores
 * hdr->crc = short_be(ret), and a region that already carries its correct
 * checksum yields 0 (pico_ipv4.c:249, pico_socket.c:1927).
 *
 * Error codes: 0 on success, otherwise the negated picoTCP pico_err value
 * (include/pico_protocol.h:21-65).
 */
#ifndef PICO_CSUM_H
#define PICO_CSUM_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ABI history (a caller must check pico_csum_abi_version() == PICO_CSUM_ABI_VERSION):
 *   2: V_FRAG, the reference's IPv6 byte-9 dispatch by default;
 *   3: F_NXTHDR_DISPATCH moved to 0x8 (bit 0x4 -- ABI 1's F_REF_DISPATCH, the opposite meaning --
 *      is rejected with -EINVAL); the forwarding batch takes the host's link addresses and a
 *      carried state (pico_ipv4_pre_forward_checks in full);
 *   4: pico_csum_release_thread_scratch; the reassembly's flat-grid scratch is freed at thread exit. */
#define PICO_CSUM_ABI_VERSION 4

/* picoTCP pico_err values used here (include/pico_protocol.h:27,31,38 + ENODEV) */
#define PICO_CSUM_EIO     5
#define PICO_CSUM_ENOMEM 12
#define PICO_CSUM_EINVAL 22
#define PICO_CSUM_ENODEV 19

/* One frame region of a batch: 16 bytes, naturally aligned. */
#ifndef PICO_CSUM_DESC_DEFINED
#define PICO_CSUM_DESC_DEFINED
struct pico_csum_desc {
    uint64_t off;   /* byte offset of the region from the batch base (any alignment) */
    uint32_t len;   /* RAW: region length (the `len` of pico_checksum);
                       IPV4: bytes available from the IPv4 header to the end of
                       the frame buffer = f->buffer_len - (f->net_hdr - f->buffer) */
    uint32_t seed;  /* RAW: initial pico_checksum_adder accumulator, e.g. a
                       pseudo-header partial from pico_ipv4_pseudo_partial()
                       (TX: from socket state, pico_tcp.c:429-433); 0 for a
                       plain pico_checksum.  IPV4: must be 0 (reserved). */
};
#endif

/* flags */
#define PICO_CSUM_F_WRITE 0x1u  /* store short_be(ret) into the frame's crc field (in place, device memory) */
#define PICO_CSUM_F_TX    0x2u  /* fused batches: compute (TX) mode -- crc fields read as zero */
/* IPv6 / Ethernet batches, RX.  By default the IPv6 TCP / UDP transport check is dispatched
 * exactly as the reference's pico_transport_crc_check does it (stack/pico_socket.c:1919-1923):
 * on `proto` read through a struct pico_ipv4_hdr cast of the network header -- for IPv6 that is
 * byte 9, the source address's second byte: 6 -> pico_tcp_checksum (TCP pseudo header), 17 ->
 * the UDP check when transport bytes 6-7 are non-zero (UDP pseudo header), anything else -> no
 * check.  With this flag the check follows the transport's own protocol instead (TCP always,
 * UDP when its crc != 0: the evident intent, not the reference's behaviour).  ICMPv6 is the
 * same either way (pico_icmp6_process_in checks it itself). */
#define PICO_CSUM_F_NXTHDR_DISPATCH 0x8u
#define PICO_CSUM_F_RETIRED_0x4     0x4u  /* ABI 1's F_REF_DISPATCH: rejected (-EINVAL) since ABI 3 */

/* Verdict byte of the fused batches: the reference's FIRST outcome for the frame, in its own
 * order (one value, plus V_IPV6 on the Ethernet batch's IPv6 frames).
 * The values are per batch kind: bits 16, 32 and 64 mean different things in different batches
 * (V_FRAG / V_EXPIRED; V_DROP_L2 / V_UNTOUCHED / V_LOCAL_SRC; V_ARP / V_DUPLICATE).  Decode a
 * verdict array only with the list given at the batch that produced it:
 *   RX / TX (IPv4, IPv6):  ACCEPT, NET_BAD (IPv4), L4_BAD, MALFORMED, FRAG
 *   Ethernet:              the RX / TX list, DROP_L2, ARP, | IPV6
 *   forwarding:            ACCEPT, MALFORMED, EXPIRED, LOCAL_SRC, DUPLICATE
 *   NAT:                   ACCEPT, MALFORMED, FRAG, UNTOUCHED
 *   reassembly:            ACCEPT, L4_BAD, MALFORMED */
#define PICO_CSUM_V_ACCEPT    1u  /* delivered to the transport and every checksum the reference
                                     checks passes: hand the frame on (a stack built with CRC=0
                                     need not check it again) */
#define PICO_CSUM_V_NET_BAD   2u  /* pico_ipv4_crc_check discards it (pico_ipv4.c:420-422, :243-257) */
#define PICO_CSUM_V_L4_BAD    4u  /* pico_transport_crc_check discards it (pico_socket.c:1929,1953) */
#define PICO_CSUM_V_MALFORMED 8u  /* discarded before any transport: infeasible length
                                     (pico_ipv4.c:405-408); after a good header checksum an invalid
                                     source (:425-428), the evil bit (:431-435), IHL < 5 (:438-443);
                                     an IPv6 extension-header chain pico_ipv6_extension_headers
                                     discards (pico_ipv6.c:659-809); a header or field that lies
                                     past the buffer (where the reference would read past it) */
#define PICO_CSUM_V_FRAG     16u  /* a fragment: IPv4 MF or offset (pico_ipv4.c:446-455), IPv6 a
                                     fragment header (pico_ipv6.c:791-795) -- header verified, NO
                                     transport check (the reference checks the reassembled
                                     datagram): route it to the reassembly batch.  TX: the
                                     header checksum only (the transport's covers the datagram). */
#define PICO_CSUM_V_EXPIRED  16u  /* forwarding batch only (same bit): TTL reached 0 (pico_ipv4.c:1549-1552) */
#define PICO_CSUM_V_LOCAL_SRC 32u /* forwarding batch only: the source is one of the host's link addresses
                                     (pico_ipv4.c:1559-1560) */
#define PICO_CSUM_V_DUPLICATE 64u /* forwarding batch only: (src, id, dst, proto) of the last forwarded
                                     datagram (pico_ipv4.c:1562-1565) */
#define PICO_CSUM_V_DROP_L2  32u  /* Ethernet batch: discarded by the link layer -- foreign destination MAC
                                     (pico_ethernet.c:221-231), unknown ethertype (:201-202) or an IP
                                     version that does not match it (:143-150, :162-176) */
#define PICO_CSUM_V_ARP      64u  /* Ethernet batch: ARP frame, handed to pico_arp_receive (:186-187) */
#define PICO_CSUM_V_IPV6    128u  /* Ethernet batch: set on every IPv6 frame (ethertype 0x86DD) */
#define PICO_CSUM_V_UNTOUCHED 32u /* NAT batch only (same bit as V_DROP_L2): left as it is -- no
                                     rewrite record (the host's tuple lookup failed), or a protocol
                                     the reference's NAT returns -1 on (pico_nat.c:472-474, :537-539) */

/* ---------------------------------------------------------------- layer 1 */

/* ref: stack/pico_frame.c:312-318 */
uint16_t pico_checksum(void *inbuf, uint32_t len);
/* ref: stack/pico_frame.c:320-328 (len1 must be even, as in the reference) */
uint16_t pico_dualbuffer_checksum(void *inbuf1, uint32_t len1, void *inbuf2, uint32_t len2);

/* The reference's accumulator step, exported so a caller can build a
 * descriptor seed: ref stack/pico_frame.c:279-299 pico_checksum_adder. */
uint32_t pico_checksum_partial(uint32_t sum, const void *buf, uint32_t len);
/* Accumulator value of the 12-byte struct pico_ipv4_pseudo_hdr
 * (modules/pico_ipv4.h:46-53) as pico_tcp_checksum_ipv4 / pico_udp_checksum_ipv4
 * build it (pico_tcp.c:428-443, pico_udp.c:42-57).  src/dst as stored in
 * struct pico_ip4 (network byte order). */
uint32_t pico_ipv4_pseudo_partial(uint32_t src_addr, uint32_t dst_addr, uint8_t proto, uint16_t transport_len);
/* Accumulator value of the 40-byte struct pico_ipv6_pseudo_hdr (modules/pico_ipv6.h:46-53:
 * src, dst, long_be(len), 3 zero bytes, nxthdr) as pico_tcp_checksum_ipv6 /
 * pico_udp_checksum_ipv6 / pico_icmp6_checksum / pico_mld_checksum build it
 * (pico_tcp.c:449-475, pico_udp.c:63-92, pico_icmp6.c:38-55, pico_mld.c:421-437).
 * A raw batch seeded with it serves the MLD router-alert variant (transport + 8,
 * length - 8) and TX datagrams whose addresses come from the socket. */
uint32_t pico_ipv6_pseudo_partial(const void *src16, const void *dst16, uint8_t nxthdr, uint32_t transport_len);

/* ---------------------------------------------------------------- layer 2 */

/* Every device batch takes the size of the buffer behind d_base (base_len).
 * Nothing outside [d_base, d_base + base_len) is ever written, and no byte outside it
 * contributes to a result.  The kernels load whole 16-byte-aligned blocks, so the
 * 16-byte-aligned blocks that overlap [d_base, d_base + base_len) may be read in full
 * (up to 15 bytes before d_base and after its end; such a block never crosses a page,
 * so this cannot fault).  A caller that writes those neighbouring bytes from another
 * stream concurrently gets correct results all the same: they are masked out.
 *
 * Batch of pico_checksum / pico_dualbuffer_checksum calls:
 *   d_out[i] = finalize(adder(desc[i].seed, d_base + desc[i].off, desc[i].len))
 * crc_off >= 0 (even): the 2 bytes at off+crc_off read as zero when they lie
 * inside the region ("hdr->crc = 0" before computing: pico_ipv4.c:237,
 * pico_icmp4.c:38, pico_tcp.c:980); with PICO_CSUM_F_WRITE the result is
 * stored there (pico_ipv4.c:238, pico_icmp4.c:39, pico_tcp.c:981).
 * crc_off < 0: no crc field.  Regions may not overlap when F_WRITE is set.
 * A region that does not lie inside base_len is not read: d_out[i] = 0 and,
 * when d_bad != NULL, *d_bad (a device uint32 the caller zeroes) counts it. */
int pico_checksum_batch_dev(void *d_base, uint64_t base_len, const struct pico_csum_desc *d_desc,
                            uint32_t n, int32_t crc_off, uint32_t flags, uint16_t *d_out,
                            uint32_t *d_bad, void *stream);

/* Uniform batch (no descriptors): frame i = d_base + i*stride, len bytes,
 * seed added to every frame.  The layout of a packed frame ring.
 * (n-1)*stride + len must not exceed base_len (else -EINVAL). */
int pico_checksum_batch_uniform_dev(const void *d_base, uint64_t base_len, uint64_t stride, uint32_t len,
                                    uint32_t n, uint32_t seed, uint16_t *d_out, void *stream);

/* Fused IPv4 header + transport batch, one IPv4 datagram per descriptor
 * (desc.off -> IPv4 header, desc.len = bytes available).
 * RX (flags without F_TX): pico_ipv4_process_in (pico_ipv4.c:381-456) up to its hand-off --
 *   lengths, pico_ipv4_crc_check (:243-257), the source check, the evil bit, IHL < 5, the
 *   fragment hand-off -- then pico_transport_crc_check (pico_socket.c:1916-1968): TCP always,
 *   UDP when its crc field != 0, pseudo header from the IP header.  The link-directed
 *   broadcast sources of pico_ipv4_is_broadcast (the stack's link table) are left to the stack.
 *   d_out_net = pico_checksum(hdr, net_len), d_out_transport = the TCP/UDP
 *   checksum (0 = valid; 0 when none is computed), d_verdict = PICO_CSUM_V_*.
 * TX (F_TX): crc fields read as zero; d_out_* are the values to store
 *   (IPv4 header; TCP with pseudo header; ICMPv4 without; UDP 0 as
 *   pico_udp.c:123).  F_WRITE stores them into accepted frames in place.
 * A datagram whose [off, off+len) is not inside base_len is MALFORMED, unread.
 * Any output pointer may be NULL. */
int pico_ipv4_checksum_batch_dev(void *d_base, uint64_t base_len, const struct pico_csum_desc *d_desc,
                                 uint32_t n, uint32_t flags, uint16_t *d_out_net,
                                 uint16_t *d_out_transport, uint8_t *d_verdict, void *stream);

/* Fused IPv6 transport batch (TCP / UDP / ICMPv6 over IPv6),
 * one datagram per descriptor: desc.off -> IPv6 header, desc.len = bytes available,
 * desc.seed = 0, or f->net_len | (transport proto << 16) when the stack already walked the
 * extension headers.  RX with seed 0: the kernel walks them itself, as
 * pico_ipv6_extension_headers does (pico_ipv6.c:659-809: the sequence check, hop-by-hop /
 * routing / fragment / destination-option processing): a chain the reference discards is
 * V_MALFORMED, a transport behind a fragment header V_FRAG.  TX with seed 0: net_len 40,
 * proto = hdr->nxthdr.  transport_len = (uint16)(payload_len - (net_len - 40))
 * (pico_ipv6.c:790); pseudo header = struct pico_ipv6_pseudo_hdr (pico_ipv6.h:46-53) from
 * the IPv6 header.
 * RX: pico_transport_crc_check (pico_socket.c:1916-1968; pico_tcp_checksum_ipv6
 *   pico_tcp.c:449-475, pico_udp_checksum_ipv6 pico_udp.c:63-92) dispatched on header byte 9
 *   as the reference does (see PICO_CSUM_F_NXTHDR_DISPATCH for the alternative); ICMPv6
 *   (pico_icmp6_checksum pico_icmp6.c:38-55) is always computed, V_L4_BAD only for the ND /
 *   MLD types the reference checks (pico_ipv6_nd.c:595, pico_mld.c:415).
 * TX (F_TX): crc field read as zero (pico_tcp.c:980, pico_ipv6.c:1337,1345);
 *   F_WRITE stores it.  d_out_transport: the checksum (0 = valid on RX). */
int pico_ipv6_checksum_batch_dev(void *d_base, uint64_t base_len, const struct pico_csum_desc *d_desc,
                                 uint32_t n, uint32_t flags, uint16_t *d_out_transport, uint8_t *d_verdict,
                                 void *stream);

/* Ethernet front end of the fused RX verify, one frame per descriptor,
 * IPv4, IPv6, ARP and other ethertypes mixed in ONE launch: desc.off -> the Ethernet header
 * (f->datalink_hdr), desc.len = frame bytes (f->buffer_len), desc.seed = the IPv6 net_len |
 * proto << 16 as for pico_ipv6_checksum_batch_dev (IPv6 frames; 0 otherwise).
 * Per frame, as pico_ethernet_receive / pico_eth_receive (modules/pico_ethernet.c:180-235):
 *   RX destination filter when mac != NULL (host pointer to the device's 6-byte address,
 *   f->dev->eth->mac): own address, 01:00:5e / 33:33 multicast or broadcast, else V_DROP_L2;
 *   ethertype 0x0806 -> V_ARP (no checksum); 0x0800 -> the IPv4 batch semantics on
 *   (off + 14, len - 14) if the version nibble is 4; 0x86DD -> the IPv6 batch semantics if
 *   it is 6, verdict | V_IPV6; anything else V_DROP_L2.  Frames shorter than 15 bytes are
 *   MALFORMED.  d_out_net is 0 for every non-IPv4 frame.  TX (F_TX, no MAC filter) computes
 *   and, with F_WRITE, stores the IPv4 / IPv6 checksums of the frames the stack built.
 *   F_NXTHDR_DISPATCH (RX) applies to the IPv6 frames as in pico_ipv6_checksum_batch_dev. */
int pico_eth_checksum_batch_dev(void *d_base, uint64_t base_len, const struct pico_csum_desc *d_desc, uint32_t n,
                                uint32_t flags, const uint8_t *mac, uint16_t *d_out_net, uint16_t *d_out_transport,
                                uint8_t *d_verdict, void *stream);

/* Forwarding step: pico_ipv4_pre_forward_checks (modules/pico_ipv4.c:1535-1574), which
 * pico_ipv4_forward (:1580-1603) runs on a datagram once route_find has a route for it, for a batch
 * of IPv4 datagrams routed through this host (desc.off -> IPv4 header, desc.len = bytes available,
 * >= 20), IN BATCH ORDER:
 *   hdr->ttl is decremented in place; a datagram whose TTL reaches 0 is V_EXPIRED (the reference
 *   drops it -- and sends pico_notify_ttl_expired, the caller's job -- crc untouched);
 *   every other one gets the reference's `hdr->crc++` (:1556, a native little-endian increment of
 *   the stored field), then:
 *   V_LOCAL_SRC  its source is one of local_addrs[0 .. n_local) (the host's link addresses, as
 *                stored: pico_ipv4_link_get's table, :1559; host memory, n_local <= 32);
 *   V_DUPLICATE  (src, id, dst, proto) equals the last datagram that got this far (:1562-1571);
 *   V_ACCEPT     forwarded: it becomes the last datagram (the caller goes on with NAT, the MTU
 *                check and pico_datalink_send, :1600-1610).
 * d_state (device memory, struct pico_csum_fwd_state) is the reference's static last tuple, carried
 * from one batch to the next; zero it once at start (the reference's initial value: a first datagram
 * with an all-zero tuple is a duplicate).  NULL: a zero state, not kept.  Calls that share a d_state
 * must be ordered (one stream).  Regions past base_len or shorter than 20 bytes are V_MALFORMED,
 * untouched, and leave the state alone.  d_verdict is required (the batch order is resolved through
 * it).  The descriptors of one batch must not overlap: each header is updated by one lane with a
 * plain read-modify-write, so two descriptors on the same header would race on its TTL / crc
 * (the reference, handed the same frame twice, would apply both decrements in sequence).  Three
 * kernel launches on `stream`. */
struct pico_csum_fwd_state {
    uint32_t src;       /* last_src, as stored */
    uint32_t dst;       /* last_dst */
    uint16_t id;        /* last_id, as stored (bytes 4-5 of the header) */
    uint16_t proto;     /* last_proto */
    uint32_t reserved;
};
int pico_ipv4_forward_batch_dev(void *d_base, uint64_t base_len, const struct pico_csum_desc *d_desc, uint32_t n,
                                const uint32_t *local_addrs, uint32_t n_local, struct pico_csum_fwd_state *d_state,
                                uint8_t *d_verdict, void *stream);

/* NAT rewrite of a batch of IPv4 datagrams: the frame work of
 * pico_ipv4_nat_outbound / pico_ipv4_nat_inbound (modules/pico_nat.c:424-545) once the host's
 * tuple table has chosen the new address and port.  desc.off -> IPv4 header, desc.len = bytes
 * available; nat[i] for datagram i (8-byte aligned device array):
 *   dir PICO_CSUM_NAT_OUTBOUND: hdr->src = addr, transport sport = port (:509-510, :525-526)
 *   dir PICO_CSUM_NAT_INBOUND:  hdr->dst = addr, transport dport = port (:446-447, :462-463)
 *   dir PICO_CSUM_NAT_NONE:     left as it is (V_UNTOUCHED; the lookup failed)
 * addr and port as they are stored in the frame (network byte order).  TCP and UDP then get
 * their transport checksum recomputed over the whole transport with the pseudo header of the
 * rewritten header -- UDP too, even if its crc was 0 (:461-465) -- and every translated or ICMPv4
 * datagram its header checksum (:478-481, :543-546); ICMPv4 is not rewritten (:466-468); other
 * protocols are V_UNTOUCHED.  All of it is written in place (V_ACCEPT).  As the reference
 * recomputes rather than adjusts, a wrong stored transport checksum comes out right.
 * A fragment (MF or an offset) is V_FRAG and untouched (it reaches reassembly, not NAT:
 * pico_ipv4.c:446-455); infeasible lengths, or a TCP / UDP transport shorter than its header
 * with a record, are V_MALFORMED and untouched.  d_out_net / d_out_transport: the stored
 * values (0 where none); any output pointer may be NULL.  One pass over each datagram: the
 * rewritten words enter the sums as deltas of the old ones (RFC 1624, on full sums). */
#define PICO_CSUM_NAT_NONE     0u
#define PICO_CSUM_NAT_OUTBOUND 1u
#define PICO_CSUM_NAT_INBOUND  2u
struct pico_csum_nat {
    uint32_t addr;      /* new source (outbound) / destination (inbound) address, as stored */
    uint16_t port;      /* new source / destination port, as stored */
    uint8_t dir;        /* PICO_CSUM_NAT_* */
    uint8_t reserved;
};
int pico_ipv4_nat_batch_dev(void *d_base, uint64_t base_len, const struct pico_csum_desc *d_desc, uint32_t n,
                            const struct pico_csum_nat *d_nat, uint16_t *d_out_net, uint16_t *d_out_transport,
                            uint8_t *d_verdict, void *stream);

/* IPv4 fragment reassembly fused with the transport check of the reassembled datagram
 * (pico_ipv4_process_frag / pico_fragments_check_complete /
 * pico_fragments_reassemble, modules/pico_fragments.c:129-139,216-239,304-358,499-568, then
 * pico_transport_crc_check, stack/pico_socket.c:1916-1968).  One pass reads each fragment's
 * payload once, writes it into the reassembled datagram and sums it; the reference copies
 * it (memcpy, :334-345) and sums the copy again.
 *   d_frag[]   fragments as pico_ipv4_process_in hands them on (desc.off -> the fragment's
 *              IPv4 header, desc.len = bytes available; header already checked)
 *   d_groups[] 2 uint32 per datagram: first fragment, count -- the fragments one reassembly
 *              tree collects (src / dst / id matched by the stack), in arrival order
 *   d_out_desc[] per datagram: output region in d_out (off a multiple of 4, len = capacity;
 *              off = 12 mod 16 puts the transport on a 16-byte line: whole-line stores)
 * Tree order by fragment offset ((frag & 0x1FFF) << 3; a repeated offset keeps the earlier
 * arrival, as pico_tree_insert rejects the later); complete when the offsets are contiguous
 * from 0 up to the first fragment without MF.  The output is the first fragment's 20 header
 * bytes (options are not copied, :332-333) followed by every payload.
 *   d_out_len[g]       transport length of the reassembled datagram, 0 when not reassembled
 *   d_out_transport[g] TCP (always) / UDP (crc != 0) checksum with the pseudo header of the
 *                      copied header (0 = valid; 0 when none is computed)
 *   d_verdict[g]       ACCEPT, L4_BAD, or MALFORMED = not reassembled: incomplete, a fragment
 *                      behind the completing one (the reference's copy loop would write past
 *                      its buffer: reference UB), 20 + len > 65535 (its uint16 allocation size
 *                      wraps), a fragment header or payload past desc.len or base_len, an empty
 *                      group or one of more than 512 fragments, an output region too small.
 * The bytes of an output region are unspecified when its datagram is not reassembled (the
 * gather starts before completeness is known) and past the reassembled datagram's end (a
 * repeated offset's later arrival may have been gathered there); no byte outside the region is
 * written.  Any of the three output pointers may be NULL.  Batches of 512 datagrams or more run
 * on a flat grid whose per-datagram tallies live in library scratch (8 bytes a datagram, kept
 * zero between calls): per calling thread and stream, kept across calls and freed when the
 * thread exits or calls pico_csum_release_thread_scratch; in a call captured into a graph,
 * owned by that graph (freed after the graph is destroyed, by the next eager call or release)
 * -- two executable instances of one captured graph must not run concurrently
 * (pico_csum_set_reasm_flat selects the grid). */
int pico_ipv4_reassemble_batch_dev(const void *d_base, uint64_t base_len, const struct pico_csum_desc *d_frag,
                                   uint32_t n_frag, const uint32_t *d_groups, uint32_t n_dgram, void *d_out,
                                   uint64_t out_len, const struct pico_csum_desc *d_out_desc, uint32_t *d_out_len,
                                   uint16_t *d_out_transport, uint8_t *d_verdict, void *stream);

/* IPv6 fragment reassembly fused with the transport check of the reassembled datagram
 * (pico_ipv6_process_frag / pico_fragments_check_complete /
 * pico_fragments_reassemble, modules/pico_fragments.c:73-83,216-239,304-358,432-498).  Arguments
 * as pico_ipv4_reassemble_batch_dev, with d_frag[] -> each fragment's IPv6 header (desc.len =
 * bytes available; desc.seed reserved, 0): the kernel walks each fragment's extension headers as
 * pico_ipv6_extension_headers does (pico_ipv6.c:659-809) -- the transport must lie behind a
 * fragment header -- for net_len, the fragment field (offset = frag & 0xFFF8, more = frag & 1,
 * pico_fragments.c:35-36) and the transport protocol; transport_len = payload_len - (net_len - 40)
 * (pico_ipv6.c:790).  The output is the first fragment's 40-byte fixed header (its extension
 * headers are not copied, :334-338) followed by every payload (out_desc.off = 8 mod 16 puts the
 * transport on a 16-byte line).  The check of the reassembled datagram follows the module the
 * completing fragment hands it to (its transport protocol): TCP / UDP through
 * pico_transport_crc_check with the reference's byte-9 dispatch on the copied header
 * (PICO_CSUM_F_NXTHDR_DISPATCH: by the module instead), ICMPv6 through pico_icmp6_checksum (a
 * verdict for the ND / MLD types only).  Verdicts and the unspecified-bytes rule as for IPv4
 * (40 + len > 65535 and a fragment that does not walk to a fragment header are MALFORMED). */
int pico_ipv6_reassemble_batch_dev(const void *d_base, uint64_t base_len, const struct pico_csum_desc *d_frag,
                                   uint32_t n_frag, const uint32_t *d_groups, uint32_t n_dgram, void *d_out,
                                   uint64_t out_len, const struct pico_csum_desc *d_out_desc, uint32_t *d_out_len,
                                   uint16_t *d_out_transport, uint8_t *d_verdict, uint32_t flags, void *stream);

/* ---------------------------------------------------------------- layer 3 */

struct pico_csum_ctx;   /* device, three streams and staging slots (the uniform ring alternates two;
                         * staged descriptor batches rotate over three, the third staging buffer
                         * allocated on their first call) */

struct pico_csum_ctx *pico_csum_ctx_create(int device, uint64_t staging_bytes);
void pico_csum_ctx_destroy(struct pico_csum_ctx *ctx);

/* Host-resident uniform batch: frames in host memory (pinned for full PCIe
 * rate, see pico_csum_host_register), results to host memory; returns when
 * d2h of every result has completed. */
int pico_checksum_batch_uniform_host(struct pico_csum_ctx *ctx, const void *base, uint64_t stride,
                                     uint32_t len, uint32_t n, uint32_t seed, uint16_t *out);
/* Host-resident descriptor batches: the TAP / pico_device burst as the stack holds it
 * (frames anywhere in `base`, base_len bytes, descriptors and results in host memory; pin
 * `base` and the outputs with pico_csum_host_register for full PCIe rate).  Consecutive
 * descriptors whose bytes span at most the ctx staging size form a chunk: the span and the
 * rebased descriptors go H2D, the device batch of the same name runs, and only the per-frame
 * results come back (with PICO_CSUM_F_WRITE also the span, crc fields stored); chunk c+1's
 * H2D overlaps chunk c's kernel and D2H on the other stream.  Results, verdicts and error
 * rules are those of the _dev functions; on the staged path a frame larger than the staging
 * buffer is -EINVAL.  With F_WRITE, frames of different chunks must not share bytes (true for a
 * frame ring).  A burst the device addresses directly (page-locked) is read in place instead:
 * pico_csum_set_host_in_place.  Returns when every result is in host memory. */
int pico_checksum_batch_host(struct pico_csum_ctx *ctx, const void *base, uint64_t base_len,
                             const struct pico_csum_desc *desc, uint32_t n, int32_t crc_off, uint32_t flags,
                             uint16_t *out);
int pico_ipv4_checksum_batch_host(struct pico_csum_ctx *ctx, const void *base, uint64_t base_len,
                                  const struct pico_csum_desc *desc, uint32_t n, uint32_t flags, uint16_t *out_net,
                                  uint16_t *out_transport, uint8_t *verdict);
int pico_ipv6_checksum_batch_host(struct pico_csum_ctx *ctx, const void *base, uint64_t base_len,
                                  const struct pico_csum_desc *desc, uint32_t n, uint32_t flags,
                                  uint16_t *out_transport, uint8_t *verdict);
int pico_eth_checksum_batch_host(struct pico_csum_ctx *ctx, const void *base, uint64_t base_len,
                                 const struct pico_csum_desc *desc, uint32_t n, uint32_t flags, const uint8_t *mac,
                                 uint16_t *out_net, uint16_t *out_transport, uint8_t *verdict);
int pico_csum_host_register(void *ptr, uint64_t bytes);
int pico_csum_host_unregister(void *ptr);
/* Zero-copy ingress (the batch form of pico_stack_recv_zerocopy, stack/pico_stack.c:479-527: the
 * driver's buffer is used where it lies): the device's address of registered host memory (NULL and
 * pico_csum_last_error() if ptr is not registered).  Any layer-2 batch takes it as d_base -- and as
 * d_desc / the outputs, registered the same way -- and the kernel then reads the frames over PCIe in
 * place, with no staging copy. */
void *pico_csum_host_device_pointer(void *ptr);

/* ---------------------------------------------------------------- misc */

int pico_csum_abi_version(void);
const char *pico_csum_last_error(void);   /* thread-local, "" when none */

/* Launch-shape override for tests and bench sweeps (all 0 = automatic choice); applies to
 * launches from the calling thread only (thread-local).
 *   group 2: descriptor batches (the sorted-rounds kernel) with fpw frames per wave (1..64);
 *            the other arguments are ignored.
 *   group 4..64 (power of 2): uniform rings -- lanes per frame; cpl = 16-byte chunks per lane
 *            per pass (1,2,4,8; 3 and 5-7 with group >= 8 and pipeline != 1: the pipelined
 *            kernel, frames past its one pass round cpl up to 4 / 8); unroll = frames in flight per group (1,2,4; cpl*unroll <= 8);
 *            fpw = frames per wave (multiple of 64/group, <= 64); nt = 0 auto / 1 plain /
 *            2 non-temporal loads; pipeline = 0 auto / 1 off / 2 on / 3 on with global instead
 *            of buffer-window loads (frames that fit one pass: double-buffered frame sets).
 * A group for the other batch kind makes the batch call return -EINVAL. */
int pico_csum_set_launch_override(uint32_t group, uint32_t cpl, uint32_t unroll, uint32_t fpw, uint32_t nt,
                                  uint32_t pipeline);

/* Host-resident descriptor batches (pico_*_batch_host), per calling thread: 1 (the default) = a
 * burst whose whole [base, base + base_len) the device addresses directly -- page-locked by
 * hipHostMalloc or pico_csum_host_register -- is read (and with F_WRITE written) in place by the
 * kernel, only descriptors and results staged, and nothing staged when the descriptor and result
 * arrays are device-addressable too (then frames larger than the staging buffer are fine);
 * 0 = always through the staging buffers.  Results never depend on it. */
int pico_csum_set_host_in_place(uint32_t on);

/* Tuning knob (tests / bench sweeps), per calling thread: the uniform rings' stream waves
 * (pico_checksum_batch_uniform_dev / _host on densely packed frames) -- mode 0 = automatic, 1 = on
 * wherever the ring allows them, PICO_CSUM_STREAM_OFF = the lane-group kernels; frames_per_wave
 * 0 = automatic.  Results never depend on it. */
#define PICO_CSUM_STREAM_OFF 0xFFu
int pico_csum_set_uniform_stream(uint32_t mode, uint32_t frames_per_wave);

/* Tuning knob (tests / bench sweeps), per calling thread: the reassembly batches' flat grid
 * (pico_ipv4_reassemble_batch_dev / pico_ipv6_reassemble_batch_dev) -- 0 = automatic (batches
 * of 512 datagrams or more), 1 = always, 2 = never (one workgroup per datagram).  Results never
 * depend on it. */
int pico_csum_set_reasm_flat(uint32_t mode);

/* Frees the calling thread's reassembly scratch (the flat grid's tallies, one buffer per stream
 * the thread launched on) and the scratch of captured graphs destroyed since; the thread's next
 * flat-grid call allocates again.  A thread's scratch is also freed when the thread exits.  Call
 * it with no reassembly of this thread still running on the device (hipFree waits for the device).
 * Returns 0, or -PICO_CSUM_ENODEV without a device. */
int pico_csum_release_thread_scratch(void);

#ifdef __cplusplus
}
#endif
#endif /* PICO_CSUM_H */

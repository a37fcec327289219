/*
 * ref_rx_driver.c -- TEST INFRASTRUCTURE ONLY.
 *
 * Runs the reference's own RX decisions on single datagrams, so the fused RX verdicts of the
 * oracle and of the HIP kernels are pinned to the reference itself (VERDICT r02 "next" 1 and 3):
 * oracle/_ref/libref_rx.so = the reference stack compiled from /root/reference (stack/*.c and
 * the IPv4 / IPv6 / ICMP / TCP / UDP / fragment / MLD / IGMP / multicast / null-device modules)
 * with pico_ipv4.c, pico_ipv6.c, pico_socket.c, pico_fragments.c and pico_ethernet.c reached
 * through ref_rx_wrap.c.  The link uses
 * --wrap so that this file OBSERVES the hand-offs of pico_ipv4_process_in /
 * pico_ipv6_extension_headers without changing any reference code:
 *   __wrap_pico_ipv4_process_frag / __wrap_pico_ipv6_process_frag   -> "handed to reassembly"
 *   __wrap_pico_transport_receive                                    -> "delivered to proto"
 *   __wrap_pico_arp_receive                                          -> "handed to ARP"
 * (a delivered frame is kept for the transport check, rr_transport_crc_check, or discarded).
 *
 * rr_ipv4_rx(datagram, avail): a frame with net_hdr at the buffer start and buffer_len = avail
 *   (allocated larger, zero-filled behind avail) goes through pico_ipv4_process_in on a null
 *   device that owns one /24 IPv4 link per destination added with rr_ipv4_link.  Result bits:
 *     1 FRAG seen, 2 delivered (protocol in bits 8-15; the UDP / ICMPv4 broadcast enqueues of
 *     pico_ipv4_process_bcast_in count as delivered), 4 transport check passed (TCP / UDP
 *     delivered), 16 the header checksum passed (pico_ipv4_crc_check on a copy with
 *     f->net_len = 20 + 4 (IHL - 5) as :394-400 sets it).
 * rr_ipv6_rx(datagram, avail, &net_len, &proto): pico_ipv6_extension_headers on the frame;
 *   returns 0 discarded, 1 transport reached (net_len / proto = f->net_len and the returned
 *   protocol), 2 handed to pico_ipv6_process_frag; for 1 with TCP / UDP, bit 4 = the transport
 *   check (pico_transport_crc_check, with f->transport_hdr / transport_len as the walk set them)
 *   passed.
 * rr_reasm(v6, base, offs, lens, n, out, cap, &len, &module, &check): the n fragments of one
 *   datagram, in arrival order, through pico_ipv4_process_in / pico_ipv6_extension_headers with
 *   the REAL pico_ipv4/6_process_frag (tree, completeness, pico_fragments_reassemble), the trees
 *   reset first; returns 1 when pico_fragments_reassemble handed a datagram to
 *   pico_transport_receive (its net_len + transport_len bytes copied to out, len =
 *   transport_len, module = the protocol it was handed with, check = pico_transport_crc_check
 *   on it for TCP / UDP, else -1), 0 when none was reassembled.
 * rr_eth_init(mac) / rr_eth_rx(frame, avail): pico_ethernet_receive on an Ethernet device with
 *   that MAC; returns 1 queued for IPv4, 2 queued for IPv6, 3 handed to ARP, 0 discarded.
 * rr_nat(dir, datagram, avail, nat_addr): pico_ipv4_nat_outbound (dir 1) or pico_ipv4_nat_inbound
 *   (dir 2) (modules/pico_nat.c:424-545) on the datagram as pico_ipv4_process_in leaves it
 *   (net_len, transport_hdr, transport_len :392-405), NAT enabled on the link nat_addr (from the
 *   first call on; tuples persist: an inbound reply finds the outbound's tuple); the frame's
 *   bytes after the call are copied back.  Returns the function's result (0 translated).
 * rr_forward(datagram, avail): pico_ipv4_pre_forward_checks (modules/pico_ipv4.c:1535-1574) on the
 *   datagram with the stack's links as added by rr_ipv4_link (pico_ipv4_link_get's table); its
 *   static last-forwarded state persists between calls (a fresh library copy starts at the
 *   reference's zero state).  The bytes after the call are copied back.  Returns 0 forwarded,
 *   1 TTL expired (:1549-1553), 2 local source (:1559-1560), 3 duplicate of the last forwarded
 *   datagram (:1562-1565).
 * rr_stack_rx(frame, len) / rr_take_delivered(&check): one frame in at the driver boundary --
 *   pico_stack_recv (stack/pico_stack.c:465-477) on the Ethernet device of rr_eth_init -- then the
 *   receive loops below the transport layer that pico_stack_tick runs (pico_devices_loop,
 *   pico_protocol_datalink_loop, pico_protocol_network_loop, :766-773), so the frame goes through
 *   pico_ethernet_receive, pico_ipv4_process_in / pico_ipv6_process_in (routing included) and, if
 *   delivered, stops at the transport hand-off; rr_take_delivered returns that frame's protocol
 *   (-1 none) and, for TCP / UDP, pico_transport_crc_check on it in *check (a CRC=0 build: the
 *   no-op variant, always 1).  rr_ipv6_link adds a non-tentative /64 IPv6 link (DAD done:
 *   pico_ipv6_link_add_no_dad) so unicast IPv6 to it is local.  The batched-driver test
 *   (tests/test_burst_driver.py) runs this in a CRC=1 and a CRC=0 build of the stack.
 *   rr_take_forwarded: 1 when that frame was routed on instead (pico_ipv4_forward /
 *   pico_ipv6_forward reached pico_datalink_send or an ICMP notice), 0 otherwise.
 * Callers (tests/golden/make_ref_rx.py, make_ref_reasm.py, make_ref_eth.py, make_ref_nat.py) only pass datagrams whose reference reads stay inside
 * avail and whose walk terminates (the oracle restatement decides which; the others are
 * restatement-only and documented so).
 */
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include "pico_stack.h"
#include "pico_frame.h"
#include "pico_device.h"
#include "pico_ipv4.h"
#include "pico_ipv6.h"
#include "pico_udp.h"
#include "pico_icmp4.h"
#include "pico_queue.h"
#include "pico_dev_null.h"
#include "pico_nat.h"
#include "pico_protocol.h"
#include "pico_socket.h"

int rr_ipv4_process_in(struct pico_frame *f);
int rr_ipv4_crc_check(struct pico_frame *f);
int rr_ipv4_pre_forward_checks(struct pico_frame *f);
int rr_ipv6_ext_headers(struct pico_frame *f);
int rr_transport_crc_check(struct pico_frame *f);
void rr_frag_reset(void);

void __real_pico_ipv4_process_frag(struct pico_ipv4_hdr *hdr, struct pico_frame *f, uint8_t proto);
void __real_pico_ipv6_process_frag(struct pico_ipv6_exthdr *frag, struct pico_frame *f, uint8_t proto);
int32_t __real_pico_transport_receive(struct pico_frame *f, uint8_t proto);
void __wrap_pico_ipv4_process_frag(struct pico_ipv4_hdr *hdr, struct pico_frame *f, uint8_t proto);
void __wrap_pico_ipv6_process_frag(struct pico_ipv6_exthdr *frag, struct pico_frame *f, uint8_t proto);
int32_t __wrap_pico_transport_receive(struct pico_frame *f, uint8_t proto);
int __wrap_pico_arp_receive(struct pico_frame *f);
int __real_pico_notify_dest_unreachable(struct pico_frame *f);
int __real_pico_notify_ttl_expired(struct pico_frame *f);
int __real_pico_notify_pkt_too_big(struct pico_frame *f);
int32_t __real_pico_datalink_send(struct pico_frame *f);
int __wrap_pico_notify_dest_unreachable(struct pico_frame *f);
int __wrap_pico_notify_ttl_expired(struct pico_frame *f);
int __wrap_pico_notify_pkt_too_big(struct pico_frame *f);
int32_t __wrap_pico_datalink_send(struct pico_frame *f);
int rr_take_forwarded(void);
int rr_tx_capture(uint8_t *buf, uint32_t cap, uint32_t *lens, uint32_t maxn);
int rr_real_transport(int on);
void *rr_socket(int proto, uint32_t addr, uint16_t port_be, int listen);
int rr_sendto(void *s, const uint8_t *data, int len, uint32_t dst, uint16_t port_be);
void *rr_accept(void *s);
int rr_write(void *s, const uint8_t *data, int len);
void rr_tick(int n);
int32_t rr_ethernet_receive(struct pico_frame *f);
int rr_eth_init(const uint8_t *mac);
int rr_eth_rx(const uint8_t *d, uint32_t avail);

int rr_init(void);
int rr_ipv4_link(uint32_t addr);
int rr_ipv4_rx(const uint8_t *d, uint32_t avail);
int rr_nat(int dir, uint8_t *d, uint32_t avail, uint32_t nat_addr);
int rr_forward(uint8_t *d, uint32_t avail);
int rr_ipv6_link(const uint8_t *addr16);
void *rr_eth_dev(void);
int rr_stack_rx(const uint8_t *frame, uint32_t len);
int rr_take_delivered(int *check);
int rr_ipv6_rx(const uint8_t *d, uint32_t avail, uint32_t *net_len, uint32_t *proto);
int rr_reasm(int v6, const uint8_t *base, const uint64_t *offs, const uint32_t *lens, uint32_t n, uint8_t *out,
             uint32_t cap, uint32_t *out_len, uint32_t *module, int *check);
int rr_reasm_batch(int v6, const uint8_t *base, const uint64_t *offs, const uint32_t *lens, const uint32_t *groups,
                   uint32_t n_dgram, uint32_t *checked);

static struct pico_device *g_dev, *g_edev;
static int g_arp;
static int g_frag, g_deliv_proto;
static struct pico_frame *g_deliv;
static int g_forward;          /* 1: call the real hand-offs (reassembly runs) */
static int g_routed;           /* the frame entered a forwarding path (see the wrappers below) */
static int g_real_l4;          /* 1: pico_transport_receive runs for real (the TX capture) */
static uint8_t *g_cap;         /* TX capture: datagrams handed to pico_datalink_send */
static uint32_t g_cap_cap, g_cap_used, g_cap_n, g_cap_max, *g_cap_len;

void __wrap_pico_ipv4_process_frag(struct pico_ipv4_hdr *hdr, struct pico_frame *f, uint8_t proto)
{
    g_frag = 1;
    if (g_forward)
        __real_pico_ipv4_process_frag(hdr, f, proto);
}

void __wrap_pico_ipv6_process_frag(struct pico_ipv6_exthdr *frag, struct pico_frame *f, uint8_t proto)
{
    g_frag = 1;
    if (g_forward)
        __real_pico_ipv6_process_frag(frag, f, proto);
}

int32_t __wrap_pico_transport_receive(struct pico_frame *f, uint8_t proto)
{
    if (g_real_l4)
        return __real_pico_transport_receive(f, proto);
    if (g_deliv)
        pico_frame_discard(g_deliv);
    g_deliv = f;
    g_deliv_proto = proto;
    return 0;
}

/* Routing is observed where pico_ipv4_forward / pico_ipv6_forward (modules/pico_ipv4.c:1589-1617,
 * modules/pico_ipv6.c:495-521) end: the datagram goes out (pico_datalink_send) or the stack gives
 * up on it with an ICMP notification (no route, TTL / hop limit expired, too big).  The real
 * functions still run; the wrappers only note that the frame was routed, not delivered. */
int __wrap_pico_notify_dest_unreachable(struct pico_frame *f)
{
    g_routed = 1;
    return __real_pico_notify_dest_unreachable(f);
}

int __wrap_pico_notify_ttl_expired(struct pico_frame *f)
{
    g_routed = 1;
    return __real_pico_notify_ttl_expired(f);
}

int __wrap_pico_notify_pkt_too_big(struct pico_frame *f)
{
    g_routed = 1;
    return __real_pico_notify_pkt_too_big(f);
}

int32_t __wrap_pico_datalink_send(struct pico_frame *f)
{
    g_routed = 1;
    if (g_cap && g_cap_n < g_cap_max && f->net_hdr) {
        /* the IP datagram as the stack hands it to the link layer (its length from its own header) */
        const uint8_t *ip = f->net_hdr;
        const uint32_t v = ip[0] >> 4;
        const uint32_t len = v == 4u ? ((uint32_t)ip[2] << 8 | ip[3]) : v == 6u ? 40u + ((uint32_t)ip[4] << 8 | ip[5]) : 0u;
        if (len && g_cap_used + len <= g_cap_cap) {
            memcpy(g_cap + g_cap_used, ip, len);
            g_cap_used += len;
            g_cap_len[g_cap_n++] = len;
        }
    }
    return __real_pico_datalink_send(f);
}

/* ARP frames the Ethernet layer hands on are counted, not processed */
int __wrap_pico_arp_receive(struct pico_frame *f)
{
    g_arp = 1;
    pico_frame_discard(f);
    return 0;
}

static int eth_send(struct pico_device *dev, void *buf, int len)
{
    (void)dev;
    (void)buf;
    return len;
}

int rr_init(void)
{
    if (g_dev)
        return 0;
    /* the reference's dbg() is printf (include/arch/pico_posix.h:19): unbuffered, so its lines
     * reach fd 1 at once (a test runner's capture) instead of a buffer flushed at exit */
    setvbuf(stdout, NULL, _IONBF, 0);
    if (pico_stack_init() != 0)
        return -1;
    g_dev = pico_null_create("rr0");
    return g_dev ? 0 : -1;
}

int rr_ipv4_link(uint32_t addr)
{
    struct pico_ip4 a, m;
    a.addr = addr;
    m.addr = 0x00FFFFFFu;    /* 255.255.255.0: only x.y.z.255 of the link's /24 is a broadcast */
    return pico_ipv4_link_add(g_dev, a, m);
}

#define RR_PAD 70000u   /* zero bytes behind avail: a read past avail is defined (callers avoid it) */

static int g_lean;              /* rr_reasm_batch: frames as a driver allocates them, no padding */

static struct pico_frame *mk(const uint8_t *d, uint32_t avail)
{
    const uint32_t pad = g_lean ? 0u : RR_PAD;
    struct pico_frame *f = pico_frame_alloc(avail + pad);
    if (!f)
        return NULL;
    if (pad)
        memset(f->buffer, 0, avail + pad);
    memcpy(f->buffer, d, avail);
    f->buffer_len = avail;
    f->start = f->buffer;
    f->len = avail;
    f->datalink_hdr = f->buffer;
    f->net_hdr = f->buffer;
    f->transport_hdr = NULL;
    f->dev = g_dev;
    return f;
}

/* the delivered frame of the last call, if any: its transport check for TCP / UDP */
static int delivered_check(void)
{
    int ok = 0;
    struct pico_frame *f = g_deliv;
    g_deliv = NULL;
    if (!f)
        return 0;
    if (g_deliv_proto == 6 || g_deliv_proto == 17) {
        ok = rr_transport_crc_check(f);      /* discards f when it fails */
        if (ok)
            pico_frame_discard(f);
    } else {
        pico_frame_discard(f);
    }
    return ok;
}

int rr_ipv4_rx(const uint8_t *d, uint32_t avail)
{
    struct pico_frame *f, *c;
    struct pico_frame *q;
    int r = 0;
    if (!g_dev || avail < 20)
        return -1;
    /* the header check alone, on a copy (net_len as pico_ipv4_process_in :394-400 sets it) */
    c = mk(d, avail);
    if (!c)
        return -1;
    c->net_len = (uint16_t)(20u + ((d[0] & 0x0Fu) > 5u ? 4u * ((d[0] & 0x0Fu) - 5u) : 0u));
    if (rr_ipv4_crc_check(c)) {
        r |= 16;
        pico_frame_discard(c);
    }
    f = mk(d, avail);
    if (!f)
        return -1;
    g_frag = 0;
    g_deliv = NULL;
    rr_ipv4_process_in(f);
    if (g_frag)
        r |= 1;
    /* pico_ipv4_process_bcast_in / _local_unicast_in enqueue UDP and ICMPv4 directly (:299,
     * :309, :359) */
    while ((q = pico_dequeue(pico_proto_udp.q_in)) != NULL) {
        if (g_deliv)
            pico_frame_discard(g_deliv);
        g_deliv = q;
        g_deliv_proto = 17;
    }
    while ((q = pico_dequeue(pico_proto_icmp4.q_in)) != NULL) {
        if (g_deliv)
            pico_frame_discard(g_deliv);
        g_deliv = q;
        g_deliv_proto = 1;
    }
    if (g_deliv) {
        r |= 2 | (g_deliv_proto << 8);
        if (delivered_check())
            r |= 4;
    }
    return r;
}

int rr_ipv6_rx(const uint8_t *d, uint32_t avail, uint32_t *net_len, uint32_t *proto)
{
    struct pico_frame *f;
    int ret, r;
    if (avail < 40)
        return -1;
    f = mk(d, avail);
    if (!f)
        return -1;
    g_frag = 0;
    ret = rr_ipv6_ext_headers(f);
    *net_len = f->net_len;
    *proto = ret > 0 ? (uint32_t)ret : 0u;
    if (g_frag) {
        pico_frame_discard(f);
        return 2;
    }
    if (ret <= 0) {
        pico_frame_discard(f);
        return 0;
    }
    r = 1;
    if (ret == 6 || ret == 17) {
        /* what pico_transport_receive hands on: net_hdr, transport_hdr, transport_len as set */
        if (rr_transport_crc_check(f)) {
            r |= 4;
            pico_frame_discard(f);
        }
    } else {
        pico_frame_discard(f);
    }
    return r;
}

int rr_reasm(int v6, const uint8_t *base, const uint64_t *offs, const uint32_t *lens, uint32_t n, uint8_t *out,
             uint32_t cap, uint32_t *out_len, uint32_t *module, int *check)
{
    uint32_t i;
    struct pico_frame *full, *q;
    if (!g_dev)
        return -1;
    rr_frag_reset();
    if (g_deliv) {
        pico_frame_discard(g_deliv);
        g_deliv = NULL;
    }
    g_forward = 1;
    for (i = 0; i < n; i++) {
        struct pico_frame *f = mk(base + offs[i], lens[i]);
        if (!f)
            break;
        if (v6) {
            if (rr_ipv6_ext_headers(f) > 0 && f != g_deliv)   /* not a fragment: not ours to keep */
                pico_frame_discard(f);
            else if (f != g_deliv)
                pico_frame_discard(f);                       /* handed on as a copy, or dropped */
        } else {
            rr_ipv4_process_in(f);                           /* discards f itself */
            while ((q = pico_dequeue(pico_proto_udp.q_in)) != NULL)
                pico_frame_discard(q);
            while ((q = pico_dequeue(pico_proto_icmp4.q_in)) != NULL)
                pico_frame_discard(q);
        }
    }
    g_forward = 0;
    full = g_deliv;
    g_deliv = NULL;
    rr_frag_reset();
    if (!full)
        return 0;
    *out_len = full->transport_len;
    *module = (uint32_t)g_deliv_proto;
    if (out && (uint32_t)full->net_len + full->transport_len <= cap)
        memcpy(out, full->net_hdr, (size_t)full->net_len + full->transport_len);
    if (g_deliv_proto == 6 || g_deliv_proto == 17) {
        *check = rr_transport_crc_check(full);               /* discards full when it fails */
        if (*check)
            pico_frame_discard(full);
    } else {
        *check = -1;
        pico_frame_discard(full);
    }
    return 1;
}

/* rr_reasm over n_dgram datagrams (groups: first fragment, count per datagram), nothing copied
 * out: the reference's fragment path as a timed CPU baseline (bench.py) -- each fragment copied
 * into a frame of its own size as pico_stack_recv does (not the padded, zero-filled frames the
 * fixture runs use) -- with one
 * pico_stack_tick per datagram as the stack's main loop runs it (it retires the cancelled
 * expiry timers, which would otherwise pile up in the timer heap).  Returns the number of
 * datagrams reassembled; *checked = how many of them passed pico_transport_crc_check. */
int rr_reasm_batch(int v6, const uint8_t *base, const uint64_t *offs, const uint32_t *lens, const uint32_t *groups,
                   uint32_t n_dgram, uint32_t *checked)
{
    uint32_t g, done = 0, ok = 0, len, module;
    int check;
    g_lean = 1;                 /* (well-formed batches: no read past a fragment's bytes) */
    for (g = 0; g < n_dgram; g++) {
        const uint32_t first = groups[2 * g], cnt = groups[2 * g + 1];
        check = 0;
        if (rr_reasm(v6, base, offs + first, lens + first, cnt, NULL, 0, &len, &module, &check) == 1) {
            done++;
            ok += check == 1;
        }
        pico_stack_tick();
    }
    g_lean = 0;
    *checked = ok;
    return (int)done;
}

/* An Ethernet device with the given MAC (pico_device_init with a MAC allocates dev->eth). */
int rr_eth_init(const uint8_t *mac)
{
    if (rr_init() != 0)
        return -1;
    if (g_edev)
        return 0;
    g_edev = PICO_ZALLOC(sizeof(struct pico_device));
    if (!g_edev || pico_device_init(g_edev, "rr1", mac) != 0)
        return -1;
    g_edev->send = eth_send;
    return 0;
}

/*
 * pico_ethernet_receive on one frame of `avail` bytes (the datalink header at d): 1 = handed to
 * IPv4 (pico_proto_ipv4.q_in), 2 = to IPv6, 3 = to ARP, 0 = discarded by the Ethernet layer.
 */
int rr_eth_rx(const uint8_t *d, uint32_t avail)
{
    struct pico_frame *f, *q;
    int r = 0;
    if (!g_edev || avail < 14)
        return -1;
    f = mk(d, avail);
    if (!f)
        return -1;
    f->dev = g_edev;
    g_arp = 0;
    rr_ethernet_receive(f);
    if ((q = pico_dequeue(pico_proto_ipv4.q_in)) != NULL) {
        r = 1;
        pico_frame_discard(q);
    }
    if ((q = pico_dequeue(pico_proto_ipv6.q_in)) != NULL) {
        r = 2;
        pico_frame_discard(q);
    }
    if (g_arp)
        r = 3;
    return r;
}

int rr_nat(int dir, uint8_t *d, uint32_t avail, uint32_t nat_addr)
{
    struct pico_frame *f;
    struct pico_ip4 a;
    struct pico_ipv4_link *link;
    uint32_t net_len;
    int r;
    if (!g_dev || avail < 20 || (dir != 1 && dir != 2))
        return -2;
    a.addr = nat_addr;
    link = pico_ipv4_link_get(&a);
    if (!link && rr_ipv4_link(nat_addr) == 0)
        link = pico_ipv4_link_get(&a);
    if (!link)
        return -2;
    /* enabled once per process (each pico_ipv4_nat_enable adds a cleanup timer); callers load a
     * private copy of this library for NAT, so no other fixture sees the link */
    if (!pico_ipv4_nat_is_enabled(&a) && pico_ipv4_nat_enable(link) != 0)
        return -2;
    f = mk(d, avail);
    if (!f)
        return -2;
    net_len = 20u + ((d[0] & 0x0Fu) > 5u ? 4u * ((d[0] & 0x0Fu) - 5u) : 0u);
    f->net_len = (uint16_t)net_len;
    f->transport_hdr = f->net_hdr + net_len;
    f->transport_len = (uint16_t)(((uint32_t)d[2] << 8 | d[3]) - net_len);
    r = dir == 1 ? pico_ipv4_nat_outbound(f, &a) : pico_ipv4_nat_inbound(f, &a);
    memcpy(d, f->buffer, avail);
    pico_frame_discard(f);
    return r;
}

int rr_forward(uint8_t *d, uint32_t avail)
{
    struct pico_frame *f;
    struct pico_ip4 src;
    int r;
    if (!g_dev || avail < 20)
        return -2;
    f = mk(d, avail);
    if (!f)
        return -2;
    f->net_len = 20;
    r = rr_ipv4_pre_forward_checks(f);
    memcpy(d, f->buffer, avail);
    pico_frame_discard(f);
    if (r == 0)
        return 0;
    /* which discard: the TTL byte after the call is 0 only when it expired (crc untouched);
     * else the source lookup (the same table the call consulted), else the duplicate rule */
    if (d[8] == 0)
        return 1;
    memcpy(&src.addr, d + 12, 4);
    return pico_ipv4_link_get(&src) ? 2 : 3;
}

int rr_ipv6_link(const uint8_t *addr16)
{
    struct pico_ip6 a, m;
    if (!g_dev)
        return -1;
    memcpy(a.addr, addr16, 16);
    memset(m.addr, 0, 16);
    memset(m.addr, 0xFF, 8);
    return pico_ipv6_link_add_no_dad(g_dev, a, m) ? 0 : -1;
}

void *rr_eth_dev(void) { return g_edev; }

int rr_stack_rx(const uint8_t *frame, uint32_t len)
{
    int k, r;
    if (!g_edev)
        return -2;
    if (g_deliv) {
        pico_frame_discard(g_deliv);
        g_deliv = NULL;
    }
    g_frag = 0;
    g_arp = 0;
    g_routed = 0;
    r = pico_stack_recv(g_edev, (uint8_t *)frame, len);
    for (k = 0; k < 3; k++) {
        pico_devices_loop(64, PICO_LOOP_DIR_IN);
        pico_protocol_datalink_loop(64, PICO_LOOP_DIR_IN);
        pico_protocol_network_loop(64, PICO_LOOP_DIR_IN);
    }
    return r;
}

int rr_take_delivered(int *check)
{
    struct pico_frame *q;
    int proto;
    /* the UDP / ICMPv4 enqueues of pico_ipv4_process_bcast_in / _local_unicast_in (:299, :309, :359) */
    while ((q = pico_dequeue(pico_proto_udp.q_in)) != NULL) {
        if (g_deliv)
            pico_frame_discard(g_deliv);
        g_deliv = q;
        g_deliv_proto = 17;
    }
    while ((q = pico_dequeue(pico_proto_icmp4.q_in)) != NULL) {
        if (g_deliv)
            pico_frame_discard(g_deliv);
        g_deliv = q;
        g_deliv_proto = 1;
    }
    *check = -1;
    if (!g_deliv)
        return -1;
    proto = g_deliv_proto;
    if (proto == 6 || proto == 17)
        *check = delivered_check();
    else {
        pico_frame_discard(g_deliv);
        g_deliv = NULL;
    }
    return proto;
}

/* 1 when the last rr_stack_rx frame was routed on (forwarded, or given up with an ICMP notice). */
int rr_take_forwarded(void)
{
    int r = g_routed;
    g_routed = 0;
    return r;
}

/*
 * The TX capture (tests/test_ref_tx.py): the frames the CRC=1 stack itself emits -- TCP from
 * tcp_send (modules/pico_tcp.c:968-985: SYN-ACKs, RSTs, data segments of an accepted connection),
 * UDP from pico_udp_push (crc 0, :120), ICMPv4 echo replies (pico_icmp4_checksum, modules/
 * pico_icmp4.c:30-41), each behind pico_ipv4_frame_push's header checksum (modules/pico_ipv4.c:1079)
 * -- recorded where they reach pico_datalink_send.  rr_real_transport(1) lets received segments
 * reach the real transport layer (the RX fixtures intercept it); rr_socket / rr_sendto /
 * rr_accept / rr_write are the public socket API; rr_tick runs pico_stack_tick.
 */
int rr_tx_capture(uint8_t *buf, uint32_t cap, uint32_t *lens, uint32_t maxn)
{
    const int n = (int)g_cap_n;
    g_cap = buf;
    g_cap_cap = cap;
    g_cap_len = lens;
    g_cap_max = maxn;
    g_cap_used = 0;
    g_cap_n = 0;
    return n;
}

int rr_real_transport(int on)
{
    g_real_l4 = on;
    return 0;
}

static void rr_wakeup(uint16_t ev, struct pico_socket *s)
{
    (void)ev;
    (void)s;
}

void *rr_socket(int proto, uint32_t addr, uint16_t port_be, int listen)
{
    struct pico_socket *s = pico_socket_open(PICO_PROTO_IPV4, (uint16_t)proto, rr_wakeup);
    struct pico_ip4 a;
    uint16_t port = port_be;
    if (!s)
        return NULL;
    a.addr = addr;
    if (pico_socket_bind(s, &a, &port) != 0 || (listen && pico_socket_listen(s, 8) != 0)) {
        pico_socket_close(s);
        return NULL;
    }
    return s;
}

int rr_sendto(void *s, const uint8_t *data, int len, uint32_t dst, uint16_t port_be)
{
    struct pico_ip4 a;
    a.addr = dst;
    return pico_socket_sendto((struct pico_socket *)s, data, len, &a, port_be);
}

void *rr_accept(void *s)
{
    struct pico_ip4 orig;
    uint16_t port = 0;
    return pico_socket_accept((struct pico_socket *)s, &orig, &port);
}

int rr_write(void *s, const uint8_t *data, int len)
{
    return pico_socket_write((struct pico_socket *)s, data, len);
}

void rr_tick(int n)
{
    int k;
    for (k = 0; k < n; k++)
        pico_stack_tick();
}

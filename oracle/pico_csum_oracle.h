/* TEST INFRASTRUCTURE ONLY -- see pico_csum_oracle.c.  Never linked into the product. */
#ifndef PICO_CSUM_ORACLE_H
#define PICO_CSUM_ORACLE_H
#include <stdint.h>

#ifndef PICO_CSUM_DESC_DEFINED
#define PICO_CSUM_DESC_DEFINED
/* Same 16-byte layout as include/pico_csum.h (kept separate on purpose). */
struct pico_csum_desc {
    uint64_t off;
    uint32_t len;
    uint32_t seed;
};
#endif

#define PICO_CSUM_V_ACCEPT    1u
#define PICO_CSUM_V_NET_BAD   2u
#define PICO_CSUM_V_L4_BAD    4u
#define PICO_CSUM_V_MALFORMED 8u
#define PICO_CSUM_V_EXPIRED  16u   /* forwarding batch */
#define PICO_CSUM_V_LOCAL_SRC 32u  /* forwarding batch */
#define PICO_CSUM_V_DUPLICATE 64u  /* forwarding batch */
#define PICO_CSUM_V_FRAG     16u   /* RX / TX batches: a fragment (same bit, other batches) */
#define PICO_CSUM_V_DROP_L2  32u
#define PICO_CSUM_V_ARP      64u
#define PICO_CSUM_V_IPV6    128u
#define PICO_CSUM_V_UNTOUCHED 32u  /* NAT batch */

/* Same 8-byte layout as include/pico_csum.h struct pico_csum_nat. */
struct oracle_nat {
    uint32_t addr;
    uint16_t port;
    uint8_t dir;        /* 0 none, 1 outbound (src, sport), 2 inbound (dst, dport) */
    uint8_t reserved;
};

#define ORACLE_IPV4_TX 1u
/* IPv6 RX: check TCP / UDP by the transport's own protocol (PICO_CSUM_F_NXTHDR_DISPATCH);
 * without it, pico_transport_crc_check's byte-9 dispatch (the reference's behaviour) */
#define ORACLE_NXTHDR_DISPATCH 4u

/* pico_ipv6_extension_headers outcome (oracle_ipv6_walk) */
#define ORACLE_WALK_DROP  0   /* the reference discards the datagram */
#define ORACLE_WALK_PROTO 1   /* transport reached: *net_len, *proto */
#define ORACLE_WALK_FRAG  2   /* transport reached behind a fragment header: handed to reassembly */
#define ORACLE_WALK_BAD  -1   /* the reference would read past the frame, or never terminates */
int oracle_ipv6_walk(const uint8_t *h, uint32_t avail, uint32_t *net_len, uint8_t *proto);
int oracle_ipv6_walk_frag(const uint8_t *h, uint32_t avail, uint32_t *net_len, uint8_t *proto, uint16_t *frag);

typedef uint16_t (*oracle_checksum_fn)(void *buf, uint32_t len);

uint32_t oracle_checksum_adder(uint32_t sum, const void *data, uint32_t len);
uint16_t oracle_checksum_finalize(uint32_t sum);
uint16_t oracle_checksum(const void *buf, uint32_t len);
uint16_t oracle_dualbuffer_checksum(const void *b1, uint32_t len1, const void *b2, uint32_t len2);
uint32_t oracle_ipv4_pseudo_sum(const uint8_t src[4], const uint8_t dst[4], uint8_t proto, uint16_t transport_len);
void oracle_batch_raw(const uint8_t *base, const struct pico_csum_desc *d, uint32_t n,
                      uint16_t *out, int32_t crc_off);
void oracle_batch_uniform(const uint8_t *base, uint64_t stride, uint32_t len, uint32_t n,
                          uint32_t seed, uint16_t *out);
void oracle_batch_ipv4(const uint8_t *base, const struct pico_csum_desc *d, uint32_t n,
                       uint16_t *out_net, uint16_t *out_l4, uint8_t *verdict, uint32_t flags);
uint32_t oracle_ipv6_pseudo_sum(const uint8_t src[16], const uint8_t dst[16], uint8_t nxthdr, uint32_t transport_len);
void oracle_batch_ipv6(const uint8_t *base, const struct pico_csum_desc *d, uint32_t n,
                       uint16_t *out_l4, uint8_t *verdict, uint32_t flags);
void oracle_batch_eth(const uint8_t *base, const struct pico_csum_desc *d, uint32_t n, const uint8_t *mac,
                      uint16_t *out_net, uint16_t *out_l4, uint8_t *verdict, uint32_t flags);
void oracle_ipv4_reassemble(const uint8_t *base, const struct pico_csum_desc *d, uint32_t nd, const uint32_t *grp,
                            uint32_t ng, uint8_t *out, const struct pico_csum_desc *od, uint32_t *out_len, uint16_t *out_l4,
                            uint8_t *verdict);
void oracle_ipv6_reassemble(const uint8_t *base, const struct pico_csum_desc *d, uint32_t nd, const uint32_t *grp,
                            uint32_t ng, uint8_t *out, const struct pico_csum_desc *od, uint32_t *out_len, uint16_t *out_l4,
                            uint8_t *verdict, uint32_t flags);
/* pico_ipv4_pre_forward_checks' static last tuple (modules/pico_ipv4.c:1537-1544), as stored */
struct oracle_fwd_state {
    uint32_t src;
    uint32_t dst;
    uint16_t id;
    uint16_t proto;
    uint32_t reserved;
};
void oracle_batch_ipv4_forward(uint8_t *base, const struct pico_csum_desc *d, uint32_t n, const uint32_t *local,
                               uint32_t n_local, struct oracle_fwd_state *st, uint8_t *verdict);
void oracle_batch_ipv4_nat(uint8_t *base, const struct pico_csum_desc *d, uint32_t n, const struct oracle_nat *rw,
                           uint16_t *out_net, uint16_t *out_l4, uint8_t *verdict);
double oracle_uniform_mt(oracle_checksum_fn fn, const uint8_t *base, uint64_t stride, uint32_t len,
                         uint32_t n, uint16_t *out, uint32_t nthreads);
#endif

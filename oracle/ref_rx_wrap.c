/*
 * ref_rx_wrap.c -- TEST INFRASTRUCTURE ONLY.
 *
 * One of five translation units that compile an UNMODIFIED reference source file together
 * with a few exported accessors for its static functions (the technique of the reference's
 * own module tests, test/unit/modunit_*.c, which #include the module they test).  Built by
 * oracle/Makefile (`make refrx`) five times, once per REF_RX_UNIT:
 *   1: modules/pico_ipv4.c   rr_ipv4_process_in  = pico_ipv4_process_in   (:381-470)
 *                            rr_ipv4_crc_check   = pico_ipv4_crc_check    (:243-257)
 *                            rr_ipv4_pre_forward_checks = pico_ipv4_pre_forward_checks (:1535-1574:
 *                            TTL, crc++, local source, the duplicate of the last forwarded datagram;
 *                            its static state lives in this library copy)
 *   2: modules/pico_ipv6.c   rr_ipv6_ext_headers = pico_ipv6_extension_headers (:707-809)
 *   3: stack/pico_socket.c   rr_transport_crc_check = pico_transport_crc_check (:1916-1968)
 *   4: modules/pico_fragments.c  rr_frag_reset: empties the two reassembly trees and forgets the
 *                            current fragment ids (pico_fragments_empty_tree, :199-214) between
 *                            the independent fragment groups of a fixture
 * and linked with the rest of the reference stack (every other object compiled from its own
 * source) into oracle/_ref/libref_rx.so, driven by ref_rx_driver.c.  Nothing here is product
 * code; nothing of the reference is copied (the #include names the file where it lies).
 */
#if REF_RX_UNIT == 1
#include "pico_ipv4.c"
int rr_ipv4_process_in(struct pico_frame *f);
int rr_ipv4_crc_check(struct pico_frame *f);
int rr_ipv4_process_in(struct pico_frame *f) { return pico_ipv4_process_in(&pico_proto_ipv4, f); }
int rr_ipv4_crc_check(struct pico_frame *f) { return pico_ipv4_crc_check(f); }
int rr_ipv4_pre_forward_checks(struct pico_frame *f);
int rr_ipv4_pre_forward_checks(struct pico_frame *f) { return pico_ipv4_pre_forward_checks(f); }
#elif REF_RX_UNIT == 2
#include "pico_ipv6.c"
int rr_ipv6_ext_headers(struct pico_frame *f);
int rr_ipv6_ext_headers(struct pico_frame *f) { return pico_ipv6_extension_headers(f); }
#elif REF_RX_UNIT == 3
#include "pico_socket.c"
int rr_transport_crc_check(struct pico_frame *f);
int rr_transport_crc_check(struct pico_frame *f) { return pico_transport_crc_check(f); }
#elif REF_RX_UNIT == 4
#include "pico_fragments.c"
void rr_frag_reset(void);
void rr_frag_reset(void)
{
    pico_fragments_empty_tree(&ipv4_fragments);
    pico_fragments_empty_tree(&ipv6_fragments);
    if (ipv4_fragments_timer)
        pico_timer_cancel(ipv4_fragments_timer);
    if (ipv6_fragments_timer)
        pico_timer_cancel(ipv6_fragments_timer);
    ipv4_fragments_timer = ipv6_fragments_timer = 0;
    ipv4_cur_frag_id = ipv6_cur_frag_id = 0;
}
#elif REF_RX_UNIT == 5
#include "pico_ethernet.c"
int32_t rr_ethernet_receive(struct pico_frame *f);
int32_t rr_ethernet_receive(struct pico_frame *f) { return pico_ethernet_receive(f); }
#else
#error "REF_RX_UNIT must be 1, 2, 3, 4 or 5"
#endif

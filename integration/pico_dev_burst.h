/*
 * pico_dev_burst.h -- the reference-side binding of libpicocsum's batched RX verify
 * (INTEGRATION.md 2): what a batching picoTCP device driver adds.  Compiled inside a picoTCP
 * build (reference headers: pico_device.h, pico_stack.h), linked to libpicocsum.so; the stack is
 * built with CRC=0 (reference Makefile:49, rules/crc.mk:1), so pico_ipv4_crc_check and
 * pico_transport_crc_check are its no-op variants (modules/pico_ipv4.c:259-264,
 * stack/pico_socket.c:1969-1975) and the driver decides per frame from the batch's verdicts.
 */
#ifndef PICO_DEV_BURST_H
#define PICO_DEV_BURST_H
#include <stdint.h>
#include "pico_csum.h"

struct pico_device;

/* Verdicts for a burst of Ethernet frames in host memory (ring, ring_len bytes; desc[i].off ->
 * frame i's Ethernet header, desc[i].len = its bytes): pico_eth_checksum_batch_host on the GPU
 * (ctx != NULL).  If that call fails (no device: -PICO_CSUM_ENODEV, or any other error) the burst
 * is NOT dropped: every frame is verified on the host with the scalar drop-in (pico_checksum /
 * pico_dualbuffer_checksum, layer 1) instead -- the checks a CRC=1 stack would make, nothing else
 * (the stack still makes every other decision).  Returns 1 when the GPU produced the verdicts, 0
 * when the host did. */
int pico_burst_verdicts(struct pico_csum_ctx *ctx, const uint8_t mac[6], const uint8_t *ring, uint64_t ring_len,
                        const struct pico_csum_desc *desc, uint32_t n, uint8_t *verdict);

/* 1 when the frame goes on to pico_stack_recv: accepted, ARP, a fragment (the stack reassembles
 * it), or a bad transport checksum on a datagram the stack routes on (it never checks those);
 * 0 when the reference would discard it (checksum, link-layer or malformed verdicts). */
int pico_burst_hand_on(uint8_t verdict, const uint8_t *frame, uint32_t len);

/* The poll step of such a driver: verdicts for the burst, then pico_stack_recv for every frame
 * that goes on.  Returns the frames handed on (or a negative pico_stack_recv error). */
int pico_burst_rx(struct pico_device *dev, struct pico_csum_ctx *ctx, const uint8_t mac[6], uint8_t *ring,
                  uint64_t ring_len, const struct pico_csum_desc *desc, uint32_t n, uint8_t *verdict);
#endif

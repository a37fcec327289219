// pico_csum_k_frag.hip -- IPv4 fragment reassembly gather fused with the transport check of
// the reassembled datagram, and its launcher.
// Helpers, argument conventions and the arithmetic contract: pico_csum_dev.h.
//
// Reference: pico_ipv4_process_frag / pico_fragments_check_complete /
// pico_fragments_reassemble (modules/pico_fragments.c:129-139, 216-239, 304-358, 499-568),
// then pico_transport_crc_check (stack/pico_socket.c:1916-1968) on the reassembled frame.
// The reference copies every fragment into a fresh frame (memcpy, :334-345) and then sums
// the whole transport again; here one pass reads each fragment's payload once, writes it to
// its place in the reassembled datagram and adds it to the checksum on the way.
//
// One wave per datagram (its fragments are a contiguous descriptor range, arrival order):
//   1. lane j parses fragment j's header (IHL, total length, MF, offset) into LDS;
//   2. tree order: rank by offset among the first arrivals of each offset (pico_tree_insert
//      rejects a repeated key), LDS broadcast reads, O(count^2 / 64) per lane;
//   3. completeness: a wave prefix scan of the sorted transport lengths against the
//      offsets, up to the first fragment without MF (must be the last in tree order);
//   4. gather: the first fragment's 20 header bytes, then fragment by fragment one dword
//      per lane per step (unaligned source: two aligned loads + alignbyte; the datagram's
//      transport starts 4-byte aligned, offsets are multiples of 8, so every dword is a
//      whole pair of checksum words), v_dot2 sums on the fly, a wave reduction at the end.
#include "pico_csum_dev.h"

namespace {

constexpr uint32_t FRAG_MAX = 512;     // fragments per datagram handled on device

struct FragArgs {
    const uint8_t* base;
    uint64_t base_len;
    const pico_csum_desc_dev* frag;
    const uint32_t* grp;                // 2 per datagram: first descriptor, count
    uint32_t n_dgram;
    uint32_t n_frag;
    uint8_t* out;
    uint64_t out_len;
    const pico_csum_desc_dev* odesc;    // per datagram: output region (off, capacity)
    uint32_t* o_len;
    uint16_t* o_l4;
    uint8_t* verdict;
};

struct FragWaveLds {
    uint32_t key[FRAG_MAX];   // offset | MF << 16 | header length << 17 | dup << 24
    uint32_t tl[FRAG_MAX];    // transport length
    uint16_t sidx[FRAG_MAX];  // tree position -> fragment
};

__device__ __forceinline__ uint32_t ld_u8(const uint8_t* p) { return (uint32_t)*p; }

// The dword at byte address a (any alignment) of the region [lo, hi): two aligned loads and
// alignbyte; the second load only where the dword reaches into it (never past the region's
// last 4-byte word, so never into an unmapped page).
__device__ __forceinline__ uint32_t ld_unaligned(const uint8_t* a, const uint8_t* hi) {
    const uintptr_t ua = reinterpret_cast<uintptr_t>(a);
    const uint32_t sh = (uint32_t)(ua & 3u);
    const uint32_t* w0 = reinterpret_cast<const uint32_t*>(ua & ~(uintptr_t)3);
    const uint32_t* w1 = (sh != 0 && reinterpret_cast<const uint8_t*>(w0 + 1) < hi) ? w0 + 1 : w0;
    return __builtin_amdgcn_alignbyte(*w1, *w0, sh);
}

__global__ __launch_bounds__(256) void ipv4_reassemble_kernel(FragArgs p) {
    __shared__ FragWaveLds lds_all[4];
    const uint32_t lane = threadIdx.x & 63u;
    FragWaveLds& L = lds_all[threadIdx.x >> 6];
    const uint32_t g = blockIdx.x * 4u + (threadIdx.x >> 6);
    if (g >= p.n_dgram) return;
    const uint32_t first = p.grp[2 * g], cnt = p.grp[2 * g + 1];
    const pico_csum_desc_dev od = p.odesc[g];
    bool bad = cnt == 0 || cnt > FRAG_MAX || first > p.n_frag || cnt > p.n_frag - first;

    // ---- 1. parse (pico_ipv4_process_in: net_len, transport_len = tot - net_len, frag)
    if (!bad) {
        bool b = false;
        for (uint32_t j = lane; j < cnt; j += 64u) {
            const pico_csum_desc_dev d = p.frag[first + j];
            uint32_t key = 0, tl = 0;
            if (d.len < 20u || d.off > p.base_len || d.len > p.base_len - d.off) {
                b = true;
            } else {
                const uint8_t* h = p.base + d.off;
                const uint32_t ihl = ld_u8(h) & 0x0Fu;
                const uint32_t hl = 20u + (ihl > 5u ? 4u * (ihl - 5u) : 0u);
                tl = ((ld_u8(h + 2) << 8) | ld_u8(h + 3)) - hl;
                tl &= 0xFFFFu;
                const uint32_t frag = (ld_u8(h + 6) << 8) | ld_u8(h + 7);
                key = ((frag & 0x1FFFu) << 3) | ((frag & 0x2000u) ? 1u << 16 : 0u) | (hl << 17);
                if (hl + tl > d.len) b = true;
            }
            L.key[j] = key;
            L.tl[j] = tl;
        }
        bad = __builtin_amdgcn_ballot_w64(b) != 0;
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_s_waitcnt(0xC07F);

    // ---- 2. tree order: repeated offsets keep the earliest arrival; rank among the kept
    uint32_t m = 0;
    if (!bad) {
        for (uint32_t j = lane; j < cnt; j += 64u) {
            const uint32_t fj = L.key[j] & 0xFFFFu;
            bool dup = false;
            for (uint32_t k = 0; k < j; ++k) dup |= (L.key[k] & 0xFFFFu) == fj;
            if (dup) L.key[j] |= 1u << 24;
        }
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_s_waitcnt(0xC07F);
        uint32_t kept = 0;
        for (uint32_t j = lane; j < cnt; j += 64u) {
            const uint32_t kj = L.key[j];
            if (kj >> 24) continue;
            uint32_t r = 0;
            for (uint32_t k = 0; k < cnt; ++k) {
                const uint32_t kk = L.key[k];
                r += ((kk >> 24) == 0 && (kk & 0xFFFFu) < (kj & 0xFFFFu)) ? 1u : 0u;
            }
            L.sidx[r] = (uint16_t)j;
            ++kept;
        }
        m = (uint32_t)__builtin_amdgcn_readlane((int)group_sum<64>(kept), 63);
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_s_waitcnt(0xC07F);

    // ---- 3. completeness (pico_fragments_check_complete): offset == bookmark up to the
    //         first fragment without MF, which must be the last one in tree order
    uint32_t len = 0;
    if (!bad) {
        uint32_t carry = 0, e = NONE;
        bool gap = false;
        for (uint32_t i0 = 0; i0 < m && e == NONE; i0 += 64u) {
            const uint32_t i = i0 + lane;
            const bool in = i < m;
            const uint32_t j = in ? L.sidx[i] : 0u;
            const uint32_t kj = in ? L.key[j] : 0u, tl = in ? L.tl[j] : 0u;
            const uint32_t incl = wave_scan_add(tl);
            const uint32_t P = carry + incl - tl;
            const uint64_t last = __builtin_amdgcn_ballot_w64(in && !(kj & (1u << 16)));
            const uint32_t le = last ? (uint32_t)__builtin_ctzll(last) : 64u;     // first MF-clear lane
            gap |= __builtin_amdgcn_ballot_w64(in && lane <= le && (kj & 0xFFFFu) != P) != 0;
            if (last) {
                e = i0 + le;
                len = (uint32_t)__builtin_amdgcn_readlane((int)(P + tl), (int)le);
            }
            carry += (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
        }
        bad = gap || e == NONE || e + 1u != m || 20u + len > 0xFFFFu || od.len < 20u + len ||
              (od.off & 3u) != 0 || od.off > p.out_len || od.len > p.out_len - od.off;
    }

    // ---- 4. gather + checksum
    uint32_t acc = 0, w1 = 0;
    uint32_t proto = 0, pseudo = 0;
    if (!bad) {
        uint8_t* dst = p.out + od.off;
        const pico_csum_desc_dev d0 = p.frag[first + L.sidx[0]];
        const uint8_t* h0 = p.base + d0.off;
        // the first fragment's PICO_SIZE_IP4HDR bytes (pico_fragments.c:332-333)
        const uint32_t hb = lane < 20u ? ld_u8(h0 + lane) : 0u;
        if (lane < 20u) dst[lane] = (uint8_t)hb;
        proto = (uint32_t)__shfl((int)hb, 9);
        // pseudo header (struct pico_ipv4_pseudo_hdr) as LE words: src, dst, proto << 8, bswap16(len)
        const uint32_t pw = lane >= 12u && lane < 20u ? (lane & 1u ? hb << 8 : hb) : 0u;
        pseudo = (uint32_t)__builtin_amdgcn_readlane((int)group_sum<64>(pw), 63) + (proto << 8) +
                 (((len & 0xFFu) << 8) | ((len >> 8) & 0xFFu));
        uint8_t* t = dst + 20;
        uint32_t at = 0;                                   // bookmark (== the fragment's offset)
        for (uint32_t i = 0; i < m; ++i) {
            const uint32_t j = L.sidx[i];
            const uint32_t hl = (L.key[j] >> 17) & 0x7Fu, tl = L.tl[j];
            const pico_csum_desc_dev d = p.frag[first + j];
            const uint8_t* src = p.base + d.off + hl;
            const uint8_t* src_end = src + tl;
            for (uint32_t w = lane; 4u * w < tl; w += 64u) {
                const uint32_t b0 = 4u * w, nb = min(4u, tl - b0);
                uint32_t v = ld_unaligned(src + b0, src_end);
                if (nb < 4u) v &= (1u << (8u * nb)) - 1u;
                if (nb == 4u) {
                    *reinterpret_cast<uint32_t*>(t + at + b0) = v;
                } else {
                    for (uint32_t q = 0; q < nb; ++q) t[at + b0 + q] = (uint8_t)(v >> (8u * q));
                }
                acc = dot2_add(v, acc);                    // at + b0 is even: frame-relative pairs
                if (at + b0 == 4u) w1 = v;                 // transport bytes 4..7 (UDP crc: 6, 7)
            }
            at += tl;
        }
        acc = (uint32_t)__builtin_amdgcn_readlane((int)group_sum<64>(acc), 63);
        w1 = (uint32_t)__builtin_amdgcn_readlane((int)group_sum<64>(w1), 63);
    }

    // ---- 5. pico_transport_crc_check on the reassembled frame
    if (lane == 0) {
        uint32_t l4 = 0, v = V_MALFORMED;
        if (!bad) {
            v = V_ACCEPT;
            if (proto == 6u || (proto == 17u && len >= 8u && (w1 >> 16) != 0u)) {
                l4 = finalize(pseudo + acc);
                if (l4) v = V_L4_BAD;
            }
        }
        if (p.o_len) p.o_len[g] = bad ? 0u : len;
        if (p.o_l4) p.o_l4[g] = (uint16_t)l4;
        if (p.verdict) p.verdict[g] = (uint8_t)v;
    }
}

}  // namespace

extern "C" {

int pico_csum_launch_ipv4_reassemble(const void* base, uint64_t base_len, const void* frag, uint32_t n_frag,
                                     const uint32_t* groups, uint32_t n_dgram, void* out, uint64_t out_len,
                                     const void* out_desc, uint32_t* o_len, uint16_t* o_l4, uint8_t* verdict,
                                     void* stream) {
    if (n_dgram == 0) return (int)hipSuccess;
    FragArgs a{static_cast<const uint8_t*>(base), base_len, static_cast<const pico_csum_desc_dev*>(frag), groups,
               n_dgram, n_frag, static_cast<uint8_t*>(out), out_len,
               static_cast<const pico_csum_desc_dev*>(out_desc), o_len, o_l4, verdict};
    const dim3 grid((n_dgram + 3u) / 4u), block(256);
    hipLaunchKernelGGL(ipv4_reassemble_kernel, grid, block, 0, static_cast<hipStream_t>(stream), a);
    return (int)hipGetLastError();
}

}  // extern "C"

// hvws_dev.h -- device helpers shared by the discovery kernels
// (hvws_kernels.hip, hvws_sieve.hip): 16-byte header loads, the fixed-format
// header decode of http/websocket_parser.c:60-142 and frame-record stores.
#pragma once

#include "hvws_internal.h"

namespace hvws {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// ---------------------------------------------------------------- helpers

__device__ __forceinline__ uint32_t rotr32(uint32_t x, uint32_t r) {
    r &= 31u;
    return r ? (x >> r) | (x << (32u - r)) : x;
}

// Key word for 4-byte aligned words of a payload whose first byte sits at
// absolute offset `pay_off` with mask phase `phase`: byte at address a uses
// mask[(a - pay_off + phase) & 3] (http/websocket_parser.c:175).
__device__ __forceinline__ uint32_t key_for_aligned(uint32_t key, uint64_t pay_off, uint32_t phase) {
    uint32_t rot = (phase - (uint32_t)pay_off) & 3u;
    return rotr32(key, 8u * rot);
}

__device__ __forceinline__ uint64_t ld64_guard(const uint8_t* rx, uint64_t rx_len, uint64_t a) {
    if (a + 8 <= rx_len) return *reinterpret_cast<const uint64_t*>(rx + a);
    uint64_t v = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k)
        if (a + k < rx_len) v |= (uint64_t)rx[a + k] << (8 * k);
    return v;
}

// 16 bytes starting at arbitrary absolute offset q (bytes past rx_len read 0).
// Inside the buffer the three words are loaded unconditionally, so the loads
// issue together and cost one memory round trip: guarded one by one, each
// sat behind its own branch and wait -- three dependent round trips per
// header in the walks (k_sieve_link: ~1.9 us per hop on an idle chip).
__device__ __forceinline__ void ld16(const uint8_t* rx, uint64_t rx_len, uint64_t q, uint64_t& lo,
                                     uint64_t& hi) {
    const uint64_t a = q & ~7ull;
    const uint32_t sh = (uint32_t)(q & 7u) * 8u;
    uint64_t w0, w1, w2;
    if (a + 24 <= rx_len) {
        const uint64_t* p = reinterpret_cast<const uint64_t*>(rx + a);
        w0 = p[0];
        w1 = p[1];
        w2 = p[2];
    } else {
        w0 = ld64_guard(rx, rx_len, a);
        w1 = ld64_guard(rx, rx_len, a + 8);
        w2 = ld64_guard(rx, rx_len, a + 16);
    }
    lo = sh ? (w0 >> sh) | (w1 << (64u - sh)) : w0;
    hi = sh ? (w1 >> sh) | (w2 << (64u - sh)) : w1;
}

struct hdr {
    uint64_t length;
    uint32_t hlen;
    uint32_t flags;
    uint32_t key;
    uint32_t viol;   // V_* classes this header violates (reported only if enabled)
};

__device__ __forceinline__ bool reserved_opcode(uint32_t op) { return (op >= 3 && op <= 7) || op >= 0xB; }

// Fixed-format header decode from its first 16 bytes (lo = bytes 0..7 LE).
// Layout per websocket_build_frame (http/websocket_parser.c:207-256):
// b0 = FIN<<7 | opcode, b1 = MASK<<7 | len7, then 0/2/8 big-endian length
// bytes, then the 4 key bytes if MASK.  RSV bits are dropped (Q1).
// V = false: no violation classes (viol = 0), for callers whose validation
// mask is 0 (invalid_bits drops them there anyway).
template <bool V = true>
__device__ __forceinline__ hdr parse_hdr(uint64_t lo, uint64_t hi) {
    hdr h;
    uint32_t b0 = (uint32_t)lo & 0xFFu;
    uint32_t b1 = (uint32_t)(lo >> 8) & 0xFFu;
    uint32_t len7 = b1 & 0x7Fu;
    bool m = (b1 & 0x80u) != 0;
    h.flags = (b0 & F_OPMASK) | ((b0 & 0x80u) ? F_FIN : 0u) | (m ? F_MASK : 0u);
    uint32_t ext = len7 == 126 ? 2u : (len7 == 127 ? 8u : 0u);
    h.hlen = 2u + ext + (m ? 4u : 0u);
    uint64_t len16 = (((lo >> 16) & 0xFFu) << 8) | ((lo >> 24) & 0xFFu);
    uint64_t len64 = __builtin_bswap64((lo >> 16) | (hi << 48));
    h.length = len7 < 126 ? (uint64_t)len7 : (len7 == 126 ? len16 : len64);
    uint32_t k0 = (uint32_t)(lo >> 16), k2 = (uint32_t)(lo >> 32), k8 = (uint32_t)(hi >> 16);
    h.key = m ? (ext == 0 ? k0 : (ext == 2 ? k2 : k8)) : 0u;
    const uint32_t op = b0 & F_OPMASK;
    if constexpr (V)
        h.viol = ((b0 & 0x70u) ? V_RSV : 0u) | (reserved_opcode(op) ? V_OPCODE : 0u) |
                 ((op & 8u) && (!(b0 & 0x80u) || h.length > 125) ? V_CONTROL : 0u) |
                 (ext == 8 && (h.length >> 63) ? V_LEN64 : 0u) |
                 ((ext == 2 && h.length < 126) || (ext == 8 && h.length <= 0xFFFFu) ? V_NONMIN : 0u) |
                 (m ? 0u : V_UNMASKED);
    else
        h.viol = 0u;
    return h;
}

struct frec {
    int64_t  hdr_off;   // segment-relative here; made absolute on store
    uint64_t pay_off;   // segment-relative
    uint64_t pay_len;
    uint64_t length;
    uint32_t key;
    uint32_t info;
};

__device__ __forceinline__ void store_frame(const dframes& fr, uint64_t idx, uint64_t seg_off, const frec& r) {
    if (idx >= fr.cap) return;   // table sized by an estimate (SCAN_SINGLE): the host re-emits if it overflowed
    uint32_t phase = (r.info >> 8) & 3u;
    bool masked = (r.info & F_MASK) != 0;
    uint64_t abs_pay = seg_off + r.pay_off;
    fr.hdr_off[idx] = r.hdr_off < 0 ? -1 : (int64_t)(seg_off + (uint64_t)r.hdr_off);
    fr.pay_off[idx] = abs_pay;
    fr.pay_len[idx] = r.pay_len;
    fr.length[idx] = r.length;
    fr.key[idx] = r.key;
    fr.keyrot[idx] = masked ? key_for_aligned(r.key, abs_pay, phase) : 0u;
    fr.info[idx] = r.info;
}

__device__ __forceinline__ uint32_t invalid_bits(uint32_t viol, uint32_t vmask) {
    const uint32_t v = viol & vmask & V_ALL;
    return v ? I_INVALID | (v << I_VSHIFT) : 0u;
}

__device__ __forceinline__ void hdr_complete(frec& r, const dcarry& st, uint64_t pay_off, uint32_t vmask) {
    r.info = (r.info & ~0xFFu & ~(3u << 8)) | (st.flags & 0xFFu) | I_HDR | invalid_bits(st.viol, vmask);
    r.pay_off = pay_off;
    r.pay_len = 0;
    r.length = st.length;
    r.key = (st.flags & F_MASK) ? st.mask : 0u;
}

__device__ __forceinline__ bool parse_at(const uint8_t* rx, uint64_t rx_len, uint64_t seg_off, uint64_t L,
                                         uint64_t q, hdr& h) {
    // true when the frame at segment offset q is whole inside [0, L)
    if (q >= L || L - q < 2) return false;
    uint64_t lo, hi;
    ld16(rx, rx_len, seg_off + q, lo, hi);
    h = parse_hdr(lo, hi);
    const uint64_t rq = L - q;
    return h.hlen <= rq && h.length <= rq - h.hlen;
}

__device__ __forceinline__ void whole_frame_rec(frec& v, uint64_t q, const hdr& h, uint32_t vmask) {
    v.hdr_off = (int64_t)q;
    v.pay_off = q + h.hlen;
    v.pay_len = h.length;
    v.length = h.length;
    v.key = h.key;
    v.info = h.flags | I_HDR | I_START | I_END | (h.length ? I_BODY : 0u) | invalid_bits(h.viol, vmask);
}

}  // namespace hvws

// hvws_keys.hip -- batched WebSocket handshake digest (SURVEY.md sec. 8(f)
// row 3): Sec-WebSocket-Accept = base64(SHA-1(key + GUID)) for many upgrade
// requests at once, byte-identical to the reference's ws_encode_key
// (http/wsdef.c:11-20; SHA-1 per util/sha1.c / FIPS 180-4, base64 per
// util/base64.c:53-85 -- 28 characters, no terminator).
//
// One lane per key.  A conforming client key is 24 base64 characters
// (RFC 6455 sec. 4.1: a 16-byte nonce), so key + GUID is 60 bytes and the
// message is exactly two SHA-1 blocks: the first holds 6 key words and the 9
// GUID words plus the 0x80 pad byte, the second only the bit length -- a
// constant block whose message schedule the compiler folds.  Keys of any
// other length take a generic byte-assembling loop.  Integer VALU-bound.
#include "hvws_internal.h"

namespace hvws {

namespace {

// "258EAFA5-E914-47DA-95CA-C5AB0DC85B11" as big-endian words (RFC 6455 sec. 1.3).
// Compile-time literals (not __constant__ memory), so the 24-character path's
// first-block schedule folds every GUID-only term: W6..W15 are known, and
// e.g. W16 = rol(W13 ^ W8 ^ W2 ^ W0) keeps one XOR with a constant.
__device__ __forceinline__ constexpr uint32_t guid_w(int t) {
    return t == 0 ? 0x32353845u : t == 1 ? 0x41464135u : t == 2 ? 0x2D453931u : t == 3 ? 0x342D3437u
         : t == 4 ? 0x44412D39u : t == 5 ? 0x3543412Du : t == 6 ? 0x43354142u : t == 7 ? 0x30444338u : 0x35423131u;
}

__device__ __forceinline__ uint32_t rol(uint32_t x, int n) { return (x << n) | (x >> (32 - n)); }

// N independent SHA-1 compressions interleaved round by round (ILP: the
// 80-round dependency chain of one digest leaves the VALU idle otherwise).
template <int N>
__device__ __forceinline__ void sha1_block_n(uint32_t (&h)[N][5], uint32_t (&w)[N][16]) {
    uint32_t a[N], b[N], c[N], d[N], e[N];
#pragma unroll
    for (int q = 0; q < N; ++q) {
        a[q] = h[q][0];
        b[q] = h[q][1];
        c[q] = h[q][2];
        d[q] = h[q][3];
        e[q] = h[q][4];
    }
#pragma unroll
    for (int t = 0; t < 80; ++t) {
#pragma unroll
        for (int q = 0; q < N; ++q) {
            uint32_t wt;
            if (t < 16) {
                wt = w[q][t];
            } else {
                wt = rol(w[q][(t - 3) & 15] ^ w[q][(t - 8) & 15] ^ w[q][(t - 14) & 15] ^ w[q][t & 15], 1);
                w[q][t & 15] = wt;
            }
            uint32_t f, k;
            if (t < 20) {
                f = (b[q] & c[q]) | (~b[q] & d[q]);
                k = 0x5A827999u;
            } else if (t < 40) {
                f = b[q] ^ c[q] ^ d[q];
                k = 0x6ED9EBA1u;
            } else if (t < 60) {
                f = (b[q] & c[q]) | (b[q] & d[q]) | (c[q] & d[q]);
                k = 0x8F1BBCDCu;
            } else {
                f = b[q] ^ c[q] ^ d[q];
                k = 0xCA62C1D6u;
            }
            const uint32_t tmp = rol(a[q], 5) + f + e[q] + k + wt;
            e[q] = d[q];
            d[q] = c[q];
            c[q] = rol(b[q], 30);
            b[q] = a[q];
            a[q] = tmp;
        }
    }
#pragma unroll
    for (int q = 0; q < N; ++q) {
        h[q][0] += a[q];
        h[q][1] += b[q];
        h[q][2] += c[q];
        h[q][3] += d[q];
        h[q][4] += e[q];
    }
}

__device__ __forceinline__ void sha1_block(uint32_t h[5], uint32_t w[16]) {
    uint32_t (&hh)[1][5] = *reinterpret_cast<uint32_t(*)[1][5]>(h);
    uint32_t (&ww)[1][16] = *reinterpret_cast<uint32_t(*)[1][16]>(w);
    sha1_block_n<1>(hh, ww);
}

__device__ __forceinline__ uint32_t b64c(uint32_t v) {   // util/base64.c alphabet
    return v < 26 ? 'A' + v : v < 52 ? 'a' + (v - 26) : v < 62 ? '0' + (v - 52) : v == 62 ? '+' : '/';
}

__device__ __forceinline__ uint8_t msg_byte(const uint8_t* key, uint64_t kl, uint64_t i, uint64_t total) {
    if (i < kl) return key[i];
    if (i < kl + 36) {
        const uint64_t g = i - kl;
        return (uint8_t)(guid_w((int)(g >> 2)) >> (24 - 8 * (g & 3)));
    }
    if (i == kl + 36) return 0x80;
    const uint64_t bits = (kl + 36) * 8;
    if (i >= total - 8) return (uint8_t)(bits >> (8 * (total - 1 - i)));
    return 0;
}

}  // namespace

__device__ __forceinline__ void key24_words(const uint8_t* key, uint32_t* w) {
    if (((uintptr_t)key & 3u) == 0) {   // 6 dword loads, byte-swapped to SHA-1's big-endian words
        const uint32_t* kw = reinterpret_cast<const uint32_t*>(key);
#pragma unroll
        for (int t = 0; t < 6; ++t) w[t] = __builtin_bswap32(kw[t]);
    } else {
#pragma unroll
        for (int t = 0; t < 6; ++t)
            w[t] = (uint32_t)key[4 * t] << 24 | (uint32_t)key[4 * t + 1] << 16 | (uint32_t)key[4 * t + 2] << 8 |
                   key[4 * t + 3];
    }
#pragma unroll
    for (int t = 0; t < 9; ++t) w[6 + t] = guid_w(t);
    w[15] = 0x80000000u;
}

// digest of a 24-character key (+ GUID = 60 bytes): two blocks, the second constant
template <int N>
__device__ __forceinline__ void digest24(const uint8_t* const (&key)[N], uint32_t (&h)[N][5]) {
    uint32_t w[N][16];
#pragma unroll
    for (int q = 0; q < N; ++q) {
        h[q][0] = 0x67452301u;
        h[q][1] = 0xEFCDAB89u;
        h[q][2] = 0x98BADCFEu;
        h[q][3] = 0x10325476u;
        h[q][4] = 0xC3D2E1F0u;
        key24_words(key[q], w[q]);
    }
    sha1_block_n<N>(h, w);
#pragma unroll
    for (int q = 0; q < N; ++q) {
#pragma unroll
        for (int t = 0; t < 15; ++t) w[q][t] = 0;
        w[q][15] = 60u * 8u;
    }
    sha1_block_n<N>(h, w);
}

__device__ void digest_any(const uint8_t* key, uint32_t kl, uint32_t h[5]) {
    h[0] = 0x67452301u;
    h[1] = 0xEFCDAB89u;
    h[2] = 0x98BADCFEu;
    h[3] = 0x10325476u;
    h[4] = 0xC3D2E1F0u;
    uint32_t w[16];
    const uint64_t total = ((uint64_t)kl + 36 + 8) / 64 * 64 + 64;
    for (uint64_t blk = 0; blk < total; blk += 64) {
        for (int t = 0; t < 16; ++t) {
            uint32_t v = 0;
            for (int b = 0; b < 4; ++b) v = v << 8 | msg_byte(key, kl, blk + 4 * t + b, total);
            w[t] = v;
        }
        sha1_block(h, w);
    }
}

// base64 of the 20-byte digest: 6 groups of 3 bytes, then 2 bytes + '='; then 4 zero bytes
__device__ __forceinline__ void store_accept(const uint32_t h[5], uint8_t* out) {
    uint8_t d[21];
#pragma unroll
    for (int j = 0; j < 20; ++j) d[j] = (uint8_t)(h[j >> 2] >> (24 - 8 * (j & 3)));
    d[20] = 0;
    uint32_t o[8];
#pragma unroll
    for (int g = 0; g < 7; ++g) {
        const uint32_t v = (uint32_t)d[3 * g] << 16 | (uint32_t)d[3 * g + 1] << 8 | (g < 6 ? d[3 * g + 2] : 0u);
        const uint32_t c3 = g < 6 ? b64c(v & 63) : '=';
        o[g] = b64c(v >> 18) | b64c((v >> 12) & 63) << 8 | b64c((v >> 6) & 63) << 16 | c3 << 24;
    }
    o[7] = 0;   // the 4 bytes after the 28 characters read as zero, like the callers' zeroed buffers
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    reinterpret_cast<u32x4*>(out)[0] = u32x4{o[0], o[1], o[2], o[3]};
    reinterpret_cast<u32x4*>(out)[1] = u32x4{o[4], o[5], o[6], o[7]};
}

// One key per lane.  (Two keys per lane with interleaved rounds measured
// slower: 2.90 vs 2.77 ms for 64M keys -- the extra registers cost more
// occupancy than the ILP returned.)
__global__ __launch_bounds__(256) void k_encode_keys(const uint8_t* __restrict__ keys,
                                                     const uint64_t* __restrict__ key_off,
                                                     const uint32_t* __restrict__ key_len, uint64_t n,
                                                     uint8_t* __restrict__ accept) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t kl = key_len[i];
    uint32_t h[1][5];
    if (kl == 24) {
        const uint8_t* const k[1] = {keys + key_off[i]};
        digest24<1>(k, h);
    } else {
        digest_any(keys + key_off[i], kl, h[0]);
    }
    store_accept(h[0], accept + i * 32);
}

hipError_t launch_encode_keys(const uint8_t* keys, const uint64_t* key_off, const uint32_t* key_len, uint64_t n,
                              uint8_t* accept, hipStream_t st) {
    if (n == 0) return hipSuccess;
    const uint64_t per = 0xFFFFFFFFull / 256 * 256;   // keep each grid below 2^32 work-items
    for (uint64_t a = 0; a < n; a += per) {
        const uint64_t m = n - a < per ? n - a : per;
        hipLaunchKernelGGL(k_encode_keys, dim3((uint32_t)((m + 255) / 256)), dim3(256), 0, st, keys, key_off + a,
                           key_len + a, m, accept + a * 32);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

}  // namespace hvws

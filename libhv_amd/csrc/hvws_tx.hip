// hvws_tx.hip -- transmit side: build many frames
// back to back on the device, byte-identical to the reference's
// websocket_build_frame (http/websocket_parser.c:207-256): header, optional
// key, payload XOR-masked from phase 0 (websocket_encode = websocket_decode,
// http/websocket_parser.h:84).  The same rotating-key XOR as k_unmask, run
// out of place from a payload buffer into the frame buffer.
#include <stdlib.h>

#include "hvws_internal.h"

namespace hvws {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t tx_hdr_len(uint32_t flags, uint64_t n) {
    const uint32_t ext = n < 126 ? 0u : (n <= 0xFFFFu ? 2u : 8u);
    return 2u + ext + ((flags & F_MASK) ? 4u : 0u);
}

// Byte h of a frame header (flags: websocket_flags, n payload bytes, key);
// layout of http/websocket_parser.c:215-246.
__device__ __forceinline__ uint32_t tx_hdr_byte(uint32_t flags, uint64_t n, uint32_t key, uint32_t h) {
    const uint32_t ext = n < 126 ? 0u : (n <= 0xFFFFu ? 2u : 8u);
    if (h == 0) return ((flags & F_FIN) ? 0x80u : 0u) | (flags & F_OPMASK);
    if (h == 1) return ((flags & F_MASK) ? 0x80u : 0u) | (n < 126 ? (uint32_t)n : (ext == 2 ? 126u : 127u));
    if (h < 2 + ext) return (uint32_t)(n >> (8 * (ext - 1 - (h - 2)))) & 0xFFu;
    return (key >> (8 * (h - 2 - ext))) & 0xFFu;
}

// ---- device-wide exclusive scan of u64 (block sums, scan of sums, add) ----
// 256-thread workgroups, 4 consecutive elements per thread (1024 per block).
// Workgroups of 1024 threads waited 125-200 us each for a CU with 16 free
// wave slots while a pipelined unmask held the device (the frame sieve's
// scans, profiles/r2o_raw), against ~5 us alone.
constexpr int SCAN_T = 256;
constexpr int SCAN_I = 4;
constexpr int SCAN_B = SCAN_T * SCAN_I;

__global__ __launch_bounds__(SCAN_T) void k_scan_blocks(const uint64_t* __restrict__ in, uint64_t* __restrict__ out,
                                                        uint64_t n, uint64_t* __restrict__ block_sums,
                                                        uint64_t* __restrict__ total_if_one) {
    __shared__ uint64_t s[SCAN_T];
    const uint32_t t = threadIdx.x;
    const uint64_t i0 = (uint64_t)blockIdx.x * SCAN_B + (uint64_t)t * SCAN_I;
    uint64_t v[SCAN_I], sum = 0;
#pragma unroll
    for (int k = 0; k < SCAN_I; ++k) {
        v[k] = i0 + k < n ? in[i0 + k] : 0;
        sum += v[k];
    }
    s[t] = sum;
    __syncthreads();
    for (int d = 1; d < SCAN_T; d <<= 1) {
        const uint64_t a = t >= (unsigned)d ? s[t - d] : 0;
        __syncthreads();
        s[t] += a;
        __syncthreads();
    }
    uint64_t run = s[t] - sum;   // exclusive within the block
#pragma unroll
    for (int k = 0; k < SCAN_I; ++k) {
        if (i0 + k < n) out[i0 + k] = run;
        run += v[k];
    }
    if (t == SCAN_T - 1) {
        block_sums[blockIdx.x] = s[t];
        if (total_if_one) *total_if_one = s[t];   // one block: its sum is the total
    }
}

__global__ __launch_bounds__(SCAN_T) void k_add_block_base(uint64_t* __restrict__ out, uint64_t n,
                                                           const uint64_t* __restrict__ block_base) {
    const uint64_t i0 = (uint64_t)blockIdx.x * SCAN_B + (uint64_t)threadIdx.x * SCAN_I;
    const uint64_t b = block_base[blockIdx.x];
#pragma unroll
    for (int k = 0; k < SCAN_I; ++k)
        if (i0 + k < n) out[i0 + k] += b;
}

// ------------------------------------------------------------- k_build
//
// One workgroup of 256 threads per output tile of 256*U*16 bytes, tiles in
// XCD-contiguous order.  A tile lying inside one frame's payload (all but
// the boundary tile of a 64 KiB frame) takes the streaming path: the frame
// is found once per tile, the U source vectors are loaded back to back and
// realigned to the output's 16-B phase (two aligned loads per chunk when the
// payload and output phases differ), XORed with the rotated key word and
// stored.  Other tiles build chunk by chunk: binary search of the frame
// table within the tile's frame range, then 16 payload bytes or, at headers
// and frame boundaries, byte by byte.

// 16 payload bytes starting at arbitrary offset p of a buffer of plen bytes.
__device__ __forceinline__ void ld16_any(const uint8_t* pay, uint64_t plen, uint64_t p, uint64_t& lo, uint64_t& hi) {
    const uint64_t a = p & ~15ull;
    const uint32_t s = (uint32_t)(p & 15u);
    if (a + 32 <= plen) {
        const u32x4 va = *reinterpret_cast<const u32x4*>(pay + a);
        const u32x4 vb = *reinterpret_cast<const u32x4*>(pay + a + 16);
        const uint64_t w0 = va.x | ((uint64_t)va.y << 32), w1 = va.z | ((uint64_t)va.w << 32);
        const uint64_t w2 = vb.x | ((uint64_t)vb.y << 32), w3 = vb.z | ((uint64_t)vb.w << 32);
        const uint64_t x0 = s < 8 ? w0 : w1, x1 = s < 8 ? w1 : w2, x2 = s < 8 ? w2 : w3;
        const uint32_t sh = (s & 7u) * 8u;
        lo = sh ? (x0 >> sh) | (x1 << (64u - sh)) : x0;
        hi = sh ? (x1 >> sh) | (x2 << (64u - sh)) : x1;
    } else {
        lo = hi = 0;
        for (int b = 0; b < 16; ++b) {
            const uint64_t q = p + b;
            const uint64_t v = q < plen ? pay[q] : 0;
            if (b < 8) lo |= v << (8 * b);
            else hi |= v << (8 * (b - 8));
        }
    }
}

// bytes s..s+15 of the 32-byte little-endian pair (a, b), s in [0, 16)
__device__ __forceinline__ u32x4 funnel16(u32x4 a, u32x4 b, uint32_t s) {
    const uint64_t w0 = a.x | ((uint64_t)a.y << 32), w1 = a.z | ((uint64_t)a.w << 32);
    const uint64_t w2 = b.x | ((uint64_t)b.y << 32), w3 = b.z | ((uint64_t)b.w << 32);
    const uint64_t x0 = s < 8 ? w0 : w1, x1 = s < 8 ? w1 : w2, x2 = s < 8 ? w2 : w3;
    const uint32_t sh = (s & 7u) * 8u;
    const uint64_t lo = sh ? (x0 >> sh) | (x1 << (64u - sh)) : x0;
    const uint64_t hi = sh ? (x1 >> sh) | (x2 << (64u - sh)) : x1;
    return u32x4{(uint32_t)lo, (uint32_t)(lo >> 32), (uint32_t)hi, (uint32_t)(hi >> 32)};
}

constexpr uint32_t BUILD_MAXF = 128;   // frames per boundary tile staged in LDS

__device__ __forceinline__ uint32_t tx_rotr(uint32_t x, uint32_t r) { return r ? (x >> r) | (x << (32u - r)) : x; }

// OR bytes [0, b1 - b0) of the 16-byte little-endian value (vlo, vhi) into
// bytes [b0, b1) of the chunk (olo, ohi); 0 <= b0 < b1 <= 16.
__device__ __forceinline__ void put_bytes(uint64_t& olo, uint64_t& ohi, uint64_t vlo, uint64_t vhi, uint32_t b0,
                                          uint32_t b1) {
    const uint32_t n = b1 - b0;
    if (n < 8) {
        vlo &= ~0ull >> (64u - 8u * n);
        vhi = 0;
    } else if (n < 16) {
        vhi = n == 8 ? 0 : vhi & (~0ull >> (64u - 8u * (n - 8u)));
    }
    if (b0 >= 8) {
        vhi = vlo << (8u * (b0 - 8u));
        vlo = 0;
    } else if (b0) {
        vhi = (vhi << (8u * b0)) | (vlo >> (64u - 8u * b0));
        vlo <<= 8u * b0;
    }
    olo |= vlo;
    ohi |= vhi;
}

// Frame header as a 16-byte little-endian value (bytes beyond its length 0);
// layout of http/websocket_parser.c:215-246 (same bytes as tx_hdr_byte).
__device__ __forceinline__ void tx_hdr128(uint32_t fl, uint64_t n, uint32_t key, uint64_t& lo, uint64_t& hi) {
    const uint64_t b0 = ((fl & F_FIN) ? 0x80u : 0u) | (fl & F_OPMASK);
    const uint64_t m = (fl & F_MASK) ? 0x80u : 0u;
    const uint64_t k = (fl & F_MASK) ? key : 0u;
    if (n < 126) {
        lo = b0 | ((m | n) << 8) | (k << 16);
        hi = 0;
    } else if (n <= 0xFFFFu) {
        lo = b0 | ((m | 126u) << 8) | (((n >> 8) & 0xFFu) << 16) | ((n & 0xFFu) << 24) | (k << 32);
        hi = 0;
    } else {
        const uint64_t be = __builtin_bswap64(n);
        lo = b0 | ((m | 127u) << 8) | (be << 16);
        hi = (be >> 48) | (k << 16);
    }
}

// (lo, hi) >> 8*r bytes, r < 16
__device__ __forceinline__ void shr_bytes(uint64_t& lo, uint64_t& hi, uint32_t r) {
    if (r >= 8) {
        lo = hi >> (8u * (r - 8u));
        hi = 0;
    } else if (r) {
        lo = (lo >> (8u * r)) | (hi << (64u - 8u * r));
        hi >>= 8u * r;
    }
}

// The bytes of output chunk [c, c+16) that belong to one frame (header at o,
// payload [ps, e) taken from pay + src0, key 0 when unmasked): the header
// piece cut out of tx_hdr128, the payload piece as one realigned 16-byte
// load XORed with the key rotated to its phase -- no per-byte work.
__device__ __forceinline__ void frame_piece(uint64_t& olo, uint64_t& ohi, uint64_t c, uint64_t o, uint64_t ps,
                                            uint64_t e, uint64_t src0, uint32_t key, uint32_t fl,
                                            const uint8_t* __restrict__ pay, uint64_t plen) {
    const uint64_t ce = c + 16;
    const uint64_t hb = o > c ? o : c, he = ps < ce ? ps : ce;
    if (hb < he) {
        uint64_t vlo, vhi;
        tx_hdr128(fl, e - ps, key, vlo, vhi);
        shr_bytes(vlo, vhi, (uint32_t)(hb - o));
        put_bytes(olo, ohi, vlo, vhi, (uint32_t)(hb - c), (uint32_t)(he - c));
    }
    const uint64_t pb = ps > c ? ps : c, pe = e < ce ? e : ce;
    if (pb < pe) {
        uint64_t vlo, vhi;
        ld16_any(pay, plen, src0 + (pb - ps), vlo, vhi);
        const uint32_t r = (uint32_t)((pb - ps) & 3u) * 8u;
        const uint32_t kw = r ? (key >> r) | (key << (32u - r)) : key;
        const uint64_t kk = (uint64_t)kw | ((uint64_t)kw << 32);
        put_bytes(olo, ohi, vlo ^ kk, vhi ^ kk, (uint32_t)(pb - c), (uint32_t)(pe - c));
    }
}

__device__ __forceinline__ void build_chunk(uint8_t* __restrict__ out, uint64_t out_len, const uint8_t* __restrict__ pay,
                                            uint64_t plen, const uint64_t* __restrict__ pay_off,
                                            const uint64_t* __restrict__ len, const uint8_t* __restrict__ flags,
                                            const uint32_t* __restrict__ mask, const uint64_t* __restrict__ out_off,
                                            const uint64_t* __restrict__ size, uint64_t n, uint64_t k_lo,
                                            uint64_t k_hi, uint64_t c) {
    uint64_t k = k_lo, k_end = k_hi;   // first frame ending after c
    while (k < k_end) {
        const uint64_t mid = (k + k_end) >> 1;
        if (out_off[mid] + size[mid] > c) k_end = mid;
        else k = mid + 1;
    }
    if (k < n && c + 16 <= out_len) {
        const uint32_t fl = flags[k];
        const uint64_t ln = len[k];
        const uint64_t ps = out_off[k] + tx_hdr_len(fl, ln);
        if (ps <= c && c + 16 <= ps + ln) {   // 16 payload bytes of one frame
            const uint64_t j0 = c - ps;
            uint64_t lo, hi;
            ld16_any(pay, plen, pay_off[k] + j0, lo, hi);
            if (fl & F_MASK) {
                const uint32_t key = mask[k];
                const uint32_t r = (uint32_t)(j0 & 3u) * 8u;
                const uint32_t kw = r ? (key >> r) | (key << (32u - r)) : key;
                const uint64_t kk = (uint64_t)kw | ((uint64_t)kw << 32);
                lo ^= kk;
                hi ^= kk;
            }
            __builtin_nontemporal_store(u32x4{(uint32_t)lo, (uint32_t)(lo >> 32), (uint32_t)hi, (uint32_t)(hi >> 32)},
                                        reinterpret_cast<u32x4*>(out + c));
            return;
        }
    }
    // header bytes / frame boundaries / tail: frame by frame
    uint64_t lo = 0, hi = 0;
    for (; k < n && out_off[k] < c + 16; ++k) {
        const uint32_t fl = flags[k];
        const uint64_t ln = len[k], o = out_off[k];
        const uint64_t ps = o + tx_hdr_len(fl, ln);
        frame_piece(lo, hi, c, o, ps, ps + ln, pay_off[k], (fl & F_MASK) ? mask[k] : 0u, fl, pay, plen);
    }
    if (c + 16 <= out_len) {
        __builtin_nontemporal_store(u32x4{(uint32_t)lo, (uint32_t)(lo >> 32), (uint32_t)hi, (uint32_t)(hi >> 32)},
                                    reinterpret_cast<u32x4*>(out + c));
    } else {
        for (uint32_t b = 0; b < 16 && c + b < out_len; ++b)
            out[c + b] = (uint8_t)((b < 8 ? lo >> (8u * b) : hi >> (8u * (b - 8u))) & 0xFFu);
    }
}

// ---- per-tile source spans (the boundary tiles' payload bytes) ----------
// span[2t], span[2t+1] = [lo, hi): the payload-buffer bytes tile t's frames
// take their payload pieces from (lo = ~0 when it holds no payload byte).
// Written frame by frame (atomics on the first and last tile a frame's
// payload touches; a tile strictly inside one payload is inside no other
// frame's and takes the streaming path or the records-first one),
// so k_build's boundary tiles can issue their payload loads in the same
// round trip as the frame records instead of one round trip after them.
// Per lane (frame k): its payload piece in tile `key` is source bytes
// [lo, hi).  Lanes of a wave hold consecutive frames, whose first (last)
// payload tiles never decrease, so frames sharing a tile sit in one run of
// lanes: a segmented min / max over the run, then one atomic pair per run
// (a per-frame atomic pair serialised ~8 frames per 8 KiB tile on one word:
// 110 us at the c2 shape, profiles/r4d_raw).
__device__ __forceinline__ void span_run_atomics(unsigned long long* span, uint64_t key, uint64_t lo, uint64_t hi) {
    const uint32_t lane = threadIdx.x & 63u;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint64_t ok = __shfl_down(key, o), ol = __shfl_down(lo, o), oh = __shfl_down(hi, o);
        if (lane + (uint32_t)o < 64u && ok == key) {
            lo = ol < lo ? ol : lo;
            hi = oh > hi ? oh : hi;
        }
    }
    const uint64_t prev = __shfl_up(key, 1);
    if (key != ~0ull && (lane == 0 || prev != key)) {
        atomicMin(&span[2 * key], (unsigned long long)lo);
        atomicMax(&span[2 * key + 1], (unsigned long long)hi);
    }
}


// The transmit tile index and spans together.  Fill: tile_first[0..ntiles]
// marked, spans empty.  Pass: frame k scatters itself into tile_first (as
// k_tile_scatter: the tiles whose first byte its output covers, at most
// TILE_SPAN_MAX) and its payload's span runs (one atomic min/max pair per run
// of lanes sharing a tile, span_run_atomics); the marked
// tiles are left to k_tile_fixup.
__global__ void k_tx_index_fill(uint32_t* __restrict__ tile_first, unsigned long long* __restrict__ span,
                                uint64_t ntiles) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t <= ntiles) tile_first[t] = TILE_MARK;
    if (span && t < ntiles) {
        span[2 * t] = ~0ull;
        span[2 * t + 1] = 0ull;
    }
}

__global__ void k_tx_index(const uint64_t* __restrict__ out_off, const uint64_t* __restrict__ size,
                           const uint64_t* __restrict__ pay_off, const uint64_t* __restrict__ len,
                           const uint8_t* __restrict__ flags, uint64_t n, uint64_t ntiles, uint64_t tile,
                           uint32_t* __restrict__ tile_first, unsigned long long* __restrict__ span) {
    const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;   // whole waves run the span shuffles
    if (k < n) {
        const uint64_t lo = k ? out_off[k - 1] + size[k - 1] : 0, hi = out_off[k] + size[k];
        if (hi > lo) {
            const uint64_t t0 = (lo + tile - 1) / tile;
            uint64_t t1 = (hi + tile - 1) / tile;
            if (t1 > ntiles + 1) t1 = ntiles + 1;
            if (t1 > t0 && t1 - t0 <= TILE_SPAN_MAX)
                for (uint64_t t = t0; t < t1; ++t) tile_first[t] = (uint32_t)k;
        }
    }
    if (!span) return;
    const uint64_t ln = k < n ? len[k] : 0;
    uint64_t t0 = ~0ull, t1 = ~0ull, l0 = 0, h0 = 0, l1 = 0, h1 = 0;
    if (ln) {
        const uint64_t ps = out_off[k] + tx_hdr_len(flags[k], ln), e = ps + ln, src = pay_off[k];
        t0 = ps / tile;
        t1 = (e - 1) / tile;
        l0 = src;
        h0 = src + (min(e, (t0 + 1) * tile) - ps);
        l1 = src + (max(ps, t1 * tile) - ps);
        h1 = src + ln;
    }
    span_run_atomics(span, t0, l0, h0);
    span_run_atomics(span, t1 != t0 ? t1 : ~0ull, l1, h1);
}


// A boundary tile's frame in LDS (k_build's staged path, C): positions
// relative to the tile's first output byte.  o and ps (header start and end)
// clamp at -32 and e (payload end) into [-32, TILE + 32]: a header that ends
// before the tile contributes no byte either way, and only min(e, chunk end)
// is used.  q0 + (a tile-relative payload position) is that byte's offset in
// the staged span.  len: the payload length for the header bytes.  fl's top
// byte holds the key phase of the tile's first byte ((base - ps) mod 4).
struct __attribute__((aligned(16))) tx_frel {
    int32_t o, ps, e, q0;
    uint32_t key, fl, len_lo, len_hi;
};

__device__ __forceinline__ tx_frel tx_frel_make(uint64_t o, uint64_t ps, uint64_t e, uint64_t src, uint64_t base,
                                                uint64_t sa, uint64_t tile, uint32_t key, uint32_t fl, uint64_t ln) {
    auto rel = [&](uint64_t x, int64_t hi) -> int32_t {
        const int64_t r = (int64_t)(x - base);   // offsets < 2^63: no overflow in the difference
        return (int32_t)(r < -32 ? -32 : (r > hi ? hi : r));
    };
    tx_frel f;
    f.o = rel(o, (int64_t)tile + 32);
    f.ps = rel(ps, (int64_t)tile + 32);
    f.e = rel(e, (int64_t)tile + 32);
    // staged byte of payload position p (tile-relative): src + (p + base - ps) - sa
    f.q0 = (int32_t)((int64_t)(src - sa) + (int64_t)(base - ps));
    f.key = key;
    f.fl = (fl & 0xFFFFFFu) | ((uint32_t)((base - ps) & 3u) << 24);   // + the key phase of the tile's byte 0
    f.len_lo = (uint32_t)ln;
    f.len_hi = (uint32_t)(ln >> 32);
    return f;
}

// 16 bytes at byte offset q of an LDS area (q + 32 inside it)
__device__ __forceinline__ void lds16(const uint8_t* a, uint32_t q, uint64_t& lo, uint64_t& hi) {
    const u32x4 va = *reinterpret_cast<const u32x4*>(a + (q & ~15u));
    const u32x4 vb = *reinterpret_cast<const u32x4*>(a + (q & ~15u) + 16);
    const u32x4 v = (q & 15u) ? funnel16(va, vb, q & 15u) : va;
    lo = v.x | ((uint64_t)v.y << 32);
    hi = v.z | ((uint64_t)v.w << 32);
}

// One output tile of k_build: its frame range [k_lo, k_hi) (tile_first of t
// and t + 1) and its source span [sp_lo, sp_hi) (k_tx_index) are loaded by the
// caller -- per tile, or one tile ahead in the grid-stride loop.
struct build_idx {
    uint64_t k_lo, k_hi, sp_lo, sp_hi;
};

// Uniform layouts (every frame the same size, payload offsets affine in the
// frame index with a non-negative step: packed payloads, the rx layout, any
// fixed gap; k_tx_check finds them): the tile's frame range and source span
// follow from its position -- no tile index or span pass, no index round trip.
// Frame k's output is [k * stride, (k + 1) * stride), its header hdr bytes,
// its payload from pay_a + k * pay_b.
struct build_uni {
    uint64_t stride, hdr, pay_a, pay_b;
    double inv;   // 1 / stride
};

// floor(x / stride) from the double reciprocal, corrected to exact
__device__ __forceinline__ uint64_t uni_div(uint64_t x, const build_uni& u) {
    uint64_t k = (uint64_t)((double)x * u.inv);
    while (k && k * u.stride > x) --k;
    while ((k + 1) * u.stride <= x) ++k;
    return k;
}

__device__ __forceinline__ build_idx build_uni_idx(const build_uni& u, uint64_t base, uint64_t tile, uint64_t n,
                                                   uint64_t out_len) {
    build_idx x;
    const uint64_t te = base + tile < out_len ? base + tile : out_len;   // base < out_len
    const uint64_t k0 = uni_div(base, u), k1 = uni_div(te - 1, u);     // first and last frame touching the tile
    x.k_lo = k0;
    x.k_hi = k1 + 1 < n ? k1 + 1 : n;
    x.sp_lo = ~0ull;
    x.sp_hi = 0;
    const uint64_t len = u.stride - u.hdr;
    if (len) {
        // first payload piece: frame k0's if its payload starts before te
        // (it ends past base), else none at all (later frames start later)
        const uint64_t ps0 = k0 * u.stride + u.hdr;
        if (ps0 < te) {
            x.sp_lo = u.pay_a + k0 * u.pay_b + (ps0 > base ? 0 : base - ps0);
            // last piece: frame k1's if its payload starts before te, else
            // the whole payload of frame k1 - 1 (>= k0 here)
            const uint64_t ps1 = k1 * u.stride + u.hdr;
            const uint64_t e1 = (k1 + 1) * u.stride;
            x.sp_hi = ps1 < te ? u.pay_a + k1 * u.pay_b + ((e1 < te ? e1 : te) - ps1)
                               : u.pay_a + (k1 - 1) * u.pay_b + len;
        }
    }
    return x;
}

__device__ __forceinline__ build_idx build_load_idx(const uint32_t* __restrict__ tile_first,
                                                    const unsigned long long* __restrict__ span, uint64_t t,
                                                    uint64_t n) {
    build_idx x;
    x.sp_lo = ~0ull;
    x.sp_hi = 0;
    if (span) {   // loaded beside tile_first: no round trip of its own
        x.sp_lo = span[2 * t];
        x.sp_hi = span[2 * t + 1];
    }
    x.k_lo = tile_first[t];
    x.k_hi = min((uint64_t)tile_first[t + 1] + 1, n);   // frames touching the tile: [k_lo, k_hi)
    return x;
}


template <int T, int U, bool NT, bool SF, int C>
__device__ __forceinline__ void build_one_tile(uint8_t* __restrict__ out, uint64_t out_len,
                                           const uint8_t* __restrict__ pay, uint64_t plen,
                                           const uint64_t* __restrict__ pay_off,
                                           const uint64_t* __restrict__ len, const uint8_t* __restrict__ flags,
                                           const uint32_t* __restrict__ mask,
                                           const uint64_t* __restrict__ out_off,
                                           const uint64_t* __restrict__ size,
                                           const unsigned long long* __restrict__ span, uint64_t n, uint64_t t,
                                           const build_idx x, const build_uni& uni) {
    constexpr uint64_t TILE = (uint64_t)T * U * 16u;
    const uint64_t base = t * TILE;
    const uint32_t tid = threadIdx.x;
    const uint64_t sp_lo = x.sp_lo, sp_hi = x.sp_hi, k_lo = x.k_lo, k_hi = x.k_hi;
    // SF: both ends of the tile's frame range load together, and a tile that
    // more than one frame touches goes straight to staging (no dependent
    // load of its first frame's record to find out it is not one payload).
    if (k_lo < n && base + TILE <= out_len && (!SF || k_hi == k_lo + 1)) {
        const uint32_t fl = flags[k_lo];
        const uint64_t ln = len[k_lo];
        const uint64_t ps = out_off[k_lo] + tx_hdr_len(fl, ln);
        const uint64_t src = pay_off[k_lo] + (base - ps);   // payload byte of the tile's first output byte
        const uint64_t src_a = src & ~15ull;
        if (ps <= base && base + TILE <= ps + ln && src_a + TILE + 16 <= plen) {
            uint32_t kw = 0;
            if (fl & F_MASK) {
                const uint32_t key = mask[k_lo];
                const uint32_t r = (uint32_t)((base - ps) & 3u) * 8u;
                kw = r ? (key >> r) | (key << (32u - r)) : key;
            }
            const u32x4 kv = u32x4{kw, kw, kw, kw};
            const uint32_t sft = (uint32_t)(src & 15u);
            const uint8_t* sp = pay + src_a;
            u32x4 v[U];
            if (sft == 0) {
#pragma unroll
                for (int i = 0; i < U; ++i)
                    v[i] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(sp + ((uint64_t)i * T + tid) * 16u));
            } else {
                u32x4 w[U], xx[U];
#pragma unroll
                for (int i = 0; i < U; ++i) {
                    const u32x4* q = reinterpret_cast<const u32x4*>(sp + ((uint64_t)i * T + tid) * 16u);
                    if (NT) {
                        w[i] = __builtin_nontemporal_load(q);
                        xx[i] = __builtin_nontemporal_load(q + 1);
                    } else {
                        w[i] = q[0];
                        xx[i] = q[1];
                    }
                }
#pragma unroll
                for (int i = 0; i < U; ++i) v[i] = funnel16(w[i], xx[i], sft);
            }
#pragma unroll
            for (int i = 0; i < U; ++i)
                __builtin_nontemporal_store(v[i] ^ kv, reinterpret_cast<u32x4*>(out + base + ((uint64_t)i * T + tid) * 16u));
            return;
        }
    }
    const uint64_t nf = k_hi > k_lo ? k_hi - k_lo : 0;
    // staged source bytes per boundary tile (LDS): the tile's payload bytes,
    // with room for gaps between payloads
    constexpr uint64_t SPAN_MAX = TILE + (C == 2 ? 256 : 1024);
    // the tile's frame records, 40 bytes each: the 64-bit per-field arrays,
    // or (C) the compact records in the same storage
    // C == 2 (lean): 16 records and 256 bytes of span slack, so a one-wave
    // workgroup's LDS leaves room for 8 waves per SIMD (its 66 VGPRs allow 7)
    constexpr uint32_t MAXF = C == 2 ? 16u : (T >= 128 ? BUILD_MAXF : (uint32_t)T);
    // (lean: 32 more bytes per frame for its header bytes, built once and
    // placed in the two output chunks they can touch)
    __shared__ __attribute__((aligned(16))) uint64_t s_rb[MAXF * (C == 2 ? 8 : 5)];
    uint64_t* const s_off = s_rb;
    uint64_t* const s_ps = s_rb + MAXF;
    uint64_t* const s_end = s_rb + 2 * MAXF;
    uint64_t* const s_src = s_rb + 3 * MAXF;
    uint32_t* const s_key = reinterpret_cast<uint32_t*>(s_rb + 4 * MAXF);
    uint32_t* const s_fl = s_key + MAXF;
    tx_frel* const s_rel = reinterpret_cast<tx_frel*>(s_rb);
    u32x4* const s_win = reinterpret_cast<u32x4*>(s_rb + 4 * MAXF);   // lean: 2 per frame, after the records
    const uint64_t sa = sp_lo & ~15ull, sb = (sp_hi + 15) & ~15ull;   // staged source chunks [sa, sb)
    const bool staged = nf && nf <= MAXF && base + TILE <= out_len &&
                        sp_lo < sp_hi && sb - sa <= SPAN_MAX && sb <= plen;
    if (staged) {
        // Boundary tile with its source span known up front: the span's
        // payload chunks and the frame records load in one round trip into
        // LDS, then every output chunk is assembled from LDS (header pieces
        // from the records, payload pieces realigned from the staged bytes).
        // (lean: the span one chunk in, so a payload read aligned to its
        // output chunk may start up to 15 bytes before the span; and a table
        // of byte masks, entry n = bytes [0, n))
        constexpr uint32_t LPAD = C == 2 ? 1u : 0u;
        __shared__ u32x4 s_data[SPAN_MAX / 16 + 2 + LPAD];
        __shared__ u32x4 s_mtab[C == 2 ? 17 : 1];
        if (C == 2 && tid < 17) {
            const uint64_t mlo = tid >= 8 ? ~0ull : (1ull << (8u * tid)) - 1ull;
            const uint64_t mhi = tid <= 8 ? 0ull : (tid >= 16 ? ~0ull : (1ull << (8u * (tid - 8u))) - 1ull);
            s_mtab[tid] = u32x4{(uint32_t)mlo, (uint32_t)(mlo >> 32), (uint32_t)mhi, (uint32_t)(mhi >> 32)};
        }
        constexpr int SPU = (int)((SPAN_MAX / 16 + T - 1) / T);
        const uint32_t nch = (uint32_t)((sb - sa) / 16);
        u32x4 d[SPU];
#pragma unroll
        for (int i = 0; i < SPU; ++i) {
            const uint32_t q = (uint32_t)i * (uint32_t)T + tid;
            if (q < nch) d[i] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(pay + sa) + q);
        }
        if (C) {
            // one 32-byte record per frame, 32-bit fields relative to the
            // tile (clamped where only their order matters) -- see tx_frel
            for (uint32_t r = tid; r < nf; r += T) {
                const uint64_t k = k_lo + r;
                const uint32_t fl = flags[k];
                // the key loads with the rest of the record, not after its
                // flags (a second round trip per tile)
                const uint32_t mk = mask ? mask[k] : 0u;
                // a uniform layout's frame position, length and payload offset
                // follow from k: only the flags and keys are read (the tables'
                // lines, shared by neighbouring tiles, were 12 % of the lean
                // form's reads at c2, profiles/r6_raw/tx_traffic)
                const bool un = uni.stride != 0;
                const uint64_t ln = un ? uni.stride - uni.hdr : len[k], o = un ? k * uni.stride : out_off[k];
                const uint64_t ps = o + tx_hdr_len(fl, ln);
                s_rel[r] = tx_frel_make(o, ps, ps + ln, un ? uni.pay_a + k * uni.pay_b : pay_off[k], base, sa, TILE,
                                        (fl & F_MASK) ? mk : 0u, fl, ln);
                if (C == 2) {
                    // the header's bytes, once per frame instead of per chunk
                    // and lane, already where they go in the two 16-byte
                    // output chunks from floor(o / 16) on (zeros around them)
                    uint64_t hlo, hhi;
                    tx_hdr128(fl, ln, mk, hlo, hhi);
                    const int32_t orel = s_rel[r].o;
                    const uint32_t sb = (uint32_t)(orel - ((orel >> 4) << 4)) * 8u;   // bits, 0..120
                    uint64_t w0, w1, w2, w3;
                    if (sb == 0) {
                        w0 = hlo, w1 = hhi, w2 = 0, w3 = 0;
                    } else if (sb < 64) {
                        w0 = hlo << sb, w1 = (hhi << sb) | (hlo >> (64u - sb)), w2 = hhi >> (64u - sb), w3 = 0;
                    } else {
                        const uint32_t s2 = sb - 64u;
                        w0 = 0, w1 = hlo << s2;
                        w2 = s2 ? (hhi << s2) | (hlo >> (64u - s2)) : hhi;
                        w3 = s2 ? hhi >> (64u - s2) : 0;
                    }
                    s_win[2 * r] = u32x4{(uint32_t)w0, (uint32_t)(w0 >> 32), (uint32_t)w1, (uint32_t)(w1 >> 32)};
                    s_win[2 * r + 1] = u32x4{(uint32_t)w2, (uint32_t)(w2 >> 32), (uint32_t)w3, (uint32_t)(w3 >> 32)};
                }
            }
        } else {
            for (uint32_t r = tid; r < nf; r += T) {
                const uint64_t k = k_lo + r;
                const uint32_t fl = flags[k];
                const uint32_t mk = mask ? mask[k] : 0u;
                const uint64_t ln = len[k], o = out_off[k];
                const uint64_t ps = o + tx_hdr_len(fl, ln);
                s_off[r] = o;
                s_ps[r] = ps;
                s_end[r] = ps + ln;
                s_src[r] = pay_off[k];
                s_key[r] = (fl & F_MASK) ? mk : 0u;
                s_fl[r] = fl;
            }
        }
#pragma unroll
        for (int i = 0; i < SPU; ++i) {
            const uint32_t q = (uint32_t)i * (uint32_t)T + tid;
            if (q < nch) s_data[q + LPAD] = d[i];
        }
        if (tid < 2) s_data[nch + LPAD + tid] = u32x4{0, 0, 0, 0};   // lds16 may read 16 bytes past the span
        __syncthreads();
        const uint8_t* lb = reinterpret_cast<const uint8_t*>(s_data);
        if (C) {
            const uint32_t nf32 = (uint32_t)nf;
            uint32_t jb = 0;   // lean: the first frame ending after the previous chunk (chunks rise with i)
#pragma unroll
            for (int i = 0; i < U; ++i) {
                const int32_t c = (int32_t)(((uint32_t)i * (uint32_t)T + tid) * 16u);   // tile-relative
                const int32_t ce = c + 16;
                // first frame ending after c: a count over short ranges
                // (independent broadcast reads), a binary search otherwise;
                // lean: advanced from the previous chunk's
                uint32_t j = 0;
                if (C == 2) {
                    while (jb < nf32 && s_rel[jb].e <= c) ++jb;
                    j = jb;
                } else if (nf32 <= 16) {
                    for (uint32_t m = 0; m < nf32; ++m) j += s_rel[m].e <= c ? 1u : 0u;
                } else {
                    uint32_t je = nf32;
                    while (j < je) {
                        const uint32_t mid = (j + je) >> 1;
                        if (s_rel[mid].e > c) je = mid;
                        else j = mid + 1;
                    }
                }
                uint64_t lo = 0, hi = 0;
                for (; j < nf32; ++j) {
                    const tx_frel f = s_rel[j];
                    if (f.o >= ce) break;
                    const int32_t hb = f.o > c ? f.o : c, he = f.ps < ce ? f.ps : ce;
                    if (hb < he) {   // header bytes
                        if (C == 2) {   // the chunk is the first or second of the frame's window
                            const u32x4 hv = s_win[2 * j + (c > ((f.o >> 4) << 4) ? 1 : 0)];
                            lo |= hv.x | ((uint64_t)hv.y << 32);
                            hi |= hv.z | ((uint64_t)hv.w << 32);
                        } else {
                            uint64_t vlo, vhi;
                            tx_hdr128(f.fl & 0xFFFFFFu, (uint64_t)f.len_lo | ((uint64_t)f.len_hi << 32), f.key, vlo,
                                      vhi);
                            shr_bytes(vlo, vhi, (uint32_t)(hb - f.o));
                            put_bytes(lo, hi, vlo, vhi, (uint32_t)(hb - c), (uint32_t)(he - c));
                        }
                    }
                    const int32_t pb = f.ps > c ? f.ps : c, pe = f.e < ce ? f.e : ce;
                    if (pb < pe) {   // payload bytes, realigned out of the staged span
                        uint64_t vlo, vhi;
                        if (C == 2) {
                            // read aligned to the output chunk (bytes land in
                            // place) and keep [pb, pe) by two table masks
                            lds16(lb, (uint32_t)(f.q0 + c + 16), vlo, vhi);
                            const uint32_t kw = tx_rotr(f.key, (((uint32_t)c + (f.fl >> 24)) & 3u) * 8u);
                            const uint64_t kk = (uint64_t)kw | ((uint64_t)kw << 32);
                            const u32x4 ms = s_mtab[pb - c], me = s_mtab[pe - c];
                            lo |= (vlo ^ kk) & ~(ms.x | ((uint64_t)ms.y << 32)) & (me.x | ((uint64_t)me.y << 32));
                            hi |= (vhi ^ kk) & ~(ms.z | ((uint64_t)ms.w << 32)) & (me.z | ((uint64_t)me.w << 32));
                        } else {
                            lds16(lb, (uint32_t)(f.q0 + pb), vlo, vhi);
                            const uint32_t kw = tx_rotr(f.key, (((uint32_t)pb + (f.fl >> 24)) & 3u) * 8u);
                            const uint64_t kk = (uint64_t)kw | ((uint64_t)kw << 32);
                            put_bytes(lo, hi, vlo ^ kk, vhi ^ kk, (uint32_t)(pb - c), (uint32_t)(pe - c));
                        }
                    }
                    if (f.e >= ce) break;   // the output is dense: the next frame starts at e
                }
                __builtin_nontemporal_store(
                    u32x4{(uint32_t)lo, (uint32_t)(lo >> 32), (uint32_t)hi, (uint32_t)(hi >> 32)},
                    reinterpret_cast<u32x4*>(out + base + (uint32_t)c));
            }
            return;
        }
#pragma unroll
        for (int i = 0; i < U; ++i) {
            const uint64_t c = base + ((uint64_t)i * T + tid) * 16u;
            uint32_t j = 0, je = (uint32_t)nf;   // first frame ending after c
            while (j < je) {
                const uint32_t mid = (j + je) >> 1;
                if (s_end[mid] > c) je = mid;
                else j = mid + 1;
            }
            const uint64_t ce = c + 16;
            uint64_t lo = 0, hi = 0;
            for (; j < nf && s_off[j] < ce; ++j) {
                const uint64_t o = s_off[j], ps = s_ps[j], e = s_end[j];
                const uint64_t hb = o > c ? o : c, he = ps < ce ? ps : ce;
                if (hb < he) {   // header bytes
                    uint64_t vlo, vhi;
                    tx_hdr128(s_fl[j], e - ps, s_key[j], vlo, vhi);
                    shr_bytes(vlo, vhi, (uint32_t)(hb - o));
                    put_bytes(lo, hi, vlo, vhi, (uint32_t)(hb - c), (uint32_t)(he - c));
                }
                const uint64_t pb = ps > c ? ps : c, pe = e < ce ? e : ce;
                if (pb < pe) {   // payload bytes, realigned out of the staged span
                    uint64_t vlo, vhi;
                    lds16(lb, (uint32_t)(s_src[j] + (pb - ps) - sa), vlo, vhi);
                    const uint32_t kw = tx_rotr(s_key[j], (uint32_t)((pb - ps) & 3u) * 8u);
                    const uint64_t kk = (uint64_t)kw | ((uint64_t)kw << 32);
                    put_bytes(lo, hi, vlo ^ kk, vhi ^ kk, (uint32_t)(pb - c), (uint32_t)(pe - c));
                }
            }
            __builtin_nontemporal_store(u32x4{(uint32_t)lo, (uint32_t)(lo >> 32), (uint32_t)hi, (uint32_t)(hi >> 32)},
                                        reinterpret_cast<u32x4*>(out + c));
        }
        return;
    }
    // The lean form's boundary tiles whose span does not fit: as below, but
    // one chunk load in flight at a time.  With all U in flight (below) its
    // register arrays made the whole kernel spill 253 VGPRs at 8 waves per
    // SIMD, and the spilled lane index was reloaded from scratch between the
    // staged loads above, each reload waiting for every load before it
    // (r4ae_raw / r4af_raw / r4ag_raw: c2 0.46-0.47 -> 0.41-0.44 ms).
    if (C == 2 && nf && nf <= MAXF && base + TILE <= out_len) {
        for (uint32_t r = tid; r < nf; r += T) {
            const uint64_t k = k_lo + r;
            const uint32_t fl = flags[k];
            const uint32_t mk = mask ? mask[k] : 0u;
            const uint64_t ln = len[k], o = out_off[k];
            const uint64_t ps = o + tx_hdr_len(fl, ln);
            s_off[r] = o;
            s_ps[r] = ps;
            s_end[r] = ps + ln;
            s_src[r] = pay_off[k];
            s_key[r] = (fl & F_MASK) ? mk : 0u;
            s_fl[r] = fl;
        }
        __syncthreads();
        uint32_t fastmask = 0;
#pragma unroll
        for (int i = 0; i < U; ++i) {
            const uint64_t c = base + ((uint64_t)i * T + tid) * 16u;
            uint32_t j = 0, je = (uint32_t)nf;   // first frame ending after c
            while (j < je) {
                const uint32_t mid = (j + je) >> 1;
                if (s_end[mid] > c) je = mid;
                else j = mid + 1;
            }
            if (j >= nf) continue;
            const uint64_t ps = s_ps[j];
            const uint64_t src = s_src[j] + (c - ps);
            if (ps <= c && c + 16 <= s_end[j] && (src & ~15ull) + 32 <= plen) {
                fastmask |= 1u << i;
                const uint32_t sft = (uint32_t)(src & 15u);
                const u32x4* q = reinterpret_cast<const u32x4*>(pay + (src & ~15ull));
                const u32x4 w = q[0];
                const u32x4 x = sft ? q[1] : w;
                const uint32_t kw = tx_rotr(s_key[j], (uint32_t)((c - ps) & 3u) * 8u);
                const u32x4 v = (sft ? funnel16(w, x, sft) : w) ^ u32x4{kw, kw, kw, kw};
                __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(out + c));
            }
        }
        // chunks holding header bytes or a frame boundary, one at a time
#pragma unroll 1
        for (int i = 0; i < U; ++i) {
            if ((fastmask >> i) & 1u) continue;
            const uint64_t c = base + ((uint64_t)i * T + tid) * 16u;
            uint32_t j = 0, je = (uint32_t)nf;
            while (j < je) {
                const uint32_t mid = (j + je) >> 1;
                if (s_end[mid] > c) je = mid;
                else j = mid + 1;
            }
            uint64_t lo = 0, hi = 0;
            for (; j < nf && s_off[j] < c + 16; ++j)
                frame_piece(lo, hi, c, s_off[j], s_ps[j], s_end[j], s_src[j], s_key[j], s_fl[j], pay, plen);
            __builtin_nontemporal_store(u32x4{(uint32_t)lo, (uint32_t)(lo >> 32), (uint32_t)hi, (uint32_t)(hi >> 32)},
                                        reinterpret_cast<u32x4*>(out + c));
        }
        return;
    }
    if (C != 2 && nf && nf <= MAXF && base + TILE <= out_len) {
        // Boundary tile: the tile's frames staged in LDS; chunks inside one
        // payload still stream (loads issued for all U chunks first), chunks
        // holding header bytes or a frame boundary are assembled byte by byte.
        for (uint32_t r = tid; r < nf; r += T) {
            const uint64_t k = k_lo + r;
            const uint32_t fl = flags[k];
            const uint32_t mk = mask ? mask[k] : 0u;
            const uint64_t ln = len[k], o = out_off[k];
            const uint64_t ps = o + tx_hdr_len(fl, ln);
            s_off[r] = o;
            s_ps[r] = ps;
            s_end[r] = ps + ln;
            s_src[r] = pay_off[k];
            s_key[r] = (fl & F_MASK) ? mk : 0u;
            s_fl[r] = fl;
        }
        __syncthreads();
        u32x4 w[U], x[U];
        uint32_t kw[U], sft[U];
        uint32_t fastmask = 0;
#pragma unroll
        for (int i = 0; i < U; ++i) {
            const uint64_t c = base + ((uint64_t)i * T + tid) * 16u;
            uint32_t j = 0, je = (uint32_t)nf;   // first frame ending after c
            while (j < je) {
                const uint32_t mid = (j + je) >> 1;
                if (s_end[mid] > c) je = mid;
                else j = mid + 1;
            }
            w[i] = x[i] = u32x4{0, 0, 0, 0};
            kw[i] = 0;
            sft[i] = 0;
            if (j < nf) {
                const uint64_t ps = s_ps[j];
                const uint64_t src = s_src[j] + (c - ps);
                if (ps <= c && c + 16 <= s_end[j] && (src & ~15ull) + 32 <= plen) {
                    fastmask |= 1u << i;
                    sft[i] = (uint32_t)(src & 15u);
                    const u32x4* q = reinterpret_cast<const u32x4*>(pay + (src & ~15ull));
                    w[i] = q[0];
                    if (sft[i]) x[i] = q[1];
                    kw[i] = tx_rotr(s_key[j], (uint32_t)((c - ps) & 3u) * 8u);
                }
            }
        }
#pragma unroll
        for (int i = 0; i < U; ++i) {
            if (!((fastmask >> i) & 1u)) continue;
            const uint64_t c = base + ((uint64_t)i * T + tid) * 16u;
            const u32x4 v = (sft[i] ? funnel16(w[i], x[i], sft[i]) : w[i]) ^ u32x4{kw[i], kw[i], kw[i], kw[i]};
            __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(out + c));
        }
        // chunks holding header bytes or a frame boundary, one at a time
#pragma unroll 1
        for (int i = 0; i < U; ++i) {
            if ((fastmask >> i) & 1u) continue;
            const uint64_t c = base + ((uint64_t)i * T + tid) * 16u;
            uint32_t j = 0, je = (uint32_t)nf;
            while (j < je) {
                const uint32_t mid = (j + je) >> 1;
                if (s_end[mid] > c) je = mid;
                else j = mid + 1;
            }
            uint64_t lo = 0, hi = 0;
            for (; j < nf && s_off[j] < c + 16; ++j)
                frame_piece(lo, hi, c, s_off[j], s_ps[j], s_end[j], s_src[j], s_key[j], s_fl[j], pay, plen);
            __builtin_nontemporal_store(u32x4{(uint32_t)lo, (uint32_t)(lo >> 32), (uint32_t)hi, (uint32_t)(hi >> 32)},
                                        reinterpret_cast<u32x4*>(out + c));
        }
        return;
    }
#pragma unroll 1
    for (int i = 0; i < U; ++i) {
        const uint64_t c = base + ((uint64_t)i * T + tid) * 16u;
        if (c >= out_len) break;
        build_chunk(out, out_len, pay, plen, pay_off, len, flags, mask, out_off, size, n, k_lo, k_hi, c);
    }
}

// One workgroup per tile, tiles in linear order (an order giving each XCD
// runs of 8 adjacent tiles, so neighbours' records share one L2, measured
// slower at c2: 0.370-0.391 against 0.353-0.386 ms, profiles/r5a_raw).
// uni.stride != 0: a uniform layout, the tile's frame
// range and span from its position (build_uni_idx); else from the tile index.
template <int T, int U, bool NT, bool SF, int C>
__global__ __launch_bounds__(T) __attribute__((amdgpu_waves_per_eu(C == 2 ? 7 : 8, 8))) void k_build(
    uint8_t* __restrict__ out, uint64_t out_len, const uint8_t* __restrict__ pay, uint64_t plen,
    const uint64_t* __restrict__ pay_off, const uint64_t* __restrict__ len, const uint8_t* __restrict__ flags,
    const uint32_t* __restrict__ mask, const uint64_t* __restrict__ out_off, const uint64_t* __restrict__ size,
    const uint32_t* __restrict__ tile_first, const unsigned long long* __restrict__ span, uint64_t n, uint64_t tile0,
    uint64_t ntiles, build_uni uni, uint32_t xgroup) {
    const uint64_t t = tile0 + xcd_group_tile(blockIdx.x, ntiles, xgroup);
    constexpr uint64_t TILE = (uint64_t)T * U * 16u;
    build_one_tile<T, U, NT, SF, C>(out, out_len, pay, plen, pay_off, len, flags, mask, out_off, size, span, n, t,
                                 uni.stride ? build_uni_idx(uni, t * TILE, TILE, n, out_len)
                                            : build_load_idx(tile_first, span, t, n),
                                 uni);
}


hipError_t launch_exclusive_scan(const uint64_t* in, uint64_t* out, uint64_t n, uint64_t* tmp, uint64_t* total,
                                 hipStream_t st) {
    if (n == 0) return hipMemsetAsync(total, 0, 8, st);
    const uint64_t nb = (n + SCAN_B - 1) / SCAN_B;
    uint64_t* sums = tmp;
    uint64_t* base = tmp + nb;
    hipLaunchKernelGGL(k_scan_blocks, dim3((uint32_t)nb), dim3(SCAN_T), 0, st, in, out, n, sums,
                       nb == 1 ? total : (uint64_t*)nullptr);
    if (nb > 1) {
        hipError_t e = launch_exclusive_scan(sums, base, nb, tmp + 2 * nb, total, st);
        if (e != hipSuccess) return e;
        hipLaunchKernelGGL(k_add_block_base, dim3((uint32_t)nb), dim3(SCAN_T), 0, st, out, n, base);
    }
    return hipGetLastError();
}

// stat[1] += frames whose payload range leaves [0, plen) or that are masked
// without a key table; stat[2] += frames that break the uniform layout (a
// size other than frame 0's, or a payload offset step other than frame 1's,
// or a negative one, or a payload length other than frame 0's); stat[3],
// stat[4], stat[5] = pay_off[0], pay_off[1] - pay_off[0], len[0].
__global__ void k_tx_check(const uint64_t* __restrict__ pay_off, const uint64_t* __restrict__ len,
                           const uint8_t* __restrict__ flags, const uint32_t* __restrict__ mask,
                           const uint64_t* __restrict__ size, uint64_t n, uint64_t plen,
                           unsigned long long* __restrict__ stat) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    bool b = false, nu = false;
    if (i < n) {
        const uint64_t o = pay_off[i], l = len[i];
        b = o > plen || l > plen - o || ((flags[i] & F_MASK) && !mask);
        if (i) {
            const uint64_t p0 = pay_off[0], p1 = pay_off[1], pp = pay_off[i - 1];
            nu = size[i] != size[0] || l != len[0] || p1 < p0 || o < pp || o - pp != p1 - p0;
        } else {
            stat[3] = o;
            stat[4] = n > 1 ? pay_off[1] - o : 0;
            stat[5] = l;
        }
    }
    const uint64_t m = __ballot(b), mu = __ballot(nu);
    if ((threadIdx.x & 63) == 0) {
        if (m) atomicAdd(stat + 1, (unsigned long long)__popcll(m));
        if (mu) atomicAdd(stat + 2, (unsigned long long)__popcll(mu));
    }
}

hipError_t launch_tx_check(const uint64_t* pay_off, const uint64_t* len, const uint8_t* flags, const uint32_t* mask,
                           const uint64_t* size, uint64_t n, uint64_t plen, uint64_t* stat, hipStream_t st) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_tx_check, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, st, pay_off, len, flags, mask,
                       size, n, plen, reinterpret_cast<unsigned long long*>(stat));
    return hipGetLastError();
}

// Build geometries: X(index, threads per workgroup, chunks per thread, XCD
// order, nontemporal realigning loads, stage-first, compact records); 0 is the
// default.  History (profiles/, DESIGN.md sec. 5 "Transmit side"): 256 x 2
// linear was the default through round 3 (stage-first: c2 0.64 -> 0.60 ms, c3
// 20.93 -> 20.50 ms, r1an_raw); larger 256-thread tiles lost occupancy, the
// XCD-contiguous order halved this out-of-place stream.  Round 4: compact
// tile-relative records (r4m_raw); then one-wave workgroups with 4 KiB tiles
// -- no staging barrier across waves, every wave's tile independent: c2
// packed 0.52 -> 0.455 ms, c3 packed 22.4 -> 20.6 ms, c4 1.40 -> 1.30 ms
// (r4t_raw, r4u_raw); 64 x 8 (LDS-bound to 3 waves per SIMD) and 64 x 2 ran
// slower at every shape (r4aa_raw); staging the span by LDS-DMA changed
// nothing measurable (r4ac_raw).  The lean form without the records-first
// path: no VGPR spills, c2 0.46-0.47 -> 0.42-0.45 ms (r4ae_raw, r4af_raw;
// with LDS-DMA staging and no streaming path as well, the same at c2 and
// 1.6x slower at c3).  Tried and gone in round 4: a grid-stride form with the
// next tile's index prefetched (r4l_raw), a position-derived index for uniform
// layouts (r4o_raw, r4p_raw), a short path for chunks inside one payload
// (r4r_raw).
#define HVWS_BUILD_GEOMS(X)               \
    X(0, 64, 4, false, false, true, 1)    \
    X(1, 256, 2, false, false, true, 1)   \
    X(2, 256, 2, false, false, true, 0)   \
    X(3, 64, 2, false, false, true, 1)    \
    X(4, 128, 2, false, false, true, 1)   \
    X(5, 64, 4, false, false, true, 2)

namespace {
// $HVWS_EXPERIMENT build: a fixed geometry (A/B runs); else by the batch's mean frame:
// the lean one-wave form from 256 B to 4 KiB per frame (c2: 0.43 against
// 0.46 ms), the default above it (c3: 20.2-20.7 against 22.3 ms;
// profiles/r4v_raw) and below it -- the lean form stages 16 frames per 4 KiB
// tile, so under ~256 B most of its tiles would take the per-chunk search.
int build_pick(uint64_t out_len, uint64_t n) {
    const char* e = experiment("build");   // read per call (tests switch it)
    const int forced = e ? atoi(e) : -1;
    if (forced >= 0 && forced < 6) return forced;
    const uint64_t mean = n ? out_len / n : 0;
    return mean >= 256 && mean < 4096 ? 5 : 0;
}
uint64_t build_tile(int v) {
    switch (v) {
#define X(I, T, U, S, N, F, C) \
    case I:                    \
        return (uint64_t)T * U * 16u;
        HVWS_BUILD_GEOMS(X)
#undef X
    }
    return 0;
}
}  // namespace

const char* build_kernel_name(int v) {
    switch (v) {
#define X(I, T, U, S, N, F, C) \
    case I:                    \
        return C == 2 ? "k_build<" #T "x" #U ",lean>" : (C ? "k_build<" #T "x" #U ">" : "k_build<" #T "x" #U ",wide>");
        HVWS_BUILD_GEOMS(X)
#undef X
    }
    return "?";
}

int tx_variant(uint64_t out_len, uint64_t n) { return build_pick(out_len, n); }
uint64_t tx_tile(int v) { return build_tile(v); }


hipError_t launch_tx_index(const uint64_t* out_off, const uint64_t* size, const uint64_t* pay_off, const uint64_t* len,
                           const uint8_t* flags, uint64_t n, uint64_t ntiles, uint64_t tile, uint32_t* tile_first,
                           uint64_t* span, hipStream_t st) {
    unsigned long long* sp = reinterpret_cast<unsigned long long*>(span);
    hipLaunchKernelGGL(k_tx_index_fill, dim3((uint32_t)((ntiles + 1 + 255) / 256)), dim3(256), 0, st, tile_first, sp,
                       ntiles);
    if (n) hipLaunchKernelGGL(k_tx_index, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, st, out_off, size, pay_off,
                              len, flags, n, ntiles, tile, tile_first, sp);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    return launch_tile_fixup(out_off, size, n, tile_first, ntiles, tile, st);
}

hipError_t launch_build(uint8_t* out, uint64_t out_len, const uint8_t* pay, uint64_t plen, const uint64_t* pay_off,
                        const uint64_t* len, const uint8_t* flags, const uint32_t* mask, const uint64_t* out_off,
                        const uint64_t* size, const uint32_t* tile_first, const uint64_t* span, uint64_t n, int v,
                        hipStream_t st, const uint64_t* uni) {
    const unsigned long long* sp = reinterpret_cast<const unsigned long long*>(span);
    build_uni u = {0, 0, 0, 0, 0.0};
    if (uni && uni[0]) {
        u.stride = uni[0];
        u.hdr = uni[1];
        u.pay_a = uni[2];
        u.pay_b = uni[3];
        u.inv = 1.0 / (double)uni[0];
    }
    const uint64_t tile = build_tile(v);
    const uint64_t ntiles = (out_len + tile - 1) / tile;
    // Runs of xg adjacent tiles per XCD (xcd_group_tile): a boundary line of
    // a payload span, and a line of the flags and keys, shared by neighbouring
    // tiles is then fetched once per run instead of once per tile.  DRAM-side
    // reads per payload byte (profiles/r6_raw/tx_traffic): the lean form at c2
    // 1.047 / 1.068 (rx layout / packed) at xg 1, 1.027 / 1.029 at 4, 1.021 /
    // 1.019 at 8 -- but 3-5 % slower (interleaved, r6h: 0.362-0.381 against
    // 0.344-0.350 ms), so the lean form keeps 1; k_build<64x4> at c3 1.027 /
    // 1.058 at 1, 1.019 / 1.036 at 2 at the same speed (20.29-20.36 / 20.72-
    // 20.74 against 20.39-20.60 / 20.63-20.66 ms), 1.012 / 1.022 at 4 but 3-5 %
    // slower.  ($HVWS_EXPERIMENT build_xgroup)
    static const uint32_t xg_env =
        experiment("build_xgroup") ? (uint32_t)atoi(experiment("build_xgroup")) : 0xFFFFFFFFu;
    const uint32_t xg = xg_env != 0xFFFFFFFFu ? xg_env : (v == 5 ? 1u : 2u);
    // a grid beyond 2^32-1 work-items is silently truncated: split the launch
    const uint64_t per_launch = 0xFFFFFFFFull / 256;
    for (uint64_t t0 = 0; t0 < ntiles; t0 += per_launch) {
        const uint64_t nt = min(per_launch, ntiles - t0);
        switch (v) {
#define X(I, T, U, S, N, F, C)                                                                                 \
    case I:                                                                                                    \
        hipLaunchKernelGGL((k_build<T, U, N, F, C>), dim3((uint32_t)nt), dim3(T), 0, st, out, out_len, pay, plen, \
                           pay_off, len, flags, mask, out_off, size, tile_first, sp, n, t0, nt, u, xg);       \
        break;
            HVWS_BUILD_GEOMS(X)
#undef X
        }
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

}  // namespace hvws

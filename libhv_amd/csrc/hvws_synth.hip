// hvws_synth.hip -- synthetic masked-frame batches and digests on the device.
//
// Bench/test data only; not on the receive path.
// Frame layout is websocket_build_frame's (reference
// http/websocket_parser.c:207-256); plaintext byte j of frame i is
// ows_plain_byte(seed, i, j) of oracle/ws_oracle.c, restated here.
#include "hvws_internal.h"

namespace hvws {

__device__ __forceinline__ uint64_t mix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__device__ __forceinline__ uint32_t hdr_len_of(uint32_t flags, uint64_t n) {
    uint32_t ext = n < 126 ? 0u : (n <= 0xFFFFu ? 2u : 8u);
    return 2u + ext + ((flags & F_MASK) ? 4u : 0u);
}

// Byte h of the header of a frame (flags, length n, key).
__device__ __forceinline__ uint32_t hdr_byte(uint32_t flags, uint64_t n, uint32_t key, uint32_t h) {
    uint32_t ext = n < 126 ? 0u : (n <= 0xFFFFu ? 2u : 8u);
    if (h == 0) return ((flags & F_FIN) ? 0x80u : 0u) | (flags & F_OPMASK);
    if (h == 1) {
        uint32_t code = n < 126 ? (uint32_t)n : (ext == 2 ? 126u : 127u);
        return ((flags & F_MASK) ? 0x80u : 0u) | code;
    }
    if (h < 2 + ext) {
        uint32_t k = h - 2;   // big-endian
        return (uint32_t)(n >> (8 * (ext - 1 - k))) & 0xFFu;
    }
    return (key >> (8 * (h - 2 - ext))) & 0xFFu;
}

__global__ void k_frame_sizes(const uint8_t* __restrict__ flags, const uint64_t* __restrict__ length,
                              uint64_t nframes, uint64_t* __restrict__ out) {
    uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < nframes) out[i] = hdr_len_of(flags[i], length[i]) + length[i];
}

constexpr uint64_t SYN_TILE = 256u * 16u * 4u;   // 16 KiB

__global__ __launch_bounds__(256) void k_synth(uint8_t* __restrict__ buf, uint64_t buf_len, uint64_t seed,
                                               uint64_t nframes, const uint64_t* __restrict__ frame_off,
                                               const uint8_t* __restrict__ flags,
                                               const uint32_t* __restrict__ mask,
                                               const uint64_t* __restrict__ length,
                                               const uint8_t* __restrict__ text,
                                               const uint64_t* __restrict__ frame_size,
                                               const uint32_t* __restrict__ tile_first, int mode,
                                               unsigned long long* __restrict__ mismatches) {
    const uint64_t t = blockIdx.x;
    unsigned long long bad = 0;
    const uint32_t kfirst = tile_first[t];
    for (int i = 0; i < 4; ++i) {
        const uint64_t c = t * SYN_TILE + ((uint64_t)i * 256u + threadIdx.x) * 16u;
        if (c >= buf_len) break;
        // first frame ending after c
        uint64_t k = kfirst;
        while (k < nframes && frame_off[k] + frame_size[k] <= c) ++k;
        // Fast path: the 16 bytes lie inside one payload -- three mix64 words
        // cover them; no per-byte frame walk.
        if (k < nframes && c + 16 <= buf_len) {
            const uint32_t fl = flags[k];
            const uint64_t n = length[k];
            const uint64_t ps = frame_off[k] + hdr_len_of(fl, n);
            if (ps <= c && c + 16 <= ps + n) {
                const uint64_t j0 = c - ps;
                const uint64_t fs = mix64(seed + k * 0x9E3779B97F4A7C15ull);
                const uint32_t sh = (uint32_t)(j0 & 7u) * 8u;
                const uint64_t q = j0 >> 3;
                const uint64_t w0 = mix64(fs + q), w1 = mix64(fs + q + 1);
                uint64_t lo = w0, hi = w1;
                if (sh) {
                    const uint64_t w2 = mix64(fs + q + 2);
                    lo = (w0 >> sh) | (w1 << (64u - sh));
                    hi = (w1 >> sh) | (w2 << (64u - sh));
                }
                if (text && text[k]) {
                    uint64_t tl = 0, th = 0;
#pragma unroll
                    for (int b = 0; b < 8; ++b) {
                        tl |= (uint64_t)(0x20u + ((((uint32_t)(lo >> (8 * b)) & 0xFFu) * 95u) >> 8)) << (8 * b);
                        th |= (uint64_t)(0x20u + ((((uint32_t)(hi >> (8 * b)) & 0xFFu) * 95u) >> 8)) << (8 * b);
                    }
                    lo = tl;
                    hi = th;
                }
                if (mode != 2 && (fl & F_MASK)) {
                    const uint32_t key = mask[k];
                    const uint32_t r = (uint32_t)(j0 & 3u) * 8u;
                    const uint32_t kw = r ? (key >> r) | (key << (32u - r)) : key;
                    const uint64_t kk = (uint64_t)kw | ((uint64_t)kw << 32);
                    lo ^= kk;
                    hi ^= kk;
                }
                uint64_t* p = reinterpret_cast<uint64_t*>(buf + c);
                if (mode == 0) {
                    p[0] = lo;
                    p[1] = hi;
                } else {
                    const uint64_t d0 = p[0] ^ lo, d1 = p[1] ^ hi;
                    if (d0 | d1) {
                        for (int b = 0; b < 8; ++b) {
                            bad += ((d0 >> (8 * b)) & 0xFFu) ? 1u : 0u;
                            bad += ((d1 >> (8 * b)) & 0xFFu) ? 1u : 0u;
                        }
                    }
                }
                continue;
            }
        }
        uint8_t cur[16];
        uint8_t exp[16];
        bool cov[16];
        const uint32_t nb = (uint32_t)(buf_len - c < 16 ? buf_len - c : 16);
        for (uint32_t b = 0; b < 16; ++b) cur[b] = b < nb ? buf[c + b] : 0;
        uint64_t wid = ~0ull, w = 0, fseed = 0, fk = ~0ull;
        for (uint32_t b = 0; b < 16; ++b) {
            const uint64_t a = c + b;
            exp[b] = cur[b];
            cov[b] = false;
            if (b >= nb) continue;
            while (k < nframes && frame_off[k] + frame_size[k] <= a) ++k;
            if (k >= nframes || frame_off[k] > a) continue;
            const uint32_t fl = flags[k];
            const uint64_t n = length[k];
            const uint32_t key = mask[k];
            const uint32_t hl = hdr_len_of(fl, n);
            const uint64_t rel = a - frame_off[k];
            cov[b] = true;
            if (rel < hl) {
                exp[b] = (uint8_t)hdr_byte(fl, n, key, (uint32_t)rel);
                continue;
            }
            const uint64_t j = rel - hl;
            if (fk != k) {
                fk = k;
                fseed = mix64(seed + k * 0x9E3779B97F4A7C15ull);
                wid = ~0ull;
            }
            if ((j >> 3) != wid) {
                wid = j >> 3;
                w = mix64(fseed + wid);
            }
            uint32_t v = (uint32_t)(w >> ((j & 7u) * 8u)) & 0xFFu;
            if (text && text[k]) v = 0x20u + ((v * 95u) >> 8);
            if (mode != 2 && (fl & F_MASK)) v ^= (key >> (8 * (j & 3u))) & 0xFFu;
            exp[b] = (uint8_t)v;
        }
        if (mode == 0) {
            for (uint32_t b = 0; b < nb; ++b)
                if (cov[b]) buf[c + b] = exp[b];
        } else {
            for (uint32_t b = 0; b < nb; ++b) bad += (cur[b] != exp[b]) ? 1u : 0u;
        }
    }
    if (mode != 0 && bad) atomicAdd(mismatches, bad);
}

__global__ __launch_bounds__(256) void k_digest(const uint8_t* __restrict__ buf, uint64_t len,
                                                unsigned long long* __restrict__ out) {
    const uint64_t nwords = (len + 7) / 8;
    uint64_t acc = 0;
    for (uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; k < nwords;
         k += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t w;
        if (k * 8 + 8 <= len) {
            w = reinterpret_cast<const uint64_t*>(buf)[k];
        } else {
            w = 0;
            for (uint64_t b = 0; k * 8 + b < len; ++b) w |= (uint64_t)buf[k * 8 + b] << (8 * b);
        }
        acc += mix64(w ^ (k * 0xD1B54A32D192ED03ull));
    }
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_down(acc, o);
    if ((threadIdx.x & 63u) == 0) atomicAdd(out, (unsigned long long)acc);
}

hipError_t launch_frame_sizes(const uint8_t* flags, const uint64_t* length, uint64_t nframes, uint64_t* out,
                              hipStream_t st) {
    if (nframes == 0) return hipSuccess;
    hipLaunchKernelGGL(k_frame_sizes, dim3((uint32_t)((nframes + 255) / 256)), dim3(256), 0, st, flags, length,
                       nframes, out);
    return hipGetLastError();
}

hipError_t launch_synth(uint8_t* buf, uint64_t buf_len, uint64_t seed, uint64_t nframes,
                        const uint64_t* frame_off, const uint8_t* flags, const uint32_t* mask,
                        const uint64_t* length, const uint8_t* text, const uint64_t* frame_size,
                        const uint32_t* tile_first, int mode, unsigned long long* mismatches,
                        hipStream_t st) {
    const uint64_t ntiles = (buf_len + SYN_TILE - 1) / SYN_TILE;
    if (ntiles == 0) return hipSuccess;
    hipLaunchKernelGGL(k_synth, dim3((uint32_t)ntiles), dim3(256), 0, st, buf, buf_len, seed, nframes,
                       frame_off, flags, mask, length, text, frame_size, tile_first, mode, mismatches);
    return hipGetLastError();
}

hipError_t launch_digest(const uint8_t* buf, uint64_t len, unsigned long long* out, hipStream_t st) {
    hipLaunchKernelGGL(k_digest, dim3(2048), dim3(256), 0, st, buf, len, out);
    return hipGetLastError();
}

uint64_t synth_tile() { return SYN_TILE; }

}  // namespace hvws

// hvws_sieve.hip -- parallel frame discovery for one long stream of mixed
// frame sizes (the frame sieve).
//
// The wire format chains headers: frame i+1 starts where frame i's length
// says (http/websocket_parser.c:72-164), so one stream of random sizes is a
// serial walk -- one dependent HBM round trip per frame (~2 us), 160 ms for
// the 74 701 frames of config 4 as one stream.  The sieve replaces the walk
// with data-parallel passes whose result is exact by construction:
//
//   k_sieve_count    every byte position of the stream is tested in parallel
//                    (SWAR over the tile staged in LDS) for a plausible
//                    client frame header -- RSV clear, opcode 0-2/8-A, MASK
//                    set, minimal length, control frames FIN and <= 125 B
//                    (about 1 position in 57 of random payload passes) --
//                    and a candidate survives when the chain of the next
//                    SV_DEPTH headers it implies is plausible too (a false
//                    candidate survives with probability ~57^-3).  Survivors
//                    of each 8 KiB tile are counted and kept in a small
//                    per-tile slot, or a run of a shared pool when more.
//   scan             tile counts -> tile bases.
//   k_sieve_fill     sorted array of survivors from the slots (and the pool
//                    runs of busy tiles); a candidate whose chain left its
//                    tile is flagged, and
//   k_sieve_verify   finishes those from HBM, one thread each;
//   scan, compact    -> sorted survivor array S.
//   k_sieve_link     succ(j): walk the exact frames from S[j] until one
//                    starts at a survivor (looked up in the S entries of its
//                    tile), hops(j) = frames walked; or none.
//
// Windows.  A long stream of large frames need not be sieved everywhere: only
// the first wt tiles of every rt ("windows", sized past the largest frame the
// traffic holds) are, and the link walks cross the gaps frame by frame -- one
// dependent header load per frame, ~rt * 8 KiB / mean frame size of them per
// region, all regions in parallel.  The host picks rt from the last exact
// count of the context's one-segment scans (sieve_geometry); rt == wt sieves
// every tile (hops(j) is then mostly 1).
//   k_sieve_jump     pointer doubling from the stream's first whole frame
//                    (known exactly from k_head): after round r the first
//                    2^(r+1) frames of the true chain are marked.
//   scan             marks * hops -> record ranks.
//   k_sieve_emit     frame records of the marked chain (each node re-walks
//                    its hops).
//
// Exactness: the chain is followed from a true header through exact
// successor positions, so every marked node is a true frame and they come in
// stream order; plausibility only decides which true frames the chain can
// reach.  Where a true frame is not a survivor (an unmasked frame, RSV bits,
// a reserved opcode: legal for the reference) the chain stops
// there and k_walk continues from that byte with the exact walk.  The
// parity tests run random and quirk streams through it.
#include "hvws_dev.h"

namespace hvws {

constexpr uint32_t SV_THREADS = 256;
constexpr uint32_t SV_PER = 32;                        // byte positions per thread
constexpr uint32_t SV_TILE = SV_THREADS * SV_PER;      // 8 KiB
constexpr uint32_t SV_HALO = 512;                      // bytes staged past the tile (headers, 7-bit-length hops)
constexpr uint32_t SV_SLOT = 16;                       // survivors kept per tile by the count pass
constexpr int SV_DEPTH = 3;                            // hops a survivor's chain must stay plausible
constexpr uint32_t SV_TERM = 0xFFFFFFFFu;
constexpr uint32_t SV_GRID = 4096;
// k_sieve_count's grid when windows are on (~37 000 tiles at c4): its
// workgroups run beside the unmask at high priority, and 4096 of them held
// the device -- the unmask pieces beside them ran at ~40 %.  c4 as one stream,
// ms per step by grid (sieve_hops 256): 4096 1.52, 2048 1.519, 1024 1.506,
// 512 1.58 (the chain then bounds the step), 256 1.727; with 320 frames per
// region 1024 1.488-1.496, 1280 1.494 (profiles/r5_raw/pieces, sg*/sgh*).
constexpr uint32_t SV_GRID_WINDOWS = 1024;
constexpr uint32_t SV_HOP_CAP = 4096;                  // frames one link walk may cross

// Tiles of the segment that are sieved (the first wt of every rt of the NT
// tiles from A0), and the stream tile of sieved tile t.
__device__ __forceinline__ uint64_t sv_ntiles(uint64_t NT, uint32_t rt, uint32_t wt) {
    if (!NT) return 0;
    const uint64_t nreg = (NT + rt - 1) / rt, last = NT - (nreg - 1) * rt;
    return (nreg - 1) * wt + (last < wt ? last : wt);
}
__device__ __forceinline__ uint64_t sv_tile(uint64_t t, uint32_t rt, uint32_t wt) {
    return rt == wt ? t : (t / wt) * rt + t % wt;
}

// The sieve runs on segment 0 when k_head found its first whole frame at
// pos, sizes that vary (probe) and no verified uniform prefix.
__device__ __forceinline__ bool sieve_wanted(const dseg* segs, const dmid* mid, const uint64_t* npred,
                                             uint64_t sieve_min, uint64_t& sb, uint64_t& L, uint64_t& pos) {
    const dmid& m = mid[0];
    sb = segs[0].off;
    L = segs[0].len;
    pos = m.pos;
    return m.st.state == S_START && m.pad != 0 && npred[0] == 0 && pos < L && L - pos >= sieve_min;
}

__device__ __forceinline__ bool plausible(const hdr& h) { return h.viol == 0 && (h.length >> 48) == 0; }

// Survivor test of the candidate at segment offset q (k_sieve_verify, from
// HBM): a whole frame with a plausible header whose next SV_DEPTH headers are
// plausible, or end the stream (exactly, or with a header or frame cut by the
// segment end).
__device__ bool survivor(const uint8_t* rx, uint64_t rx_len, uint64_t sb, uint64_t L, uint64_t q) {
    const uint64_t end = sb + L, a = sb + q;
    auto load = [&](uint64_t x) {
        uint64_t lo, hi;
        ld16(rx, rx_len, x, lo, hi);
        return parse_hdr(lo, hi);
    };
    hdr h = load(a);
    const uint64_t r0 = end - a;
    if (!plausible(h) || h.hlen > r0 || h.length > r0 - h.hlen) return false;
    uint64_t x = a + h.hlen + h.length;
#pragma unroll 1
    for (int d = 0; d < SV_DEPTH; ++d) {
        const uint64_t r = end - x;
        if (r < 14) return true;   // end of stream, or a header that may be cut by it
        h = load(x);
        if (!plausible(h)) return false;
        if (h.length > r - h.hlen) return true;   // frame cut by the segment end
        x += h.hlen + h.length;
    }
    return true;
}

// Verdicts of the tile pass (quick_verdict): rejected, a survivor without a
// doubt, or pending -- k_sieve_verify decides from HBM.
enum : uint32_t { SV_NO = 0, SV_YES = 1, SV_PENDING = 2 };

// Tile staging in two halves so the next tile's loads can be in flight while
// the current tile is sieved: each thread loads 16-B chunks c = t, t + 256
// (and t + 512 for the halo) of [T0, T0 + SV_TILE + SV_HALO) into registers,
// then stores them to LDS.  Bytes past rx_len read 0.
typedef uint32_t sv_u32x4 __attribute__((ext_vector_type(4)));
// Thread t holds chunks t and t + 256 of the tile, and threads 8h hold halo
// chunk 512 + h (h < 32), each with the dword that follows it.
struct tile_regs {
    sv_u32x4 v[3];
    uint32_t nx[3];
};
constexpr uint32_t SV_HCH = SV_HALO / 16;   // halo chunks

__device__ __forceinline__ bool halo_lane(uint32_t t) { return (t & 7u) == 0 && (t >> 3) < SV_HCH; }

// 16 bytes at a, bytes past rx_len read 0 (the last tile only: kept out of
// line so its byte loop does not raise the kernel's register allocation).
__device__ __attribute__((noinline)) sv_u32x4 load_chunk(const uint8_t* rx, uint64_t rx_len, uint64_t a) {
    if (a + 16 <= rx_len) return *reinterpret_cast<const sv_u32x4*>(rx + a);
    uint32_t b[4] = {0u, 0u, 0u, 0u};
    for (uint32_t k = 0; a + k < rx_len && k < 16; ++k) b[k >> 2] |= (uint32_t)rx[a + k] << (8 * (k & 3));
    return sv_u32x4{b[0], b[1], b[2], b[3]};
}

__device__ __forceinline__ void load_tile(const uint8_t* rx, uint64_t rx_len, uint64_t T0, tile_regs& r) {
    const uint32_t t = threadIdx.x;
    const uint32_t hc = 2 * SV_THREADS + (t >> 3);   // halo chunk of a halo lane
    // Every lane loads a halo chunk (other lanes the first one, the same
    // line): a load under the halo lanes' mask kept the register's old value
    // for the rest, and the merge copy waited for the prefetch at once
    // (s_waitcnt vmcnt(0) before the tile's sieve, so nothing overlapped).
    const uint32_t hcu = halo_lane(t) ? hc : 2 * SV_THREADS;
    const uint8_t* p = rx + T0;
    if (T0 + SV_TILE + SV_HALO + 16 <= rx_len) {   // every tile but the last
        r.v[0] = *reinterpret_cast<const sv_u32x4*>(p + 16 * t);
        r.v[1] = *reinterpret_cast<const sv_u32x4*>(p + 16 * (t + SV_THREADS));
        r.nx[0] = *reinterpret_cast<const uint32_t*>(p + 16 * (t + 1));
        r.nx[1] = *reinterpret_cast<const uint32_t*>(p + 16 * (t + SV_THREADS + 1));
        r.v[2] = *reinterpret_cast<const sv_u32x4*>(p + 16 * hcu);
        r.nx[2] = *reinterpret_cast<const uint32_t*>(p + 16 * (hcu + 1));
        return;
    }
    r.v[0] = load_chunk(rx, rx_len, T0 + (uint64_t)t * 16);
    r.v[1] = load_chunk(rx, rx_len, T0 + (uint64_t)(t + SV_THREADS) * 16);
    r.nx[0] = load_chunk(rx, rx_len, T0 + (uint64_t)(t + 1) * 16).x;
    r.nx[1] = load_chunk(rx, rx_len, T0 + (uint64_t)(t + SV_THREADS + 1) * 16).x;
    r.v[2] = load_chunk(rx, rx_len, T0 + (uint64_t)hcu * 16);
    r.nx[2] = load_chunk(rx, rx_len, T0 + (uint64_t)(hcu + 1) * 16).x;
}

__device__ __forceinline__ void store_tile(uint32_t* l, const tile_regs& r) {
    const uint32_t t = threadIdx.x;
    *reinterpret_cast<sv_u32x4*>(l + 4 * t) = r.v[0];
    *reinterpret_cast<sv_u32x4*>(l + 4 * (t + SV_THREADS)) = r.v[1];
    if (halo_lane(t)) *reinterpret_cast<sv_u32x4*>(l + 4 * (2 * SV_THREADS + (t >> 3))) = r.v[2];
}

// Candidate word of one 16-byte chunk (positions q = 16c + 4d + j, d = dword,
// j = byte): a byte b0 with (b0 & 0x77) <= 2 -- RSV clear, opcode 0-2 or 8-A
// -- followed by a byte with MASK set.  SWAR, 4 positions per dword:
// (b0 & 0x77) + 0x7D sets bit 7 iff (b0 & 0x77) >= 3, with no carry between
// bytes.  The result is kept transposed: bit 8j + d of the word is position
// 4d + j of the chunk (cand_bit() reads it).
__device__ __forceinline__ uint32_t chunk_candidates(sv_u32x4 v, uint32_t next) {
    const uint32_t w[5] = {v.x, v.y, v.z, v.w, next};
    uint32_t out = 0;
#pragma unroll
    for (int d = 0; d < 4; ++d) {
        const uint32_t bad = (w[d] & 0x77777777u) + 0x7D7D7D7Du;
        const uint32_t b1 = __builtin_amdgcn_alignbyte(w[d + 1], w[d], 1);   // the byte after each
        const uint32_t c = b1 & ~bad & 0x80808080u;
        out |= c >> (7 - d);
    }
    return out;
}

__device__ __forceinline__ uint32_t cand_bit(const uint32_t* cb, uint32_t q) {
    return (cb[q >> 4] >> (8u * (q & 3u) + ((q >> 2) & 3u))) & 1u;
}

__device__ __forceinline__ uint32_t lds_byte(const uint32_t* l, uint32_t p) { return (l[p >> 2] >> (8 * (p & 3u))) & 0xFFu; }

// Verdict from the staged bytes and the candidate bitmap where that is
// enough: SV_NO, SV_PENDING, or SV_FULL when only the full test can decide
// (the tile pass hands those to k_sieve_verify too).  Every rejection is
// implied by survivor() rejecting: control frames must be FIN and <= 125 bytes, lengths minimal
// and < 2^48, and a header the chain reaches must be a candidate -- followed
// through the bitmap for 7-bit lengths while the next header is staged.
// A plausible 16-bit-length candidate whose next header lies beyond the
// staged bytes is SV_PENDING without a parse (k_sieve_verify finishes it).
constexpr uint32_t SV_FULL = 3;

__device__ __forceinline__ uint32_t quick_verdict(const uint32_t* l, const uint32_t* cb, uint32_t q, uint32_t hrel) {
    // hrel: segment end relative to the tile start (clamped; 32-bit math only)
    const uint32_t b0 = lds_byte(l, q), len7 = lds_byte(l, q + 1) & 0x7Fu;
    if ((b0 & 8u) && (!(b0 & 0x80u) || len7 >= 126)) return SV_NO;   // control frame
    if (len7 == 127) return (lds_byte(l, q + 2) | lds_byte(l, q + 3)) ? SV_NO : SV_FULL;
    if (len7 == 126) {
        const uint32_t n = (lds_byte(l, q + 2) << 8) | lds_byte(l, q + 3);
        if (n < 126) return SV_NO;
        const uint32_t x = q + 8u + n;
        if (x > hrel) return SV_NO;                                   // not whole
        return x + 14 <= hrel && x + 16 > SV_TILE + SV_HALO ? SV_PENDING : SV_FULL;
    }
    uint32_t x = q + 6u + len7;
#pragma unroll 1
    for (int d = 0; d < SV_DEPTH; ++d) {
        if (x + 16 > SV_TILE + SV_HALO || x + 14 > hrel) return SV_FULL;
        if (!cand_bit(cb, x)) return SV_NO;
        const uint32_t n7 = lds_byte(l, x + 1) & 0x7Fu;
        if (n7 >= 126) return SV_FULL;
        x += 6u + n7;
    }
    return SV_FULL;
}

// Wave-wide exclusive prefix of v; *tot = wave sum.
__device__ __forceinline__ uint32_t wave_prefix(uint32_t v, uint32_t& tot) {
    const uint32_t lane = threadIdx.x & 63u;
    uint32_t x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o);
        if (lane >= (uint32_t)o) x += y;
    }
    tot = __shfl(x, 63);
    return x - v;
}

constexpr uint32_t SV_WLIST = 512;   // candidates a wave handles per round

struct sieve_lds {
    uint32_t l[(SV_TILE + SV_HALO) / 4 + 8];   // the tile's bytes (+ halo)
    uint32_t cb[(SV_TILE + SV_HALO) / 16];     // candidate words, one per 16-byte chunk
    uint32_t sbits[2][SV_TILE / 32];           // survivors (and pending ones), bit p of word p / 32; by tile parity
    uint32_t pbits[2][SV_TILE / 32];           // survivors still to be verified from HBM
    uint16_t list[SV_THREADS / 64][SV_WLIST];  // each wave's candidate positions
};

// Candidates of the staged tile, then the survivor test: each wave compacts
// its own candidates into a list so every lane checks about one (a loop over
// each thread's 32 positions waited for the busiest lane); survivors land in
// the tile's bitmaps.  Two block barriers per tile: tile + candidate words
// staged, and survivors complete.
__device__ __forceinline__ void sieve_tile(const uint8_t* rx, uint64_t rx_len, sieve_lds& sh, tile_regs& r, int par,
                                           uint64_t T0, bool have_next, uint64_t next_T0, uint64_t sb, uint64_t L,
                                           uint64_t pos) {
    const uint32_t t = threadIdx.x, lane = t & 63u, w = t >> 6;
    store_tile(sh.l, r);
    const uint32_t w0 = chunk_candidates(r.v[0], r.nx[0]);
    const uint32_t w1 = chunk_candidates(r.v[1], r.nx[1]);
    sh.cb[t] = w0;
    sh.cb[t + SV_THREADS] = w1;
    if (halo_lane(t)) sh.cb[2 * SV_THREADS + (t >> 3)] = chunk_candidates(r.v[2], r.nx[2]);
    sh.sbits[par][t] = 0;
    sh.pbits[par][t] = 0;
    if (have_next) load_tile(rx, rx_len, next_T0, r);   // the next tile's loads under this one's work
    __syncthreads();
    const uint64_t lo = sb + pos, hi = sb + L;
    const uint32_t qlo = lo > T0 ? (uint32_t)(lo - T0) : 0u;
    const uint32_t qhi = hi - T0 < SV_TILE ? (uint32_t)(hi - T0) : SV_TILE;
    const uint32_t hrel = hi - T0 < (1u << 30) ? (uint32_t)(hi - T0) : (1u << 30);   // > any 16-bit-length frame end
    uint32_t wtot;
    const uint32_t first = wave_prefix(__builtin_popcount(w0) + __builtin_popcount(w1), wtot);
    uint16_t* list = sh.list[w];
    for (uint32_t base = 0; base < wtot; base += SV_WLIST) {
        uint32_t k = first;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            uint32_t m = h ? w1 : w0;
            const uint32_t c = h ? t + SV_THREADS : t;
            while (m) {
                const uint32_t b = __builtin_ctz(m);
                m &= m - 1;
                if (k >= base && k < base + SV_WLIST) list[k - base] = (uint16_t)(16u * c + 4u * (b & 7u) + (b >> 3));
                ++k;
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const uint32_t nl = wtot - base < SV_WLIST ? wtot - base : SV_WLIST;
        for (uint32_t e = lane; e < nl; e += 64) {
            const uint32_t q = list[e];
            if (q < qlo || q >= qhi) continue;
            uint32_t v = quick_verdict(sh.l, sh.cb, q, hrel);
            if (v == SV_NO) continue;
            if (v == SV_FULL) v = SV_PENDING;   // k_sieve_verify decides from HBM (keeps this loop lean)
            if (v != SV_NO) atomicOr(&sh.sbits[par][q >> 5], 1u << (q & 31u));
            if (v == SV_PENDING) atomicOr(&sh.pbits[par][q >> 5], 1u << (q & 31u));
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
    __syncthreads();
}

// Wave 0 records tile t's survivors (bitmaps of parity par) in position
// order: up to SV_SLOT in the tile's slot; a tile with more reserves a run
// of the pool and records its start in slot word 0.  Every survivor comes
// from one snapshot of the bytes, so S is exact and sorted even while a
// concurrent unmask rewrites the payloads (only false survivors depend on
// payload bytes).  Bit 31 of an entry: verify from HBM.
__device__ __forceinline__ void record_tile(const sieve_lds& sh, int par, uint64_t t, uint64_t* tcount,
                                            uint32_t* slot, uint32_t* pool, unsigned long long* pool_n,
                                            uint64_t pool_cap) {
    const uint32_t lane = threadIdx.x;   // wave 0
    const uint32_t* sw = sh.sbits[par] + 4 * lane;
    const uint32_t* pw = sh.pbits[par] + 4 * lane;
    const uint32_t n = __builtin_popcount(sw[0]) + __builtin_popcount(sw[1]) + __builtin_popcount(sw[2]) +
                       __builtin_popcount(sw[3]);
    uint32_t tot;
    uint32_t k = wave_prefix(n, tot);
    if (tot == 0) {
        if (lane == 0) tcount[t] = 0;
        return;
    }
    uint32_t* dst = slot + t * SV_SLOT;
    uint32_t cap = SV_SLOT;
    if (tot > SV_SLOT) {
        uint64_t base = 0;
        if (lane == 0) base = atomicAdd(pool_n, (unsigned long long)tot);
        base = __shfl(base, 0);
        if (lane == 0) dst[0] = (uint32_t)base;
        dst = pool + base;
        cap = base + tot <= pool_cap ? tot : 0;   // pool full: the survivor total exceeds capS, sieve off
    }
    if (lane == 0) tcount[t] = tot;
#pragma unroll 1
    for (int i = 0; i < 4; ++i) {
        uint32_t m = sw[i];
        const uint32_t pmk = pw[i];
        while (m) {
            const uint32_t b = __builtin_ctz(m);
            m &= m - 1;
            if (k < cap) dst[k] = (128u * lane + 32u * i + b) | (((pmk >> b) & 1u) << 31);
            ++k;
        }
    }
}

// COUNT: tcount[t] = survivors of tile t, recorded by record_tile.
__global__ __launch_bounds__(SV_THREADS) __attribute__((amdgpu_waves_per_eu(8, 8))) void k_sieve_count(const uint8_t* __restrict__ rx, uint64_t rx_len,
                                                            const dseg* __restrict__ segs, const dmid* __restrict__ mid,
                                                            const uint64_t* __restrict__ npred, uint64_t sieve_min,
                                                            uint64_t* __restrict__ tcount, uint32_t* __restrict__ slot,
                                                            uint32_t* __restrict__ pool, unsigned long long* __restrict__ pool_n,
                                                            uint64_t pool_cap, uint64_t ntiles_max, dsieve* __restrict__ sv,
                                                            uint32_t rt, uint32_t wt) {
    __shared__ sieve_lds sh;
    uint64_t sb, L, pos;
    const bool want = sieve_wanted(segs, mid, npred, sieve_min, sb, L, pos);
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        dsieve z = {};
        z.active = want;
        *sv = z;
    }
    if (!want) return;
    if (threadIdx.x < 8) sh.l[(SV_TILE + SV_HALO) / 4 + threadIdx.x] = 0;   // read past the last halo chunk
    const uint64_t A0 = (sb + pos) & ~15ull;
    const uint64_t ntiles = sv_ntiles((sb + L - A0 + SV_TILE - 1) / SV_TILE, rt, wt);
    for (uint64_t t = ntiles + blockIdx.x; t < ntiles_max; t += gridDim.x)
        if (threadIdx.x == 0) tcount[t] = 0;
    tile_regs r;
    uint64_t t = blockIdx.x;
    if (t < ntiles) load_tile(rx, rx_len, A0 + sv_tile(t, rt, wt) * SV_TILE, r);
    int par = 0;
    for (; t < ntiles; t += gridDim.x, par ^= 1) {
        const uint64_t tn = t + gridDim.x;
        const uint64_t T0 = A0 + sv_tile(t, rt, wt) * SV_TILE, Tn = A0 + sv_tile(tn, rt, wt) * SV_TILE;
        sieve_tile(rx, rx_len, sh, r, par, T0, tn < ntiles, Tn, sb, L, pos);
        // wave 0 records while the other waves stage the next tile (the
        // bitmaps alternate by parity; the next barrier orders the rest)
        if (threadIdx.x < 64) record_tile(sh, par, t, tcount, slot, pool, pool_n, pool_cap);
    }
}

// S[tbase[t] + k] = segment offset of tile t's k-th survivor, one thread per
// tile, from its slot or its pool run.
__global__ __launch_bounds__(256) void k_sieve_fill(const dseg* __restrict__ segs, const dmid* __restrict__ mid,
                                                    const uint64_t* __restrict__ tcount,
                                                    const uint64_t* __restrict__ tbase, const uint32_t* __restrict__ slot,
                                                    const uint32_t* __restrict__ pool, uint64_t* __restrict__ S,
                                                    const uint64_t* __restrict__ m_total, uint64_t capS,
                                                    const dsieve* __restrict__ sv, uint32_t rt, uint32_t wt) {
    if (!sv->active || *m_total > capS) return;
    const uint64_t sb = segs[0].off, L = segs[0].len, pos = mid[0].pos;
    const uint64_t A0 = (sb + pos) & ~15ull;
    const uint64_t ntiles = sv_ntiles((sb + L - A0 + SV_TILE - 1) / SV_TILE, rt, wt);
    for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < ntiles; t += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t n = tcount[t], b = tbase[t];
        if (n == 0) continue;
        const uint64_t T0 = A0 + sv_tile(t, rt, wt) * SV_TILE - sb;
        const uint32_t* src = n <= SV_SLOT ? slot + t * SV_SLOT : pool + slot[t * SV_SLOT];
        for (uint64_t k = 0; k < n; ++k) {
            const uint32_t e = src[k];
            S[b + k] = (T0 + (e & 0x7FFFFFFFu)) | ((uint64_t)(e >> 31) << 63);
        }
    }
}

// Finish the survivor test of entries whose chain left their tile (from
// HBM, one thread per entry, every entry's loads in flight at once);
// keep[j] = 1 for survivors, 0 otherwise and for j in [m_pre, capS).
__global__ __launch_bounds__(256) void k_sieve_verify(const uint8_t* __restrict__ rx, uint64_t rx_len,
                                                      const dseg* __restrict__ segs, uint64_t* __restrict__ Spre,
                                                      const uint64_t* __restrict__ m_pre, uint64_t capS,
                                                      uint64_t* __restrict__ keep, const dsieve* __restrict__ sv) {
    if (!sv->active || *m_pre > capS) return;
    const uint64_t m = *m_pre, sb = segs[0].off, L = segs[0].len;
    for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < capS; j += (uint64_t)gridDim.x * blockDim.x) {
        if (j >= m) {
            keep[j] = 0;
            continue;
        }
        const uint64_t e = Spre[j];
        if (!(e >> 63)) {
            keep[j] = 1;
            continue;
        }
        const uint64_t q = e & ~(1ull << 63);
        keep[j] = survivor(rx, rx_len, sb, L, q);
        Spre[j] = q;
    }
}

__global__ __launch_bounds__(256) void k_sieve_compact(const uint64_t* __restrict__ Spre,
                                                       const uint64_t* __restrict__ m_pre, uint64_t capS,
                                                       const uint64_t* __restrict__ keep,
                                                       const uint64_t* __restrict__ kbase, uint64_t* __restrict__ S,
                                                       uint64_t capC, const dsieve* __restrict__ sv) {
    if (!sv->active || *m_pre > capS) return;
    const uint64_t m = *m_pre;
    for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < m; j += (uint64_t)gridDim.x * blockDim.x)
        if (keep[j] && kbase[j] < capC) S[kbase[j]] = Spre[j];
}

__device__ __forceinline__ bool sieve_on(const dsieve* sv, const uint64_t* m_total, uint64_t capS) {
    return sv->active && *m_total <= capS;
}

// Index of the survivor at segment offset x, or SV_TERM: x must lie in a
// sieved tile; that tile's survivors are S[kb(tbase[ct]) .. kb(tbase[ct+1]))
// (kb maps a pre-verification index to the first survivor at or after it).
__device__ __forceinline__ uint32_t sv_lookup(const uint64_t* __restrict__ S, uint64_t m,
                                              const uint64_t* __restrict__ tbase, const uint64_t* __restrict__ kbase,
                                              uint64_t capS, uint64_t A0, uint64_t sb, uint64_t ntiles, uint32_t rt,
                                              uint32_t wt, uint64_t x) {
    const uint64_t rel = sb + x - A0, rb = (uint64_t)rt * SV_TILE;
    const uint64_t r = rel / rb, off = rel - r * rb;
    if (off >= (uint64_t)wt * SV_TILE) return SV_TERM;
    const uint64_t ct = r * wt + off / SV_TILE;
    if (ct >= ntiles) return SV_TERM;
    const uint64_t b0 = tbase[ct], b1 = tbase[ct + 1];
    if (b0 >= b1) return SV_TERM;
    uint64_t lo = b0 < capS ? kbase[b0] : m, hi = b1 < capS ? kbase[b1] : m;
    if (hi > m) hi = m;
    while (lo < hi) {
        const uint64_t md = (lo + hi) >> 1;
        if (S[md] < x) lo = md + 1;
        else hi = md;
    }
    return lo < m && S[lo] == x ? (uint32_t)lo : SV_TERM;
}

// J[j] = index of the next survivor the exact walk from S[j] reaches (every
// frame on the way whole and plausible, at most SV_HOP_CAP of them), or
// SV_TERM; hops[j] = whole frames from S[j] up to that survivor (or up to
// where the walk stopped); mark[j] = 1 for the stream's first whole frame,
// mark[j] = 0 for j in [m, capC).  With P > 0 the first P frame offsets of
// each walk go to scr[j * P ...], so the records need no second walk.
__global__ __launch_bounds__(256) void k_sieve_link(const uint8_t* __restrict__ rx, uint64_t rx_len,
                                                    const dseg* __restrict__ segs, const dmid* __restrict__ mid,
                                                    const uint64_t* __restrict__ S, const uint64_t* __restrict__ m_total,
                                                    uint64_t capC, uint32_t* __restrict__ J, uint32_t* __restrict__ hops,
                                                    uint64_t* __restrict__ mark, const dsieve* __restrict__ sv,
                                                    const uint64_t* __restrict__ tbase, const uint64_t* __restrict__ kbase,
                                                    const uint64_t* __restrict__ m_pre, uint64_t capS, uint32_t rt,
                                                    uint32_t wt, uint64_t* __restrict__ scr, uint32_t P) {
    if (!sieve_on(sv, m_total, capC) || *m_pre > capS) return;
    const uint64_t m = *m_total, sb = segs[0].off, L = segs[0].len, pos = mid[0].pos;
    const uint64_t A0 = (sb + pos) & ~15ull;
    const uint64_t ntiles = sv_ntiles((sb + L - A0 + SV_TILE - 1) / SV_TILE, rt, wt);
    for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < capC; j += (uint64_t)gridDim.x * blockDim.x) {
        if (j >= m) {
            mark[j] = 0;
            continue;
        }
        const uint64_t q = S[j];
        hdr h;
        uint32_t nx = SV_TERM, k = 0;
        if (parse_at(rx, rx_len, sb, L, q, h)) {
            uint64_t x = q;
            // the window the walk is in or heads for: [wlo, whi) absolute
            const uint64_t rb = (uint64_t)rt * SV_TILE, wb = (uint64_t)wt * SV_TILE;
            uint64_t wlo = A0 + (sb + q - A0) / rb * rb, whi = wlo + wb;
            uint64_t* sp = P ? scr + j * P : nullptr;
#pragma unroll 1
            for (;;) {
                if (k < P) sp[k] = x;   // frame k of this node (k_sieve_emit_pos reads them back)
                x += h.hlen + h.length;
                ++k;
                if (!parse_at(rx, rx_len, sb, L, x, h)) break;   // the segment ends (or cuts the frame) at x
                const uint64_t ax = sb + x;
                if (ax >= wlo + rb) {   // a later region (division only when the walk crosses one)
                    wlo = A0 + (ax - A0) / rb * rb;
                    whi = wlo + wb;
                }
                nx = ax < whi ? sv_lookup(S, m, tbase, kbase, capS, A0, sb, ntiles, rt, wt, x) : SV_TERM;
                if (nx != SV_TERM || !plausible(h) || k >= SV_HOP_CAP) break;
            }
        }
        J[j] = nx;
        hops[j] = k;
        mark[j] = q == pos && (j == 0 || S[j - 1] != pos) ? 1u : 0u;
    }
}

// All doubling rounds in one workgroup when the chain arrays fit in LDS
// (windowed scans: up to ~10 000 survivors) -- one launch instead of
// ceil(log2 capC), each of which costs a dispatch beside the unmask.
constexpr uint32_t SV_JLDS = 16384;   // 2 x 64 KiB of successors + 16 KiB of marks

__global__ __launch_bounds__(256) void k_sieve_jump_lds(const uint32_t* __restrict__ J, uint64_t* __restrict__ mark,
                                                         const uint64_t* __restrict__ m_total, uint64_t capC,
                                                         const dsieve* __restrict__ sv) {
    __shared__ uint32_t jj[2][SV_JLDS];
    __shared__ uint8_t mk[SV_JLDS];
    if (!sieve_on(sv, m_total, capC)) return;
    const uint32_t m = (uint32_t)*m_total;   // <= capC <= SV_JLDS (host)
    for (uint32_t j = threadIdx.x; j < m; j += blockDim.x) {
        jj[0][j] = J[j];
        mk[j] = mark[j] ? 1 : 0;
    }
    __syncthreads();
    uint32_t c = 0;
    for (uint32_t r = 0; (1u << r) < m; ++r, c ^= 1) {
        for (uint32_t j = threadIdx.x; j < m; j += blockDim.x) {
            const uint32_t n = jj[c][j];
            if (n == SV_TERM) {
                jj[c ^ 1][j] = SV_TERM;
                continue;
            }
            if (mk[j]) mk[n] = 1;   // only ever set: racing writers agree
            jj[c ^ 1][j] = jj[c][n];
        }
        __syncthreads();
    }
    for (uint32_t j = threadIdx.x; j < m; j += blockDim.x) mark[j] = mk[j];
}

// Record ranks are weighted by the frames each marked node stands for.
__global__ __launch_bounds__(256) void k_sieve_weight(const uint64_t* __restrict__ mark, const uint32_t* __restrict__ hops,
                                                      uint64_t* __restrict__ w, const uint64_t* __restrict__ m_total,
                                                      uint64_t capC, const dsieve* __restrict__ sv) {
    if (!sieve_on(sv, m_total, capC)) return;
    const uint64_t m = *m_total;
    for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < capC; j += (uint64_t)gridDim.x * blockDim.x)
        w[j] = j < m && mark[j] ? hops[j] : 0;
}

// Pointer doubling, round r (jump 2^r): a marked node marks the node 2^r
// frames ahead.  After round r the chain's first 2^(r+1) frames are marked.
__global__ __launch_bounds__(256) void k_sieve_jump(const uint32_t* __restrict__ Jin, uint32_t* __restrict__ Jout,
                                                    uint64_t* __restrict__ mark, const uint64_t* __restrict__ m_total,
                                                    uint64_t capS, const dsieve* __restrict__ sv, uint32_t r) {
    if (!sieve_on(sv, m_total, capS)) return;
    const uint64_t m = *m_total;
    if (r < 64 && (1ull << r) >= m) return;   // the chain holds at most m frames: all marked
    for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < m; j += (uint64_t)gridDim.x * blockDim.x) {
        const uint32_t jj = Jin[j];
        if (jj == SV_TERM) {
            Jout[j] = SV_TERM;
            continue;
        }
        if (mark[j]) mark[jj] = 1;
        Jout[j] = Jin[jj];
    }
}

// Records of the marked chain: node j's hops[j] frames are records
// n_a + rank[j] ...  The node that ends the chain hands k_walk the resume
// position and its last frame; the last masked frame's offset is the max
// over nodes (Q14: its key stays in the parser).
__global__ __launch_bounds__(256) void k_sieve_emit(const uint8_t* __restrict__ rx, uint64_t rx_len,
                                                    const dseg* __restrict__ segs, const dmid* __restrict__ mid,
                                                    const uint64_t* __restrict__ S, const uint64_t* __restrict__ m_total,
                                                    uint64_t capS, const uint64_t* __restrict__ mark,
                                                    const uint32_t* __restrict__ hops, const uint64_t* __restrict__ rank,
                                                    const uint64_t* __restrict__ npath_p, dframes fr, uint32_t vmask,
                                                    dsieve* __restrict__ sv) {
    if (!sieve_on(sv, m_total, capS)) return;
    const uint64_t m = *m_total, npath = *npath_p, sb = segs[0].off, L = segs[0].len, n_a = mid[0].n_a;
    for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < m; j += (uint64_t)gridDim.x * blockDim.x) {
        if (!mark[j]) continue;
        const uint64_t k0 = rank[j];
        const uint32_t n = hops[j];
        uint64_t x = S[j], prev = x, lm = 0;
#pragma unroll 1
        for (uint32_t i = 0; i < n; ++i) {
            hdr h;
            parse_at(rx, rx_len, sb, L, x, h);
            frec v;
            whole_frame_rec(v, x, h, vmask);
            store_frame(fr, n_a + k0 + i, sb, v);
            if (h.flags & F_MASK) lm = x + 1;
            prev = x;
            x += h.hlen + h.length;
        }
        if (lm) atomicMax((unsigned long long*)&sv->last_masked, (unsigned long long)lm);
        if (n && k0 + n == npath) {
            sv->pend = x;
            sv->last = prev + 1;
            sv->npath = npath;
            sv->use = 1;
        }
    }
}

// The same records from the walks' stored offsets (P > 0): one wave per
// marked node, its lanes take the node's frames 64 at a time (every header
// load independent); frames past a walk's first P are walked by lane 0 from
// its P-th (rare: the host sizes P at about twice a region's frames).
__device__ __forceinline__ uint64_t wave_max64(uint64_t v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const uint64_t w = __shfl_xor(v, o);
        v = w > v ? w : v;
    }
    return v;
}

__global__ __launch_bounds__(256) void k_sieve_emit_pos(const uint8_t* __restrict__ rx, uint64_t rx_len,
                                                        const dseg* __restrict__ segs, const dmid* __restrict__ mid,
                                                        const uint64_t* __restrict__ m_total, uint64_t capC,
                                                        const uint64_t* __restrict__ mark,
                                                        const uint32_t* __restrict__ hops,
                                                        const uint64_t* __restrict__ rank,
                                                        const uint64_t* __restrict__ npath_p,
                                                        const uint64_t* __restrict__ scr, uint32_t lgP, dframes fr,
                                                        uint32_t vmask, dsieve* __restrict__ sv) {
    if (!sieve_on(sv, m_total, capC)) return;
    const uint64_t m = *m_total, npath = *npath_p, sb = segs[0].off, L = segs[0].len, n_a = mid[0].n_a;
    const uint32_t P = 1u << lgP, lane = threadIdx.x & 63u;
    const uint64_t wv = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6, nw = ((uint64_t)gridDim.x * blockDim.x) >> 6;
    for (uint64_t j = wv; j < m; j += nw) {   // wave-uniform
        if (!mark[j]) continue;
        const uint32_t n = hops[j];
        const uint64_t k0 = rank[j];
        const uint32_t ns = n < P ? n : P;
        uint64_t lm = 0;
        for (uint32_t i = lane; i < ns; i += 64) {
            const uint64_t x = scr[(j << lgP) + i];
            hdr h;
            parse_at(rx, rx_len, sb, L, x, h);
            frec v;
            whole_frame_rec(v, x, h, vmask);
            store_frame(fr, n_a + k0 + i, sb, v);
            if (h.flags & F_MASK) lm = x + 1;
            if (i + 1 == n && k0 + n == npath) {   // the chain's last frame
                sv->pend = x + h.hlen + h.length;
                sv->last = x + 1;
                sv->npath = npath;
                sv->use = 1;
            }
        }
        if (n > P && lane == 0) {   // the rest of a long walk
            uint64_t x = scr[(j << lgP) + P - 1];
            hdr h;
            parse_at(rx, rx_len, sb, L, x, h);
#pragma unroll 1
            for (uint32_t t = P; t < n; ++t) {
                x += h.hlen + h.length;
                parse_at(rx, rx_len, sb, L, x, h);
                frec v;
                whole_frame_rec(v, x, h, vmask);
                store_frame(fr, n_a + k0 + t, sb, v);
                if (h.flags & F_MASK) lm = x + 1;
            }
            if (k0 + n == npath) {
                sv->pend = x + h.hlen + h.length;
                sv->last = x + 1;
                sv->npath = npath;
                sv->use = 1;
            }
        }
        lm = wave_max64(lm);
        if (lane == 0 && lm) atomicMax((unsigned long long*)&sv->last_masked, (unsigned long long)lm);
    }
}

// ---------------------------------------------------------------- launcher

uint64_t sieve_tiles_max(uint64_t rx_len) { return rx_len / SV_TILE + 2; }
uint64_t sieve_slot_words(uint64_t rx_len) { return sieve_tiles_max(rx_len) * SV_SLOT; }

static uint64_t g_sieve_min = 0;   // 0: not yet read from the environment
constexpr uint64_t SIEVE_MIN_DEFAULT = 8ull << 20;

uint64_t sieve_min() {
    if (!g_sieve_min) {
        const char* e = experiment("sieve_min");
        const long long x = e ? atoll(e) : 0;
        g_sieve_min = x > 0 ? (uint64_t)x : SIEVE_MIN_DEFAULT;
    }
    return g_sieve_min;
}

static uint64_t g_sieve_gen = 1;

uint64_t set_sieve_min(uint64_t v) {
    const uint64_t old = sieve_min();
    g_sieve_min = v ? v : SIEVE_MIN_DEFAULT;
    ++g_sieve_gen;
    return old;
}

uint64_t sieve_generation() { return g_sieve_gen; }

// Windows: regions of about $HVWS_EXPERIMENT sieve_hops (default 320) mean-sized frames,
// each sieved over its first $HVWS_EXPERIMENT sieve_window bytes (default 1 MiB + 16 KiB:
// past the largest frame of config 4, so a walk entering a region almost
// always lands on a survivor of its window).  Regions shorter than two
// windows, or no count yet: every tile.  Results never depend on it.
// 320: with the count grid of SV_GRID_WINDOWS and the faster link hops (ld16),
// c4 as one stream 1.488-1.496 ms per step against 1.51 at 256 (r5zs, r5zt).
constexpr uint64_t SIEVE_HOPS_DEFAULT = 320, SIEVE_WINDOW_DEFAULT = (1 << 20) + (16 << 10);
static uint64_t g_sv_hops = ~0ull, g_sv_win = 0;   // ~0 / 0: not yet read from the environment

static void sieve_windows_init() {
    if (g_sv_hops == ~0ull) {
        const char* e = experiment("sieve_hops");
        g_sv_hops = e ? (uint64_t)atoll(e) : SIEVE_HOPS_DEFAULT;
    }
    if (!g_sv_win) {
        const char* e = experiment("sieve_window");
        const long long x = e ? atoll(e) : 0;
        g_sv_win = x > 0 ? (uint64_t)x : SIEVE_WINDOW_DEFAULT;
    }
}

void set_sieve_windows(uint64_t hops, uint64_t window, uint64_t prev[2]) {
    sieve_windows_init();
    if (prev) {
        prev[0] = g_sv_hops;
        prev[1] = g_sv_win;
    }
    g_sv_hops = hops;
    g_sv_win = window ? window : SIEVE_WINDOW_DEFAULT;
    ++g_sieve_gen;
}

uint64_t sieve_hops() {
    sieve_windows_init();
    return g_sv_hops;
}

void sieve_geometry(uint64_t rx_len, uint64_t nframes, uint32_t& rt, uint32_t& wt) {
    sieve_windows_init();
    rt = wt = 1;
    if (!nframes || !g_sv_hops || g_sv_hops > (1ull << 20)) return;
    const uint64_t rb = rx_len / nframes * g_sv_hops;
    const uint64_t wtiles = (g_sv_win + SV_TILE - 1) / SV_TILE, rtiles = rb / SV_TILE;
    if (rtiles < 2 * wtiles || rtiles > 0xFFFFFFFFull) return;
    rt = (uint32_t)rtiles;
    wt = (uint32_t)wtiles;
}

// Survivor-array capacity rounds: log2 of the capacity bounds the chain.
static uint32_t jump_rounds(uint64_t capS) {
    uint32_t r = 0;
    while (r < 40 && (1ull << r) < capS) ++r;
    return r;
}

hipError_t launch_sieve(const uint8_t* rx, uint64_t rx_len, const dseg* segs, const dmid* mid, const uint64_t* npred,
                        const sieve_bufs& b, hipStream_t st) {
    const uint64_t ntm = sieve_tiles_max(rx_len);
    static const uint32_t grid_env = experiment("sieve_grid") ? (uint32_t)atoi(experiment("sieve_grid")) : 0u;
    const uint32_t grid_cap = grid_env ? grid_env : (b.rt != b.wt ? SV_GRID_WINDOWS : SV_GRID);
    const uint32_t grid = (uint32_t)(ntm < grid_cap ? ntm : grid_cap);
    dsieve* sv = reinterpret_cast<dsieve*>(b.state);
    hipError_t e = hipMemsetAsync(b.pool_n, 0, 8, st);
    if (e != hipSuccess) return e;
    // (round 4's timing modes -- lists without checks, staging alone, loads
    // alone, no next-tile prefetch -- were removed in round 6; profiles/r4*_raw)
    hipLaunchKernelGGL(k_sieve_count, dim3(grid), dim3(SV_THREADS), 0, st, rx, rx_len, segs, mid, npred, sieve_min(),
                       b.tcount, b.slot, b.pool, reinterpret_cast<unsigned long long*>(b.pool_n), b.capS, ntm, sv, b.rt,
                       b.wt);
    if ((e = launch_exclusive_scan(b.tcount, b.tbase, ntm, b.tmp, b.m_pre, st)) != hipSuccess) return e;
    const uint64_t fb = (ntm + 255) / 256;
    hipLaunchKernelGGL(k_sieve_fill, dim3((uint32_t)(fb < 8192 ? fb : 8192)), dim3(256), 0, st, segs, mid, b.tcount,
                       b.tbase, b.slot, b.pool, b.Spre, b.m_pre, b.capS, sv, b.rt, b.wt);
    // Pre-verification entries use capacity capS; the survivors and the chain
    // arrays capC (about the survivor count: the doubling rounds and the mark
    // scan run over it).  More survivors than capC: the sieve stands down.
    const uint32_t lg = (uint32_t)((b.capS + 255) / 256 < 8192 ? (b.capS + 255) / 256 : 8192);
    const uint32_t lc = (uint32_t)((b.capC + 255) / 256 < 8192 ? (b.capC + 255) / 256 : 8192);
    hipLaunchKernelGGL(k_sieve_verify, dim3(lg), dim3(256), 0, st, rx, rx_len, segs, b.Spre, b.m_pre, b.capS, b.keep, sv);
    if ((e = launch_exclusive_scan(b.keep, b.kbase, b.capS, b.tmp, b.m_total, st)) != hipSuccess) return e;
    hipLaunchKernelGGL(k_sieve_compact, dim3(lg), dim3(256), 0, st, b.Spre, b.m_pre, b.capS, b.keep, b.kbase, b.S, b.capC,
                       sv);
    hipLaunchKernelGGL(k_sieve_link, dim3(lc), dim3(256), 0, st, rx, rx_len, segs, mid, b.S, b.m_total, b.capC, b.J0,
                       b.hops, b.mark, sv, b.tbase, b.kbase, b.m_pre, b.capS, b.rt, b.wt, b.scr,
                       b.scr ? 1u << b.lgP : 0u);
    if (b.capC <= SV_JLDS) {
        // 256 threads: a 16-wave workgroup waits for a CU with 16 free slots
        // beside the unmask grid
        hipLaunchKernelGGL(k_sieve_jump_lds, dim3(1), dim3(256), 0, st, b.J0, b.mark, b.m_total, b.capC, sv);
    } else {
        uint32_t* Jin = b.J0;
        uint32_t* Jout = b.J1;
        const uint32_t rounds = jump_rounds(b.capC);
        for (uint32_t r = 0; r < rounds; ++r) {
            hipLaunchKernelGGL(k_sieve_jump, dim3(lc < 1024 ? lc : 1024), dim3(256), 0, st, Jin, Jout, b.mark,
                               b.m_total, b.capC, sv, r);
            uint32_t* t = Jin;
            Jin = Jout;
            Jout = t;
        }
    }
    // weights into keep (free once the link has read kbase)
    hipLaunchKernelGGL(k_sieve_weight, dim3(lc), dim3(256), 0, st, b.mark, b.hops, b.keep, b.m_total, b.capC, sv);
    e = launch_exclusive_scan(b.keep, b.rank, b.capC, b.tmp, b.npath, st);
    if (e != hipSuccess) return e;
    return hipGetLastError();
}

hipError_t launch_sieve_emit(const uint8_t* rx, uint64_t rx_len, const dseg* segs, const dmid* mid,
                             const sieve_bufs& b, dframes fr, uint32_t vmask, hipStream_t st) {
    if (b.scr) {
        const uint64_t g = (b.capC + 3) / 4;   // a wave per node
        hipLaunchKernelGGL(k_sieve_emit_pos, dim3((uint32_t)(g < 8192 ? g : 8192)), dim3(256), 0, st, rx, rx_len,
                           segs, mid, b.m_total, b.capC, b.mark, b.hops, b.rank, b.npath, b.scr, b.lgP, fr, vmask,
                           reinterpret_cast<dsieve*>(b.state));
        return hipGetLastError();
    }
    const uint32_t lc = (uint32_t)((b.capC + 255) / 256 < 8192 ? (b.capC + 255) / 256 : 8192);
    hipLaunchKernelGGL(k_sieve_emit, dim3(lc), dim3(256), 0, st, rx, rx_len, segs, mid, b.S, b.m_total, b.capC,
                       b.mark, b.hops, b.rank, b.npath, fr, vmask, reinterpret_cast<dsieve*>(b.state));
    return hipGetLastError();
}

}  // namespace hvws

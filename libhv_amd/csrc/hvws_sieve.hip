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
//   scan             tile counts -> tile bases (sorted survivor array S).
//   k_sieve_fill     S from the slots (and the pool runs of busy tiles).
//   k_sieve_link     succ(j) = index of S[j] + size(S[j]) in S (binary
//                    search), or none.
//   k_sieve_jump     pointer doubling from the stream's first whole frame
//                    (known exactly from k_head): after round r the first
//                    2^(r+1) frames of the true chain are marked.
//   scan             marks -> record ranks.
//   k_sieve_emit     frame records of the marked chain.
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
constexpr uint32_t SV_HALO = 256;                      // bytes staged past the tile (headers, short hops)
constexpr uint32_t SV_SLOT = 16;                       // survivors kept per tile by the count pass
constexpr int SV_DEPTH = 3;                            // hops a survivor's chain must stay plausible
constexpr uint32_t SV_TERM = 0xFFFFFFFFu;
constexpr uint32_t SV_GRID = 4096;

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

// 16 bytes at byte offset p of the LDS tile.
__device__ __forceinline__ void lds_ld16(const uint32_t* l, uint32_t p, uint64_t& lo, uint64_t& hi) {
    const uint32_t w = p >> 2, sh = p & 3u;
    const uint32_t a0 = l[w], a1 = l[w + 1], a2 = l[w + 2], a3 = l[w + 3], a4 = l[w + 4];
    const uint32_t b0 = __builtin_amdgcn_alignbyte(a1, a0, sh), b1 = __builtin_amdgcn_alignbyte(a2, a1, sh);
    const uint32_t b2 = __builtin_amdgcn_alignbyte(a3, a2, sh), b3 = __builtin_amdgcn_alignbyte(a4, a3, sh);
    lo = (uint64_t)b0 | ((uint64_t)b1 << 32);
    hi = (uint64_t)b2 | ((uint64_t)b3 << 32);
}

// Header at segment offset x: from the LDS tile when it is staged there
// (tile base T0 absolute), else from HBM.
__device__ __forceinline__ hdr hdr_at(const uint8_t* rx, uint64_t rx_len, const uint32_t* l, uint64_t T0,
                                      uint64_t a) {
    uint64_t lo, hi;
    if (a >= T0 && a - T0 + 16 <= SV_TILE + SV_HALO) lds_ld16(l, (uint32_t)(a - T0), lo, hi);
    else ld16(rx, rx_len, a, lo, hi);
    return parse_hdr(lo, hi);
}

// Candidate at absolute a (segment [sb, sb + L)): a whole frame with a
// plausible header whose next SV_DEPTH headers are plausible, or end the
// stream (exactly, or with a header or frame cut by the segment end).
__device__ bool survivor(const uint8_t* rx, uint64_t rx_len, const uint32_t* l, uint64_t T0, uint64_t sb,
                         uint64_t L, uint64_t a) {
    const uint64_t end = sb + L;
    hdr h = hdr_at(rx, rx_len, l, T0, a);
    const uint64_t r0 = end - a;
    if (!plausible(h) || h.hlen > r0 || h.length > r0 - h.hlen) return false;
    uint64_t x = a + h.hlen + h.length;
#pragma unroll 1
    for (int d = 0; d < SV_DEPTH; ++d) {
        const uint64_t r = end - x;
        if (r < 14) return true;   // end of stream, or a header that may be cut by it
        h = hdr_at(rx, rx_len, l, T0, x);
        if (!plausible(h)) return false;
        if (h.length > r - h.hlen) return true;   // frame cut by the segment end
        x += h.hlen + h.length;
    }
    return true;
}

// Candidate mask of the thread's 32 positions (bit i = position 32*t + i):
// byte b0 with (b0 & 0x74) == 0 and (b0 & 3) != 3 (RSV clear, opcode 0-2 or
// 8-A) followed by a byte with MASK set.  SWAR over 4 positions per dword.
__device__ __forceinline__ uint32_t candidates(const uint32_t* l, uint32_t t) {
    uint32_t w[SV_PER / 4 + 1];
#pragma unroll
    for (int k = 0; k <= (int)(SV_PER / 4); ++k) w[k] = l[t * (SV_PER / 4) + k];
    uint32_t mask = 0;
#pragma unroll
    for (int k = 0; k < (int)(SV_PER / 4); ++k) {
        const uint32_t v = w[k];
        const uint32_t v1 = __builtin_amdgcn_alignbyte(w[k + 1], v, 1);   // next byte of each
        const uint32_t z = v & 0x74747474u;
        const uint32_t bad = (z + 0x7F7F7F7Fu) | z;                      // bit 7: byte of z non-zero
        const uint32_t x = (v & 0x03030303u) ^ 0x03030303u;
        const uint32_t ok = (x + 0x7F7F7F7Fu) | x;                       // bit 7: (b0 & 3) != 3
        const uint32_t c = ~bad & ok & v1 & 0x80808080u;
        const uint32_t c4 = ((c >> 7) & 1u) | ((c >> 14) & 2u) | ((c >> 21) & 4u) | ((c >> 28) & 8u);
        mask |= c4 << (4 * k);
    }
    return mask;
}

// Tile staging in two halves so the next tile's loads can be in flight while
// the current tile is sieved: each thread loads 16-B chunks c = t, t + 256
// (and t + 512 for the halo) of [T0, T0 + SV_TILE + SV_HALO) into registers,
// then stores them to LDS.  Bytes past rx_len read 0.
typedef uint32_t sv_u32x4 __attribute__((ext_vector_type(4)));
constexpr uint32_t SV_CHUNKS = (SV_TILE + SV_HALO) / 16;   // 528
struct tile_regs {
    sv_u32x4 v[3];
};

__device__ __forceinline__ sv_u32x4 load_chunk(const uint8_t* rx, uint64_t rx_len, uint64_t a) {
    if (a + 16 <= rx_len) return *reinterpret_cast<const sv_u32x4*>(rx + a);
    uint32_t b[4] = {0u, 0u, 0u, 0u};
    for (uint32_t k = 0; a + k < rx_len && k < 16; ++k) b[k >> 2] |= (uint32_t)rx[a + k] << (8 * (k & 3));
    return sv_u32x4{b[0], b[1], b[2], b[3]};
}

__device__ __forceinline__ void load_tile(const uint8_t* rx, uint64_t rx_len, uint64_t T0, tile_regs& r) {
    const uint32_t t = threadIdx.x;
    r.v[0] = load_chunk(rx, rx_len, T0 + (uint64_t)t * 16);
    r.v[1] = load_chunk(rx, rx_len, T0 + (uint64_t)(t + SV_THREADS) * 16);
    r.v[2] = t + 2 * SV_THREADS < SV_CHUNKS ? load_chunk(rx, rx_len, T0 + (uint64_t)(t + 2 * SV_THREADS) * 16)
                                            : sv_u32x4{0u, 0u, 0u, 0u};
}

__device__ __forceinline__ void store_tile(uint32_t* l, const tile_regs& r) {
    const uint32_t t = threadIdx.x;
    *reinterpret_cast<sv_u32x4*>(l + 4 * t) = r.v[0];
    *reinterpret_cast<sv_u32x4*>(l + 4 * (t + SV_THREADS)) = r.v[1];
    if (t + 2 * SV_THREADS < SV_CHUNKS) *reinterpret_cast<sv_u32x4*>(l + 4 * (t + 2 * SV_THREADS)) = r.v[2];
}

// Candidate bitmap of the staged tile + halo into cb (bit p = byte p of the
// tile); bits of positions whose second byte is not staged are never read.
__device__ __forceinline__ void candidate_bits(const uint32_t* l, uint32_t* cb) {
    const uint32_t t = threadIdx.x;
    cb[t] = candidates(l, t);
    if (t < SV_HALO / SV_PER) cb[SV_TILE / SV_PER + t] = candidates(l, SV_TILE / SV_PER + t);
}

__device__ __forceinline__ uint32_t lds_byte(const uint32_t* l, uint32_t p) { return (l[p >> 2] >> (8 * (p & 3u))) & 0xFFu; }

// Survivor mask of the thread's positions in tile T0 (segment [sb+pos, sb+L)).
// A short candidate (7-bit length) whose next header position is staged and
// is not itself a candidate is rejected by one bitmap test -- the full check
// would reject it too (a plausible header is a candidate) -- so only ~1 in
// 57 candidates pays the full parse and hops.
__device__ __forceinline__ uint32_t survivors(const uint8_t* rx, uint64_t rx_len, const uint32_t* l,
                                              const uint32_t* cb, uint64_t T0, uint64_t sb, uint64_t L, uint64_t pos) {
    const uint32_t t = threadIdx.x;
    uint32_t cm = cb[t];
    const uint64_t a0 = T0 + (uint64_t)t * SV_PER;
    const uint64_t lo = sb + pos, hi = sb + L;
    if (a0 < lo) cm &= lo - a0 >= SV_PER ? 0u : ~0u << (uint32_t)(lo - a0);
    if (a0 + SV_PER > hi) cm &= a0 >= hi ? 0u : (1u << (uint32_t)(hi - a0)) - 1u;
    // Phase 1: the bitmap filter (LDS only).  Phase 2: full checks of what
    // is left -- about one per thread at most -- so a wave waits for one
    // chain of dependent header loads, not one per candidate.
    uint32_t pm = 0;
    while (cm) {
        const uint32_t i = __builtin_ctz(cm);
        cm &= cm - 1;
        const uint32_t p = t * SV_PER + i;
        const uint32_t len7 = lds_byte(l, p + 1) & 0x7Fu;
        if (len7 < 126) {
            const uint32_t x = p + 6u + len7;   // next header (the candidate is masked)
            if (x + 16 <= SV_TILE + SV_HALO && T0 + x + 14 <= hi && !((cb[x >> 5] >> (x & 31u)) & 1u)) continue;
        }
        pm |= 1u << i;
    }
    uint32_t sm = 0;
    while (pm) {
        const uint32_t i = __builtin_ctz(pm);
        pm &= pm - 1;
        if (survivor(rx, rx_len, l, T0, sb, L, a0 + i)) sm |= 1u << i;
    }
    return sm;
}

// Block-wide exclusive prefix of v (thread order); *tot = block sum.
__device__ __forceinline__ uint32_t block_prefix(uint32_t v, uint32_t* ws, uint32_t& tot) {
    const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
    uint32_t x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o);
        if (lane >= (uint32_t)o) x += y;
    }
    if (lane == 63) ws[w] = x;
    __syncthreads();
    uint32_t base = 0;
    tot = 0;
#pragma unroll
    for (uint32_t k = 0; k < SV_THREADS / 64; ++k) {
        if (k < w) base += ws[k];
        tot += ws[k];
    }
    __syncthreads();
    return base + x - v;
}

struct sieve_lds {
    uint32_t l[(SV_TILE + SV_HALO) / 4 + 8];
    uint32_t cb[(SV_TILE + SV_HALO) / SV_PER];
    uint32_t ws[SV_THREADS / 64];
    uint32_t nover;
    uint32_t over[SV_THREADS];
};

// Sieve one tile whose bytes are in r (stored to LDS here); `next` (if any)
// is loaded into r meanwhile.  Returns this thread's survivor mask and its
// exclusive prefix / the tile total.
__device__ __forceinline__ uint32_t sieve_tile(const uint8_t* rx, uint64_t rx_len, sieve_lds& sh, tile_regs& r,
                                               uint64_t T0, bool have_next, uint64_t next_T0, uint64_t sb,
                                               uint64_t L, uint64_t pos, uint32_t& before, uint32_t& tot) {
    store_tile(sh.l, r);
    __syncthreads();
    if (have_next) load_tile(rx, rx_len, next_T0, r);
    candidate_bits(sh.l, sh.cb);
    __syncthreads();
    const uint32_t sm = survivors(rx, rx_len, sh.l, sh.cb, T0, sb, L, pos);
    before = block_prefix(__builtin_popcount(sm), sh.ws, tot);
    return sm;
}

// COUNT: tcount[t] = survivors of tile t, the first SV_SLOT of them (tile
// offsets) into slot[t].
__global__ __launch_bounds__(SV_THREADS) void k_sieve_count(const uint8_t* __restrict__ rx, uint64_t rx_len,
                                                            const dseg* __restrict__ segs, const dmid* __restrict__ mid,
                                                            const uint64_t* __restrict__ npred, uint64_t sieve_min,
                                                            uint64_t* __restrict__ tcount, uint32_t* __restrict__ slot,
                                                            uint32_t* __restrict__ pool, unsigned long long* __restrict__ pool_n,
                                                            uint64_t pool_cap, uint64_t ntiles_max, dsieve* __restrict__ sv) {
    __shared__ sieve_lds sh;
    uint64_t sb, L, pos;
    const bool want = sieve_wanted(segs, mid, npred, sieve_min, sb, L, pos);
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        dsieve z = {};
        z.active = want;
        *sv = z;
    }
    if (!want) return;
    if (threadIdx.x < 8) sh.l[(SV_TILE + SV_HALO) / 4 + threadIdx.x] = 0;
    const uint64_t A0 = (sb + pos) & ~15ull;
    const uint64_t ntiles = (sb + L - A0 + SV_TILE - 1) / SV_TILE;
    for (uint64_t t = ntiles + blockIdx.x; t < ntiles_max; t += gridDim.x)
        if (threadIdx.x == 0) tcount[t] = 0;
    tile_regs r;
    uint64_t t = blockIdx.x;
    if (t < ntiles) load_tile(rx, rx_len, A0 + t * SV_TILE, r);
    for (; t < ntiles; t += gridDim.x) {
        const uint64_t T0 = A0 + t * SV_TILE;
        const uint64_t tn = t + gridDim.x;
        uint32_t before, tot;
        uint32_t m = sieve_tile(rx, rx_len, sh, r, T0, tn < ntiles, A0 + tn * SV_TILE, sb, L, pos, before, tot);
        // Up to SV_SLOT survivors go to the tile's slot; a tile with more
        // reserves a run of the pool and records its start in slot word 0.
        // Every survivor is written from this one snapshot of the bytes, so
        // S is exact and sorted even while a concurrent unmask rewrites the
        // payloads (only false survivors depend on payload bytes).
        uint32_t* dst = slot + t * SV_SLOT;
        uint64_t cap = SV_SLOT;
        if (tot > SV_SLOT) {
            if (threadIdx.x == 0) sh.nover = (uint32_t)atomicAdd(pool_n, (unsigned long long)tot);
            __syncthreads();
            const uint64_t base = sh.nover;
            __syncthreads();
            if (threadIdx.x == 0) dst[0] = (uint32_t)base;
            dst = pool + base;
            cap = base + tot <= pool_cap ? tot : 0;   // pool full: the survivor total exceeds capS, sieve off
        }
        if (threadIdx.x == 0) tcount[t] = tot;
        uint32_t k = before;
        while (m && k < cap) {
            const uint32_t i = __builtin_ctz(m);
            m &= m - 1;
            dst[k++] = threadIdx.x * SV_PER + i;
        }
    }
}

// S[tbase[t] + k] = segment offset of tile t's k-th survivor, one thread per
// tile, from its slot or its pool run.
__global__ __launch_bounds__(256) void k_sieve_fill(const dseg* __restrict__ segs, const dmid* __restrict__ mid,
                                                    const uint64_t* __restrict__ tcount,
                                                    const uint64_t* __restrict__ tbase, const uint32_t* __restrict__ slot,
                                                    const uint32_t* __restrict__ pool, uint64_t* __restrict__ S,
                                                    const uint64_t* __restrict__ m_total, uint64_t capS,
                                                    const dsieve* __restrict__ sv) {
    if (!sv->active || *m_total > capS) return;
    const uint64_t sb = segs[0].off, L = segs[0].len, pos = mid[0].pos;
    const uint64_t A0 = (sb + pos) & ~15ull;
    const uint64_t ntiles = (sb + L - A0 + SV_TILE - 1) / SV_TILE;
    for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < ntiles; t += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t n = tcount[t], b = tbase[t];
        if (n == 0) continue;
        const uint64_t T0 = A0 + t * SV_TILE - sb;
        const uint32_t* src = n <= SV_SLOT ? slot + t * SV_SLOT : pool + slot[t * SV_SLOT];
        for (uint64_t k = 0; k < n; ++k) S[b + k] = T0 + src[k];
    }
}

__device__ __forceinline__ bool sieve_on(const dsieve* sv, const uint64_t* m_total, uint64_t capS) {
    return sv->active && *m_total <= capS;
}

// J[j] = index of the survivor at S[j] + size(S[j]), or SV_TERM; mark[j] = 1
// for the stream's first whole frame; mark[j] = 0 for j in [m, capS).
__global__ __launch_bounds__(256) void k_sieve_link(const uint8_t* __restrict__ rx, uint64_t rx_len,
                                                    const dseg* __restrict__ segs, const dmid* __restrict__ mid,
                                                    const uint64_t* __restrict__ S, const uint64_t* __restrict__ m_total,
                                                    uint64_t capS, uint32_t* __restrict__ J, uint64_t* __restrict__ mark,
                                                    const dsieve* __restrict__ sv) {
    if (!sieve_on(sv, m_total, capS)) return;
    const uint64_t m = *m_total, sb = segs[0].off, L = segs[0].len, pos = mid[0].pos;
    for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < capS; j += (uint64_t)gridDim.x * blockDim.x) {
        if (j >= m) {
            mark[j] = 0;
            continue;
        }
        // Only whole frames are chain nodes: a node's successor is the first
        // entry equal to its exact end, if a whole frame starts there.
        const uint64_t q = S[j];
        hdr h;
        uint32_t nx = SV_TERM;
        if (parse_at(rx, rx_len, sb, L, q, h)) {
            const uint64_t x = q + h.hlen + h.length;
            uint64_t lo = j + 1, hi = m;
            while (lo < hi) {
                const uint64_t md = (lo + hi) >> 1;
                if (S[md] < x) lo = md + 1;
                else hi = md;
            }
            hdr hx;
            if (lo < m && S[lo] == x && parse_at(rx, rx_len, sb, L, x, hx)) nx = (uint32_t)lo;
        }
        J[j] = nx;
        mark[j] = q == pos && (j == 0 || S[j - 1] != pos) ? 1u : 0u;
    }
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

// Records of the marked chain: record n_a + rank[j] for node j.  The last
// node hands k_walk the resume position; the last masked one its key (Q14).
__global__ __launch_bounds__(256) void k_sieve_emit(const uint8_t* __restrict__ rx, uint64_t rx_len,
                                                    const dseg* __restrict__ segs, const dmid* __restrict__ mid,
                                                    const uint64_t* __restrict__ S, const uint64_t* __restrict__ m_total,
                                                    uint64_t capS, const uint64_t* __restrict__ mark,
                                                    const uint64_t* __restrict__ rank,
                                                    const uint64_t* __restrict__ npath_p, dframes fr, uint32_t vmask,
                                                    dsieve* __restrict__ sv) {
    if (!sieve_on(sv, m_total, capS)) return;
    const uint64_t m = *m_total, npath = *npath_p, sb = segs[0].off, L = segs[0].len, n_a = mid[0].n_a;
    for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < m; j += (uint64_t)gridDim.x * blockDim.x) {
        if (!mark[j]) continue;
        const uint64_t q = S[j];
        hdr h;
        parse_at(rx, rx_len, sb, L, q, h);
        frec v;
        whole_frame_rec(v, q, h, vmask);
        const uint64_t k = rank[j];
        store_frame(fr, n_a + k, sb, v);
        if (h.flags & F_MASK) atomicMax((unsigned long long*)&sv->last_masked, (unsigned long long)(j + 1));
        if (k + 1 == npath) {
            sv->pend = q + h.hlen + h.length;
            sv->last = j + 1;
            sv->npath = npath;
            sv->use = 1;
        }
    }
}

// ---------------------------------------------------------------- launcher

uint64_t sieve_tiles_max(uint64_t rx_len) { return rx_len / SV_TILE + 2; }
uint64_t sieve_slot_words(uint64_t rx_len) { return sieve_tiles_max(rx_len) * SV_SLOT; }

static uint64_t g_sieve_min = 0;   // 0: not yet read from the environment
constexpr uint64_t SIEVE_MIN_DEFAULT = 8ull << 20;

uint64_t sieve_min() {
    if (!g_sieve_min) {
        const char* e = getenv("HVWS_SIEVE_MIN");
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

// Survivor-array capacity rounds: log2 of the capacity bounds the chain.
static uint32_t jump_rounds(uint64_t capS) {
    uint32_t r = 0;
    while (r < 40 && (1ull << r) < capS) ++r;
    return r;
}

hipError_t launch_sieve(const uint8_t* rx, uint64_t rx_len, const dseg* segs, const dmid* mid, const uint64_t* npred,
                        const sieve_bufs& b, hipStream_t st) {
    const uint64_t ntm = sieve_tiles_max(rx_len);
    const uint32_t grid = (uint32_t)(ntm < SV_GRID ? ntm : SV_GRID);
    dsieve* sv = reinterpret_cast<dsieve*>(b.state);
    hipError_t e = hipMemsetAsync(b.pool_n, 0, 8, st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_sieve_count, dim3(grid), dim3(SV_THREADS), 0, st, rx, rx_len, segs, mid, npred, sieve_min(),
                       b.tcount, b.slot, b.pool, reinterpret_cast<unsigned long long*>(b.pool_n), b.capS, ntm, sv);
    if ((e = launch_exclusive_scan(b.tcount, b.tbase, ntm, b.tmp, b.m_total, st)) != hipSuccess) return e;
    const uint64_t fb = (ntm + 255) / 256;
    hipLaunchKernelGGL(k_sieve_fill, dim3((uint32_t)(fb < 8192 ? fb : 8192)), dim3(256), 0, st, segs, mid, b.tcount,
                       b.tbase, b.slot, b.pool, b.S, b.m_total, b.capS, sv);
    const uint32_t lg = (uint32_t)((b.capS + 255) / 256 < 8192 ? (b.capS + 255) / 256 : 8192);
    hipLaunchKernelGGL(k_sieve_link, dim3(lg), dim3(256), 0, st, rx, rx_len, segs, mid, b.S, b.m_total, b.capS, b.J0,
                       b.mark, sv);
    uint32_t* Jin = b.J0;
    uint32_t* Jout = b.J1;
    const uint32_t rounds = jump_rounds(b.capS);
    for (uint32_t r = 0; r < rounds; ++r) {
        hipLaunchKernelGGL(k_sieve_jump, dim3(lg < 1024 ? lg : 1024), dim3(256), 0, st, Jin, Jout, b.mark, b.m_total,
                           b.capS, sv, r);
        uint32_t* t = Jin;
        Jin = Jout;
        Jout = t;
    }
    e = launch_exclusive_scan(b.mark, b.rank, b.capS, b.tmp, b.npath, st);
    if (e != hipSuccess) return e;
    return hipGetLastError();
}

hipError_t launch_sieve_emit(const uint8_t* rx, uint64_t rx_len, const dseg* segs, const dmid* mid,
                             const sieve_bufs& b, dframes fr, uint32_t vmask, hipStream_t st) {
    const uint32_t lg = (uint32_t)((b.capS + 255) / 256 < 8192 ? (b.capS + 255) / 256 : 8192);
    hipLaunchKernelGGL(k_sieve_emit, dim3(lg), dim3(256), 0, st, rx, rx_len, segs, mid, b.S, b.m_total, b.capS,
                       b.mark, b.rank, b.npath, fr, vmask, reinterpret_cast<dsieve*>(b.state));
    return hipGetLastError();
}

}  // namespace hvws

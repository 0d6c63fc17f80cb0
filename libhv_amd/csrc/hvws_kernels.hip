// hvws_kernels.hip -- HIP kernels of the MI355X WebSocket receive path (gfx950).
//
//   k_scan        frame discovery + header parse (FIN/opcode/mask/length/key)
//                 for every segment of a batch: one wavefront per segment,
//                 speculative stride walk verified with a 64-lane ballot.
//                 Replaces the per-byte switch of websocket_parser_execute
//                 (reference http/websocket_parser.c:53-171).
//   k_offsets     exclusive scan of per-segment frame counts.
//   k_tile_scatter / k_tile_fixup  first frame touching each unmask tile.
//   k_unmask      rotating 32-bit XOR of every masked payload byte, in place,
//                 16-B coalesced loads/stores, tile frame table staged in LDS.
//                 Replaces websocket_parser_decode's byte loop
//                 (http/websocket_parser.c:173-180) as called by
//                 WebSocketParser::on_frame_body (http/WebSocketParser.cpp:32-34).
//   k_stream_xor  STREAM-style in-place read+write ceiling for the roofline.
//
// All work is integer; there is no contraction, so no MFMA.  The unmask is
// HBM-bound: 2 x payload + headers bytes per pass.
#include <stdio.h>
#include <stdlib.h>

#include <hip/hip_ext.h>

#include "hvws_dev.h"

namespace hvws {

// Exact byte-level state machine for one frame episode starting from `st` at
// segment-relative `pos`: used for the carry-in frame and for the incomplete
// frame at the segment end (the speculative walk handles everything whole in
// between).  Mirrors http/websocket_parser.c:60-164 state by state, with the
// payload decoded by WebSocketParser (mask_offset advanced over masked bytes).
// Returns true when any callback of the reference would fire for this frame
// inside the segment (then `r` holds its record).  All lanes run it
// redundantly on the same bytes, so control flow stays wave-uniform.
__device__ bool scalar_frame(const uint8_t* seg, uint64_t L, dcarry& st, uint64_t& pos, frec& r, uint32_t vmask) {
    r.hdr_off = -1;
    r.pay_off = 0;
    r.pay_len = 0;
    r.length = 0;
    r.key = 0;
    r.info = 0;
    bool have = false;
    if (st.state == S_START) {
        if (pos >= L) return false;
        uint32_t b0 = seg[pos];
        st.offset = 0;
        st.length = 0;
        st.mask_offset = 0;
        st.flags = (b0 & F_OPMASK) | ((b0 & 0x80u) ? F_FIN : 0u);
        st.viol = ((b0 & 0x70u) ? V_RSV : 0u) | (reserved_opcode(b0 & F_OPMASK) ? V_OPCODE : 0u);
        st.state = S_HEAD;
        st.started = 1;
        r.hdr_off = (int64_t)pos;
        r.info |= I_START;
        ++pos;
    }
    if (st.state == S_HEAD) {
        if (pos >= L) return false;
        uint32_t b1 = seg[pos];
        ++pos;
        st.length = b1 & 0x7Fu;
        if (b1 & 0x80u) st.flags |= F_MASK;
        if ((st.flags & 8u) && !(st.flags & F_FIN)) st.viol |= V_CONTROL;   // length checked once decoded
        if (!(b1 & 0x80u)) st.viol |= V_UNMASKED;
        if (st.length >= 126) st.viol |= (st.length == 127 ? 2u : 1u) << V_ENC_SHIFT;
        if (st.length >= 126) {
            st.require = st.length == 127 ? 8 : 2;
            st.length = 0;
            st.state = S_LENGTH;
        } else if (st.flags & F_MASK) {
            st.state = S_MASK;
            st.require = 4;
        } else if (st.length) {
            st.state = S_BODY;
            st.require = st.length;
            hdr_complete(r, st, pos, vmask);
            have = true;
        } else {
            st.state = S_START;
            hdr_complete(r, st, pos, vmask);
            r.info |= I_END;
            return true;
        }
    }
    if (st.state == S_LENGTH) {
        while (pos < L && st.require) {
            st.length = (st.length << 8) | seg[pos];
            --st.require;
            ++pos;
        }
        if (st.require) return false;
        {
            const uint32_t enc = (st.viol >> V_ENC_SHIFT) & 3u;
            if (enc == 2 && (st.length >> 63)) st.viol |= V_LEN64;
            if ((enc == 1 && st.length < 126) || (enc == 2 && st.length <= 0xFFFFu)) st.viol |= V_NONMIN;
            if ((st.flags & 8u) && st.length > 125) st.viol |= V_CONTROL;
        }
        if (st.flags & F_MASK) {
            st.state = S_MASK;
            st.require = 4;
        } else if (st.length) {
            st.state = S_BODY;
            st.require = st.length;
            hdr_complete(r, st, pos, vmask);
            have = true;
        } else {
            st.state = S_START;
            hdr_complete(r, st, pos, vmask);
            r.info |= I_END;
            return true;
        }
    }
    if (st.state == S_MASK) {
        while (pos < L && st.require) {
            uint32_t sh = 8u * (uint32_t)(4 - st.require);
            st.mask = (st.mask & ~(0xFFu << sh)) | ((uint32_t)seg[pos] << sh);
            --st.require;
            ++pos;
        }
        if (st.require) return false;
        if (st.length) {
            st.state = S_BODY;
            st.require = st.length;
            hdr_complete(r, st, pos, vmask);
            have = true;
        } else {
            st.state = S_START;
            hdr_complete(r, st, pos, vmask);
            r.info |= I_END;
            return true;
        }
    }
    if (st.state == S_BODY) {
        if (st.require == 0) {
            // Unreachable through the reference API (body states are entered
            // with require > 0); mirrored: end the frame, skip one byte.
            if (pos >= L) return have;
            if (!have) {
                r.info = (st.flags & 0xFFu) | ((st.mask_offset & 3u) << 8);
                r.length = st.length;
                r.key = (st.flags & F_MASK) ? st.mask : 0u;
                r.pay_off = pos;
            }
            st.state = S_START;
            r.info |= I_END;
            ++pos;
            return true;
        }
        if (pos >= L) return have;
        if (!have) {   // continuing frame: header was in an earlier batch
            r.info = (st.flags & 0xFFu) | ((st.mask_offset & 3u) << 8);
            r.length = st.length;
            r.key = (st.flags & F_MASK) ? st.mask : 0u;
        }
        uint64_t avail = L - pos;
        uint64_t nb = st.require < avail ? st.require : avail;
        r.pay_off = pos;
        r.pay_len = nb;
        r.info |= I_BODY;
        if (st.flags & F_MASK) st.mask_offset = (uint32_t)((st.mask_offset + nb) & 3u);
        st.require -= nb;
        pos += nb;
        if (st.require == 0) {
            st.state = S_START;
            r.info |= I_END;
        } else {
            st.offset += L - r.pay_off;   // http/websocket_parser.c:153
        }
        return true;
    }
    return have;
}

// ----------------------------------------------------------------- k_head
//
// Discovery runs in three kernels per pass (COUNT, then EMIT):
//   k_head    one wavefront per segment: finish the frame carried in from the
//             previous batch (exact byte state machine), then parse the first
//             whole frame; its size is the speculation stride.  Long segments
//             (>= spec_min() predicted frames) are handed to k_verify.
//   k_verify  the whole grid checks the predicted headers of every long
//             segment at pos + j*stride in parallel (first break per segment
//             by atomicMin); every prediction before the first break is a
//             true frame by induction from the known header at pos, so a
//             uniform stream is verified in one parallel pass whatever its
//             length.  EMIT writes those frames.
//   k_walk    one wavefront per segment continues after the verified prefix
//             with a wave-wide speculative walk (64 x SCAN_U predictions per
//             HBM round trip, broken chains re-predicted from the true size),
//             then the exact state machine for the frame cut by the segment
//             end.  Mixed-size streams advance >= 1 frame per round trip.

// Predicted frames that make a segment "long" (grid-wide k_verify); shorter
// uniform runs are verified by k_walk's wave-wide speculation, 256 frames
// per round, all segments in parallel.  $HVWS_EXPERIMENT spec_min overrides (tuning).
constexpr uint64_t SPEC_MIN_DEFAULT = 4096;
static uint64_t g_spec_min = 0;   // 0: not yet read from the environment

uint64_t spec_min() {
    if (!g_spec_min) {
        const char* e = experiment("spec_min");
        const long long x = e ? atoll(e) : 0;
        g_spec_min = x > 0 ? (uint64_t)x : SPEC_MIN_DEFAULT;
    }
    return g_spec_min;
}

uint64_t set_spec_min(uint64_t v) {
    const uint64_t old = spec_min();
    g_spec_min = v ? v : SPEC_MIN_DEFAULT;
    return old;
}

enum : uint32_t {
    HEAD_ZERO_LM = 1u,     // also clear last_masked (no k_head<true> follows)
    HEAD_NO_VERIFY = 2u    // no k_verify follows (see head_body)
};

template <bool EMIT>
__device__ __forceinline__ void head_body(const uint8_t* __restrict__ rx, uint64_t rx_len,
                                                       const dseg* __restrict__ segs, uint32_t nseg,
                                                       const dcarry* __restrict__ carry_in, dmid* __restrict__ mid,
                                                       uint64_t* __restrict__ npred, uint64_t* __restrict__ first_fail,
                                                       uint64_t* __restrict__ last_masked,
                                                       const uint64_t* __restrict__ bases, dframes fr, uint32_t vmask,
                                                       uint64_t spec_min, uint64_t* __restrict__ est,
                                                       const dseg* __restrict__ src_segs,
                                                       const dcarry* __restrict__ src_carry, dseg* __restrict__ segs_w,
                                                       dcarry* __restrict__ carry_w, int probe_mixed,
                                                       uint64_t slack_cap, uint64_t* __restrict__ est_u,
                                          uint32_t w0, uint32_t wn, uint32_t hflags, drun* __restrict__ runs,
                                          uint32_t* __restrict__ run_fail) {
    const uint32_t lane = threadIdx.x & 63u;
    for (uint32_t s = w0; s < nseg; s += wn) {
        dseg sg;
        dcarry st;
        if (src_segs) {
            // Zero-copy upload: lanes 0-3 each fetch one 16-B piece of the
            // segment's 64 bytes (segment + carry) from host memory, store it
            // into the device tables and broadcast it -- one PCIe read per
            // piece instead of one per lane.
            u32x4 piece = {0u, 0u, 0u, 0u};
            if (lane == 0) piece = *reinterpret_cast<const u32x4*>(&src_segs[s]);
            else if (lane < 4) piece = reinterpret_cast<const u32x4*>(&src_carry[s])[lane - 1];
            if (lane == 0) *reinterpret_cast<u32x4*>(&segs_w[s]) = piece;
            else if (lane < 4) reinterpret_cast<u32x4*>(&carry_w[s])[lane - 1] = piece;
            uint32_t w[16];
#pragma unroll
            for (int p = 0; p < 4; ++p) {
                w[4 * p + 0] = __shfl(piece.x, p);
                w[4 * p + 1] = __shfl(piece.y, p);
                w[4 * p + 2] = __shfl(piece.z, p);
                w[4 * p + 3] = __shfl(piece.w, p);
            }
            __builtin_memcpy(&sg, &w[0], sizeof(sg));
            __builtin_memcpy(&st, &w[4], sizeof(st));
        } else {
            sg = segs[s];
            st = carry_in[s];
        }
        const uint64_t sb = sg.off, L = sg.len;
        st.started = 0;
        const dcarry st_in = st;
        uint64_t pos = 0, n = 0;
        frec r;
        r.info = 0;
        if (st.state != S_START && scalar_frame(rx + sb, L, st, pos, r, vmask)) {
            if (EMIT && lane == 0) store_frame(fr, bases[s], sb, r);
            ++n;
        }
        uint64_t stride = 0, np = 0, mixed = 0;
        hdr h;
        h.hlen = 0;
        h.length = 0;
        h.flags = 0;
        if (st.state == S_START && parse_at(rx, rx_len, sb, L, pos, h)) {
            stride = (uint64_t)h.hlen + h.length;
            const uint64_t cnt = (L - pos) / stride;
            // probe_mixed (one-stream passes): run the probe at any length and
            // record whether the sizes vary -- the frame sieve's trigger.
            if (cnt >= spec_min || (probe_mixed && cnt >= 2)) {
                // Probe before committing the grid: lanes 0-31 check
                // predictions 2^(l/2) (near the start), lanes 32-63 spread over
                // the whole range.  Speculation stops at the first probe that
                // breaks, so a mixed-size stream costs no grid-wide work and
                // no atomic storm; a uniform one keeps every prediction.
                uint64_t j = lane < 32 ? (1ull << (lane / 2)) + (lane & 1) * ((1ull << (lane / 2)) >> 1)
                                       : ((uint64_t)(lane - 31) * cnt) / 33;
                if (j >= cnt) j = cnt - 1;
                hdr hp;
                const uint64_t q = pos + j * stride;
                const bool ok = parse_at(rx, rx_len, sb, L, q, hp) && (uint64_t)hp.hlen + hp.length == stride;
                uint64_t jb = ok ? cnt : j;
                for (int o = 32; o > 0; o >>= 1) {
                    const uint64_t other = __shfl_xor(jb, o);
                    jb = other < jb ? other : jb;
                }
                np = cnt >= spec_min && jb >= spec_min ? jb : 0;
                mixed = jb < cnt;
            } else if (probe_mixed) {
                mixed = 1;   // the first frame covers over half the segment: sizes unknown
            }
        }
        uint64_t e = n;   // records if every frame after pos had size `stride`
        if (est && st.state == S_START && pos < L) {
            uint64_t q = pos;
            if (stride) {
                const uint64_t cnt = (L - pos) / stride;
                e += cnt;
                q += cnt * stride;
            }
            // the frame cut by the segment end fires a record iff its
            // header completes inside the segment
            const uint64_t rem = L - q;
            if (rem >= 2) {
                const uint32_t b1 = rx[sb + q + 1];
                const uint32_t len7 = b1 & 0x7Fu;
                const uint64_t hl = 2u + (len7 == 126 ? 2u : (len7 == 127 ? 8u : 0u)) + ((b1 & 0x80u) ? 4u : 0u);
                if (hl <= rem) ++e;
            }
        }
        if (runs && lane == 0) {
            // RUN: the segment as one run of frames of the first whole one's
            // size (the hypothesis k_unmask_run checks header by header), with
            // the carried-in frame and the frame cut by the segment end exact.
            drun d;
            d.seg_lo = sb;
            d.seg_hi = sb + L;
            d.flags = 0;
            d.a_off = d.a_end = d.t_off = d.t_end = 0;
            d.a_kw = d.t_kw = 0;
            d.pad = 0;
            if (n && (r.info & I_BODY) && (r.info & F_MASK)) {   // the carried-in frame's payload here
                d.a_off = sb + r.pay_off;
                d.a_end = d.a_off + r.pay_len;
                d.a_kw = key_for_aligned(r.key, d.a_off, (r.info >> 8) & 3u);
            }
            const uint64_t cnt = stride ? (L - pos) / stride : 0;
            d.p0 = sb + pos;
            d.stride = stride;
            d.len = h.length;
            d.inv = stride ? 1.0 / (double)stride : 0.0;
            d.cnt = (uint32_t)cnt;
            d.hlen = h.hlen;
            d.masked = (h.flags & F_MASK) ? 1u : 0u;
            if (cnt > 0xFFFFFFFFull) d.flags |= RUN_BAD;
            if (st.state == S_START) {
                // the frame after the run: cut by the segment end (its payload
                // piece here), or it must end exactly there -- anything after
                // it means the segment is not one run
                const uint64_t q = pos + cnt * stride;
                if (q < L && L - q >= 2) {
                    uint64_t lo, hi;
                    ld16(rx, rx_len, sb + q, lo, hi);
                    const hdr ht = parse_hdr(lo, hi);
                    if (ht.hlen <= L - q) {
                        const uint64_t ps = q + ht.hlen, rem = L - ps;
                        if (ht.length < rem) d.flags |= RUN_BAD;
                        if ((ht.flags & F_MASK) && rem && ht.length) {
                            d.t_off = sb + ps;
                            d.t_end = sb + ps + (ht.length < rem ? ht.length : rem);
                            d.t_kw = key_for_aligned(ht.key, d.t_off, 0);
                        }
                    }
                }
            }
            d.cin = st_in;
            runs[s] = d;
            run_fail[s] = 0;
            if (d.flags & RUN_BAD) atomicOr(&run_fail[nseg], 1u);   // the repair pass must look
        }
        if (lane == 0) {
            // SLACK (mixed sizes): the segment's region of the slack table --
            // its record bound, at most slack_cap records
            if (est) est[s] = slack_cap ? min(L / 2 + 3, slack_cap) : e;
            if (est_u) est_u[s] = e;   // SLACK: the uniform estimate, to tell whether SPEC would hold
            dmid m;
            m.st = st;
            m.pos = pos;
            m.stride = stride;
            m.n_a = n;
            m.pad = mixed;   // read by the frame sieve (hvws_sieve.hip)
            mid[s] = m;
            npred[s] = np;
            // HEAD_NO_VERIFY: no k_verify follows; the walk takes every frame
            // (first_fail 0), npred keeps the candidate count as a hint
            if (!EMIT) first_fail[s] = (hflags & HEAD_NO_VERIFY) ? 0 : np;
            if (EMIT || (hflags & HEAD_ZERO_LM)) last_masked[s] = 0;
        }
    }
}

template <bool EMIT>
__global__ __launch_bounds__(SCAN_THREADS) void k_head(const uint8_t* __restrict__ rx, uint64_t rx_len,
                                                       const dseg* __restrict__ segs, uint32_t nseg,
                                                       const dcarry* __restrict__ carry_in, dmid* __restrict__ mid,
                                                       uint64_t* __restrict__ npred, uint64_t* __restrict__ first_fail,
                                                       uint64_t* __restrict__ last_masked,
                                                       const uint64_t* __restrict__ bases, dframes fr, uint32_t vmask,
                                                       uint64_t spec_min, uint64_t* __restrict__ est,
                                                       const dseg* __restrict__ src_segs,
                                                       const dcarry* __restrict__ src_carry, dseg* __restrict__ segs_w,
                                                       dcarry* __restrict__ carry_w, int probe_mixed,
                                                       uint64_t slack_cap, uint64_t* __restrict__ est_u,
                                                       uint32_t hflags, drun* __restrict__ runs,
                                                       uint32_t* __restrict__ run_fail) {
    const uint32_t wpb = SCAN_THREADS / 64;
    head_body<EMIT>(rx, rx_len, segs, nseg, carry_in, mid, npred, first_fail, last_masked, bases, fr, vmask, spec_min, est,
                    src_segs, src_carry, segs_w, carry_w, probe_mixed, slack_cap, est_u,
                    blockIdx.x * wpb + (threadIdx.x >> 6), gridDim.x * wpb, hflags, runs, run_fail);
}

// --------------------------------------------------------------- k_verify
template <bool EMIT>
__device__ __forceinline__ void verify_body(const uint8_t* __restrict__ rx, uint64_t rx_len,
                                                const dseg* __restrict__ segs, uint32_t nseg,
                                                const dmid* __restrict__ mid, const uint64_t* __restrict__ pbase,
                                                uint64_t total,
                                                uint64_t* __restrict__ first_fail,
                                                uint64_t* __restrict__ last_masked,
                                                const uint64_t* __restrict__ bases, dframes fr, uint32_t vmask,
                                            uint32_t bid, uint32_t nb) {
    if (total == 0) return;
    const uint64_t per = (total + nb - 1) / nb;
    const uint64_t g0 = (uint64_t)bid * per;
    const uint64_t g1 = g0 + per < total ? g0 + per : total;
    if (g0 >= g1) return;
    // segment holding g0: last s with pbase[s] <= g0 (pbase is non-decreasing)
    uint32_t lo = 0, hi = nseg;
    while (hi - lo > 1) {
        const uint32_t m = (lo + hi) >> 1;
        if (pbase[m] <= g0) lo = m;
        else hi = m;
    }
    uint32_t s = lo;
    // EMIT tracks the last masked verified frame per segment; it is flushed
    // with one atomic per wave (a per-frame atomic on one word serialises
    // the whole grid: 1M frames took 12 ms that way).
    uint32_t ms = s;
    uint64_t mmax = 0;
    for (uint64_t g = g0 + threadIdx.x; g < g1; g += blockDim.x) {
        while (s + 1 < nseg && pbase[s + 1] <= g) ++s;
        const uint64_t j = g - pbase[s];
        const dmid& m = mid[s];
        const uint64_t q = m.pos + j * m.stride;
        hdr h;
        const bool whole = parse_at(rx, rx_len, segs[s].off, segs[s].len, q, h);
        const bool ok = whole && (uint64_t)h.hlen + h.length == m.stride;
        if (!EMIT) {
            // filter on a (possibly stale, never too small) read first
            if (!ok && j < __hip_atomic_load(&first_fail[s], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
                atomicMin((unsigned long long*)&first_fail[s], (unsigned long long)j);
        } else if (j < first_fail[s]) {
            frec v;
            whole_frame_rec(v, q, h, vmask);
            store_frame(fr, bases[s] + m.n_a + j, segs[s].off, v);
            if (h.flags & F_MASK) {
                if (ms != s && mmax) {
                    atomicMax((unsigned long long*)&last_masked[ms], (unsigned long long)mmax);
                    mmax = 0;
                }
                ms = s;
                mmax = j + 1 > mmax ? j + 1 : mmax;
            }
        }
    }
    if (EMIT) {
        // Segment-uniform block (the common case): reduce in registers and
        // LDS, one atomic per block -- one per wave still serialised 16K
        // same-address atomics for a 1M-frame stream (~80 us).
        __shared__ uint32_t s_seg[256 / 64];
        __shared__ uint64_t s_max[256 / 64];
        const uint32_t ms0 = __shfl(ms, 0);
        const bool wave_uniform = __all(ms == ms0);
        uint64_t wmax = mmax;
        for (int o = 32; o > 0; o >>= 1) {
            const uint64_t other = __shfl_xor(wmax, o);
            wmax = other > wmax ? other : wmax;
        }
        const uint32_t w = threadIdx.x >> 6;
        if ((threadIdx.x & 63u) == 0) {
            s_seg[w] = wave_uniform ? ms0 : 0xFFFFFFFFu;
            s_max[w] = wmax;
        }
        __syncthreads();
        bool block_uniform = true;
        for (uint32_t i = 0; i < blockDim.x / 64; ++i) block_uniform &= s_seg[i] == s_seg[0] && s_seg[i] != 0xFFFFFFFFu;
        if (block_uniform) {
            if (threadIdx.x == 0) {
                uint64_t bmax = 0;
                for (uint32_t i = 0; i < blockDim.x / 64; ++i) bmax = s_max[i] > bmax ? s_max[i] : bmax;
                if (bmax) atomicMax((unsigned long long*)&last_masked[s_seg[0]], (unsigned long long)bmax);
            }
        } else if (wave_uniform) {
            if ((threadIdx.x & 63u) == 0 && wmax)
                atomicMax((unsigned long long*)&last_masked[ms0], (unsigned long long)wmax);
        } else if (mmax) {
            atomicMax((unsigned long long*)&last_masked[ms], (unsigned long long)mmax);
        }
    }
}

template <bool EMIT>
__global__ __launch_bounds__(256) void k_verify(const uint8_t* __restrict__ rx, uint64_t rx_len,
                                                const dseg* __restrict__ segs, uint32_t nseg,
                                                const dmid* __restrict__ mid, const uint64_t* __restrict__ pbase,
                                                const uint64_t* __restrict__ total_pred,
                                                uint64_t* __restrict__ first_fail,
                                                uint64_t* __restrict__ last_masked,
                                                const uint64_t* __restrict__ bases, dframes fr, uint32_t vmask) {
    verify_body<EMIT>(rx, rx_len, segs, nseg, mid, pbase, *total_pred, first_fail, last_masked, bases, fr, vmask,
                      blockIdx.x, gridDim.x);
}

// Whole frames from segment offset `pos` on (wave-wide speculative walk,
// 64 x SCAN_U predictions per round), then the exact state machine for the
// frame cut by the segment end.  Advances st/pos/n; emit(idx, rec) is called
// (EMIT only) by the lane owning record idx of the segment.
template <bool EMIT, typename Emit>
__device__ __forceinline__ void walk_frames(const uint8_t* __restrict__ rx, uint64_t rx_len, uint64_t sb, uint64_t L,
                                            dcarry& st, uint64_t& pos, uint64_t& n, uint32_t vmask, Emit&& emit) {
    const uint32_t lane = threadIdx.x & 63u;
    constexpr uint32_t NPRED = 64u * SCAN_U;
    uint64_t stride = 0;
    // Speculation width (wave-uniform): predictions loaded per round.  A run
    // of equal sizes doubles it up to NPRED; a break shrinks it to about
    // twice the frames the round proved, so a mixed-size stream costs ~2
    // header loads per frame (one HBM round trip) instead of NPRED scattered
    // loads, most of them TLB misses.
    uint32_t width = NPRED;
    while (st.state == S_START && pos < L) {
        const uint64_t rem = L - pos;
        if (stride == 0) {
            hdr h0;
            if (!parse_at(rx, rx_len, sb, L, pos, h0)) break;   // incomplete: tail
            stride = (uint64_t)h0.hlen + h0.length;
        }
        uint64_t lo[SCAN_U], hi[SCAN_U];
        bool inr[SCAN_U];
#pragma unroll
        for (int u = 0; u < SCAN_U; ++u) {
            const uint32_t j = (uint32_t)u * 64u + lane;
            // j * stride <= rem - 2 (j < 2^8, so it overflows only for strides
            // past 2^56; no 64-bit division per prediction)
            uint64_t off;
            inr[u] = j < width && rem >= 2 && !__builtin_mul_overflow((uint64_t)j, stride, &off) && off <= rem - 2;
            lo[u] = hi[u] = 0;
            if (inr[u]) ld16(rx, rx_len, sb + pos + (uint64_t)j * stride, lo[u], hi[u]);
        }
        // Per prediction only what the records need is kept: the key and a
        // packed (flags | hlen << 8 | viol << 16); a frame that holds has
        // length = stride - hlen.  The first break's wholeness and size are
        // taken while its header is parsed.  (Holding the parsed headers of
        // all SCAN_U predictions cost 134 VGPRs, 3 waves per SIMD.)
        uint32_t key[SCAN_U], pk[SCAN_U];
        uint32_t f = NPRED;
        bool wf = false;
        uint64_t sf = 0;
#pragma unroll
        for (int u = 0; u < SCAN_U; ++u) {
            const uint32_t j = (uint32_t)u * 64u + lane;
            const uint64_t q = pos + (uint64_t)j * stride;
            const hdr h = parse_hdr(lo[u], hi[u]);
            const uint64_t rq = inr[u] ? L - q : 0;
            const bool whole = inr[u] && h.hlen <= rq && h.length <= rq - h.hlen;
            const uint64_t sz = (uint64_t)h.hlen + h.length;
            const bool ok = whole && sz == stride;
            key[u] = h.key;
            pk[u] = h.flags | (h.hlen << 8) | (h.viol << 16);
            const unsigned long long bad = __ballot(!ok);
            if (f == NPRED && bad) {
                const int lf = __ffsll((long long)bad) - 1;
                f = (uint32_t)u * 64u + (uint32_t)lf;
                wf = __shfl((int)whole, lf) != 0;
                sf = __shfl(sz, lf);
            }
        }
        uint32_t last_flags = 0, last_key = 0;
        uint64_t last_len = 0;
        bool any_masked = false;
#pragma unroll 1
        for (int u = 0; u < SCAN_U; ++u) {   // not unrolled: 4 records' stores in flight cost ~30 VGPRs
            const uint32_t j = (uint32_t)u * 64u + lane;
            const bool mine = j < f;
            const uint32_t fl = pk[u] & 0xFFu, hl = (pk[u] >> 8) & 0xFFu;
            if (EMIT && mine) {
                const uint64_t q = pos + (uint64_t)j * stride;
                const uint64_t len = stride - hl;
                frec v;
                v.hdr_off = (int64_t)q;
                v.pay_off = q + hl;
                v.pay_len = len;
                v.length = len;
                v.key = key[u];
                v.info = fl | I_HDR | I_START | I_END | (len ? I_BODY : 0u) | invalid_bits(pk[u] >> 16, vmask);
                emit(n + j, v);
            }
            const unsigned long long mm = __ballot(mine && (fl & F_MASK));
            if (mm) {
                const int src = 63 - __clzll((long long)mm);
                last_key = __shfl(key[u], src);
                any_masked = true;
            }
            if (f > (uint32_t)u * 64u && f <= (uint32_t)u * 64u + 64u) {
                const int src = (int)(f - 1 - (uint32_t)u * 64u);
                last_flags = __shfl(fl, src);
                last_len = stride - __shfl(hl, src);
            }
        }
        if (f > 0) {
            st.flags = last_flags;   // Q14: the last frame's fields persist
            st.length = last_len;
            st.require = 0;
            st.offset = 0;
            st.mask_offset = (last_flags & F_MASK) ? (uint32_t)(last_len & 3u) : 0u;
            st.started = 0;
            if (any_masked) st.mask = last_key;
        }
        n += f;
        pos += (uint64_t)f * stride;
        if (f == width) {   // every prediction held: widen, same stride
            width = width * 2 < NPRED ? width * 2 : NPRED;
            continue;
        }
        width = f * 2 < 2 ? 2 : (f * 2 < NPRED ? f * 2 : NPRED);
        if (pos >= L) break;
        if (!wf) break;
        stride = sf;
    }

    if (st.state == S_START && pos < L) {   // frame cut by the segment end
        frec r;
        if (scalar_frame(rx + sb, L, st, pos, r, vmask)) {
            if (EMIT && lane == 0) emit(n, r);
            ++n;
        }
    }
}

// ----------------------------------------------------------------- k_walk
// carry_rec (EMIT, one-launch scan): also write the record of the frame
// carried in from the previous batch (k_head<true>'s job in the kernel
// chain), re-running the exact state machine from the carried-in state.
template <bool EMIT>
__device__ __forceinline__ void walk_body(const uint8_t* __restrict__ rx, uint64_t rx_len,
                                          const dseg* __restrict__ segs, uint32_t nseg,
                                          const dmid* __restrict__ mid,
                                          const uint64_t* __restrict__ npred,
                                          const uint64_t* __restrict__ first_fail,
                                          const uint64_t* __restrict__ last_masked,
                                          dcarry* __restrict__ carry_out, uint64_t* __restrict__ counts,
                                          const uint64_t* __restrict__ bases, dframes fr, uint32_t vmask,
                                          int emit_counts, const dsieve* __restrict__ sv,
                                          const uint64_t* __restrict__ sv_S, const dcarry* __restrict__ carry_rec,
                                          uint32_t w0, uint32_t wn) {
    const uint32_t lane = threadIdx.x & 63u;

    for (uint32_t s = w0; s < nseg; s += wn) {
        const uint64_t sb = segs[s].off;
        const uint64_t L = segs[s].len;
        const dmid m = mid[s];
        dcarry st = m.st;
        uint64_t pos = m.pos;
        uint64_t n = m.n_a;
        const uint64_t obase = EMIT ? bases[s] : 0;
        if (EMIT && carry_rec && m.n_a) {
            dcarry c0 = carry_rec[s];
            c0.started = 0;
            uint64_t p0 = 0;
            frec r;
            scalar_frame(rx + sb, L, c0, p0, r, vmask);
            if (lane == 0) store_frame(fr, obase, sb, r);
        }

        // Skip the prefix k_verify proved; restore the fields the reference
        // leaves behind after its last frame (Q14).
        const uint64_t f0 = npred[s] ? first_fail[s] : 0;
        if (f0) {
            pos += f0 * m.stride;
            n += f0;
            hdr h;
            parse_at(rx, rx_len, sb, L, pos - m.stride, h);
            st.flags = h.flags;
            st.length = h.length;
            st.require = 0;
            st.offset = 0;
            st.mask_offset = (h.flags & F_MASK) ? (uint32_t)(h.length & 3u) : 0u;
            st.started = 0;
            if (EMIT && last_masked[s]) {
                hdr hm;
                parse_at(rx, rx_len, sb, L, m.pos + (last_masked[s] - 1) * m.stride, hm);
                st.mask = hm.key;
            }
        }

        // One stream sieved (hvws_sieve.hip): its chain of whole frames is
        // recorded; resume after it with the fields its last frame leaves.
        if (sv && s == 0 && sv->use) {
            const uint64_t np = sv->pend;
            hdr h;
            parse_at(rx, rx_len, sb, L, sv->last - 1, h);
            n += sv->npath;
            pos = np;
            st.flags = h.flags;
            st.length = h.length;
            st.require = 0;
            st.offset = 0;
            st.mask_offset = (h.flags & F_MASK) ? (uint32_t)(h.length & 3u) : 0u;
            st.started = 0;
            if (sv->last_masked) {
                hdr hm;
                parse_at(rx, rx_len, sb, L, sv->last_masked - 1, hm);
                st.mask = hm.key;
            }
        }

        walk_frames<EMIT>(rx, rx_len, sb, L, st, pos, n, vmask,
                          [&](uint64_t idx, const frec& v) { store_frame(fr, obase + idx, sb, v); });
        if (lane == 0) {
            if (!EMIT || emit_counts) counts[s] = n;
            if (EMIT) carry_out[s] = st;
        }
    }
}

template <bool EMIT>
__global__ __launch_bounds__(SCAN_THREADS) void k_walk(const uint8_t* __restrict__ rx, uint64_t rx_len,
                                                       const dseg* __restrict__ segs, uint32_t nseg,
                                                       const dmid* __restrict__ mid,
                                                       const uint64_t* __restrict__ npred,
                                                       const uint64_t* __restrict__ first_fail,
                                                       const uint64_t* __restrict__ last_masked,
                                                       dcarry* __restrict__ carry_out, uint64_t* __restrict__ counts,
                                                       const uint64_t* __restrict__ bases, dframes fr, uint32_t vmask,
                                                       int emit_counts, const dsieve* __restrict__ sv,
                                                       const uint64_t* __restrict__ sv_S,
                                                       const dcarry* __restrict__ carry_rec) {
    const uint32_t wpb = SCAN_THREADS / 64;
    walk_body<EMIT>(rx, rx_len, segs, nseg, mid, npred, first_fail, last_masked, carry_out, counts, bases, fr, vmask,
                    emit_counts, sv, sv_S, carry_rec, blockIdx.x * wpb + (threadIdx.x >> 6), gridDim.x * wpb);
}

// ----------------------------------------------------------------- k_small
//
// Small batches (an event loop's reads, FeedRecvData): one wavefront per
// segment runs the whole hot path in a single launch -- the carried-in frame
// (exact state machine), the speculative walk and the tail (the same device
// code as the COUNT/EMIT kernels), records, then the XOR of the segment's
// masked payload bytes -- and writes its results straight into pinned host
// memory: the changed 16-byte chunks, the records (compacted by one atomic per
// segment), the count and the carry.  One launch and one sync (plus one H2D
// copy unless zero-copy) replace the ~15 operations of the general path,
// whose fixed cost dominates reads of a few KiB.
//
// A read's time is a chain of dependent memory round trips (~1 us each to HBM,
// several us across PCIe), so STAGE (segments <= kZcSegment) first pulls the
// whole segment into LDS in one round of 16-byte loads; the walk, the tail and
// the XOR then read LDS, and the records stay in LDS (the first SMALL_LREC of
// them; more spill to the device slot).  `rx` handed to the body is a flat
// pointer biased so absolute offsets in [sb, se) land in LDS, with rx_len = se
// (bytes past the segment end never decide a result: a header that reaches
// past it is incomplete whatever those bytes hold).  The source is device
// memory (after the H2D copy) or, zero-copy, the pinned host buffer itself.
constexpr uint32_t SMALL_LREC = 512;      // records kept in LDS (20 KiB)
constexpr uint32_t SMALL_BY_RECORD = 64;  // up to this many records: record-major XOR

// Bytes [lo, hi) of a 64-bit word (bounds clamped to [0, 8]).
__device__ __forceinline__ uint64_t byte_range(int64_t lo, int64_t hi) {
    lo = lo < 0 ? 0 : lo;
    hi = hi > 8 ? 8 : hi;
    if (hi <= lo) return 0;
    const uint64_t h = hi >= 8 ? ~0ull : ((1ull << (8 * hi)) - 1);
    return h & ~((1ull << (8 * lo)) - 1);
}

// k_small's XOR of segment [sb, se): records via rec(i) (sorted by payload
// offset), n of them.  The key stream is periodic in absolute offsets, so a
// chunk's mask is the key word rotated for the chunk start, cut to the bytes
// each masked payload covers.  STAGE: XOR the LDS copy (lds holds offset sb16
// at 0), then a pass of host stores only -- no load between the stores (a
// vector-memory load waits for every older store's round trip).
template <bool STAGE, typename Rec>
__device__ __forceinline__ void small_xor(Rec rec, uint64_t n, uint64_t sb, uint64_t se, const uint8_t* src,
                                          uint8_t* lds, uint8_t* __restrict__ h_rx) {
    const uint32_t lane = threadIdx.x;
    const uint64_t sb16 = sb & ~15ull;
    uint64_t k_lo = 0;      // chunks rise, so the first live record never moves back
    uint64_t changed = 0;   // STAGE: bit i = this lane's i-th chunk changed (<= 33 per lane)
    uint32_t i = 0;
    if (STAGE && n <= SMALL_BY_RECORD) {
        // Record-major: the wave walks the records in order, every lane
        // XORing chunks of the current payload (a broadcast LDS read per
        // record instead of a per-chunk search).  A chunk two payloads share
        // is updated by both, in program order (one wave's LDS accesses do not
        // pass each other).  Every chunk is then stored back.
        for (uint64_t k = 0; k < n; ++k) {
            const drec f = rec(k);
            if (!(f.info & F_MASK) || f.pay_len == 0) continue;
            const uint32_t phase = (f.info >> 8) & 3u;
            const uint64_t pe = f.pay_off + f.pay_len;
            for (uint64_t c = (f.pay_off & ~15ull) + (uint64_t)lane * 16u; c < pe; c += 64u * 16u) {
                const uint32_t kw = rotr32(f.key, 8u * (uint32_t)((phase + c - f.pay_off) & 3u));
                const uint64_t kk = (uint64_t)kw | ((uint64_t)kw << 32);
                const int64_t a = (int64_t)(f.pay_off > c ? f.pay_off - c : 0);
                const int64_t e = (int64_t)(pe < c + 16 ? pe - c : 16);
                const uint64_t mlo = kk & byte_range(a, e), mhi = kk & byte_range(a - 8, e - 8);
                *reinterpret_cast<u32x4*>(lds + (c - sb16)) ^=
                    u32x4{(uint32_t)mlo, (uint32_t)(mlo >> 32), (uint32_t)mhi, (uint32_t)(mhi >> 32)};
            }
        }
        changed = ~0ull;
    } else
    for (uint64_t c = sb16 + (uint64_t)lane * 16u; c < se; c += 64u * 16u, ++i) {
        uint64_t k = k_lo, k_end = n;   // first record whose payload ends after c
        while (k < k_end) {
            const uint64_t mid = (k + k_end) >> 1;
            const drec m = rec(mid);
            if (m.pay_off + m.pay_len > c) k_end = mid;
            else k = mid + 1;
        }
        k_lo = k;
        uint64_t mlo = 0, mhi = 0;
        for (; k < n; ++k) {
            const drec f = rec(k);
            if (f.pay_off >= c + 16) break;
            if (!(f.info & F_MASK) || f.pay_len == 0) continue;
            const uint32_t phase = (f.info >> 8) & 3u;
            const uint32_t kw = rotr32(f.key, 8u * (uint32_t)((phase + c - f.pay_off) & 3u));
            const uint64_t kk = (uint64_t)kw | ((uint64_t)kw << 32);
            const int64_t a = (int64_t)(f.pay_off > c ? f.pay_off - c : 0);
            const uint64_t pe = f.pay_off + f.pay_len;
            const int64_t e = (int64_t)(pe < c + 16 ? pe - c : 16);
            mlo |= kk & byte_range(a, e);
            mhi |= kk & byte_range(a - 8, e - 8);
            if (e == 16) break;   // this payload runs past the chunk
        }
        if (!(mlo | mhi)) continue;   // no masked byte (or a zero key): bytes unchanged
        const u32x4 m4 = u32x4{(uint32_t)mlo, (uint32_t)(mlo >> 32), (uint32_t)mhi, (uint32_t)(mhi >> 32)};
        const bool whole = c >= sb && c + 16 <= se;
        if (STAGE) {
            changed |= 1ull << i;
            u32x4* p = reinterpret_cast<u32x4*>(lds + (c - sb16));
            if (whole) {
                *p ^= m4;
            } else {   // chunk shared with a neighbouring segment: own bytes only
                for (uint32_t b = 0; b < 16; ++b) {
                    const uint64_t x = c + b;
                    if (x >= sb && x < se) lds[x - sb16] ^= (uint8_t)((b < 8 ? mlo >> (8 * b) : mhi >> (8 * (b - 8))) & 0xFFu);
                }
            }
        } else if (whole) {
            u32x4 v = *reinterpret_cast<const u32x4*>(src + c);
            *reinterpret_cast<u32x4*>(h_rx + c) = v ^ m4;
        } else {
            for (uint32_t b = 0; b < 16; ++b) {
                const uint64_t x = c + b;
                const uint32_t kb = (uint32_t)((b < 8 ? mlo >> (8 * b) : mhi >> (8 * (b - 8))) & 0xFFu);
                if (x >= sb && x < se && kb) h_rx[x] = src[x] ^ (uint8_t)kb;
            }
        }
    }
    if (!STAGE) return;
    i = 0;
    for (uint64_t c = sb16 + (uint64_t)lane * 16u; c < se; c += 64u * 16u, ++i) {
        if (!((changed >> i) & 1u)) continue;
        if (c >= sb && c + 16 <= se) {
            *reinterpret_cast<u32x4*>(h_rx + c) = *reinterpret_cast<const u32x4*>(lds + (c - sb16));
        } else {
            for (uint32_t b = 0; b < 16; ++b) {
                const uint64_t x = c + b;
                if (x >= sb && x < se) h_rx[x] = lds[x - sb16];
            }
        }
    }
}

template <bool STAGE>
__global__ __launch_bounds__(64) void k_small(const uint8_t* __restrict__ rx, uint64_t rx_len,
                                              const dseg* __restrict__ segs, const dcarry* __restrict__ carry_in,
                                              const uint64_t* __restrict__ slot_base, drec* __restrict__ slots,
                                              unsigned long long* __restrict__ rec_total, drec* __restrict__ h_rec,
                                              uint64_t h_rec_cap, dsmall_out* __restrict__ h_out,
                                              uint8_t* __restrict__ h_rx, int unmask, uint32_t vmask,
                                              uint64_t rec_base, uint64_t* __restrict__ h_done, uint64_t seq) {
    extern __shared__ u32x4 lds_seg[];
    __shared__ drec lrec[SMALL_LREC];
    const uint32_t s = blockIdx.x;
    const uint32_t lane = threadIdx.x;
    // independent loads, one round trip
    const dseg sg = segs[s];
    dcarry st = carry_in[s];
    drec* slot = slots + slot_base[s];
    const uint64_t sb = sg.off, L = sg.len, se = sb + L;

    const uint8_t* src = rx;
    uint64_t src_len = rx_len;
    uint8_t* lds = reinterpret_cast<uint8_t*>(lds_seg);
    const uint64_t sb16 = sb & ~15ull;
    if (STAGE) {
        // Whole 16-byte chunks: SB independent loads per lane in flight, then
        // their LDS stores (a load -> store -> load chain would pay the full
        // memory latency per chunk: ~1.5 us each across PCIe).
        constexpr int SB = 8;
        for (uint64_t c0 = sb16 + (uint64_t)lane * 16u; c0 < se; c0 += 64u * 16u * SB) {
            u32x4 v[SB];
#pragma unroll
            for (int u = 0; u < SB; ++u) {
                const uint64_t c = c0 + (uint64_t)u * 1024u;
                v[u] = c >= sb && c + 16 <= se ? *reinterpret_cast<const u32x4*>(rx + c) : u32x4{0u, 0u, 0u, 0u};
            }
#pragma unroll
            for (int u = 0; u < SB; ++u) {
                const uint64_t c = c0 + (uint64_t)u * 1024u;
                if (c >= sb && c + 16 <= se) *reinterpret_cast<u32x4*>(lds + (c - sb16)) = v[u];
            }
        }
        // The (at most two) chunks the segment shares with a neighbour: lane 0
        // the first, lane 1 the last, their bytes loaded together.
        const uint64_t c_last = (se - 1) & ~15ull;
        const uint64_t ce = lane == 0 ? sb16 : c_last;
        const bool partial = L && lane < 2 && (lane == 0 || c_last != sb16) && (ce < sb || ce + 16 > se);
        if (partial) {
            uint8_t b16[16];
#pragma unroll
            for (int b = 0; b < 16; ++b) b16[b] = ce + b >= sb && ce + b < se ? rx[ce + b] : 0;
#pragma unroll
            for (int b = 0; b < 16; ++b)
                if (ce + b >= sb && ce + b < se) lds[ce + b - sb16] = b16[b];
        }
        __syncthreads();
        src = lds - sb16;
        src_len = se;
    }

    st.started = 0;
    uint64_t pos = 0, n = 0;
    auto emit = [&](uint64_t idx, const frec& v) {
        drec o;
        o.hdr_off = v.hdr_off < 0 ? -1 : (int64_t)(sb + (uint64_t)v.hdr_off);
        o.pay_off = sb + v.pay_off;
        o.pay_len = v.pay_len;
        o.length = v.length;
        o.key = v.key;
        o.info = v.info;
        if (idx < SMALL_LREC) lrec[idx] = o;
        else slot[idx] = o;
    };
    if (st.state != S_START) {
        frec r;
        if (scalar_frame(src + sb, L, st, pos, r, vmask)) {
            if (lane == 0) emit(0, r);
            n = 1;
        }
    }
    walk_frames<true>(src, src_len, sb, L, st, pos, n, vmask, emit);
    __threadfence_block();
    __syncthreads();

    // The record base first: a returning global atomic issued after the
    // host stores below would wait for all of them to complete (vmcnt counts
    // loads and stores in order on CDNA).
    uint64_t base = 0;
    if (lane == 0 && n) base = atomicAdd(rec_total, (unsigned long long)n) - rec_base;

    if (unmask && n) {
        if (n <= SMALL_LREC) {
            small_xor<STAGE>([&](uint64_t i) { return lrec[i]; }, n, sb, se, src, lds, h_rx);
        } else {   // > SMALL_LREC records (frames of a few bytes): all of them in the device slot
            for (uint64_t i = lane; i < SMALL_LREC; i += 64) slot[i] = lrec[i];
            __threadfence_block();
            __syncthreads();
            small_xor<STAGE>([&](uint64_t i) { return slot[i]; }, n, sb, se, src, lds, h_rx);
        }
    }

    base = __shfl(base, 0);
    const uint64_t nl = n < SMALL_LREC ? n : SMALL_LREC;
    if (base + n <= h_rec_cap) {
        for (uint64_t i = lane; i < nl; i += 64) h_rec[base + i] = lrec[i];
        for (uint64_t i = SMALL_LREC + lane; i < n; i += 64) h_rec[base + i] = slot[i];
    } else if (!(unmask && n > SMALL_LREC)) {
        // Past the pinned record area: the host reads this segment from its
        // device slot, so the slot must hold every record (the XOR path above
        // copied the LDS ones only when it needed them).
        for (uint64_t i = lane; i < nl; i += 64) slot[i] = lrec[i];
    }
    if (lane == 0) {
        dsmall_out o;
        o.first = base;
        o.count = n;
        o.st = st;
        h_out[s] = o;
    }
    if (h_done) {
        // Completion word the host polls instead of synchronising the stream:
        // every store of this wave above (bytes, records, h_out) is released
        // to system scope first, so seeing `seq` means seeing all of them.
        __threadfence_system();
        if (lane == 0) __hip_atomic_store(h_done + s, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

hipError_t launch_small(const uint8_t* rx, uint64_t rx_len, const dseg* segs, const dcarry* carry_in, uint32_t nseg,
                        const uint64_t* slot_base, drec* slots, unsigned long long* rec_total, uint64_t rec_base,
                        drec* h_rec, uint64_t h_rec_cap, dsmall_out* h_out, uint8_t* h_rx, int unmask, uint32_t vmask,
                        uint32_t stage_lds, uint64_t* h_done, uint64_t seq, hipStream_t st, hipEvent_t ev_start,
                        hipEvent_t ev_stop) {
    if (nseg == 0) return hipSuccess;
    // Timing events, when asked for, ride on the dispatch itself (no marker
    // packets); without them the plain launch is cheaper still.
    const bool ev = ev_start || ev_stop;
    if (stage_lds && ev)
        hipExtLaunchKernelGGL(k_small<true>, dim3(nseg), dim3(64), stage_lds, st, ev_start, ev_stop, 0u, rx, rx_len,
                              segs, carry_in, slot_base, slots, rec_total, h_rec, h_rec_cap, h_out, h_rx, unmask, vmask,
                              rec_base, h_done, seq);
    else if (stage_lds)
        hipLaunchKernelGGL(k_small<true>, dim3(nseg), dim3(64), stage_lds, st, rx, rx_len, segs, carry_in, slot_base,
                           slots, rec_total, h_rec, h_rec_cap, h_out, h_rx, unmask, vmask, rec_base, h_done, seq);
    else if (ev)
        hipExtLaunchKernelGGL(k_small<false>, dim3(nseg), dim3(64), 0, st, ev_start, ev_stop, 0u, rx, rx_len, segs,
                              carry_in, slot_base, slots, rec_total, h_rec, h_rec_cap, h_out, h_rx, unmask, vmask,
                              rec_base, h_done, seq);
    else
        hipLaunchKernelGGL(k_small<false>, dim3(nseg), dim3(64), 0, st, rx, rx_len, segs, carry_in, slot_base, slots,
                           rec_total, h_rec, h_rec_cap, h_out, h_rx, unmask, vmask, rec_base, h_done, seq);
    return hipGetLastError();
}

// ------------------------------------------------------------------ k_door
//
// The resident small-path worker (ddoor, hvws_internal.h): one workgroup of
// kDoorThreads threads (8 waves) that stays on the device between
// reference-API calls.  Wave 0 polls the mailbox's 128-byte request block
// (one system-scope load, then s_sleep -- no fence per poll); on a new read
// every wave stages the request's bytes into LDS (all loads in flight at
// once) while wave 0 runs a carried-in payload (it needs none of them); then
// wave 0 walks the headers and the cut frame (door_walk) while the last wave
// unmasks the carried-in payload, the waves XOR the other records (8 waves:
// at most one each of an 8 KiB read's 8 others) beside the records' copy to
// host memory, and store every chunk to the mailbox's data area; thread 0 writes the L2 back once every
// thread's stores are in it, and publishes `done`.  A request costs no
// launch, no dispatch and no end-of-kernel signal.  Parking: idle for
// idle_ticks of the 100 MHz realtime clock, the worker clears `alive`, takes
// one last look at `seq` (serving a request that arrived meanwhile) and
// exits; its last store is `exited = epoch`, and the host relaunches it on the
// next request once it has seen that word.
// The worker's header walk over a read staged in LDS.  A single wave walking
// headers one after the other is a chain of dependent instructions (~8
// cycles each): round 3's walks spent ~4.5 us on the 8 headers of an 8 KiB
// read (profiles/r4c_raw).  So the wave takes a run of equal-size frames per
// round: lane j parses the header at q + j * stride in full and emits its
// record if the frames from q up to it are whole and of that size; the first
// lane off the run gives the next round's stride, or it holds the frame cut
// by the read's end, whose record and S_BODY carry follow from its header
// bytes (the exact state machine only when that header itself is cut).
// Records and the carried fields (Q14) as walk_frames leaves them.  (Until
// round 6 a round sized the frames first, wrote their positions to LDS and
// parsed them in a second pass, and the cut frame's header was loaded and
// parsed once more: chase 0.56 + parse 0.48 + tail 0.52 us per 8 KiB read.)

// 16 bytes at LDS byte q (dword-aligned loads, v_alignbyte realigns)
__device__ __forceinline__ void lds_hdr16(const uint32_t* l, uint32_t q, uint64_t& lo, uint64_t& hi) {
    const uint32_t w = q >> 2, r = q & 3u;
    const uint32_t d0 = l[w], d1 = l[w + 1], d2 = l[w + 2], d3 = l[w + 3], d4 = l[w + 4];
    const uint32_t c0 = __builtin_amdgcn_alignbyte(d1, d0, r), c1 = __builtin_amdgcn_alignbyte(d2, d1, r);
    const uint32_t c2 = __builtin_amdgcn_alignbyte(d3, d2, r), c3 = __builtin_amdgcn_alignbyte(d4, d3, r);
    lo = (uint64_t)c0 | ((uint64_t)c1 << 32);
    hi = (uint64_t)c2 | ((uint64_t)c3 << 32);
}

// Header length and payload length of the frame at LDS byte q (32-bit; a
// 64-bit length past 2^32 - 1 clamps, which no whole frame of a read has).
__device__ __forceinline__ void door_size(const uint32_t* l, uint32_t q, uint32_t& hl, uint32_t& len) {
    const uint32_t w = q >> 2, r = q & 3u;
    const uint32_t d0 = l[w], d1 = l[w + 1];
    const uint32_t b0 = __builtin_amdgcn_alignbyte(d1, d0, r);   // bytes q .. q+3
    const uint32_t len7 = (b0 >> 8) & 0x7Fu, m4 = (b0 >> 13) & 4u;   // bit 7 of byte 1 -> 4 key bytes
    if (len7 < 126) {
        hl = 2u + m4;
        len = len7;
    } else if (len7 == 126) {
        hl = 4u + m4;
        len = ((b0 >> 8) & 0xFF00u) | (b0 >> 24);
    } else {
        const uint32_t d2 = l[w + 2], d3 = l[w + 3];
        const uint32_t b1 = __builtin_amdgcn_alignbyte(d2, d1, r), b2 = __builtin_amdgcn_alignbyte(d3, d2, r);
        const uint64_t be = (uint64_t)(b0 >> 16) | ((uint64_t)b1 << 16) | ((uint64_t)(b2 & 0xFFFFu) << 48);
        const uint64_t len64 = __builtin_bswap64(be);
        hl = 10u + m4;
        len = len64 > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)len64;
    }
}

// k_door's flags (door_flags reads them from the environment once)
constexpr uint32_t DOOR_F_STAMPS = 8u;   // realtime stamps per phase (door_stamps; scripts/probe/door_phases.py)
// DOOR_XOR (a masked websocket_build_frame payload, websocket_decode) runs in
// registers, its result written through the L2 (sc0 sc1), and `done` after
// those stores' acks: no LDS staging, no barrier between the two, no L2
// writeback.  A masked 125 B build: 3.41-3.46 us per call against 4.49-4.90
// staged in LDS (profiles/r5_raw/door, r5x2).  (For a read's ~500 result
// stores the same trade lost: 13-14 us per call.)  Round 5's other worker
// variants -- walk_frames instead of door_walk, non-temporal staging loads,
// the data preload -- lost and were removed in round 6.

// A phase stamp (DOOR_F_STAMPS): each realtime-clock read is a scalar
// memory round trip that the wave waits for, so stamps are off by default.
__device__ __forceinline__ uint64_t door_now(uint32_t flags) {
    return (flags & DOOR_F_STAMPS) ? (uint64_t)wall_clock64() : 0ull;
}

// Chunks [0, c_hi) of the data area (a multiple of 64) into LDS at the same
// offsets by LDS-DMA: no registers (an array of 16-byte values per thread
// cost the worker ~1000 register moves, ~2 us per read); a wave writes 64
// consecutive chunks per instruction (lane-linear destination).  The caller
// waits for vmcnt(0) before a barrier.
__device__ __forceinline__ void door_stage(const uint8_t* din, uint8_t* lds, uint32_t c_hi) {
    const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63u;
    for (uint32_t cb = wave * 64u; cb < c_hi; cb += kDoorThreads) {
        const auto* g = (const __attribute__((address_space(1))) void*)(din + (uint64_t)(cb + lane) * 16u);
        auto* l = (__attribute__((address_space(3))) void*)(lds + (uint64_t)cb * 16u);
        __builtin_amdgcn_global_load_lds(g, l, 16, 0, 0);
    }
}

// 16 bytes at system scope (the poll's view of the request block)
__device__ __forceinline__ u32x4 ld16_sys(const void* p) {
    u32x4 v;
    asm volatile("global_load_dwordx4 %0, %1, off sc0 sc1\n\ts_waitcnt vmcnt(0)" : "=v"(v) : "v"(p) : "memory");
    return v;
}

// readlane of a 64-bit value (wave-uniform lane index)
__device__ __forceinline__ uint64_t readlane64(uint64_t v, int src) {
    return (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, src) |
           ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), src) << 32);
}

template <bool V, typename Emit>
__device__ __forceinline__ void door_walk(const uint8_t* lds, uint64_t L, dcarry& st, uint64_t& pos, uint64_t& n,
                                          uint32_t vmask, uint64_t* stamps, Emit&& emit) {
    const uint32_t* l = reinterpret_cast<const uint32_t*>(lds);
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t Lw = (uint32_t)L;   // reads are <= kDoorMax
    uint32_t q = (uint32_t)pos, nn = (uint32_t)n;
    bool cut = false;
    uint64_t clo = 0, chi = 0;   // the cut frame's first 16 bytes (its header is whole)
    if (st.state == S_START && q + 2 <= Lw) {
        // the stride of the frame at q (0: that frame is cut by the read's end)
        uint32_t stride;
        {
            uint32_t hl, len;
            door_size(l, q, hl, len);
            const uint32_t rq = Lw - q;
            stride = (hl <= rq && len <= rq - hl) ? hl + len : 0u;
        }
        bool first = true;
        for (;;) {
            // lane j parses the header at q + j * stride in full; the run of
            // whole frames of that size from lane 0 are this round's records,
            // and the first lane off the run is the next round's start (its
            // size the next stride) or the frame cut by the read's end
            const uint32_t p = q + lane * stride;   // < 64 * 2^16: no overflow
            const bool inb = lane == 0 || (stride != 0 && p + 2 <= Lw);
            const uint32_t pp = inb ? p : q;
            uint64_t lo, hi;
            lds_hdr16(l, pp, lo, hi);
            const hdr h = parse_hdr<V>(lo, hi);
            const uint32_t rj = Lw - pp;
            const bool whole = inb && h.hlen <= rj && h.length <= (uint64_t)(rj - h.hlen);
            const uint32_t size = h.hlen + (uint32_t)h.length;   // whole: <= rj
            const bool ok = whole && size == stride;
            const unsigned long long bad = __ballot(!ok);
            const uint32_t f = bad ? (uint32_t)__ffsll((long long)bad) - 1u : 64u;
            if (lane < f) {
                frec v;
                whole_frame_rec(v, p, h, vmask);
                emit(nn + lane, v);
            }
            if (f) {   // the carried fields (Q14): the run's last frame and last masked frame
                const int last = (int)f - 1;
                st.flags = (uint32_t)__builtin_amdgcn_readlane((int)h.flags, last);
                st.length = readlane64(h.length, last);
                st.require = 0;
                st.offset = 0;
                st.mask_offset = (st.flags & F_MASK) ? (uint32_t)(st.length & 3u) : 0u;
                st.started = 0;
                const unsigned long long mm = __ballot(lane < f && (h.flags & F_MASK)) ;
                if (mm) st.mask = (uint32_t)__builtin_amdgcn_readlane((int)h.key, 63 - __clzll((long long)mm));
            }
            nn += f;
            q += f * stride;
            if (stamps && first && threadIdx.x == 0) stamps[0] = wall_clock64();
            first = false;
            if (f == 64u) {   // the same stride again
                if (q + 2 > Lw) break;
                continue;
            }
            // lane f: a whole frame of another size, or the read's cut frame
            if ((__ballot(whole) >> f) & 1ull) {
                stride = (uint32_t)__builtin_amdgcn_readlane((int)size, (int)f);
                continue;
            }
            // lane f's frame is cut; with at least 2 bytes of it here lane f
            // parsed its header
            if (q + 2 <= Lw) {
                clo = readlane64(lo, (int)f);
                chi = readlane64(hi, (int)f);
                cut = true;
            }
            break;
        }
    }
    if (threadIdx.x == 0 && stamps) stamps[1] = wall_clock64();
    n = nn;
    pos = q;
    if (cut) {
        // The common cut: the header is whole, the payload runs past the
        // read.  What scalar_frame leaves behind, in one step: a record with
        // the payload bytes here, S_BODY with the rest to come.  (Wave-uniform
        // values: lane f's header bytes.)
        const uint32_t rq = Lw - q;
        const hdr h = parse_hdr(clo, chi);
        if (h.hlen <= rq) {
            const uint32_t nb = rq - h.hlen;   // < h.length: the frame is cut
            frec r;
            r.hdr_off = (int64_t)q;
            r.pay_off = q + h.hlen;
            r.pay_len = nb;
            r.length = h.length;
            r.key = (h.flags & F_MASK) ? h.key : 0u;
            r.info = I_START | (h.flags & 0xFFu) | I_HDR | invalid_bits(h.viol, vmask) | (nb ? I_BODY : 0u);
            const uint32_t len7 = (uint32_t)(clo >> 8) & 0x7Fu;
            st.state = S_BODY;
            st.flags = h.flags;
            st.length = h.length;
            if (h.flags & F_MASK) st.mask = h.key;
            st.mask_offset = (h.flags & F_MASK) ? (nb & 3u) : 0u;
            st.require = h.length - nb;
            st.offset = nb;
            st.started = 1;
            st.viol = h.viol | ((len7 == 127 ? 2u : (len7 == 126 ? 1u : 0u)) << V_ENC_SHIFT);
            if (lane == 0) emit(n, r);
            ++n;
            pos = L;
        }
    }
    if (st.state == S_START && pos < L) {   // the header itself is cut: the exact state machine
        frec r;
        if (scalar_frame(lds, L, st, pos, r, vmask)) {
            if (lane == 0) emit(n, r);
            ++n;
        }
    }
    if (threadIdx.x == 0 && stamps) stamps[2] = wall_clock64();
}

__global__ __launch_bounds__(kDoorThreads) void k_door(const ddoor* __restrict__ req, ddoor* __restrict__ box,
                                                       const uint8_t* __restrict__ din, uint8_t* __restrict__ dout,
                                                       drec* __restrict__ h_rec, drec* __restrict__ d_slot,
                                                       uint64_t idle_ticks, uint64_t first_seq, uint64_t epoch,
                                                       uint32_t flags) {
    extern __shared__ u32x4 lds_door[];
    __shared__ drec lrec[SMALL_LREC];
    __shared__ uint64_t s_seq, s_len, s_n;
    __shared__ uint32_t s_op, s_unmask, s_vmask, s_key, s_phase, s_exit;
    __shared__ dcarry s_carry;
    const uint32_t tid = threadIdx.x;
    uint8_t* lds = reinterpret_cast<uint8_t*>(lds_door);
    uint64_t last = first_seq;
    uint64_t served = 0;
    __shared__ uint64_t s_t[7];
    uint64_t rel_prev = 0;   // thread 0: realtime ticks of the previous request's release
    __shared__ uint64_t s_req[16];
    __shared__ uint64_t s_w[3];               // door_walk's stamps
    __shared__ uint32_t s_c0;                 // record 0 is the carried-in payload (made while staging)
    for (;;) {
        if (tid < 64) {
            // Wave 0 polls the whole 128-byte request block, lanes 0-7 16
            // bytes each: a new request's fields arrive with its seq, so no
            // second round trip for them.  The host writes seq_tail with the
            // fields and seq after them; a block read straddling those writes
            // shows the two copies differing and is read again.
            const uint32_t lane = tid;
            uint64_t t0 = wall_clock64();
            uint64_t s = last;
            uint32_t ex = 0, polls = 0;
            u32x4 piece = u32x4{0u, 0u, 0u, 0u};
            for (;;) {
                if (lane < 8) piece = ld16_sys(reinterpret_cast<const u32x4*>(req) + lane);
                const uint64_t head = (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)piece[0], 0) |
                                      ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)piece[1], 0) << 32);
                bool torn = false;   // read again at once
                if (head != last) {
                    const uint64_t tail = (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)piece[2], 7) |
                                          ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)piece[3], 7) << 32);
                    if (tail == head) {
                        s = head;
                        break;
                    }
                    torn = true;
                }
                // the clock every 32 polls: each read is a round trip the poll would wait for
                if ((++polls & 31u) == 0 && wall_clock64() - t0 > idle_ticks) {
                    if (lane == 0) {
                        __hip_atomic_store(&box->alive, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                        __threadfence_system();
                    }
                    const uint64_t again = __hip_atomic_load(&req->seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                    const uint32_t a_lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)again);
                    const uint32_t a_hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(again >> 32));
                    if ((((uint64_t)a_hi << 32) | a_lo) == last) {
                        ex = 1;
                        break;
                    }
                    // arrived while parking: serve it (read and checked at the loop's top)
                    if (lane == 0) __hip_atomic_store(&box->alive, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                    torn = true;
                }
                if (!torn) __builtin_amdgcn_s_sleep(2);
            }
            if (lane < 8) reinterpret_cast<u32x4*>(s_req)[lane] = piece;
            if (lane == 0) {
                s_exit = ex;
                s_seq = s;
                s_t[0] = door_now(flags);
                // The acquire invalidates this CU's L1 and the L2 for the
                // request's bytes loaded next.
                if (!ex) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
            }
        }
        __syncthreads();
        if (s_exit) {   // parked (idle): `alive` is already 0; say this launch has ended
            if (tid == 0) __hip_atomic_store(&box->exited, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            return;
        }
        if (tid == 0) {
            const uint64_t* q = s_req + 1;   // word 0 is seq
            s_op = (uint32_t)q[0];
            s_unmask = (uint32_t)(q[0] >> 32);
            s_len = q[1] < kDoorMax ? q[1] : kDoorMax;
            s_vmask = (uint32_t)q[2];
            s_key = (uint32_t)(q[2] >> 32);
            s_phase = (uint32_t)q[3];
            s_c0 = 0;
            dcarry cin;
            memcpy(&cin, &q[4], sizeof(dcarry));
            s_carry = cin;
            s_t[5] = door_now(flags);
        }
        __syncthreads();
        const uint64_t seq = s_seq;
        const uint32_t op = s_op;
        if (op == DOOR_EXIT) {
            if (tid == 0) {
                __hip_atomic_store(&box->alive, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                __threadfence_system();
                __hip_atomic_store(&box->done, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                __threadfence_system();
                __hip_atomic_store(&box->exited, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            }
            return;
        }
        const uint64_t L = s_len;
        const uint64_t nch = (L + 15u) / 16u;   // the data area has slack past L: whole chunks throughout
        const uint32_t ngr = (uint32_t)((nch + 63u) & ~63ull);   // whole wave groups of 64 chunks (<= kDoorMax)
        const bool xdirect = op == DOOR_XOR;
        dcarry st;                   // wave 0: the carry through a read
        uint64_t pos = 0, n = 0;     // wave 0: position in the read, records so far
        bool carried = false;        // wave 0: the carried-in payload is done
        const uint32_t vmask = s_vmask;
        auto emit = [&](uint64_t idx, const frec& v) {
            drec o;
            o.hdr_off = v.hdr_off;
            o.pay_off = v.pay_off;
            o.pay_len = v.pay_len;
            o.length = v.length;
            o.key = v.key;
            o.info = v.info;
            if (idx < SMALL_LREC) lrec[idx] = o;
            else d_slot[idx] = o;
        };
        if (xdirect) {
            const uint32_t kw = rotr32(s_key, 8u * (s_phase & 3u));
            const u32x4 k4 = u32x4{kw, kw, kw, kw};
            for (uint64_t c = tid; c < nch; c += kDoorThreads) {
                const u32x4 v = *reinterpret_cast<const u32x4*>(din + c * 16u) ^ k4;
                asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1" ::"v"(dout + c * 16u), "v"(v) : "memory");
            }
        } else {
            // the data area into LDS (all in flight)
            door_stage(din, lds, ngr);
            // wave 0: the common carry, a payload that continues into this
            // read, needs none of the staged bytes -- it runs while they land
            // (scalar_frame's S_BODY step without its state dispatch)
            if (tid < 64) {
                st = s_carry;
                st.started = 0;
                if (st.state == S_BODY && st.require > 0 && L > 0) {
                    const uint64_t nb = st.require < L ? st.require : L;
                    frec r;
                    r.hdr_off = -1;
                    r.pay_off = 0;
                    r.pay_len = nb;
                    r.length = st.length;
                    r.key = (st.flags & F_MASK) ? st.mask : 0u;
                    r.info = (st.flags & 0xFFu) | ((st.mask_offset & 3u) << 8) | I_BODY;
                    if (st.flags & F_MASK) st.mask_offset = (uint32_t)((st.mask_offset + nb) & 3u);
                    st.require -= nb;
                    pos = nb;
                    if (st.require == 0) {
                        st.state = S_START;
                        r.info |= I_END;
                    } else {
                        st.offset += L;   // http/websocket_parser.c:153
                    }
                    if (tid == 0) {
                        emit(0, r);
                        s_c0 = 1;
                    }
                    n = 1;
                    carried = true;
                }
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        if (!xdirect) {
            __syncthreads();
            if (tid == 0) s_t[1] = door_now(flags);
            uint32_t* l32 = reinterpret_cast<uint32_t*>(lds);
            const uint32_t wave = tid >> 6, lane = tid & 63u;
            auto unmask_rec = [&](const drec& f) {
                // 32-bit: offsets inside one read.  Chunks start at
                // multiples of 16, so one key word serves every chunk.
                const uint32_t po = (uint32_t)f.pay_off, pl = (uint32_t)f.pay_len, info = f.info;
                if (!(info & F_MASK) || pl == 0) return;
                const uint32_t pe = po + pl;
                const uint32_t kw = rotr32(f.key, 8u * ((((info >> 8) & 3u) - po) & 3u));
                const uint32_t cf = (po + 15u) & ~15u, cl = pe & ~15u;   // whole chunks [cf, cl)
                for (uint32_t c = cf + lane * 16u; c < cl; c += 64u * 16u) {
                    u32x4* q = reinterpret_cast<u32x4*>(lds + c);
                    *q = *q ^ u32x4{kw, kw, kw, kw};
                }
                // the partial chunks at either end (they may hold another
                // record's bytes), a dword per lane: lanes 0-3 the first
                // chunk, lanes 4-7 the last (one atomic step, not four)
                const uint32_t c0 = po & ~15u;
                const bool head = (po & 15u) != 0, tail = (pe & 15u) != 0 && cl >= cf;
                const bool hl = lane < 4u;
                if ((hl && head) || (lane - 4u < 4u && tail)) {
                    const uint32_t cc = hl ? c0 : cl;
                    const int32_t a = hl ? (int32_t)(po - c0) : 0;
                    const int32_t e = (hl && cl < cf) ? (int32_t)(pe - c0) : (hl ? 16 : (int32_t)(pe - cl));
                    const int32_t d4 = 4 * (int32_t)(lane & 3u);
                    const int32_t lo = a - d4 < 0 ? 0 : (a - d4), hi = e - d4 > 4 ? 4 : (e - d4);
                    if (hi > lo) {
                        const uint32_t m = (hi >= 4 ? ~0u : ((1u << (8 * hi)) - 1u)) & ~((1u << (8 * lo)) - 1u);
                        atomicXor(l32 + cc / 4u + (lane & 3u), kw & m);
                    }
                }
            };
            if (tid < 64) {   // wave 0: the rest of a carried-in frame, walk, tail (k_small's code)
                if (!carried && st.state != S_START) {
                    frec r;
                    if (scalar_frame(lds, L, st, pos, r, vmask)) {
                        if (tid == 0) emit(0, r);
                        n = 1;
                    }
                }
                if (tid == 0) s_t[4] = door_now(flags);
                uint64_t* const ws = (flags & DOOR_F_STAMPS) ? s_w : nullptr;
                if (vmask) door_walk<true>(lds, L, st, pos, n, vmask, ws, emit);
                else door_walk<false>(lds, L, st, pos, n, vmask, ws, emit);
                if (tid == 0) {
                    s_n = n;
                    s_carry = st;
                }
            } else if (tid >= kDoorThreads - 64u && s_c0 && s_unmask) {
                // the last wave unmasks the carried-in payload while wave 0
                // walks (wave 0 reads header bytes only, none of that
                // payload's): the waves then share the other records, at
                // most one each for an 8 KiB read of 1 KiB frames
                unmask_rec(lrec[0]);
            }
            __threadfence_block();
            __syncthreads();
            if (tid == 0) s_t[2] = door_now(flags);
            const uint64_t n = s_n;
            // records [0, nl) sit in LDS, the rest in d_slot: separate loops,
            // so LDS records are read with ds loads (a select between the two
            // pointers compiled to flat loads waiting on both counters)
            const uint64_t nl = n < SMALL_LREC ? n : SMALL_LREC;
            // Unmask in LDS record by record (waves take records in turn, a
            // wave's lanes a record's 16-byte chunks): no per-chunk search of
            // the records.  A chunk inside one payload belongs to that record
            // alone (plain read-modify-write); a payload's first and last
            // chunks may hold another record's bytes too (LDS atomic XOR per
            // dword).  Then every chunk of the read goes to dout.  (Round 6
            // tried chunk-major instead -- a binary search of the records'
            // payload ends per chunk, the chunk XORed and stored straight to
            // dout: 1.52 against 1.08 us for an 8 KiB read, profiles/r6_raw/door.)
            // the records to host memory first: their stores run beside the XOR
            for (uint64_t i = tid; i < nl; i += kDoorThreads) h_rec[i] = lrec[i];
            for (uint64_t i = nl + tid; i < n; i += kDoorThreads) h_rec[i] = d_slot[i];
            if (s_unmask) {
                for (uint64_t k = s_c0 + wave; k < nl; k += kDoorThreads / 64u) unmask_rec(lrec[k]);
                for (uint64_t k = nl + wave; k < n; k += kDoorThreads / 64u) unmask_rec(d_slot[k]);
                __syncthreads();
                if (tid == 0) s_t[6] = door_now(flags);
                for (uint64_t c = (uint64_t)tid * 16u; c < L; c += (uint64_t)kDoorThreads * 16u)
                    *reinterpret_cast<u32x4*>(dout + c) = *reinterpret_cast<const u32x4*>(lds + c);
            } else if (tid == 0) {
                s_t[6] = s_t[2];
            }
            if (tid == 0) s_t[3] = door_now(flags);
            if (tid == 0) {
                box->count = n;
                box->out = s_carry;
                box->served = ++served;
                if (flags & DOOR_F_STAMPS) {
                    box->stamp[0] = s_t[0];
                    box->stamp[1] = s_t[1];
                    box->stamp[2] = s_t[2];
                    box->stamp[3] = s_t[3];
                    box->stamp[4] = wall_clock64();
                    box->stamp[5] = s_t[5];
                    box->stamp[6] = rel_prev;   // the previous request's release (its fence and barrier)
                    box->stamp[7] = s_t[4];     // carried-in frame done, the walk starts
                    box->stamp[8] = s_w[0];
                    box->stamp[9] = s_w[1];
                    box->stamp[10] = s_w[2];
                    box->stamp[11] = s_t[6];    // the XOR's barrier: stores to dout start
                }
            }
        }
        // Every thread's stores reach host memory before `done` says so: each
        // thread waits for its stores' L2 acknowledgements, the barrier orders
        // them before thread 0, and thread 0's one system-scope release writes
        // the L2 back (an L2-wide writeback: every wave's lines).  A release in
        // every thread meant four writebacks: 1.14 us against 0.49 for one
        // (scripts/probe/lat_probe.hip).  DOOR_XOR's results were written
        // through the L2: their acknowledgements suffice.
        const uint64_t tr = tid == 0 ? door_now(flags) : 0;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0) {
            if (!xdirect) {
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
                // the writeback's completion before `done`: the compiler
                // drops the fence's own wait after the barrier's
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
            rel_prev = door_now(flags) - tr;
            __hip_atomic_store(&box->done, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        last = seq;
    }
}

// k_door's flags ($HVWS_EXPERIMENT door_stamps: the worker's phase stamps,
// scripts/probe/door_phases.py)
uint32_t door_flags() {
    static const uint32_t flags = experiment("door_stamps") && atoi(experiment("door_stamps")) ? DOOR_F_STAMPS : 0u;
    return flags;
}

// A device symbol of this code object: its address names the executable the
// HIP runtime loaded for the device, in which the worker queue finds k_door
// (hvws_doorq.cpp); asking for it loads the code object.
__device__ uint32_t g_door_anchor;
hipError_t door_anchor(void** dev_addr) { return hipGetSymbolAddress(dev_addr, HIP_SYMBOL(g_door_anchor)); }
const char* door_kernel_symbol_prefix() { return "_ZN4hvws6k_doorE"; }

// ------------------------------------------------------------- k_offsets
// Exclusive scan of counts[0..nseg) into bases[], total into *total.  One
// block of 1024 threads; each thread owns a contiguous run.
template <uint32_t NT>
__device__ __forceinline__ void offsets_body(const uint64_t* __restrict__ counts, uint64_t* __restrict__ bases,
                                             uint32_t nseg, uint64_t* __restrict__ total) {
    __shared__ uint64_t part[NT];
    const uint32_t t = threadIdx.x;
    const uint32_t per = (nseg + NT - 1u) / NT;
    const uint32_t b = t * per;
    const uint32_t e = min(nseg, b + per);
    uint64_t sum = 0;
    for (uint32_t i = b; i < e; ++i) sum += counts[i];
    part[t] = sum;
    __syncthreads();
    for (uint32_t d = 1; d < NT; d <<= 1) {
        uint64_t v = t >= d ? part[t - d] : 0;
        __syncthreads();
        part[t] += v;
        __syncthreads();
    }
    uint64_t run = part[t] - sum;
    for (uint32_t i = b; i < e; ++i) {
        bases[i] = run;
        run += counts[i];
    }
    if (t == NT - 1u) *total = part[NT - 1u];
}

// Single-block kernels of the scan chains run as 256-thread workgroups: a
// 1024-thread one (16 waves on one CU) waited tens of us for slots beside a
// pipelined unmask (k_offsets 6 -> 66 us in profiles/r2h_raw/c2_trace.csv).
constexpr uint32_t ONE_BLOCK = 256;

__global__ __launch_bounds__(ONE_BLOCK) void k_offsets(const uint64_t* __restrict__ counts,
                                                       uint64_t* __restrict__ bases, uint32_t nseg,
                                                       uint64_t* __restrict__ total) {
    offsets_body<ONE_BLOCK>(counts, bases, nseg, total);
}

// ----------------------------------------------------------- k_spec_check
// Compare the true per-segment record counts with k_head's estimates (one
// block).  SPEC: the table was emitted at the estimates' offsets, so it is
// exact iff every count matches and the records fit the table; then *total
// = the record count, else 0 (everything downstream becomes a no-op and the
// host re-scans exactly).  COUNT (observe only): report whether the
// estimates would have held, leave *total alone.  Results go to pinned host
// memory (status), tagged with the scan's sequence number.
template <bool SPEC, uint32_t NT>
__device__ __forceinline__ void spec_check_body(const uint64_t* __restrict__ counts,
                                                     const uint64_t* __restrict__ est,
                                                     const uint64_t* __restrict__ npred, uint32_t nseg,
                                                     uint64_t* __restrict__ total, uint64_t cap,
                                                     dspec_status* __restrict__ status, uint64_t seq,
                                                     bool publish) {
    __shared__ uint64_t s_sum[NT / 64], s_max[NT / 64];
    __shared__ uint32_t s_bad[NT / 64];
    const uint32_t t = threadIdx.x;
    uint64_t sum = 0, mx = 0;
    uint32_t bad = 0;
    for (uint32_t i = t; i < nseg; i += NT) {
        const uint64_t c = counts[i];
        sum += c;
        mx = c > mx ? c : mx;
        bad |= c != est[i];
        if (npred && npred[i]) bad |= 2u;   // a long uniform run (the next scan keeps k_verify)
    }
    for (int o = 32; o > 0; o >>= 1) {
        sum += __shfl_xor(sum, o);
        const uint64_t m2 = __shfl_xor(mx, o);
        mx = m2 > mx ? m2 : mx;
        bad |= __shfl_xor(bad, o);
    }
    if ((t & 63u) == 0) {
        s_sum[t >> 6] = sum;
        s_max[t >> 6] = mx;
        s_bad[t >> 6] = bad;
    }
    __syncthreads();
    if (t == 0) {
        uint64_t all = 0, amax = 0;
        uint32_t any_bad = 0;
        for (uint32_t w = 0; w < NT / 64; ++w) {
            all += s_sum[w];
            amax = s_max[w] > amax ? s_max[w] : amax;
            any_bad |= s_bad[w];
        }
        status->pad2[0] = amax;   // largest segment count: sizes the next slack table
        status->pad2[1] = (any_bad & 2u) ? 1u : 0u;   // some segment had >= spec_min predicted frames
        any_bad &= 1u;
        uint32_t flags = any_bad ? 0u : SPEC_MATCH;
        if (SPEC) {
            const bool ok = !any_bad && all <= cap;
            if (ok) flags |= SPEC_OK;
            *total = ok ? all : 0;
        }
        status->total = all;
        status->flags = flags;
        // last: the host polls seq (fine-grained pinned memory)
        if (publish) __hip_atomic_store(&status->seq, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

template <bool SPEC>
__global__ __launch_bounds__(ONE_BLOCK) void k_spec_check(const uint64_t* __restrict__ counts,
                                                     const uint64_t* __restrict__ est,
                                                     const uint64_t* __restrict__ npred, uint32_t nseg,
                                                     uint64_t* __restrict__ total, uint64_t cap,
                                                     dspec_status* __restrict__ status, uint64_t seq) {
    spec_check_body<SPEC, ONE_BLOCK>(counts, est, npred, nseg, total, cap, status, seq, true);
}

// ----------------------------------------------------------- SLACK table
// Mixed-size batches of many segments: one EMIT walk writes each segment's
// records into its own region of a scratch table (k_head sized it: the
// segment's record bound, at most a cap from the last batch's largest
// segment count).  k_slack_check (one block) verifies every count fits its
// region and scans the counts into the exact bases; k_slack_compact moves
// the records into the frame table there.  A segment that did not fit
// zeroes the count (downstream kernels do nothing) and the host re-scans
// COUNT, read, EMIT -- so a mixed batch is discovered with one walk and no
// host round trip before EMIT, like SPEC for uniform ones.
__global__ __launch_bounds__(ONE_BLOCK) void k_slack_check(const uint64_t* __restrict__ counts,
                                                      const uint64_t* __restrict__ est,
                                                      const uint64_t* __restrict__ est_u,
                                                      const uint64_t* __restrict__ npred, uint32_t nseg,
                                                      uint64_t* __restrict__ bases_x, uint64_t* __restrict__ total,
                                                      uint64_t cap, dspec_status* __restrict__ status, uint64_t seq) {
    __shared__ uint64_t part[ONE_BLOCK], pmax[ONE_BLOCK / 64];
    __shared__ uint32_t pbad[ONE_BLOCK / 64];
    const uint32_t t = threadIdx.x;
    const uint32_t per = (nseg + ONE_BLOCK - 1u) / ONE_BLOCK;
    const uint32_t b = t * per;
    const uint32_t e = min(nseg, b + per);
    uint64_t sum = 0, mx = 0;
    uint32_t bad = 0;
    for (uint32_t i = b; i < e; ++i) {
        const uint64_t c = counts[i];
        sum += c;
        mx = c > mx ? c : mx;
        bad |= (c > est[i] ? 1u : 0u) | (c != est_u[i] ? 2u : 0u);   // 1: region overflow, 2: not uniform
        if (npred[i]) bad |= 4u;                                       // 4: a long uniform run (keep k_verify)
    }
    part[t] = sum;
    for (int o = 32; o > 0; o >>= 1) {   // max and flags: wave reductions, then one partial per wave
        const uint64_t m2 = __shfl_xor(mx, o);
        mx = m2 > mx ? m2 : mx;
        bad |= __shfl_xor(bad, o);
    }
    if ((t & 63u) == 0) {
        pmax[t >> 6] = mx;
        pbad[t >> 6] = bad;
    }
    __syncthreads();
    for (uint32_t d = 1; d < ONE_BLOCK; d <<= 1) {
        const uint64_t v = t >= d ? part[t - d] : 0;
        __syncthreads();
        part[t] += v;
        __syncthreads();
    }
    uint64_t run = part[t] - sum;
    for (uint32_t i = b; i < e; ++i) {
        bases_x[i] = run;
        run += counts[i];
    }
    if (t == 0) {
        uint64_t amax = 0;
        uint32_t any_bad = 0;
        for (uint32_t k = 0; k < ONE_BLOCK / 64; ++k) {
            amax = pmax[k] > amax ? pmax[k] : amax;
            any_bad |= pbad[k];
        }
        const uint64_t all = part[ONE_BLOCK - 1u];
        const bool ok = !(any_bad & 1u) && all <= cap;
        *total = ok ? all : 0;
        status->total = all;
        status->flags = (ok ? SPEC_OK : 0u) | ((any_bad & 2u) ? 0u : SPEC_MATCH);
        status->pad2[0] = amax;
        status->pad2[1] = (any_bad & 4u) ? 1u : 0u;
        __hip_atomic_store(&status->seq, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// One block per segment: records [bases[s], +counts[s]) of the slack table
// to [bases_x[s], ...) of the frame table; bases[s] then holds the exact base.
__global__ __launch_bounds__(256) void k_slack_compact(dframes src, dframes dst, const uint64_t* __restrict__ counts,
                                                       uint64_t* __restrict__ bases,
                                                       const uint64_t* __restrict__ bases_x,
                                                       const uint64_t* __restrict__ total, uint32_t nseg) {
    if (*total == 0) return;   // rejected (or empty): the host re-scans
    for (uint32_t s = blockIdx.x; s < nseg; s += gridDim.x) {
        const uint64_t n = counts[s], a = bases[s], b = bases_x[s];
        for (uint64_t i = threadIdx.x; i < n; i += blockDim.x) {
            dst.hdr_off[b + i] = src.hdr_off[a + i];
            dst.pay_off[b + i] = src.pay_off[a + i];
            dst.pay_len[b + i] = src.pay_len[a + i];
            dst.length[b + i] = src.length[a + i];
            dst.key[b + i] = src.key[a + i];
            dst.keyrot[b + i] = src.keyrot[a + i];
            dst.info[b + i] = src.info[a + i];
        }
        __syncthreads();   // every thread has read bases[s]
        if (threadIdx.x == 0) bases[s] = b;
    }
}

// One-segment scans whose table was sized by an estimate: over capacity
// zeroes the count (downstream kernels then do nothing; the host re-emits);
// the true count goes to pinned host memory with the scan's sequence number.
__global__ void k_cap_check(uint64_t* __restrict__ total, uint64_t cap, dspec_status* __restrict__ status,
                            uint64_t seq) {
    const uint64_t v = *total;
    const bool ok = v <= cap;
    if (!ok) *total = 0;
    status->total = v;
    status->flags = ok ? SPEC_OK : 0u;
    __hip_atomic_store(&status->seq, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// The scan's tables are complete: every earlier kernel of the stream has
// ended (and released its writes) before this one starts.
__global__ void k_publish_tiles(dspec_status* __restrict__ status, uint64_t seq) {
    __hip_atomic_store(&status->tseq, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

hipError_t launch_publish_tiles(dspec_status* status, uint64_t seq, hipStream_t st) {
    hipLaunchKernelGGL(k_publish_tiles, dim3(1), dim3(1), 0, st, status, seq);
    return hipGetLastError();
}

hipError_t launch_cap_check(uint64_t* total, uint64_t cap, dspec_status* status, uint64_t seq, hipStream_t st) {
    hipLaunchKernelGGL(k_cap_check, dim3(1), dim3(1), 0, st, total, cap, status, seq);
    return hipGetLastError();
}

// Table invariant the tile index stands on: frame ends off[k] + len[k] are
// non-decreasing over the whole table.  Every producer keeps it by
// construction -- a segment's records are written in stream order, each
// inside its own segment (a carried-in frame's record first, at the segment
// start), segments are sorted and disjoint and their record bases come from
// an exclusive scan in segment order (EMIT, SPEC, SLACK's compaction, the
// sieve's ranked chain).  k_tile_scatter then has one writer per tile, and
// k_tile_fix_class's two-load validity test and its binary search are exact.
// k_ends_check verifies it (hvws_set_table_checks, tests): bad[0] counts the
// records whose end lies before their predecessor's.
__global__ void k_ends_check(const uint64_t* __restrict__ off, const uint64_t* __restrict__ len,
                             const uint64_t* __restrict__ nfr_p, unsigned long long* __restrict__ bad) {
    const uint64_t nfr = *nfr_p;
    unsigned long long n = 0;
    for (uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x + 1; k < nfr;
         k += (uint64_t)gridDim.x * blockDim.x)
        n += off[k - 1] + len[k - 1] > off[k] + len[k];
    if (n) atomicAdd(bad, n);
}

hipError_t launch_ends_check(const uint64_t* off, const uint64_t* len, const uint64_t* nfr_dev,
                             unsigned long long* bad, hipStream_t st) {
    hipLaunchKernelGGL(k_ends_check, dim3(1024), dim3(256), 0, st, off, len, nfr_dev, bad);
    return hipGetLastError();
}

// ---------------------------------------------------------- k_tile_index
// tile_first[t] = first frame k with off[k] + len[k] > t*tile (t <= ntiles).
// Two kernels: k_tile_scatter has each frame k write the tiles whose start
// lies in [end(k-1), end(k)) (ends are non-decreasing) -- no search, one
// write per tile; frames spanning more than TILE_SPAN_MAX tiles and the
// tiles after the last frame are left marked, and k_tile_fixup binary
// searches those.  A per-tile binary search for every tile cost ~100 us at
// config 3 (4M tiles x 20 dependent loads).
// nfr_p (device) overrides nfr_v when given: the frame count of a batch can
// stay on the device, so a small batch needs no host round trip before EMIT.
// (TILE_MARK, TILE_SPAN_MAX: hvws_internal.h)

__device__ __forceinline__ void tile_scatter_body(const uint64_t* __restrict__ off, const uint64_t* __restrict__ len,
                                                  uint64_t nfr, uint32_t* __restrict__ tile_first, uint64_t ntiles,
                                                  uint64_t tile, uint64_t k0, uint64_t kstep) {
    for (uint64_t k = k0; k < nfr; k += kstep) {
        const uint64_t lo = k ? off[k - 1] + len[k - 1] : 0;
        const uint64_t hi = off[k] + len[k];
        if (hi <= lo) continue;
        const uint64_t t0 = (lo + tile - 1) / tile;
        uint64_t t1 = (hi + tile - 1) / tile;
        if (t1 > ntiles + 1) t1 = ntiles + 1;
        if (t1 <= t0 || t1 - t0 > TILE_SPAN_MAX) continue;
        for (uint64_t t = t0; t < t1; ++t) tile_first[t] = (uint32_t)k;
    }
}

__global__ void k_tile_scatter(const uint64_t* __restrict__ off, const uint64_t* __restrict__ len, uint64_t nfr_v,
                               const uint64_t* __restrict__ nfr_p, uint32_t* __restrict__ tile_first, uint64_t ntiles,
                               uint64_t tile) {
    tile_scatter_body(off, len, nfr_p ? *nfr_p : nfr_v, tile_first, ntiles, tile,
                      (uint64_t)blockIdx.x * blockDim.x + threadIdx.x, (uint64_t)gridDim.x * blockDim.x);
}

__global__ void k_tile_fixup(const uint64_t* __restrict__ off, const uint64_t* __restrict__ len, uint64_t nfr_v,
                             const uint64_t* __restrict__ nfr_p, uint32_t* __restrict__ tile_first, uint64_t ntiles,
                             uint64_t tile) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t > ntiles || tile_first[t] != TILE_MARK) return;
    const uint64_t nfr = nfr_p ? *nfr_p : nfr_v;
    const uint64_t x = t * tile;
    uint64_t lo = 0, hi = nfr;
    while (lo < hi) {
        uint64_t mid = (lo + hi) >> 1;
        if (off[mid] + len[mid] > x) hi = mid;
        else lo = mid + 1;
    }
    tile_first[t] = (uint32_t)lo;
}

// Unmask tile classes.  A tile lying wholly inside one masked payload (7 of 8
// tiles for 64 KiB frames) needs only that frame's key word: k_unmask then
// skips the frame-table staging, the LDS search and the barrier.
enum : uint32_t { TILE_GENERAL = 0, TILE_SINGLE = 1, TILE_NONE = 2 };

__global__ void k_tile_class(const uint64_t* __restrict__ off, const uint64_t* __restrict__ len,
                             const uint32_t* __restrict__ keyrot, const uint64_t* __restrict__ nfr_p,
                             const uint32_t* __restrict__ tile_first, uint32_t* __restrict__ tile_key,
                             uint8_t* __restrict__ tile_kind, uint64_t ntiles, uint64_t tile, uint64_t rx_len) {
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= ntiles) return;
    const uint64_t nfr = *nfr_p;
    const uint64_t x = t * tile;
    const uint64_t xe = x + tile < rx_len ? x + tile : rx_len;
    const uint32_t k = tile_first[t];
    uint32_t kind = TILE_GENERAL, key = 0;
    if (k >= nfr || off[k] >= xe) {
        kind = TILE_NONE;                       // no payload byte in the tile
    } else if (off[k] <= x && xe <= off[k] + len[k] && xe == x + tile) {
        key = keyrot[k];
        kind = key ? TILE_SINGLE : TILE_NONE;   // one payload; zero key word = no-op
    }
    tile_key[t] = key;
    tile_kind[t] = (uint8_t)kind;
}

// k_tile_fixup + k_tile_class in one pass over the tiles (the scan's unmask
// tiles): resolve a tile k_tile_scatter left marked, then classify it.
__device__ __forceinline__ void fix_class_body(const uint64_t* __restrict__ off, const uint64_t* __restrict__ len,
                                               const uint32_t* __restrict__ keyrot, uint64_t nfr,
                                               uint32_t* __restrict__ tile_first, uint32_t* __restrict__ tile_key,
                                               uint8_t* __restrict__ tile_kind, uint64_t ntiles, uint64_t tile,
                                               uint64_t rx_len, uint64_t t0, uint64_t tstep) {
    for (uint64_t t = t0; t <= ntiles; t += tstep) {
    const uint64_t x = t * tile;
    // tile_first[t] is not cleared between batches: k_tile_scatter writes
    // every tile whose start lies before the last frame's end, except the
    // tiles of very long frames.  An entry is taken only if it is this
    // batch's answer (the first frame ending after x); anything else -- a
    // stale or never-written entry -- is searched for.
    uint32_t k = tile_first[t];
    const bool valid = k < nfr && off[k] + len[k] > x && (k == 0 || off[k - 1] + len[k - 1] <= x);
    if (!valid) {
        uint64_t lo = 0, hi = nfr;
        while (lo < hi) {
            const uint64_t mid = (lo + hi) >> 1;
            if (off[mid] + len[mid] > x) hi = mid;
            else lo = mid + 1;
        }
        k = (uint32_t)lo;
        tile_first[t] = k;
    }
    if (t == ntiles) continue;   // sentinel entry: index only
    const uint64_t xe = x + tile < rx_len ? x + tile : rx_len;
    uint32_t kind = TILE_GENERAL, key = 0;
    if (k >= nfr || off[k] >= xe) {
        kind = TILE_NONE;
    } else if (off[k] <= x && xe <= off[k] + len[k] && xe == x + tile) {
        key = keyrot[k];
        kind = key ? TILE_SINGLE : TILE_NONE;
    }
    tile_key[t] = key;
    tile_kind[t] = (uint8_t)kind;
    }
}

__global__ void k_tile_fix_class(const uint64_t* __restrict__ off, const uint64_t* __restrict__ len,
                                 const uint32_t* __restrict__ keyrot, const uint64_t* __restrict__ nfr_p,
                                 uint32_t* __restrict__ tile_first, uint32_t* __restrict__ tile_key,
                                 uint8_t* __restrict__ tile_kind, uint64_t ntiles, uint64_t tile, uint64_t rx_len) {
    fix_class_body(off, len, keyrot, *nfr_p, tile_first, tile_key, tile_kind, ntiles, tile, rx_len,
                   (uint64_t)blockIdx.x * blockDim.x + threadIdx.x, (uint64_t)gridDim.x * blockDim.x);
}

// -------------------------------------------------------------- k_unmask
//
// One workgroup per tile of T*U*16 bytes.  Each thread owns U 16-byte chunks
// spaced T*16 bytes apart (so every wave instruction moves 1 KiB of
// contiguous bytes).  Geometry from the on-device sweep (scripts/membench2.hip,
// profiles/): the bounds check is hoisted to the tile so the U loads issue
// back to back (a per-chunk check makes hipcc wait vmcnt(0) after each), and
// the tile order is XCD-contiguous -- blocks b, b+8, b+16, ... (which the
// dispatcher places on one XCD) walk adjacent tiles -- worth 5-8 % of HBM
// throughput on in-place read+write streams.  Data loads are issued first;
// meanwhile the tile's frames (from the tile index) are staged in LDS as
// [pay_off, pay_end, key word].  A chunk wholly inside one masked payload is
// XORed with 4 copies of that frame's aligned key word; a chunk touching a
// header or a frame boundary is merged byte by byte; chunks with no masked
// byte are not written back.

template <typename END>
__device__ __forceinline__ uint32_t first_end_after(END endf, uint32_t n, uint64_t c) {
    uint32_t lo = 0, hi = n;
    while (lo < hi) {
        uint32_t mid = (lo + hi) >> 1;
        if (endf(mid) > c) hi = mid;
        else lo = mid + 1;
    }
    return lo;
}

template <typename OFF, typename END, typename KEY>
__device__ __forceinline__ bool xor_chunk(u32x4& v, uint64_t c, uint32_t nf, OFF offf, END endf, KEY keyf) {
    uint32_t k = first_end_after(endf, nf, c);
    if (k >= nf) return false;
    const uint64_t o = offf(k), e = endf(k);
    if (o >= c + 16) return false;               // only header/gap bytes here
    if (o <= c && c + 16 <= e) {                 // fast path: one payload
        const uint32_t kw = keyf(k);
        v ^= u32x4{kw, kw, kw, kw};
        return true;
    }
    // Boundary chunk.  Every frame spends >= 2 header bytes, so at most 9
    // frames touch 16 bytes.  For each payload piece OR in its key word under
    // a byte mask of the overlap [lo, hi) -- no per-byte loop.
    uint64_t mlo = 0, mhi = 0;   // key bytes for chunk bytes 0-7 / 8-15
#pragma unroll 1
    for (int p = 0; p < 10; ++p) {
        if (k >= nf) break;
        const uint64_t po = offf(k), pe = endf(k);
        if (po >= c + 16) break;
        const uint32_t lo = po > c ? (uint32_t)(po - c) : 0u;
        const uint32_t hi = pe < c + 16 ? (uint32_t)(pe - c) : 16u;
        if (hi > lo) {
            const uint64_t kw = keyf(k);
            const uint64_t kk = kw | (kw << 32);
            // bytes [lo, hi) of a 16-byte little-endian window
            const uint64_t lo_keep_lo = lo >= 8 ? 0ull : (~0ull << (8 * lo));
            const uint64_t hi_keep_lo = hi >= 8 ? ~0ull : ((1ull << (8 * hi)) - 1);
            const uint64_t lo_keep_hi = lo <= 8 ? ~0ull : (~0ull << (8 * (lo - 8)));
            const uint64_t hi_keep_hi = hi <= 8 ? 0ull : (hi >= 16 ? ~0ull : ((1ull << (8 * (hi - 8))) - 1));
            mlo |= kk & lo_keep_lo & hi_keep_lo;
            mhi |= kk & lo_keep_hi & hi_keep_hi;
        }
        if (pe > c + 16) break;
        ++k;
    }
    const uint32_t m0 = (uint32_t)mlo, m1 = (uint32_t)(mlo >> 32), m2 = (uint32_t)mhi, m3 = (uint32_t)(mhi >> 32);
    v ^= u32x4{m0, m1, m2, m3};
    return true;
}

// Tiles are visited in xcd_tile order (hvws_internal.h; cdna_hip_programming.md
// sec. 5, "XCD swizzle must be bijective").  Placement only changes speed.

template <int T, int U, bool SWZ>
__global__ __launch_bounds__(T) void k_unmask(uint8_t* __restrict__ rx, uint64_t rx_len,
                                              const uint64_t* __restrict__ pay_off,
                                              const uint64_t* __restrict__ pay_len,
                                              const uint32_t* __restrict__ keyrot,
                                              const uint32_t* __restrict__ tile_first,
                                              const uint32_t* __restrict__ tile_key,
                                              const uint8_t* __restrict__ tile_kind,
                                              const uint64_t* __restrict__ nfr_p, uint64_t tile0, uint64_t ntiles) {
    constexpr uint64_t TILE = (uint64_t)T * U * 16u;
    __shared__ uint64_t s_off[UNMASK_MAXF];
    __shared__ uint64_t s_end[UNMASK_MAXF];
    __shared__ uint32_t s_key[UNMASK_MAXF];

    const uint64_t t = tile0 + (SWZ ? xcd_tile(blockIdx.x, ntiles) : (uint64_t)blockIdx.x);
    const uint64_t base = t * TILE;
    const uint32_t tid = threadIdx.x;
    const bool full = base + TILE <= rx_len;
    const uint32_t kind = tile_kind[t];
    if (kind == TILE_NONE) return;

    u32x4 v[U];
    if (kind == TILE_SINGLE) {   // whole tile inside one masked payload
        const uint32_t kw = tile_key[t];
#pragma unroll
        for (int i = 0; i < U; ++i)
            v[i] = __builtin_nontemporal_load(
                reinterpret_cast<const u32x4*>(rx + base + ((uint64_t)i * T + tid) * 16u));
#pragma unroll
        for (int i = 0; i < U; ++i)
            __builtin_nontemporal_store(v[i] ^ u32x4{kw, kw, kw, kw},
                                        reinterpret_cast<u32x4*>(rx + base + ((uint64_t)i * T + tid) * 16u));
        return;
    }
    if (full) {
#pragma unroll
        for (int i = 0; i < U; ++i)
            v[i] = __builtin_nontemporal_load(
                reinterpret_cast<const u32x4*>(rx + base + ((uint64_t)i * T + tid) * 16u));
    } else {
#pragma unroll
        for (int i = 0; i < U; ++i) {
            const uint64_t c = base + ((uint64_t)i * T + tid) * 16u;
            uint32_t w[4] = {0u, 0u, 0u, 0u};
            for (int b = 0; b < 16; ++b)
                if (c + b < rx_len) w[b >> 2] |= (uint32_t)rx[c + b] << (8 * (b & 3));
            v[i] = u32x4{w[0], w[1], w[2], w[3]};
        }
    }

    const uint64_t nfr = *nfr_p;
    const uint32_t k0 = tile_first[t];
    const uint32_t k1r = tile_first[t + 1];
    const uint32_t k1 = (uint64_t)k1r + 1 < nfr ? k1r + 1 : (uint32_t)nfr;
    const uint32_t nf = k1 > k0 ? k1 - k0 : 0u;
    const bool staged = nf <= (uint32_t)UNMASK_MAXF;
    if (staged) {
        for (uint32_t i = tid; i < nf; i += T) {
            const uint64_t o = pay_off[k0 + i];
            const uint32_t kw = keyrot[k0 + i];
            s_off[i] = o;
            // A zero key word (unmasked frame, or a masked one whose key is
            // 0) changes nothing: stage it as an empty span so its bytes are
            // neither XORed nor written back.  Ends stay non-decreasing.
            s_end[i] = kw ? o + pay_len[k0 + i] : o;
            s_key[i] = kw;
        }
    }
    __syncthreads();

    bool dirty[U];
#pragma unroll
    for (int i = 0; i < U; ++i) {
        const uint64_t c = base + ((uint64_t)i * T + tid) * 16u;
        if (!full && c >= rx_len) {
            dirty[i] = false;
            continue;
        }
        if (staged) {
            dirty[i] = xor_chunk(
                v[i], c, nf, [&](uint32_t k) { return s_off[k]; }, [&](uint32_t k) { return s_end[k]; },
                [&](uint32_t k) { return s_key[k]; });
        } else {
            dirty[i] = xor_chunk(
                v[i], c, nf, [&](uint32_t k) { return pay_off[k0 + k]; },
                [&](uint32_t k) { return keyrot[k0 + k] ? pay_off[k0 + k] + pay_len[k0 + k] : pay_off[k0 + k]; },
                [&](uint32_t k) { return keyrot[k0 + k]; });
        }
    }
    if (full) {
#pragma unroll
        for (int i = 0; i < U; ++i)
            if (dirty[i])
                __builtin_nontemporal_store(v[i], reinterpret_cast<u32x4*>(rx + base + ((uint64_t)i * T + tid) * 16u));
    } else {
#pragma unroll
        for (int i = 0; i < U; ++i) {
            if (!dirty[i]) continue;
            const uint64_t c = base + ((uint64_t)i * T + tid) * 16u;
            const uint32_t w[4] = {v[i].x, v[i].y, v[i].z, v[i].w};
            for (int b = 0; b < 16; ++b)
                if (c + b < rx_len) rx[c + b] = (uint8_t)(w[b >> 2] >> (8 * (b & 3)));
        }
    }
}

// ------------------------------------------------------------ RUN unmask
//
// A batch whose segments are each one run of equal frames (hvws_internal.h,
// drun).  k_unmask_run loads its tile as k_unmask does; behind the loads one
// thread per run frame starting in the tile reads its header, checks it
// against the run's hypothesis (header length, payload length, mask bit) and
// keeps its key in LDS; then every chunk XORs the pieces that meet it: the
// carried-in frame's, the run frames' (position by division by the stride),
// the cut frame's.  The scan beside the previous unmask is k_head and
// k_run_tiles.  A failed check marks the segment; k_run_fix (behind, on the
// same stream) XORs that segment's hypothesis back -- the same keys from the
// same, unchanged header positions -- and unmasks it exactly.

// floor((x - p0) / stride) for x >= p0, exact (double estimate, corrected)
__device__ __forceinline__ uint64_t run_frame_of(const drun& r, uint64_t x) {
    const uint64_t d = x - r.p0;
    uint64_t j = (uint64_t)((double)d * r.inv);
    while (j && j * r.stride > d) --j;
    while ((j + 1) * r.stride <= d) ++j;
    return j;
}

// OR key word kw (for 4-byte aligned words) into the chunk mask for bytes
// [lo, hi) of the chunk at c (absolute), clamped to the chunk
__device__ __forceinline__ void run_piece(uint64_t& mlo, uint64_t& mhi, uint64_t c, uint64_t lo, uint64_t hi,
                                          uint32_t kw) {
    const uint64_t a = lo > c ? lo : c, b = hi < c + 16 ? hi : c + 16;
    if (a >= b || !kw) return;
    const uint32_t l = (uint32_t)(a - c), h = (uint32_t)(b - c);
    const uint64_t kk = (uint64_t)kw | ((uint64_t)kw << 32);
    const uint64_t keep_lo = (l >= 8 ? 0ull : (~0ull << (8 * l))) & (h >= 8 ? ~0ull : ((1ull << (8 * h)) - 1));
    const uint64_t keep_hi = (l <= 8 ? ~0ull : (~0ull << (8 * (l - 8)))) &
                             (h <= 8 ? 0ull : (h >= 16 ? ~0ull : ((1ull << (8 * (h - 8))) - 1)));
    mlo |= kk & keep_lo;
    mhi |= kk & keep_hi;
}

// A run frame's key as the hypothesis lays its header out: the 4 bytes before
// its payload (bytes hlen-4 .. hlen-1 of the 16 at the header).  Only bytes
// inside the hypothesised header are used, which no piece of the hypothesis
// XORs -- so the repair pass reads the same key the unmask used even where
// the hypothesis is wrong (a key parsed by the header's own length field
// could lie in bytes the unmask changed).
__device__ __forceinline__ uint32_t run_key(const drun& r, uint64_t lo, uint64_t hi) {
    if (!r.masked || r.hlen < 6) return 0u;
    const uint32_t b = r.hlen - 4u;   // 2, 4 or 10
    return b == 2 ? (uint32_t)(lo >> 16) : (b == 4 ? (uint32_t)(lo >> 32) : (uint32_t)(hi >> 16));
}

// Unmask entries of segment r meeting [x0, x1): the carried-in piece, the run
// frames, the cut frame's piece (in stream order); cnt_only: just count them.
// Run frame j's entry is [its payload start, end) with the key word of its
// header (written by the caller, which parses the header).
__device__ __forceinline__ void run_tile_frames(const drun& r, uint64_t x0, uint64_t x1, uint32_t& jlo, uint32_t& nj) {
    jlo = 0;
    nj = 0;
    if (!r.cnt || (r.flags & RUN_BAD)) return;
    const uint64_t re = r.p0 + (uint64_t)r.cnt * r.stride;
    const uint64_t a = x0 > r.p0 ? x0 : r.p0, b = x1 < re ? x1 : re;
    if (a >= b) return;
    jlo = (uint32_t)run_frame_of(r, a);
    nj = (uint32_t)run_frame_of(r, b - 1) + 1u - jlo;
}

// Runs k_unmask_run takes: strides of at least RUN_MIN_STRIDE bytes, so the
// frames of a tile's two runs need at most TILE / RUN_MIN_STRIDE + 8 key
// slots (s_fk, sized by run_key_slots); a run of smaller frames (2-31 B:
// thousands per tile) is left to the repair's exact path.
constexpr uint32_t RUN_MIN_STRIDE = 32;
__host__ __device__ constexpr uint32_t run_key_slots(uint64_t tile) { return (uint32_t)(tile / RUN_MIN_STRIDE) + 16u; }
// frames of one run meeting a tile: at most (tile + stride - 1) / stride + 1;
// two runs, each with 3 extra slots, fit with room to spare
static_assert((16384 + RUN_MIN_STRIDE - 1) / RUN_MIN_STRIDE + 1 + 3 + 3 + 3 <= run_key_slots(16384), "RUN key slots");

__device__ __forceinline__ bool run_fast_ok(const drun& r) {
    return !(r.flags & RUN_BAD) && (!r.cnt || (r.stride >= RUN_MIN_STRIDE && r.stride <= RUN_FAST_STRIDE));
}

// Run r as it meets the tile [x, x + tile) (dtrun's fields after k0); a run
// k_unmask_run does not take (ok false) meets it with nothing.
__device__ __forceinline__ void tile_run(dtrun& o, const drun& r, bool ok, uint64_t x, uint64_t tile) {
    o.S = (uint32_t)r.stride;
    o.len = (uint32_t)r.len;
    o.hm = r.hlen | (r.masked << 8);
    o.nj = 0;
    o.h0 = 0;
    o.a_lo = o.a_hi = o.t_lo = o.t_hi = 0;
    o.a_kw = o.t_kw = 0;
    if (!ok) return;
    uint32_t jlo, nj;
    run_tile_frames(r, x, x + tile, jlo, nj);
    o.nj = nj;
    o.h0 = nj ? (int32_t)((int64_t)(r.p0 + (uint64_t)jlo * r.stride) - (int64_t)x) : 0;
    const uint64_t te = x + tile;
    if (r.a_kw && r.a_off < te && r.a_end > x) {
        o.a_lo = (int32_t)((r.a_off > x ? r.a_off : x) - x);
        o.a_hi = (int32_t)((r.a_end < te ? r.a_end : te) - x);
        o.a_kw = r.a_kw;
    }
    if (r.t_kw && r.t_off < te && r.t_end > x) {
        o.t_lo = (int32_t)((r.t_off > x ? r.t_off : x) - x);
        o.t_hi = (int32_t)((r.t_end < te ? r.t_end : te) - x);
        o.t_kw = r.t_kw;
    }
}

// trun[t] for every unmask tile, one wave per segment s writing the tiles
// whose first byte lies in [end of s - 1, end of s) (s0 = s; the last
// segment's wave also the tiles past every segment: s0 = nseg).  s1 = the
// first segment ending after the tile's last byte (clamped to the last).
// k_unmask_run takes a tile's s0 and s1; the segments between (each wholly
// inside the tile) are marked for the repair's exact path (fail bit 2), as
// is -- by the repair itself -- a segment whose run it does not take
// (run_fast_ok).  The key of s0's run frame begun before the tile is read
// here, beside the previous unmask, not on the unmask's critical path.
__device__ __forceinline__ void run_tiles_seg(const uint8_t* __restrict__ rx, uint64_t rx_len,
                                              const dseg* __restrict__ segs, uint32_t nseg,
                                              const drun* __restrict__ runs, dtrun* __restrict__ trun,
                                              uint64_t ntiles, uint64_t tile, uint32_t* __restrict__ fail,
                                              uint32_t s, uint32_t lane) {
    const uint64_t e0 = s ? segs[s - 1].off + segs[s - 1].len : 0;
    const uint64_t e1 = segs[s].off + segs[s].len;
    const uint64_t ta = (e0 + tile - 1) / tile, tb = (e1 + tile - 1) / tile;
    const uint64_t tz = s + 1 == nseg ? ntiles : tb;
    const drun r = runs[s];
    const bool ok = run_fast_ok(r);
    const uint64_t re = r.p0 + (uint64_t)r.cnt * r.stride;
    for (uint64_t t = ta + lane; t < tz; t += 64) {
        const uint64_t x = t * tile;
        dtrun o;
        o.pad[0] = o.pad[1] = 0;
        o.k0 = 0;
        if (t >= tb) {   // past every segment
            o.s0 = o.s1 = nseg;
            tile_run(o, r, false, x, tile);
            trun[t] = o;
            continue;
        }
        o.s0 = s;
        uint32_t s1 = s;
        while (s1 + 1 < nseg && segs[s1].off + segs[s1].len <= x + tile - 1) ++s1;
        o.s1 = s1;
        tile_run(o, r, ok, x, tile);
        if (ok && r.cnt && r.masked && x > r.p0 && x < re) {
            const uint64_t hs = r.p0 + run_frame_of(r, x) * r.stride;
            if (hs < x) {
                uint64_t lo, hi;
                ld16(rx, rx_len, hs, lo, hi);
                o.k0 = run_key(r, lo, hi);
            }
        }
        bool exact = !ok || (s1 != s && !run_fast_ok(runs[s1]));
        for (uint32_t m = s + 1; m < s1; ++m) {
            atomicOr(&fail[m], 2u);
            exact = true;
        }
        if (exact) atomicOr(&fail[nseg], 1u);   // the repair pass must look
        trun[t] = o;
    }
}

__global__ __launch_bounds__(256) void k_run_tiles(const uint8_t* __restrict__ rx, uint64_t rx_len,
                                                   const dseg* __restrict__ segs, uint32_t nseg,
                                                   const drun* __restrict__ runs, dtrun* __restrict__ trun,
                                                   uint64_t ntiles, uint64_t tile, uint32_t* __restrict__ fail) {
    const uint32_t lane = threadIdx.x & 63u;
    for (uint32_t s = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); s < nseg; s += gridDim.x * (blockDim.x >> 6))
        run_tiles_seg(rx, rx_len, segs, nseg, runs, trun, ntiles, tile, fail, s, lane);
}

// The run hypothesis' header bytes 1 .. 1 + ext (MASK bit + 7-bit length,
// then the extended length, big-endian) as a 16-byte pattern and its byte
// mask, relative to the header's first byte; byte 0 (FIN, RSV, opcode) is
// free, as is the key.
__device__ __forceinline__ void run_pattern(uint32_t masked, uint32_t hlen, uint64_t len, uint64_t& plo, uint64_t& phi,
                                            uint64_t& mlo, uint64_t& mhi) {
    const uint32_t ext = hlen - 2u - (masked ? 4u : 0u);   // 0, 2 or 8
    const uint64_t b1 = (masked ? 0x80u : 0u) | (ext == 0 ? len : (ext == 2 ? 126u : 127u));
    plo = b1 << 8;
    phi = 0;
    mlo = 0xFFull << 8;
    mhi = 0;
    if (ext == 2) {
        plo |= ((len >> 8) & 0xFFu) << 16 | (len & 0xFFu) << 24;
        mlo |= 0xFFFFull << 16;
    } else if (ext == 8) {
        const uint64_t be = __builtin_bswap64(len);   // bytes 2..9
        plo |= be << 16;
        phi = be >> 48;
        mlo |= ~0ull << 16;
        mhi = 0xFFFFull;
    }
}

// The unmask of a RUN step.  Every tile takes at most two runs, its first
// and last segment's (the segments between, each wholly inside the tile,
// are left to the repair's exact path; so is a run of a stride outside
// [32, RUN_FAST_STRIDE] or one k_head found is not one run), in 32-bit
// tile-relative arithmetic.  An earlier form (v3: an entry table per tile
// in LDS, as k_unmask's, plus each lane taking header bytes from its chunks)
// took 73 VGPRs and twice k_unmask's VALU instructions per byte and ran at
// half the stream rate (profiles/r5g_raw).

// v_perm selectors by the two 4-bit byte masks of a word (e = g's | g + 1's
// << 4): byte b takes 4 + b (byte b of the first operand, slot g + 1), b (of
// the second, slot g + 2) or 12 (zero).
struct run_sel_table {
    uint32_t v[256];
    constexpr run_sel_table() : v() {
        for (uint32_t e = 0; e < 256; ++e) {
            uint32_t sel = 0;
            for (uint32_t b = 0; b < 4; ++b)
                sel |= (((e >> b) & 1u) ? 4u + b : (((e >> (4 + b)) & 1u) ? b : 12u)) << (8 * b);
            v[e] = sel;
        }
    }
};
__device__ constexpr run_sel_table kRunSel{};

// One run of a fast tile, tile-relative (32-bit positions): its frames
// meeting the tile are g = 0 .. nj-1, g's header at h0 + g * S; their keys
// in LDS slots slot + g + 1 (slot + 0 and the two past the run: 0).
struct fast_run {
    int32_t S, hl, h0;
    uint32_t nj, slot, masked, seg, k0, len;
    int32_t a_lo, a_hi, t_lo, t_hi;   // the carried-in / cut frame's payload pieces in the tile
    uint32_t a_kw, t_kw;              // (0: none)
};

__device__ __forceinline__ void fast_run_init(fast_run& R, const dtrun& o, uint32_t seg, uint32_t slot) {
    R.S = (int32_t)o.S;
    R.hl = (int32_t)(o.hm & 0xFFu);
    R.masked = (o.hm >> 8) & 1u;
    R.len = o.len;
    R.h0 = o.h0;
    R.nj = o.nj;
    R.slot = slot;
    R.seg = seg;
    R.k0 = o.k0;
    R.a_lo = o.a_lo, R.a_hi = o.a_hi, R.t_lo = o.t_lo, R.t_hi = o.t_hi;
    R.a_kw = o.a_kw, R.t_kw = o.t_kw;
}

// One thread per slot: the header of each run frame that starts in the tile
// (16 bytes from HBM, issued behind the tile's loads; no unmask changes a
// byte the hypothesis calls header) checked against the hypothesis (header
// length, payload length, mask bit); the frame's key word, rotated to its
// payload's phase, into its slot.
__device__ __forceinline__ void fast_run_keys(const fast_run& R, const uint8_t* rx, uint64_t rx_len, uint64_t base,
                                              uint32_t* s_fk, uint32_t* __restrict__ fail, uint32_t nseg, uint32_t tid,
                                              uint32_t T, const uint32_t* s_tile, int32_t tile_bytes) {
    uint64_t plo, phi, mlo, mhi;
    run_pattern(R.masked, (uint32_t)R.hl, R.len, plo, phi, mlo, mhi);
    const uint32_t kb = (uint32_t)R.hl - 4u;   // the key's first byte in a masked header: 2, 4 or 10
    for (uint32_t s = tid; s < R.nj + 3; s += T) {
        const int32_t g = (int32_t)s - 1;
        uint32_t key = 0;
        if (g >= 0 && g < (int32_t)R.nj) {
            const int32_t hs = R.h0 + g * R.S;
            if (hs < 0) {
                key = R.k0;   // begun before the tile: its header is checked where it starts
            } else {
                uint64_t lo, hi;
                if (hs + 16 <= tile_bytes) lds_hdr16(s_tile, (uint32_t)hs, lo, hi);   // staged tile
                else ld16(rx, rx_len, base + (uint64_t)hs, lo, hi);
                if (((lo ^ plo) & mlo) | ((hi ^ phi) & mhi)) {
                    atomicOr(&fail[R.seg], 1u);
                    atomicOr(&fail[nseg], 1u);
                }
                if (R.masked) key = kb < 8 ? (uint32_t)(lo >> (8 * kb)) : (uint32_t)(hi >> (8 * (kb - 8)));
            }
            key = rotr32(key, 8u * ((0u - (uint32_t)(hs + R.hl)) & 3u));
        }
        s_fk[R.slot + s] = R.masked ? key : 0u;
    }
}

// The key bytes run R lays on the chunk at tile-relative x, ORed into m[4]:
// x's frame g by a float reciprocal; g's payload [t1, t2) takes slot g + 1,
// g + 1's from t3 slot g + 2 (S >= 32: no third frame meets 16 bytes); each
// word's bytes picked by one v_perm whose selector s_sel gives for the two
// 4-bit byte masks.  The carried-in and cut pieces, when they meet the tile.
__device__ __forceinline__ void fast_run_mask(const fast_run& R, const uint32_t* s_fk, const uint32_t* s_sel,
                                              int32_t x, uint32_t m[4]) {
    if (R.nj) {
        const int32_t S = R.S;
        int32_t r = x - R.h0 + S;
        r = r < 0 ? 0 : r;
        int32_t q = (int32_t)((float)r * __builtin_amdgcn_rcpf((float)S));   // g + 1, within one
        const int32_t qs = (int32_t)__umul24((uint32_t)q, (uint32_t)S);
        if (qs > r) --q;
        else if (qs + S <= r) ++q;
        q = q < (int32_t)R.nj + 1 ? q : (int32_t)R.nj + 1;
        const int32_t hs = R.h0 + (int32_t)__umul24((uint32_t)q, (uint32_t)S) - S;
        const int32_t t1 = hs + R.hl - x, t2 = hs + S - x, t3 = t2 + R.hl;
        const uint32_t a1 = (uint32_t)(t1 < 0 ? 0 : (t1 > 16 ? 16 : t1));
        const uint32_t a2 = (uint32_t)(t2 < 0 ? 0 : (t2 > 16 ? 16 : t2));
        const uint32_t a3 = (uint32_t)(t3 < 0 ? 0 : (t3 > 16 ? 16 : t3));
        const uint32_t pm = ((((1u << (a2 - a1)) - 1u) << a1) & 0xFFFFu) | (((0xFFFFu << a3) & 0xFFFFu) << 16);
        const uint32_t kf = s_fk[R.slot + (uint32_t)q], kf1 = s_fk[R.slot + (uint32_t)q + 1];
#pragma unroll
        for (int j = 0; j < 4; ++j)
            m[j] |= __builtin_amdgcn_perm(kf, kf1, s_sel[((pm >> (4 * j)) & 15u) | ((pm >> (12 + 4 * j)) & 0xF0u)]);
    }
    if (R.a_kw | R.t_kw) {   // bytes [lo, hi) of the chunk: the 4-bit byte masks of the selector table
        const int32_t al = R.a_lo - x, ah = R.a_hi - x, tl = R.t_lo - x, th = R.t_hi - x;
        const uint32_t b1 = (uint32_t)(al < 0 ? 0 : (al > 16 ? 16 : al)), b2 = (uint32_t)(ah < 0 ? 0 : (ah > 16 ? 16 : ah));
        const uint32_t c1 = (uint32_t)(tl < 0 ? 0 : (tl > 16 ? 16 : tl)), c2 = (uint32_t)(th < 0 ? 0 : (th > 16 ? 16 : th));
        const uint32_t pa = b2 > b1 ? ((1u << (b2 - b1)) - 1u) << b1 : 0u;
        const uint32_t pt = c2 > c1 ? ((1u << (c2 - c1)) - 1u) << c1 : 0u;
#pragma unroll
        for (int j = 0; j < 4; ++j)
            m[j] |= __builtin_amdgcn_perm(R.a_kw, R.t_kw,
                                          s_sel[((pa >> (4 * j)) & 15u) | (((pt >> (4 * j)) & 15u) << 4)]);
    }
}

// The tiles.  The tile's loads are issued first; behind them one thread per
// run frame reads its header and keeps its key (fast_run_keys) while the
// selector table is built; one barrier; each chunk XORs what the runs lay on
// it.
template <int T, int U>
__device__ __forceinline__ void run_unmask_tile(uint8_t* __restrict__ rx, uint64_t rx_len, const drun* __restrict__ runs,
                                                const dtrun* __restrict__ trun, uint32_t nseg,
                                                uint32_t* __restrict__ fail, uint64_t t, uint32_t* s_fk,
                                                uint32_t* s_sel, uint32_t* s_tile) {
    constexpr uint64_t TILE = (uint64_t)T * U * 16u;
    const uint64_t base = t * TILE, te = base + TILE;
    const uint32_t tid = threadIdx.x;
    const bool full = te <= rx_len;
    u32x4 v[U];
    if (full) {
#pragma unroll
        for (int i = 0; i < U; ++i)
            v[i] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(rx + base + ((uint64_t)i * T + tid) * 16u));
    } else {
#pragma unroll
        for (int i = 0; i < U; ++i) {
            const uint64_t c = base + ((uint64_t)i * T + tid) * 16u;
            uint32_t w[4] = {0u, 0u, 0u, 0u};
            for (int b = 0; b < 16; ++b)
                if (c + b < rx_len) w[b >> 2] |= (uint32_t)rx[c + b] << (8 * (b & 3));
            v[i] = u32x4{w[0], w[1], w[2], w[3]};
        }
    }
    // the record after the data loads (it is not in any cache by now)
    const dtrun& tr = trun[t];   // wave-uniform: scalar loads
    const uint32_t s0 = tr.s0;
    if (s0 >= nseg) return;   // no segment reaches this tile
    // the headers from the tile's own bytes: staged in LDS, one more barrier
#pragma unroll
    for (int i = 0; i < U; ++i) *reinterpret_cast<u32x4*>(&s_tile[((uint32_t)i * T + tid) * 4u]) = v[i];
    __syncthreads();
    fast_run R0, R1;
    fast_run_init(R0, tr, s0, 0);
    const uint32_t s1 = tr.s1;
    const bool two = s1 != s0;
    if (two) {   // s1 starts inside the tile: its run frames from its first, no k0
        const drun r1 = runs[s1];
        dtrun o1;
        o1.k0 = 0;
        tile_run(o1, r1, run_fast_ok(r1), base, TILE);
        fast_run_init(R1, o1, s1, R0.nj + 3);
    }
    fast_run_keys(R0, rx, rx_len, base, s_fk, fail, nseg, tid, T, s_tile, (int32_t)TILE);
    if (two) fast_run_keys(R1, rx, rx_len, base, s_fk, fail, nseg, tid, T, s_tile, (int32_t)TILE);
    for (uint32_t e = tid; e < 256; e += T) s_sel[e] = kRunSel.v[e];
    __syncthreads();
    bool dirty[U];
#pragma unroll
    for (int i = 0; i < U; ++i) {
        const int32_t x = (int32_t)(((uint32_t)i * T + tid) * 16u);
        dirty[i] = false;
        if (!full && base + (uint64_t)x >= rx_len) continue;
        uint32_t m[4] = {0u, 0u, 0u, 0u};
        fast_run_mask(R0, s_fk, s_sel, x, m);
        if (two) fast_run_mask(R1, s_fk, s_sel, x, m);
        if (m[0] | m[1] | m[2] | m[3]) {
            v[i] ^= u32x4{m[0], m[1], m[2], m[3]};
            dirty[i] = true;
        }
    }
    if (full) {
#pragma unroll
        for (int i = 0; i < U; ++i)
            if (dirty[i])
                __builtin_nontemporal_store(v[i], reinterpret_cast<u32x4*>(rx + base + ((uint64_t)i * T + tid) * 16u));
    } else {
#pragma unroll
        for (int i = 0; i < U; ++i) {
            if (!dirty[i]) continue;
            const uint64_t c = base + ((uint64_t)i * T + tid) * 16u;
            const uint32_t w[4] = {v[i].x, v[i].y, v[i].z, v[i].w};
            for (int b = 0; b < 16; ++b)
                if (c + b < rx_len) rx[c + b] = (uint8_t)(w[b >> 2] >> (8 * (b & 3)));
        }
    }
}

// XOR [lo, hi) of HBM with key word kw (for 4-byte aligned words), one wave
__device__ __forceinline__ void wave_xor_range(uint8_t* rx, uint64_t lo, uint64_t hi, uint32_t kw) {
    if (lo >= hi || !kw) return;
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t a = (lo + 15) & ~15ull, b = hi & ~15ull;
    if (a >= b) {
        for (uint64_t x = lo + lane; x < hi; x += 64) rx[x] ^= (uint8_t)(kw >> (8 * (x & 3u)));
        return;
    }
    for (uint64_t x = lo + lane; x < a; x += 64) rx[x] ^= (uint8_t)(kw >> (8 * (x & 3u)));
    for (uint64_t x = b + lane; x < hi; x += 64) rx[x] ^= (uint8_t)(kw >> (8 * (x & 3u)));
    for (uint64_t x = a + (uint64_t)lane * 16u; x < b; x += 64u * 16u) {
        u32x4* q = reinterpret_cast<u32x4*>(rx + x);
        *q = *q ^ u32x4{kw, kw, kw, kw};
    }
}

// The repair: nothing unless a segment failed (one word read per
// workgroup).  A failed segment is put back -- its hypothesis XORed again
// with the same keys, read from the same header positions, which no unmask
// changes -- and unmasked exactly (the carried-in frame, then walk_frames over
// HBM, each record's payload XORed by its lane).  A segment k_head found not
// to be one run (RUN_BAD), or that the tiles left (fail bit 2, or a stride
// they do not take), had nothing applied: exact only.  Waves w0, w0 + wn, ...
// take the segments.
// fail[s]: 1 = s's hypothesis failed (undo, then exact), 2 = left to the
// repair (exact); fail[nseg] = any, [nseg + 1] = repaired count, [nseg + 2]
// = repair workgroups done; all of them, and every segment's word, are zero
// when the repair ends.
// wave_xor_range clamped to segment r's bytes: every range the repair XORs
// from a descriptor lies inside its segment by construction (k_head), and the
// clamp keeps it there by construction too -- the repair's XORs are the RUN
// path's only global writes not bounded by a tile (the r5h fault).
__device__ __forceinline__ void seg_xor_range(uint8_t* rx, const drun& r, uint64_t lo, uint64_t hi, uint32_t kw) {
    wave_xor_range(rx, lo > r.seg_lo ? lo : r.seg_lo, hi < r.seg_hi ? hi : r.seg_hi, kw);
}

__device__ __forceinline__ void run_repair(uint8_t* __restrict__ rx, uint64_t rx_len, const drun* __restrict__ runs,
                                           uint32_t nseg, uint32_t* __restrict__ fail, uint32_t w0, uint32_t wn) {
    const uint32_t lane = threadIdx.x & 63u;
    if (__hip_atomic_load(&fail[nseg], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0) return;
    for (uint32_t s = w0; s < nseg; s += wn) {
        const drun r = runs[s];
        const uint32_t fs = fail[s];
        const bool bad = !run_fast_ok(r) || (fs & 2u);   // nothing applied: the exact path only
        // zero again for the set's next RUN step: a later batch of fewer
        // segments has its batch words (nseg ..) where this one had these
        if (fs && lane == 0) fail[s] = 0;
        if (!bad && !fs) continue;
        if (lane == 0) atomicAdd(&fail[nseg + 1], 1u);
        if (!bad) {   // undo the hypothesis
            seg_xor_range(rx, r, r.a_off, r.a_end, r.a_kw);
            seg_xor_range(rx, r, r.t_off, r.t_end, r.t_kw);
            if (r.masked)
                for (uint64_t j = 0; j < r.cnt; ++j) {
                    const uint64_t fo = r.p0 + j * r.stride;
                    uint64_t lo, hi;
                    ld16(rx, rx_len, fo, lo, hi);
                    const uint64_t ps = fo + r.hlen;
                    seg_xor_range(rx, r, ps, fo + r.stride, rotr32(run_key(r, lo, hi), 8u * ((0u - (uint32_t)ps) & 3u)));
                }
            __threadfence();
        }
        // the exact path over the segment's bytes
        const uint64_t sb = r.seg_lo, L = r.seg_hi - r.seg_lo;
        dcarry st = r.cin;
        uint64_t pos = 0, n = 0;
        frec fr0;
        if (st.state != S_START && scalar_frame(rx + sb, L, st, pos, fr0, 0u) && (fr0.info & I_BODY) &&
            (fr0.info & F_MASK)) {
            const uint64_t po = sb + fr0.pay_off;
            seg_xor_range(rx, r, po, po + fr0.pay_len, key_for_aligned(fr0.key, po, (fr0.info >> 8) & 3u));
        }
        __threadfence();
        // walk_frames calls emit from every lane owning a record (the
        // whole frames of one round) or from lane 0 (the cut frame)
        walk_frames<true>(rx, rx_len, sb, L, st, pos, n, 0u, [&](uint64_t, const frec& v) {
            if (!(v.info & I_BODY) || !(v.info & F_MASK)) return;
            const uint64_t po = sb + v.pay_off, pe = po + v.pay_len;
            const uint32_t kw = key_for_aligned(v.key, po, (v.info >> 8) & 3u);
            for (uint64_t x = po; x < pe; ++x) rx[x] ^= (uint8_t)(kw >> (8 * (x & 3u)));
        });
        __threadfence();
    }
}

template <int T, int U>
__global__ __launch_bounds__(T) void k_unmask_run(uint8_t* __restrict__ rx, uint64_t rx_len, const drun* __restrict__ runs,
                                                  const dtrun* __restrict__ trun, uint32_t nseg,
                                                  uint32_t* __restrict__ fail, uint64_t tile0) {
    constexpr uint64_t TILE = (uint64_t)T * U * 16u;
    __shared__ uint32_t s_fk[run_key_slots(TILE)];   // 2 runs: sum of (nj + 3) <= TILE / 32 + 8 (run_fast_ok)
    __shared__ uint32_t s_sel[256];
    __shared__ uint32_t s_tile[TILE / 4 + 8];
    run_unmask_tile<T, U>(rx, rx_len, runs, trun, nseg, fail, tile0 + blockIdx.x, s_fk, s_sel, s_tile);
}

// The repair kernel behind the unmask on the same stream (a kernel boundary
// is the one cheap grid-wide barrier: the repair workgroups folded into the
// unmask grid needed a release fence per tile workgroup to hand over its
// bytes, 11.7 ms a step at c2, profiles/r5r_raw).  With no failure -- the
// common case, one word read -- workgroup 0 publishes (seq, 0) at once.
constexpr uint32_t RUN_FIX_BLOCKS = 32;

__global__ __launch_bounds__(256) void k_run_fix(uint8_t* __restrict__ rx, uint64_t rx_len, const drun* __restrict__ runs,
                                                 uint32_t nseg, uint32_t* __restrict__ fail,
                                                 dspec_status* __restrict__ status, uint64_t seq) {
    const bool any = __hip_atomic_load(&fail[nseg], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
    if (!any) {
        if (blockIdx.x == 0 && threadIdx.x == 0) {
            status->pad3[1] = 0;
            __hip_atomic_store(&status->pad3[0], seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        return;
    }
    run_repair(rx, rx_len, runs, nseg, fail, blockIdx.x * 4u + (threadIdx.x >> 6), gridDim.x * 4u);
    // the last workgroup publishes
    __shared__ uint32_t s_last;
    __syncthreads();
    if (threadIdx.x == 0) {
        __threadfence();
        s_last = atomicAdd(&fail[nseg + 2], 1u) == gridDim.x - 1u;
    }
    __syncthreads();
    if (s_last && threadIdx.x == 0) {
        __threadfence();
        status->pad3[1] = __hip_atomic_load(&fail[nseg + 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&status->pad3[0], seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        // the batch's words clean for this table set's next RUN step
        fail[nseg] = 0;
        fail[nseg + 1] = 0;
        fail[nseg + 2] = 0;
    }
}

// ---------------------------------------------------------- k_stream_xor
// The same geometry with no frame table: the measured in-place ceiling.
template <int T, int U, bool SWZ>
__global__ __launch_bounds__(T) void k_stream_xor(uint8_t* __restrict__ d, uint64_t n, uint64_t tile0, uint64_t ntiles,
                                                  uint32_t pat) {
    constexpr uint64_t TILE = (uint64_t)T * U * 16u;
    const uint64_t t = tile0 + (SWZ ? xcd_tile(blockIdx.x, ntiles) : (uint64_t)blockIdx.x);
    const uint64_t base = t * TILE;
    if (base + TILE <= n) {
        u32x4 v[U];
#pragma unroll
        for (int i = 0; i < U; ++i)
            v[i] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(d + base + ((uint64_t)i * T + threadIdx.x) * 16u));
#pragma unroll
        for (int i = 0; i < U; ++i)
            __builtin_nontemporal_store(v[i] ^ u32x4{pat, pat, pat, pat},
                                        reinterpret_cast<u32x4*>(d + base + ((uint64_t)i * T + threadIdx.x) * 16u));
    } else {
        for (int i = 0; i < U; ++i) {
            const uint64_t c = base + ((uint64_t)i * T + threadIdx.x) * 16u;
            for (int b = 0; b < 16; ++b)
                if (c + b < n) d[c + b] ^= (uint8_t)(pat >> (8 * (b & 3)));
        }
    }
}

// XOR one span with a key and phase (websocket_decode on device).
__global__ void k_xor_span(uint8_t* __restrict__ d, uint64_t n, uint32_t key, uint32_t phase) {
    // d is 16-B aligned; byte a uses key byte (a + phase) & 3.
    const uint32_t kw = rotr32(key, 8u * (phase & 3u));
    for (uint64_t c = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) * 16u; c < n;
         c += (uint64_t)gridDim.x * blockDim.x * 16u) {
        if (c + 16 <= n) {
            uint4 v = *reinterpret_cast<const uint4*>(d + c);
            v.x ^= kw;
            v.y ^= kw;
            v.z ^= kw;
            v.w ^= kw;
            *reinterpret_cast<uint4*>(d + c) = v;
        } else {
            for (uint64_t a = c; a < n; ++a) d[a] ^= (uint8_t)(kw >> (8 * (a & 3u)));
        }
    }
}

// --------------------------------------------------------------- launchers

// A RUN scan's k_head and k_run_tiles grids at most this many blocks (512
// waves, each taking segments in turn; $HVWS_EXPERIMENT run_scan_grid, 0: one
// wave per segment).  They run beside the previous step's unmask at high
// priority, and one wave per segment (1024 blocks at c2) slowed the unmask
// piece beside them: c2 ms per step by cap, none 0.367-0.369, 512 0.367,
// 256 0.363, 128 0.357-0.358, 64 0.357 (profiles/r5_raw/events, rg_*).  A RUN
// segment holds >= 64 KiB (RUN_MIN_SEG), so 512 waves still scan segments
// faster than the unmask consumes them.
static uint32_t run_scan_grid() {
    static const uint32_t v = experiment("run_scan_grid") ? (uint32_t)atoi(experiment("run_scan_grid")) : 128u;
    return v;
}

static uint32_t wave_blocks(uint32_t nseg) {
    const uint32_t wpb = SCAN_THREADS / 64;
    uint32_t blocks = (nseg + wpb - 1) / wpb;
    return blocks > 65536u ? 65536u : (blocks ? blocks : 1u);
}

// $HVWS_EXPERIMENT walk_blocks (experiment): cap the walk's grid; each wave then walks
// several segments in turn (fewer wave slots taken beside a running unmask).
static uint32_t walk_blocks(uint32_t nseg) {
    static const long cap = experiment("walk_blocks") ? atol(experiment("walk_blocks")) : 0;
    const uint32_t b = wave_blocks(nseg);
    return cap > 0 && (uint32_t)cap < b ? (uint32_t)cap : b;
}

hipError_t launch_scan(int pass, const uint8_t* rx, uint64_t rx_len, const dseg* segs, uint32_t nseg,
                       const dcarry* carry_in, dcarry* carry_out, uint64_t* counts, uint64_t* bases,
                       uint64_t* total, scan_scratch sc, dframes fr, uint32_t vmask, hipStream_t st) {
    if (nseg == 0) return hipSuccess;
    const uint32_t wb = wave_blocks(nseg), wwb = walk_blocks(nseg);
    const uint32_t vb = 2048;
    // The frame sieve (one segment): its chain of whole frames is found in
    // parallel between the COUNT-side head and EMIT; k_walk resumes after it.
    const bool sieve = sc.sieve && nseg == 1 && (pass == SCAN_SINGLE || pass == SCAN_EMIT);
    const dsieve* sv = sieve ? sc.sieve->state : nullptr;
    const uint64_t* sv_S = sieve ? sc.sieve->S : nullptr;
    // k_head<false> opens every pass but EMIT; it takes the zero-copy tables.
    auto head_count = [&](uint64_t* est) {
        hipLaunchKernelGGL(k_head<false>, dim3(wb), dim3(SCAN_THREADS), 0, st, rx, rx_len, segs, nseg, carry_in,
                           sc.mid, sc.npred, sc.first_fail, sc.last_masked, bases, fr, vmask, spec_min(), est,
                           sc.src_segs, sc.src_carry, sc.segs_w, sc.carry_w, (int)(pass == SCAN_SINGLE && sieve),
                           pass == SCAN_SLACK ? sc.slack_cap : (uint64_t)0,
                           pass == SCAN_SLACK ? sc.est_u : (uint64_t*)nullptr, 0u, (drun*)nullptr, (uint32_t*)nullptr);
        hipLaunchKernelGGL(k_offsets, dim3(1), dim3(ONE_BLOCK), 0, st, sc.npred, sc.pbase, nseg, sc.total_pred);
        hipLaunchKernelGGL(k_verify<false>, dim3(vb), dim3(256), 0, st, rx, rx_len, segs, nseg, sc.mid, sc.pbase,
                           sc.total_pred, sc.first_fail, sc.last_masked, bases, fr, vmask);
    };
    auto emit = [&](int emit_counts, dframes fr) -> hipError_t {
        hipLaunchKernelGGL(k_head<true>, dim3(wb), dim3(SCAN_THREADS), 0, st, rx, rx_len, segs, nseg, carry_in,
                           sc.mid, sc.npred, sc.first_fail, sc.last_masked, bases, fr, vmask, spec_min(),
                           (uint64_t*)nullptr, (const dseg*)nullptr, (const dcarry*)nullptr, (dseg*)nullptr,
                           (dcarry*)nullptr, 0, (uint64_t)0, (uint64_t*)nullptr, 0u, (drun*)nullptr, (uint32_t*)nullptr);
        hipLaunchKernelGGL(k_verify<true>, dim3(vb), dim3(256), 0, st, rx, rx_len, segs, nseg, sc.mid, sc.pbase,
                           sc.total_pred, sc.first_fail, sc.last_masked, bases, fr, vmask);
        if (sieve) {
            const hipError_t e = launch_sieve_emit(rx, rx_len, segs, sc.mid, *sc.sieve, fr, vmask, st);
            if (e != hipSuccess) return e;
        }
        hipLaunchKernelGGL(k_walk<true>, dim3(wwb), dim3(SCAN_THREADS), 0, st, rx, rx_len, segs, nseg, sc.mid,
                           sc.npred, sc.first_fail, sc.last_masked, carry_out, counts, bases, fr, vmask, emit_counts,
                           sv, sv_S, (const dcarry*)nullptr);
        return hipSuccess;
    };
    // One-walk passes (SPEC, SLACK) when the last check saw no long uniform
    // run: k_head<false> alone (no k_verify pair, no npred scan), then the
    // walk also writes the carried-in frame's record, so no k_head<true>:
    // 4 kernels fewer.  The walk is exact whatever the segments hold.
    auto head_walk = [&](uint64_t* est, dframes fr) {
        hipLaunchKernelGGL(k_head<false>, dim3(wb), dim3(SCAN_THREADS), 0, st, rx, rx_len, segs, nseg, carry_in,
                           sc.mid, sc.npred, sc.first_fail, sc.last_masked, bases, fr, vmask, spec_min(), est,
                           sc.src_segs, sc.src_carry, sc.segs_w, sc.carry_w, 0,
                           pass == SCAN_SLACK ? sc.slack_cap : (uint64_t)0,
                           pass == SCAN_SLACK ? sc.est_u : (uint64_t*)nullptr, HEAD_ZERO_LM | HEAD_NO_VERIFY,
                           (drun*)nullptr, (uint32_t*)nullptr);
        hipLaunchKernelGGL(k_offsets, dim3(1), dim3(ONE_BLOCK), 0, st, est, bases, nseg, total);
        hipLaunchKernelGGL(k_walk<true>, dim3(wwb), dim3(SCAN_THREADS), 0, st, rx, rx_len, segs, nseg, sc.mid,
                           sc.npred, sc.first_fail, sc.last_masked, carry_out, counts, bases, fr, vmask, 1,
                           (const dsieve*)nullptr, (const uint64_t*)nullptr, carry_in);
    };
    if (pass == SCAN_SINGLE) {
        head_count(nullptr);
        hipError_t e;
        if (sieve && (e = launch_sieve(rx, rx_len, segs, sc.mid, sc.npred, *sc.sieve, st)) != hipSuccess) return e;
        if ((e = hipMemsetAsync(bases, 0, (size_t)nseg * 8, st)) != hipSuccess) return e;
        if ((e = emit(1, fr)) != hipSuccess) return e;
        hipLaunchKernelGGL(k_offsets, dim3(1), dim3(ONE_BLOCK), 0, st, counts, bases, nseg, total);
    } else if (pass == SCAN_SPEC) {
        if (sc.no_verify) {
            head_walk(sc.est, fr);
        } else {
            head_count(sc.est);
            hipLaunchKernelGGL(k_offsets, dim3(1), dim3(ONE_BLOCK), 0, st, sc.est, bases, nseg, total);
            if (hipError_t e = emit(1, fr); e != hipSuccess) return e;
        }
        hipLaunchKernelGGL(k_spec_check<true>, dim3(1), dim3(ONE_BLOCK), 0, st, counts, sc.est, sc.npred, nseg, total,
                           fr.cap, sc.status, sc.seq);
    } else if (pass == SCAN_COUNT) {
        head_count(sc.status ? sc.est : nullptr);
        hipLaunchKernelGGL(k_walk<false>, dim3(wwb), dim3(SCAN_THREADS), 0, st, rx, rx_len, segs, nseg, sc.mid,
                           sc.npred, sc.first_fail, sc.last_masked, carry_out, counts, bases, fr, vmask, 0,
                           (const dsieve*)nullptr, (const uint64_t*)nullptr, (const dcarry*)nullptr);
        hipLaunchKernelGGL(k_offsets, dim3(1), dim3(ONE_BLOCK), 0, st, counts, bases, nseg, total);
        if (sc.status)
            hipLaunchKernelGGL(k_spec_check<false>, dim3(1), dim3(ONE_BLOCK), 0, st, counts, sc.est, sc.npred, nseg, total,
                               fr.cap, sc.status, sc.seq);
    } else if (pass == SCAN_RUN) {
        const uint32_t rcap = run_scan_grid();
        hipLaunchKernelGGL(k_head<false>, dim3(rcap && rcap < wb ? rcap : wb), dim3(SCAN_THREADS), 0, st, rx, rx_len,
                           segs, nseg, carry_in,
                           sc.mid, sc.npred, sc.first_fail, sc.last_masked, bases, fr, vmask, spec_min(),
                           (uint64_t*)nullptr, sc.src_segs, sc.src_carry, sc.segs_w, sc.carry_w, 0, (uint64_t)0,
                           (uint64_t*)nullptr, HEAD_ZERO_LM | HEAD_NO_VERIFY, sc.runs, sc.run_fail);
        if (hipError_t e = launch_run_tiles(rx, rx_len, segs, nseg, sc.runs, sc.run_trun, sc.run_ntiles, sc.run_tile,
                                            sc.run_fail, st);
            e != hipSuccess)
            return e;
    } else if (pass == SCAN_SLACK) {
        if (sc.no_verify) {
            head_walk(sc.est, sc.slack);
        } else {
            head_count(sc.est);
            hipLaunchKernelGGL(k_offsets, dim3(1), dim3(ONE_BLOCK), 0, st, sc.est, bases, nseg, total);
            if (hipError_t e = emit(1, sc.slack); e != hipSuccess) return e;
        }
        hipLaunchKernelGGL(k_slack_check, dim3(1), dim3(ONE_BLOCK), 0, st, counts, sc.est, sc.est_u, sc.npred, nseg, sc.bases_x,
                           total, fr.cap, sc.status, sc.seq);
        hipLaunchKernelGGL(k_slack_compact, dim3(nseg < 65535u ? nseg : 65535u), dim3(256), 0, st, sc.slack, fr, counts,
                           bases, sc.bases_x, total, nseg);
    } else {
        if (hipError_t e = emit(0, fr); e != hipSuccess) return e;
    }
    return hipGetLastError();
}

hipError_t launch_offsets(const uint64_t* counts, uint64_t* bases, uint32_t nseg, uint64_t* total,
                          hipStream_t st) {
    hipLaunchKernelGGL(k_offsets, dim3(1), dim3(ONE_BLOCK), 0, st, counts, bases, nseg, total);
    return hipGetLastError();
}

hipError_t launch_tile_index(const uint64_t* off, const uint64_t* len, uint64_t nfr, const uint64_t* nfr_dev,
                             uint32_t* tile_first, uint64_t ntiles, uint64_t tile, hipStream_t st) {
    const uint64_t n = ntiles + 1;
    hipError_t e = hipMemsetAsync(tile_first, 0xFF, n * 4, st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_tile_scatter, dim3(2048), dim3(256), 0, st, off, len, nfr, nfr_dev, tile_first, ntiles, tile);
    const uint32_t blocks = (uint32_t)((n + 255) / 256);
    hipLaunchKernelGGL(k_tile_fixup, dim3(blocks), dim3(256), 0, st, off, len, nfr, nfr_dev, tile_first, ntiles, tile);
    return hipGetLastError();
}

hipError_t launch_tile_fixup(const uint64_t* off, const uint64_t* len, uint64_t nfr, uint32_t* tile_first,
                             uint64_t ntiles, uint64_t tile, hipStream_t st) {
    const uint32_t blocks = (uint32_t)((ntiles + 1 + 255) / 256);
    hipLaunchKernelGGL(k_tile_fixup, dim3(blocks), dim3(256), 0, st, off, len, nfr, (const uint64_t*)nullptr, tile_first,
                       ntiles, tile);
    return hipGetLastError();
}

hipError_t launch_unmask_tiles(const uint64_t* off, const uint64_t* len, const uint32_t* keyrot, const uint64_t* nfr_dev,
                               uint32_t* tile_first, uint32_t* tile_key, uint8_t* tile_kind, uint64_t ntiles,
                               uint64_t tile, uint64_t rx_len, hipStream_t st) {
    const uint64_t n = ntiles + 1;
    // no fill: k_tile_fix_class checks every entry (see there)
    hipLaunchKernelGGL(k_tile_scatter, dim3(2048), dim3(256), 0, st, off, len, (uint64_t)0, nfr_dev, tile_first,
                       ntiles, tile);
    const uint64_t nb = (n + 255) / 256;
    const uint32_t blocks = nb > 65536u ? 65536u : (uint32_t)nb;
    hipLaunchKernelGGL(k_tile_fix_class, dim3(blocks), dim3(256), 0, st, off, len, keyrot, nfr_dev, tile_first,
                       tile_key, tile_kind, ntiles, tile, rx_len);
    return hipGetLastError();
}

hipError_t launch_tile_class(const uint64_t* off, const uint64_t* len, const uint32_t* keyrot, const uint64_t* nfr_dev,
                             const uint32_t* tile_first, uint32_t* tile_key, uint8_t* tile_kind, uint64_t ntiles,
                             uint64_t tile, uint64_t rx_len, hipStream_t st) {
    if (ntiles == 0) return hipSuccess;
    const uint32_t blocks = (uint32_t)((ntiles + 255) / 256);
    hipLaunchKernelGGL(k_tile_class, dim3(blocks), dim3(256), 0, st, off, len, keyrot, nfr_dev, tile_first, tile_key,
                       tile_kind, ntiles, tile, rx_len);
    return hipGetLastError();
}

// Unmask geometries (threads, chunks per thread, XCD order): the two the
// batch size picks between.  Rounds 1-5 swept ten more (128 x 2 ... 1024 x 1,
// 64 x 8, 256 x 8, linear and XCD orders; profiles/r2c_raw, r2l_raw); none
// won anywhere, and round 6 removed them.  hvws_set_unmask_variant (tests,
// bench.py --sweep-unmask) or $HVWS_EXPERIMENT unmask=<index> forces one.
struct unmask_geom {
    int threads, unroll;
    bool swz;
};
// X(index, threads, chunks per thread, XCD order)
#define HVWS_UNMASK_GEOMS(X)                                                              \
    X(0, 256, 4, true)                                                                    \
    X(1, 512, 2, false)
#define HVWS_GEOM_ENTRY(i, t, u, s) {t, u, s},
static const unmask_geom kGeoms[] = {HVWS_UNMASK_GEOMS(HVWS_GEOM_ENTRY)};

// Geometry by batch size unless one is chosen ($HVWS_EXPERIMENT unmask, or
// hvws_set_unmask_variant; -1 = back to this choice).  Pipelined steps,
// interleaved runs on one box (profiles/r2l_raw): 512 x 2 in linear tile
// order against the XCD-contiguous 256 x 4 -- c2 (1 GiB) 0.4195 vs 0.425
// ms/step, c4 (4.3 GB, 1024 segments) 1.383 vs 1.510 ms; at c3 (68.7 GB) the
// XCD-contiguous order wins, 20.92 vs 22.76 ms.  The single-step sweep over
// uniform batches (profiles/r2c_raw/size_sweep.jsonl) puts the crossover at
// 16 GiB.
constexpr int kGeomSmall = 1;                         // 512 x 2, linear
constexpr int kGeomLarge = 0;                         // 256 x 4, XCD-contiguous
constexpr uint64_t kGeomLinearMax = 16ull << 30;     // bytes

static int g_geom_forced = -2;   // -2: not yet read from the environment; -1: by size

static int forced_geom() {
    if (g_geom_forced == -2) {
        const char* e = experiment("unmask");
        int v = e ? atoi(e) : -1;
        if (v < -1 || v >= (int)(sizeof(kGeoms) / sizeof(kGeoms[0]))) v = -1;
        g_geom_forced = v;
    }
    return g_geom_forced;
}

int unmask_variant() {
    const int f = forced_geom();
    return f >= 0 ? f : kGeomLarge;
}

int unmask_variant_for(uint64_t rx_len) {
    const int f = forced_geom();
    if (f >= 0) return f;
    return rx_len < kGeomLinearMax ? kGeomSmall : kGeomLarge;
}

int set_unmask_variant(int v) {
    if (v < -1 || v >= (int)(sizeof(kGeoms) / sizeof(kGeoms[0]))) return -2;
    (void)forced_geom();
    g_geom_forced = v;
    return v;
}

int unmask_variant_count() { return (int)(sizeof(kGeoms) / sizeof(kGeoms[0])); }

uint64_t unmask_tile(int variant) {
    const unmask_geom& g = kGeoms[variant];
    return (uint64_t)g.threads * g.unroll * 16u;
}

const char* unmask_name(int variant) {
    static char buf[16][48];
    const unmask_geom& g = kGeoms[variant];
    snprintf(buf[variant & 15], sizeof(buf[0]), "k_unmask<%d,%d,%s>", g.threads, g.unroll, g.swz ? "xcd" : "linear");
    return buf[variant & 15];
}

#define HVWS_GEOM_CASE(i, t, u, s) \
    case i: hipLaunchKernelGGL((HVWS_K<t, u, s>), HVWS_ARGS); break;
// A launch may hold at most 2^32-1 work-items (and 2^31-1 workgroups); a
// larger grid is split into several launches over consecutive tile ranges
// (each keeps its own XCD order).  Never let the runtime truncate a grid.
static uint64_t max_tiles_per_launch(int threads) {
    const uint64_t by_items = 0xFFFFFFFFull / (uint64_t)threads;
    return by_items < 0x7FFFFFFFull ? by_items : 0x7FFFFFFFull;
}

#define HVWS_GEOM_CASE_EXT(i, t, u, s) \
    case i: hipExtLaunchKernelGGL((HVWS_K<t, u, s>), HVWS_EXT_ARGS); break;

hipError_t launch_unmask(int variant, uint8_t* rx, uint64_t rx_len, dframes fr, const uint32_t* tile_first,
                         const uint32_t* tile_key, const uint8_t* tile_kind, const uint64_t* nfr_dev, hipStream_t st,
                         uint32_t pieces, hipEvent_t ev_start, hipEvent_t ev_stop) {
    if (rx_len == 0) return hipSuccess;
    if (variant < 0 || variant >= unmask_variant_count()) return hipErrorInvalidValue;
    const uint64_t tile = unmask_tile(variant);
    const uint64_t ntiles_all = (rx_len + tile - 1) / tile;
    const int threads = kGeoms[variant].threads;
    // pieces > 1: several launches over consecutive tile ranges, so kernels
    // queued on another stream (the next batch's discovery) are dispatched
    // between them instead of after the whole grid.
    uint64_t cap = max_tiles_per_launch(threads);
    if (pieces > 1) {
        const uint64_t per = (ntiles_all + pieces - 1) / pieces;
        cap = per < cap ? (per ? per : 1) : cap;
    }
    // Timing events ride on the dispatch packets themselves (start of the
    // first launch, end of the last): a separate hipEventRecord marker
    // between the tile kernels and the unmask cost ~12 us of idle device per
    // pipelined c2 step (profiles/r2g_raw).
    for (uint64_t tile0 = 0; tile0 < ntiles_all; tile0 += cap) {
        const uint64_t ntiles = ntiles_all - tile0 < cap ? ntiles_all - tile0 : cap;
        const hipEvent_t e0 = tile0 == 0 ? ev_start : nullptr;
        const hipEvent_t e1 = tile0 + ntiles >= ntiles_all ? ev_stop : nullptr;
#define HVWS_K k_unmask
#define HVWS_ARGS dim3((uint32_t)ntiles), dim3(threads), 0, st, rx, rx_len, fr.pay_off, fr.pay_len, \
                  fr.keyrot, tile_first, tile_key, tile_kind, nfr_dev, tile0, ntiles
#define HVWS_EXT_ARGS dim3((uint32_t)ntiles), dim3(threads), 0, st, e0, e1, 0u, rx, rx_len, fr.pay_off, \
                      fr.pay_len, fr.keyrot, tile_first, tile_key, tile_kind, nfr_dev, tile0, ntiles
        if (e0 || e1) {
            switch (variant) { HVWS_UNMASK_GEOMS(HVWS_GEOM_CASE_EXT) default: return hipErrorInvalidValue; }
        } else {
            switch (variant) { HVWS_UNMASK_GEOMS(HVWS_GEOM_CASE) default: return hipErrorInvalidValue; }
        }
#undef HVWS_K
#undef HVWS_ARGS
#undef HVWS_EXT_ARGS
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

hipError_t launch_run_tiles(const uint8_t* rx, uint64_t rx_len, const dseg* segs, uint32_t nseg, const drun* runs,
                            dtrun* trun, uint64_t ntiles, uint64_t tile, uint32_t* fail, hipStream_t st) {
    const uint32_t rcap = run_scan_grid();
    const uint32_t nb1 = (nseg + 3) / 4;   // one wave per segment
    const uint32_t nb = rcap && rcap < nb1 ? rcap : nb1;
    if (nb && ntiles) hipLaunchKernelGGL(k_run_tiles, dim3(nb), dim3(256), 0, st, rx, rx_len, segs, nseg, runs, trun,
                                         ntiles, tile, fail);
    return hipGetLastError();
}

// The RUN unmask: 256 threads x 4 chunks per 16 KiB tile, the tile staged
// in LDS for the header reads (c2 0.380-0.382 ms per step against 0.386-0.387
// reading them from HBM; 512 x 2, 256 x 2, 128 x 4 and 64 x 4 all lost,
// profiles/r5_raw/sweeps/*_r5l-r5x.json; those geometries were removed in
// round 6).
const char* run_kernel_name() { return "k_unmask_run<256,4,lds>"; }

hipError_t launch_unmask_run(uint8_t* rx, uint64_t rx_len, const drun* runs, const dtrun* trun, uint32_t nseg,
                             uint32_t* fail, dspec_status* status, uint64_t seq, hipStream_t st, hipEvent_t ev_start,
                             hipEvent_t ev_stop) {
    if (rx_len == 0 || nseg == 0) return hipSuccess;
    constexpr int T = 256, U = 4;
    static_assert((uint64_t)T * U * 16u == RUN_TILE, "RUN tile");
    const uint64_t ntiles_all = (rx_len + RUN_TILE - 1) / RUN_TILE;
    // The grid in two launches: c2 0.375-0.376 ms per step against 0.377-0.379
    // in one, 0.378-0.379 in three, 0.383-0.385 in four (interleaved on one box,
    // profiles/r5_raw/sweeps/*_r5za.json).
    constexpr uint64_t pieces = 2;
    const uint64_t cap = std::min<uint64_t>(max_tiles_per_launch(T), (ntiles_all + pieces - 1) / pieces);
    for (uint64_t tile0 = 0; tile0 < ntiles_all; tile0 += cap) {
        const uint64_t ntiles = ntiles_all - tile0 < cap ? ntiles_all - tile0 : cap;
        if (tile0 == 0 && ev_start)
            hipExtLaunchKernelGGL((k_unmask_run<T, U>), dim3((uint32_t)ntiles), dim3(T), 0, st, ev_start, nullptr, 0u, rx,
                                  rx_len, runs, trun, nseg, fail, tile0);
        else
            hipLaunchKernelGGL((k_unmask_run<T, U>), dim3((uint32_t)ntiles), dim3(T), 0, st, rx, rx_len, runs, trun, nseg,
                               fail, tile0);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    if (ev_stop)
        hipExtLaunchKernelGGL(k_run_fix, dim3(RUN_FIX_BLOCKS), dim3(256), 0, st, nullptr, ev_stop, 0u, rx, rx_len, runs,
                              nseg, fail, status, seq);
    else
        hipLaunchKernelGGL(k_run_fix, dim3(RUN_FIX_BLOCKS), dim3(256), 0, st, rx, rx_len, runs, nseg, fail, status, seq);
    return hipGetLastError();
}

hipError_t launch_stream_xor(int variant, uint8_t* d, uint64_t n, uint32_t pattern, hipStream_t st) {
    if (variant < 0 || variant >= unmask_variant_count()) return hipErrorInvalidValue;
    const uint64_t tile = unmask_tile(variant);
    const uint64_t ntiles_all = (n + tile - 1) / tile;
    const int threads = kGeoms[variant].threads;
    const uint64_t cap = max_tiles_per_launch(threads);
    for (uint64_t tile0 = 0; tile0 < ntiles_all; tile0 += cap) {
        const uint64_t ntiles = ntiles_all - tile0 < cap ? ntiles_all - tile0 : cap;
#define HVWS_K k_stream_xor
#define HVWS_ARGS dim3((uint32_t)ntiles), dim3(threads), 0, st, d, n, tile0, ntiles, pattern
        switch (variant) { HVWS_UNMASK_GEOMS(HVWS_GEOM_CASE) default: return hipErrorInvalidValue; }
#undef HVWS_K
#undef HVWS_ARGS
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    return hipSuccess;
}

// An empty launch: the HIP runtime keeps the buffers named by the last kernel
// dispatched on a stream referenced until another kernel is dispatched there,
// so hipFree of such a buffer does not return its memory (profiles/r3c_raw:
// 68.7 GB held after hvws_digest / hvws_step).  hvws_dev_free issues one on
// each of the context's streams first.
__global__ void k_noop() {}

hipError_t launch_noop(hipStream_t st) {
    hipLaunchKernelGGL(k_noop, dim3(1), dim3(64), 0, st);
    return hipGetLastError();
}

hipError_t launch_xor_span(uint8_t* d, uint64_t n, uint32_t key, uint32_t phase, hipStream_t st) {
    if (n == 0) return hipSuccess;
    uint64_t chunks = (n + 15) / 16;
    uint32_t blocks = (uint32_t)((chunks + 255) / 256);
    if (blocks > 8192u) blocks = 8192u;
    hipLaunchKernelGGL(k_xor_span, dim3(blocks), dim3(256), 0, st, d, n, key, phase);
    return hipGetLastError();
}

}  // namespace hvws

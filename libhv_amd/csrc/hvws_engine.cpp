// hvws_engine.cpp -- host side of the MI355X WebSocket receive engine:
// per-(thread, device) contexts, frame-table management, kernel sequencing,
// and the C ABI declared in include/hvws.h and include/hvws_synth.h.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <dirent.h>
#include <immintrin.h>
#include <execinfo.h>
#include <signal.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <vector>
#include <mutex>
#include <shared_mutex>
#include <atomic>

#include "hvws.h"
#include "hvws_internal.h"
#include "hvws_synth.h"

using namespace hvws;

namespace {

thread_local char g_err[512] = "";

int set_err(int code, const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
    return code;
}

#define HIP_OR(expr, code)                                                              \
    do {                                                                                \
        hipError_t e_ = (expr);                                                         \
        if (e_ != hipSuccess)                                                           \
            return set_err((code), "%s: %s (%s:%d)", #expr, hipGetErrorString(e_), __FILE__, \
                           __LINE__);                                                   \
    } while (0)

// The runtime's frees (hipFree, hipHostFree, hipHostUnregister) wait for
// every stream of the device -- a resident k_door worker's too, until it
// parks.  Every free here first parks every worker on the current device,
// whichever thread owns it (defined with the worker).
void door_park_device();

// Grow-only device allocation.
struct dbuf {
    void* p = nullptr;
    uint64_t cap = 0;
    hipError_t ensure(uint64_t bytes) {
        if (bytes <= cap && p) return hipSuccess;
        if (p) {
            door_park_device();
            hipFree(p);
        }
        p = nullptr;
        cap = 0;
        uint64_t want = std::max<uint64_t>(bytes + bytes / 2, 4096);
        hipError_t e = hipMalloc(&p, want);
        if (e == hipSuccess) cap = want;
        return e;
    }
    void release() {
        if (p) {
            door_park_device();
            hipFree(p);
        }
        p = nullptr;
        cap = 0;
    }
    template <typename T>
    T* as() const { return reinterpret_cast<T*>(p); }
};

struct hbuf {   // grow-only pinned host allocation
    void* p = nullptr;
    void* dev = nullptr;   // its device-mapped address, looked up once per allocation
    uint64_t cap = 0;
    unsigned flags = hipHostMallocDefault;   // hipHostMallocCoherent: device reads/writes bypass its caches
    hipError_t ensure(uint64_t bytes) {
        if (bytes <= cap && p) return hipSuccess;
        if (p) {
            door_park_device();
            hipHostFree(p);
        }
        p = nullptr;
        dev = nullptr;
        cap = 0;
        uint64_t want = std::max<uint64_t>(bytes + bytes / 2, 4096);
        hipError_t e = hipHostMalloc(&p, want, flags);
        if (e == hipSuccess) cap = want;
        return e;
    }
    void release() {
        if (p) {
            door_park_device();
            hipHostFree(p);
        }
        p = nullptr;
        dev = nullptr;
        cap = 0;
    }
    template <typename T>
    T* as() const { return reinterpret_cast<T*>(p); }
};

}  // namespace

namespace hvws {
hvws_ctx* thread_ctx();
[[noreturn]] void fatal(const char* what);
}

static_assert(sizeof(drec) == sizeof(hvws_frame), "drec mirrors hvws_frame");
static_assert(sizeof(dsmall_out) == 64, "dsmall_out layout");

// What one scan produces (frame table, tile index, per-segment results and
// scratch); the context holds two.
struct tset {
    dbuf carry_out, counts, bases, total;
    dbuf sc_mid, sc_npred, sc_pbase, sc_fail, sc_masked, sc_total, sc_est;
    dbuf f_hdr, f_off, f_len, f_length, f_key, f_keyrot, f_info;
    dbuf tile_first, tile_key, tile_kind;
    dbuf runs, run_fail, run_trun;   // RUN path: per-segment run descriptors, failure words, per-tile records
    uint64_t frame_cap = 0;
    hipEvent_t free_ev = nullptr;   // recorded after the last kernel reading the set (pipelined steps)
    hipEvent_t free_wait = nullptr; // what the next scan into the set waits for: free_ev, or the stop
                                    // event attached to the unmask's own dispatch (no marker packet)
    bool free_pending = false;
    void release() {
        for (dbuf* b : {&carry_out, &counts, &bases, &total, &sc_mid, &sc_npred, &sc_pbase, &sc_fail, &sc_masked,
                        &sc_total, &sc_est, &f_hdr, &f_off, &f_len, &f_length, &f_key, &f_keyrot, &f_info,
                        &tile_first, &tile_key, &tile_kind, &runs, &run_fail, &run_trun})
            b->release();
        frame_cap = 0;
    }
};

struct hvws_ctx {
    int device = 0;
    hipStream_t stream = nullptr;    // compute
    hipStream_t copy_in = nullptr;   // pipeline H2D
    hipStream_t copy_out = nullptr;  // pipeline D2H
    // Pipelined steps (hvws_step_resident): discovery on sstream, overlapping
    // the previous batch's unmask on `stream`.  cs = the stream the current
    // scan enqueues on.
    hipStream_t sstream = nullptr;
    hipStream_t cs = nullptr;
    hipEvent_t scan_done = nullptr;
    bool piped = false;   // the last step was pipelined (set free events are being kept)
    // per-batch tables: the segment/carry tables the scan reads, and two
    // sets of everything a scan produces, used in turn, so a batch's scan
    // can run while the previous batch's unmask still reads its tables
    dbuf segs, carry_in;
    tset ts[2];
    int cur = 0;
    tset& T() { return ts[cur]; }
    hbuf h_segs, h_total;
    // Segment/carry upload staging: two pinned slots used in turn, each
    // reusable once the H2D copy that read it has run (event), so a step
    // never waits for the previous step's kernels.
    // The scan's first kernel reads the slot through its device mapping (no
    // copy); up_src_* point at the slot the next scan is to read.
    hbuf h_up[2];
    hipEvent_t up_ev[2] = {nullptr, nullptr};
    bool up_pending[2] = {false, false};
    int up_next = 0;
    int up_slot = -1;
    const dseg* up_src_segs = nullptr;
    const dcarry* up_src_carry = nullptr;
    // Speculative EMIT (SCAN_SPEC): per-segment estimates, the device's
    // verdict in pinned memory, and whether the last exact scan says the
    // estimates hold (then the next batch speculates).
    hbuf h_status;
    uint64_t scan_seq = 0;
    bool spec_ok = false;
    // The last check saw a segment with >= spec_min predicted frames: the
    // next one-walk pass keeps the grid-wide k_verify pair (else head + walk).
    bool verify_hint = true;
    int verify_mode = -1;   // hvws_set_walk_verify: -1 adaptive (the hint), 0 never, 1 always
    int spec_mode = -1;   // -1 auto, 0 never, 1 SPEC first, 2 SLACK first ($HVWS_EXPERIMENT spec / hvws_set_speculation)
    // SLACK (mixed sizes, several segments): scratch table, exact bases, and
    // the per-segment region cap from the last exact scan's largest segment
    dbuf sl_hdr, sl_off, sl_len, sl_length, sl_key, sl_keyrot, sl_info, sl_bx;
    uint64_t sl_cap = 0;       // records the scratch table holds
    uint64_t slack_seg = 0;    // largest per-segment count of the last exact scan (0 = unknown)
    uint64_t fast_bound = 0;   // record bound below which COUNT -> EMIT needs no host wait; 0 = default
    int scan_path = -1;        // HVWS_PATH_* of the last scan
    int prev_path = -1;        // ... and of the one before (set when a scan starts)
    uint64_t single_hint = 0;  // records of the last one-segment scan whose count was read
    // RUN path (hvws_internal.h, drun): the last scan left no frame table (its
    // records are built on demand), its unmask is k_unmask_run + k_run_fix
    bool run_active = false;
    bool materializing = false;   // run_materialize's exact scan: no timing slot, no RUN bookkeeping
    bool run_call = false;     // the scan belongs to a step call (the only callers RUN serves)
    int run_mode = -1;         // hvws_set_run: -1 auto, 0 never, 1 whenever a step's batch allows it
    uint32_t run_skip = 0;     // steps left before RUN is tried again after a failed hypothesis
    uint64_t run_seq = 0;      // the current RUN step's verdict number
    uint64_t run_seen = 0;     // the last verdict read (status pad3)
    uint64_t last_mean = 0;    // bytes per record of the last exact (or SPEC) scan: RUN is for small frames
    // frame sieve (hvws_sieve.hip): one long mixed-size segment discovered in
    // parallel.  h_sv receives the device state + survivor and chain counts
    // after each sieved scan (read as hints by the next one).
    dbuf sv_state, sv_tcount, sv_tbase, sv_slot, sv_pool, sv_keep, sv_kbase, sv_Spre, sv_S, sv_J0, sv_J1, sv_mark, sv_hops, sv_rank, sv_cnt, sv_tmp, sv_scr;
    uint64_t sv_cap = 0, sv_capc = 0;
    uint64_t sv_hint_pre = 0, sv_hint_surv = 0;   // counts of the latest sieved scan read back
    hbuf h_sv;
    uint32_t sv_skip = 0;      // one-stream scans left before the sieve is tried again on uniform traffic
    bool sv_ran = false;       // the last scan launched the sieve
    hipEvent_t sv_ev = nullptr;   // h_sv holds the last sieved scan's state once this has completed
    uint64_t sv_gen = 0;       // sieve_generation() the history below belongs to
    uint64_t sv_win_len = 0;   // segment length of the last sieved scan if it sieved windows only, else 0
    uint32_t sv_full_left = 0; // scans left that sieve every tile (a windowed chain fell short)
    uint32_t sv_rt = 0, sv_wt = 0;   // window geometry of the last sieved scan (tiles)
    bool sv_hint_win = false;  // sv_hint_* come from a windowed scan
    uint64_t sv_mean = 0;      // bytes per frame along the last sieved chain (0: none yet)
    // hvws_pipeline: its three device slots and their events, kept across
    // calls (a per-call hipMalloc/hipFree pair cost the first call ~2x)
    dbuf pipe_slot[3], pipe_segs;
    hipEvent_t pipe_ev[9] = {};
    // staging for host-memory entry points
    dbuf stage;
    dbuf xor_stage;
    dbuf synth_sizes, synth_tiles, synth_bad;
    // small-batch path (k_small): upload packet, record slots, pinned results
    hbuf h_small_in, h_small_out;
    hbuf h_small_done;             // per-segment completion words k_small writes last
    uint64_t small_seq = 0;        // value the current call's completion words carry
    int small_poll = 1;            // $HVWS_EXPERIMENT small_poll: poll those words instead of syncing the stream
    bool small_quiet = false;      // the last small call saw all its words: its kernel no longer touches the pinned buffers
    hbuf h_feed;   // hvws_feed_many's gather buffer (reference-API thread contexts)
    dbuf d_small_in, d_small_slots;
    uint64_t small_limit = 0;   // bytes; 0 = default
    // k_small's record counter lives on the device and only ever grows; a
    // call's records start at small_ctr_base
    dbuf d_small_ctr;
    uint64_t small_ctr_base = 0;
    bool small_ctr_dirty = true;   // unknown value (first use, failed call): zero it
    int small_zc = 1;              // $HVWS_EXPERIMENT small_zc / hvws_set_small_zero_copy
    uint64_t zc_batch = kZcBatch;  // largest zero-copy batch ($HVWS_EXPERIMENT zc_batch)
    uint32_t vmask = 0;         // protocol validation classes (V_*); 0 = reference behaviour
    // transmit side (hvws_build_frames)
    dbuf tx_size, tx_off, tx_scan, tx_tiles, tx_stat, tx_span;
    hbuf h_tx;
    bool ev_build = false;
    int tx_variant = 0;   // k_build geometry of the last hvws_build_frames
    bool tx_uniform = false;   // ... and whether it built a uniform layout without a tile index
    // last scan
    uint32_t nseg = 0;
    uint64_t nfr = 0;
    uint64_t rx_len = 0;
    const uint8_t* rx = nullptr;
    bool have_scan = false;
    hipEvent_t ev[6] = {nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};   // [4], [5]: build / keys
    // Per-step timing: scan begin/end and unmask begin/end events for the
    // last kTimeRing steps, read after the fact (hvws_step_times) so a caller
    // timing many steps need not synchronise after each.
    static constexpr int kTimeRing = 32;
    hipEvent_t tev[kTimeRing][4] = {};
    bool t_unmask[kTimeRing] = {};
    uint8_t t_rec[kTimeRing] = {};      // which of the slot's 4 events were recorded (bit i)
    uint64_t t_seq = 0;   // scans recorded so far
    int t_cur = 0;        // ring slot of the last scan
    uint32_t t_every = 1; // hvws_set_step_event_interval: events on every t_every-th scan (0: none)
    bool t_on = true;     // the current scan is one of them
    // resident small-path worker (k_door): its own HSA queue (a dedicated
    // hardware queue, so the resident kernel never holds up other work;
    // hvws_doorq.cpp), the mailbox, the data and record areas (fine-grained
    // pinned) and a device slot for records past the worker's LDS area
    door_queue* door_q = nullptr;
    hbuf h_door, h_door_data, h_door_rec;
    dbuf d_door_slot;
    // Request block + request bytes in fine-grained device memory, written by
    // the host through the PCIe BAR (round 4): the worker polls and stages
    // from its own HBM instead of pulling them across the link.  nullptr: the
    // request and its bytes go through the pinned box and data area (round 3).
    void* d_door_req = nullptr;
    bool door_live = false;     // launched and not yet seen to have ended
    bool door_wedged = false;   // its launch ran on past every bound: queue and mailbox are left alone
    bool door_broken = false;   // a request went unanswered: this context launches per call from now on
    // The HIP runtime call this context's worker lifecycle or teardown is
    // in (nullptr: none): a wedge report or hvws_debug_dump names the call.
    std::atomic<const char*> at{nullptr};
    uint64_t door_seq = 0;      // last request number posted
    uint64_t door_epoch = 0;    // launches so far; the worker writes its epoch to `exited` as it ends
    std::mutex door_m;          // one caller at a time: the owning thread, a free on another thread, exit
    int door_mode = -1;         // hvws_set_door: -1 default ($HVWS_DOOR, on), 0 off, 1 on
    uint64_t door_launches = 0, door_calls = 0;
    // hvws_span_begin / hvws_span_end: a timed region's begin and end markers
    // on both of the context's compute streams
    hipEvent_t span_ev[4] = {};
    int variant = 0;   // k_unmask geometry the tile index was built for
    bool nfr_known = false;   // else c->nfr is an upper bound, the count is on the device
    // table invariant check (hvws_set_table_checks)
    dbuf chk;
    hbuf h_chk;
    // host copy of the last scan's results (readback_all)
    hbuf h_readback;
    bool hcache_valid = false;
    std::vector<hvws_frame> hcache;
    std::vector<uint64_t> hfirst, hcount;
    std::vector<dcarry> hcarry;
};

namespace {
constexpr uint64_t kFastFrameBound = 1ull << 24;   // records: table sized by the bound, no count sync
constexpr uint64_t kReadbackPrefix = 1ull << 16;   // records read back speculatively with the rest
constexpr uint64_t kSingleMin = 1ull << 20;   // records: smallest one-stream table before its count is known
constexpr uint64_t kSlackMaxRecords = 1ull << 26;   // SLACK scratch table at most (48 B each: 3.2 GB)
// Small-batch path (k_small): batches up to kSmallBatch bytes whose segments
// are each at most kSmallSegment bytes run as one launch.
constexpr uint64_t kSmallBatch = 64ull << 20;
constexpr uint64_t kSmallSegment = 1ull << 20;
constexpr uint64_t kSmallHostRecords = 1ull << 20;   // records returned through pinned memory
int g_table_checks = -1;   // -1: from $HVWS_CHECK_TABLES on first use
bool table_checks() {
    if (__atomic_load_n(&g_table_checks, __ATOMIC_RELAXED) < 0) {
        const char* e = getenv("HVWS_CHECK_TABLES");
        int want = e && atoi(e) ? 1 : 0, unset = -1;
        __atomic_compare_exchange_n(&g_table_checks, &unset, want, false, __ATOMIC_RELAXED, __ATOMIC_RELAXED);
    }
    return __atomic_load_n(&g_table_checks, __ATOMIC_RELAXED) > 0;
}
}  // namespace

namespace {

dframes frames_of(hvws_ctx* c) {
    dframes f;
    f.hdr_off = c->T().f_hdr.as<int64_t>();
    f.pay_off = c->T().f_off.as<uint64_t>();
    f.pay_len = c->T().f_len.as<uint64_t>();
    f.length = c->T().f_length.as<uint64_t>();
    f.key = c->T().f_key.as<uint32_t>();
    f.keyrot = c->T().f_keyrot.as<uint32_t>();
    f.info = c->T().f_info.as<uint32_t>();
    f.cap = c->T().frame_cap;
    return f;
}

hipError_t ensure_frames(hvws_ctx* c, uint64_t n, bool exact = false) {
    if (n <= c->T().frame_cap && c->T().f_off.p) return hipSuccess;
    uint64_t want = std::max<uint64_t>(exact ? n : n + n / 4, 1024);
    hipError_t e;
    if ((e = c->T().f_hdr.ensure(want * 8)) != hipSuccess) return e;
    if ((e = c->T().f_off.ensure(want * 8)) != hipSuccess) return e;
    if ((e = c->T().f_len.ensure(want * 8)) != hipSuccess) return e;
    if ((e = c->T().f_length.ensure(want * 8)) != hipSuccess) return e;
    if ((e = c->T().f_key.ensure(want * 4)) != hipSuccess) return e;
    if ((e = c->T().f_keyrot.ensure(want * 4)) != hipSuccess) return e;
    if ((e = c->T().f_info.ensure(want * 4)) != hipSuccess) return e;
    c->T().frame_cap = want;
    return hipSuccess;
}

void to_dcarry(const websocket_parser& p, dcarry& d) {
    d.state = p.state;
    d.flags = (uint32_t)p.flags;
    memcpy(&d.mask, p.mask, 4);
    d.mask_offset = p.mask_offset;
    d.length = p.length;
    d.require = p.require;
    d.offset = p.offset;
    d.started = 0;
    // Validation state of a partial header lives in the struct's padding
    // byte after mask_offset (offset 13), invisible to the reference API.
    d.viol = reinterpret_cast<const uint8_t*>(&p)[kViolByte];
}

void from_dcarry(const dcarry& d, websocket_parser& p) {
    p.state = d.state;
    p.flags = (websocket_flags)d.flags;
    memcpy(p.mask, &d.mask, 4);
    p.mask_offset = (uint8_t)d.mask_offset;
    p.length = d.length;
    p.require = d.require;
    p.offset = d.offset;
    reinterpret_cast<uint8_t*>(&p)[kViolByte] = (uint8_t)d.viol;
}

int check_ctx(hvws_ctx* c) {
    if (!c) return set_err(HVWS_EINVAL, "null context");
    HIP_OR(hipSetDevice(c->device), HVWS_EHIP);
    return HVWS_OK;
}

// Device address of a pinned host buffer.
template <typename T>
T* mapped(hbuf& b) {
    if (!b.dev && b.p && hipHostGetDevicePointer(&b.dev, b.p, 0) != hipSuccess) b.dev = nullptr;
    return reinterpret_cast<T*>(b.dev);
}

// Which per-step timing events are recorded: 2 = scan begin/end and unmask
// begin/end, 1 = the unmask's only, 0 = none.  Default: 2 for serial steps,
// 1 for pipelined ones (hvws_step_resident) -- each timing marker is a packet
// the command processor runs between kernels, and the scan-side pair cost a
// pipelined c2 step ~9 us (0.465 -> 0.456 ms, profiles/r2d_raw); a pipelined
// scan's span includes its wait for the previous unmask anyway.
// $HVWS_EXPERIMENT step_events forces a mode.
int step_events(const hvws_ctx* c) {
    static const int v = [] {
        const char* e = experiment("step_events");
        return e ? atoi(e) : -1;
    }();
    return v >= 0 ? v : (c->cs != c->stream ? 1 : 2);
}

// Record timing event i (0 scan begin, 1 scan end, 2 unmask begin, 3 unmask
// end) of the current ring slot if this mode keeps it.
hipError_t tev_record(hvws_ctx* c, int i, hipStream_t st) {
    const int m = step_events(c);
    if (!c->t_on || m <= 0 || (m == 1 && i < 2)) return hipSuccess;
    c->t_rec[c->t_cur] |= (uint8_t)(1u << i);
    return hipEventRecord(c->tev[c->t_cur][i], st);
}

// Next slot of the timing ring: record the scan-begin event there (unless
// the caller attaches the slot's events to a dispatch itself).
hipError_t begin_timed_scan(hvws_ctx* c, bool record = true) {
    c->t_cur = (int)(c->t_seq % hvws_ctx::kTimeRing);
    c->t_unmask[c->t_cur] = false;
    c->t_rec[c->t_cur] = 0;
    c->t_on = c->t_every != 0 && c->t_seq % c->t_every == 0;
    ++c->t_seq;
    return record ? tev_record(c, 0, c->cs) : hipSuccess;
}

// out[0] = scan ms, out[1] = unmask ms (-1: no unmask, or not recorded) of
// the step in ring `slot`.
int step_times_at(hvws_ctx* c, int slot, float* out) {
    hipEvent_t* e = c->tev[slot];
    const uint8_t r = c->t_rec[slot];
    out[0] = out[1] = -1.0f;
    if ((r & 3u) == 3u) {
        HIP_OR(hipEventSynchronize(e[1]), HVWS_EHIP);
        HIP_OR(hipEventElapsedTime(&out[0], e[0], e[1]), HVWS_EHIP);
    }
    if (c->t_unmask[slot] && (r & 4u) && (r & 8u)) {
        HIP_OR(hipEventSynchronize(e[3]), HVWS_EHIP);
        HIP_OR(hipEventElapsedTime(&out[1], e[2], e[3]), HVWS_EHIP);
    }
    return HVWS_OK;
}

// Wait until k_spec_check has published scan `seq` in the (fine-grained)
// pinned status: the device stores it with system-scope release as its last
// write, so the host polls it instead of a stream event (an event marker
// costs ~10 us of device idle between the check and the tile kernels).  A
// stream that drains without publishing is an error, never a hang.
// Pipelined SPEC steps queue the unmask after the host has seen the scan
// finish instead of behind a cross-stream event ($HVWS_EXPERIMENT host_order=0: the
// event, as in round 3).
// $HVWS_RUN=0: the RUN path off (A/B runs); hvws_set_run overrides per context.
bool run_env() {
    static const int v = getenv("HVWS_RUN") ? atoi(getenv("HVWS_RUN")) : 1;
    return v != 0;
}


// Pipelined steps: the host queues the unmask once the scan's last kernel
// has published (always since round 4; round 6 removed the switch back to a
// cross-stream event).
constexpr bool host_order() { return true; }

int wait_status(hvws_ctx* c, uint64_t seq, bool tiles = false) {
    const dspec_status* st = c->h_status.as<dspec_status>();
    const uint64_t* w = tiles ? &st->tseq : &st->seq;
    for (uint64_t spin = 0;; ++spin) {
        if (__atomic_load_n(w, __ATOMIC_ACQUIRE) == seq) return HVWS_OK;
        if ((spin & 1023) == 1023) {
            const hipError_t q = hipStreamQuery(c->cs);
            if (q == hipSuccess) {
                if (__atomic_load_n(w, __ATOMIC_ACQUIRE) == seq) return HVWS_OK;
                return set_err(HVWS_EHIP, "scan check did not publish (seq %llu)", (unsigned long long)seq);
            }
            if (q != hipErrorNotReady) return set_err(HVWS_EHIP, "stream error: %s", hipGetErrorString(q));
        }
        __builtin_ia32_pause();
    }
}

// The last sieved scan's state has landed in h_sv.
bool sieve_state_ready(hvws_ctx* c) { return c->sv_ran && c->sv_ev && hipEventQuery(c->sv_ev) == hipSuccess; }

// Frame-sieve buffers for a one-segment scan of rx_len bytes.  The survivor
// capacity is sized from the batch (one survivor per KiB) and from the last
// sieved scan's survivor count; a batch with more survivors than that leaves
// the sieve off (the exact walk runs) and the next one gets room.
int ensure_sieve(hvws_ctx* c, uint64_t rx_len, sieve_bufs& b) {
    const uint64_t* h = c->h_sv.as<uint64_t>();
    // entries before HBM verification, and survivors, of the latest sieved
    // scan whose state has landed (pipelined steps run ahead of it)
    if (sieve_state_ready(c)) {
        const uint64_t pre = h[sizeof(dsieve) / 8 + 3], surv = h[sizeof(dsieve) / 8];
        const bool counted = surv <= pre && pre <= c->sv_cap;   // else it overflowed and never counted survivors
        c->sv_hint_pre = pre;
        c->sv_hint_surv = counted ? surv : 0;
        // A windowed chain that stopped well before the end (a walk hit its
        // frame cap, or traffic changed): the next 15 scans sieve every tile.
        const dsieve* d = c->h_sv.as<dsieve>();
        if (c->sv_win_len && d->active && (!d->use || d->pend + (4ull << 20) < c->sv_win_len)) c->sv_full_left = 15;
        c->sv_hint_win = c->sv_win_len != 0;
        c->sv_win_len = 0;
        // bytes per frame along the last chain: the window geometry's mean
        // (single_hint is read only when the frame table had to be sized by
        // an estimate, so it can belong to an older stream)
        if (d->active && d->use && d->npath) c->sv_mean = std::max<uint64_t>(1, d->pend / d->npath);
    }
    if (c->sv_full_left) {
        --c->sv_full_left;
        b.rt = b.wt = 1;
    } else {
        sieve_geometry(rx_len, c->sv_mean ? rx_len / c->sv_mean : c->single_hint, b.rt, b.wt);
    }
    // Counts of a windowed scan say nothing about a scan of every tile.
    const bool stale = b.rt == b.wt && c->sv_hint_win;
    const uint64_t seen = stale ? 0 : c->sv_hint_pre, seen_s = stale ? 0 : c->sv_hint_surv;
    // Capacity from the last sieved scan's entry count when there is one (the
    // chain steps and their scans run over the whole capacity), else one
    // entry per KiB of the batch.
    uint64_t cap = seen ? std::max<uint64_t>({1ull << 18, rx_len / 8192, seen + seen / 4 + 1024})
                        : std::max<uint64_t>(1ull << 20, rx_len / 1024);
    cap = std::min<uint64_t>(cap, 0xFFFFFFF0ull);
    c->sv_cap = cap;
    // chain arrays: from the last survivor count (the chain steps scale with it)
    // (no usable count -- none yet, or the last scan overflowed its entries and
    // never counted survivors -- means the full capacity)
    uint64_t capc = seen_s ? std::min<uint64_t>(cap, std::max<uint64_t>(1ull << 16, seen_s + seen_s / 4 + 1024))
                           : cap;
    b.scr = nullptr;
    b.lgP = 0;
    if (b.rt != b.wt && seen_s) {
        // Windowed: survivors lie in the windows only (a count from a scan of
        // every tile scales by their share).  A small capacity keeps the
        // doubling rounds in one LDS-resident launch and the walks' offset
        // scratch (2^lgP per node, about twice the frames a region holds) small.
        const uint64_t est = c->sv_hint_win ? seen_s : seen_s * b.wt / b.rt * 2;
        capc = std::min<uint64_t>(cap, std::max<uint64_t>(4096, est + est / 2 + 2048));
        uint32_t lgP = 4;
        while (lgP < 12 && (1ull << lgP) < 2 * sieve_hops()) ++lgP;
        if ((capc << lgP) <= (1ull << 25)) {
            HIP_OR(c->sv_scr.ensure((capc << lgP) * 8), HVWS_ENOMEM);
            b.scr = c->sv_scr.as<uint64_t>();
            b.lgP = lgP;
        }
    }
    c->sv_capc = capc;
    const uint64_t ntm = sieve_tiles_max(rx_len);
    const uint64_t nmax = std::max(cap, ntm);
    HIP_OR(c->sv_state.ensure(sizeof(dsieve)), HVWS_ENOMEM);
    HIP_OR(c->sv_tcount.ensure(ntm * 8), HVWS_ENOMEM);
    HIP_OR(c->sv_tbase.ensure(ntm * 8), HVWS_ENOMEM);
    HIP_OR(c->sv_slot.ensure(sieve_slot_words(rx_len) * 4), HVWS_ENOMEM);
    HIP_OR(c->sv_S.ensure(capc * 8), HVWS_ENOMEM);
    HIP_OR(c->sv_Spre.ensure(cap * 8), HVWS_ENOMEM);
    HIP_OR(c->sv_pool.ensure(cap * 4), HVWS_ENOMEM);
    HIP_OR(c->sv_keep.ensure(cap * 8), HVWS_ENOMEM);
    HIP_OR(c->sv_kbase.ensure(cap * 8), HVWS_ENOMEM);
    HIP_OR(c->sv_J0.ensure(capc * 4), HVWS_ENOMEM);
    HIP_OR(c->sv_J1.ensure(capc * 4), HVWS_ENOMEM);
    HIP_OR(c->sv_mark.ensure(capc * 8), HVWS_ENOMEM);
    HIP_OR(c->sv_hops.ensure(capc * 4), HVWS_ENOMEM);
    HIP_OR(c->sv_rank.ensure(capc * 8), HVWS_ENOMEM);
    HIP_OR(c->sv_cnt.ensure(32), HVWS_ENOMEM);
    HIP_OR(c->sv_tmp.ensure((4 * ((nmax + 1023) / 1024) + 64) * 8), HVWS_ENOMEM);
    b.state = c->sv_state.as<dsieve>();
    b.tcount = c->sv_tcount.as<uint64_t>();
    b.tbase = c->sv_tbase.as<uint64_t>();
    b.slot = c->sv_slot.as<uint32_t>();
    b.pool = c->sv_pool.as<uint32_t>();
    b.pool_n = c->sv_cnt.as<uint64_t>() + 2;
    b.S = c->sv_S.as<uint64_t>();
    b.Spre = c->sv_Spre.as<uint64_t>();
    b.m_pre = c->sv_cnt.as<uint64_t>() + 3;
    b.J0 = c->sv_J0.as<uint32_t>();
    b.J1 = c->sv_J1.as<uint32_t>();
    b.mark = c->sv_mark.as<uint64_t>();
    b.hops = c->sv_hops.as<uint32_t>();
    b.rank = c->sv_rank.as<uint64_t>();
    b.m_total = c->sv_cnt.as<uint64_t>();
    b.npath = c->sv_cnt.as<uint64_t>() + 1;
    b.tmp = c->sv_tmp.as<uint64_t>();
    b.capS = cap;
    b.capC = capc;
    b.keep = c->sv_keep.as<uint64_t>();
    b.kbase = c->sv_kbase.as<uint64_t>();
    c->sv_win_len = b.rt != b.wt ? rx_len : 0;
    c->sv_rt = b.rt;
    c->sv_wt = b.wt;
    return HVWS_OK;
}

// Unmask kernel launch with its timing events (no argument checks).  The
// events ride on the unmask's own dispatch (launch_unmask).
// joined = false: the host has already seen the scan's last kernel publish
// (host_order), so the unmask needs no cross-stream wait packet.
hipError_t issue_unmask(hvws_ctx* c, uint8_t* d_rx, uint64_t rx_len, bool joined = false) {
    hipError_t e;
    const bool piped = c->cs != c->stream;
    if (piped && !joined) {   // the scan ran on the side stream: join it
        if ((e = hipEventRecord(c->scan_done, c->cs)) != hipSuccess) return e;
        if ((e = hipStreamWaitEvent(c->stream, c->scan_done, 0)) != hipSuccess) return e;
    }
    const bool timed = step_events(c) >= 1 && c->t_on;
    // Pipelined steps of mixed multi-segment batches: the unmask in pieces.
    // The hardware dispatches a kernel queued on the second stream (the next
    // batch's discovery) only once the unmask grid is fully launched, so its
    // walk (~0.2 ms at c4) waited for the whole unmask; between pieces it is
    // dispatched and overlaps.  On-device sweep: 4 pieces c4
    // 1.73 -> 1.55 ms, but c3 21.3 -> 22.4 ms and c2 flat, so uniform batches
    // (SPEC: a short scan) keep one launch.  With the 512 x 2 linear geometry
    // (round 2, profiles/r2n_raw) c4 ran 1.429 / 1.405 / 1.377 / 1.366 ms at
    // 1 / 2 / 4 / 8 pieces: 8.  One sieved stream (c4 as one segment, its
    // ~25 chain kernels beside the unmask) likewise: 1 / 2 / 4 / 8 / 12 / 16 /
    // 32 pieces 1.58 / 1.56 / 1.54 / 1.52 / 1.525 / 1.535 / 1.59 ms
    // (profiles/r5_raw/pieces).  $HVWS_EXPERIMENT unmask_pieces overrides.
    static const int env_pieces = experiment("unmask_pieces") ? atoi(experiment("unmask_pieces")) : -1;
    const int path = c->prev_path;   // the current scan's path may not be settled yet
    const bool mixed = path == HVWS_PATH_SLACK || path == HVWS_PATH_SLACK_FAILED || path == HVWS_PATH_SPEC_FAILED ||
                       (path == HVWS_PATH_COUNT_READ_EMIT && !c->spec_ok) ||   // an exact scan that saw mixed counts
                       (path == HVWS_PATH_SINGLE && c->sv_ran);                 // a sieved stream
    const uint32_t pieces = !piped ? 1u : env_pieces > 0 ? (uint32_t)env_pieces : (mixed ? 8u : 1u);
    // An untimed pipelined step attaches its set's free event to its last
    // dispatch (RUN: the repair) instead of recording it in a marker packet after it:
    // c2 0.355-0.356 vs 0.358 ms per step (profiles/r5_raw/events, fa*).
    const bool attach_free = piped && !timed;
    if (c->run_active) {   // the RUN unmask and its repair pass (the stop event rides on the repair)
        if ((e = launch_unmask_run(d_rx, rx_len, c->T().runs.as<drun>(), c->T().run_trun.as<dtrun>(),
                                   c->nseg, c->T().run_fail.as<uint32_t>(), mapped<dspec_status>(c->h_status),
                                   c->run_seq, c->stream, timed ? c->tev[c->t_cur][2] : nullptr,
                                   timed ? c->tev[c->t_cur][3] : (attach_free ? c->T().free_ev : nullptr))) !=
            hipSuccess)
            return e;
    } else if ((e = launch_unmask(c->variant, d_rx, rx_len, frames_of(c), c->T().tile_first.as<uint32_t>(),
                                  c->T().tile_key.as<uint32_t>(), c->T().tile_kind.as<uint8_t>(),
                                  c->T().total.as<uint64_t>(), c->stream, pieces, timed ? c->tev[c->t_cur][2] : nullptr,
                                  timed ? c->tev[c->t_cur][3] : (attach_free ? c->T().free_ev : nullptr))) !=
               hipSuccess) {
        return e;
    }
    if (timed) c->t_rec[c->t_cur] |= (uint8_t)(4u | 8u);
    c->t_unmask[c->t_cur] = true;
    if (piped) {   // the next pipelined scan into this set waits for this unmask
        // The unmask's dispatch-attached stop event marks the set free when it
        // was recorded; a separate marker packet cost ~6 us of device time per
        // pipelined c2 step (0.4215 -> 0.416 ms, profiles/r2r_raw).
        if (timed) {
            c->T().free_wait = c->tev[c->t_cur][3];
        } else if (attach_free) {   // recorded by the repair's dispatch
            c->T().free_wait = c->T().free_ev;
        } else {
            if ((e = hipEventRecord(c->T().free_ev, c->stream)) != hipSuccess) return e;
            c->T().free_wait = c->T().free_ev;
        }
        c->T().free_pending = true;
    }
    return hipSuccess;
}

// unmask_into: the caller will unmask d_rx right after the scan (hvws_step).
// On the speculative path the unmask is then queued before the host waits
// for the device's check -- a rejected table has a zero count, so that
// unmask does nothing -- and *unmasked reports whether it stands.
int scan_device_carry(hvws_ctx* c, const uint8_t* d_rx, uint64_t rx_len, uint32_t nseg, uint8_t* unmask_into = nullptr,
                      bool* unmasked = nullptr) {
    if (unmasked) *unmasked = false;
    // The other table set: the previous batch's tables stay intact while its
    // unmask may still be running (pipelined steps).
    c->cur ^= 1;
    c->prev_path = c->scan_path;
    c->run_active = false;
    if (c->cs == c->stream) c->piped = false;   // a later pipelined step re-arms the set events
    if (c->cs != c->stream && c->T().free_pending) {
        HIP_OR(hipStreamWaitEvent(c->cs, c->T().free_wait, 0), HVWS_EHIP);
        c->T().free_pending = false;
    }
    HIP_OR(c->T().counts.ensure((uint64_t)nseg * 8 + 8), HVWS_ENOMEM);
    HIP_OR(c->T().bases.ensure((uint64_t)nseg * 8 + 8), HVWS_ENOMEM);
    HIP_OR(c->T().total.ensure(8), HVWS_ENOMEM);
    HIP_OR(c->T().carry_out.ensure((uint64_t)nseg * sizeof(dcarry) + 64), HVWS_ENOMEM);
    HIP_OR(c->h_total.ensure(8), HVWS_ENOMEM);
    HIP_OR(ensure_frames(c, 1), HVWS_ENOMEM);
    HIP_OR(c->T().sc_mid.ensure((uint64_t)nseg * sizeof(dmid) + 64), HVWS_ENOMEM);
    HIP_OR(c->T().sc_npred.ensure((uint64_t)nseg * 8 + 8), HVWS_ENOMEM);
    HIP_OR(c->T().sc_pbase.ensure((uint64_t)nseg * 8 + 8), HVWS_ENOMEM);
    HIP_OR(c->T().sc_fail.ensure((uint64_t)nseg * 8 + 8), HVWS_ENOMEM);
    HIP_OR(c->T().sc_masked.ensure((uint64_t)nseg * 8 + 8), HVWS_ENOMEM);
    HIP_OR(c->T().sc_total.ensure(8), HVWS_ENOMEM);
    HIP_OR(c->T().sc_est.ensure((uint64_t)nseg * 8 + 8), HVWS_ENOMEM);
    HIP_OR(c->h_status.ensure(sizeof(dspec_status)), HVWS_ENOMEM);
    scan_scratch sc;
    sc.mid = c->T().sc_mid.as<dmid>();
    sc.npred = c->T().sc_npred.as<uint64_t>();
    sc.pbase = c->T().sc_pbase.as<uint64_t>();
    sc.first_fail = c->T().sc_fail.as<uint64_t>();
    sc.last_masked = c->T().sc_masked.as<uint64_t>();
    sc.total_pred = c->T().sc_total.as<uint64_t>();
    sc.est = c->T().sc_est.as<uint64_t>();
    sc.src_segs = c->up_src_segs;
    sc.src_carry = c->up_src_carry;
    sc.segs_w = c->segs.as<dseg>();
    sc.carry_w = c->carry_in.as<dcarry>();
    sc.status = nullptr;
    sc.seq = 0;
    sc.sieve = nullptr;
    sc.slack = frames_of(c);
    sc.slack_cap = 0;
    sc.bases_x = nullptr;
    sc.est_u = nullptr;
    sc.no_verify = 0;
    sc.runs = nullptr;
    sc.run_fail = nullptr;
    sc.run_trun = nullptr;
    sc.run_ntiles = sc.run_tile = 0;
    dspec_status* status_d = mapped<dspec_status>(c->h_status);
    const dspec_status* status_h = c->h_status.as<dspec_status>();
    if (!status_d) return set_err(HVWS_EHIP, "pinned status not device-mapped");
    const dseg* segs = c->segs.as<dseg>();
    const dcarry* cin = c->carry_in.as<dcarry>();
    // (run_materialize's rebuild of a RUN step's records keeps that step's
    // timing slot: no new slot, no events)
    if (!c->materializing) HIP_OR(begin_timed_scan(c), HVWS_EHIP);
    // After the first pass the device tables hold the uploaded segments; the
    // pinned slot is free once that pass's first kernel has run.
    const int up_slot = c->up_slot;
    c->up_slot = -1;
    c->up_src_segs = nullptr;
    c->up_src_carry = nullptr;
    bool slot_released = up_slot < 0;
    auto release_slot = [&]() -> hipError_t {
        if (slot_released) return hipSuccess;
        slot_released = true;
        const hipError_t e2 = hipEventRecord(c->up_ev[up_slot], c->cs);
        c->up_pending[up_slot] = e2 == hipSuccess;
        return e2;
    };
    auto pass = [&](int which) {
        const hipError_t e = launch_scan(which, d_rx, rx_len, segs, nseg, cin, c->T().carry_out.as<dcarry>(),
                                         c->T().counts.as<uint64_t>(), c->T().bases.as<uint64_t>(), c->T().total.as<uint64_t>(), sc,
                                         frames_of(c), c->vmask, c->cs);
        sc.src_segs = nullptr;
        sc.src_carry = nullptr;
        if (e == hipSuccess) return release_slot();
        return e;
    };
    // k_spec_check's verdict for the pass just issued (after a wait on the
    // stream or for the published status): the record count and the SPEC_* flags.
    auto read_status = [&](uint64_t& n, uint32_t& flags) -> int {
        if (status_h->seq != sc.seq) return set_err(HVWS_EHIP, "scan status not published (seq %llu, want %llu)",
                                                    (unsigned long long)status_h->seq, (unsigned long long)sc.seq);
        n = status_h->total;
        flags = status_h->flags;
        if (flags & SPEC_ERR) return set_err(HVWS_EHIP, "scan check reported an error (seq %llu)",
                                             (unsigned long long)sc.seq);
        if (n >= 0xFFFFFFF0ull)
            return set_err(HVWS_EINVAL, "batch holds %llu frames (max 2^32-16)", (unsigned long long)n);
        return HVWS_OK;
    };
    // A rejected check in pipelined mode.  The speculative unmask was queued
    // on c->stream, behind the previous batch's unmask, and reads this set's
    // tile index and count when it runs, not when it was queued.  The exact
    // re-scan rewrites those tables on c->cs; unordered, a still-waiting
    // speculative unmask would see the re-scan's tiles and XOR for real, and
    // the caller's unmask would then XOR the payloads back.  So the re-scan
    // waits for it (the set's free event, recorded right after it).
    auto join_rejected = [&]() -> int {
        if (unmask_into && c->cs != c->stream) HIP_OR(hipStreamWaitEvent(c->cs, c->T().free_wait, 0), HVWS_EHIP);
        return HVWS_OK;
    };
    c->variant = unmask_variant_for(rx_len);
    const uint64_t tile = unmask_tile(c->variant);
    const uint64_t ntiles = (rx_len + tile - 1) / tile;
    HIP_OR(c->T().tile_first.ensure((ntiles + 8) * 4), HVWS_ENOMEM);
    HIP_OR(c->T().tile_key.ensure((ntiles + 2) * 4), HVWS_ENOMEM);
    HIP_OR(c->T().tile_kind.ensure(ntiles + 16), HVWS_ENOMEM);
    auto tiles = [&]() -> int {
        HIP_OR(launch_unmask_tiles(c->T().f_off.as<uint64_t>(), c->T().f_len.as<uint64_t>(), c->T().f_keyrot.as<uint32_t>(),
                                   c->T().total.as<uint64_t>(), c->T().tile_first.as<uint32_t>(), c->T().tile_key.as<uint32_t>(),
                                   c->T().tile_kind.as<uint8_t>(), ntiles, tile, rx_len,
                                   c->cs),
               HVWS_EHIP);
        return HVWS_OK;
    };
    // Frame records are bounded: after a segment's first record every frame
    // spends >= 2 of its bytes.  When the bound fits the table, EMIT follows
    // COUNT with no host round trip and the count stays on the device (the
    // tile kernels and k_unmask read it there); otherwise read the count first.
    const uint64_t bound = rx_len / 2 + 2 * (uint64_t)nseg + 1;
    uint64_t nfr = bound;
    c->nfr_known = false;
    bool tiles_done = false;
    if (nseg == 1) {
        c->scan_path = HVWS_PATH_SINGLE;
        // One stream: its base is 0, so EMIT needs no COUNT walk (a mixed-size
        // stream's serial walk runs once).  The table is sized by the bound
        // when that is small, else by an estimate (1.25 x the last one-stream
        // count, at least 2^20 records) that is checked after the pass and
        // re-emitted into an exact-size table if it overflowed.  (Sizing by
        // the bound would give a 256 MiB chunk of 64 KiB frames a 3.2 GB
        // table for its ~4000 records.)
        const uint64_t guess = std::max<uint64_t>(kSingleMin, c->single_hint + c->single_hint / 4);
        const uint64_t cap = std::min<uint64_t>(bound, guess);
        HIP_OR(ensure_frames(c, cap), HVWS_ENOMEM);
        // A long segment is sieved (parallel discovery) unless the last
        // sieved scan found uniform sizes: then 15 scans walk before the next
        // try.  Results never depend on it.
        sieve_bufs svb;
        if (c->sv_gen != sieve_generation()) {
            c->sv_gen = sieve_generation();
            c->sv_skip = 0;
            c->sv_ran = false;
            c->sv_hint_pre = c->sv_hint_surv = 0;
            c->sv_win_len = 0;
            c->sv_full_left = 0;
            c->sv_hint_win = false;
            c->sv_mean = 0;
        }
        if (rx_len >= sieve_min()) {
            if (sieve_state_ready(c) && c->h_sv.as<dsieve>()->active == 0 && c->sv_skip == 0) c->sv_skip = 15;
            if (c->sv_skip) {
                --c->sv_skip;
                c->sv_ran = false;
            } else {
                HIP_OR(c->h_sv.ensure(sizeof(dsieve) + 32), HVWS_ENOMEM);
                if (!c->sv_ev) HIP_OR(hipEventCreateWithFlags(&c->sv_ev, hipEventDisableTiming), HVWS_EHIP);
                if (ensure_sieve(c, rx_len, svb) == HVWS_OK) {
                    sc.sieve = &svb;
                    c->sv_ran = true;
                } else {   // no room for the sieve's tables: walk instead (results are the same)
                    (void)hipGetLastError();
                    for (dbuf* b : {&c->sv_tcount, &c->sv_tbase, &c->sv_slot, &c->sv_pool, &c->sv_keep, &c->sv_kbase,
                                    &c->sv_Spre, &c->sv_S,
                                    &c->sv_J0, &c->sv_J1, &c->sv_mark, &c->sv_hops, &c->sv_rank, &c->sv_tmp, &c->sv_scr})
                        b->release();
                    c->sv_ran = false;
                }
            }
        }
        HIP_OR(pass(SCAN_SINGLE), HVWS_EHIP);
        if (bound > c->T().frame_cap) {
            // The table was sized by an estimate.  The device checks the count
            // against it (over capacity zeroes the count, so the tile kernels
            // and an unmask queued behind do nothing) and publishes it; the
            // tiles and the unmask are queued before the host waits, so the
            // device runs on instead of idling through a host round trip.
            int rc;
            uint32_t flags = 0;
            sc.seq = ++c->scan_seq;
            HIP_OR(launch_cap_check(c->T().total.as<uint64_t>(), c->T().frame_cap, status_d, sc.seq, c->cs), HVWS_EHIP);
            if ((rc = tiles()) != HVWS_OK) return rc;
            if (unmask_into) {
                HIP_OR(tev_record(c, 1, c->cs), HVWS_EHIP);
                HIP_OR(issue_unmask(c, unmask_into, rx_len), HVWS_EHIP);
            }
            if ((rc = wait_status(c, sc.seq)) != HVWS_OK) return rc;
            if ((rc = read_status(nfr, flags)) != HVWS_OK) return rc;
            if (flags & SPEC_OK) {
                tiles_done = true;
                if (unmask_into && unmasked) *unmasked = true;
            } else {   // overflowed: re-emit into an exact table (the caller unmasks)
                if ((rc = join_rejected()) != HVWS_OK) return rc;
                HIP_OR(ensure_frames(c, nfr + 1), HVWS_ENOMEM);
                HIP_OR(pass(SCAN_EMIT), HVWS_EHIP);
                HIP_OR(launch_offsets(c->T().counts.as<uint64_t>(), c->T().bases.as<uint64_t>(), 1,
                                      c->T().total.as<uint64_t>(), c->cs),
                       HVWS_EHIP);
            }
            c->nfr_known = true;
            c->single_hint = nfr;
        }
        if (c->sv_ran) {   // state and counts for the next scan's choices and hvws_last_sieve
            HIP_OR(hipMemcpyAsync(c->h_sv.p, c->sv_state.p, sizeof(dsieve), hipMemcpyDeviceToHost, c->cs), HVWS_EHIP);
            HIP_OR(hipMemcpyAsync(c->h_sv.as<uint8_t>() + sizeof(dsieve), c->sv_cnt.p, 32, hipMemcpyDeviceToHost, c->cs),
                   HVWS_EHIP);
            HIP_OR(hipEventRecord(c->sv_ev, c->cs), HVWS_EHIP);
        }
        sc.sieve = nullptr;
    } else if (bound <= (c->fast_bound ? c->fast_bound : kFastFrameBound)) {
        c->scan_path = HVWS_PATH_COUNT_EMIT;
        HIP_OR(pass(SCAN_COUNT), HVWS_EHIP);
        HIP_OR(ensure_frames(c, bound), HVWS_ENOMEM);
        HIP_OR(pass(SCAN_EMIT), HVWS_EHIP);
    } else {
        // Large batch: the table is sized from a count.  With the estimates
        // holding on the last batch, EMIT speculatively into the table as
        // it is (SCAN_SPEC) and let the device check it -- one walk, no
        // host round trip before EMIT, and the tile kernels queued behind
        // the check; the host then waits for the check only.  Otherwise (or
        // when the check fails) COUNT, read the count, EMIT.
        int rc;
        uint32_t flags = 0;
        sc.status = status_d;
        bool done = false;
        // The last RUN verdict the device has published: a failed hypothesis
        // turns RUN off for the next 16 steps and the next scan exact.
        const uint64_t vseq = __atomic_load_n(&status_h->pad3[0], __ATOMIC_ACQUIRE);
        if (vseq != c->run_seen) {
            c->run_seen = vseq;
            if (status_h->pad3[1]) {
                c->run_skip = 16;
                c->spec_ok = false;
            }
        }
        // RUN: a step's batch of small uniform frames (the last exact or SPEC
        // scan matched the uniform estimates): discovery is k_head alone, the
        // unmask checks every header it loads (hvws_internal.h, drun).
        // Segments of RUN_MIN_SEG bytes or more on average: k_unmask_run
        // takes two segments per tile and leaves any between to the repair.
        const bool run_auto = c->run_mode < 0 && c->spec_ok && c->spec_mode != 0 && !c->run_skip && c->last_mean &&
                              c->last_mean <= RUN_MAX_FRAME && rx_len / nseg >= RUN_MIN_SEG && run_env();
        if (c->run_skip && !c->materializing) --c->run_skip;
        if (unmask_into && c->run_call && c->vmask == 0 && (run_auto || c->run_mode == 1)) {
            c->scan_path = HVWS_PATH_RUN;
            HIP_OR(c->T().runs.ensure((uint64_t)nseg * sizeof(drun) + 64), HVWS_ENOMEM);
            {
                const void* was = c->T().run_fail.p;
                const uint64_t had = c->T().run_fail.cap;
                HIP_OR(c->T().run_fail.ensure((uint64_t)nseg * 4 + 64), HVWS_ENOMEM);
                if (c->T().run_fail.p != was || c->T().run_fail.cap != had)
                    HIP_OR(hipMemsetAsync(c->T().run_fail.p, 0, c->T().run_fail.cap, c->cs), HVWS_EHIP);
            }
            const uint64_t rtile = RUN_TILE;
            const uint64_t rtiles = (rx_len + rtile - 1) / rtile;
            HIP_OR(c->T().run_trun.ensure((rtiles + 1) * sizeof(dtrun)), HVWS_ENOMEM);
            sc.runs = c->T().runs.as<drun>();
            sc.run_fail = c->T().run_fail.as<uint32_t>();
            sc.run_trun = c->T().run_trun.as<dtrun>();
            sc.run_ntiles = rtiles;
            sc.run_tile = rtile;
            HIP_OR(pass(SCAN_RUN), HVWS_EHIP);
            c->run_seq = ++c->scan_seq;
            c->run_active = true;
            c->nseg = nseg;
            const bool ordered = c->cs != c->stream && host_order();
            if (ordered) {
                HIP_OR(launch_publish_tiles(status_d, c->run_seq, c->cs), HVWS_EHIP);
                if ((rc = wait_status(c, c->run_seq, /*tiles=*/true)) != HVWS_OK) return rc;
                HIP_OR(issue_unmask(c, unmask_into, rx_len, /*joined=*/true), HVWS_EHIP);
            } else {
                HIP_OR(tev_record(c, 1, c->cs), HVWS_EHIP);
                HIP_OR(issue_unmask(c, unmask_into, rx_len), HVWS_EHIP);
            }
            if (unmasked) *unmasked = true;
            c->nfr = 0;
            c->nfr_known = false;
            c->rx = d_rx;
            c->rx_len = rx_len;
            c->have_scan = true;
            c->hcache_valid = false;
            return HVWS_OK;
        }
        c->scan_path = HVWS_PATH_COUNT_READ_EMIT;
        if ((c->spec_ok && c->spec_mode != 0) || c->spec_mode == 1) {
            // a set not used yet gets the other set's capacity (the table
            // must hold the estimated records for the check to pass)
            if (c->T().frame_cap < c->ts[c->cur ^ 1].frame_cap)
                HIP_OR(ensure_frames(c, c->ts[c->cur ^ 1].frame_cap, /*exact=*/true), HVWS_ENOMEM);
            sc.seq = ++c->scan_seq;
            sc.no_verify = (c->verify_mode < 0 ? c->verify_hint : c->verify_mode != 0) ? 0u : 1u;
            HIP_OR(pass(SCAN_SPEC), HVWS_EHIP);
            if ((rc = tiles()) != HVWS_OK) return rc;
            // Pipelined: the host waits for the scan's last kernel (it runs
            // beside the previous unmask) and then queues this unmask with no
            // cross-stream wait packet between the two unmasks.  Otherwise
            // the unmask is queued behind the check at once.
            const bool ordered = unmask_into && c->cs != c->stream && host_order();
            if (ordered) HIP_OR(launch_publish_tiles(status_d, sc.seq, c->cs), HVWS_EHIP);
            if (unmask_into && !ordered) {
                HIP_OR(tev_record(c, 1, c->cs), HVWS_EHIP);
                HIP_OR(issue_unmask(c, unmask_into, rx_len), HVWS_EHIP);
            }
            if ((rc = wait_status(c, sc.seq)) != HVWS_OK) return rc;
            if ((rc = read_status(nfr, flags)) != HVWS_OK) return rc;
            c->verify_hint = status_h->pad2[1] != 0;
            done = (flags & SPEC_OK) != 0;
            c->spec_ok = done;
            c->scan_path = done ? HVWS_PATH_SPEC : HVWS_PATH_SPEC_FAILED;
            if (done && ordered) {
                if ((rc = wait_status(c, sc.seq, /*tiles=*/true)) != HVWS_OK) return rc;
                HIP_OR(issue_unmask(c, unmask_into, rx_len, /*joined=*/true), HVWS_EHIP);
            }
            if (done && unmask_into && unmasked) *unmasked = true;
            if (!done && (rc = join_rejected()) != HVWS_OK) return rc;
            tiles_done = done;
        }
        // Mixed sizes: one EMIT walk into per-segment regions of a scratch
        // table, checked and compacted on the device (SCAN_SLACK).  Its check
        // also tells whether the uniform estimates held (SPEC next time).
        const uint64_t cap_seg = c->slack_seg + c->slack_seg / 2 + 16;
        const uint64_t want = std::min<uint64_t>((uint64_t)nseg * cap_seg, bound) + 1;
        bool slack_try = !done && c->spec_mode != 0 && c->spec_mode != 1 && c->slack_seg &&
                         (c->spec_mode == 2 || !c->spec_ok) && want <= kSlackMaxRecords;
        if (slack_try && want > c->sl_cap) {
            // a scratch table that cannot be had is no error: scan exactly instead
            const uint64_t n = want + want / 4;
            bool ok = true;
            for (dbuf* b : {&c->sl_hdr, &c->sl_off, &c->sl_len, &c->sl_length}) ok = ok && b->ensure(n * 8) == hipSuccess;
            for (dbuf* b : {&c->sl_key, &c->sl_keyrot, &c->sl_info}) ok = ok && b->ensure(n * 4) == hipSuccess;
            c->sl_cap = ok ? n : 0;
            if (!ok) {
                (void)hipGetLastError();
                for (dbuf* b : {&c->sl_hdr, &c->sl_off, &c->sl_len, &c->sl_length, &c->sl_key, &c->sl_keyrot,
                                &c->sl_info})
                    b->release();
            }
            slack_try = ok;
        }
        if (slack_try) {
            HIP_OR(c->sl_bx.ensure((uint64_t)nseg * 16 + 16), HVWS_ENOMEM);
            // the frame table must hold the batch: the last count, with room
            if (c->T().frame_cap < c->ts[c->cur ^ 1].frame_cap)
                HIP_OR(ensure_frames(c, c->ts[c->cur ^ 1].frame_cap, /*exact=*/true), HVWS_ENOMEM);
            sc.slack.hdr_off = c->sl_hdr.as<int64_t>();
            sc.slack.pay_off = c->sl_off.as<uint64_t>();
            sc.slack.pay_len = c->sl_len.as<uint64_t>();
            sc.slack.length = c->sl_length.as<uint64_t>();
            sc.slack.key = c->sl_key.as<uint32_t>();
            sc.slack.keyrot = c->sl_keyrot.as<uint32_t>();
            sc.slack.info = c->sl_info.as<uint32_t>();
            sc.slack.cap = c->sl_cap;
            sc.slack_cap = cap_seg;
            sc.bases_x = c->sl_bx.as<uint64_t>();
            sc.est_u = c->sl_bx.as<uint64_t>() + nseg + 1;
            sc.seq = ++c->scan_seq;
            sc.no_verify = (c->verify_mode < 0 ? c->verify_hint : c->verify_mode != 0) ? 0u : 1u;
            HIP_OR(pass(SCAN_SLACK), HVWS_EHIP);
            if ((rc = tiles()) != HVWS_OK) return rc;
            if (unmask_into) {
                HIP_OR(tev_record(c, 1, c->cs), HVWS_EHIP);
                HIP_OR(issue_unmask(c, unmask_into, rx_len), HVWS_EHIP);
            }
            if ((rc = wait_status(c, sc.seq)) != HVWS_OK) return rc;
            if ((rc = read_status(nfr, flags)) != HVWS_OK) return rc;
            c->verify_hint = status_h->pad2[1] != 0;
            done = (flags & SPEC_OK) != 0;
            if (done) {
                c->slack_seg = status_h->pad2[0];
                c->spec_ok = (flags & SPEC_MATCH) != 0;   // uniform again: the next batch tries SPEC
                if (unmask_into && unmasked) *unmasked = true;
            } else if ((rc = join_rejected()) != HVWS_OK) {
                return rc;
            }
            c->scan_path = done ? HVWS_PATH_SLACK : HVWS_PATH_SLACK_FAILED;
            tiles_done = done;
        }
        if (!done) {
            sc.seq = ++c->scan_seq;
            sc.no_verify = 0;
            HIP_OR(pass(SCAN_COUNT), HVWS_EHIP);
            HIP_OR(hipStreamSynchronize(c->cs), HVWS_EHIP);
            if ((rc = read_status(nfr, flags)) != HVWS_OK) return rc;
            c->verify_hint = status_h->pad2[1] != 0;
            c->spec_ok = (flags & SPEC_MATCH) != 0;
            c->slack_seg = status_h->pad2[0];
            HIP_OR(ensure_frames(c, nfr + 1), HVWS_ENOMEM);
            HIP_OR(pass(SCAN_EMIT), HVWS_EHIP);
        }
        c->nfr_known = true;
    }
    if (!tiles_done) {
        int rc = tiles();
        if (rc) return rc;
    }
    if (!(unmasked && *unmasked)) HIP_OR(tev_record(c, 1, c->cs), HVWS_EHIP);
    if (table_checks()) {   // the tile index's invariant (k_ends_check), tests only: one sync
        HIP_OR(c->chk.ensure(8), HVWS_ENOMEM);
        HIP_OR(c->h_chk.ensure(8), HVWS_ENOMEM);
        HIP_OR(hipMemsetAsync(c->chk.p, 0, 8, c->cs), HVWS_EHIP);
        HIP_OR(launch_ends_check(c->T().f_off.as<uint64_t>(), c->T().f_len.as<uint64_t>(), c->T().total.as<uint64_t>(),
                                 c->chk.as<unsigned long long>(), c->cs),
               HVWS_EHIP);
        HIP_OR(hipMemcpyAsync(c->h_chk.p, c->chk.p, 8, hipMemcpyDeviceToHost, c->cs), HVWS_EHIP);
        HIP_OR(hipStreamSynchronize(c->cs), HVWS_EHIP);
        if (const uint64_t bad = *c->h_chk.as<uint64_t>())
            return set_err(HVWS_EINVAL, "frame table: %llu record ends before its predecessor's (scan path %d)",
                           (unsigned long long)bad, c->scan_path);
    }
    c->nseg = nseg;
    c->nfr = nfr;
    c->rx = d_rx;
    c->rx_len = rx_len;
    c->have_scan = true;
    c->hcache_valid = false;
    if (c->nfr_known && nfr) c->last_mean = rx_len / nfr;
    return HVWS_OK;
}

// The records of a RUN step, built when a reader asks for them: an exact scan
// of the same batch (its headers never change; its segment and carry tables
// are the device copies the RUN scan wrote) on the context stream, behind
// the unmask and its repair.  The scan path stays RUN.
int run_materialize(hvws_ctx* c) {
    if (!c->run_active) return HVWS_OK;
    c->run_active = false;
    const int path = c->scan_path;
    hipStream_t cs = c->cs;
    c->cs = c->stream;
    const bool call = c->run_call, t_on = c->t_on;
    c->run_call = false;
    c->t_on = false;   // the RUN step's events stay in its slot (hvws_last_times / hvws_step_times)
    c->materializing = true;
    const int rc = scan_device_carry(c, c->rx, c->rx_len, c->nseg);
    c->materializing = false;
    c->t_on = t_on;
    c->run_call = call;
    c->cs = cs;
    c->scan_path = path;
    return rc;
}

// The frame count of the last scan on the host (one small read-back when the
// scan left it on the device).
int ensure_count(hvws_ctx* c) {
    if (int rc = run_materialize(c)) return rc;
    if (c->nfr_known) return HVWS_OK;
    HIP_OR(hipMemcpyAsync(c->h_total.p, c->T().total.p, 8, hipMemcpyDeviceToHost, c->stream), HVWS_EHIP);
    HIP_OR(hipStreamSynchronize(c->stream), HVWS_EHIP);
    c->nfr = *c->h_total.as<uint64_t>();
    c->nfr_known = true;
    return HVWS_OK;
}

// Everything a host-side replay needs from the last scan, in one round trip:
// count, per-segment first/count, carry-out, and the frame table up to the
// record bound (small batches) -- copied into pinned memory, one sync.
int readback_all(hvws_ctx* c) {
    if (int rc = run_materialize(c)) return rc;
    const uint32_t nseg = c->nseg;
    // c->nfr is the exact count or its bound; copy at most a prefix of the
    // table with the rest, and the remainder after the sync if needed.
    const uint64_t nrec = c->nfr < kReadbackPrefix ? c->nfr : kReadbackPrefix;
    const uint64_t cap = c->nfr_known ? c->nfr : nrec;
    const uint64_t soa = (cap > nrec ? cap : nrec) * (8 + 8 + 8 + 8 + 4 + 4);
    const uint64_t need = 64 + (uint64_t)nseg * (16 + sizeof(dcarry)) + soa + 64;
    HIP_OR(c->h_readback.ensure(need), HVWS_ENOMEM);
    uint8_t* h = c->h_readback.as<uint8_t>();
    uint64_t* total = (uint64_t*)h;
    uint64_t* first = (uint64_t*)(h + 64);
    uint64_t* count = first + nseg;
    dcarry* carry = (dcarry*)(count + nseg);
    hipStream_t s = c->stream;
    HIP_OR(hipMemcpyAsync(total, c->T().total.p, 8, hipMemcpyDeviceToHost, s), HVWS_EHIP);
    if (nseg) {
        HIP_OR(hipMemcpyAsync(first, c->T().bases.p, (uint64_t)nseg * 8, hipMemcpyDeviceToHost, s), HVWS_EHIP);
        HIP_OR(hipMemcpyAsync(count, c->T().counts.p, (uint64_t)nseg * 8, hipMemcpyDeviceToHost, s), HVWS_EHIP);
        HIP_OR(hipMemcpyAsync(carry, c->T().carry_out.p, (uint64_t)nseg * sizeof(dcarry), hipMemcpyDeviceToHost, s),
               HVWS_EHIP);
    }
    // SoA staging sized for `cap` records (exact count known) or the prefix
    uint64_t room = cap > nrec ? cap : nrec;
    uint8_t* f = (uint8_t*)(carry + nseg);
    int64_t* f_hdr = (int64_t*)f;
    uint64_t* f_off = (uint64_t*)(f_hdr + room);
    uint64_t* f_len = f_off + room;
    uint64_t* f_length = f_len + room;
    uint32_t* f_key = (uint32_t*)(f_length + room);
    uint32_t* f_info = f_key + room;
    auto copy_range = [&](uint64_t a, uint64_t b) -> hipError_t {
        if (b <= a) return hipSuccess;
        const uint64_t n = b - a;
        hipError_t e2;
        if ((e2 = hipMemcpyAsync(f_hdr + a, c->T().f_hdr.as<int64_t>() + a, n * 8, hipMemcpyDeviceToHost, s))) return e2;
        if ((e2 = hipMemcpyAsync(f_off + a, c->T().f_off.as<uint64_t>() + a, n * 8, hipMemcpyDeviceToHost, s))) return e2;
        if ((e2 = hipMemcpyAsync(f_len + a, c->T().f_len.as<uint64_t>() + a, n * 8, hipMemcpyDeviceToHost, s))) return e2;
        if ((e2 = hipMemcpyAsync(f_length + a, c->T().f_length.as<uint64_t>() + a, n * 8, hipMemcpyDeviceToHost, s)))
            return e2;
        if ((e2 = hipMemcpyAsync(f_key + a, c->T().f_key.as<uint32_t>() + a, n * 4, hipMemcpyDeviceToHost, s))) return e2;
        return hipMemcpyAsync(f_info + a, c->T().f_info.as<uint32_t>() + a, n * 4, hipMemcpyDeviceToHost, s);
    };
    HIP_OR(copy_range(0, c->nfr_known ? c->nfr : nrec), HVWS_EHIP);
    HIP_OR(hipStreamSynchronize(s), HVWS_EHIP);
    const uint64_t got = c->nfr_known ? c->nfr : nrec;
    if (*total > got) {
        // more records than the speculative prefix: the exact count is known
        // now, so one more round trip copies the whole table
        c->nfr = *total;
        c->nfr_known = true;
        return readback_all(c);
    }
    const uint64_t n = *total;
    c->nfr = n;
    c->nfr_known = true;
    c->hcache.resize(n);
    for (uint64_t i = 0; i < n; ++i) {
        hvws_frame& o = c->hcache[i];
        o.hdr_off = f_hdr[i];
        o.pay_off = f_off[i];
        o.pay_len = f_len[i];
        o.length = f_length[i];
        o.key = f_key[i];
        o.info = f_info[i];
    }
    c->hfirst.assign(first, first + nseg);
    c->hcount.assign(count, count + nseg);
    c->hcarry.assign(carry, carry + nseg);
    c->hcache_valid = true;
    return HVWS_OK;
}

int upload_segments(hvws_ctx* c, const hvws_segment* segs, const websocket_parser* carry, uint32_t nseg,
                    uint64_t rx_len) {
    for (uint32_t s = 0; s < nseg; ++s) {
        if (segs[s].off > rx_len || segs[s].len > rx_len - segs[s].off)
            return set_err(HVWS_EINVAL, "segment %u [%llu,+%llu) outside the %llu-byte buffer", s,
                           (unsigned long long)segs[s].off, (unsigned long long)segs[s].len,
                           (unsigned long long)rx_len);
        if (s && segs[s].off < segs[s - 1].off + segs[s - 1].len)
            return set_err(HVWS_EINVAL, "segments must be sorted and disjoint (segment %u)", s);
    }
    HIP_OR(c->segs.ensure((uint64_t)nseg * sizeof(dseg) + 64), HVWS_ENOMEM);
    HIP_OR(c->carry_in.ensure((uint64_t)nseg * sizeof(dcarry) + 64), HVWS_ENOMEM);
    // Pinned staging slot: the scan two uploads ago may still be about to
    // read it -- wait for that scan's first kernel only.
    const int u = c->up_next;
    c->up_next ^= 1;
    if (c->up_pending[u]) {
        HIP_OR(hipEventSynchronize(c->up_ev[u]), HVWS_EHIP);
        c->up_pending[u] = false;
    }
    const uint64_t o_carry = ((uint64_t)nseg * sizeof(dseg) + 63) & ~63ull;
    HIP_OR(c->h_up[u].ensure(o_carry + (uint64_t)nseg * sizeof(dcarry) + 64), HVWS_ENOMEM);
    dseg* hs = c->h_up[u].as<dseg>();
    dcarry* hc = reinterpret_cast<dcarry*>(c->h_up[u].as<uint8_t>() + o_carry);
    for (uint32_t s = 0; s < nseg; ++s) {
        hs[s].off = segs[s].off;
        hs[s].len = segs[s].len;
        if (carry) {
            to_dcarry(carry[s], hc[s]);
        } else {
            memset(&hc[s], 0, sizeof(dcarry));
        }
    }
    // No copy: the scan's first kernel reads the slot through its device
    // mapping and writes c->segs / c->carry_in (a DMA copy of these tables
    // cost ~40 us of idle device per step).
    uint8_t* dev = mapped<uint8_t>(c->h_up[u]);
    if (!dev) return set_err(HVWS_EHIP, "pinned upload slot not device-mapped");
    c->up_slot = u;
    c->up_src_segs = reinterpret_cast<const dseg*>(dev);
    c->up_src_carry = reinterpret_cast<const dcarry*>(dev + o_carry);
    return HVWS_OK;
}

// Device-visible address of pinned host memory (nullptr if `p` is not
// pinned/registered host memory).
uint8_t* host_mapped(void* p) {
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();
        return nullptr;
    }
    if (a.type != hipMemoryTypeHost || !a.devicePointer || !a.hostPointer) return nullptr;
    return (uint8_t*)a.devicePointer + ((uint8_t*)p - (uint8_t*)a.hostPointer);
}

bool small_eligible(hvws_ctx* c, uint64_t len, const hvws_segment* segs, uint32_t nseg) {
    const uint64_t limit = c->small_limit ? c->small_limit : kSmallBatch;
    if (c->small_limit == ~0ull || len > limit || nseg == 0) return false;
    for (uint32_t s = 0; s < nseg; ++s)
        if (segs[s].len > kSmallSegment) return false;
    return true;
}

// hvws_rx_batch for small batches: one H2D copy, k_small, one sync.
int rx_batch_small(hvws_ctx* c, uint8_t* h_rx, uint64_t len, const hvws_segment* segs, websocket_parser* carry,
                   uint32_t nseg, int unmask, uint8_t* dev_base = nullptr) {
    for (uint32_t s = 0; s < nseg; ++s) {
        if (segs[s].off > len || segs[s].len > len - segs[s].off)
            return set_err(HVWS_EINVAL, "segment %u [%llu,+%llu) outside the %llu-byte buffer", s,
                           (unsigned long long)segs[s].off, (unsigned long long)segs[s].len, (unsigned long long)len);
        if (s && segs[s].off < segs[s - 1].off + segs[s - 1].len)
            return set_err(HVWS_EINVAL, "segments must be sorted and disjoint (segment %u)", s);
    }
    // packet: [counter | segs | carry | slot_base | data (256-aligned)]
    const uint64_t o_segs = 64;
    const uint64_t o_carry = o_segs + (uint64_t)nseg * sizeof(dseg);
    const uint64_t o_slot = o_carry + (uint64_t)nseg * sizeof(dcarry);
    const uint64_t o_data = (o_slot + (uint64_t)nseg * 8 + 255) & ~255ull;
    // pinned caller buffer: read and write it directly.  dev_base (hvws_rx_reads):
    // the segments are the callers' registered pinned reads, offsets from dev_base.
    uint8_t* user_mapped = dev_base ? dev_base : host_mapped(h_rx);
    const uint64_t pkt = user_mapped ? o_data : o_data + len;
    // Segments of event-loop size are staged in LDS by k_small; small
    // batches of them may also go zero-copy (the kernel reads the packet and
    // the bytes from pinned host memory, no H2D copy ahead of the launch).
    uint64_t max_seg = 0;
    for (uint32_t s = 0; s < nseg; ++s) max_seg = std::max<uint64_t>(max_seg, segs[s].len);
    const bool stage = max_seg <= kStageSegment;
    const bool zc = dev_base || (stage && c->small_zc && len <= c->zc_batch);
    if (dev_base && !stage) return set_err(HVWS_EINVAL, "registered reads must be at most %llu bytes each",
                                           (unsigned long long)kStageSegment);
    const uint32_t stage_lds = stage ? (uint32_t)(((max_seg + 15) & ~15ull) + 16) : 0u;
    // The pinned packet may still be the source of an in-flight copy --
    // unless the last small call saw every completion word: then its copy
    // and its kernel's host accesses are over, and waiting for the stream
    // would only wait for the kernel's end-of-pipe signal (~10 us).
    if (!c->small_quiet) HIP_OR(hipStreamSynchronize(c->stream), HVWS_EHIP);
    c->small_quiet = false;
    // The packet carries the bytes only when the caller's buffer is not
    // device-mapped; the device copy exists only without zero-copy.  (With
    // dev_base, len spans all the reads' addresses, not bytes to move.)
    HIP_OR(c->h_small_in.ensure(o_data + (user_mapped ? 0 : len) + 64), HVWS_ENOMEM);
    if (!zc) HIP_OR(c->d_small_in.ensure(o_data + len + 64), HVWS_ENOMEM);
    uint8_t* hp = c->h_small_in.as<uint8_t>();
    memset(hp, 0, 64);
    dseg* hs = (dseg*)(hp + o_segs);
    dcarry* hc = (dcarry*)(hp + o_carry);
    uint64_t* hb = (uint64_t*)(hp + o_slot);
    uint64_t nslots = 0;
    for (uint32_t s = 0; s < nseg; ++s) {
        hs[s].off = segs[s].off;
        hs[s].len = segs[s].len;
        if (carry) to_dcarry(carry[s], hc[s]);
        else memset(&hc[s], 0, sizeof(dcarry));
        hb[s] = nslots;
        nslots += segs[s].len / 2 + 3;   // carried-in frame + >= 2 bytes per frame + tail
    }
    if (!user_mapped && len) par_memcpy(hp + o_data, h_rx, len);
    const uint64_t hcap = std::min<uint64_t>(nslots, kSmallHostRecords);
    HIP_OR(c->d_small_slots.ensure(nslots * sizeof(drec) + 64), HVWS_ENOMEM);
    HIP_OR(c->h_small_out.ensure((uint64_t)nseg * sizeof(dsmall_out) + hcap * sizeof(drec) + 64), HVWS_ENOMEM);
    dsmall_out* ho = c->h_small_out.as<dsmall_out>();
    drec* hr = (drec*)(ho + nseg);
    dsmall_out* ho_d = mapped<dsmall_out>(c->h_small_out);
    uint8_t* hp_d = mapped<uint8_t>(c->h_small_in);
    if (!ho_d || !hp_d) return set_err(HVWS_EHIP, "pinned buffers not device-mapped");
    // Record counter: device memory, only ever grows; this call's records
    // start at small_ctr_base (no per-call reset operation).
    HIP_OR(c->d_small_ctr.ensure(64), HVWS_ENOMEM);
    unsigned long long* ctr = c->d_small_ctr.as<unsigned long long>();
    if (c->small_ctr_dirty) {
        HIP_OR(hipMemsetAsync(ctr, 0, 8, c->stream), HVWS_EHIP);
        c->small_ctr_base = 0;
        c->small_ctr_dirty = false;
    }
    const uint64_t ctr_base = c->small_ctr_base;
    c->small_ctr_dirty = true;   // until this call's record total is known
    uint8_t* d = hp_d;           // zero-copy: the kernel reads the pinned packet in place
    if (!zc) {
        d = c->d_small_in.as<uint8_t>();
        HIP_OR(hipMemcpyAsync(d, hp, pkt, hipMemcpyHostToDevice, c->stream), HVWS_EHIP);
        if (user_mapped && len)
            HIP_OR(hipMemcpyAsync(d + o_data, h_rx, len, hipMemcpyHostToDevice, c->stream), HVWS_EHIP);
    }
    const uint8_t* d_rx = zc ? (user_mapped ? user_mapped : hp_d + o_data) : d + o_data;
    // No timing events unless $HVWS_EXPERIMENT step_events >= 2 asks for them: an
    // event-carrying launch costs a per-read call ~10 us of ~38 (r2an).
    static const bool timed_env = experiment("step_events") && atoi(experiment("step_events")) >= 2;
    const bool timed = timed_env && c->t_on;
    // Completion: each wave releases its stores to system scope and then
    // writes its segment's word with this call's sequence number; the host
    // polls the words (in segment order) instead of waiting for the stream,
    // which also waits for the kernel's end-of-pipe release and signal.
    uint64_t* done_d = nullptr;
    const volatile uint64_t* done_h = nullptr;
    const uint64_t seq = ++c->small_seq;
    if (c->small_poll) {
        HIP_OR(c->h_small_done.ensure((uint64_t)nseg * 8 + 64), HVWS_ENOMEM);
        done_d = mapped<uint64_t>(c->h_small_done);
        done_h = c->h_small_done.as<uint64_t>();
        if (!done_d) return set_err(HVWS_EHIP, "pinned completion words not device-mapped");
    }
    HIP_OR(begin_timed_scan(c, false), HVWS_EHIP);
    HIP_OR(launch_small(d_rx, len, (const dseg*)(d + o_segs), (const dcarry*)(d + o_carry), nseg,
                        (const uint64_t*)(d + o_slot), c->d_small_slots.as<drec>(), ctr, ctr_base,
                        (drec*)(ho_d + nseg), hcap, ho_d, user_mapped ? user_mapped : hp_d + o_data, unmask,
                        c->vmask, stage_lds, done_d, seq, c->stream, timed ? c->tev[c->t_cur][0] : nullptr,
                        timed ? c->tev[c->t_cur][1] : nullptr),
           HVWS_EHIP);
    if (timed) c->t_rec[c->t_cur] |= 3u;
    if (done_h) {
        // Spin on the words; now and then ask the stream, so a kernel that
        // faulted (or was never dispatched) ends the wait with its error.
        // (The stream is asked at most every ~100 us: a query takes the
        // runtime's locks, and right after a launch one cost ~7 us.)
        uint32_t s = 0, spins = 0;
        auto next_query = std::chrono::steady_clock::now() + std::chrono::microseconds(100);
        while (s < nseg) {
            if (done_h[s] == seq) {
                ++s;
                continue;
            }
            if ((++spins & 63u) == 0 && std::chrono::steady_clock::now() >= next_query) {
                next_query = std::chrono::steady_clock::now() + std::chrono::microseconds(100);
                const hipError_t q = hipStreamQuery(c->stream);
                if (q == hipSuccess) {   // finished: every word is written
                    if (done_h[s] != seq) return set_err(HVWS_EHIP, "k_small finished without completing segment %u", s);
                    continue;
                }
                if (q != hipErrorNotReady) return set_err(HVWS_EHIP, "k_small: %s", hipGetErrorString(q));
            }
            __builtin_ia32_pause();
        }
        __atomic_thread_fence(__ATOMIC_ACQUIRE);
    } else {
        HIP_OR(hipStreamSynchronize(c->stream), HVWS_EHIP);
    }
    c->small_quiet = true;
    if (!user_mapped && unmask && len) par_memcpy(h_rx, hp + o_data, len);
    // host cache in segment order
    uint64_t total = 0;
    for (uint32_t s = 0; s < nseg; ++s) total += ho[s].count;
    c->small_ctr_base = ctr_base + total;
    c->small_ctr_dirty = false;
    c->hcache.resize(total);
    c->hfirst.resize(nseg);
    c->hcount.resize(nseg);
    c->hcarry.resize(nseg);
    // A segment whose records fit the pinned area (first + count <= hcap)
    // wrote them there; the others left them in their device slots only.
    bool on_host = true;
    const drec* slots_base = c->d_small_slots.as<drec>();
    uint64_t k = 0;
    for (uint32_t s = 0; s < nseg; ++s) {
        const uint64_t cnt = ho[s].count;
        c->hfirst[s] = k;
        c->hcount[s] = cnt;
        c->hcarry[s] = ho[s].st;
        if (cnt) {
            if (ho[s].first + cnt <= hcap) {
                memcpy(&c->hcache[k], hr + ho[s].first, cnt * sizeof(drec));
            } else {
                on_host = false;
                HIP_OR(hipMemcpyAsync(&c->hcache[k], slots_base + hb[s], cnt * sizeof(drec), hipMemcpyDeviceToHost,
                                      c->stream),
                       HVWS_EHIP);
            }
        }
        k += cnt;
    }
    if (!on_host) HIP_OR(hipStreamSynchronize(c->stream), HVWS_EHIP);
    c->nseg = nseg;
    c->nfr = total;
    c->nfr_known = true;
    c->rx = nullptr;   // the device frame table is not populated: hvws_unmask refuses
    c->rx_len = 0;
    c->have_scan = true;
    c->hcache_valid = true;
    if (carry) {
        for (uint32_t s = 0; s < nseg; ++s) {
            void* keep = carry[s].data;
            from_dcarry(c->hcarry[s], carry[s]);
            carry[s].data = keep;
        }
    }
    return HVWS_OK;
}

// ------------------------------------------------- resident small-path worker
// k_door (hvws_kernels.hip, ddoor in hvws_internal.h) serves the reference
// API's single calls -- FeedRecvData / websocket_parser_execute on one read,
// websocket_decode, websocket_parser_decode, a masked websocket_build_frame --
// from a mailbox in fine-grained pinned memory: no launch, no dispatch and no
// end-of-kernel signal per call.

// Idle time after which a worker parks ($HVWS_EXPERIMENT door_idle_us, default 5 ms),
// in ticks of the 100 MHz realtime clock.
std::atomic<uint64_t> g_door_idle_us{0};   // 0: not yet read from the environment

uint64_t door_idle_us() {
    uint64_t us = g_door_idle_us.load(std::memory_order_relaxed);
    if (!us) {
        const char* e = experiment("door_idle_us");
        us = e && strtoull(e, nullptr, 0) ? strtoull(e, nullptr, 0) : 5000;
        g_door_idle_us.store(us, std::memory_order_relaxed);
    }
    return us;
}

uint64_t door_idle_ticks() { return door_idle_us() * 100; }

bool door_on(hvws_ctx* c) {
    if (c->door_broken) return false;
    if (c->door_mode >= 0) return c->door_mode != 0;
    static const int env = getenv("HVWS_DOOR") ? atoi(getenv("HVWS_DOOR")) : 1;   // on by default (round 4)
    return env != 0;
}

// Contexts that own a worker queue.  Lock order: g_door_m, then a
// context's door_m; nothing that holds a door_m takes g_door_m.
std::mutex g_door_m;
std::vector<hvws_ctx*> g_doors;
// Idle worker queues of released contexts, for the next context's worker on
// that device (creating one is the costliest step of a context's first call);
// destroyed at exit.  Guarded by g_door_m.
std::vector<door_queue*> g_door_pool;
std::atomic<int> g_door_count{0};   // g_doors.size(): frees skip the lock when no worker exists
void door_atexit();
// Process-wide failure counts (hvws_door_health; the test session fails on
// either): worker streams that did not drain within their bound (left
// wedged), and requests a worker did not answer (the context then launches
// per call).  Both are printed to stderr as they happen.
std::atomic<uint64_t> g_door_wedged{0};
std::atomic<uint64_t> g_door_failed{0};

// Worker streams per device at most ($HVWS_DOOR_MAX, default 8): each is a
// hardware queue of its own, and queues beyond what the hardware scheduler
// maps at once are time-sliced -- a resident worker could then go
// unscheduled.  A context past the cap serves its reads with a launch each.
int door_cap() {
    static const int cap = getenv("HVWS_DOOR_MAX") && atoi(getenv("HVWS_DOOR_MAX")) > 0 ? atoi(getenv("HVWS_DOOR_MAX")) : 8;
    return cap;
}

// Marks the runtime call a context is in for the wedge report and
// hvws_debug_dump (a hang then names its call, not only its thread).
struct in_call {
    hvws_ctx* c;
    const char* prev;
    in_call(hvws_ctx* c_, const char* what) : c(c_), prev(c_->at.exchange(what)) {}
    ~in_call() { c->at.store(prev); }
};

// The request area in device memory: its 128-byte request block, then the
// request bytes.
constexpr uint64_t kDoorReqBytes = 256 + kDoorMax + 256;

bool door_vram_enabled() {
    static const int v = experiment("door_vram") ? atoi(experiment("door_vram")) : 1;
    return v != 0;
}

// Host stores to device memory go through write-combining buffers: an sfence
// makes them visible (the request bytes before seq, and seq itself; without
// it a lone 8-byte seq store sat in a WC buffer for ~10 ms,
// profiles/r4a_raw/vram_probe.jsonl).
inline void door_flush_wc() { __builtin_ia32_sfence(); }

// A request's bytes into the mailbox.  Device memory behind the BAR is
// write-combining: with AVX-512 every store is one whole 64-byte line, a
// non-temporal one (the sfence in door_call drains them); otherwise memcpy.
__attribute__((target("avx512f"))) void wc_copy_avx512(uint8_t* dst, const uint8_t* src, size_t n) {
    size_t i = 0;
    for (; i + 64 <= n; i += 64) _mm512_stream_si512((__m512i*)(dst + i), _mm512_loadu_si512(src + i));
    if (i < n) memcpy(dst + i, src + i, n - i);
}
void door_copy_in(hvws_ctx* c, uint8_t* dst, const void* src, size_t n) {
    static const bool avx512 = __builtin_cpu_supports("avx512f");
    if (c->d_door_req && avx512 && ((uintptr_t)dst & 63u) == 0) wc_copy_avx512(dst, static_cast<const uint8_t*>(src), n);
    else memcpy(dst, src, n);
}

// Where the host writes a request (block and bytes) and where the worker reads it.
ddoor* door_req(hvws_ctx* c) { return c->d_door_req ? (ddoor*)c->d_door_req : c->h_door.as<ddoor>(); }
uint8_t* door_din(hvws_ctx* c) {
    return c->d_door_req ? (uint8_t*)c->d_door_req + 256 : c->h_door_data.as<uint8_t>();
}

// A context that gets no worker serves its calls with a launch each (its
// callers fall back on any failure here), so the thread's last-error text is
// left as it was: the call itself succeeds.
int door_ensure_impl(hvws_ctx* c);
int door_ensure(hvws_ctx* c) {
    if (c->door_q) return HVWS_OK;
    char saved[sizeof g_err];
    memcpy(saved, g_err, sizeof g_err);
    const int rc = door_ensure_impl(c);
    if (rc != HVWS_OK) memcpy(g_err, saved, sizeof g_err);
    return rc;
}

int door_ensure_impl(hvws_ctx* c) {
    {
        std::lock_guard<std::mutex> lk(g_door_m);
        int same = 0;
        for (const hvws_ctx* o : g_doors) same += o->device == c->device;
        if (same >= door_cap()) return set_err(HVWS_EINVAL, "k_door: %d workers on device %d already", same, c->device);
    }
    HIP_OR(hipSetDevice(c->device), HVWS_EHIP);
    hipDeviceProp_t prop;
    HIP_OR(hipGetDeviceProperties(&prop, c->device), HVWS_EHIP);
    // The mailbox is fine-grained (polled, uncached); the data and record
    // areas are ordinary pinned memory: the worker's system-scope acquire on
    // each request invalidates its caches before it stages the bytes, and its
    // release writes its results back.  (Fine-grained data made the staging
    // loads of an 8 KiB read take 6.2 us, profiles/r3f_raw.)
    c->h_door.flags = hipHostMallocCoherent;
    HIP_OR(c->h_door.ensure(sizeof(ddoor)), HVWS_ENOMEM);
    HIP_OR(c->h_door_data.ensure(kDoorMax + 256), HVWS_ENOMEM);
    HIP_OR(c->h_door_rec.ensure(kDoorRecords * sizeof(drec)), HVWS_ENOMEM);
    HIP_OR(c->d_door_slot.ensure(kDoorRecords * sizeof(drec)), HVWS_ENOMEM);
    memset(c->h_door.p, 0, sizeof(ddoor));
    if (!mapped<ddoor>(c->h_door) || !mapped<uint8_t>(c->h_door_data) || !mapped<drec>(c->h_door_rec))
        return set_err(HVWS_EHIP, "worker mailbox not device-mapped");
    if (door_vram_enabled() && prop.isLargeBar && !c->d_door_req) {
        // With a large BAR, fine-grained device memory is mapped for the host
        // at its device address (profiles/r4a_raw/vram_probe.jsonl: host
        // stores and loads work, an 8 KiB memcpy into it takes 0.49 us);
        // without one the request area stays pinned host memory.
        void* p = nullptr;
        if (hipExtMallocWithFlags(&p, kDoorReqBytes, hipDeviceMallocFinegrained) == hipSuccess) {
            c->d_door_req = p;
            memset(p, 0, sizeof(ddoor));
            door_flush_wc();
        }
        (void)hipGetLastError();
    }
    std::lock_guard<std::mutex> lk(g_door_m);
    int same = 0;   // again, under the lock that also registers this context
    for (const hvws_ctx* o : g_doors) same += o->device == c->device;
    if (same >= door_cap()) return set_err(HVWS_EINVAL, "k_door: %d workers on device %d already", same, c->device);
    for (size_t i = 0; i < g_door_pool.size(); ++i)
        if (g_door_pool[i]->device == c->device) {
            c->door_q = g_door_pool[i];
            g_door_pool.erase(g_door_pool.begin() + (long)i);
            break;
        }
    if (!c->door_q) {
        in_call ic(c, "hsa_queue_create (worker queue)");
        if (int rc = door_queue_create(c->device, &c->door_q)) return set_err(rc, "%s", door_queue_why());
    }
    // registered after the HIP runtime's own exit handlers, so it runs before them
    static const bool reg = (atexit(door_atexit), true);
    (void)reg;
    g_doors.push_back(c);
    g_door_count.store((int)g_doors.size(), std::memory_order_release);
    return HVWS_OK;
}

uint64_t door_word(const hvws_ctx* c, const uint64_t& w) {
    (void)c;
    return __atomic_load_n(&w, __ATOMIC_ACQUIRE);
}

// Wait up to `ms` for the worker's last launch to end (its completion
// signal: never an unbounded wait -- a worker that never ends must not hang
// its host thread).  On a timeout the mailbox state goes to stderr and the
// context is marked wedged: its queue and mailbox are never reused or freed.
bool door_drain(hvws_ctx* c, int ms, const char* where) {
    const auto t0 = std::chrono::steady_clock::now();
    for (;;) {
        if (door_queue_idle(c->door_q)) return true;
        if (const int e = door_queue_error(c->door_q)) {
            set_err(HVWS_EHIP, "k_door: worker queue error 0x%x", e);
            return true;   // the queue failed: nothing of the worker runs any more
        }
        if (std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(ms)) break;
        usleep(20);
    }
    const ddoor* b = c->h_door.as<ddoor>();
    const ddoor* rq = door_req(c);
    fprintf(stderr,
            "[hvws] k_door (%s): ctx %p worker launch still running after %d ms: seq %llu done %llu alive %llu "
            "exited %llu epoch %llu served %llu live %d\n",
            where, (void*)c, ms, (unsigned long long)__atomic_load_n(&rq->seq, __ATOMIC_ACQUIRE),
            (unsigned long long)door_word(c, b->done), (unsigned long long)door_word(c, b->alive),
            (unsigned long long)door_word(c, b->exited), (unsigned long long)c->door_epoch,
            (unsigned long long)door_word(c, b->served), (int)c->door_live);
    c->door_wedged = true;
    g_door_wedged.fetch_add(1);
    set_err(HVWS_EHIP, "k_door: the worker launch did not end (%s)", where);
    return false;
}

// Post the request already written into the mailbox and wait for it (the
// caller holds c->door_m).  A worker is (re)launched when none is resident.
// Whether the resident one has ended is read from the mailbox: its last
// store is `exited = epoch`; a relaunch also waits for the last launch's
// completion signal (door_drain), so two workers never share the mailbox.
// The queue's error state says whether a kernel fault ended it.
// pf, pf_len: results the caller copies out once `done` is seen.  The
// worker's stores land in host memory before `done` (its release waits for
// them), so prefetching those lines while waiting pulls them into the cache
// as they land instead of after `done`.
int door_call(hvws_ctx* c, const void* pf = nullptr, size_t pf_len = 0) {
    ddoor* b = c->h_door.as<ddoor>();
    ddoor* rq = door_req(c);
    const uint64_t seq = ++c->door_seq;
    rq->seq_tail = seq;
    if (c->d_door_req) door_flush_wc();   // the request's bytes and fields first
    __atomic_store_n(&rq->seq, seq, __ATOMIC_RELEASE);
    if (c->d_door_req) door_flush_wc();
    ++c->door_calls;
    const auto t0 = std::chrono::steady_clock::now();
    auto next_query = t0 + std::chrono::microseconds(100);
    uint32_t spins = 0, launches = 0;
    for (;;) {
        if (__atomic_load_n(&b->done, __ATOMIC_ACQUIRE) == seq) return HVWS_OK;
        if (!c->door_live) {
            if (c->door_wedged) return set_err(HVWS_EHIP, "k_door: the worker stream is wedged");
            if (launches++ >= 4) return set_err(HVWS_EHIP, "k_door: the worker takes no requests");
            HIP_OR(hipSetDevice(c->device), HVWS_EHIP);
            __atomic_store_n(&b->alive, 1ull, __ATOMIC_RELAXED);
            ++c->door_epoch;
            const ddoor* dreq = c->d_door_req ? (const ddoor*)c->d_door_req : mapped<ddoor>(c->h_door);
            const uint8_t* ddin = c->d_door_req ? (const uint8_t*)c->d_door_req + 256 : mapped<uint8_t>(c->h_door_data);
            door_args a;
            a.req = dreq;
            a.box = mapped<ddoor>(c->h_door);
            a.din = ddin;
            a.dout = mapped<uint8_t>(c->h_door_data);
            a.h_rec = mapped<drec>(c->h_door_rec);
            a.d_slot = c->d_door_slot.as<drec>();
            a.idle_ticks = door_idle_ticks();
            a.first_seq = __atomic_load_n(&b->done, __ATOMIC_ACQUIRE);
            a.epoch = c->door_epoch;
            a.flags = door_flags();
            in_call ic(c, "AQL dispatch of k_door (worker queue)");
            if (int rc = door_queue_launch(c->door_q, &a, (uint32_t)sizeof a)) return set_err(rc, "%s", door_queue_why());
            c->door_live = true;
            ++c->door_launches;
            continue;
        }
        if (door_word(c, b->exited) == c->door_epoch) {
            // The worker has ended; its last look at seq came before this
            // request.  Its launch completes (the wave retires) before the
            // next launch, so two workers never share the mailbox.
            if (__atomic_load_n(&b->done, __ATOMIC_ACQUIRE) == seq) return HVWS_OK;
            if (!door_drain(c, 5000, "relaunch")) return HVWS_EHIP;
            c->door_live = false;
            continue;
        }
        if ((++spins & 63u) == 0) {
            const auto now = std::chrono::steady_clock::now();
            if (now >= next_query) {
                next_query = now + std::chrono::microseconds(100);
                if (const int e = door_queue_error(c->door_q)) return set_err(HVWS_EHIP, "k_door: worker queue error 0x%x", e);
                if (now - t0 > std::chrono::seconds(10)) return set_err(HVWS_EHIP, "k_door: no answer in 10 s");
            }
        }
        if (pf_len)
            for (size_t i = 0; i < pf_len; i += 64) __builtin_prefetch(static_cast<const char*>(pf) + i);
        else
            __builtin_ia32_pause();
    }
}

// Send the resident worker home and wait until it has ended (the caller
// holds c->door_m): context teardown, a free, a thread's exit, the door
// switched off.
void door_park(hvws_ctx* c) {
    if (!c->door_q || !c->door_live || c->door_wedged) return;
    ddoor* b = c->h_door.as<ddoor>();
    if (door_word(c, b->exited) != c->door_epoch) {
        door_req(c)->op = DOOR_EXIT;
        if (door_call(c) != HVWS_OK) {
            (void)hipGetLastError();
        } else {
            // served: the worker's `exited` store follows `done`
            const auto t0 = std::chrono::steady_clock::now();
            while (door_word(c, b->exited) != c->door_epoch &&
                   std::chrono::steady_clock::now() - t0 < std::chrono::seconds(1))
                __builtin_ia32_pause();
        }
    }
    if (door_drain(c, 5000, "park")) c->door_live = false;
}

// The calling thread's context for the reference-API entry points.
thread_local int t_device = -1;
thread_local hvws_ctx* t_ctx = nullptr;

// Park every worker on the current device before a free (whichever thread
// owns it); the current device is restored afterwards.
void door_park_device() {
    if (g_door_count.load(std::memory_order_acquire) == 0) return;
    int dev = -1;
    if (hipGetDevice(&dev) != hipSuccess) return;
    std::lock_guard<std::mutex> lk(g_door_m);
    for (hvws_ctx* c : g_doors) {
        if (c->device != dev || !c->door_live) continue;
        std::lock_guard<std::mutex> cl(c->door_m);
        door_park(c);
    }
    hipSetDevice(dev);
}

// At process exit: no HIP call at all (an exit handler that destroyed the
// worker streams hung a process's exit, profiles/r3ab_raw).  A worker still
// resident is asked to exit through the mailbox and given up to 100 ms to
// say it has ended; a context whose owner holds its lock past 100 ms is left
// as it is.
void door_quit_nohip(hvws_ctx* c) {
    if (!c->door_q || !c->door_live) return;
    ddoor* b = c->h_door.as<ddoor>();
    if (door_word(c, b->exited) != c->door_epoch) {
        ddoor* rq = door_req(c);
        rq->op = DOOR_EXIT;
        rq->seq_tail = c->door_seq + 1;
        if (c->d_door_req) door_flush_wc();
        __atomic_store_n(&rq->seq, ++c->door_seq, __ATOMIC_RELEASE);
        if (c->d_door_req) door_flush_wc();
        const auto t0 = std::chrono::steady_clock::now();
        while (door_word(c, b->exited) != c->door_epoch &&
               std::chrono::steady_clock::now() - t0 < std::chrono::milliseconds(100))
            __builtin_ia32_pause();
    }
    c->door_live = false;
}

// At exit, once every worker has ended (its launch's completion signal),
// the worker queues are destroyed (HSA calls only; this handler runs before
// the HIP runtime's own, so the HSA runtime is still up).  A process that
// ended with a worker queue alive crashed under rocprofv3; a
// queue whose worker did not end is left alone.
void door_atexit() {
    std::lock_guard<std::mutex> lk(g_door_m);
    for (hvws_ctx* c : g_doors) {
        std::unique_lock<std::mutex> cl(c->door_m, std::defer_lock);
        const auto t0 = std::chrono::steady_clock::now();
        while (!cl.try_lock() && std::chrono::steady_clock::now() - t0 < std::chrono::milliseconds(100)) usleep(100);
        if (!cl.owns_lock()) continue;
        door_quit_nohip(c);
        if (!c->door_q || c->door_wedged) continue;
        const auto t1 = std::chrono::steady_clock::now();
        while (!door_queue_idle(c->door_q) && std::chrono::steady_clock::now() - t1 < std::chrono::milliseconds(100))
            usleep(50);
        if (door_queue_idle(c->door_q)) {
            c->door_q->at_exit = true;
            door_queue_destroy(c->door_q);
            c->door_q = nullptr;
        }
    }
    for (door_queue* q : g_door_pool) {
        q->at_exit = true;
        door_queue_destroy(q);
    }
    g_door_pool.clear();
}

void door_release(hvws_ctx* c) {
    if (!c->door_q) return;
    {
        std::lock_guard<std::mutex> lk(g_door_m);
        {
            std::lock_guard<std::mutex> cl(c->door_m);
            door_park(c);
        }
        g_doors.erase(std::remove(g_doors.begin(), g_doors.end(), c), g_doors.end());
        g_door_count.store((int)g_doors.size(), std::memory_order_release);
    }
    if (c->door_wedged || !door_drain(c, 5000, "release")) {
        // a worker that may still run: its queue and the memory it writes stay
        fprintf(stderr, "[hvws] k_door: ctx %p released with its worker launch wedged; queue and mailbox leaked\n",
                (void*)c);
        c->door_q = nullptr;
        c->h_door.p = c->h_door_data.p = c->h_door_rec.p = nullptr;
        c->d_door_slot.p = nullptr;
        c->d_door_req = nullptr;
        return;
    }
    {
        // ended: the next context's worker takes the queue (destroyed at exit)
        std::lock_guard<std::mutex> lk(g_door_m);
        g_door_pool.push_back(c->door_q);
    }
    c->door_q = nullptr;
    in_call ic(c, "hipHostFree / hipFree (worker mailbox and areas)");
    c->h_door.release();
    c->h_door_data.release();
    c->h_door_rec.release();
    c->d_door_slot.release();
    if (c->d_door_req) {
        door_park_device();
        hipFree(c->d_door_req);
        c->d_door_req = nullptr;
    }
}

// A request the worker did not answer (the caller holds c->door_m): counted
// and reported, and the context launches per call from now on.  The caller's
// buffer is untouched until a request succeeds, so the caller serves this
// call on the launch path itself (advisor r4: no abort).
void door_fail(hvws_ctx* c, const char* what) {
    g_door_failed.fetch_add(1);
    fprintf(stderr, "[hvws] k_door: ctx %p: %s request unanswered (%s); this context launches per call from now on\n",
            (void*)c, what, g_err);
    c->door_broken = true;
    if (c->door_live && !c->door_wedged && door_drain(c, 1000, "failed request")) c->door_live = false;
}

// $HVWS_EXPERIMENT feed_times=1: host time per phase of door_feed (request
// written, answered, results copied back), printed at exit (diagnostic).
struct door_times {
    bool on = experiment("feed_times") && atoi(experiment("feed_times"));
    std::atomic<uint64_t> calls{0}, ns[3] = {};
    ~door_times() {
        const uint64_t n = calls.load();
        if (on && n)
            fprintf(stderr, "[door_times] calls=%llu us/call: request %.2f answer %.2f results %.2f\n",
                    (unsigned long long)n, ns[0].load() / 1e3 / n, ns[1].load() / 1e3 / n, ns[2].load() / 1e3 / n);
    }
};
door_times g_door_times;

// One read through the worker (gpu_feed's fast path): false when the worker
// does not take it (off, or longer than kDoorMax).
bool door_feed(hvws_ctx* c, char* buf, size_t len, const websocket_parser& carry, bool unmask,
               std::vector<hvws_frame>& frames, websocket_parser& carry_out, int& started) {
    if (!door_on(c) || len > kDoorMax || door_ensure(c) != HVWS_OK) return false;
    std::lock_guard<std::mutex> cl(c->door_m);
    using clk = std::chrono::steady_clock;
    const bool timed = g_door_times.on;
    clk::time_point t0, t1, t2;
    if (timed) t0 = clk::now();
    ddoor* b = c->h_door.as<ddoor>();
    ddoor* rq = door_req(c);
    uint8_t* data = c->h_door_data.as<uint8_t>();
    door_copy_in(c, door_din(c), buf, len);
    rq->op = DOOR_FEED;
    rq->unmask = unmask ? 1u : 0u;
    rq->len = len;
    rq->vmask = c->vmask;
    dcarry cin;
    to_dcarry(carry, cin);
    memcpy(&rq->carry, &cin, sizeof(dcarry));
    if (timed) t1 = clk::now();
    if (door_call(c, data, unmask ? len : 0) != HVWS_OK) {
        door_fail(c, "read");
        return false;
    }
    if (timed) t2 = clk::now();
    const uint64_t n = b->count;
    frames.resize((size_t)n);
    if (n) memcpy(frames.data(), c->h_door_rec.p, (size_t)n * sizeof(drec));
    if (unmask) memcpy(buf, data, len);
    copy_parser(carry_out, carry);
    const dcarry out = b->out;
    from_dcarry(out, carry_out);
    started = (int)out.started;
    if (timed) {
        const auto t3 = clk::now();
        g_door_times.calls.fetch_add(1, std::memory_order_relaxed);
        g_door_times.ns[0].fetch_add((uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(t1 - t0).count());
        g_door_times.ns[1].fetch_add((uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(t2 - t1).count());
        g_door_times.ns[2].fetch_add((uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(t3 - t2).count());
    }
    return true;
}

bool door_xor(hvws_ctx* c, char* dst, const char* src, size_t n, uint32_t key, uint32_t phase) {
    if (!door_on(c) || n > kDoorMax || door_ensure(c) != HVWS_OK) return false;
    std::lock_guard<std::mutex> cl(c->door_m);
    ddoor* rq = door_req(c);
    uint8_t* data = c->h_door_data.as<uint8_t>();
    door_copy_in(c, door_din(c), src, n);
    rq->op = DOOR_XOR;
    rq->len = n;
    rq->key = key;
    rq->phase = phase;
    if (door_call(c, data, n) != HVWS_OK) {
        door_fail(c, "XOR");
        return false;
    }
    memcpy(dst, data, n);
    return true;
}

// ------------------------------------------- registered pinned host memory
// Ranges the device can read and write in place (hvws_host_alloc,
// hvws_host_register).  hvws_rx_reads looks every read up here; a
// thread-local last hit makes the common case (many reads out of one pinned
// arena) one compare per read.
struct pinned_range {
    uintptr_t lo, hi;
    uint8_t* dev;
    bool registered;   // hipHostRegister'ed (unregister on removal), else hipHostMalloc'ed
};
std::shared_mutex g_pin_m;
std::vector<pinned_range> g_pins;     // sorted by lo, disjoint
std::atomic<uint64_t> g_pin_gen{1};   // bumped on every removal

void pin_add(void* p, uint64_t bytes, uint8_t* dev, bool registered) {
    std::unique_lock<std::shared_mutex> lk(g_pin_m);
    const pinned_range r{(uintptr_t)p, (uintptr_t)p + bytes, dev, registered};
    g_pins.insert(std::upper_bound(g_pins.begin(), g_pins.end(), r,
                                   [](const pinned_range& a, const pinned_range& b) { return a.lo < b.lo; }),
                  r);
}

// Removes the range starting at p; returns it (lo == 0 if none).
pinned_range pin_remove(void* p) {
    std::unique_lock<std::shared_mutex> lk(g_pin_m);
    for (auto it = g_pins.begin(); it != g_pins.end(); ++it)
        if (it->lo == (uintptr_t)p) {
            const pinned_range r = *it;
            g_pins.erase(it);
            g_pin_gen.fetch_add(1);
            return r;
        }
    return pinned_range{0, 0, nullptr, false};
}

// Device address of [p, p+len) if it lies inside one registered range.
uint8_t* pinned_dev(const void* p, uint64_t len) {
    thread_local pinned_range last{0, 0, nullptr, false};
    thread_local uint64_t last_gen = 0;
    const uintptr_t a = (uintptr_t)p;
    const uint64_t gen = g_pin_gen.load(std::memory_order_acquire);
    if (last_gen != gen || a < last.lo || a + len > last.hi) {
        std::shared_lock<std::shared_mutex> lk(g_pin_m);
        auto it = std::upper_bound(g_pins.begin(), g_pins.end(), a,
                                   [](uintptr_t v, const pinned_range& r) { return v < r.lo; });
        if (it == g_pins.begin()) return nullptr;
        --it;
        if (a + len > it->hi) return nullptr;
        last = *it;
        last_gen = gen;
    }
    return last.dev + (a - last.lo);
}

// Unmask launch after a scan of the same buffer.
int unmask_impl(hvws_ctx* c, uint8_t* d_rx, uint64_t rx_len) {
    int rc = check_ctx(c);
    if (rc) return rc;
    if (!c->have_scan) return set_err(HVWS_EINVAL, "hvws_unmask without a preceding hvws_scan");
    if (d_rx != c->rx || rx_len != c->rx_len)
        return set_err(HVWS_EINVAL, "hvws_unmask buffer differs from the scanned one");
    // After a RUN step its descriptors are spent (the repair cleared the
    // failure words): a further unmask of the batch goes through the exact
    // frame table, built now, so every frame is XORed again.
    if (c->run_active && (rc = run_materialize(c)) != HVWS_OK) return rc;
    HIP_OR(issue_unmask(c, d_rx, rx_len), HVWS_EHIP);
    return HVWS_OK;
}

void stall_fn(void* usec) { usleep((useconds_t)(uintptr_t)usec); }


// Every live context (hvws_debug_dump).
std::mutex g_ctx_m;
std::vector<hvws_ctx*> g_ctx_all;

int g_bt_fd = 2;
std::atomic<int> g_bt_done{0};

void bt_handler(int) {
    void* fr[64];
    const int n = backtrace(fr, 64);
    char hdr[64];
    const int l = snprintf(hdr, sizeof(hdr), "--- thread %ld\n", (long)syscall(SYS_gettid));
    if (l > 0) (void)!write(g_bt_fd, hdr, (size_t)l);
    backtrace_symbols_fd(fr, n, g_bt_fd);
    g_bt_done.fetch_add(1, std::memory_order_release);
}

const char* qname(hipError_t q) {
    return q == hipSuccess ? "idle" : q == hipErrorNotReady ? "busy" : hipGetErrorString(q);
}

}  // namespace

// ===================================================================== C ABI
extern "C" {

int hvws_debug_dump(int fd) {
    std::vector<hvws_ctx*> all;
    {
        std::lock_guard<std::mutex> lk(g_ctx_m);
        all = g_ctx_all;
    }
    dprintf(fd, "libhvws: %zu contexts, %d with a worker stream\n", all.size(), g_door_count.load());
    // memory state first (no HIP call, no lock a stuck caller could hold)
    for (hvws_ctx* c : all) {
        dprintf(fd, "  ctx %p dev %d door_mode %d door_live %d door_seq %llu epoch %llu launches %llu calls %llu",
                (void*)c, c->device, c->door_mode, (int)c->door_live, (unsigned long long)c->door_seq,
                (unsigned long long)c->door_epoch, (unsigned long long)c->door_launches,
                (unsigned long long)c->door_calls);
        if (c->h_door.p) {
            const ddoor* b = c->h_door.as<ddoor>();
            dprintf(fd, " | mailbox%s seq %llu done %llu alive %llu exited %llu served %llu op %u",
                    c->d_door_req ? " (request in device memory)" : "",
                    (unsigned long long)__atomic_load_n(&door_req(c)->seq, __ATOMIC_ACQUIRE),
                    (unsigned long long)__atomic_load_n(&b->done, __ATOMIC_ACQUIRE),
                    (unsigned long long)__atomic_load_n(&b->alive, __ATOMIC_ACQUIRE),
                    (unsigned long long)__atomic_load_n(&b->exited, __ATOMIC_ACQUIRE),
                    (unsigned long long)__atomic_load_n(&b->served, __ATOMIC_ACQUIRE), door_req(c)->op);
        }
        const char* at = c->at.load();
        dprintf(fd, " | wedged %d broken %d | in %s | last scan path %d, have_scan %d\n", (int)c->door_wedged,
                (int)c->door_broken, at ? at : "-", c->scan_path, (int)c->have_scan);
    }
    dprintf(fd, "libhvws: worker launches wedged %llu, requests unanswered %llu (process)\n",
            (unsigned long long)g_door_wedged.load(), (unsigned long long)g_door_failed.load());
    for (hvws_ctx* c : all) {
        if (c->at.load()) {   // its streams may be going away under that call: not queried
            dprintf(fd, "  ctx %p streams: not queried (in %s)\n", (void*)c, c->at.load());
            continue;
        }
        dprintf(fd, "  ctx %p streams:", (void*)c);
        const struct {
            const char* n;
            hipStream_t s;
        } ss[] = {{"stream", c->stream}, {"sstream", c->sstream}, {"copy_in", c->copy_in},
                  {"copy_out", c->copy_out}};
        for (const auto& x : ss)
            if (x.s) dprintf(fd, " %s=%s", x.n, qname(hipStreamQuery(x.s)));
        if (c->door_q)
            dprintf(fd, " worker-queue=%s error=0x%x", door_queue_idle(c->door_q) ? "idle" : "running",
                    door_queue_error(c->door_q));
        dprintf(fd, "\n");
    }
    return (int)all.size();
}

int hvws_debug_backtraces(int fd) {
    struct sigaction sa = {}, old = {};
    sa.sa_handler = bt_handler;
    sigemptyset(&sa.sa_mask);
    sa.sa_flags = SA_RESTART;
    void* warm[4];
    (void)backtrace(warm, 4);   // loads the unwinder outside the handler
    g_bt_fd = fd;
    if (sigaction(SIGUSR2, &sa, &old) != 0) return -1;
    const long self = (long)syscall(SYS_gettid);
    int answered = 0;
    if (DIR* d = opendir("/proc/self/task")) {
        while (dirent* e = readdir(d)) {
            const long tid = atol(e->d_name);
            if (tid <= 0) continue;
            if (tid == self) {
                dprintf(fd, "--- thread %ld (the caller)\n", tid);
                continue;
            }
            const int before = g_bt_done.load(std::memory_order_acquire);
            if (syscall(SYS_tgkill, getpid(), tid, SIGUSR2) != 0) continue;
            for (int i = 0; i < 200 && g_bt_done.load(std::memory_order_acquire) == before; ++i) usleep(1000);
            if (g_bt_done.load(std::memory_order_acquire) != before) ++answered;
            else dprintf(fd, "--- thread %ld: no answer\n", tid);
        }
        closedir(d);
    }
    // A thread that had SIGUSR2 blocked, or sat in a long system call, takes
    // it after this returns: with the default action (terminate) restored,
    // that would kill a healthy process from its own diagnostics (advisor
    // r4).  So the handler stays installed unless the program had one.
    if (old.sa_handler != SIG_DFL || (old.sa_flags & SA_SIGINFO)) sigaction(SIGUSR2, &old, nullptr);
    return answered;
}


const char* hvws_last_error(void) { return g_err; }

int hvws_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

int hvws_device_identity(int device, char* bus_id, int len, int* cur) {
    if (!bus_id || len < 13) return set_err(HVWS_EINVAL, "bus id buffer too small");
    HIP_OR(hipSetDevice(device), HVWS_EHIP);
    int d = -1;
    HIP_OR(hipGetDevice(&d), HVWS_EHIP);
    if (cur) *cur = d;
    HIP_OR(hipDeviceGetPCIBusId(bus_id, len, d), HVWS_EHIP);
    return HVWS_OK;
}

hvws_ctx* hvws_ctx_create(int device) {
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess || n <= 0) {
        set_err(HVWS_ENODEV, "no HIP device available (%s)", e != hipSuccess ? hipGetErrorString(e) : "count 0");
        return nullptr;
    }
    if (device < 0 || device >= n) {
        set_err(HVWS_EINVAL, "device %d out of range (have %d)", device, n);
        return nullptr;
    }
    if ((e = hipSetDevice(device)) != hipSuccess) {
        set_err(HVWS_EHIP, "hipSetDevice(%d): %s", device, hipGetErrorString(e));
        return nullptr;
    }
    hvws_ctx* c = new hvws_ctx();
    c->device = device;
    {
        std::lock_guard<std::mutex> lk(g_ctx_m);
        g_ctx_all.push_back(c);
    }
    // Tables the device reads (upload slots) or writes (check verdict) in
    // host memory while the host uses them between launches: fine-grained,
    // so no stale copy can sit in a device cache across reuses.
    for (hbuf& b : c->h_up) b.flags = hipHostMallocCoherent;
    c->h_status.flags = hipHostMallocCoherent;
    c->h_small_done.flags = hipHostMallocCoherent;
    if (const char* sp = experiment("small_poll")) c->small_poll = atoi(sp) ? 1 : 0;
    if (const char* zc = experiment("small_zc")) c->small_zc = atoi(zc) ? 1 : 0;
    if (const char* zb = experiment("zc_batch")) c->zc_batch = strtoull(zb, nullptr, 0);
    if (const char* sp = experiment("spec")) c->spec_mode = atoi(sp) == 0 ? 0 : (atoi(sp) == 1 ? 1 : (atoi(sp) == 2 ? 2 : -1));
    if (const char* wv = experiment("walk_verify")) c->verify_mode = atoi(wv) < 0 ? -1 : (atoi(wv) ? 1 : 0);
    // The pipelined scan stream at the highest priority: a scan kernel of
    // ~1000 workgroups queued while an unmask grid is being dispatched waits
    // for that whole grid at normal priority, but is dispatched beside it at
    // high priority (scripts/dispatch_probe.hip).
    int prio_least = 0, prio_greatest = 0;
    (void)hipDeviceGetStreamPriorityRange(&prio_least, &prio_greatest);
    const int scan_prio = prio_greatest;
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
        hipStreamCreateWithFlags(&c->copy_in, hipStreamNonBlocking) != hipSuccess ||
        hipStreamCreateWithFlags(&c->copy_out, hipStreamNonBlocking) != hipSuccess ||
        hipStreamCreateWithPriority(&c->sstream, hipStreamNonBlocking, scan_prio) != hipSuccess) {
        set_err(HVWS_EHIP, "stream creation failed");
        hvws_ctx_destroy(c);
        return nullptr;
    }
    bool ev_ok = true;
    for (auto& ev : c->ev) ev_ok = ev_ok && hipEventCreate(&ev) == hipSuccess;
    for (auto& row : c->tev)
        for (auto& ev : row) ev_ok = ev_ok && hipEventCreate(&ev) == hipSuccess;
    for (auto& ev : c->up_ev) ev_ok = ev_ok && hipEventCreateWithFlags(&ev, hipEventDisableTiming) == hipSuccess;
    for (tset& t : c->ts) ev_ok = ev_ok && hipEventCreateWithFlags(&t.free_ev, hipEventDisableTiming) == hipSuccess;
    ev_ok = ev_ok && hipEventCreateWithFlags(&c->scan_done, hipEventDisableTiming) == hipSuccess;
    c->cs = c->stream;
    if (!ev_ok) {
        set_err(HVWS_EHIP, "event creation failed");
        hvws_ctx_destroy(c);
        return nullptr;
    }
    return c;
}

void hvws_ctx_destroy(hvws_ctx* c) {
    if (!c) return;
    hipSetDevice(c->device);
    door_release(c);
    // Each runtime call of the teardown is named while it runs (c->at): a
    // teardown that hangs names its call in the wedge report and
    // hvws_debug_dump (round 5: the r4k hang was inside this teardown).
    {
        in_call ic(c, "hipStreamSynchronize(stream)");
        if (c->stream) hipStreamSynchronize(c->stream);
    }
    {
        in_call ic(c, "hipStreamSynchronize(sstream)");
        if (c->sstream) hipStreamSynchronize(c->sstream);
    }
    {
        in_call ic(c, "hipFree (table sets)");
        for (tset& t : c->ts) t.release();
    }
    {
        in_call ic(c, "hipFree (scratch, sieve, pipeline, staging)");
        for (dbuf* b : {&c->sl_hdr, &c->sl_off, &c->sl_len, &c->sl_length, &c->sl_key, &c->sl_keyrot, &c->sl_info, &c->sl_bx})
            b->release();
        for (dbuf* b : {&c->sv_state, &c->sv_tcount, &c->sv_tbase, &c->sv_slot, &c->sv_pool, &c->sv_keep, &c->sv_kbase,
                        &c->sv_Spre, &c->sv_S, &c->sv_J0, &c->sv_J1,
                        &c->sv_mark, &c->sv_hops, &c->sv_rank, &c->sv_cnt, &c->sv_tmp, &c->sv_scr})
            b->release();
        for (dbuf* b : {&c->pipe_slot[0], &c->pipe_slot[1], &c->pipe_slot[2], &c->pipe_segs}) b->release();
        for (dbuf* b : {&c->segs, &c->carry_in, &c->stage, &c->xor_stage, &c->synth_sizes, &c->synth_tiles, &c->synth_bad,
                        &c->tx_size, &c->tx_off, &c->tx_scan, &c->tx_tiles, &c->tx_stat, &c->tx_span, &c->d_small_in,
                        &c->d_small_slots})
            b->release();
        c->chk.release();
    }
    {
        in_call ic(c, "hipHostFree (pinned buffers)");
        c->h_sv.release();
        c->h_tx.release();
        c->h_small_in.release();
        c->h_small_done.release();
        c->h_small_out.release();
        c->h_feed.release();
        c->h_segs.release();
        for (hbuf& b : c->h_up) b.release();
        c->h_total.release();
        c->h_chk.release();
        c->h_status.release();
    }
    {
        in_call ic(c, "hipEventDestroy");
        for (tset& t : c->ts)
            if (t.free_ev) hipEventDestroy(t.free_ev);
        if (c->sv_ev) hipEventDestroy(c->sv_ev);
        for (hipEvent_t ev : c->pipe_ev)
            if (ev) hipEventDestroy(ev);
        for (auto& ev : c->ev)
            if (ev) hipEventDestroy(ev);
        for (auto& row : c->tev)
            for (auto& ev : row)
                if (ev) hipEventDestroy(ev);
        for (auto& ev : c->up_ev)
            if (ev) hipEventDestroy(ev);
        for (auto& ev : c->span_ev)
            if (ev) hipEventDestroy(ev);
        if (c->scan_done) hipEventDestroy(c->scan_done);
    }
    {
        in_call ic(c, "hipStreamDestroy (context streams)");
        if (c->stream) hipStreamDestroy(c->stream);
        if (c->copy_in) hipStreamDestroy(c->copy_in);
        if (c->copy_out) hipStreamDestroy(c->copy_out);
        if (c->sstream) hipStreamDestroy(c->sstream);
    }
    {
        std::lock_guard<std::mutex> lk(g_ctx_m);
        g_ctx_all.erase(std::remove(g_ctx_all.begin(), g_ctx_all.end(), c), g_ctx_all.end());
    }
    delete c;
}

void* hvws_ctx_stream(hvws_ctx* c) { return c ? (void*)c->stream : nullptr; }
int hvws_ctx_device(hvws_ctx* c) { return c ? c->device : -1; }

void* hvws_dev_alloc(hvws_ctx* c, uint64_t bytes) {
    if (check_ctx(c) != HVWS_OK) return nullptr;
    void* p = nullptr;
    hipError_t e = hipMalloc(&p, bytes ? bytes : 16);
    if (e != hipSuccess) {
        set_err(HVWS_ENOMEM, "hipMalloc(%llu): %s", (unsigned long long)bytes, hipGetErrorString(e));
        return nullptr;
    }
    return p;
}

void hvws_dev_free(hvws_ctx* c, void* p) {
    if (!c || !p) return;
    hipSetDevice(c->device);
    door_park_device();
    // The runtime holds the buffers of the last kernel dispatched on a stream
    // until the next dispatch there: without an empty launch on each of the
    // context's compute streams, a freed 68.7 GB batch stayed allocated.
    for (hipStream_t s : {c->stream, c->sstream})
        if (s && launch_noop(s) != hipSuccess) (void)hipGetLastError();
    hipStreamSynchronize(c->stream);
    if (c->sstream) hipStreamSynchronize(c->sstream);
    hipFree(p);
}

void* hvws_host_alloc(hvws_ctx* c, uint64_t bytes) {
    if (check_ctx(c) != HVWS_OK) return nullptr;
    void* p = nullptr;
    hipError_t e = hipHostMalloc(&p, bytes ? bytes : 16, hipHostMallocDefault);
    if (e != hipSuccess) {
        set_err(HVWS_ENOMEM, "hipHostMalloc(%llu): %s", (unsigned long long)bytes, hipGetErrorString(e));
        return nullptr;
    }
    if (uint8_t* dev = host_mapped(p)) pin_add(p, bytes ? bytes : 16, dev, false);
    return p;
}

void hvws_host_free(hvws_ctx* c, void* p) {
    if (!c || !p) return;
    hipSetDevice(c->device);
    door_park_device();
    pin_remove(p);
    hipHostFree(p);
}

int hvws_host_register(hvws_ctx* c, void* p, uint64_t bytes) {
    int rc = check_ctx(c);
    if (rc) return rc;
    if (!p || !bytes) return set_err(HVWS_EINVAL, "empty range");
    HIP_OR(hipHostRegister(p, bytes, hipHostRegisterMapped), HVWS_EHIP);
    uint8_t* dev = host_mapped(p);
    if (!dev) {
        hipHostUnregister(p);
        return set_err(HVWS_EHIP, "registered range not device-mapped");
    }
    pin_add(p, bytes, dev, true);
    return HVWS_OK;
}

int hvws_host_unregister(hvws_ctx* c, void* p) {
    int rc = check_ctx(c);
    if (rc) return rc;
    const pinned_range r = pin_remove(p);
    if (!r.lo || !r.registered) return set_err(HVWS_EINVAL, "not a range from hvws_host_register");
    door_park_device();
    HIP_OR(hipHostUnregister(p), HVWS_EHIP);
    return HVWS_OK;
}

int hvws_rx_reads(hvws_ctx* c, char* const* reads, const uint64_t* lens, websocket_parser* carry, uint32_t n,
                  int unmask) {
    int rc = check_ctx(c);
    if (rc) return rc;
    if (n && (!reads || !lens)) return set_err(HVWS_EINVAL, "null read table");
    if (n == 0) return set_err(HVWS_EINVAL, "no reads");
    // In-place reads exist only on the small path: with it switched off
    // (hvws_set_small_batch_limit ~0) callers fall back to the general path.
    if (c->small_limit == ~0ull) return set_err(HVWS_EINVAL, "small-batch path disabled on this context");
    // device address of every read; the batch goes to k_small in address order
    std::vector<uint8_t*> dev(n);
    bool sorted = true;
    for (uint32_t i = 0; i < n; ++i) {
        if (lens[i] > kStageSegment)
            return set_err(HVWS_EINVAL, "read %u: %llu bytes (at most %llu)", i, (unsigned long long)lens[i],
                           (unsigned long long)kStageSegment);
        if (!(dev[i] = pinned_dev(reads[i], lens[i])))
            return set_err(HVWS_EINVAL, "read %u is not in registered pinned memory", i);
        if (i && dev[i] < dev[i - 1]) sorted = false;
    }
    std::vector<uint32_t> ord(n);
    for (uint32_t i = 0; i < n; ++i) ord[i] = i;
    if (!sorted) std::sort(ord.begin(), ord.end(), [&](uint32_t a, uint32_t b) { return dev[a] < dev[b]; });
    uint8_t* base = n ? (uint8_t*)((uintptr_t)dev[ord[0]] & ~(uintptr_t)15) : nullptr;
    std::vector<hvws_segment> segs(n);
    std::vector<websocket_parser> cin(carry ? n : 0);
    uint64_t span = 0, total = 0;
    for (uint32_t k = 0; k < n; ++k) {
        const uint32_t i = ord[k];
        segs[k].off = (uint64_t)(dev[i] - base);
        segs[k].len = lens[i];
        if (k && segs[k].off < segs[k - 1].off + segs[k - 1].len)
            return set_err(HVWS_EINVAL, "reads %u and %u overlap", ord[k - 1], i);
        span = segs[k].off + lens[i];
        total += lens[i];
        if (carry) copy_parser(cin[k], carry[i]);
    }
    const uint64_t limit = c->small_limit ? c->small_limit : kSmallBatch;
    if (total > limit) return set_err(HVWS_EINVAL, "%llu bytes of reads (at most %llu per call)",
                                      (unsigned long long)total, (unsigned long long)limit);
    if ((rc = rx_batch_small(c, nullptr, span, segs.data(), carry ? cin.data() : nullptr, n, unmask, base)) != HVWS_OK)
        return rc;
    // results back in caller order, offsets relative to each read; reads
    // already in address order (one arena filled in order) rebase in place
    if (sorted) {
        for (uint32_t i = 0; i < n; ++i) {
            const uint64_t rb = segs[i].off;
            hvws_frame* r = c->hcache.data() + c->hfirst[i];
            for (uint64_t j = 0; j < c->hcount[i]; ++j) {
                if (r[j].hdr_off >= 0) r[j].hdr_off -= (int64_t)rb;
                r[j].pay_off -= rb;
            }
            if (carry) {
                void* keep = carry[i].data;
                copy_parser(carry[i], cin[i]);
                carry[i].data = keep;
            }
        }
        return HVWS_OK;
    }
    std::vector<hvws_frame> recs(c->hcache.size());
    std::vector<uint64_t> first(n), count(n);
    std::vector<dcarry> hc(n);
    uint64_t at = 0;
    std::vector<uint32_t> pos(n);   // caller index -> address-order position
    for (uint32_t k = 0; k < n; ++k) pos[ord[k]] = k;
    for (uint32_t i = 0; i < n; ++i) {
        const uint32_t k = pos[i];
        const uint64_t cnt = c->hcount[k], rb = segs[k].off;
        first[i] = at;
        count[i] = cnt;
        hc[i] = c->hcarry[k];
        for (uint64_t j = 0; j < cnt; ++j) {
            hvws_frame r = c->hcache[c->hfirst[k] + j];
            if (r.hdr_off >= 0) r.hdr_off -= (int64_t)rb;
            r.pay_off -= rb;
            recs[at + j] = r;
        }
        at += cnt;
        if (carry) {
            void* keep = carry[i].data;
            copy_parser(carry[i], cin[k]);
            carry[i].data = keep;
        }
    }
    c->hcache.swap(recs);
    c->hfirst.swap(first);
    c->hcount.swap(count);
    c->hcarry.swap(hc);
    return HVWS_OK;
}

int hvws_h2d(hvws_ctx* c, void* dst, const void* src, uint64_t n) {
    int rc = check_ctx(c);
    if (rc) return rc;
    HIP_OR(hipMemcpyAsync(dst, src, n, hipMemcpyHostToDevice, c->stream), HVWS_EHIP);
    return HVWS_OK;
}

int hvws_d2h(hvws_ctx* c, void* dst, const void* src, uint64_t n) {
    int rc = check_ctx(c);
    if (rc) return rc;
    HIP_OR(hipMemcpyAsync(dst, src, n, hipMemcpyDeviceToHost, c->stream), HVWS_EHIP);
    return HVWS_OK;
}

int hvws_memset(hvws_ctx* c, void* dst, int v, uint64_t n) {
    int rc = check_ctx(c);
    if (rc) return rc;
    HIP_OR(hipMemsetAsync(dst, v, n, c->stream), HVWS_EHIP);
    return HVWS_OK;
}

int hvws_d2d(hvws_ctx* c, void* dst, const void* src, uint64_t n) {
    int rc = check_ctx(c);
    if (rc) return rc;
    HIP_OR(hipMemcpyAsync(dst, src, n, hipMemcpyDeviceToDevice, c->stream), HVWS_EHIP);
    return HVWS_OK;
}

int hvws_sync(hvws_ctx* c) {
    int rc = check_ctx(c);
    if (rc) return rc;
    HIP_OR(hipStreamSynchronize(c->stream), HVWS_EHIP);
    HIP_OR(hipStreamSynchronize(c->sstream), HVWS_EHIP);
    return HVWS_OK;
}

int hvws_debug_stall(hvws_ctx* c, uint32_t usec) {
    int rc = check_ctx(c);
    if (rc) return rc;
    HIP_OR(hipLaunchHostFunc(c->stream, stall_fn, (void*)(uintptr_t)usec), HVWS_EHIP);
    return HVWS_OK;
}

int hvws_scan(hvws_ctx* c, const uint8_t* d_rx, uint64_t rx_len, const hvws_segment* segs,
              const websocket_parser* carry_in, uint32_t nseg) {
    int rc = check_ctx(c);
    if (rc) return rc;
    if (!segs && nseg) return set_err(HVWS_EINVAL, "null segment table");
    if (((uintptr_t)d_rx & 15u) != 0) return set_err(HVWS_EINVAL, "rx buffer must be 16-byte aligned");
    if ((rc = upload_segments(c, segs, carry_in, nseg, rx_len)) != HVWS_OK) return rc;
    return scan_device_carry(c, d_rx, rx_len, nseg);
}

int hvws_unmask(hvws_ctx* c, uint8_t* d_rx, uint64_t rx_len) { return unmask_impl(c, d_rx, rx_len); }

int hvws_step_resident(hvws_ctx* c, uint8_t* d_rx, uint64_t rx_len, const hvws_segment* segs,
                       const websocket_parser* carry_in, uint32_t nseg) {
    int rc = check_ctx(c);
    if (rc) return rc;
    if (!segs && nseg) return set_err(HVWS_EINVAL, "null segment table");
    if (((uintptr_t)d_rx & 15u) != 0) return set_err(HVWS_EINVAL, "rx buffer must be 16-byte aligned");
    if (!c->piped) {
        // Entering pipelined mode: both table sets may still be read by work
        // queued on the context stream.
        for (tset& t : c->ts) {
            HIP_OR(hipEventRecord(t.free_ev, c->stream), HVWS_EHIP);
            t.free_wait = t.free_ev;
            t.free_pending = true;
        }
        c->piped = true;
    }
    if ((rc = upload_segments(c, segs, carry_in, nseg, rx_len)) != HVWS_OK) return rc;
    c->cs = c->sstream;
    bool unmasked = false;
    c->run_call = true;
    rc = scan_device_carry(c, d_rx, rx_len, nseg, d_rx, &unmasked);
    c->run_call = false;
    if (rc == HVWS_OK && !unmasked) rc = unmask_impl(c, d_rx, rx_len);
    c->cs = c->stream;
    return rc;
}

int hvws_step(hvws_ctx* c, uint8_t* d_rx, uint64_t rx_len, const hvws_segment* segs,
              const websocket_parser* carry_in, uint32_t nseg) {
    int rc = check_ctx(c);
    if (rc) return rc;
    if (!segs && nseg) return set_err(HVWS_EINVAL, "null segment table");
    if (((uintptr_t)d_rx & 15u) != 0) return set_err(HVWS_EINVAL, "rx buffer must be 16-byte aligned");
    if ((rc = upload_segments(c, segs, carry_in, nseg, rx_len)) != HVWS_OK) return rc;
    bool unmasked = false;
    c->run_call = true;
    rc = scan_device_carry(c, d_rx, rx_len, nseg, d_rx, &unmasked);
    c->run_call = false;
    if (rc != HVWS_OK) return rc;
    return unmasked ? HVWS_OK : unmask_impl(c, d_rx, rx_len);
}

int64_t hvws_frame_count(hvws_ctx* c) {
    if (!c || !c->have_scan) return -1;
    if (check_ctx(c) != HVWS_OK || ensure_count(c) != HVWS_OK) return -1;
    return (int64_t)c->nfr;
}

int hvws_get_frames(hvws_ctx* c, hvws_frame* out, uint64_t first, uint64_t n) {
    int rc = check_ctx(c);
    if (rc) return rc;
    if (!c->have_scan) return set_err(HVWS_EINVAL, "no scan");
    if ((rc = ensure_count(c)) != HVWS_OK) return rc;
    if (first > c->nfr || n > c->nfr - first) return set_err(HVWS_EINVAL, "frame range out of bounds");
    if (n == 0) return HVWS_OK;
    if (c->hcache_valid) {
        memcpy(out, c->hcache.data() + first, n * sizeof(hvws_frame));
        return HVWS_OK;
    }
    std::vector<int64_t> hdr(n);
    std::vector<uint64_t> off(n), len(n), length(n);
    std::vector<uint32_t> key(n), info(n);
    HIP_OR(hipMemcpyAsync(hdr.data(), c->T().f_hdr.as<int64_t>() + first, n * 8, hipMemcpyDeviceToHost, c->stream),
           HVWS_EHIP);
    HIP_OR(hipMemcpyAsync(off.data(), c->T().f_off.as<uint64_t>() + first, n * 8, hipMemcpyDeviceToHost, c->stream),
           HVWS_EHIP);
    HIP_OR(hipMemcpyAsync(len.data(), c->T().f_len.as<uint64_t>() + first, n * 8, hipMemcpyDeviceToHost, c->stream),
           HVWS_EHIP);
    HIP_OR(hipMemcpyAsync(length.data(), c->T().f_length.as<uint64_t>() + first, n * 8, hipMemcpyDeviceToHost,
                          c->stream),
           HVWS_EHIP);
    HIP_OR(hipMemcpyAsync(key.data(), c->T().f_key.as<uint32_t>() + first, n * 4, hipMemcpyDeviceToHost, c->stream),
           HVWS_EHIP);
    HIP_OR(hipMemcpyAsync(info.data(), c->T().f_info.as<uint32_t>() + first, n * 4, hipMemcpyDeviceToHost, c->stream),
           HVWS_EHIP);
    HIP_OR(hipStreamSynchronize(c->stream), HVWS_EHIP);
    for (uint64_t i = 0; i < n; ++i) {
        out[i].hdr_off = hdr[i];
        out[i].pay_off = off[i];
        out[i].pay_len = len[i];
        out[i].length = length[i];
        out[i].key = key[i];
        out[i].info = info[i];
    }
    return HVWS_OK;
}

int hvws_get_segment_frames(hvws_ctx* c, uint64_t* first, uint64_t* count) {
    int rc = check_ctx(c);
    if (rc) return rc;
    if (!c->have_scan) return set_err(HVWS_EINVAL, "no scan");
    if ((rc = run_materialize(c)) != HVWS_OK) return rc;
    if (c->hcache_valid) {
        if (first) memcpy(first, c->hfirst.data(), (uint64_t)c->nseg * 8);
        if (count) memcpy(count, c->hcount.data(), (uint64_t)c->nseg * 8);
        return HVWS_OK;
    }
    if (first)
        HIP_OR(hipMemcpyAsync(first, c->T().bases.p, (uint64_t)c->nseg * 8, hipMemcpyDeviceToHost, c->stream),
               HVWS_EHIP);
    if (count)
        HIP_OR(hipMemcpyAsync(count, c->T().counts.p, (uint64_t)c->nseg * 8, hipMemcpyDeviceToHost, c->stream),
               HVWS_EHIP);
    HIP_OR(hipStreamSynchronize(c->stream), HVWS_EHIP);
    return HVWS_OK;
}

int hvws_get_carry(hvws_ctx* c, websocket_parser* out, int* started) {
    int rc = check_ctx(c);
    if (rc) return rc;
    if (!c->have_scan) return set_err(HVWS_EINVAL, "no scan");
    if ((rc = run_materialize(c)) != HVWS_OK) return rc;
    std::vector<dcarry> h;
    const dcarry* src;
    if (c->hcache_valid) {
        src = c->hcarry.data();
    } else {
        h.resize(c->nseg);
        if (c->nseg)
            HIP_OR(hipMemcpyAsync(h.data(), c->T().carry_out.p, (uint64_t)c->nseg * sizeof(dcarry),
                                  hipMemcpyDeviceToHost, c->stream),
                   HVWS_EHIP);
        HIP_OR(hipStreamSynchronize(c->stream), HVWS_EHIP);
        src = h.data();
    }
    for (uint32_t s = 0; s < c->nseg; ++s) {
        if (out) from_dcarry(src[s], out[s]);
        if (started) started[s] = (int)src[s].started;
    }
    return HVWS_OK;
}

int hvws_last_times(hvws_ctx* c, float out[2]) {
    int rc = check_ctx(c);
    if (rc) return rc;
    out[0] = out[1] = -1.0f;
    if (!c->have_scan || c->t_seq == 0) return set_err(HVWS_EINVAL, "no scan");
    return step_times_at(c, c->t_cur, out);
}

// Timed region on the device: markers on both compute streams (the scan
// stream and the unmask stream of pipelined steps), so the span runs from
// whichever stream starts first to whichever ends last.
int hvws_span_begin(hvws_ctx* c) {
    int rc = check_ctx(c);
    if (rc) return rc;
    for (auto& ev : c->span_ev)
        if (!ev) HIP_OR(hipEventCreate(&ev), HVWS_EHIP);
    HIP_OR(hipEventRecord(c->span_ev[0], c->stream), HVWS_EHIP);
    HIP_OR(hipEventRecord(c->span_ev[1], c->sstream ? c->sstream : c->stream), HVWS_EHIP);
    return HVWS_OK;
}

int hvws_span_end(hvws_ctx* c, float* ms) {
    int rc = check_ctx(c);
    if (rc) return rc;
    if (!ms || !c->span_ev[0]) return set_err(HVWS_EINVAL, "no hvws_span_begin");
    HIP_OR(hipEventRecord(c->span_ev[2], c->stream), HVWS_EHIP);
    HIP_OR(hipEventRecord(c->span_ev[3], c->sstream ? c->sstream : c->stream), HVWS_EHIP);
    HIP_OR(hipEventSynchronize(c->span_ev[2]), HVWS_EHIP);
    HIP_OR(hipEventSynchronize(c->span_ev[3]), HVWS_EHIP);
    // max over (begin, end) pairs = latest end - earliest begin
    float best = 0.0f;
    for (int b = 0; b < 2; ++b)
        for (int e = 2; e < 4; ++e) {
            float t = 0.0f;
            HIP_OR(hipEventElapsedTime(&t, c->span_ev[b], c->span_ev[e]), HVWS_EHIP);
            best = std::max(best, t);
        }
    *ms = best;
    return HVWS_OK;
}

int hvws_set_step_event_interval(hvws_ctx* c, uint32_t every) {
    int rc = check_ctx(c);
    if (rc) return rc;
    const int old = (int)c->t_every;
    c->t_every = every;
    return old;
}

int hvws_step_times(hvws_ctx* c, float* out, int max_steps) {
    int rc = check_ctx(c);
    if (rc) return rc;
    if (!out || max_steps < 0) return set_err(HVWS_EINVAL, "bad output");
    uint64_t n = std::min<uint64_t>(c->t_seq, hvws_ctx::kTimeRing);
    n = std::min<uint64_t>(n, (uint64_t)max_steps);
    for (uint64_t i = 0; i < n; ++i) {
        const int slot = (int)((c->t_seq - n + i) % hvws_ctx::kTimeRing);
        if ((rc = step_times_at(c, slot, out + 2 * i)) != HVWS_OK) return rc;
    }
    return (int)n;
}

int hvws_stream_xor(hvws_ctx* c, uint8_t* d, uint64_t n, uint32_t pattern) {
    int rc = check_ctx(c);
    if (rc) return rc;
    if (((uintptr_t)d & 15u) != 0) return set_err(HVWS_EINVAL, "buffer must be 16-byte aligned");
    HIP_OR(launch_stream_xor(unmask_variant_for(n), d, n, pattern, c->stream), HVWS_EHIP);
    return HVWS_OK;
}

int hvws_rx_batch(hvws_ctx* c, uint8_t* h_rx, uint64_t len, const hvws_segment* segs, websocket_parser* carry,
                  uint32_t nseg, int unmask) {
    int rc = check_ctx(c);
    if (rc) return rc;
    if (!segs && nseg) return set_err(HVWS_EINVAL, "null segment table");
    if (small_eligible(c, len, segs, nseg)) return rx_batch_small(c, h_rx, len, segs, carry, nseg, unmask);
    HIP_OR(c->stage.ensure(len + 64), HVWS_ENOMEM);
    uint8_t* d = c->stage.as<uint8_t>();
    if ((rc = upload_segments(c, segs, carry, nseg, len)) != HVWS_OK) return rc;
    if (len) HIP_OR(hipMemcpyAsync(d, h_rx, len, hipMemcpyHostToDevice, c->stream), HVWS_EHIP);
    bool unmasked = false;
    if ((rc = scan_device_carry(c, d, len, nseg, unmask ? d : nullptr, &unmasked)) != HVWS_OK) return rc;
    if (unmask) {
        if (!unmasked && (rc = unmask_impl(c, d, len)) != HVWS_OK) return rc;
        if (len) HIP_OR(hipMemcpyAsync(h_rx, d, len, hipMemcpyDeviceToHost, c->stream), HVWS_EHIP);
    }
    // one round trip for the results (the D2H of the bytes above is ordered before it)
    if ((rc = readback_all(c)) != HVWS_OK) return rc;
    if (carry) {
        for (uint32_t s = 0; s < nseg; ++s) {
            void* keep = carry[s].data;
            from_dcarry(c->hcarry[s], carry[s]);
            carry[s].data = keep;
        }
    }
    return HVWS_OK;
}

int hvws_pipeline(hvws_ctx* c, uint8_t* h_rx, uint64_t len, uint64_t chunk, websocket_parser* carry) {
    int rc = check_ctx(c);
    if (rc) return rc;
    if (!carry) return set_err(HVWS_EINVAL, "carry required");
    if (chunk < 4096) chunk = 4096;
    chunk = (chunk + 15) & ~15ull;
    const uint64_t nchunks = (len + chunk - 1) / chunk;
    if (nchunks == 0) return HVWS_OK;
    // Three device slots: H2D(k+1) and D2H(k-1) overlap compute(k).  Slots
    // and events live in the context (grow-only), so repeated calls pay no
    // allocation; earlier work on the context's streams is finished first
    // (an earlier call's copies may still use the slots).
    HIP_OR(hipStreamSynchronize(c->stream), HVWS_EHIP);   // h_segs may still feed an earlier copy
    HIP_OR(hipStreamSynchronize(c->copy_in), HVWS_EHIP);
    HIP_OR(hipStreamSynchronize(c->copy_out), HVWS_EHIP);
    dbuf* slot = c->pipe_slot;
    for (int i = 0; i < 3; ++i) HIP_OR(slot[i].ensure(chunk + 64), HVWS_ENOMEM);
    for (hipEvent_t& ev : c->pipe_ev)
        if (!ev) HIP_OR(hipEventCreateWithFlags(&ev, hipEventDisableTiming), HVWS_EHIP);
    hipEvent_t* in_done = c->pipe_ev;
    hipEvent_t* comp_done = c->pipe_ev + 3;
    hipEvent_t* out_done = c->pipe_ev + 6;
    // every chunk's segment {0, n}, resident before the loop
    dbuf& pipe_segs = c->pipe_segs;
    HIP_OR(pipe_segs.ensure(nchunks * sizeof(dseg)), HVWS_ENOMEM);
    HIP_OR(c->h_segs.ensure(nchunks * sizeof(dseg)), HVWS_ENOMEM);
    for (uint64_t k = 0; k < nchunks; ++k) c->h_segs.as<dseg>()[k] = dseg{0, std::min(chunk, len - k * chunk)};
    HIP_OR(hipMemcpyAsync(pipe_segs.p, c->h_segs.p, nchunks * sizeof(dseg), hipMemcpyHostToDevice, c->stream),
           HVWS_EHIP);
    hvws_segment seg0 = {0, 0};
    void* keep = carry->data;
    int out_rc = HVWS_OK;
    auto issue_in = [&](uint64_t k) -> hipError_t {
        const int s = (int)(k % 3);
        const uint64_t off = k * chunk;
        const uint64_t n = std::min(chunk, len - off);
        hipError_t e = hipStreamWaitEvent(c->copy_in, out_done[s], 0);
        if (e == hipSuccess) e = hipMemcpyAsync(slot[s].p, h_rx + off, n, hipMemcpyHostToDevice, c->copy_in);
        if (e == hipSuccess) e = hipEventRecord(in_done[s], c->copy_in);
        return e;
    };
    // out_done events start "complete"
    for (int i = 0; i < 3; ++i) hipEventRecord(out_done[i], c->copy_out);
    hipError_t e = issue_in(0);
    for (uint64_t k = 0; k < nchunks && e == hipSuccess && out_rc == HVWS_OK; ++k) {
        const int s = (int)(k % 3);
        const uint64_t off = k * chunk;
        const uint64_t n = std::min(chunk, len - off);
        if (k + 1 < nchunks) e = issue_in(k + 1);
        if (e != hipSuccess) break;
        e = hipStreamWaitEvent(c->stream, in_done[s], 0);
        if (e != hipSuccess) break;
        seg0.len = n;
        if (k == 0) {
            out_rc = upload_segments(c, &seg0, carry, 1, n);
        } else {
            // The carry chains on the device: chunk k-1's carry-out is chunk
            // k's carry-in (a frame may straddle the chunk boundary).
            // Both tables are copied device to device, so the host never
            // waits inside the loop (each chunk's segment is preloaded).
            e = hipMemcpyAsync(c->segs.p, pipe_segs.as<dseg>() + k, sizeof(dseg), hipMemcpyDeviceToDevice, c->stream);
            if (e == hipSuccess)
                e = hipMemcpyAsync(c->carry_in.p, c->T().carry_out.p, sizeof(dcarry), hipMemcpyDeviceToDevice,
                                   c->stream);
            if (e != hipSuccess) break;
        }
        if (out_rc != HVWS_OK) break;
        out_rc = scan_device_carry(c, slot[s].as<uint8_t>(), n, 1);
        if (out_rc != HVWS_OK) break;
        out_rc = hvws_unmask(c, slot[s].as<uint8_t>(), n);
        if (out_rc != HVWS_OK) break;
        e = hipEventRecord(comp_done[s], c->stream);
        if (e == hipSuccess) e = hipStreamWaitEvent(c->copy_out, comp_done[s], 0);
        if (e == hipSuccess) e = hipMemcpyAsync(h_rx + off, slot[s].p, n, hipMemcpyDeviceToHost, c->copy_out);
        if (e == hipSuccess) e = hipEventRecord(out_done[s], c->copy_out);
    }
    if (e == hipSuccess && out_rc == HVWS_OK) {
        e = hipStreamSynchronize(c->copy_out);
        if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
        if (e == hipSuccess) out_rc = hvws_get_carry(c, carry, nullptr);
    }
    hipStreamSynchronize(c->copy_in);
    hipStreamSynchronize(c->copy_out);
    hipStreamSynchronize(c->stream);
    carry->data = keep;
    // The last scan referenced a slot, which the next call overwrites:
    // forget it (hvws_unmask would refuse it anyway).
    c->have_scan = false;
    if (e != hipSuccess) return set_err(HVWS_EHIP, "pipeline: %s", hipGetErrorString(e));
    return out_rc;
}

// ------------------------------------------------------------------ synth
int hvws_synth(hvws_ctx* c, uint8_t* d_buf, uint64_t buf_len, uint64_t seed, uint64_t nframes,
               const uint64_t* d_frame_off, const uint8_t* d_flags, const uint32_t* d_mask,
               const uint64_t* d_length, const uint8_t* d_text, int mode, uint64_t* mismatches) {
    int rc = check_ctx(c);
    if (rc) return rc;
    if (mode < 0 || mode > 2) return set_err(HVWS_EINVAL, "bad synth mode %d", mode);
    const uint64_t tile = synth_tile();
    const uint64_t ntiles = (buf_len + tile - 1) / tile;
    HIP_OR(c->synth_sizes.ensure(nframes * 8 + 8), HVWS_ENOMEM);
    HIP_OR(c->synth_tiles.ensure((ntiles + 2) * 4), HVWS_ENOMEM);
    HIP_OR(c->synth_bad.ensure(8), HVWS_ENOMEM);
    HIP_OR(launch_frame_sizes(d_flags, d_length, nframes, c->synth_sizes.as<uint64_t>(), c->stream), HVWS_EHIP);
    HIP_OR(launch_tile_index(d_frame_off, c->synth_sizes.as<uint64_t>(), nframes, nullptr, c->synth_tiles.as<uint32_t>(),
                             ntiles, tile, c->stream),
           HVWS_EHIP);
    HIP_OR(hipMemsetAsync(c->synth_bad.p, 0, 8, c->stream), HVWS_EHIP);
    HIP_OR(launch_synth(d_buf, buf_len, seed, nframes, d_frame_off, d_flags, d_mask, d_length, d_text,
                        c->synth_sizes.as<uint64_t>(), c->synth_tiles.as<uint32_t>(), mode,
                        c->synth_bad.as<unsigned long long>(), c->stream),
           HVWS_EHIP);
    if (mode != HVWS_SYNTH_WRITE) {
        uint64_t bad = 0;
        HIP_OR(hipMemcpyAsync(&bad, c->synth_bad.p, 8, hipMemcpyDeviceToHost, c->stream), HVWS_EHIP);
        HIP_OR(hipStreamSynchronize(c->stream), HVWS_EHIP);
        if (mismatches) *mismatches = bad;
    }
    return HVWS_OK;
}

int hvws_digest(hvws_ctx* c, const uint8_t* d_buf, uint64_t len, uint64_t* out) {
    int rc = check_ctx(c);
    if (rc) return rc;
    HIP_OR(c->synth_bad.ensure(8), HVWS_ENOMEM);
    HIP_OR(hipMemsetAsync(c->synth_bad.p, 0, 8, c->stream), HVWS_EHIP);
    HIP_OR(launch_digest(d_buf, len, c->synth_bad.as<unsigned long long>(), c->stream), HVWS_EHIP);
    uint64_t v = 0;
    HIP_OR(hipMemcpyAsync(&v, c->synth_bad.p, 8, hipMemcpyDeviceToHost, c->stream), HVWS_EHIP);
    HIP_OR(hipStreamSynchronize(c->stream), HVWS_EHIP);
    if (out) *out = v;
    return HVWS_OK;
}

// --------------------------------------------------------------- transmit
int hvws_build_frames(hvws_ctx* c, uint8_t* d_out, uint64_t out_cap, const uint8_t* d_payload, uint64_t payload_len,
                      const uint64_t* d_pay_off, const uint64_t* d_len, const uint8_t* d_flags, const uint32_t* d_mask,
                      uint64_t n, uint64_t* d_out_off, uint64_t* out_len) {
    int rc = check_ctx(c);
    if (rc) return rc;
    if (out_len) *out_len = 0;
    if (n == 0) return HVWS_OK;
    if (!d_out || !d_pay_off || !d_len || !d_flags) return set_err(HVWS_EINVAL, "build_frames: null table");
    if (n >= 0xFFFFFFFFull) return set_err(HVWS_EINVAL, "build_frames: %llu frames (max 2^32-2)", (unsigned long long)n);
    const uint64_t nb = (n + 1023) / 1024;
    HIP_OR(c->tx_size.ensure(n * 8 + 8), HVWS_ENOMEM);
    HIP_OR(c->tx_scan.ensure((4 * nb + 64) * 8), HVWS_ENOMEM);
    HIP_OR(c->tx_stat.ensure(64), HVWS_ENOMEM);
    HIP_OR(c->h_tx.ensure(64), HVWS_ENOMEM);
    uint64_t* off = d_out_off;
    if (!off) {
        HIP_OR(c->tx_off.ensure(n * 8 + 8), HVWS_ENOMEM);
        off = c->tx_off.as<uint64_t>();
    }
    // [0] total bytes, [1] payload ranges out of bounds, [2] frames breaking
    // the uniform layout, [3..5] pay_off[0], its step, len[0] (k_tx_check)
    uint64_t* stat = c->tx_stat.as<uint64_t>();
    HIP_OR(hipMemsetAsync(stat, 0, 64, c->stream), HVWS_EHIP);
    HIP_OR(launch_frame_sizes(d_flags, d_len, n, c->tx_size.as<uint64_t>(), c->stream), HVWS_EHIP);
    HIP_OR(launch_exclusive_scan(c->tx_size.as<uint64_t>(), off, n, c->tx_scan.as<uint64_t>(), stat, c->stream),
           HVWS_EHIP);
    HIP_OR(launch_tx_check(d_pay_off, d_len, d_flags, d_mask, c->tx_size.as<uint64_t>(), n, payload_len, stat,
                           c->stream),
           HVWS_EHIP);
    uint64_t* h = c->h_tx.as<uint64_t>();
    HIP_OR(hipMemcpyAsync(h, stat, 48, hipMemcpyDeviceToHost, c->stream), HVWS_EHIP);
    HIP_OR(hipStreamSynchronize(c->stream), HVWS_EHIP);
    if (h[1]) return set_err(HVWS_EINVAL, "build_frames: %llu frames read outside the payload buffer or lack a mask",
                             (unsigned long long)h[1]);
    const uint64_t total = h[0];
    if (out_len) *out_len = total;
    if (total > out_cap)
        return set_err(HVWS_EINVAL, "build_frames: output needs %llu bytes, capacity %llu", (unsigned long long)total,
                       (unsigned long long)out_cap);
    // the geometry by the batch's mean frame size (tx_variant); every layout
    // takes k_build (round 4: it reached or beat the same-offset kernel
    // k_build_id, which is gone, profiles/r4v_raw)
    const int v = tx_variant(total, n);
    c->tx_variant = v;
    // each tile's source span first (round 4: records-first tiles lost, and
    // their switch went in round 6)
    const bool spans_ok = true;
    const uint64_t tile = tx_tile(v);
    const uint64_t ntiles = (total + tile - 1) / tile;
    // A uniform layout (every frame the same size and length, payload offsets
    // a + k * b, b >= 0) needs no tile index: each tile finds its frames and
    // source span from its position.
    constexpr bool uni_ok = true;
    // (payload steps shorter than a payload would make a tile's pieces
    // overlap out of order: the index handles those)
    // (small frames only, the lean form: at 64 KiB frames the index is ~0.1 %
    // of the call and the position-derived form measured slower at the rx
    // layout, 21.3 against 20.2 ms at c3, profiles/r5b_raw)
    const bool uniform = uni_ok && v == 5 && h[2] == 0 && total % n == 0 && (n == 1 || h[4] >= h[5]);
    const uint64_t uni[4] = {uniform ? total / n : 0, uniform ? total / n - h[5] : 0, h[3], h[4]};
    c->tx_uniform = uniform;
    if (!uniform) {
        HIP_OR(c->tx_tiles.ensure((ntiles + 2) * 4), HVWS_ENOMEM);
        if (spans_ok) HIP_OR(c->tx_span.ensure(ntiles * 16 + 16), HVWS_ENOMEM);
    }
    // the timed device work (hvws_last_kernel_ms): tile index, spans, build
    HIP_OR(hipEventRecord(c->ev[4], c->stream), HVWS_EHIP);
    uint64_t* span = spans_ok && !uniform ? c->tx_span.as<uint64_t>() : nullptr;
    if (!uniform)
        HIP_OR(launch_tx_index(off, c->tx_size.as<uint64_t>(), d_pay_off, d_len, d_flags, n, ntiles, tile,
                               c->tx_tiles.as<uint32_t>(), span, c->stream),
               HVWS_EHIP);
    HIP_OR(launch_build(d_out, total, d_payload, payload_len, d_pay_off, d_len, d_flags, d_mask, off,
                        c->tx_size.as<uint64_t>(), c->tx_tiles.as<uint32_t>(), span, n, v, c->stream, uni),
           HVWS_EHIP);
    HIP_OR(hipEventRecord(c->ev[5], c->stream), HVWS_EHIP);
    c->ev_build = true;
    return HVWS_OK;
}

int hvws_encode_keys(hvws_ctx* c, const char* d_keys, const uint64_t* d_key_off, const uint32_t* d_key_len,
                     uint64_t n, char* d_accept) {
    int rc = check_ctx(c);
    if (rc) return rc;
    if (n == 0) return HVWS_OK;
    if (!d_keys || !d_key_off || !d_key_len || !d_accept) return set_err(HVWS_EINVAL, "encode_keys: null table");
    if (((uintptr_t)d_accept & 15u) != 0) return set_err(HVWS_EINVAL, "encode_keys: accept buffer must be 16-byte aligned");
    HIP_OR(hipEventRecord(c->ev[4], c->stream), HVWS_EHIP);
    HIP_OR(launch_encode_keys((const uint8_t*)d_keys, d_key_off, d_key_len, n, (uint8_t*)d_accept, c->stream),
           HVWS_EHIP);
    HIP_OR(hipEventRecord(c->ev[5], c->stream), HVWS_EHIP);
    c->ev_build = true;
    return HVWS_OK;
}

int hvws_last_kernel_ms(hvws_ctx* c, float* ms) {
    int rc = check_ctx(c);
    if (rc) return rc;
    if (!c->ev_build) return set_err(HVWS_EINVAL, "no build_frames / encode_keys call yet");
    HIP_OR(hipEventSynchronize(c->ev[5]), HVWS_EHIP);
    HIP_OR(hipEventElapsedTime(ms, c->ev[4], c->ev[5]), HVWS_EHIP);
    return HVWS_OK;
}

const char* hvws_build_kernel_name(void) { return build_kernel_name(tx_variant(0, 0)); }

const char* hvws_last_build_kernel(hvws_ctx* c) {
    if (!c) return "";
    return build_kernel_name(c->tx_variant);
}

int hvws_last_build_uniform(hvws_ctx* c) { return c && c->tx_uniform ? 1 : 0; }

uint32_t hvws_set_validation(hvws_ctx* c, uint32_t classes) {
    if (!c) c = hvws::thread_ctx();
    const uint32_t old = c->vmask;
    c->vmask = classes & V_ALL;
    return old;
}

int hvws_set_door(hvws_ctx* c, int on) {
    if (!c) c = hvws::thread_ctx();
    std::lock_guard<std::mutex> cl(c->door_m);
    const int old = door_on(c) ? 1 : 0;
    c->door_mode = on < 0 ? -1 : (on ? 1 : 0);
    if (!door_on(c) && c->door_live) {   // off (explicitly, or -1 resolving to off): park now
        int dev = -1;
        (void)hipGetDevice(&dev);
        hipSetDevice(c->device);
        door_park(c);
        if (dev >= 0) hipSetDevice(dev);
    }
    return old;
}

int hvws_door_info(hvws_ctx* c, uint64_t out[2]) {
    if (!c) c = hvws::thread_ctx();
    if (!out) return set_err(HVWS_EINVAL, "null output");
    out[0] = c->d_door_req ? 1 : 0;
    out[1] = c->door_q ? 1 : 0;
    return HVWS_OK;
}

int hvws_door_stamps(hvws_ctx* c, uint64_t out[12]) {
    if (!c) c = hvws::thread_ctx();
    if (!out) return set_err(HVWS_EINVAL, "null output");
    memset(out, 0, 12 * sizeof(uint64_t));
    if (c->h_door.p) memcpy(out, c->h_door.as<ddoor>()->stamp, 12 * sizeof(uint64_t));
    return HVWS_OK;
}

uint64_t hvws_set_door_idle_us(uint64_t us) {
    const uint64_t old = door_idle_us();
    g_door_idle_us.store(us ? us : 5000, std::memory_order_relaxed);
    return old;
}

int hvws_door_health(uint64_t out[2]) {
    if (!out) return set_err(HVWS_EINVAL, "null output");
    out[0] = g_door_wedged.load();
    out[1] = g_door_failed.load();
    return HVWS_OK;
}

int hvws_door_stats(hvws_ctx* c, uint64_t out[4]) {
    if (!c) c = hvws::thread_ctx();
    if (!out) return set_err(HVWS_EINVAL, "null output");
    out[0] = c->door_launches;
    out[1] = c->door_calls;
    out[2] = c->h_door.p ? __atomic_load_n(&c->h_door.as<ddoor>()->served, __ATOMIC_ACQUIRE) : 0;
    out[3] = c->door_live ? 1 : 0;
    return HVWS_OK;
}

uint64_t hvws_set_small_batch_limit(hvws_ctx* c, uint64_t bytes) {
    if (!c) c = hvws::thread_ctx();   // the calling thread's reference-API context
    const uint64_t old = c->small_limit ? c->small_limit : kSmallBatch;
    c->small_limit = bytes;
    return old;
}

int hvws_set_small_zero_copy(hvws_ctx* c, int on) {
    if (!c) c = hvws::thread_ctx();
    const int old = c->small_zc;
    c->small_zc = on ? 1 : 0;
    return old;
}

const char* hvws_unmask_kernel_name(void) { return unmask_name(unmask_variant()); }

const char* hvws_unmask_kernel_name_for(uint64_t rx_len) { return unmask_name(unmask_variant_for(rx_len)); }

const char* hvws_run_kernel_name(void) { return run_kernel_name(); }

uint64_t hvws_set_spec_min(uint64_t frames) { return set_spec_min(frames); }

uint64_t hvws_set_sieve_min(uint64_t bytes) { return set_sieve_min(bytes); }

int hvws_set_table_checks(int on) {
    const int prev = table_checks() ? 1 : 0;
    __atomic_store_n(&g_table_checks, on ? 1 : 0, __ATOMIC_RELAXED);
    return prev;
}

int hvws_last_sieve(hvws_ctx* c, uint64_t out[4]) {
    if (!c) c = thread_ctx();
    if (!c || !out) return set_err(HVWS_EINVAL, "hvws_last_sieve: NULL argument");
    out[0] = out[1] = out[2] = out[3] = 0;
    if (!c->sv_ran) return HVWS_OK;
    HIP_OR(hipSetDevice(c->device), HVWS_EHIP);
    HIP_OR(hipStreamSynchronize(c->cs), HVWS_EHIP);
    const dsieve* d = c->h_sv.as<dsieve>();
    const uint64_t* n = reinterpret_cast<const uint64_t*>(c->h_sv.as<uint8_t>() + sizeof(dsieve));
    out[0] = d->active ? (n[3] <= c->sv_cap && n[0] <= c->sv_capc ? 1 : 2) : 0;
    out[1] = d->active ? n[0] : 0;
    out[2] = d->use ? d->npath : 0;
    out[3] = d->use ? d->pend : 0;
    return HVWS_OK;
}

void hvws_set_sieve_windows(uint64_t hops, uint64_t window_bytes, uint64_t prev[2]) {
    set_sieve_windows(hops, window_bytes, prev);
}

int hvws_last_sieve_windows(hvws_ctx* c, uint64_t out[2]) {
    if (!c) c = thread_ctx();
    if (!c || !out) return set_err(HVWS_EINVAL, "hvws_last_sieve_windows: NULL argument");
    out[0] = c->sv_ran ? c->sv_rt : 0;
    out[1] = c->sv_ran ? c->sv_wt : 0;
    return HVWS_OK;
}

int hvws_last_scan_path(hvws_ctx* c) { return c ? c->scan_path : -1; }

uint64_t hvws_set_fast_bound(hvws_ctx* c, uint64_t records) {
    if (!c) return 0;
    const uint64_t old = c->fast_bound ? c->fast_bound : kFastFrameBound;
    c->fast_bound = records;
    return old;
}

int hvws_set_walk_verify(hvws_ctx* c, int mode) {
    if (!c) c = thread_ctx();
    if (!c) return HVWS_ENODEV;
    const int old = c->verify_mode;
    c->verify_mode = mode < 0 ? -1 : (mode ? 1 : 0);
    return old;
}

int64_t hvws_last_run_repairs(hvws_ctx* c) {
    if (check_ctx(c) != HVWS_OK || c->scan_path != HVWS_PATH_RUN) return -1;
    if (hipStreamSynchronize(c->stream) != hipSuccess) return -1;
    const dspec_status* st = c->h_status.as<dspec_status>();
    return __atomic_load_n(&st->pad3[0], __ATOMIC_ACQUIRE) == c->run_seq ? (int64_t)st->pad3[1] : -1;
}

int hvws_set_run(hvws_ctx* c, int mode) {
    if (!c) c = thread_ctx();
    if (!c) return HVWS_ENODEV;
    const int old = c->run_mode;
    c->run_mode = mode < 0 ? -1 : (mode ? 1 : 0);
    return old;
}

int hvws_set_speculation(hvws_ctx* c, int mode) {
    if (!c) c = thread_ctx();
    if (!c) return HVWS_ENODEV;
    const int old = c->spec_mode;
    c->spec_mode = mode < 0 ? -1 : (mode > 2 ? 2 : mode);
    return old;
}

int hvws_set_unmask_variant(int v) {
    if (set_unmask_variant(v) < -1) return set_err(HVWS_EINVAL, "unmask variant %d out of range [-1,%d)", v,
                                                   unmask_variant_count());
    return HVWS_OK;
}

void hvws_thread_release(void) {
    if (t_ctx) hvws_ctx_destroy(t_ctx);
    t_ctx = nullptr;
}

int hvws_set_thread_device(int device) {
    if (t_ctx && t_ctx->device != device) {
        hvws_ctx_destroy(t_ctx);
        t_ctx = nullptr;
    }
    t_device = device;
    return HVWS_OK;
}

}  // extern "C"

// ----------------------------------------------- internal helpers for the drop-in
namespace hvws {

[[noreturn]] void fatal(const char* what) {
    fprintf(stderr, "libhvws: %s: %s -- the MI355X WebSocket path has no CPU fallback\n", what, g_err);
    fflush(stderr);
    abort();
}

// Parks the thread context's resident worker when the thread exits (the
// context itself lives on until hvws_thread_release, as before).
// The main thread's guard runs inside exit(): it only asks the worker to
// exit through the mailbox (no HIP call, like door_atexit).
struct thread_door_guard {
    ~thread_door_guard() {
        if (!t_ctx || !t_ctx->door_live) return;
        std::lock_guard<std::mutex> cl(t_ctx->door_m);
        if ((pid_t)syscall(SYS_gettid) == getpid()) {
            door_quit_nohip(t_ctx);
        } else {
            hipSetDevice(t_ctx->device);
            door_park(t_ctx);
        }
    }
};
thread_local thread_door_guard t_door_guard;

hvws_ctx* thread_ctx() {
    if (t_ctx) return t_ctx;
    (void)&t_door_guard;
    int dev = t_device;
    if (dev < 0) {
        const char* e = getenv("HVWS_DEVICE");
        dev = e ? atoi(e) : 0;
    }
    t_ctx = hvws_ctx_create(dev);
    if (!t_ctx) fatal("cannot open a HIP device context");
    return t_ctx;
}

// A feeder's worker context takes the per-context knobs of the thread that
// made the feeder (small-batch path, zero-copy, validation classes).
void ctx_copy_settings(hvws_ctx* dst, const hvws_ctx* src) {
    dst->small_limit = src->small_limit;
    dst->small_zc = src->small_zc;
    dst->zc_batch = src->zc_batch;
    dst->vmask = src->vmask;
}

// The host record cache of the last small-path call, moved out (no copy) with
// its per-segment first/count; the context then holds no scan (the batched
// drop-in is the only reader of its thread context's records).
bool take_frames(hvws_ctx* c, std::vector<hvws_frame>& frames, std::vector<uint64_t>& first,
                 std::vector<uint64_t>& count) {
    if (!c->have_scan || !c->hcache_valid || c->rx) return false;
    frames.swap(c->hcache);
    first.swap(c->hfirst);
    count.swap(c->hcount);
    c->hcache.clear();
    c->hcache_valid = false;
    c->have_scan = false;
    return true;
}

// True when [p, p+len) lies in registered pinned memory (hvws_rx_reads can take it).
bool is_pinned(const void* p, uint64_t len) { return pinned_dev(p, len) != nullptr; }

// Per-thread pinned staging for batched host entry points.
char* pinned_stage(uint64_t bytes) {
    hvws_ctx* c = thread_ctx();
    if (hipSetDevice(c->device) != hipSuccess || c->h_feed.ensure(bytes + 64) != hipSuccess)
        fatal("pinned staging allocation");
    return c->h_feed.as<char>();
}

// XOR `n` host bytes at src into dst with key/phase on the GPU.
void gpu_xor_host(char* dst, const char* src, size_t n, uint32_t key, uint32_t phase) {
    if (n == 0) return;
    hvws_ctx* c = thread_ctx();
    if (door_xor(c, dst, src, n, key, phase)) return;   // no HIP call on the worker's path
    if (hipSetDevice(c->device) != hipSuccess) fatal("hipSetDevice");
    if (c->xor_stage.ensure(n + 64) != hipSuccess) fatal("device staging allocation");
    uint8_t* d = c->xor_stage.as<uint8_t>();
    if (hipMemcpyAsync(d, src, n, hipMemcpyHostToDevice, c->stream) != hipSuccess ||
        launch_xor_span(d, n, key, phase, c->stream) != hipSuccess ||
        hipMemcpyAsync(dst, d, n, hipMemcpyDeviceToHost, c->stream) != hipSuccess ||
        hipStreamSynchronize(c->stream) != hipSuccess) {
        set_err(HVWS_EHIP, "xor span failed");
        fatal("websocket_decode on the GPU");
    }
}

// One-segment batch from host memory for the streaming drop-in.
// Returns frames and the carry-out (WebSocketParser semantics).
void gpu_feed(char* buf, size_t len, const websocket_parser& carry, bool unmask, std::vector<hvws_frame>& frames,
              websocket_parser& carry_out, int& started) {
    hvws_ctx* c = thread_ctx();
    if (door_feed(c, buf, len, carry, unmask, frames, carry_out, started)) return;   // no HIP call there
    if (hipSetDevice(c->device) != hipSuccess) fatal("hipSetDevice");
    hvws_segment seg = {0, (uint64_t)len};
    websocket_parser cin;
    copy_parser(cin, carry);
    if (hvws_rx_batch(c, (uint8_t*)buf, len, &seg, &cin, 1, unmask ? 1 : 0) != HVWS_OK) fatal("hvws_rx_batch");
    const int64_t n = hvws_frame_count(c);
    frames.resize((size_t)n);
    if (n > 0 && hvws_get_frames(c, frames.data(), 0, (uint64_t)n) != HVWS_OK) fatal("hvws_get_frames");
    int st = 0;
    if (hvws_get_carry(c, nullptr, &st) != HVWS_OK) fatal("hvws_get_carry");
    copy_parser(carry_out, cin);
    started = st;
}

}  // namespace hvws

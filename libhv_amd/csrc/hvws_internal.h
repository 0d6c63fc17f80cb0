// hvws_internal.h -- shared between the HIP kernels and the host engine.
#pragma once

#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <stddef.h>
#include <stdlib.h>
#include <stdint.h>
#include <string.h>

#include <atomic>
#include <functional>

#include "websocket_parser.h"

struct hvws_ctx;

namespace hvws {

// $HVWS_EXPERIMENT="name=value,name=value": the A/B switches of the on-device
// sweeps (DESIGN.md sec. 9 lists them).  The text of `name`'s value (up to
// the next ','; atoi / strtoull stop there) or nullptr; read from the
// environment on every call (callers that keep a value cache it themselves).
inline const char* experiment(const char* name) {
    const char* e = getenv("HVWS_EXPERIMENT");
    if (!e) return nullptr;
    const size_t n = strlen(name);
    for (const char* p = e; p && *p; p = strchr(p, ',') ? strchr(p, ',') + 1 : nullptr)
        if (!strncmp(p, name, n) && p[n] == '=') return p + n + 1;
    return nullptr;
}

// With validation on, the state of a header split across reads lives in the
// padding byte after websocket_parser.mask_offset (the reference never reads
// it).  Copies of the struct inside the library go through memcpy: a struct
// assignment may copy member by member and drop the padding.
constexpr size_t kViolByte = offsetof(websocket_parser, mask_offset) + 1;
static_assert(offsetof(websocket_parser, length) > kViolByte, "validation byte must be padding");
inline void copy_parser(websocket_parser& dst, const websocket_parser& src) { memcpy(&dst, &src, sizeof dst); }

// Parser states (reference enum at http/websocket_parser.c:34-40).
enum : uint32_t { S_START = 0, S_HEAD = 1, S_LENGTH = 2, S_MASK = 3, S_BODY = 4 };
enum : uint32_t { F_OPMASK = 0x0Fu, F_FIN = 0x10u, F_MASK = 0x20u };
enum : uint32_t {
    I_HDR = 1u << 10, I_BODY = 1u << 11, I_END = 1u << 12, I_START = 1u << 13, I_INVALID = 1u << 14
};
// Optional protocol validation (RFC 6455 sec. 5.1-5.5; the reference checks
// none of these).  Violation classes, reported in info bits
// I_VSHIFT.. of a frame whose header completes, only for classes enabled in
// the context's validation mask (0 = off = reference behaviour).
enum : uint32_t {
    V_RSV = 1u,        // RSV1-3 set with no extension negotiated
    V_OPCODE = 2u,     // reserved opcode 3-7 / 0xB-0xF
    V_CONTROL = 4u,    // control frame fragmented (FIN = 0) or longer than 125 bytes
    V_LEN64 = 8u,      // 64-bit length with the most significant bit set
    V_NONMIN = 16u,    // length not in its minimal encoding
    V_UNMASKED = 32u,  // client-to-server frame without a mask
    V_ALL = 63u,
    V_ENC_SHIFT = 6u,  // (carry only) 2-bit length encoding of a partial header: 1 = 16-bit, 2 = 64-bit
    I_VSHIFT = 16u
};

// Device-side carry (the websocket_parser fields the walk needs), 48 bytes.
struct dcarry {
    uint32_t state;
    uint32_t flags;
    uint32_t mask;         // mask[0] in bits 0-7
    uint32_t mask_offset;
    uint64_t length;
    uint64_t require;
    uint64_t offset;
    uint32_t started;      // first header byte of the pending frame was in this segment
    uint32_t viol;         // V_* bits (+ encoding) of the partial header, for validation
};

// Per-segment state between the discovery kernels (k_head -> k_verify -> k_walk).
struct dmid {
    dcarry   st;       // parser state after the carried-in frame
    uint64_t pos;      // segment offset of the first whole frame
    uint64_t stride;   // its size (speculation stride), 0 if none
    uint64_t n_a;      // frames recorded before pos (0 or 1)
    uint64_t pad;
};

struct dseg {
    uint64_t off;
    uint64_t len;
};

// Frame table, structure of arrays in HBM (one entry per frame per batch).
struct dframes {
    int64_t*  hdr_off;   // absolute, -1 = header began in an earlier batch
    uint64_t* pay_off;   // absolute
    uint64_t* pay_len;
    uint64_t* length;
    uint32_t* key;       // raw key
    uint32_t* keyrot;    // key rotated for 4-byte aligned words (0 if not masked)
    uint32_t* info;
    uint64_t  cap;       // records the arrays hold; EMIT drops records beyond it (counts stay exact)
};

// One frame record as handed to the host (layout of hvws_frame, 40 bytes).
struct drec {
    int64_t  hdr_off;
    uint64_t pay_off;
    uint64_t pay_len;
    uint64_t length;
    uint32_t key;
    uint32_t info;
};

// Per-segment result of the small-batch kernel, written to pinned host memory.
struct dsmall_out {
    uint64_t first;   // index of the segment's first record in the host record area
    uint64_t count;
    dcarry   st;      // carry out
};

constexpr int SCAN_THREADS = 256;           // 4 waves, one segment per wave
constexpr int SCAN_U = 4;                   // predicted frames per lane per round
constexpr int UNMASK_MAXF = 512;            // frames staged in LDS per tile

// Result of k_spec_check, written by the device into pinned host memory.
struct dspec_status {
    uint64_t seq;     // scan sequence number it belongs to
    uint64_t total;   // records of the batch (sum of the true counts)
    uint32_t flags;   // SPEC_*
    uint32_t pad;
    uint64_t pad2[2];
    uint64_t tseq;    // seq again, published after the scan's last kernel (tile index complete)
    uint64_t pad3[2];
};
enum : uint32_t {
    SPEC_MATCH = 1u,   // every segment's record count equals k_head's estimate
    SPEC_OK = 2u,      // SCAN_SPEC: the speculative table is the exact table (match and within capacity)
    SPEC_ERR = 4u      // one-launch scan: a grid barrier timed out (results void)
};

struct sieve_bufs;

// RUN path (round 5): a batch whose segments each hold one run of equal
// frames (the last check saw uniform counts) is unmasked from per-segment
// descriptors alone -- no per-frame records, no second pass over the header
// lines.  k_head writes the descriptor (the carried-in frame and the frame cut
// by the segment end exactly, the run in between as a hypothesis: the first
// whole frame's size repeated); k_unmask_run parses every run header from
// the tile bytes it loads anyway, checks it against the hypothesis and takes
// its key from it; k_run_fix, queued behind on the same stream, undoes and
// redoes exactly any segment whose hypothesis failed, so work queued after a
// step always sees the reference's bytes.  Frame records are built on demand
// (an exact scan of the unchanged headers) when a reader asks for them.
struct drun {
    uint64_t seg_lo, seg_hi;   // the segment's absolute byte range
    uint64_t p0;               // absolute offset of the run's first header
    uint64_t stride;           // bytes per frame of the run (0: no run)
    uint64_t len;              // payload bytes per frame of the run
    double   inv;              // 1 / stride
    uint32_t cnt, hlen;        // frames in the run, header bytes of each
    uint32_t masked, flags;    // run frames carry a key (the first's mask bit); RUN_*
    uint64_t a_off, a_end;     // carried-in frame's payload piece [a_off, a_end), absolute
    uint64_t t_off, t_end;     // payload piece of the frame cut by the segment end
    uint32_t a_kw, t_kw;       // their key words for 4-byte aligned words (0: nothing to XOR)
    uint64_t pad;
    dcarry   cin;              // the segment's carry-in (the repair's exact path; the shared
                               // carry table belongs to the next scan by then)
};
static_assert(sizeof(drun) == 160, "drun layout");
// Per unmask tile (64 bytes, k_run_tiles): the first segment meeting the
// tile (s0, nseg if none) and the last (s1), and s0's run as it meets the
// tile, tile-relative: its first run frame's header h0 (>= -S), the run
// frames meeting the tile (nj; 0 if s0 is left to the repair), k0 -- the key
// of the run frame begun before the tile (its header read beside the previous
// unmask) -- and the carried-in / cut frame's payload pieces clipped to the
// tile.  A tile of one segment needs no other load before its unmask.
struct dtrun {
    uint32_t s0, s1, k0;
    int32_t  h0;
    uint32_t nj, S, len, hm;    // run frames meeting the tile, stride, payload bytes, header bytes | masked << 8
    int32_t  a_lo, a_hi, t_lo, t_hi;
    uint32_t a_kw, t_kw;        // 0: no piece
    uint32_t pad[2];
};
static_assert(sizeof(dtrun) == 64, "dtrun layout");
enum : uint32_t { RUN_BAD = 1u };   // the segment is not one run (k_head saw it): exact repair only
constexpr uint64_t RUN_MAX_FRAME = 8192;   // frames at most this size take the RUN path (bigger: SPEC)
constexpr uint64_t RUN_MIN_SEG = 65536;    // and segments of at least this size on average
// k_head<false> writes runs[s] when given; k_run_tiles: trun[t] for every
// unmask tile (t < ntiles, dtrun); fail[s] is segment
// s's failure word (zeroed by k_head; k_run_tiles sets bit 2 for a segment
// k_unmask_run leaves to the repair), fail[nseg .. nseg + 2] the batch's
// (any failed, failed count, repair workgroups done), zero between RUN steps
// (the repair clears them all; the host zeroes a new array).
hipError_t launch_run_tiles(const uint8_t* rx, uint64_t rx_len, const dseg* segs, uint32_t nseg, const drun* runs,
                            dtrun* trun, uint64_t ntiles, uint64_t tile, uint32_t* fail, hipStream_t st);
// The RUN unmask (RUN_TILE bytes per tile, the tiles k_run_tiles described)
// and its repair pass; the timing events ride on the unmask's first dispatch
// (start) and the repair's (stop).  The repair publishes (seq, failed
// segments) to status->pad3 when it is done.
constexpr uint64_t RUN_TILE = 16384;   // 256 threads x 4 chunks of 16 B
const char* run_kernel_name();
hipError_t launch_unmask_run(uint8_t* rx, uint64_t rx_len, const drun* runs, const dtrun* trun, uint32_t nseg,
                             uint32_t* fail, dspec_status* status, uint64_t seq, hipStream_t st, hipEvent_t ev_start,
                             hipEvent_t ev_stop);
constexpr uint64_t RUN_FAST_STRIDE = 1u << 20;   // run strides up to this take k_unmask_run's one-segment path

struct scan_scratch {   // per-segment arrays (nseg entries) + one total
    dmid*     mid;
    uint64_t* npred;
    uint64_t* pbase;
    uint64_t* first_fail;
    uint64_t* last_masked;   // 1 + index of the last masked verified frame, 0 none
    uint64_t* total_pred;
    uint64_t* est;           // records k_head predicts per segment (uniform-stride hypothesis)
    // Zero-copy upload: when src_segs is set, the first k_head of the scan
    // reads the segment and carry tables from these (device-mapped pinned
    // host) arrays and writes the device tables the later kernels read.
    const dseg*   src_segs;
    const dcarry* src_carry;
    dseg*         segs_w;
    dcarry*       carry_w;
    dspec_status* status;    // device-mapped pinned host
    uint64_t      seq;
    const sieve_bufs* sieve; // SINGLE / its re-EMIT: frame sieve buffers, nullptr = no sieve
    dframes   slack;         // SLACK: scratch table
    uint64_t  slack_cap;     // SLACK: records per segment region at most
    uint64_t* bases_x;       // SLACK: exact bases (nseg)
    uint64_t* est_u;         // SLACK: uniform-stride estimates (nseg), for SPEC_MATCH
    uint32_t  no_verify;     // SPEC/SLACK: head + walk only (no k_verify pair, no k_head<true>)
    drun*     runs;          // RUN: k_head writes each segment's run descriptor
    uint32_t* run_fail;      // RUN: per-segment failure words + the batch's, zeroed by k_head / k_run_tiles
    dtrun*    run_trun;      // RUN: per unmask tile (run_ntiles entries)
    uint64_t  run_ntiles, run_tile;
};

// Bijective XCD-contiguous tile order: the dispatcher deals blocks b, b+8,
// b+16, ... to one XCD; map them to adjacent tiles so each XCD's L2 and
// memory channels see one contiguous range.
__device__ __forceinline__ uint64_t xcd_tile(uint64_t b, uint64_t ntiles) {
    const uint64_t q = ntiles >> 3, r = ntiles & 7u, x = b & 7u, i = b >> 3;
    return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + i;
}

// Workgroup b -> tile, runs of g adjacent tiles per XCD: within each window
// of 8 g tiles, XCD x (= b mod 8, the hardware's round-robin placement) takes
// tiles x g .. x g + g - 1, in order.  Neighbouring tiles that share a cache
// line (a payload span's boundary line, a line of the per-frame tables) then
// meet in one L2 instead of being fetched from memory by two XCDs, while the
// eight XCDs still stream through the same window of memory (the whole-range
// XCD order of xcd_tile halved k_build's rate).  A bijection on
// [0, ntiles): the last partial window keeps the linear order.
__device__ __forceinline__ uint64_t xcd_group_tile(uint64_t b, uint64_t ntiles, uint32_t g) {
    const uint64_t win = 8ull * g, full = ntiles - ntiles % win;
    if (g <= 1 || b >= full) return b;
    const uint64_t w = b / win, r = b % win;
    return w * win + (r & 7u) * g + (r >> 3);
}

// Frame sieve (hvws_sieve.hip): parallel discovery of one long mixed-size
// stream.  State of the current scan, device side.
struct dsieve {
    uint64_t active;        // this scan's one segment is sieved
    uint64_t use;           // k_walk resumes at pend with npath chain frames recorded
    uint64_t pend;          // segment offset where the exact walk resumes
    uint64_t last;          // 1 + segment offset of the chain's last frame
    uint64_t last_masked;   // 1 + segment offset of the chain's last masked frame
    uint64_t npath;         // frames on the chain
    uint64_t pad[2];
};

// Device buffers of the sieve (per context; scans run in order on one stream).
struct sieve_bufs {
    dsieve*   state;
    uint64_t* tcount;    // per 8 KiB tile: survivors        (sieve_tiles_max entries)
    uint64_t* tbase;     // exclusive scan of tcount          (sieve_tiles_max)
    uint32_t* slot;      // first survivors of each tile      (sieve_slot_words)
    uint32_t* pool;      // survivors of tiles with more      (capS)
    uint64_t* pool_n;    // pool entries used
    uint64_t* keep;      // 1 = survivor after HBM verification (capS)
    uint64_t* kbase;     // exclusive scan of keep            (capS)
    uint64_t* Spre;      // survivors before HBM verification (capS)
    uint64_t* m_pre;     // entries of Spre
    uint64_t* S;         // survivor segment offsets, sorted  (capC)
    uint32_t* J0;        // successor / doubling tables       (capC each)
    uint32_t* J1;
    uint64_t* mark;      // 1 = on the chain                  (capC)
    uint32_t* hops;      // whole frames from a node to its successor (capC)
    uint64_t* rank;      // exclusive scan of mark * hops     (capC)
    uint64_t* m_total;   // survivors
    uint64_t* npath;     // chain frames
    uint64_t* tmp;       // scan scratch (>= 4 * ceil(max(capS, tiles) / 1024) + 64 words)
    uint64_t  capS;      // entries before verification, < 2^32
    uint64_t  capC;      // survivors / chain nodes, <= capS
    uint32_t  rt, wt;    // windows: the first wt of every rt tiles are sieved (rt == wt: every tile)
    uint64_t* scr;       // windowed: each node's first 2^lgP frame offsets (capC << lgP), or nullptr
    uint32_t  lgP;
};
uint64_t sieve_tiles_max(uint64_t rx_len);
uint64_t sieve_slot_words(uint64_t rx_len);
uint64_t sieve_min();                  // bytes after the first whole frame from which a mixed stream is sieved
uint64_t set_sieve_min(uint64_t v);    // 0 = default; returns the previous value
uint64_t sieve_generation();           // bumped by set_sieve_min (contexts forget their sieve history)
// Window geometry for a one-segment scan of rx_len bytes whose last exact
// count was nframes (0: unknown -> every tile): rt, wt in tiles.
void sieve_geometry(uint64_t rx_len, uint64_t nframes, uint32_t& rt, uint32_t& wt);
void set_sieve_windows(uint64_t hops, uint64_t window, uint64_t prev[2]);   // bumps sieve_generation()
uint64_t sieve_hops();                 // frames per region the window geometry aims at (0: windows off)
hipError_t launch_sieve(const uint8_t* rx, uint64_t rx_len, const dseg* segs, const dmid* mid, const uint64_t* npred,
                        const sieve_bufs& b, hipStream_t st);
hipError_t launch_sieve_emit(const uint8_t* rx, uint64_t rx_len, const dseg* segs, const dmid* mid,
                             const sieve_bufs& b, dframes fr, uint32_t vmask, hipStream_t st);

// Kernel launchers (hvws_kernels.hip).
// COUNT pass (emit=false): counts[], bases[] (exclusive scan) and *total.
// EMIT pass: frame table at bases[], carry_out[].
// SINGLE (one segment, base 0 known): COUNT's speculation only, then EMIT,
// which also writes counts[] -- the serial walk of a mixed-size stream runs
// once instead of twice.
// SPEC (several segments, frame table of known capacity): EMIT at bases
// taken from k_head's per-segment estimates, then k_spec_check compares the
// true counts with them -- equal everywhere means the table is exact, so a
// uniform batch is discovered with one walk and no host round trip before
// EMIT; otherwise *total is zeroed (the tile kernels and k_unmask then do
// nothing) and the host re-runs COUNT + EMIT.  COUNT also runs the check,
// to tell the host whether the next batch is worth speculating on.
// SLACK (several segments of mixed sizes): one EMIT walk into per-segment
// regions of a scratch table (sized by each segment's record bound, capped at
// slack_cap), then a device check that every segment fit and a compaction into
// the frame table at the exact bases; a segment that did not fit zeroes *total
// and the host re-scans COUNT + EMIT.
// RUN: k_head writing run descriptors (no est, no walk) + the tile-segment index.
enum scan_pass { SCAN_COUNT = 0, SCAN_EMIT = 1, SCAN_SINGLE = 2, SCAN_SPEC = 3, SCAN_SLACK = 4, SCAN_RUN = 5 };
hipError_t launch_scan(int pass, const uint8_t* rx, uint64_t rx_len, const dseg* segs, uint32_t nseg,
                       const dcarry* carry_in, dcarry* carry_out, uint64_t* counts, uint64_t* bases,
                       uint64_t* total, scan_scratch sc, dframes fr, uint32_t vmask, hipStream_t st);
hipError_t launch_offsets(const uint64_t* counts, uint64_t* bases, uint32_t nseg, uint64_t* total,
                          hipStream_t st);
// status->tseq = seq (system-scope release), after every earlier kernel of the stream:
// the host sees that the scan's tables are complete without a stream event.
hipError_t launch_publish_tiles(dspec_status* status, uint64_t seq, hipStream_t st);
// *total > cap: *total = 0; publishes the count to status (SPEC_OK if within cap).
hipError_t launch_cap_check(uint64_t* total, uint64_t cap, dspec_status* status, uint64_t seq, hipStream_t st);
hipError_t launch_ends_check(const uint64_t* off, const uint64_t* len, const uint64_t* nfr_dev,
                             unsigned long long* bad, hipStream_t st);
hipError_t launch_tile_index(const uint64_t* off, const uint64_t* len, uint64_t nfr, const uint64_t* nfr_dev,
                             uint32_t* tile_first, uint64_t ntiles, uint64_t tile, hipStream_t st);
// Tile index marks: a tile no frame's scatter reached (k_tile_fixup searches
// it); a frame scatters itself into at most TILE_SPAN_MAX tiles.
constexpr uint32_t TILE_MARK = 0xFFFFFFFFu;
constexpr uint64_t TILE_SPAN_MAX = 64;
// k_tile_fixup alone (tile_first already scattered).
hipError_t launch_tile_fixup(const uint64_t* off, const uint64_t* len, uint64_t nfr, uint32_t* tile_first,
                             uint64_t ntiles, uint64_t tile, hipStream_t st);
// Small batches, whole path in one launch (one wave per segment): records
// into slots[slot_base[s]..], then compacted into h_rec (pinned host) when
// they fit h_rec_cap; results into h_out[s]; unmasked chunks into h_rx
// (pinned host, same layout as rx).  *rec_total (device) must equal rec_base
// on entry and advances by the records written.  stage_lds != 0: each segment
// is staged in stage_lds bytes of LDS (>= its 16-aligned span + 16); rx,
// segs, carry_in and slot_base may then be pinned host memory read in place
// (zero-copy).
constexpr uint64_t kStageSegment = 32ull << 10;   // largest segment k_small stages in LDS
constexpr uint64_t kZcBatch = 1ull << 20;         // largest batch sent zero-copy
hipError_t launch_small(const uint8_t* rx, uint64_t rx_len, const dseg* segs, const dcarry* carry_in, uint32_t nseg,
                        const uint64_t* slot_base, drec* slots, unsigned long long* rec_total, uint64_t rec_base,
                        drec* h_rec, uint64_t h_rec_cap, dsmall_out* h_out, uint8_t* h_rx, int unmask, uint32_t vmask,
                        uint32_t stage_lds, uint64_t* h_done, uint64_t seq, hipStream_t st,
                        hipEvent_t ev_start = nullptr, hipEvent_t ev_stop = nullptr);
// Resident small-path worker ("door", k_door): one workgroup that stays on
// the device between calls and takes one request at a time from a mailbox in
// fine-grained pinned host memory, so a reference-API call (FeedRecvData,
// websocket_parser_execute, websocket_decode, a masked websocket_build_frame)
// pays neither a launch nor a dispatch.  The host writes the request fields,
// then `seq` (release); the worker serves it and publishes `done = seq`
// (system-scope release) after its results.  A worker idle for idle_ticks of
// the 100 MHz realtime clock parks itself (alive = 0, after one last look at
// seq) and the next request relaunches it.  Every launch carries an epoch;
// a worker's last store before it returns is `exited = epoch`, and the host
// takes that word -- not the stream's status -- as the sign that the worker
// has ended ("Resident worker").
enum : uint32_t { DOOR_FEED = 1u, DOOR_XOR = 2u, DOOR_EXIT = 3u };
constexpr uint32_t kDoorThreads = 512;              // 8 waves: staging and XOR in parallel, walk on wave 0
constexpr uint64_t kDoorMax = 32ull << 10;          // largest request (bytes)
constexpr uint64_t kDoorRecords = kDoorMax / 2 + 3; // records a kDoorMax segment can hold
struct ddoor {
    // host -> device (written before seq)
    uint64_t seq;
    uint32_t op;
    uint32_t unmask;
    uint64_t len;
    uint32_t vmask;
    uint32_t key;       // DOOR_XOR: mask word (mask[0] in bits 0-7)
    uint32_t phase;     // DOOR_XOR: mask_offset of the first byte
    uint32_t pad0;
    dcarry   carry;     // DOOR_FEED: carry in
    uint64_t pad1[4];
    uint64_t seq_tail;  // seq again, written with the fields (before seq): the worker reads the
                        // whole block with its poll and takes it when both copies agree
    // device -> host (own cache lines; `done` written last)
    uint64_t done;      // seq of the last request served
    uint64_t alive;     // 1 while a worker runs (0 once it parked)
    uint64_t count;     // DOOR_FEED: records written
    uint64_t served;    // requests served by this worker (diagnostic)
    dcarry   out;       // DOOR_FEED: carry out
    uint64_t exited;    // epoch of the last worker that has ended (its last store before it returns)
    uint64_t pad2[1];
    // realtime-clock stamps of the last request (100 MHz): seen, staged,
    // walked, xored, stored (before the release); read by hvws_door_stamps'
    // diagnostics (scripts/probe/door_phases.py)
    uint64_t stamp[12];   // [6]: the previous request's release, ticks; [8..10]: door_walk's chase, parse, tail ends
};
static_assert(sizeof(dcarry) == 48, "dcarry layout");
static_assert(offsetof(ddoor, done) == 128, "ddoor: device fields on their own lines");
static_assert(offsetof(ddoor, seq_tail) == 120, "k_door reads seq_tail as the last 8 bytes of the request block");
static_assert(offsetof(ddoor, carry) == 40 && offsetof(ddoor, len) == 16 && offsetof(ddoor, vmask) == 24,
              "k_door reads the request as words 1-10");
// data areas: kDoorMax + 256 bytes (256-aligned); h_rec: kDoorRecords records
// (pinned); d_slot: kDoorRecords records (device) for records past the LDS area.
// req: the request block (words 0-15 of a ddoor) -- fine-grained device
// memory the host writes through the PCIe BAR, or the pinned box itself;
// din: the request's bytes (same choice); dout: results (pinned host; may equal
// din when both are the pinned area).
// k_door's kernel arguments, as an AQL dispatch of it reads them (the
// kernel's explicit arguments in order; it uses no hidden ones).
struct door_args {
    const ddoor* req;
    ddoor* box;
    const uint8_t* din;
    uint8_t* dout;
    drec* h_rec;
    drec* d_slot;
    uint64_t idle_ticks, first_seq, epoch;
    uint32_t flags;
};
uint32_t door_flags();                      // k_door's flags ($HVWS_EXPERIMENT door_stamps)
hipError_t door_anchor(void** dev_addr);    // a device symbol of k_door's code object (loads it on the device)
const char* door_kernel_symbol_prefix();    // k_door's symbol name, up to its argument types

// The worker's own HSA queue (hvws_doorq.cpp): k_door dispatched by one AQL
// packet per launch; `done` (its completion signal) reaches 0 when the launch
// has ended; destroyed only then.
struct door_queue {
    hsa_queue_t* q = nullptr;
    hsa_signal_t done{0};
    hsa_agent_t agent{0};
    uint64_t object = 0;                   // k_door's kernel descriptor
    uint32_t group = 0, priv = 0, kernarg_size = 0;
    void* kernarg = nullptr;               // pinned host
    void* kernarg_dev = nullptr;
    int device = -1;
    bool at_exit = false;                  // destroyed from the exit handler: no HIP call
    std::atomic<int> error{0};             // queue error reported by the runtime (hsa_status_t)
};
int  door_queue_create(int device, door_queue** out);
int  door_queue_launch(door_queue* q, const void* args, uint32_t nargs);
bool door_queue_idle(door_queue* q);     // the last launch has ended (or none was made)
int  door_queue_error(door_queue* q);    // 0, or the queue's error status
const char* door_queue_why();            // what the last failing door_queue_* call of this thread hit
void door_queue_destroy(door_queue* q);  // only when idle

// Host copy pool (hvws_hostpool.cpp): fn(i) for i in [0, n) on up to
// copy_width() threads (the caller included; serial when another caller
// holds the pool); par_memcpy splits copies of >= kParCopyMin bytes.
constexpr uint64_t kParCopyMin = 1ull << 20;
int copy_width();
void par_for(int n, const std::function<void(int)>& fn);
void par_memcpy(void* dst, const void* src, uint64_t n);
// Batched handshake digest (hvws_keys.hip): accept[32*i..] = base64(SHA-1(key_i + GUID)), 28 chars + 4 zero bytes.
hipError_t launch_encode_keys(const uint8_t* keys, const uint64_t* key_off, const uint32_t* key_len, uint64_t n,
                              uint8_t* accept, hipStream_t st);
// Predicted frames above which a uniform segment is verified grid-wide (k_verify).
uint64_t spec_min();
uint64_t set_spec_min(uint64_t v);   // 0 = default; returns the previous value
// k_unmask geometry variants (threads x chunks/thread, XCD-ordered tiles)
int unmask_variant();                      // the forced geometry, else the large-batch default
int unmask_variant_for(uint64_t rx_len);   // the geometry a batch of rx_len bytes runs with
int set_unmask_variant(int v);             // -1 = by batch size; -2 if out of range
int unmask_variant_count();
uint64_t unmask_tile(int variant);         // bytes per workgroup tile
const char* unmask_name(int variant);
hipError_t launch_unmask(int variant, uint8_t* rx, uint64_t rx_len, dframes fr, const uint32_t* tile_first,
                         const uint32_t* tile_key, const uint8_t* tile_kind, const uint64_t* nfr_dev, hipStream_t st,
                         uint32_t pieces = 1, hipEvent_t ev_start = nullptr, hipEvent_t ev_stop = nullptr);
hipError_t launch_tile_class(const uint64_t* off, const uint64_t* len, const uint32_t* keyrot, const uint64_t* nfr_dev,
                             const uint32_t* tile_first, uint32_t* tile_key, uint8_t* tile_kind, uint64_t ntiles,
                             uint64_t tile, uint64_t rx_len, hipStream_t st);
// Tile index + tile classes for k_unmask in one sequence (fill, scatter,
// fused fixup/classify); tile_first must hold ntiles + 8 entries.
hipError_t launch_unmask_tiles(const uint64_t* off, const uint64_t* len, const uint32_t* keyrot, const uint64_t* nfr_dev,
                               uint32_t* tile_first, uint32_t* tile_key, uint8_t* tile_kind, uint64_t ntiles,
                               uint64_t tile, uint64_t rx_len, hipStream_t st);
hipError_t launch_stream_xor(int variant, uint8_t* d, uint64_t n, uint32_t pattern, hipStream_t st);
hipError_t launch_xor_span(uint8_t* d, uint64_t n, uint32_t key, uint32_t phase, hipStream_t st);
hipError_t launch_noop(hipStream_t st);   // see hvws_dev_free

// Synthetic data (hvws_synth.hip).
hipError_t launch_synth(uint8_t* buf, uint64_t buf_len, uint64_t seed, uint64_t nframes,
                        const uint64_t* frame_off, const uint8_t* flags, const uint32_t* mask,
                        const uint64_t* length, const uint8_t* text, const uint64_t* frame_size,
                        const uint32_t* tile_first, int mode, unsigned long long* mismatches,
                        hipStream_t st);
hipError_t launch_digest(const uint8_t* buf, uint64_t len, unsigned long long* out, hipStream_t st);
hipError_t launch_frame_sizes(const uint8_t* flags, const uint64_t* length, uint64_t nframes,
                              uint64_t* out, hipStream_t st);
uint64_t synth_tile();

// Transmit side (hvws_tx.hip).
// out[i] = sum(in[0..i)), *total = sum(in); tmp >= 4 * ceil(n / 1024) + 64 words.
hipError_t launch_exclusive_scan(const uint64_t* in, uint64_t* out, uint64_t n, uint64_t* tmp, uint64_t* total,
                                 hipStream_t st);
// stat[1] += frames whose payload range leaves [0, plen) or that are masked
// without a key table; stat[2] += frames breaking the uniform layout (size
// or length other than frame 0's, payload offset step other than frame 1's or
// negative); stat[3..5] = pay_off[0], pay_off[1] - pay_off[0], len[0].
hipError_t launch_tx_check(const uint64_t* pay_off, const uint64_t* len, const uint8_t* flags, const uint32_t* mask,
                           const uint64_t* size, uint64_t n, uint64_t plen, uint64_t* stat, hipStream_t st);
// k_build geometry for a batch of out_len output bytes in n frames
// ($HVWS_EXPERIMENT build, else by the mean frame size), its tile and its name
int tx_variant(uint64_t out_len, uint64_t n);
uint64_t tx_tile(int v);   // output bytes per k_build workgroup
const char* build_kernel_name(int v);
// The transmit tile index and (span != nullptr: 2 words per k_build tile)
// source spans in three launches: one fill of both, one pass over the frames
// doing the tile scatter and the span runs together, k_tile_fixup (in place
// of a tile index's fill, scatter and fixup plus a span fill and pass).
hipError_t launch_tx_index(const uint64_t* out_off, const uint64_t* size, const uint64_t* pay_off, const uint64_t* len,
                           const uint8_t* flags, uint64_t n, uint64_t ntiles, uint64_t tile, uint32_t* tile_first,
                           uint64_t* span, hipStream_t st);
// span: from launch_tx_index, or nullptr (boundary tiles load their records
// first).  uni (host array {stride, header bytes, pay_off[0], payload offset
// step}, stride != 0): a uniform layout -- every tile finds its frame range and
// span from its position, tile_first and span are not read (no index pass).
hipError_t launch_build(uint8_t* out, uint64_t out_len, const uint8_t* pay, uint64_t plen, const uint64_t* pay_off,
                        const uint64_t* len, const uint8_t* flags, const uint32_t* mask, const uint64_t* out_off,
                        const uint64_t* size, const uint32_t* tile_first, const uint64_t* span, uint64_t n, int v,
                        hipStream_t st, const uint64_t* uni = nullptr);

}  // namespace hvws

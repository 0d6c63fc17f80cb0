/*
 * hvws.h -- batch / device-resident C ABI of the MI355X WebSocket receive
 * engine (libhv_amd/libhvws.so).  New entry points; the reference has no
 * batch API.  What each one stands in for:
 *
 *   hvws_scan    websocket_parser_execute's header state machine
 *                (reference http/websocket_parser.c:53-171) run over many
 *                segments (= connections' rx bytes) at once: frame
 *                discovery + FIN/opcode/mask/length extraction on the GPU.
 *   hvws_unmask  the per-byte XOR of websocket_parser_decode
 *                (http/websocket_parser.c:173-180) as called in place by
 *                WebSocketParser's on_frame_body (http/WebSocketParser.cpp:32-34),
 *                applied to every masked payload span the last scan found.
 *   hvws_step    scan + unmask: one pass of the hot path over a batch.
 *   hvws_rx_batch  the same from/to host memory (H2D, step, D2H).
 *   hvws_build_frames  transmit side: websocket_build_frame
 *                (http/websocket_parser.c:207-256, as called per message by
 *                WebSocketChannel::sendFrame via ws_build_frame,
 *                http/WebSocketChannel.cpp:66-79, http/wsdef.c:36-46)
 *                for a whole batch of outgoing frames at once.
 *   hvws_encode_keys  the handshake digest ws_encode_key (http/wsdef.c:11-20)
 *                for a batch of upgrade requests.
 *   hvws_wsp_*   C handle over the WebSocketParser class
 *                (http/WebSocketParser.h:19-31) for FFI callers.
 *
 * A batch is a buffer holding `nseg` segments; segment s is the byte range
 * [segs[s].off, segs[s].off + segs[s].len) and continues the stream whose
 * parser state is carry[s] (a `struct websocket_parser`).  Segments must be
 * sorted by offset and must not overlap.  Contexts are per (thread, device):
 * several event-loop threads may each own one; there is no global lock.
 * Device buffers passed in must be 16-byte aligned.
 */
#ifndef HVWS_H
#define HVWS_H

#include <stddef.h>
#include <stdint.h>

#include "websocket_parser.h"

#ifdef __cplusplus
extern "C" {
#endif

enum {
    HVWS_OK = 0,
    HVWS_ENODEV = -1,   /* no HIP device / runtime */
    HVWS_EINVAL = -2,
    HVWS_ENOMEM = -3,
    HVWS_EHIP = -4      /* a HIP call failed; see hvws_last_error() */
};

/* hvws_frame.info bits */
#define HVWS_I_FLAGS       0xFFu      /* websocket_flags of the frame          */
#define HVWS_I_PHASE_SHIFT 8          /* 2-bit mask phase at pay_off           */
#define HVWS_I_HDR         (1u << 10) /* header completed here (on_frame_header fires) */
#define HVWS_I_BODY        (1u << 11) /* >= 1 payload byte here (on_frame_body fires)   */
#define HVWS_I_END         (1u << 12) /* frame completed here (on_frame_end fires)      */
#define HVWS_I_START       (1u << 13) /* first header byte is inside this segment       */
#define HVWS_I_INVALID     (1u << 14) /* header violates an enabled validation class    */
#define HVWS_I_VSHIFT      16         /* HVWS_V_* classes violated, bits 16-21           */

/* Optional protocol validation (hvws_set_validation), RFC 6455 sec. 5.1-5.5.
 * The reference checks none of these, so all are off by
 * default and results are then identical to the reference's. */
#define HVWS_V_RSV       (1u << 0)  /* RSV1-3 set (no extension is negotiated)        */
#define HVWS_V_OPCODE    (1u << 1)  /* reserved opcode 3-7 or 0xB-0xF                 */
#define HVWS_V_CONTROL   (1u << 2)  /* control frame with FIN = 0 or > 125 bytes      */
#define HVWS_V_LEN64     (1u << 3)  /* 64-bit length with its most significant bit set */
#define HVWS_V_NONMIN    (1u << 4)  /* length not in its minimal encoding             */
#define HVWS_V_UNMASKED  (1u << 5)  /* client-to-server frame without a mask          */
#define HVWS_V_ALL       0x3Fu

typedef struct hvws_ctx hvws_ctx;

typedef struct hvws_segment {
    uint64_t off;
    uint64_t len;
} hvws_segment;

/* One frame as seen by one batch (40 bytes). Offsets are absolute in the
 * batch buffer. */
typedef struct hvws_frame {
    int64_t  hdr_off;   /* first header byte, -1 if it was in an earlier batch */
    uint64_t pay_off;   /* first payload byte of this frame in the batch       */
    uint64_t pay_len;   /* payload bytes of this frame inside the batch        */
    uint64_t length;    /* full payload length (parser->length)                */
    uint32_t key;       /* masking key, mask[0] in bits 0-7 (0 if unmasked)    */
    uint32_t info;      /* HVWS_I_* */
} hvws_frame;

/* ---- context / memory ---------------------------------------------- */
int         hvws_device_count(void);
hvws_ctx*   hvws_ctx_create(int device);          /* NULL on failure */
void        hvws_ctx_destroy(hvws_ctx* ctx);
const char* hvws_last_error(void);                /* thread-local */
void*       hvws_ctx_stream(hvws_ctx* ctx);       /* hipStream_t */
int         hvws_ctx_device(hvws_ctx* ctx);
/* The PCI bus id ("dddd:bb:dd.f", NUL-terminated, len >= 13) of HIP device
 * `device` and, in *cur, the device hipGetDevice reports once it is selected:
 * a multi-GPU run names the physical card each rank used. */
int         hvws_device_identity(int device, char* bus_id, int len, int* cur);

void* hvws_dev_alloc(hvws_ctx* ctx, uint64_t bytes);
void  hvws_dev_free(hvws_ctx* ctx, void* p);
void* hvws_host_alloc(hvws_ctx* ctx, uint64_t bytes); /* pinned */
void  hvws_host_free(hvws_ctx* ctx, void* p);
int   hvws_h2d(hvws_ctx* ctx, void* dst, const void* src, uint64_t n);  /* async, ctx stream */
int   hvws_d2h(hvws_ctx* ctx, void* dst, const void* src, uint64_t n);  /* async, ctx stream */
int   hvws_memset(hvws_ctx* ctx, void* dst, int v, uint64_t n);
int   hvws_d2d(hvws_ctx* ctx, void* dst, const void* src, uint64_t n);  /* async, ctx stream */
int   hvws_sync(hvws_ctx* ctx);
/* Tests only: hold back work queued on the ctx stream after this call for
 * `usec` microseconds without occupying the device (a host function on the
 * stream), e.g. to keep an unmask waiting while the second stream runs on. */
int   hvws_debug_stall(hvws_ctx* ctx, uint32_t usec);

/* ---- the hot path, device resident ---------------------------------- */
/* Frame discovery + header parse for every segment.  Waits for the device
 * once (to size the frame table, or for its speculative table's check; see
 * hvws_set_speculation) -- not for earlier work on the stream to finish.
 * Results stay on the device in `ctx`. */
int hvws_scan(hvws_ctx* ctx, const uint8_t* d_rx, uint64_t rx_len, const hvws_segment* segs,
              const websocket_parser* carry_in, uint32_t nseg);
/* Unmask, in place, every masked payload span found by the last scan.
 * Asynchronous on the ctx stream. */
int hvws_unmask(hvws_ctx* ctx, uint8_t* d_rx, uint64_t rx_len);
/* scan + unmask */
int hvws_step(hvws_ctx* ctx, uint8_t* d_rx, uint64_t rx_len, const hvws_segment* segs,
              const websocket_parser* carry_in, uint32_t nseg);
/* hvws_step for a batch whose bytes are already complete in device memory
 * (nothing queued on the context stream still writes them).  Its discovery
 * then runs on the context's second stream, overlapping the unmask of the
 * previous step, whose tables are kept in the other of two table sets; the
 * unmask is queued on the context stream after it, as with hvws_step.  Frames
 * and carry of the call are readable (hvws_get_*) until the next scan; work
 * queued on the context stream afterwards sees the unmasked bytes.
 * A step that took the RUN path (hvws_set_run; hvws_step too) builds its
 * frames and carry when hvws_get_* / hvws_frame_count first asks, from the
 * batch's header bytes: those bytes must not change until then (reading them
 * before the next receive into the buffer, or calling hvws_frame_count right
 * after the step, fixes them).  Payload bytes may change freely. */
int hvws_step_resident(hvws_ctx* ctx, uint8_t* d_rx, uint64_t rx_len, const hvws_segment* segs,
                       const websocket_parser* carry_in, uint32_t nseg);

int64_t hvws_frame_count(hvws_ctx* ctx);
int     hvws_get_frames(hvws_ctx* ctx, hvws_frame* out, uint64_t first, uint64_t n);
/* first frame index and frame count of every segment of the last scan */
int     hvws_get_segment_frames(hvws_ctx* ctx, uint64_t* first, uint64_t* count);
/* parser state after each segment (WebSocketParser semantics: mask_offset
 * advanced over unmasked bytes).  started[s] = 1 when the pending frame's
 * first header byte lay inside segment s. */
int     hvws_get_carry(hvws_ctx* ctx, websocket_parser* out, int* started);

/* Device time (ms, HIP events on the ctx stream) of the last scan and
 * unmask: out[0] = scan kernels (count + offsets + emit + tile index),
 * out[1] = unmask kernel.  A pipelined step (hvws_step_resident) records the
 * unmask's events only: its out[0] is -1 ($HVWS_STEP_EVENTS=2 records both).
 * The small-batch path (reads of an event loop) records none unless
 * $HVWS_STEP_EVENTS=2: out[0] = out[1] = -1 (an event-carrying launch costs
 * ~10 us of a ~30 us read). */
int hvws_last_times(hvws_ctx* ctx, float out[2]);
/* The same for each of the last min(max_steps, 32) scans, oldest first:
 * out[2*i] = scan ms, out[2*i+1] = unmask ms (-1 if the step had none).
 * Waits for those steps only; returns the number of steps written (< 0 on
 * error).  Lets a caller time a run of asynchronous steps afterwards. */
int hvws_step_times(hvws_ctx* ctx, float* out, int max_steps);
/* Record those timing events on every `every`-th scan only (1, the default:
 * every scan; 0: none).  Each event-carrying step costs device time between
 * kernels -- ~15 us of a 0.38 ms pipelined config-2 step -- so a caller that
 * times a long run samples it (bench.py: every 8th step); unsampled steps
 * read -1.  Returns the previous interval (< 0 on error). */
int hvws_set_step_event_interval(hvws_ctx* ctx, uint32_t every);

/* k_unmask geometry.  By default it follows the batch size: 512 threads x 2
 * chunks in linear tile order below 16 GiB, 256 x 4 in XCD-contiguous order
 * from there (measured).  hvws_unmask_kernel_name: the name
 * of the forced geometry, or of the large-batch one; ..._for: the geometry a
 * batch of rx_len bytes runs with (e.g. "k_unmask<256,4,xcd>"). */
const char* hvws_unmask_kernel_name(void);
const char* hvws_unmask_kernel_name_for(uint64_t rx_len);
/* The RUN path's unmask kernel (HVWS_PATH_RUN steps), e.g. "k_unmask_run<256,4,lds>". */
const char* hvws_run_kernel_name(void);
/* Force a k_unmask geometry for later scans (tuning; process-wide); -1 =
 * back to the choice by batch size. */
int hvws_set_unmask_variant(int variant);

/* Uniform runs of at least `frames` predicted frames in one segment are
 * verified grid-wide (k_verify); shorter ones by the per-segment wave walk.
 * Tuning only (process-wide, default 4096, 0 = default); results never
 * depend on it.  Returns the previous value. */
uint64_t hvws_set_spec_min(uint64_t frames);

/* Frame sieve: one segment of at least `bytes` after its first whole frame,
 * whose frame sizes vary, is discovered by data-parallel passes (every byte
 * position tested for a plausible client frame header chained 3 headers
 * deep, then pointer doubling from the first frame along exact successors)
 * instead of the serial header-to-header walk; frames the chain cannot reach
 * (unmasked, RSV bits, reserved opcodes) are walked exactly from there.
 * Tuning only (process-wide, default 8 MiB, 0 = default; $HVWS_SIEVE_MIN);
 * results never depend on it.  Returns the previous value. */
uint64_t hvws_set_sieve_min(uint64_t bytes);

/* What the frame sieve did in the last one-segment scan on ctx (NULL = the
 * calling thread's context; waits for that scan): out[0] = 0 not run or not
 * wanted (uniform sizes, short segment), 1 sieved, 2 more survivors than its
 * table held (walked instead); out[1] = survivors; out[2] = frames on the
 * chain; out[3] = segment offset where the exact walk resumed. */
int hvws_last_sieve(hvws_ctx* ctx, uint64_t out[4]);

/* Frame-sieve windows.  A long stream of large frames is sieved only over the
 * first `window_bytes` of every region of about `hops` mean-sized frames (the
 * mean from the context's last exact count of a one-segment scan); the chain's
 * link walks cross the rest of each region frame by frame, so the sieve reads
 * window / region of the bytes instead of all of them.  hops = 0 sieves every
 * position (the round-2 behaviour).  Process-wide tuning (default 320 and
 * 1 MiB + 16 KiB; $HVWS_EXPERIMENT sieve_hops, sieve_window; window 0 = default);
 * results never depend on it.  prev (may be NULL) receives the old values. */
void hvws_set_sieve_windows(uint64_t hops, uint64_t window_bytes, uint64_t prev[2]);

/* Window geometry of the last sieved scan on ctx, in 8 KiB tiles: out[0] =
 * region, out[1] = window (equal: every tile sieved; 0, 0: no sieve ran). */
int hvws_last_sieve_windows(hvws_ctx* ctx, uint64_t out[2]);

/* Verify after every scan that frame ends (pay_off + pay_len) never
 * decrease over the table -- the invariant the unmask tile index is built on
 * -- and fail the scan with HVWS_EINVAL otherwise.  Costs one device sync
 * per scan; for tests (process-wide; default off, or $HVWS_CHECK_TABLES=1).
 * Returns the previous setting. */
int hvws_set_table_checks(int on);

/* Speculative frame tables for large multi-segment batches.  SPEC: when the
 * last batch's per-segment record counts matched the uniform-stride
 * estimates, the next scan emits straight into the table at the estimated
 * offsets and the device checks it (one walk, no host round trip before
 * EMIT).  SLACK: otherwise (mixed sizes), one walk emits each segment's
 * records into its own region of a scratch table (at most 1.5 x the last
 * exact scan's largest segment count + 16), the device checks that every
 * segment fit and compacts the records to the exact offsets (and whether the
 * uniform estimates would have held: SPEC next time).  A failed check
 * re-scans exactly (COUNT, wait, EMIT).  mode -1 = that automatic choice
 * (default, or $HVWS_EXPERIMENT spec unset), 0 = never speculate, 1 = try SPEC first,
 * 2 = try SLACK first (tests).  Results never depend on it.  ctx NULL = the
 * calling thread's context.  Returns the previous mode. */
int hvws_set_speculation(hvws_ctx* ctx, int mode);

/* One-walk passes (SPEC, SLACK): mode -1 = adaptive (default: the grid-wide
 * k_verify pair and k_head<true> run only when the last check saw a segment
 * with >= spec_min predicted frames; otherwise k_head<false>, the offsets and
 * one walk that also records the carried-in frame), 0 = never, 1 = always.
 * Results never depend on it.  Returns the previous mode. */
int hvws_set_walk_verify(hvws_ctx* ctx, int mode);

/* How the last hvws_scan on ctx found its frames (tests, benchmarks). */
enum {
    HVWS_PATH_COUNT_EMIT = 0,       /* COUNT then EMIT, table sized by the record bound, no wait */
    HVWS_PATH_COUNT_READ_EMIT = 1,  /* COUNT, wait for the count, EMIT */
    HVWS_PATH_SINGLE = 2,           /* one segment: one walk into an estimated table */
    HVWS_PATH_SPEC = 3,             /* speculative table checked exact on the device */
    HVWS_PATH_SPEC_FAILED = 4,      /* speculation rejected by the check, then COUNT/EMIT */
    HVWS_PATH_SLACK = 5,            /* mixed sizes: one EMIT walk into per-segment regions, compacted on the device */
    HVWS_PATH_SLACK_FAILED = 6,     /* a segment outgrew its region, then COUNT/EMIT */
    HVWS_PATH_RUN = 7               /* step of small uniform frames: per-segment run descriptors, headers
                                       checked by the unmask itself, records built when read */
};
int hvws_last_scan_path(hvws_ctx* ctx);

/* RUN path for hvws_step / hvws_step_resident: a batch of many segments whose
 * last exact scan found each segment one run of equal frames (and frames of at
 * most 8 KiB) is discovered by k_head alone -- the carried-in frame and the
 * frame cut by the segment end exactly, the run in between as a hypothesis --
 * and the unmask parses every run header from the bytes it loads anyway,
 * checks it against the hypothesis and takes its key from it: no per-frame
 * records and no second pass over the header lines.  A repair pass queued on
 * the context stream right behind undoes and redoes exactly any segment whose
 * hypothesis failed, so work queued after the step sees the reference's bytes
 * either way; the next steps then scan exactly until a check sees uniform
 * frames again.  The frame records, counts and carry of a RUN step are built
 * (an exact scan of the unchanged headers) when hvws_get_* first asks: the
 * header bytes must stay as they were until then (hvws_step_resident).  An
 * hvws_unmask after a RUN step builds them first and XORs by that exact
 * table.  mode
 * -1 = automatic (default; $HVWS_RUN=0 turns it off), 0 = never, 1 = every
 * step batch of several segments, whatever the last scan saw (tests).  ctx
 * NULL = the calling thread's context.  Returns the previous mode. */
int hvws_set_run(hvws_ctx* ctx, int mode);
/* Segments of the last step that the RUN path's repair pass put back and
 * unmasked exactly (their hypothesis failed, or k_head saw they were not one
 * run); -1 if the last scan was not a RUN step.  Waits for the step. */
int64_t hvws_last_run_repairs(hvws_ctx* ctx);

/* Device span of a timed region: hvws_span_begin records a marker on each of
 * the context's compute streams, hvws_span_end records the end markers, waits
 * for them and returns (latest end - earliest begin) in ms.  For benchmarks:
 * the per-device time of a run of steps. */
int hvws_span_begin(hvws_ctx* ctx);
int hvws_span_end(hvws_ctx* ctx, float* ms);
/* Batches whose record bound (rx_len / 2 + 2 * nseg + 1) is at most
 * `records` are scanned COUNT -> EMIT with the table sized by that bound
 * (default 2^24); larger ones wait for a count (or speculate).  1 makes
 * every multi-segment batch take the large-batch path, 0 restores the
 * default.  Tuning/testing only; results never depend on it.  Returns the
 * previous bound. */
uint64_t hvws_set_fast_bound(hvws_ctx* ctx, uint64_t records);

/* STREAM-style in-place ceiling: d[i] ^= pattern over n bytes (16-B aligned). */
int hvws_stream_xor(hvws_ctx* ctx, uint8_t* d, uint64_t n, uint32_t pattern);

/* ---- transmit side, device resident ---------------------------------- */
/* Build n frames back to back into d_out, each byte-identical to
 * websocket_build_frame(frame, flags[i], mask + i, payload + pay_off[i],
 * len[i]): header (FIN/opcode, MASK bit, 7/16/64-bit length, key) followed by
 * the payload XOR-masked from phase 0 when flags[i] has WS_HAS_MASK.
 * d_mask[i] holds frame i's key with mask[0] in bits 0-7; d_mask may be NULL
 * only if no frame is masked (the reference would read uninitialised bytes).
 * d_out_off (n words, optional) receives each frame's offset in d_out.
 * *out_len = total bytes.  Synchronises once (after sizing/validating the
 * tables: a payload range outside [0, payload_len) or an output larger than
 * out_cap is HVWS_EINVAL and nothing is written); the build kernel itself is
 * asynchronous on the ctx stream.  d_out must be 16-byte aligned and must not
 * overlap d_payload. */
int hvws_build_frames(hvws_ctx* ctx, uint8_t* d_out, uint64_t out_cap, const uint8_t* d_payload,
                      uint64_t payload_len, const uint64_t* d_pay_off, const uint64_t* d_len,
                      const uint8_t* d_flags, const uint32_t* d_mask, uint64_t n, uint64_t* d_out_off,
                      uint64_t* out_len);
/* Device time (ms, HIP events on the ctx stream) of the last hvws_encode_keys
 * kernel, or of the last hvws_build_frames' device work after its size check
 * (tile index, source spans, k_build); the default build geometry's name. */
int hvws_last_kernel_ms(hvws_ctx* ctx, float* ms);
const char* hvws_build_kernel_name(void);
/* The k_build geometry the last hvws_build_frames on ctx ran: one-wave
 * workgroups of 4 KiB tiles, in a lean-LDS form for batches of small frames
 * (mean frame < 4 KiB), or $HVWS_EXPERIMENT build's.  Results never
 * depend on it. */
const char* hvws_last_build_kernel(hvws_ctx* ctx);
/* 1 when the last hvws_build_frames on ctx found a uniform layout (every frame
 * the same size and payload length, payload offsets a + k*b with b >= 0) and
 * built it without a tile index (each tile finds its frames from its
 * position); 0 otherwise.  Results never depend on it. */
int hvws_last_build_uniform(hvws_ctx* ctx);

/* ---- handshake, device resident --------------------------------------- */
/* Sec-WebSocket-Accept for n upgrade requests: accept + 32*i receives the 28
 * characters ws_encode_key (http/wsdef.c:11-20) writes for key i (the bytes
 * d_keys[key_off[i] .. + key_len[i]), no NUL inside), followed by 4 zero bytes
 * -- the callers' zeroed char[32] (http/server/HttpHandler.cpp:986).
 * d_accept must be 16-byte aligned.  Asynchronous on the ctx stream. */
int hvws_encode_keys(hvws_ctx* ctx, const char* d_keys, const uint64_t* d_key_off, const uint32_t* d_key_len,
                     uint64_t n, char* d_accept);

/* ---- host memory in, host memory out -------------------------------- */
/* Copies h_rx to the device, runs scan (+ unmask if `unmask`), copies the
 * bytes back in place and updates carry[].  Frames of the batch are then
 * available through hvws_get_frames(). */
int hvws_rx_batch(hvws_ctx* ctx, uint8_t* h_rx, uint64_t len, const hvws_segment* segs,
                  websocket_parser* carry, uint32_t nseg, int unmask);

/* Enable protocol validation classes (HVWS_V_*; 0 = off, the default) for
 * later batches on ctx (NULL = the calling thread's reference-API context).
 * Device API: a frame whose header violates an enabled class carries
 * HVWS_I_INVALID and the classes in its info.  Reference API: the library
 * rejects such a frame the way a failing on_frame_header callback would --
 * websocket_parser_execute / FeedRecvData return the index of the header's
 * last byte (< len), so HttpHandler::FeedRecvData reports ERR_PARSE and the
 * connection closes (http/server/HttpHandler.cpp:757-763); on_frame_header
 * is not called for it.  A header split across reads keeps its partial
 * validation state in the padding byte after websocket_parser.mask_offset.
 * Returns the previous classes. */
uint32_t hvws_set_validation(hvws_ctx* ctx, uint32_t classes);

/* Batches of at most `bytes` (default 64 MiB; each segment <= 1 MiB) take
 * the single-launch small-batch path inside hvws_rx_batch (and so inside
 * FeedRecvData / websocket_parser_execute); 0 restores the default, ~0
 * disables the path.  ctx NULL = the calling thread's context used by the
 * reference-API entry points.  Returns the previous limit.  Results are identical
 * either way; only latency differs. */
uint64_t hvws_set_small_batch_limit(hvws_ctx* ctx, uint64_t bytes);

/* Resident small-path worker.  The reference API's single calls -- FeedRecvData
 * and websocket_parser_execute on a read of <= 32 KiB, websocket_decode,
 * websocket_parser_decode and a masked websocket_build_frame of <= 32 KiB --
 * are served by one workgroup (k_door) that stays on the device between
 * calls and takes requests from a mailbox (in device memory written through
 * the PCIe BAR on large-BAR devices, else in pinned host memory): no kernel
 * launch per call.  It runs on a stream of its own (its own hardware queue)
 * and parks itself after $HVWS_DOOR_IDLE_US (default 5000) without a
 * request; the next call relaunches it.  Context teardown, thread exit and
 * process exit park it too.  on = 1 / 0 (off: each call launches k_small, or
 * the XOR kernel), -1 = default ($HVWS_DOOR, on unless set to 0).  ctx NULL = the
 * calling thread's context.  Returns the previous setting.  Results are
 * identical either way; only latency differs. */
int hvws_set_door(hvws_ctx* ctx, int on);
/* out = {worker launches, requests posted, requests the current worker
 * served, worker resident now} (tests, benchmarks). */
int hvws_door_stats(hvws_ctx* ctx, uint64_t out[4]);
/* Process-wide worker failures since the process started: out = {worker
 * streams that did not drain within 5 s (their context keeps the stream and
 * mailbox and never reuses them), requests a worker did not answer (that
 * context launches per call from then on)}.  Each is also reported on stderr
 * when it happens; both are 0 in a healthy process (the test session fails
 * otherwise).  At most $HVWS_DOOR_MAX (default 8) contexts per device hold a
 * worker stream at once; reads on further contexts launch per call. */
int hvws_door_health(uint64_t out[2]);
/* Idle time after which workers launched from now on park (microseconds;
 * 0 = the default, 5000).  Returns the previous value.  The runtime's frees
 * (hipFree, hipHostFree, hipHostUnregister) wait for every stream, a resident
 * worker's too: before each of its frees the library parks every worker on
 * that device, whichever thread owns it; a free outside this library waits
 * for the workers to park themselves (at most their idle time). */
uint64_t hvws_set_door_idle_us(uint64_t us);
/* Diagnostics for a process that seems stuck (bench.py's watchdog): writes
 * to fd the state of every context -- each resident worker's mailbox (seq,
 * done, alive, exited epoch) and the host's view of it, then
 * hipStreamQuery of every stream of the context (a query can itself block
 * behind a stuck runtime call; the memory state is written first). */
int hvws_debug_dump(int fd);
/* Diagnostics: a native backtrace of every thread of the process to fd
 * (SIGUSR2 to each thread in turn, backtrace_symbols_fd in the handler).
 * Returns the number of threads that answered within 200 ms each. */
int hvws_debug_backtraces(int fd);
/* out = {requests go through device memory written across the PCIe BAR (1)
 * or through pinned host memory (0), the context has a worker stream}. */
int hvws_door_info(hvws_ctx* ctx, uint64_t out[2]);
/* Diagnostics: 100 MHz device-clock stamps of the worker's last read request
 * -- seen, staged, walked, XORed, records written (before the release), and
 * the previous request's release.  Written only under $HVWS_EXPERIMENT
 * door_stamps=1 (each stamp costs the worker a clock round trip); else 0. */
int hvws_door_stamps(hvws_ctx* ctx, uint64_t out[12]);

/* Small batches whose segments are all <= 32 KiB (total <= 1 MiB; an event
 * loop's reads) are read by the device straight from pinned host memory, each
 * segment staged in LDS, with no H2D copy ahead of the launch (on = 1, the
 * default; $HVWS_SMALL_ZC=0 turns it off for new contexts).  ctx NULL = the
 * calling thread's context.  Returns the previous setting.  Results are
 * identical either way; only latency differs. */
int hvws_set_small_zero_copy(hvws_ctx* ctx, int on);

/* Registered pinned host memory: hvws_host_alloc'ed ranges are registered
 * automatically; hvws_host_register pins and registers caller memory (an
 * event loop's read buffers), hvws_host_unregister undoes it. */
int hvws_host_register(hvws_ctx* ctx, void* p, uint64_t bytes);
int hvws_host_unregister(hvws_ctx* ctx, void* p);

/* hvws_rx_batch over n separate reads that live in registered pinned memory
 * (no gather into a staging buffer, no copies: the kernel reads every read
 * where it is and unmasks it in place).  Each read is at most 32 KiB, the
 * total at most the small-batch limit (64 MiB by default), and reads must not
 * overlap.  Read i is segment i: hvws_get_segment_frames / hvws_get_frames
 * report its frames with hdr_off / pay_off relative to reads[i]; carry is
 * in/out per read.  HVWS_EINVAL (nothing done) if a read is not registered,
 * or if the context's small-batch path is off (hvws_set_small_batch_limit ~0). */
int hvws_rx_reads(hvws_ctx* ctx, char* const* reads, const uint64_t* lens, websocket_parser* carry, uint32_t n,
                  int unmask);

/* Host-inclusive streaming unmask of a large pinned host buffer holding
 * frames back to back from one stream: chunked H2D -> scan -> unmask -> D2H,
 * double-buffered over two streams.  carry is in/out. */
int hvws_pipeline(hvws_ctx* ctx, uint8_t* h_rx, uint64_t len, uint64_t chunk,
                  websocket_parser* carry);

/* ---- WebSocketParser handle for FFI ------------------------------------ */
typedef void (*hvws_msg_cb)(void* user, int opcode, const char* data, size_t len);
void* hvws_wsp_new(void);
void  hvws_wsp_free(void* h);
void  hvws_wsp_set_sink(void* h, hvws_msg_cb cb, void* user);
int   hvws_wsp_feed(void* h, const char* data, size_t len);
void  hvws_wsp_state(void* h, uint64_t out[8]);
/* n handles fed in one GPU round trip (see hvws_feed_many in WebSocketParser.h) */
int   hvws_wsp_feed_many(void* const* handles, const char* const* data, const size_t* len, int n, int* rets);

/* Pipelined event-loop feed.  A feeder owns a
 * worker thread with its own context, stream and pinned stage.  Each submit
 * starts the device half of this poll iteration's reads (gather, one GPU round
 * trip, unmasked bytes written back in place) on the worker and, meanwhile,
 * replays the PREVIOUS submission's message logic and onMessage callbacks on
 * the calling thread.  Effects per parser are those of hvws_feed_many, one
 * submission late: the callbacks and rets[] of submission k arrive during
 * submit k+1 (or flush).  The caller keeps submission k's buffers and its
 * rets array alive and untouched until then.  Submitting 0 reads = flush.
 * A parser whose feed returned short must be closed (as libhv does); its
 * results already in flight are then undefined.  Submit and flush are not
 * callable from inside the feeder's own callbacks (they return -1), nor may a
 * submission hold a parser that a replay still to come will write (see
 * hvws_feed_many; -1).  new() binds the calling thread's device; free()
 * flushes.  free() from inside one of the feeder's own callbacks is deferred:
 * the feeder is freed when the submit / flush that replays it returns (the
 * rest of that run's callbacks still run; runs of that submission not yet
 * started are dropped and its return value counts the reads taken). */
typedef struct hvws_feeder hvws_feeder;
hvws_feeder* hvws_feeder_new(void);
void hvws_feeder_free(hvws_feeder* f);
int  hvws_feeder_flush(hvws_feeder* f);
/* hvws_feeder_submit over hvws_wsp_* handles (C++: hvws_feeder_submit in WebSocketParser.h) */
int  hvws_wsp_feeder_submit(hvws_feeder* f, void* const* handles, const char* const* data, const size_t* len, int n,
                            int* rets);

/* Device used by the reference-API entry points on the calling thread
 * (default: $HVWS_DEVICE or 0). */
int hvws_set_thread_device(int device);
/* Free the calling thread's reference-API context (streams, device tables,
 * pinned staging); call at event-loop thread exit.  The next call on the
 * thread creates a fresh one. */
void hvws_thread_release(void);

#ifdef __cplusplus
}
#endif
#endif /* HVWS_H */

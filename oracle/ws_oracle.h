/*
 * ws_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of libhv's WebSocket receive path, used as the parity
 * checker for the HIP implementation in libhv_amd/.  Nothing in the product
 * library links, loads or calls this code; only tests/, bench.py's
 * cpu_baseline leg and __graft_entry__.smoke() do.
 *
 * Pinning: every function here is checked (tests/test_oracle.py) against
 *   (1) RFC 6455 sec. 5.7 known answers,
 *   (2) golden vectors under tests/golden/ produced by the reference's own
 *       http/websocket_parser.c + http/wsdef.c compiled from /root/reference
 *       by oracle/Makefile into oracle/_ref/ (see tests/golden/make_golden.py),
 *   (3) the reference library itself whenever oracle/_ref/ is present.
 * The message layer (WebSocketParser.cpp) cannot be compiled here (it pulls
 * the generated hconfig.h through base/hdef.h -> base/hplatform.h), so it is
 * restated in ws_msg.c and driven on top of the compiled reference frame
 * parser; its quirks are pinned by the known answers recorded in SURVEY.md
 * Appendix A (Q5, Q6, Q7, Q10).
 */
#ifndef HVWS_ORACLE_H
#define HVWS_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Same layout as `struct websocket_parser` (http/websocket_parser.h:50-62):
 * 48 bytes on x86-64, flags@4 mask@8 mask_offset@12 length@16 require@24
 * offset@32 data@40. */
typedef struct ows_parser {
    uint32_t state;
    uint32_t flags;
    char     mask[4];
    uint8_t  mask_offset;
    size_t   length;
    size_t   require;
    size_t   offset;
    void*    data;
} ows_parser;

typedef int (*ows_cb)(ows_parser*);
typedef int (*ows_data_cb)(ows_parser*, const char* at, size_t length);

/* http/websocket_parser.h:64-68 */
typedef struct ows_settings {
    ows_cb      on_frame_header;
    ows_data_cb on_frame_body;
    ows_cb      on_frame_end;
} ows_settings;

enum { OWS_S_START = 0, OWS_S_HEAD, OWS_S_LENGTH, OWS_S_MASK, OWS_S_BODY };
enum { OWS_OP_MASK = 0x0F, OWS_FIN = 0x10, OWS_HAS_MASK = 0x20 };

void   ows_parser_init(ows_parser* p);
void   ows_settings_init(ows_settings* s);
size_t ows_execute(ows_parser* p, const ows_settings* s, const char* data, size_t len);
void   ows_parser_decode(char* dst, const char* src, size_t len, ows_parser* p);
uint8_t ows_decode(char* dst, const char* src, size_t len, const char mask[4], uint8_t mask_offset);
size_t ows_calc_frame_size(uint32_t flags, size_t data_len);
size_t ows_build_frame(char* frame, uint32_t flags, const char mask[4], const char* data, size_t data_len);
int    ows_ws_calc_frame_size(int data_len, int has_mask);
int    ows_ws_build_frame(char* out, const char* data, int data_len, const char mask[4],
                          int has_mask, int opcode, int fin);

/* Instrumentation for record extraction: byte index (within the current
 * execute() call) of the byte being processed when the last callback fired,
 * and the index at which the current frame's first header byte was seen
 * (-1 if that happened in an earlier call). */
extern __thread int64_t ows_cb_pos;
extern __thread int64_t ows_frame_start;

/* ---------------------------------------------------------------------
 * Frame records: the per-frame view the GPU scan kernel produces for one
 * segment (one execute() call over `len` bytes starting from a carry-in
 * parser state).  Field meanings mirror libhv_amd/include/hvws.h.
 * ------------------------------------------------------------------- */
typedef struct ows_frame {
    int64_t  hdr_off;     /* first header byte within segment, -1 if earlier */
    uint64_t pay_off;     /* first payload byte of this frame in the segment */
    uint64_t pay_len;     /* payload bytes of this frame inside the segment */
    uint64_t length;      /* parser->length (full payload length)           */
    uint32_t key;         /* mask bytes little-endian (0 if not masked)      */
    uint32_t info;        /* flags | phase<<8 | HDR/BODY/END/START bits      */
} ows_frame;

enum {
    OWS_I_HDR = 1u << 10, OWS_I_BODY = 1u << 11, OWS_I_END = 1u << 12, OWS_I_START = 1u << 13
};

/* Walk one segment like WebSocketParser::FeedRecvData would (header parse +
 * in-place unmask of masked body spans), recording frames.  `buf` is unmasked
 * in place.  Returns the number of frame records (<= cap written).
 * `started_out` (may be NULL) receives 1 if the carry-out frame's first
 * header byte was inside this segment. */
size_t ows_scan_segment(ows_parser* st, uint8_t* buf, size_t len,
                        ows_frame* out, size_t cap, int* started_out);

/* ---------------------------------------------------------------------
 * Synthetic masked-frame batches.  Frame i's plaintext
 * byte j is a pure function of (seed, i, j) so the GPU generator and this
 * oracle produce identical bytes independently.
 * ------------------------------------------------------------------- */
uint64_t ows_mix64(uint64_t x);
uint8_t  ows_plain_byte(uint64_t seed, uint64_t frame, uint64_t j, int text);
/* Builds frames back to back (websocket_build_frame layout) at frame_off[i]. */
void ows_synth_fill(uint8_t* buf, size_t buf_len, uint64_t seed, size_t nframes,
                    const uint64_t* frame_off, const uint8_t* flags, const uint32_t* mask,
                    const uint64_t* length, const uint8_t* text);
/* Expected plaintext of frame i into out (length[i] bytes). */
void ows_synth_plain(uint8_t* out, uint64_t seed, uint64_t frame, uint64_t length, int text);

/* FNV-1a 64 over bytes (cheap checksum for logs). */
uint64_t ows_fnv1a(const uint8_t* p, size_t n, uint64_t h);

#ifdef __cplusplus
}
#endif
#endif

/*
 * hvws_synth.h -- synthetic masked-frame batches on the device (bench/test
 * data).  Not part of the receive path.
 *
 * Frame i is laid out exactly as the reference's websocket_build_frame
 * (http/websocket_parser.c:207-256) writes it: header at frame_off[i],
 * payload masked with phase 0.  Its plaintext byte j is a pure function of
 * (seed, i, j) -- see oracle/ws_oracle.c ows_plain_byte -- so the device and
 * the CPU oracle build identical batches independently.
 */
#ifndef HVWS_SYNTH_H
#define HVWS_SYNTH_H

#include <stdint.h>

#include "hvws.h"

#ifdef __cplusplus
extern "C" {
#endif

enum {
    HVWS_SYNTH_WRITE = 0,        /* write masked frames                       */
    HVWS_SYNTH_VERIFY_MASKED = 1,/* count bytes != masked frames              */
    HVWS_SYNTH_VERIFY_PLAIN = 2  /* count bytes != header + plaintext payload  */
};

/* All plan arrays are device pointers of nframes entries (text may be NULL).
 * For the VERIFY modes *mismatches receives the differing-byte count
 * (synchronises). */
int hvws_synth(hvws_ctx* ctx, uint8_t* d_buf, uint64_t buf_len, uint64_t seed, uint64_t nframes,
               const uint64_t* d_frame_off, const uint8_t* d_flags, const uint32_t* d_mask,
               const uint64_t* d_length, const uint8_t* d_text, int mode, uint64_t* mismatches);

/* Order-independent digest: sum over 8-byte words w_k (zero padded) of
 * mix64(w_k ^ (k * 0xD1B54A32D192ED03)).  Synchronises. */
int hvws_digest(hvws_ctx* ctx, const uint8_t* d_buf, uint64_t len, uint64_t* out);

#ifdef __cplusplus
}
#endif
#endif

// websocket_parser.cpp -- the reference frame-layer C ABI
// (http/websocket_parser.h:70-90) on top of the MI355X engine.
//
// websocket_parser_execute runs frame discovery + header parse on the GPU
// (k_scan over one segment continuing from *parser), then replays the
// reference's callbacks on the host in the reference's order with the
// parser fields the reference would show at each one, including the
// early-return protocol (a callback returning non-zero stops the parse and
// execute returns the index of the byte under the reference's cursor,
// http/websocket_parser.c:14-32).  The decode/encode helpers run the XOR on
// the GPU.  There is no CPU fallback: without a device these abort().
#include <stddef.h>
#include <string.h>

#include <vector>

#include "hvws.h"
#include "hvws_internal.h"

namespace hvws {
[[noreturn]] void fatal(const char* what);
void gpu_xor_host(char* dst, const char* src, size_t n, uint32_t key, uint32_t phase);
void gpu_feed(char* buf, size_t len, const websocket_parser& carry, bool unmask, std::vector<hvws_frame>& frames,
              websocket_parser& carry_out, int& started);
}  // namespace hvws

using namespace hvws;

extern "C" {

// http/websocket_parser.c:42-47
void websocket_parser_init(websocket_parser* parser) {
    void* keep = parser->data;
    memset(parser, 0, sizeof(*parser));
    parser->data = keep;
    parser->state = S_START;
}

// http/websocket_parser.c:49-51
void websocket_parser_settings_init(websocket_parser_settings* settings) {
    memset(settings, 0, sizeof(*settings));
}

size_t websocket_parser_execute(websocket_parser* parser, const websocket_parser_settings* settings,
                                const char* data, size_t len) {
    if (len == 0) return 0;
    std::vector<hvws_frame> frames;
    websocket_parser out;
    int started = 0;
    // The raw frame layer does not unmask (only WebSocketParser's callback
    // does), so the caller's bytes are read, never written.
    gpu_feed(const_cast<char*>(data), len, *parser, false, frames, out, started);

    websocket_parser* p = parser;
    for (const hvws_frame& f : frames) {
        const uint32_t fl = f.info & HVWS_I_FLAGS;
        const uint64_t rel_pay = f.pay_off;   // one segment at offset 0
        if (f.info & HVWS_I_START) {          // s_start: :60-71
            p->offset = 0;
            p->mask_offset = 0;
        }
        if (f.info & HVWS_I_HDR) {
            // Fields as the reference leaves them when on_frame_header fires
            // (:72-142): flags/length final, key present if masked, state
            // already switched to body (or back to start for empty frames).
            p->flags = (websocket_flags)fl;
            p->length = f.length;
            if (fl & WS_HAS_MASK) memcpy(p->mask, &f.key, 4);
            p->offset = 0;
            if (f.length) {
                p->state = S_BODY;
                p->require = f.length;
            } else {
                p->state = S_START;
                p->require = 0;
            }
            const size_t at = (size_t)rel_pay - 1;   // last header byte
            // hvws_set_validation: reject as a failing on_frame_header would
            if (f.info & HVWS_I_INVALID) return at;
            if (settings->on_frame_header && settings->on_frame_header(p) != 0) return at;
            if (!f.length && (f.info & HVWS_I_END)) {
                if (settings->on_frame_end && settings->on_frame_end(p) != 0) return at;
                continue;
            }
        }
        if (f.info & HVWS_I_BODY) {
            // :143-157 -- require still counts this span while the callback runs
            if (!(f.info & HVWS_I_HDR)) {
                p->flags = (websocket_flags)fl;
                p->length = f.length;
            }
            p->state = S_BODY;
            const size_t at = (size_t)rel_pay;
            if (settings->on_frame_body &&
                settings->on_frame_body(p, data + rel_pay, (size_t)f.pay_len) != 0)
                return at;
            p->require -= f.pay_len;
        }
        if (f.info & HVWS_I_END) {
            p->state = S_START;
            p->require = 0;
            // cursor: last body byte; the skipped byte of the (unreachable)
            // empty-body state otherwise
            const size_t at = (f.info & HVWS_I_BODY) ? (size_t)(rel_pay + f.pay_len) - 1 : (size_t)rel_pay;
            if (settings->on_frame_end && settings->on_frame_end(p) != 0) return at;
        }
    }
    // Final state: the engine's carry-out, except mask_offset, which in the
    // raw frame layer only the user's callbacks move (via
    // websocket_parser_decode); a frame begun here with no callback yet was
    // reset to 0 by s_start.
    const uint8_t mo = p->mask_offset;
    bool pending_has_record = false;
    if (out.state != S_START && !frames.empty()) {
        const hvws_frame& last = frames.back();
        pending_has_record = !(last.info & HVWS_I_END);
    }
    void* keep = p->data;
    p->state = out.state;
    p->flags = out.flags;
    memcpy(p->mask, out.mask, 4);
    p->length = out.length;
    p->require = out.require;
    p->offset = out.offset;
    p->data = keep;
    // partial-header validation state (padding byte after mask_offset; see hvws_set_validation)
    reinterpret_cast<uint8_t*>(p)[kViolByte] = reinterpret_cast<const uint8_t*>(&out)[kViolByte];
    if (out.state != S_START && started && !pending_has_record) p->mask_offset = 0;
    else p->mask_offset = mo;
    return len;
}

// http/websocket_parser.c:173-180
void websocket_parser_decode(char* dst, const char* src, size_t len, websocket_parser* parser) {
    uint32_t key;
    memcpy(&key, parser->mask, 4);
    gpu_xor_host(dst, src, len, key, parser->mask_offset & 3u);
    parser->mask_offset = (uint8_t)((len + parser->mask_offset) % 4);
}

// http/websocket_parser.c:182-189
uint8_t websocket_decode(char* dst, const char* src, size_t len, const char mask[4], uint8_t mask_offset) {
    uint32_t key;
    memcpy(&key, mask, 4);
    gpu_xor_host(dst, src, len, key, mask_offset & 3u);
    return (uint8_t)((len + mask_offset) % 4);
}

// http/websocket_parser.c:191-205
size_t websocket_calc_frame_size(websocket_flags flags, size_t data_len) {
    size_t ext = data_len < 126 ? 0 : (data_len <= 0xFFFF ? 2 : 8);
    return data_len + 2 + ext + ((flags & WS_HAS_MASK) ? 4 : 0);
}

// http/websocket_parser.c:207-256: header on the host, payload masked on the GPU.
size_t websocket_build_frame(char* frame, websocket_flags flags, const char mask[4], const char* data,
                             size_t data_len) {
    unsigned char* f = (unsigned char*)frame;
    size_t at;
    f[0] = (unsigned char)(((flags & WS_FIN) ? 0x80u : 0u) | (flags & WS_OP_MASK));
    f[1] = (flags & WS_HAS_MASK) ? 0x80u : 0u;
    if (data_len < 126) {
        f[1] |= (unsigned char)data_len;
        at = 2;
    } else if (data_len <= 0xFFFF) {
        f[1] |= 126;
        f[2] = (unsigned char)(data_len >> 8);
        f[3] = (unsigned char)(data_len & 0xFF);
        at = 4;
    } else {
        f[1] |= 127;
        for (int k = 0; k < 8; ++k) f[2 + k] = (unsigned char)((uint64_t)data_len >> (56 - 8 * k));
        at = 10;
    }
    if (flags & WS_HAS_MASK) {
        if (mask) memcpy(f + at, mask, 4);   // NULL: whatever bytes are there act as key
        uint32_t key;
        memcpy(&key, f + at, 4);
        at += 4;
        gpu_xor_host(frame + at, data, data_len, key, 0);
    } else if (data_len) {
        memcpy(f + at, data, data_len);
    }
    return at + data_len;
}

}  // extern "C"

// WebSocketParser.cpp -- drop-in for the reference message reassembler
// (http/WebSocketParser.cpp:8-75) on the MI355X engine.
//
// FeedRecvData ships the chunk to the device, runs k_scan (frame discovery +
// header parse) and k_unmask (XOR) there, copies the unmasked bytes back into
// the caller's buffer (the reference also rewrites it in place, Q10), and
// replays the reference's per-frame message logic on the host:
//   header: latch opcode unless CONTINUE, reserve, clear on BEGIN/FIN  (:8-26)
//   body:   append the (now unmasked) span                            (:28-37)
//   end:    on FIN, onMessage(opcode, message)                        (:39-50)
#include "WebSocketParser.h"

#include <stdlib.h>
#include <string.h>

#include <vector>

#include "hvws.h"
#include "hvws_internal.h"

namespace hvws {
[[noreturn]] void fatal(const char* what);
void gpu_feed(char* buf, size_t len, const websocket_parser& carry, bool unmask, std::vector<hvws_frame>& frames,
              websocket_parser& carry_out, int& started);
}  // namespace hvws

namespace {
const int kMaxReserve = 1 << 24;   // MAX_PAYLOAD_LENGTH, reference WebSocketParser.cpp:6
}

WebSocketParser::WebSocketParser() {
    parser = (websocket_parser*)malloc(sizeof(websocket_parser));
    if (!parser) hvws::fatal("out of memory");
    memset(parser, 0, sizeof(*parser));
    websocket_parser_init(parser);
    parser->data = this;
    state = WS_FRAME_BEGIN;
    opcode = WS_OP_CLOSE;   // a lone CONTINUE first reports CLOSE (Q6)
}

WebSocketParser::~WebSocketParser() {
    if (parser) {
        free(parser);
        parser = NULL;
    }
}

int WebSocketParser::FeedRecvData(const char* data, size_t len) {
    if (len == 0) return 0;
    std::vector<hvws_frame> frames;
    websocket_parser out;
    int started = 0;
    char* buf = const_cast<char*>(data);   // unmasked in place, like the reference
    hvws::gpu_feed(buf, len, *parser, true, frames, out, started);

    for (const hvws_frame& f : frames) {
        const uint32_t fl = f.info & HVWS_I_FLAGS;
        parser->flags = (websocket_flags)fl;
        parser->length = f.length;
        if (f.info & HVWS_I_HDR) {
            const int op = (int)(fl & WS_OP_MASK);
            if (op != WS_OP_CONTINUE) opcode = op;
            const int length = (int)f.length;   // int truncation, as the reference (Q11)
            const int want = length + 1 < kMaxReserve ? length + 1 : kMaxReserve;
            // The reference compares int with size_t here; a negative `want`
            // makes it call reserve(huge) and throw.  Skip the reserve instead.
            if (want >= 0 && (size_t)want > message.capacity()) message.reserve((size_t)want);
            if (state == WS_FRAME_BEGIN || state == WS_FRAME_FIN) message.clear();
            state = WS_FRAME_HEADER;
        }
        if (f.info & HVWS_I_BODY) {
            state = WS_FRAME_BODY;
            message.append(buf + f.pay_off, (size_t)f.pay_len);
        }
        if (f.info & HVWS_I_END) {
            state = WS_FRAME_END;
            if (fl & WS_FIN) {
                state = WS_FRAME_FIN;
                if (onMessage) onMessage(opcode, message);
            }
        }
    }
    void* keep = parser->data;
    *parser = out;
    parser->data = keep;
    return (int)len;
}

// ---------------------------------------------------------------- C handle
namespace {
struct wsp_handle {
    WebSocketParser p;
    hvws_msg_cb cb = nullptr;
    void* user = nullptr;
};
}  // namespace

extern "C" {

void* hvws_wsp_new(void) { return new wsp_handle(); }

void hvws_wsp_free(void* h) { delete (wsp_handle*)h; }

void hvws_wsp_set_sink(void* h, hvws_msg_cb cb, void* user) {
    wsp_handle* w = (wsp_handle*)h;
    w->cb = cb;
    w->user = user;
    if (cb)
        w->p.onMessage = [w](int op, const std::string& msg) { w->cb(w->user, op, msg.data(), msg.size()); };
    else
        w->p.onMessage = nullptr;
}

int hvws_wsp_feed(void* h, const char* data, size_t len) { return ((wsp_handle*)h)->p.FeedRecvData(data, len); }

void hvws_wsp_state(void* h, uint64_t out[8]) {
    wsp_handle* w = (wsp_handle*)h;
    websocket_parser* p = w->p.parser;
    uint32_t m;
    memcpy(&m, p->mask, 4);
    out[0] = p->state;
    out[1] = (uint64_t)p->flags;
    out[2] = m;
    out[3] = p->mask_offset;
    out[4] = p->length;
    out[5] = p->require;
    out[6] = p->offset;
    out[7] = (uint64_t)w->p.state | ((uint64_t)(uint32_t)w->p.opcode << 32);
}

}  // extern "C"

// TEST INFRASTRUCTURE ONLY (tests/test_abi.py::test_builds_against_reference_headers).
//
// libhv's own code includes libhv's own headers.  This translation unit is
// compiled twice -- once against the reference's headers where they lie
// (/root/reference/http/{WebSocketParser.h, websocket_parser.h, wsdef.h} +
// hexport.h), once against include/ -- and both builds are linked against
// libhv_amd/libhvws.so with no undefined symbol allowed.  So:
//   * every declaration a libhv caller sees resolves to a symbol of the
//     library (C names, and the C++ mangled names of the WebSocketParser
//     members with the reference's own parameter types);
//   * struct websocket_parser, websocket_parser_settings and class
//     WebSocketParser have the same size and member offsets under both
//     headers (the same static_asserts pass in both builds);
//   * the host-only entry points (no device needed) give the same answers
//     under both: the test compares the two programs' output, and that with
//     the reference library's.
#include <stddef.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include "WebSocketParser.h"
#include "websocket_parser.h"
#include "wsdef.h"

// x86-64 layout probed in SURVEY.md sec. 8(a) rows a1, a8
static_assert(sizeof(websocket_parser) == 48, "websocket_parser size");
static_assert(offsetof(websocket_parser, state) == 0, "state");
static_assert(offsetof(websocket_parser, flags) == 4, "flags");
static_assert(offsetof(websocket_parser, mask) == 8, "mask");
static_assert(offsetof(websocket_parser, mask_offset) == 12, "mask_offset");
static_assert(offsetof(websocket_parser, length) == 16, "length");
static_assert(offsetof(websocket_parser, require) == 24, "require");
static_assert(offsetof(websocket_parser, offset) == 32, "offset");
static_assert(offsetof(websocket_parser, data) == 40, "data");
static_assert(sizeof(websocket_parser_settings) == 24, "settings size");
static_assert(offsetof(websocket_parser_settings, on_frame_header) == 0, "on_frame_header");
static_assert(offsetof(websocket_parser_settings, on_frame_body) == 8, "on_frame_body");
static_assert(offsetof(websocket_parser_settings, on_frame_end) == 16, "on_frame_end");
static_assert(sizeof(websocket_flags) == 4, "websocket_flags");
static_assert(WS_OP_CONTINUE == 0 && WS_OP_TEXT == 1 && WS_OP_BINARY == 2 && WS_OP_CLOSE == 8 && WS_OP_PING == 9 &&
                  WS_OP_PONG == 10 && WS_FIN == 0x10 && WS_HAS_MASK == 0x20 && WS_OP_MASK == 0xF,
              "flag values");
static_assert(WS_OPCODE_TEXT == 1 && WS_OPCODE_PONG == 0xA, "ws_opcode values");

// WebSocketParser is not standard-layout (std::string, std::function);
// offsetof on it is conditionally supported and GCC gives the real offsets
// (built with -Wno-invalid-offsetof).
static_assert(sizeof(WebSocketParser) == 80, "WebSocketParser size");
static_assert(offsetof(WebSocketParser, parser) == 0, "parser");
static_assert(offsetof(WebSocketParser, state) == 8, "state");
static_assert(offsetof(WebSocketParser, opcode) == 12, "opcode");
static_assert(offsetof(WebSocketParser, message) == 16, "message");
static_assert(offsetof(WebSocketParser, onMessage) == 48, "onMessage");

// Every entry point, by address: the link must resolve each one.
typedef void (*any_fn)();
static volatile any_fn g_fns[] = {
    (any_fn)&websocket_parser_init,   (any_fn)&websocket_parser_settings_init, (any_fn)&websocket_parser_execute,
    (any_fn)&websocket_parser_decode, (any_fn)&websocket_decode,                (any_fn)&websocket_calc_frame_size,
    (any_fn)&websocket_build_frame,   (any_fn)&ws_encode_key,                   (any_fn)&ws_calc_frame_size,
    (any_fn)&ws_build_frame,
};
static int (WebSocketParser::*volatile g_feed)(const char*, size_t) = &WebSocketParser::FeedRecvData;

int main(int argc, char** argv) {
    (void)argv;
    if (argc > 99) {   // never taken: makes the constructor / destructor symbols part of the link
        WebSocketParser* p = new WebSocketParser();
        (p->*g_feed)("", 0);
        delete p;
    }
    // host-only entry points
    websocket_parser p;
    memset(&p, 0x5A, sizeof(p));
    void* keep = p.data;
    websocket_parser_init(&p);
    printf("init %u %d %u %zu %zu %zu %d\n", p.state, (int)p.flags, (unsigned)p.mask_offset, p.length, p.require,
           p.offset, p.data == keep);
    websocket_parser_settings st;
    memset(&st, 0x5A, sizeof(st));
    websocket_parser_settings_init(&st);
    printf("settings %d %d %d\n", st.on_frame_header == NULL, st.on_frame_body == NULL, st.on_frame_end == NULL);
    const size_t lens[] = {0, 1, 125, 126, 127, 65535, 65536, 1u << 20, ((size_t)1 << 32) + 7};
    const int fls[] = {WS_OP_TEXT | WS_FIN, WS_OP_BINARY | WS_FIN | WS_HAS_MASK, WS_OP_PING | WS_HAS_MASK, 0};
    for (size_t l : lens)
        for (int f : fls) printf("calc %zu %d %zu\n", l, f, websocket_calc_frame_size((websocket_flags)f, l));
    const int ilens[] = {0, 1, 125, 126, 65535, 65536, 1 << 20};
    for (int l : ilens) printf("wscalc %d %d %d\n", l, ws_calc_frame_size(l, false), ws_calc_frame_size(l, true));
    printf("sizes %zu %zu %zu\n", sizeof(websocket_parser), sizeof(websocket_parser_settings), sizeof(WebSocketParser));
    return 0;
}

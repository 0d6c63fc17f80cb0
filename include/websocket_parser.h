/*
 * websocket_parser.h -- drop-in C ABI of libhv's WebSocket frame layer,
 * implemented by libhv_amd/libhvws.so on MI355X (gfx950).
 *
 * Every declaration replaces the same-named one in the reference header
 * http/websocket_parser.h (ithewei/libhv); the struct layout is identical so
 * http/WebSocketParser.cpp, http/server/HttpHandler.cpp and
 * http/client/WebSocketClient.cpp link against this library unchanged.
 *
 *   websocket_parser_init            <- http/websocket_parser.h:70 (.c:42-47)
 *   websocket_parser_settings_init   <- http/websocket_parser.h:71 (.c:49-51)
 *   websocket_parser_execute         <- http/websocket_parser.h:72-77 (.c:53-171)
 *   websocket_parser_decode          <- http/websocket_parser.h:80 (.c:173-180)
 *   websocket_decode / _encode       <- http/websocket_parser.h:83-84 (.c:182-189)
 *   websocket_calc_frame_size        <- http/websocket_parser.h:87 (.c:191-205)
 *   websocket_build_frame            <- http/websocket_parser.h:90 (.c:207-256)
 *
 * Behaviour is the reference's, byte for byte, including its quirks (see
 * SURVEY.md Appendix A); the work is done by HIP kernels (frame discovery +
 * header parse, XOR unmask) on the calling thread's device context.  With no
 * usable GPU these entry points print a diagnostic and abort(): there is no
 * CPU fallback.
 */
#ifndef HVWS_WEBSOCKET_PARSER_H
#define HVWS_WEBSOCKET_PARSER_H

#include <stddef.h>
#include <stdint.h>
#include <sys/types.h>

#ifdef __cplusplus
extern "C" {
#endif

#define WEBSOCKET_UUID "258EAFA5-E914-47DA-95CA-C5AB0DC85B11"

/* opcodes and marks, http/websocket_parser.h:30-45 */
typedef enum websocket_flags {
    WS_OP_CONTINUE = 0x0,
    WS_OP_TEXT     = 0x1,
    WS_OP_BINARY   = 0x2,
    WS_OP_CLOSE    = 0x8,
    WS_OP_PING     = 0x9,
    WS_OP_PONG     = 0xA,
    WS_FINAL_FRAME = 0x10,
    WS_HAS_MASK    = 0x20
} websocket_flags;

#define WS_OP_MASK 0xF
#define WS_FIN     WS_FINAL_FRAME

typedef struct websocket_parser websocket_parser;
typedef struct websocket_parser_settings websocket_parser_settings;

typedef int (*websocket_data_cb)(websocket_parser*, const char* at, size_t length);
typedef int (*websocket_cb)(websocket_parser*);

/* Streaming parser state, one per connection (http/websocket_parser.h:50-62).
 * This is also the carry state the GPU batch API (hvws.h) consumes/produces. */
struct websocket_parser {
    uint32_t        state;
    websocket_flags flags;
    char            mask[4];
    uint8_t         mask_offset;
    size_t          length;
    size_t          require;
    size_t          offset;
    void*           data;
};

struct websocket_parser_settings {
    websocket_cb      on_frame_header;
    websocket_data_cb on_frame_body;
    websocket_cb      on_frame_end;
};

void   websocket_parser_init(websocket_parser* parser);
void   websocket_parser_settings_init(websocket_parser_settings* settings);
size_t websocket_parser_execute(websocket_parser* parser, const websocket_parser_settings* settings,
                                const char* data, size_t len);
void    websocket_parser_decode(char* dst, const char* src, size_t len, websocket_parser* parser);
uint8_t websocket_decode(char* dst, const char* src, size_t len, const char mask[4], uint8_t mask_offset);
#define websocket_encode(dst, src, len, mask, mask_offset) websocket_decode(dst, src, len, mask, mask_offset)
size_t websocket_calc_frame_size(websocket_flags flags, size_t data_len);
size_t websocket_build_frame(char* frame, websocket_flags flags, const char mask[4], const char* data,
                             size_t data_len);

#define websocket_parser_get_opcode(p) ((p)->flags & WS_OP_MASK)
#define websocket_parser_has_mask(p)   ((p)->flags & WS_HAS_MASK)
#define websocket_parser_has_final(p)  ((p)->flags & WS_FIN)

#ifdef __cplusplus
}
#endif
#endif /* HVWS_WEBSOCKET_PARSER_H */

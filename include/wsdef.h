/*
 * wsdef.h -- drop-in for libhv's installed WebSocket helper header
 * (reference http/wsdef.h:1-89, http/wsdef.c:11-46), served by libhvws.so.
 *
 *   ws_encode_key         <- http/wsdef.h:48 / wsdef.c:11-20 (SHA-1 + base64, host)
 *   ws_calc_frame_size    <- http/wsdef.h:51 / wsdef.c:23-34
 *   ws_build_frame        <- http/wsdef.h:53-60 / wsdef.c:36-46 (payload masked on the GPU)
 *   ws_client_build_frame <- http/wsdef.h:62-77 (inline)
 *   ws_server_build_frame <- http/wsdef.h:79-87 (inline)
 */
#ifndef HVWS_WSDEF_H
#define HVWS_WSDEF_H

#include <stdbool.h>
#include <stdlib.h>

#define SEC_WEBSOCKET_VERSION    "Sec-WebSocket-Version"
#define SEC_WEBSOCKET_KEY        "Sec-WebSocket-Key"
#define SEC_WEBSOCKET_ACCEPT     "Sec-WebSocket-Accept"
#define SEC_WEBSOCKET_PROTOCOL   "Sec-WebSocket-Protocol"
#define SEC_WEBSOCKET_EXTENSIONS "Sec-WebSocket-Extensions"

#define WS_SERVER_MIN_FRAME_SIZE 2
#define WS_SERVER_PING_FRAME     "\211\0"
#define WS_SERVER_PONG_FRAME     "\212\0"
#define WS_CLIENT_MIN_FRAME_SIZE 6
#define WS_CLIENT_PING_FRAME     "\211\200WSWS"
#define WS_CLIENT_PONG_FRAME     "\212\200WSWS"

enum ws_session_type { WS_CLIENT, WS_SERVER };

enum ws_opcode {
    WS_OPCODE_CONTINUE = 0x0,
    WS_OPCODE_TEXT     = 0x1,
    WS_OPCODE_BINARY   = 0x2,
    WS_OPCODE_CLOSE    = 0x8,
    WS_OPCODE_PING     = 0x9,
    WS_OPCODE_PONG     = 0xA,
};

#ifdef __cplusplus
extern "C" {
#define HVWS_DEFAULT(x) = x
#else
#define HVWS_DEFAULT(x)
#endif

/* accept must hold >= 29 bytes */
void ws_encode_key(const char* key, char accept[]);
int  ws_calc_frame_size(int data_len, bool has_mask HVWS_DEFAULT(false));
int  ws_build_frame(char* out, const char* data, int data_len, const char mask[4],
                    bool has_mask HVWS_DEFAULT(false), enum ws_opcode opcode HVWS_DEFAULT(WS_OPCODE_TEXT),
                    bool fin HVWS_DEFAULT(true));

static inline int ws_client_build_frame(char* out, const char* data, int data_len,
                                        enum ws_opcode opcode HVWS_DEFAULT(WS_OPCODE_TEXT),
                                        bool fin HVWS_DEFAULT(true)) {
    char mask[4];
    int r = rand();
    for (int i = 0; i < 4; i++) mask[i] = (char)((r >> (8 * i)) & 0xff);
    return ws_build_frame(out, data, data_len, mask, true, opcode, fin);
}

static inline int ws_server_build_frame(char* out, const char* data, int data_len,
                                        enum ws_opcode opcode HVWS_DEFAULT(WS_OPCODE_TEXT),
                                        bool fin HVWS_DEFAULT(true)) {
    char mask[4] = {0, 0, 0, 0};
    return ws_build_frame(out, data, data_len, mask, false, opcode, fin);
}

#ifdef __cplusplus
}
#endif
#endif

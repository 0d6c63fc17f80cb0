/*
 * WebSocketParser.h -- drop-in for libhv's WebSocket message reassembler
 * (reference: http/WebSocketParser.h:10-33, http/WebSocketParser.cpp:8-75).
 *
 * Same public members, constructor/destructor and FeedRecvData signature, so
 * http/server/HttpHandler.cpp:168-217,757-763 and
 * http/client/WebSocketClient.cpp:187-193 compile and link unchanged.
 * FeedRecvData runs frame discovery/header parse and the XOR unmask as HIP
 * kernels on MI355X, rewrites the caller's buffer in place exactly as the
 * reference does (payload unmasked, header bytes untouched), and fires
 * onMessage(opcode, message) for every FIN frame in order.
 */
#ifndef HVWS_WEBSOCKET_PARSER_HPP
#define HVWS_WEBSOCKET_PARSER_HPP

#include <stddef.h>

#include <functional>
#include <memory>
#include <string>

#ifndef HV_EXPORT
#define HV_EXPORT __attribute__((visibility("default")))
#endif

enum websocket_parser_state {
    WS_FRAME_BEGIN,
    WS_FRAME_HEADER,
    WS_FRAME_BODY,
    WS_FRAME_END,
    WS_FRAME_FIN,
};

struct websocket_parser;

class HV_EXPORT WebSocketParser {
public:
    websocket_parser*                                       parser;
    websocket_parser_state                                  state;
    int                                                     opcode;
    std::string                                             message;
    std::function<void(int opcode, const std::string& msg)> onMessage;

    WebSocketParser();
    ~WebSocketParser();

    /* Returns len (as int, like the reference) once every byte is consumed. */
    int FeedRecvData(const char* data, size_t len);
};

typedef std::shared_ptr<WebSocketParser> WebSocketParserPtr;

/* Batched FeedRecvData for an event loop: n connections' reads in one GPU
 * round trip (one segment each).  Same effects, per parser, as calling
 * parsers[i]->FeedRecvData(data[i], len[i]) in order i = 0..n-1; rets[i]
 * receives each call's return value.  New entry point (no reference twin).
 * Nested feeds: an onMessage replayed by this call (or by a feeder) may feed
 * any parser whose results are final; feeding one whose state a replay still
 * to come on this thread will write (later in the same batch, or in a
 * feeder's run already in flight) returns -1 and changes nothing -- as does
 * FeedRecvData on such a parser.  Returns n, or -1. */
HV_EXPORT int hvws_feed_many(WebSocketParser* const* parsers, const char* const* data, const size_t* len, int n,
                             int* rets);

/* Pipelined form for an event loop (see hvws_feeder in hvws.h): starts this
 * poll iteration's reads on the GPU and replays the previous submission's
 * callbacks meanwhile.  Returns n, or -1 when called from inside one of the
 * feeder's own callbacks. */
struct hvws_feeder;
HV_EXPORT int hvws_feeder_submit(hvws_feeder* f, WebSocketParser* const* parsers, const char* const* data,
                                 const size_t* len, int n, int* rets);

#endif

/*
 * ws_msg.cpp -- TEST INFRASTRUCTURE ONLY.
 *
 * Restatement of libhv's WebSocket message reassembler
 * (http/WebSocketParser.cpp:8-75, class at http/WebSocketParser.h:10-33),
 * driven by a frame parser selected at compile time:
 *   -DOWS_USE_REF : the reference's own websocket_parser_execute/_decode,
 *                   compiled from /root/reference into oracle/_ref/ (the
 *                   "reference" CPU path for bench.py's cpu_baseline);
 *   otherwise     : this directory's restatement (ws_oracle.c).
 * The reference .cpp itself cannot be compiled here (base/hdef.h pulls the
 * generated hconfig.h), hence this restatement of its ~70 lines.
 *
 * Exposes the C ABI `msgp_*` used by tests/ and bench.py; the product
 * library exposes the same shape as hvws_wsp_* (include/hvws.h).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <string>

#ifdef OWS_USE_REF
extern "C" {
#include "websocket_parser.h" /* /root/reference/http (include path set by Makefile) */
}
typedef websocket_parser ows_parser_t;
typedef websocket_parser_settings ows_settings_t;
#define X_INIT websocket_parser_init
#define X_EXECUTE websocket_parser_execute
#define X_DECODE websocket_parser_decode
#define X_HAS_MASK WS_HAS_MASK
#define X_FIN WS_FIN
#define X_OPMASK WS_OP_MASK
#else
#include "ws_oracle.h"
typedef ows_parser ows_parser_t;
typedef ows_settings ows_settings_t;
#define X_INIT ows_parser_init
#define X_EXECUTE ows_execute
#define X_DECODE ows_parser_decode
#define X_HAS_MASK OWS_HAS_MASK
#define X_FIN OWS_FIN
#define X_OPMASK OWS_OP_MASK
#endif

namespace {

enum msg_state { M_BEGIN, M_HEADER, M_BODY, M_END, M_FIN };   // WebSocketParser.h:10-16

typedef void (*msg_sink)(void* user, int opcode, const char* data, size_t len);

struct msgp {
    ows_parser_t* parser;
    msg_state     state;
    int           opcode;
    std::string   message;
    msg_sink      sink;
    void*         user;
};

const int kMaxReserve = 1 << 24;   // MAX_PAYLOAD_LENGTH, WebSocketParser.cpp:6

int cb_header(ows_parser_t* p) {                      // WebSocketParser.cpp:8-26
    msgp* m = (msgp*)p->data;
    int op = (int)(p->flags & X_OPMASK);
    if (op != 0) m->opcode = op;                      // CONTINUE keeps the latched opcode
    int length = (int)p->length;                      // int truncation (Q11)
    int want = length + 1 < kMaxReserve ? length + 1 : kMaxReserve;
    // The reference compares int against size_t; a negative `want` would
    // throw from reserve() there.  Only non-negative values reserve here.
    if (want >= 0 && (size_t)want > m->message.capacity()) m->message.reserve((size_t)want);
    if (m->state == M_BEGIN || m->state == M_FIN) m->message.clear();
    m->state = M_HEADER;
    return 0;
}

int cb_body(ows_parser_t* p, const char* at, size_t n) {   // WebSocketParser.cpp:28-37
    msgp* m = (msgp*)p->data;
    m->state = M_BODY;
    if (p->flags & X_HAS_MASK) X_DECODE((char*)at, at, n, p);
    m->message.append(at, n);
    return 0;
}

int cb_end(ows_parser_t* p) {                          // WebSocketParser.cpp:39-50
    msgp* m = (msgp*)p->data;
    m->state = M_END;
    if (p->flags & X_FIN) {
        m->state = M_FIN;
        if (m->sink) m->sink(m->user, m->opcode, m->message.data(), m->message.size());
    }
    return 0;
}

ows_settings_t g_cbs = {cb_header, cb_body, cb_end};  // WebSocketParser.cpp:52-56

}  // namespace

extern "C" {

void* msgp_new(void) {                                // WebSocketParser.cpp:58-64
    msgp* m = new msgp();
    m->parser = (ows_parser_t*)malloc(sizeof(ows_parser_t));
    memset(m->parser, 0, sizeof(ows_parser_t));
    X_INIT(m->parser);
    m->parser->data = m;
    m->state = M_BEGIN;
    m->opcode = 8;                                    // WS_OP_CLOSE (Q6)
    m->sink = NULL;
    m->user = NULL;
    return m;
}

void msgp_free(void* h) {
    msgp* m = (msgp*)h;
    if (!m) return;
    free(m->parser);
    delete m;
}

void msgp_set_sink(void* h, msg_sink sink, void* user) {
    msgp* m = (msgp*)h;
    m->sink = sink;
    m->user = user;
}

int msgp_feed(void* h, const char* data, size_t len) {   // WebSocketParser.cpp:73-75
    msgp* m = (msgp*)h;
    return (int)X_EXECUTE(m->parser, &g_cbs, data, len);
}

/* Parser state after the last feed, for carry comparisons. */
void msgp_state(void* h, uint64_t out[8]) {
    msgp* m = (msgp*)h;
    uint32_t mask;
    memcpy(&mask, m->parser->mask, 4);
    out[0] = m->parser->state;
    out[1] = (uint64_t)m->parser->flags;
    out[2] = mask;
    out[3] = m->parser->mask_offset;
    out[4] = m->parser->length;
    out[5] = m->parser->require;
    out[6] = m->parser->offset;
    out[7] = (uint64_t)m->state | ((uint64_t)(uint32_t)m->opcode << 32);
}

/* ---- bench helpers: feed a whole rx buffer in `chunk`-byte pieces ---- */
struct bench_acc {
    uint64_t msgs;
    uint64_t bytes;
    uint64_t xsum;
};

static void bench_sink(void* user, int opcode, const char* data, size_t len) {
    bench_acc* a = (bench_acc*)user;
    a->msgs++;
    a->bytes += len;
    a->xsum += (uint64_t)opcode * 31u + (len ? (uint8_t)data[len - 1] : 0u);
}

/* Returns 0 on success; out = {messages, message bytes, checksum, fed}. */
int msgp_bench_feed(char* rx, size_t len, size_t chunk, uint64_t out[4]) {
    bench_acc acc = {0, 0, 0};
    void* h = msgp_new();
    msgp_set_sink(h, bench_sink, &acc);
    size_t at = 0;
    int rc = 0;
    while (at < len) {
        size_t n = len - at < chunk ? len - at : chunk;
        int got = msgp_feed(h, rx + at, n);
        if ((size_t)got != n) { rc = -1; break; }
        at += n;
    }
    msgp_free(h);
    out[0] = acc.msgs;
    out[1] = acc.bytes;
    out[2] = acc.xsum;
    out[3] = at;
    return rc;
}

/* Decode-only path (websocket_decode over payload spans), given spans. */
uint64_t msgp_bench_decode_spans(char* rx, const uint64_t* off, const uint64_t* n,
                                 const uint32_t* key, size_t nspans) {
    uint64_t total = 0;
    for (size_t i = 0; i < nspans; i++) {
        char k[4];
        memcpy(k, &key[i], 4);
#ifdef OWS_USE_REF
        websocket_decode(rx + off[i], rx + off[i], n[i], k, 0);
#else
        ows_decode(rx + off[i], rx + off[i], n[i], k, 0);
#endif
        total += n[i];
    }
    return total;
}

#ifdef OWS_USE_REF
/* Handshake digest baseline: the reference ws_encode_key (http/wsdef.c:11-20)
 * over n keys of klen bytes laid out `stride` apart; out: 32 bytes per key. */
void ws_encode_key(const char* key, char accept[]);
uint64_t msgp_bench_keys(const char* keys, uint64_t n, uint32_t stride, uint32_t klen, char* out) {
    char k[256];
    uint64_t x = 0;
    if (klen >= sizeof(k)) return 0;
    for (uint64_t i = 0; i < n; i++) {
        memcpy(k, keys + i * stride, klen);
        k[klen] = 0;
        memset(out + i * 32, 0, 32);
        ws_encode_key(k, out + i * 32);
        x += (uint8_t)out[i * 32];
    }
    return x;
}
#endif

}  // extern "C"

/*
 * evlog.c -- test harness (not product code).
 *
 * Drives any implementation of the websocket_parser C ABI
 * (http/websocket_parser.h:70-80) -- the product's GPU-backed one, the
 * oracle restatement, or the compiled reference -- through the same chunked
 * feed and records every callback with the parser fields visible at that
 * moment.  Identical logs == identical observable behaviour.
 *
 * Log records (little-endian, packed):
 *   'H' flags:u32 mask:u32 length:u64 require:u64 state:u32 mask_offset:u8
 *   'B' at:u64 n:u64 flags:u32 require:u64 state:u32 mask_offset:u8
 *   'E' flags:u32 require:u64 state:u32 mask_offset:u8
 *   'R' ret:u64 state:u32 flags:u32 mask:u32 mask_offset:u8 length:u64 require:u64
 * `at` is relative to the data pointer passed to that execute() call.
 */
#include <stddef.h>
#include <stdint.h>
#include <string.h>

typedef struct evp {
    uint32_t state;
    uint32_t flags;
    char     mask[4];
    uint8_t  mask_offset;
    size_t   length;
    size_t   require;
    size_t   offset;
    void*    data;
} evp;

typedef int (*cb_t)(evp*);
typedef int (*dcb_t)(evp*, const char*, size_t);
typedef struct evs { cb_t h; dcb_t b; cb_t e; } evs;

typedef size_t (*exec_t)(evp*, const evs*, const char*, size_t);
typedef void (*init_t)(evp*);
typedef void (*pdecode_t)(char*, const char*, size_t, evp*);

typedef struct evctx {
    uint8_t*    log;
    size_t      cap;
    size_t      len;
    const char* base;
    pdecode_t   decode;      /* non-NULL: unmask masked spans in place */
    int64_t     abort_at;    /* callback index that returns 1, -1 none */
    int64_t     ncb;
    int         overflow;
} evctx;

static void put(evctx* c, const void* p, size_t n) {
    if (c->len + n > c->cap) { c->overflow = 1; return; }
    memcpy(c->log + c->len, p, n);
    c->len += n;
}
static void put8(evctx* c, uint8_t v) { put(c, &v, 1); }
static void put32(evctx* c, uint32_t v) { put(c, &v, 4); }
static void put64(evctx* c, uint64_t v) { put(c, &v, 8); }

static int maybe_abort(evctx* c) {
    int64_t k = c->ncb++;
    return (c->abort_at >= 0 && k == c->abort_at) ? 1 : 0;
}

static int on_h(evp* p) {
    evctx* c = (evctx*)p->data;
    uint32_t m;
    memcpy(&m, p->mask, 4);
    put8(c, 'H'); put32(c, p->flags); put32(c, m); put64(c, p->length); put64(c, p->require);
    put32(c, p->state); put8(c, p->mask_offset);
    return maybe_abort(c);
}

static int on_b(evp* p, const char* at, size_t n) {
    evctx* c = (evctx*)p->data;
    put8(c, 'B'); put64(c, (uint64_t)(at - c->base)); put64(c, n); put32(c, p->flags);
    put64(c, p->require); put32(c, p->state); put8(c, p->mask_offset);
    if (c->decode && (p->flags & 0x20u)) c->decode((char*)at, at, n, p);
    return maybe_abort(c);
}

static int on_e(evp* p) {
    evctx* c = (evctx*)p->data;
    put8(c, 'E'); put32(c, p->flags); put64(c, p->require); put32(c, p->state); put8(c, p->mask_offset);
    return maybe_abort(c);
}

/* Feeds `data` in the given chunk sizes.  After a short return the rest of
 * that chunk is fed again from the returned count (a naive caller), once.
 * `data` is modified in place when `decode` is given.
 * Returns bytes of log written, or -1 on log overflow. */
int64_t evlog_feed(exec_t ex, init_t init, pdecode_t decode, char* data, size_t len,
                   const uint64_t* chunks, size_t nchunks, int64_t abort_at,
                   uint8_t* log, size_t cap) {
    evp p;
    evs s = {on_h, on_b, on_e};
    evctx c;
    memset(&p, 0, sizeof(p));
    memset(&c, 0, sizeof(c));
    c.log = log;
    c.cap = cap;
    c.decode = decode;
    c.abort_at = abort_at;
    init(&p);
    p.data = &c;
    size_t at = 0;
    for (size_t k = 0; k < nchunks && at < len; k++) {
        size_t n = chunks[k];
        if (n > len - at) n = len - at;
        size_t done = 0;
        int refed = 0;
        while (done < n) {
            c.base = data + at + done;
            size_t r = ex(&p, &s, data + at + done, n - done);
            uint32_t m;
            memcpy(&m, p.mask, 4);
            put8(&c, 'R'); put64(&c, r); put32(&c, p.state); put32(&c, p.flags); put32(&c, m);
            put8(&c, p.mask_offset); put64(&c, p.length); put64(&c, p.require);
            if (r >= n - done || refed) break;
            done += r;
            refed = 1;
        }
        at += n;
    }
    return c.overflow ? -1 : (int64_t)c.len;
}

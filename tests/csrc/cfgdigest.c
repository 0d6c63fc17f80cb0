/* TEST INFRASTRUCTURE ONLY (tests/golden/make_golden.py --configs c3,...).
 *
 * Reference digests of a full-size synthetic batch in bounded memory, for
 * configurations too large to hold (config 3: 68.7 GB; config 5: 8 of them).
 * The batch is never materialised: frames are built window by window with the
 * REFERENCE websocket_build_frame (http/websocket_parser.c:207-256) from the
 * plan's plaintext, the masked bytes are folded into the digest, the window
 * is fed through the reference parser + message layer in 8 KiB chunks
 * (http/websocket_parser.c:53-171 via oracle/ws_msg.cpp, libwsref.so) and the
 * unmasked bytes are folded into the second digest.
 *
 * The digest (include/hvws_synth.h hvws_digest) is additive over 8-byte
 * little-endian words w_k at absolute offsets 8k: sum of mix64(w_k ^ k*C),
 * the last word zero-padded.  So the buffer splits into byte ranges of 8-byte
 * aligned bounds, one per thread, whose sums add up.  A thread rebuilds and
 * refeeds the frame its range starts inside (from that frame's header), so
 * every byte it digests was unmasked by a parser that saw its whole frame.
 * Message statistics: each frame of an all-FIN plan ends one message, counted
 * by the thread its header lies in.
 *
 * Every reference function arrives as a pointer (resolved by the Python
 * driver from oracle/_ref/libwsref.so), so nothing here links the reference.
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef size_t (*build_fn)(char* out, int flags, const char mask[4], const char* data, size_t len);
typedef void (*sink_fn)(void* user, int opcode, const char* data, size_t len);
typedef void* (*msgp_new_fn)(void);
typedef void (*msgp_set_sink_fn)(void* h, sink_fn sink, void* user);
typedef int (*msgp_feed_fn)(void* h, const char* data, size_t len);
typedef void (*msgp_free_fn)(void* h);
typedef void (*synth_fn)(uint8_t* out, uint64_t seed, uint64_t frame, uint64_t length, int text);

struct cfgd_fns {
    build_fn build;
    msgp_new_fn mnew;
    msgp_set_sink_fn msink;
    msgp_feed_fn mfeed;
    msgp_free_fn mfree;
    synth_fn synth;
};

static uint64_t mix64(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

/* Streaming digest over ascending absolute offsets. */
struct dig {
    uint64_t sum;
    uint64_t word;   /* bytes of the word being filled */
    uint64_t at;     /* next absolute offset expected */
};

static void dig_bytes(struct dig* d, uint64_t abs, const uint8_t* p, uint64_t n) {
    const uint64_t C = 0xD1B54A32D192ED03ull;
    uint64_t i = 0;
    (void)abs;   /* == d->at: callers feed contiguously */
    while (i < n && (d->at & 7u)) {
        d->word |= (uint64_t)p[i] << (8u * (d->at & 7u));
        ++i;
        if ((++d->at & 7u) == 0) {
            d->sum += mix64(d->word ^ (((d->at >> 3) - 1) * C));
            d->word = 0;
        }
    }
    for (; i + 8 <= n; i += 8, d->at += 8) {
        uint64_t w;
        memcpy(&w, p + i, 8);
        d->sum += mix64(w ^ ((d->at >> 3) * C));
    }
    for (; i < n; ++i, ++d->at) d->word |= (uint64_t)p[i] << (8u * (d->at & 7u));
}

static void dig_finish(struct dig* d) {   /* zero-padded last word */
    if (d->at & 7u) d->sum += mix64(d->word ^ ((d->at >> 3) * 0xD1B54A32D192ED03ull));
    d->word = 0;
}

struct msgs {
    uint64_t n, bytes, xsum;
    int skip;   /* messages still to skip (the frame owned by the previous range) */
};

static void on_msg(void* user, int opcode, const char* data, size_t len) {
    struct msgs* m = (struct msgs*)user;
    if (m->skip > 0) {
        m->skip--;
        return;
    }
    m->n++;
    m->bytes += len;
    m->xsum += (uint64_t)opcode * 31u + (len ? (uint8_t)data[len - 1] : 0u);
}

struct job {
    const struct cfgd_fns* F;
    uint64_t seed, n, total, lo, hi;   /* byte range [lo, hi) */
    const uint64_t *off, *len;
    const uint8_t *flags, *text;
    const uint32_t* mask;
    struct dig dm, du;
    struct msgs ms;
    int rc;
};

static uint64_t frame_size(uint8_t flags, uint64_t n) {
    return n + 2 + (n < 126 ? 0 : n <= 0xFFFF ? 2 : 8) + ((flags & 0x20) ? 4 : 0);
}

/* last frame whose header starts at or before x */
static uint64_t frame_at(const uint64_t* off, uint64_t n, uint64_t x) {
    uint64_t a = 0, b = n;
    while (b - a > 1) {
        uint64_t m = (a + b) / 2;
        if (off[m] <= x) a = m;
        else b = m;
    }
    return a;
}

#define WINDOW (64ull << 20)

static void* run(void* arg) {
    struct job* J = (struct job*)arg;
    const struct cfgd_fns* F = J->F;
    J->rc = -1;
    if (J->lo >= J->hi) {
        J->rc = 0;
        return NULL;
    }
    uint64_t f = frame_at(J->off, J->n, J->lo);
    const uint64_t f_end = frame_at(J->off, J->n, J->hi - 1) + 1;
    uint64_t maxf = 0;
    for (uint64_t i = f; i < f_end; ++i) {
        uint64_t s = frame_size(J->flags[i], J->len[i]);
        if (s > maxf) maxf = s;
    }
    const uint64_t cap = (WINDOW > maxf ? WINDOW : maxf) + 16;
    uint8_t* buf = (uint8_t*)malloc(cap);
    uint8_t* plain = (uint8_t*)malloc(maxf + 16);
    void* h = F->mnew();
    if (!buf || !plain || !h) goto out;
    J->ms.skip = J->off[f] < J->lo ? 1 : 0;
    F->msink(h, on_msg, &J->ms);
    J->dm.at = J->du.at = J->lo;
    while (f < f_end) {
        /* window: frames [f, g) spanning at most `cap` bytes (one at least) */
        const uint64_t base = J->off[f];
        uint64_t g = f, span = 0;
        while (g < f_end) {
            uint64_t e = J->off[g] + frame_size(J->flags[g], J->len[g]) - base;
            if (e > cap - 16 && g > f) break;
            span = e;
            ++g;
        }
        for (uint64_t i = f; i < g; ++i) {
            char key[4];
            memcpy(key, &J->mask[i], 4);
            F->synth(plain, J->seed, i, J->len[i], J->text ? J->text[i] : 0);
            F->build((char*)buf + (J->off[i] - base), J->flags[i], key, (const char*)plain, (size_t)J->len[i]);
        }
        /* the part of the window inside [lo, hi) */
        uint64_t a = base > J->lo ? base : J->lo, b = base + span < J->hi ? base + span : J->hi;
        if (a < b) dig_bytes(&J->dm, a, buf + (a - base), b - a);
        for (uint64_t at = 0; at < span; at += 8192) {
            size_t k = span - at < 8192 ? (size_t)(span - at) : 8192;
            if ((size_t)F->mfeed(h, (const char*)buf + at, k) != k) goto out;
        }
        if (a < b) dig_bytes(&J->du, a, buf + (a - base), b - a);
        f = g;
    }
    if (J->hi == J->total) {
        dig_finish(&J->dm);
        dig_finish(&J->du);
    }
    J->rc = 0;
out:
    if (h) F->mfree(h);
    free(buf);
    free(plain);
    return NULL;
}

/* out: {digest_masked, digest_unmasked, messages, message_bytes, message_xsum}.
 * threads > 1 requires an all-FIN plan with no CONTINUE frames (each frame is
 * one message, so ranges are independent); the caller checks.  Returns 0. */
int cfgd_run(const struct cfgd_fns* F, uint64_t seed, uint64_t n, const uint64_t* off, const uint8_t* flags,
             const uint32_t* mask, const uint64_t* len, const uint8_t* text, uint64_t total, int threads,
             uint64_t out[5]) {
    if (threads < 1) threads = 1;
    if (n == 0 || total == 0) return -1;
    struct job* J = (struct job*)calloc((size_t)threads, sizeof(struct job));
    pthread_t* th = (pthread_t*)calloc((size_t)threads, sizeof(pthread_t));
    if (!J || !th) return -1;
    for (int t = 0; t < threads; ++t) {
        J[t].F = F;
        J[t].seed = seed;
        J[t].n = n;
        J[t].total = total;
        J[t].off = off;
        J[t].len = len;
        J[t].flags = flags;
        J[t].text = text;
        J[t].mask = mask;
        J[t].lo = t == 0 ? 0 : (total / (uint64_t)threads * (uint64_t)t) & ~7ull;
        J[t].hi = t == threads - 1 ? total : (total / (uint64_t)threads * (uint64_t)(t + 1)) & ~7ull;
    }
    for (int t = 0; t < threads; ++t) pthread_create(&th[t], NULL, run, &J[t]);
    int rc = 0;
    memset(out, 0, 5 * sizeof(uint64_t));
    for (int t = 0; t < threads; ++t) {
        pthread_join(th[t], NULL);
        rc |= J[t].rc;
        out[0] += J[t].dm.sum;
        out[1] += J[t].du.sum;
        out[2] += J[t].ms.n;
        out[3] += J[t].ms.bytes;
        out[4] += J[t].ms.xsum;
    }
    free(J);
    free(th);
    return rc;
}

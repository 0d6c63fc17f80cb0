/* MEASUREMENT HARNESS (bench.py drop_in leg, scripts/bench_dropin.py): the
 * literal drop-in's per-call latency with no interpreter in the loop.  The
 * functions under test arrive as pointers: the product's (libhvws.so) or the
 * reference's (oracle/_ref) -- the same signatures. */
#include <stddef.h>
#include <stdint.h>
#include <string.h>
#include <time.h>

typedef int (*feed_fn)(void* h, const char* data, size_t len);
typedef size_t (*build_fn)(char* frame, int flags, const char mask[4], const char* data, size_t len);

static double now_s(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return (double)t.tv_sec + 1e-9 * (double)t.tv_nsec;
}

/* Feeds buf[0, total) to handle h in `read`-byte calls; returns the seconds
 * taken, or -1 if a call consumed less than it was given. */
double cb_feed(feed_fn f, void* h, char* buf, size_t total, size_t read) {
    const double t = now_s();
    for (size_t at = 0; at < total; at += read) {
        const size_t n = total - at < read ? total - at : read;
        if ((size_t)f(h, buf + at, n) != n) return -1.0;
    }
    return now_s() - t;
}

/* reps calls of build(out, flags, mask, data, len); returns seconds, or -1. */
double cb_build(build_fn f, char* out, int flags, const char* mask, const char* data, size_t len, int reps) {
    const double t = now_s();
    size_t x = 0;
    for (int i = 0; i < reps; ++i) x += f(out, flags, mask, data, len);
    const double dt = now_s() - t;
    return x == (size_t)reps * (len + 2 + (len < 126 ? 0 : len <= 0xFFFF ? 2 : 8) + ((flags & 0x20) ? 4 : 0)) ? dt : -1.0;
}

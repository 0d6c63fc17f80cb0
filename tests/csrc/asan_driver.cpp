// asan_driver.cpp -- test harness (not product code).
//
// Drives the product library's host code under AddressSanitizer (host side
// only: the library is rebuilt with -Xarch_host -fsanitize=address, device
// code is untouched) on a real GPU: WebSocketParser::FeedRecvData and
// hvws_feed_many over random streams and chunkings (both receive paths),
// websocket_parser_execute with early returns, validation rejects,
// hvws_build_frames and hvws_encode_keys.  Expected messages come from the
// oracle's message-layer restatement (oracle/_build/libwsoracle.so).
// Exit status 0 = every check matched and ASan reported nothing.
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <random>
#include <thread>
#include <string>
#include <utility>
#include <vector>

#include "WebSocketParser.h"
#include "hvws.h"
#include "wsdef.h"

extern "C" {
typedef void (*msg_sink)(void* user, int opcode, const char* data, size_t len);
void* msgp_new(void);
void msgp_free(void* h);
void msgp_set_sink(void* h, msg_sink sink, void* user);
int msgp_feed(void* h, const char* data, size_t len);
}

namespace {

typedef std::vector<std::pair<int, std::string>> Msgs;
int g_fail = 0;

#define CHECK(c)                                                         \
    do {                                                                 \
        if (!(c)) {                                                      \
            fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
            ++g_fail;                                                    \
        }                                                                \
    } while (0)

std::string frame(std::mt19937_64& rng, int op, bool fin, bool masked, size_t n) {
    std::string payload(n, '\0');
    for (auto& ch : payload) ch = (char)(rng() & 0xFF);
    char key[4];
    for (auto& k : key) k = (char)(rng() & 0xFF);
    std::string out(n + 14, '\0');
    int flags = op | (fin ? 0x10 : 0) | (masked ? 0x20 : 0);
    size_t w = websocket_build_frame(&out[0], (websocket_flags)flags, key, payload.data(), n);
    out.resize(w);
    return out;
}

std::string stream(std::mt19937_64& rng, int frames) {
    std::string s;
    for (int i = 0; i < frames; ++i) {
        const int kind = (int)(rng() % 10);
        size_t n = kind < 6 ? rng() % 126 : (kind < 9 ? 126 + rng() % 4000 : 65536 + rng() % 5000);
        if (kind == 5) s += frame(rng, 9, true, true, rng() % 20);          // ping between
        s += frame(rng, (rng() & 1) ? 1 : 2, (rng() % 4) != 0, (rng() % 8) != 0, n);
    }
    return s;
}

std::vector<size_t> chunks(std::mt19937_64& rng, size_t total) {
    std::vector<size_t> c;
    size_t at = 0;
    while (at < total) {
        size_t k = 1 + rng() % (rng() % 3 == 0 ? 16 : 9000);
        if (k > total - at) k = total - at;
        c.push_back(k);
        at += k;
    }
    return c;
}

void sink(void* user, int op, const char* data, size_t len) {
    ((Msgs*)user)->emplace_back(op, std::string(data, len));
}

Msgs oracle_msgs(const std::string& data, const std::vector<size_t>& ch) {
    Msgs m;
    std::string buf = data;
    void* h = msgp_new();
    msgp_set_sink(h, sink, &m);
    size_t at = 0;
    for (size_t k : ch) {
        msgp_feed(h, &buf[at], k);
        at += k;
    }
    msgp_free(h);
    return m;
}

void test_feed(std::mt19937_64& rng) {
    for (int t = 0; t < 30; ++t) {
        const std::string data = stream(rng, 1 + (int)(rng() % 40));
        const std::vector<size_t> ch = chunks(rng, data.size());
        WebSocketParser p;
        Msgs got;
        p.onMessage = [&](int op, const std::string& msg) { got.emplace_back(op, msg); };
        std::string buf = data;
        size_t at = 0;
        for (size_t k : ch) {
            CHECK(p.FeedRecvData(&buf[at], k) == (int)k);
            at += k;
        }
        CHECK(got == oracle_msgs(data, ch));
    }
}

void test_feed_many(std::mt19937_64& rng) {
    const int n = 40;
    std::vector<std::string> data(n), buf(n);
    std::vector<std::vector<size_t>> ch(n);
    std::vector<WebSocketParser> ps(n);
    std::vector<Msgs> got(n);
    for (int i = 0; i < n; ++i) {
        data[i] = stream(rng, 1 + (int)(rng() % 20));
        buf[i] = data[i];
        ch[i] = chunks(rng, data[i].size());
        ps[i].onMessage = [&got, i](int op, const std::string& msg) { got[i].emplace_back(op, msg); };
    }
    std::vector<size_t> at(n, 0), next(n, 0);
    for (bool more = true; more;) {
        more = false;
        std::vector<WebSocketParser*> pp;
        std::vector<const char*> dd;
        std::vector<size_t> ll;
        std::vector<int> who;
        for (int i = 0; i < n; ++i) {
            if (next[i] >= ch[i].size() || rng() % 3 == 0) continue;
            pp.push_back(&ps[i]);
            dd.push_back(&buf[i][at[i]]);
            ll.push_back(ch[i][next[i]]);
            who.push_back(i);
        }
        std::vector<int> rets(pp.size());
        if (!pp.empty()) hvws_feed_many(pp.data(), dd.data(), ll.data(), (int)pp.size(), rets.data());
        for (size_t j = 0; j < who.size(); ++j) {
            CHECK(rets[j] == (int)ll[j]);
            at[who[j]] += ll[j];
            ++next[who[j]];
        }
        for (int i = 0; i < n; ++i) more |= next[i] < ch[i].size();
    }
    for (int i = 0; i < n; ++i) CHECK(got[i] == oracle_msgs(data[i], ch[i]));
}

struct cbstate {
    int calls = 0, fail_at = -1;
};
int cb_hdr(websocket_parser* p) {
    cbstate* s = (cbstate*)p->data;
    return s->calls++ == s->fail_at;
}
int cb_body(websocket_parser* p, const char*, size_t) {
    cbstate* s = (cbstate*)p->data;
    return s->calls++ == s->fail_at;
}

void test_execute(std::mt19937_64& rng) {
    for (int t = 0; t < 20; ++t) {
        const std::string data = stream(rng, 1 + (int)(rng() % 20));
        websocket_parser_settings st;
        websocket_parser_settings_init(&st);
        st.on_frame_header = cb_hdr;
        st.on_frame_body = cb_body;
        st.on_frame_end = cb_hdr;
        cbstate cs;
        cs.fail_at = (int)(rng() % 30);
        websocket_parser p;
        websocket_parser_init(&p);
        p.data = &cs;
        size_t r = websocket_parser_execute(&p, &st, data.data(), data.size());
        CHECK(r <= data.size());
    }
}

void test_validation(std::mt19937_64& rng) {
    hvws_set_validation(nullptr, HVWS_V_ALL);
    std::string data = stream(rng, 3);
    std::string bad = frame(rng, 2, true, false, 10);   // unmasked client frame
    std::string all = data + bad;
    std::vector<char> buf(all.begin(), all.end());
    WebSocketParser p;
    const int r = p.FeedRecvData(buf.data(), buf.size());
    CHECK(r >= 0 && (size_t)r < buf.size());
    hvws_set_validation(nullptr, 0);
}

void test_tx_and_keys(std::mt19937_64& rng) {
    hvws_ctx* c = hvws_ctx_create(0);
    CHECK(c != nullptr);
    const uint64_t n = 300;
    std::vector<uint64_t> off(n), len(n);
    std::vector<uint8_t> flags(n);
    std::vector<uint32_t> mask(n);
    std::string payload;
    std::string expect;
    for (uint64_t i = 0; i < n; ++i) {
        len[i] = rng() % 3000;
        off[i] = payload.size();
        std::string p(len[i], '\0');
        for (auto& ch : p) ch = (char)(rng() & 0xFF);
        payload += p;
        flags[i] = (uint8_t)(2 | 0x10 | ((rng() & 1) ? 0x20 : 0));
        mask[i] = (uint32_t)rng();
        std::string f(len[i] + 14, '\0');
        f.resize(websocket_build_frame(&f[0], (websocket_flags)flags[i], (const char*)&mask[i], p.data(), len[i]));
        expect += f;
    }
    void* d_pay = hvws_dev_alloc(c, payload.size() + 64);
    void* d_out = hvws_dev_alloc(c, expect.size() + 64);
    void* d_off = hvws_dev_alloc(c, n * 8);
    void* d_len = hvws_dev_alloc(c, n * 8);
    void* d_fl = hvws_dev_alloc(c, n);
    void* d_mk = hvws_dev_alloc(c, n * 4);
    hvws_h2d(c, d_pay, payload.data(), payload.size());
    hvws_h2d(c, d_off, off.data(), n * 8);
    hvws_h2d(c, d_len, len.data(), n * 8);
    hvws_h2d(c, d_fl, flags.data(), n);
    hvws_h2d(c, d_mk, mask.data(), n * 4);
    uint64_t out_len = 0;
    CHECK(hvws_build_frames(c, (uint8_t*)d_out, expect.size() + 64, (const uint8_t*)d_pay, payload.size(),
                            (const uint64_t*)d_off, (const uint64_t*)d_len, (const uint8_t*)d_fl,
                            (const uint32_t*)d_mk, n, nullptr, &out_len) == HVWS_OK);
    CHECK(out_len == expect.size());
    std::string got(out_len, '\0');
    hvws_d2h(c, &got[0], d_out, out_len);
    hvws_sync(c);
    CHECK(got == expect);

    const char* key = "dGhlIHNhbXBsZSBub25jZQ==";
    void* d_k = hvws_dev_alloc(c, 64);
    void* d_ko = hvws_dev_alloc(c, 8);
    void* d_kl = hvws_dev_alloc(c, 8);
    void* d_acc = hvws_dev_alloc(c, 64);
    const uint64_t ko = 0;
    const uint32_t kl = 24;
    hvws_h2d(c, d_k, key, 24);
    hvws_h2d(c, d_ko, &ko, 8);
    hvws_h2d(c, d_kl, &kl, 4);
    CHECK(hvws_encode_keys(c, (const char*)d_k, (const uint64_t*)d_ko, (const uint32_t*)d_kl, 1, (char*)d_acc) ==
          HVWS_OK);
    char acc[32];
    hvws_d2h(c, acc, d_acc, 32);
    hvws_sync(c);
    CHECK(memcmp(acc, "s3pPLMBiTxaQ9kYGzzhZRbK+xOo=", 28) == 0);
    char host_acc[32] = {0};
    ws_encode_key(key, host_acc);
    CHECK(memcmp(acc, host_acc, 32) == 0);
    for (void* p : {d_pay, d_out, d_off, d_len, d_fl, d_mk, d_k, d_ko, d_kl, d_acc}) hvws_dev_free(c, p);
    hvws_ctx_destroy(c);
}

// The resident worker (hvws_set_door) under ASan: this thread's context and
// three loop threads with workers of their own feed through it; the threads
// exit with their workers resident (the thread guard parks them), a free on
// this thread parks the others' workers, and the process exits with this
// thread's worker still resident and its context never released -- the path
// of round 3's "corrupted double-linked list" at exit.
void test_door(std::mt19937_64& rng) {
    hvws_set_door(nullptr, 1);
    test_feed(rng);
    std::vector<std::thread> th;
    for (int i = 0; i < 3; ++i) {
        const uint64_t seed = rng();
        th.emplace_back([seed] {
            std::mt19937_64 r(seed);
            hvws_set_door(nullptr, 1);
            test_feed(r);
        });
    }
    for (auto& t : th) t.join();
    hvws_ctx* c = hvws_ctx_create(0);
    void* p = hvws_dev_alloc(c, 1 << 20);
    hvws_dev_free(c, p);
    hvws_ctx_destroy(c);
    test_feed(rng);   // relaunches this thread's worker, left resident at exit
    uint64_t st[4];
    CHECK(hvws_door_stats(nullptr, st) == 0 && st[0] >= 1 && st[3] == 1);
}

}  // namespace

int main(int argc, char** argv) {
    if (argc > 1 && strcmp(argv[1], "door") == 0) {   // the worker's paths and a process exit with one resident
        std::mt19937_64 rng(20261017);
        test_door(rng);
        printf("asan_driver door: %s (%d failed checks)\n", g_fail ? "FAIL" : "ok", g_fail);
        fflush(stdout);
        return g_fail ? 1 : 0;
    }
    std::mt19937_64 rng(20261015);
    for (uint64_t limit : {0ull, ~0ull}) {   // small-batch path, then the general path
        hvws_set_small_batch_limit(nullptr, limit);
        test_feed(rng);
        test_feed_many(rng);
        test_execute(rng);
        test_validation(rng);
    }
    hvws_set_small_batch_limit(nullptr, 0);
    test_tx_and_keys(rng);
    hvws_thread_release();
    printf("asan_driver: %s (%d failed checks)\n", g_fail ? "FAIL" : "ok", g_fail);
    fflush(stdout);   // before the runtimes' exit handlers
    return g_fail ? 1 : 0;
}

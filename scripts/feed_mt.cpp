// feed_mt.cpp -- benchmark harness (not product code): event-loop threads.
//
// T loop threads (libhv runs one event loop per worker thread,
// http/server/HttpServer.cpp:95-100), each owning C connections whose
// clients stream masked 1 KiB binary frames.  One poll iteration hands every
// connection's next 8 KiB read (event/hevent.h:16) to the parser:
//   gpu : hvws_feed_many (this library; one GPU round trip per thread per
//         iteration, each thread on its own context and stream)
//   gpupipe : hvws_feeder_submit (the device half of iteration k on the
//         thread's feeder worker while the loop thread replays k-1)
//   gpupin, gpupinpipe : the same two with every connection's stream in a
//         pinned arena (hvws_host_alloc), so the reads go to the device in
//         place (hvws_rx_reads)
//   ref : the reference frame parser + message layer (oracle/_ref), per
//         connection, on the same threads
// Prints one JSON line: aggregate payload GiB/s and per-iteration latency.
//
//   feed_mt <gpu|gpupipe|gpupin|gpupinpipe|ref> <threads> <connections per thread> <iterations>
#include <dlfcn.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <atomic>
#include <chrono>
#include <string>
#include <thread>
#include <vector>

#include "WebSocketParser.h"
#include "hvws.h"

namespace {

const size_t kRead = 8192;
const size_t kPayload = 1024;
const size_t kFrame = kPayload + 8;   // 2 + 2 (16-bit length) + 4 (key)

std::string client_stream(uint64_t seed, size_t bytes) {
    std::string s;
    s.reserve(bytes + kFrame);
    uint64_t x = seed * 0x9E3779B97F4A7C15ull + 1;
    while (s.size() < bytes) {
        x ^= x << 13;
        x ^= x >> 7;
        x ^= x << 17;
        const uint32_t key = (uint32_t)x;
        unsigned char h[8] = {0x82, 0x80 | 126, (unsigned char)(kPayload >> 8), (unsigned char)(kPayload & 0xFF)};
        memcpy(h + 4, &key, 4);
        s.append((const char*)h, 8);
        for (size_t i = 0; i < kPayload; ++i) s.push_back((char)(((x >> (i % 56)) & 0xFF) ^ ((key >> (8 * (i & 3))) & 0xFF)));
    }
    s.resize(bytes);
    return s;
}

typedef void (*msg_sink)(void*, int, const char*, size_t);
struct RefApi {
    void* (*make)(void);
    void (*free_)(void*);
    void (*set_sink)(void*, msg_sink, void*);
    int (*feed)(void*, const char*, size_t);
};

void count_sink(void* user, int, const char*, size_t len) { *(uint64_t*)user += len; }

}  // namespace

int main(int argc, char** argv) {
    if (argc < 5) {
        fprintf(stderr, "usage: feed_mt <gpu|ref> <threads> <connections/thread> <iterations>\n");
        return 2;
    }
    const std::string mode = argv[1];
    const bool gpu = mode.compare(0, 3, "gpu") == 0;
    const bool pipe = mode == "gpupipe" || mode == "gpupinpipe";
    const bool pin = mode == "gpupin" || mode == "gpupinpipe";
    const int T = atoi(argv[2]), C = atoi(argv[3]), I = atoi(argv[4]);
    RefApi ref = {};
    if (!gpu) {
        void* h = dlopen("oracle/_ref/libwsref.so", RTLD_NOW | RTLD_LOCAL);
        if (!h) {
            fprintf(stderr, "reference library: %s\n", dlerror());
            return 2;
        }
        ref.make = (void* (*)(void))dlsym(h, "msgp_new");
        ref.free_ = (void (*)(void*))dlsym(h, "msgp_free");
        ref.set_sink = (void (*)(void*, msg_sink, void*))dlsym(h, "msgp_set_sink");
        ref.feed = (int (*)(void*, const char*, size_t))dlsym(h, "msgp_feed");
    }
    std::vector<std::vector<std::string>> streams(T);
    for (int t = 0; t < T; ++t)
        for (int c = 0; c < C; ++c) streams[t].push_back(client_stream((uint64_t)t * 100003 + c, kRead * (I + 1)));
    std::atomic<int> ready{0};
    std::atomic<bool> go{false};
    std::vector<double> secs(T, 0.0);
    std::vector<uint64_t> delivered(T, 0);
    std::vector<std::thread> th;
    for (int t = 0; t < T; ++t) {
        th.emplace_back([&, t] {
            if (gpu) hvws_set_thread_device(0);
            std::vector<std::string>& ss = streams[t];
            // pinned: the thread's streams copied into one arena, connection-major
            hvws_ctx* actx = nullptr;
            char* arena = nullptr;
            const size_t stride = kRead * (I + 1);
            if (pin) {
                actx = hvws_ctx_create(0);
                arena = (char*)hvws_host_alloc(actx, stride * C);
                if (!arena) {
                    fprintf(stderr, "hvws_host_alloc: %s\n", hvws_last_error());
                    exit(1);
                }
                for (int c = 0; c < C; ++c) memcpy(arena + (size_t)c * stride, ss[c].data(), stride);
            }
            hvws_feeder* feeder = pipe ? hvws_feeder_new() : nullptr;
            std::vector<WebSocketParser> ps(gpu ? C : 0);
            std::vector<void*> rs;
            uint64_t got = 0;
            if (gpu) {
                for (auto& p : ps) p.onMessage = [&got](int, const std::string& m) { got += m.size(); };
            } else {
                for (int c = 0; c < C; ++c) {
                    rs.push_back(ref.make());
                    ref.set_sink(rs.back(), count_sink, &got);
                }
            }
            std::vector<WebSocketParser*> pp(C);
            std::vector<const char*> dd(C);
            std::vector<size_t> ll(C, kRead);
            std::vector<int> rets(C);
            for (int c = 0; c < C && gpu; ++c) pp[c] = &ps[c];
            auto iter = [&](int it) {
                for (int c = 0; c < C; ++c)
                    dd[c] = pin ? arena + (size_t)c * stride + (size_t)it * kRead : &ss[c][(size_t)it * kRead];
                if (feeder) {
                    hvws_feeder_submit(feeder, pp.data(), dd.data(), ll.data(), C, rets.data());
                } else if (gpu) {
                    hvws_feed_many(pp.data(), dd.data(), ll.data(), C, rets.data());
                } else {
                    for (int c = 0; c < C; ++c) ref.feed(rs[c], dd[c], kRead);
                }
            };
            iter(0);   // warm-up: contexts, allocations, first launch
            if (feeder) hvws_feeder_flush(feeder);
            ready++;
            while (!go.load()) std::this_thread::yield();
            const auto t0 = std::chrono::steady_clock::now();
            for (int it = 1; it <= I; ++it) iter(it);
            if (feeder) hvws_feeder_flush(feeder);   // the last iteration's callbacks, inside the timed region
            secs[t] = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
            delivered[t] = got;
            for (void* r : rs) ref.free_(r);
            if (feeder) hvws_feeder_free(feeder);
            if (arena) hvws_host_free(actx, arena);
            if (actx) hvws_ctx_destroy(actx);
            if (gpu) hvws_thread_release();
        });
    }
    while (ready.load() < T) std::this_thread::yield();
    go = true;
    for (auto& x : th) x.join();
    double wall = 0;
    uint64_t msg_bytes = 0;
    for (int t = 0; t < T; ++t) {
        wall = secs[t] > wall ? secs[t] : wall;
        msg_bytes += delivered[t];
    }
    const double payload = (double)T * C * I * kRead * kPayload / kFrame;
    printf("{\"bench\": \"feed_mt\", \"mode\": \"%s\", \"threads\": %d, \"connections_per_thread\": %d, "
           "\"iterations\": %d, \"read_bytes\": %zu, \"iteration_us\": %.1f, \"GiBps_payload\": %.3f, "
           "\"message_bytes\": %llu}\n",
           mode.c_str(), T, C, I, kRead, wall / I * 1e6, payload / wall / (1 << 30),
           (unsigned long long)msg_bytes);
    return 0;
}

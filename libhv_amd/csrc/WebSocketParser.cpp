// WebSocketParser.cpp -- drop-in for the reference message reassembler
// (http/WebSocketParser.cpp:8-75) on the MI355X engine.
//
// FeedRecvData ships the chunk to the device, runs k_scan (frame discovery +
// header parse) and k_unmask (XOR) there, copies the unmasked bytes back into
// the caller's buffer (the reference also rewrites it in place, Q10), and
// replays the reference's per-frame message logic on the host:
//   header: latch opcode unless CONTINUE, reserve, clear on BEGIN/FIN  (:8-26)
//   body:   append the (now unmasked) span                            (:28-37)
//   end:    on FIN, onMessage(opcode, message)                        (:39-50)
#include "WebSocketParser.h"

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <mutex>
#include <thread>
#include <vector>

#include "hvws.h"
#include "hvws_internal.h"

namespace hvws {
[[noreturn]] void fatal(const char* what);
hvws_ctx* thread_ctx();
char* pinned_stage(uint64_t bytes);
void ctx_copy_settings(hvws_ctx* dst, const hvws_ctx* src);
bool is_pinned(const void* p, uint64_t len);
bool take_frames(hvws_ctx* c, std::vector<hvws_frame>& frames, std::vector<uint64_t>& first,
                 std::vector<uint64_t>& count);
void gpu_feed(char* buf, size_t len, const websocket_parser& carry, bool unmask, std::vector<hvws_frame>& frames,
              websocket_parser& carry_out, int& started);
}  // namespace hvws

namespace {
// Gather (to_stage) or scatter the n chunks through the pinned stage, split
// into byte-balanced runs of chunks over the host copy pool.
void stage_copy(char* stage, const hvws_segment* segs, const char* const* data, const size_t* len, int n,
                uint64_t total, bool to_stage) {
    auto one = [&](int i) {
        if (!len[i]) return;
        if (to_stage) memcpy(stage + segs[i].off, data[i], len[i]);
        else memcpy(const_cast<char*>(data[i]), stage + segs[i].off, len[i]);
    };
    const int w = total >= hvws::kParCopyMin ? hvws::copy_width() : 1;
    if (w <= 1) {
        for (int i = 0; i < n; ++i) one(i);
        return;
    }
    std::vector<int> cut(1, 0);   // run r covers chunks [cut[r], cut[r+1])
    const uint64_t share = (total + w - 1) / w;
    for (int i = 0; i < n; ++i)
        if (segs[i].off + len[i] >= share * cut.size() && i + 1 < n) cut.push_back(i + 1);
    cut.push_back(n);
    hvws::par_for((int)cut.size() - 1, [&](int r) {
        for (int i = cut[r]; i < cut[r + 1]; ++i) one(i);
    });
}
}  // namespace

namespace {
// Pointer -> int index without per-element allocation (open addressing,
// linear probing, load <= 1/2, entries of older generations read as empty):
// a poll iteration looks every connection's parser up once or twice, and a
// node-allocating std::unordered_set/map cost ~100 ns per parser there.
class ptr_index {
  public:
    void reset(size_t n) {   // empty, room for n keys
        size_t cap = 16;
        while (cap < 2 * n) cap <<= 1;
        if (cap > key_.size()) {
            key_.assign(cap, nullptr);
            val_.assign(cap, 0);
            gen_.assign(cap, 0);
            cur_ = 0;
        }
        if (++cur_ == 0) {   // generation counter wrapped: clear for real
            std::fill(gen_.begin(), gen_.end(), 0u);
            cur_ = 1;
        }
    }
    // Adds p -> v; false (and no change) when p is already there.
    bool insert(const void* p, int v) {
        for (size_t i = slot(p);; i = (i + 1) & (key_.size() - 1)) {
            if (gen_[i] != cur_) {
                gen_[i] = cur_;
                key_[i] = p;
                val_[i] = v;
                return true;
            }
            if (key_[i] == p) return false;
        }
    }
    int find(const void* p) const {   // -1 when absent
        for (size_t i = slot(p);; i = (i + 1) & (key_.size() - 1)) {
            if (gen_[i] != cur_) return -1;
            if (key_[i] == p) return val_[i];
        }
    }

  private:
    size_t slot(const void* p) const {
        uint64_t x = (uint64_t)(uintptr_t)p;
        x ^= x >> 33;
        x *= 0xff51afd7ed558ccdull;
        x ^= x >> 33;
        return (size_t)x & (key_.size() - 1);
    }
    std::vector<const void*> key_;
    std::vector<int> val_;
    std::vector<uint32_t> gen_;
    uint32_t cur_ = 0;
};

// End of the run of distinct parsers starting at `done` (a parser seen twice
// starts a new run: its second chunk needs the carry its first one leaves).
int distinct_run_end(WebSocketParser* const* parsers, int done, int n) {
    thread_local ptr_index seen;   // used only between calls of feed_distinct / feeder_run
    seen.reset((size_t)(n - done));
    int end = done;
    while (end < n && seen.insert(parsers[end], end)) ++end;
    return end;
}

const int kMaxReserve = 1 << 24;   // MAX_PAYLOAD_LENGTH, reference WebSocketParser.cpp:6
const size_t kMappedRead = 32 << 10;   // largest read hvws_rx_reads takes in place

bool any_busy(WebSocketParser* const* parsers, int n);   // below, with the replay
}

WebSocketParser::WebSocketParser() {
    parser = (websocket_parser*)malloc(sizeof(websocket_parser));
    if (!parser) hvws::fatal("out of memory");
    memset(parser, 0, sizeof(*parser));
    websocket_parser_init(parser);
    parser->data = this;
    state = WS_FRAME_BEGIN;
    opcode = WS_OP_CLOSE;   // a lone CONTINUE first reports CLOSE (Q6)
}

WebSocketParser::~WebSocketParser() {
    if (parser) {
        free(parser);
        parser = NULL;
    }
}

namespace {

// The reference's per-frame message logic (http/WebSocketParser.cpp:8-50)
// over the frame records of one connection; `base` is where offset `base_off`
// of the batch buffer sits in the caller's (already unmasked) bytes.
// Returns the bytes consumed: len, or -- when hvws_set_validation rejects a
// header -- the index of that header's last byte, as execute reports a
// failing on_frame_header (the parser is left as that callback would see it).
size_t replay_messages(WebSocketParser* wp, const char* base, uint64_t base_off, const hvws_frame* frames, size_t n,
                       const websocket_parser& out, size_t len) {
    websocket_parser* parser = wp->parser;
    for (size_t i = 0; i < n; ++i) {
        const hvws_frame& f = frames[i];
        const uint32_t fl = f.info & HVWS_I_FLAGS;
        parser->flags = (websocket_flags)fl;
        parser->length = f.length;
        if ((f.info & HVWS_I_HDR) && (f.info & HVWS_I_INVALID)) {
            if (fl & WS_HAS_MASK) memcpy(parser->mask, &f.key, 4);
            parser->offset = 0;
            parser->state = f.length ? 4u : 0u;   // s_body / s_start
            parser->require = f.length;
            return (size_t)(f.pay_off - base_off) - 1;
        }
        if (f.info & HVWS_I_HDR) {
            const int op = (int)(fl & WS_OP_MASK);
            if (op != WS_OP_CONTINUE) wp->opcode = op;
            const int length = (int)f.length;   // int truncation, as the reference (Q11)
            const int want = length + 1 < kMaxReserve ? length + 1 : kMaxReserve;
            // The reference compares int with size_t here; a negative `want`
            // makes it call reserve(huge) and throw.  Skip the reserve instead.
            if (want >= 0 && (size_t)want > wp->message.capacity()) wp->message.reserve((size_t)want);
            if (wp->state == WS_FRAME_BEGIN || wp->state == WS_FRAME_FIN) wp->message.clear();
            wp->state = WS_FRAME_HEADER;
        }
        if (f.info & HVWS_I_BODY) {
            wp->state = WS_FRAME_BODY;
            wp->message.append(base + (f.pay_off - base_off), (size_t)f.pay_len);
        }
        if (f.info & HVWS_I_END) {
            wp->state = WS_FRAME_END;
            if (fl & WS_FIN) {
                wp->state = WS_FRAME_FIN;
                if (wp->onMessage) wp->onMessage(wp->opcode, wp->message);
            }
        }
    }
    void* keep = parser->data;
    hvws::copy_parser(*parser, out);
    parser->data = keep;
    return len;
}

}  // namespace

int WebSocketParser::FeedRecvData(const char* data, size_t len) {
    if (len == 0) return 0;
    WebSocketParser* self = this;
    if (any_busy(&self, 1)) return -1;   // a replay still to come would overwrite this feed
    std::vector<hvws_frame> frames;
    websocket_parser out;
    int started = 0;
    char* buf = const_cast<char*>(data);   // unmasked in place, like the reference
    hvws::gpu_feed(buf, len, *parser, true, frames, out, started);
    return (int)replay_messages(this, buf, 0, frames.data(), frames.size(), out, len);
}

// One GPU round trip for many connections' reads:
// every chunk becomes one segment of a single batch, so the launch and copy
// latency is paid once per poll iteration instead of once per connection.
static int feed_distinct(WebSocketParser* const* parsers, const char* const* data, const size_t* len, int n,
                         int* rets);

int hvws_feed_many(WebSocketParser* const* parsers, const char* const* data, const size_t* len, int n, int* rets) {
    if (n < 0 || any_busy(parsers, n)) return -1;
    // A connection's second chunk needs the carry its first chunk leaves, so
    // cut the batch before any parser that already appears in it.
    int done = 0;
    while (done < n) {
        const int end = distinct_run_end(parsers, done, n);
        feed_distinct(parsers + done, data + done, len + done, end - done, rets ? rets + done : nullptr);
        done = end;
    }
    return n;
}

namespace {
// $HVWS_EXPERIMENT feed_times=1: per-phase host time of feed_distinct, printed at exit (diagnostic)
struct feed_times {
    double ph[6] = {0, 0, 0, 0, 0, 0};   // carry, gather, gpu, scatter, replay, feeder wait
    long calls = 0;
    bool on = hvws::experiment("feed_times") && atoi(hvws::experiment("feed_times"));
    std::mutex m;   // the loop thread and feeder workers add to the same counters
    void add(int k, double us) {
        std::lock_guard<std::mutex> lk(m);
        ph[k] += us;
    }
    void call() {
        std::lock_guard<std::mutex> lk(m);
        ++calls;
    }
    ~feed_times() {
        if (on && calls)
            fprintf(stderr, "[feed_times] calls=%ld us/call: carry %.1f gather %.1f gpu %.1f scatter %.1f replay %.1f "
                    "feeder-wait %.1f\n",
                    calls, ph[0] / calls, ph[1] / calls, ph[2] / calls, ph[3] / calls, ph[4] / calls, ph[5] / calls);
    }
} g_ft;
double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
}  // namespace

namespace {
// One distinct-parser run of a poll iteration: its reads, the carries going
// in (then the states coming out) and the frame records of every segment.
struct feed_batch {
    std::vector<WebSocketParser*> parsers;
    std::vector<const char*> data;
    std::vector<size_t> len;
    int* rets = nullptr;
    std::vector<hvws_segment> segs;
    std::vector<websocket_parser> carry;
    std::vector<hvws_frame> frames;
    std::vector<uint64_t> first, count;
    uint64_t total = 0;
    bool mapped = false;   // reads taken in place (hvws_rx_reads): record offsets are per read
    int n() const { return (int)parsers.size(); }
    void set(WebSocketParser* const* p, const char* const* d, const size_t* l, int k, int* r) {
        parsers.assign(p, p + k);
        data.assign(d, d + k);
        len.assign(l, l + k);
        rets = r;
        segs.resize((size_t)k);
        carry.resize((size_t)k);
        total = 0;
        for (int i = 0; i < k; ++i) {
            segs[i].off = total;
            segs[i].len = len[i];
            total += len[i];
        }
    }
};

// The device half of a run, on the calling thread's context and pinned stage:
// gather the reads, one hvws_rx_batch, read the frame table back, and write
// the unmasked bytes back into the callers' buffers.  Touches no parser:
// b.carry must already hold the carries going in.
void gpu_part(feed_batch& b) {
    const int n = b.n();
    double t0 = g_ft.on ? now_us() : 0, t1;
    auto lap = [&](int k) {
        if (!g_ft.on) return;
        t1 = now_us();
        g_ft.add(k, t1 - t0);
        t0 = t1;
    };
    hvws_ctx* c = hvws::thread_ctx();
    static_assert(sizeof(size_t) == sizeof(uint64_t), "read lengths pass as uint64_t");
    // Reads in registered pinned memory (an event loop whose read buffers come
    // from hvws_host_alloc / hvws_host_register) go to the device where they
    // are: no gather, no write-back.  Anything else goes through the stage.
    b.mapped = n && b.len[0] <= kMappedRead && hvws::is_pinned(b.data[0], b.len[0]) &&
               hvws_rx_reads(c, const_cast<char* const*>(b.data.data()), (const uint64_t*)b.len.data(),
                             b.carry.data(), (uint32_t)n, 1) == HVWS_OK;
    char* stage = nullptr;
    if (!b.mapped) {
        stage = hvws::pinned_stage(b.total);
        stage_copy(stage, b.segs.data(), b.data.data(), b.len.data(), n, b.total, true);
        lap(1);
        if (hvws_rx_batch(c, (uint8_t*)stage, b.total, b.segs.data(), b.carry.data(), (uint32_t)n, 1) != HVWS_OK)
            hvws::fatal("hvws_rx_batch");
    }
    // small path: the records move out of the context's host cache; general
    // path: read back
    if (!hvws::take_frames(c, b.frames, b.first, b.count)) {
        const int64_t nf = hvws_frame_count(c);
        b.frames.resize((size_t)(nf > 0 ? nf : 0));
        b.first.resize((size_t)n);
        b.count.resize((size_t)n);
        if ((nf > 0 && hvws_get_frames(c, b.frames.data(), 0, (uint64_t)nf) != HVWS_OK) ||
            hvws_get_segment_frames(c, b.first.data(), b.count.data()) != HVWS_OK)
            hvws::fatal("frame table read-back");
    }
    lap(2);
    // Every segment leaves the (thread's, reusable) stage before any callback
    // runs: an onMessage that feeds again on this thread restages it.
    if (!b.mapped) stage_copy(stage, b.segs.data(), b.data.data(), b.len.data(), n, b.total, false);   // in place, like the reference
    lap(3);
}

// The host half, on the loop thread: the reference's message logic and
// onMessage callbacks, connection by connection in submission order.
// $HVWS_EXPERIMENT replay_prefetch (bytes, default 64 KiB; 0 = off): while connection i
// replays, the next connections' read bytes -- just written by the device
// across PCIe, so in DRAM, not in any cache -- are prefetched up to this far
// ahead; the appends otherwise wait on DRAM a few cache lines at a time.
const uint64_t g_replay_prefetch =
    hvws::experiment("replay_prefetch") ? strtoull(hvws::experiment("replay_prefetch"), nullptr, 0) : (64u << 10);

// Replays running on this thread (nested when an onMessage feeds again).
// While one runs, the states of its parsers after the one being replayed --
// and of every parser in a feeder's in-flight run -- are already decided by
// carries taken before any callback: a nested feed on such a parser would be
// overwritten when its turn comes, so it is refused (parser_busy).  The
// indexes are built only when a nested feed actually asks.
struct replay_scope {
    const feed_batch* b;
    const int* pos;                // index in b being replayed
    const feed_batch* inflight;    // feeder: run whose device half is issued, or nullptr
    ptr_index idx_b, idx_f;
    bool built = false;
};
thread_local std::vector<replay_scope*> t_replays;

void replay_part(feed_batch& b, const feed_batch* inflight = nullptr) {
    double t0 = g_ft.on ? now_us() : 0;
    int i = 0;
    replay_scope scope{&b, &i, inflight};
    struct push {   // popped however the replay ends (an onMessage may throw)
        explicit push(replay_scope* s) { t_replays.push_back(s); }
        ~push() { t_replays.pop_back(); }
    } pushed(&scope);
    int pf_conn = 0;          // next connection whose bytes to prefetch
    uint64_t pf_off = 0;      // ... from this offset in its read
    uint64_t pf_ahead = 0;    // bytes prefetched beyond the connection being replayed
    for (; i < b.n(); ++i) {
        if (g_replay_prefetch) {
            if (i) pf_ahead = pf_ahead > b.len[i] ? pf_ahead - b.len[i] : 0;   // connection i is no longer ahead
            if (pf_conn <= i) {
                pf_conn = i + 1;
                pf_off = 0;
                pf_ahead = 0;
            }
            while (pf_conn < b.n() && pf_ahead < g_replay_prefetch) {
                const char* p = b.data[pf_conn];
                const uint64_t n = b.len[pf_conn];
                for (; pf_off < n && pf_ahead < g_replay_prefetch; pf_off += 64, pf_ahead += 64) __builtin_prefetch(p + pf_off);
                if (pf_off >= n) {
                    ++pf_conn;
                    pf_off = 0;
                }
            }
        }
        char* dst = const_cast<char*>(b.data[i]);
        b.carry[i].data = b.parsers[i]->parser->data;
        const size_t used = replay_messages(b.parsers[i], dst, b.mapped ? 0 : b.segs[i].off, b.frames.data() + b.first[i],
                                            (size_t)b.count[i], b.carry[i], b.len[i]);
        if (b.rets) b.rets[i] = (int)used;
    }
    if (g_ft.on) g_ft.add(4, now_us() - t0);
}

// True when a feed of `p` now (from inside a replayed callback) would be
// overwritten by a replay still to come on this thread.
bool parser_busy(const WebSocketParser* p) {
    for (replay_scope* s : t_replays) {
        if (!s->built) {
            s->idx_b.reset((size_t)s->b->n());
            for (int k = 0; k < s->b->n(); ++k) s->idx_b.insert(s->b->parsers[k], k);
            if (s->inflight) {
                s->idx_f.reset((size_t)s->inflight->n());
                for (int k = 0; k < s->inflight->n(); ++k) s->idx_f.insert(s->inflight->parsers[k], k);
            }
            s->built = true;
        }
        if (s->idx_b.find(p) > *s->pos) return true;
        if (s->inflight && s->idx_f.find(p) >= 0) return true;
    }
    return false;
}

bool any_busy(WebSocketParser* const* parsers, int n) {
    if (t_replays.empty()) return false;
    for (int i = 0; i < n; ++i)
        if (parser_busy(parsers[i])) return true;
    return false;
}
}  // namespace

static int feed_distinct(WebSocketParser* const* parsers, const char* const* data, const size_t* len, int n,
                         int* rets) {
    if (n <= 0) return 0;
    double t0 = g_ft.on ? now_us() : 0;
    feed_batch b;   // local: an onMessage may feed again on this thread
    b.set(parsers, data, len, n, rets);
    for (int i = 0; i < n; ++i) hvws::copy_parser(b.carry[i], *parsers[i]->parser);
    if (g_ft.on) g_ft.add(0, now_us() - t0);
    gpu_part(b);
    replay_part(b);
    if (g_ft.on) g_ft.call();
    return n;
}

// ------------------------------------------------------------ pipelined feed
// hvws_feeder: the device half of poll iteration k
// (gather, GPU round trip, write-back) runs on the feeder's worker thread,
// on that thread's own context, stream and pinned stage, while the loop
// thread replays iteration k-1's message logic and onMessage callbacks.
// Callbacks arrive one submission late; their order is hvws_feed_many's.
struct hvws_feeder {
    int device = 0;
    hvws_ctx* src = nullptr;         // creating thread's context (settings), until the worker started
    bool started = false;
    std::thread worker;
    std::mutex m;
    std::condition_variable cv;
    feed_batch slot[2];
    int next = 0;                    // slot the next run fills (the other one may be pending)
    std::atomic<feed_batch*> job{nullptr};   // handed to the worker, device half not finished
    feed_batch* pending = nullptr;   // device half issued, callbacks not replayed yet
    bool stop = false;
    bool in_replay = false;
    bool free_requested = false;     // hvws_feeder_free from one of its callbacks: freed when the replay returns
    uint64_t inline_bytes = 0;      // runs up to this size skip the worker ($HVWS_EXPERIMENT feeder_inline)
    ptr_index pend_idx;              // parser -> index in *pending (valid while pending is set)
};

namespace {
// Hand-offs spin briefly before blocking: an event loop submits every poll
// iteration, and a futex wake-up costs ~10-20 us against ~30-50 us round trips.
constexpr int kFeederSpinUs = 50;

template <class Pred>
bool spin_until(Pred p) {
    const auto t_end = std::chrono::steady_clock::now() + std::chrono::microseconds(kFeederSpinUs);
    for (int i = 0;; ++i) {
        if (p()) return true;
        if ((i & 63) == 63 && std::chrono::steady_clock::now() > t_end) return false;
        __builtin_ia32_pause();
    }
}

void feeder_main(hvws_feeder* f) {
    hvws_set_thread_device(f->device);
    {
        std::lock_guard<std::mutex> lk(f->m);
        hvws::ctx_copy_settings(hvws::thread_ctx(), f->src);
        f->src = nullptr;
        f->started = true;
    }
    f->cv.notify_all();
    for (;;) {
        feed_batch* b = nullptr;
        if (!spin_until([&] { return (b = f->job.load(std::memory_order_acquire)) != nullptr; })) {
            std::unique_lock<std::mutex> lk(f->m);
            f->cv.wait(lk, [&] { return (b = f->job.load(std::memory_order_acquire)) != nullptr || f->stop; });
            if (!b) break;
        }
        gpu_part(*b);
        {
            std::lock_guard<std::mutex> lk(f->m);
            f->job.store(nullptr, std::memory_order_release);
        }
        f->cv.notify_all();
    }
    hvws_thread_release();
}

void feeder_wait_idle(hvws_feeder* f) {
    const double t0 = g_ft.on ? now_us() : 0;
    if (!spin_until([f] { return f->job.load(std::memory_order_acquire) == nullptr; })) {
        std::unique_lock<std::mutex> lk(f->m);
        f->cv.wait(lk, [f] { return f->job.load(std::memory_order_acquire) == nullptr; });
    }
    if (g_ft.on) g_ft.add(5, now_us() - t0);
}

void feeder_replay_pending(hvws_feeder* f, const feed_batch* inflight = nullptr) {
    if (!f->pending) return;
    f->in_replay = true;
    replay_part(*f->pending, inflight);
    f->in_replay = false;
    f->pending = nullptr;
}

// One run of distinct parsers: start its device half, then replay the
// previous run while it is in flight.
void feeder_run(hvws_feeder* f, WebSocketParser* const* parsers, const char* const* data, const size_t* len, int n,
                int* rets) {
    feed_batch& b = f->slot[f->next];
    f->next ^= 1;
    b.set(parsers, data, len, n, rets);
    // The previous run's device half has produced its carries; a parser it
    // holds continues from there (its own state is only written by the
    // replay below), any other parser from its own state.
    feeder_wait_idle(f);
    for (int i = 0; i < n; ++i) {
        const int k = f->pending ? f->pend_idx.find(parsers[i]) : -1;
        if (k >= 0) hvws::copy_parser(b.carry[i], f->pending->carry[k]);
        else hvws::copy_parser(b.carry[i], *parsers[i]->parser);
    }
    if (g_ft.on) g_ft.call();
    if (b.total <= f->inline_bytes) {
        // Too small for the hand-off to pay: the device half on this thread
        // (its own context), then the previous run's replay.
        gpu_part(b);
    } else {
        {
            std::lock_guard<std::mutex> lk(f->m);
            f->job.store(&b, std::memory_order_release);
        }
        f->cv.notify_all();
    }
    feeder_replay_pending(f, &b);
    f->pending = &b;
    f->pend_idx.reset((size_t)n);
    for (int i = 0; i < n; ++i) f->pend_idx.insert(parsers[i], i);   // distinct within a run
}
}  // namespace

extern "C" hvws_feeder* hvws_feeder_new(void) {
    hvws_feeder* f = new hvws_feeder();
    if (const char* e = hvws::experiment("feeder_inline")) f->inline_bytes = strtoull(e, nullptr, 0);
    f->src = hvws::thread_ctx();
    f->device = hvws_ctx_device(f->src);
    f->worker = std::thread(feeder_main, f);
    std::unique_lock<std::mutex> lk(f->m);
    f->cv.wait(lk, [f] { return f->started; });
    return f;
}

namespace {
void feeder_destroy(hvws_feeder* f) {
    feeder_wait_idle(f);
    feeder_replay_pending(f);
    {
        std::lock_guard<std::mutex> lk(f->m);
        f->stop = true;
    }
    f->cv.notify_all();
    f->worker.join();
    delete f;
}

// Ends a top-level submit / flush: a free asked for by one of its callbacks
// happens now that the replay has returned.  Returns rc.
int feeder_settle(hvws_feeder* f, int rc) {
    if (!f->free_requested) return rc;
    feeder_destroy(f);
    return rc;
}
}  // namespace

extern "C" int hvws_feeder_flush(hvws_feeder* f) {
    if (!f) return -1;
    if (f->in_replay) return -1;   // from inside one of its own callbacks
    feeder_wait_idle(f);
    feeder_replay_pending(f);
    return feeder_settle(f, 0);
}

extern "C" void hvws_feeder_free(hvws_feeder* f) {
    if (!f) return;
    if (f->in_replay) {
        // From inside one of its own callbacks: the replay that called it is
        // still iterating this feeder's run.  Freed when that submit / flush
        // returns (after the rest of its callbacks).
        f->free_requested = true;
        return;
    }
    feeder_destroy(f);
}

int hvws_feeder_submit(hvws_feeder* f, WebSocketParser* const* parsers, const char* const* data, const size_t* len,
                       int n, int* rets) {
    if (!f || n < 0 || f->in_replay || f->free_requested) return -1;
    if (n == 0) return hvws_feeder_flush(f);
    if (any_busy(parsers, n)) return -1;   // from another replay on this thread that would overwrite these
    // as hvws_feed_many: a parser seen twice starts a new run
    int done = 0;
    while (done < n && !f->free_requested) {
        const int end = distinct_run_end(parsers, done, n);
        feeder_run(f, parsers + done, data + done, len + done, end - done, rets ? rets + done : nullptr);
        done = end;
    }
    // freed from a callback: the runs not started yet are dropped (their
    // rets untouched); the count says how many reads were taken
    return feeder_settle(f, done);
}

// ---------------------------------------------------------------- C handle
namespace {
struct wsp_handle {
    WebSocketParser p;
    hvws_msg_cb cb = nullptr;
    void* user = nullptr;
};
}  // namespace

extern "C" {

void* hvws_wsp_new(void) { return new wsp_handle(); }

void hvws_wsp_free(void* h) { delete (wsp_handle*)h; }

void hvws_wsp_set_sink(void* h, hvws_msg_cb cb, void* user) {
    wsp_handle* w = (wsp_handle*)h;
    w->cb = cb;
    w->user = user;
    if (cb)
        w->p.onMessage = [w](int op, const std::string& msg) { w->cb(w->user, op, msg.data(), msg.size()); };
    else
        w->p.onMessage = nullptr;
}

int hvws_wsp_feed(void* h, const char* data, size_t len) { return ((wsp_handle*)h)->p.FeedRecvData(data, len); }

int hvws_wsp_feed_many(void* const* handles, const char* const* data, const size_t* len, int n, int* rets) {
    std::vector<WebSocketParser*> ps((size_t)(n > 0 ? n : 0));
    for (int i = 0; i < n; ++i) ps[i] = &((wsp_handle*)handles[i])->p;
    return hvws_feed_many(ps.data(), data, len, n, rets);
}

int hvws_wsp_feeder_submit(hvws_feeder* f, void* const* handles, const char* const* data, const size_t* len, int n,
                           int* rets) {
    std::vector<WebSocketParser*> ps((size_t)(n > 0 ? n : 0));
    for (int i = 0; i < n; ++i) ps[i] = &((wsp_handle*)handles[i])->p;
    return hvws_feeder_submit(f, ps.data(), data, len, n, rets);
}

void hvws_wsp_state(void* h, uint64_t out[8]) {
    wsp_handle* w = (wsp_handle*)h;
    websocket_parser* p = w->p.parser;
    uint32_t m;
    memcpy(&m, p->mask, 4);
    out[0] = p->state;
    out[1] = (uint64_t)p->flags;
    out[2] = m;
    out[3] = p->mask_offset;
    out[4] = p->length;
    out[5] = p->require;
    out[6] = p->offset;
    out[7] = (uint64_t)w->p.state | ((uint64_t)(uint32_t)w->p.opcode << 32);
}

}  // extern "C"

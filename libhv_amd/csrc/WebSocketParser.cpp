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

#include <chrono>
#include <unordered_set>
#include <vector>

#include "hvws.h"
#include "hvws_internal.h"

namespace hvws {
[[noreturn]] void fatal(const char* what);
hvws_ctx* thread_ctx();
char* pinned_stage(uint64_t bytes);
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
const int kMaxReserve = 1 << 24;   // MAX_PAYLOAD_LENGTH, reference WebSocketParser.cpp:6
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
    // A connection's second chunk needs the carry its first chunk leaves, so
    // cut the batch before any parser that already appears in it.
    int done = 0;
    while (done < n) {
        int end = done;
        std::unordered_set<WebSocketParser*> seen;
        while (end < n && seen.insert(parsers[end]).second) ++end;
        feed_distinct(parsers + done, data + done, len + done, end - done, rets ? rets + done : nullptr);
        done = end;
    }
    return n;
}

namespace {
// $HVWS_FEED_TIMES=1: per-phase host time of feed_distinct, printed at exit (diagnostic)
struct feed_times {
    double ph[5] = {0, 0, 0, 0, 0};
    long calls = 0;
    bool on = getenv("HVWS_FEED_TIMES") && atoi(getenv("HVWS_FEED_TIMES"));
    ~feed_times() {
        if (on && calls)
            fprintf(stderr, "[feed_times] calls=%ld us/call: carry %.1f gather %.1f gpu %.1f scatter %.1f replay %.1f\n",
                    calls, ph[0] / calls, ph[1] / calls, ph[2] / calls, ph[3] / calls, ph[4] / calls);
    }
} g_ft;
double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
}  // namespace

static int feed_distinct(WebSocketParser* const* parsers, const char* const* data, const size_t* len, int n,
                         int* rets) {
    if (n <= 0) return 0;
    double t0 = g_ft.on ? now_us() : 0, t1;
    auto lap = [&](int k) {
        if (!g_ft.on) return;
        t1 = now_us();
        g_ft.ph[k] += t1 - t0;
        t0 = t1;
    };
    std::vector<hvws_segment> segs((size_t)n);
    std::vector<websocket_parser> carry((size_t)n);
    uint64_t total = 0;
    for (int i = 0; i < n; ++i) {
        segs[i].off = total;
        segs[i].len = len[i];
        total += len[i];
        hvws::copy_parser(carry[i], *parsers[i]->parser);
    }
    lap(0);
    char* stage = hvws::pinned_stage(total);
    stage_copy(stage, segs.data(), data, len, n, total, true);
    lap(1);
    hvws_ctx* c = hvws::thread_ctx();
    if (hvws_rx_batch(c, (uint8_t*)stage, total, segs.data(), carry.data(), (uint32_t)n, 1) != HVWS_OK)
        hvws::fatal("hvws_rx_batch");
    const int64_t nf = hvws_frame_count(c);
    std::vector<hvws_frame> frames((size_t)(nf > 0 ? nf : 0));
    std::vector<uint64_t> first((size_t)n), count((size_t)n);
    if ((nf > 0 && hvws_get_frames(c, frames.data(), 0, (uint64_t)nf) != HVWS_OK) ||
        hvws_get_segment_frames(c, first.data(), count.data()) != HVWS_OK)
        hvws::fatal("frame table read-back");
    lap(2);
    // Every segment leaves the (thread's, reusable) stage before any callback
    // runs: an onMessage that feeds again on this thread restages it.
    stage_copy(stage, segs.data(), data, len, n, total, false);   // in place, like the reference
    lap(3);
    for (int i = 0; i < n; ++i) {
        char* dst = const_cast<char*>(data[i]);
        carry[i].data = parsers[i]->parser->data;
        const size_t used =
            replay_messages(parsers[i], dst, segs[i].off, frames.data() + first[i], (size_t)count[i], carry[i], len[i]);
        if (rets) rets[i] = (int)used;
    }
    lap(4);
    g_ft.calls += g_ft.on;
    return n;
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

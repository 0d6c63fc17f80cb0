// hvws_lagged.cpp -- lagged steps: two scan chains in flight.
//
// hvws_step_resident waits in the host for its own scan's verdict before it
// returns, so only one scan chain is ever in flight beside one unmask and a
// step takes max(chain, unmask).  A lagged stepper runs consecutive steps on
// two contexts of the same device from two worker threads, so two chains can
// be in flight.  Measured for config 4 as one stream (DESIGN.md sec. 9.1,
// profiles/r5_raw/lagged): 1.70-1.78 ms per step against 1.58 resident --
// the resident chain already fits beside the unmask, each context's chain
// runs beside its own context's unmask only, and the second chain's link
// walks slow the unmask -- so this stays an opt-in API.  Unmasks stay in
// step order: before its first unmask is queued, step k waits in the host
// until step k-1 has queued all of its own, and its context's stream waits
// on the event recorded behind them.  The batch passed to hvws_lagged_step is
// unmasked by the time a later call or hvws_lagged_sync returns -- not when
// this call returns (hvws_step_resident's contract is unchanged).
//
// Reference: one loop per connection parses its frames strictly in order
// (http/websocket_parser.c:53-171, http/server/HttpHandler.cpp:757-763);
// here the frames of one batch are still unmasked from that batch's exact
// scan, only the host's wait for batch k moves behind batch k+1's launch.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <string.h>

#include <condition_variable>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "hvws.h"
#include "hvws_internal.h"

namespace {

struct lag_worker {
    hvws_ctx* ctx = nullptr;
    std::thread th;
    std::mutex m;
    std::condition_variable cv;
    bool has_job = false, quit = false;
    // the job
    uint8_t* rx = nullptr;
    uint64_t len = 0;
    std::vector<hvws_segment> segs;
    std::vector<websocket_parser> carry;
    bool has_carry = false;
    uint64_t seq = 0;
    hipEvent_t done_ev = nullptr;   // behind this worker's last step's unmasks, on its context's stream
};

}  // namespace

struct hvws_lagged {
    int device = 0;
    lag_worker w[2];
    std::mutex om;                  // issued_seq, err
    std::condition_variable ocv;
    uint64_t issued_seq = 0;        // the last step whose unmasks are all queued (and its done_ev recorded)
    uint64_t next_seq = 1;
    int err = HVWS_OK;
    std::string err_msg;
};

namespace {

void lag_fail(hvws_lagged* L, int rc, const char* what) {
    std::lock_guard<std::mutex> lk(L->om);
    if (L->err == HVWS_OK) {
        L->err = rc;
        L->err_msg = what;
    }
}

void lag_run(hvws_lagged* L, int i) {
    lag_worker& W = L->w[i];
    lag_worker& P = L->w[i ^ 1];
    hipSetDevice(L->device);   // (each call also sets its context's device)
    for (;;) {
        std::unique_lock<std::mutex> lk(W.m);
        W.cv.wait(lk, [&] { return W.has_job || W.quit; });
        if (W.quit && !W.has_job) return;
        const uint64_t seq = W.seq;
        lk.unlock();
        // Before this step's first unmask: the previous step has queued all of
        // its unmasks (it did so right after its own scan's verdict), and this
        // context's stream waits for them.
        hvws::ctx_arm_lag(W.ctx, [&, seq] {
            std::unique_lock<std::mutex> ol(L->om);
            L->ocv.wait(ol, [&] { return L->issued_seq + 1 >= seq || L->err != HVWS_OK; });
            ol.unlock();
            if (seq > 1 && hipStreamWaitEvent(hvws::ctx_stream(W.ctx), P.done_ev, 0) != hipSuccess)
                lag_fail(L, HVWS_EHIP, "hipStreamWaitEvent (previous lagged step)");
        });
        const int rc = hvws_step_resident(W.ctx, W.rx, W.len, W.segs.data(), W.has_carry ? W.carry.data() : nullptr,
                                          (uint32_t)W.segs.size());
        if (rc != HVWS_OK) lag_fail(L, rc, hvws_last_error());
        hvws::ctx_lag_fire(W.ctx);   // a step that queued no unmask still keeps the order
        if (hipEventRecord(W.done_ev, hvws::ctx_stream(W.ctx)) != hipSuccess) lag_fail(L, HVWS_EHIP, "hipEventRecord");
        {
            std::lock_guard<std::mutex> ol(L->om);
            L->issued_seq = seq;
        }
        L->ocv.notify_all();
        lk.lock();
        W.has_job = false;
        lk.unlock();
        W.cv.notify_all();
    }
}

int lag_idle(hvws_lagged* L, int i) {   // wait until worker i holds no job
    lag_worker& W = L->w[i];
    std::unique_lock<std::mutex> lk(W.m);
    W.cv.wait(lk, [&] { return !W.has_job; });
    return HVWS_OK;
}

}  // namespace

extern "C" {

hvws_lagged* hvws_lagged_new(int device) {
    hvws_lagged* L = new hvws_lagged();
    L->device = device;
    for (int i = 0; i < 2; ++i) {
        L->w[i].ctx = hvws_ctx_create(device);
        if (!L->w[i].ctx || hipSetDevice(device) != hipSuccess ||
            hipEventCreateWithFlags(&L->w[i].done_ev, hipEventDisableTiming) != hipSuccess) {
            for (int j = 0; j <= i; ++j) {
                if (L->w[j].done_ev) hipEventDestroy(L->w[j].done_ev);
                if (L->w[j].ctx) hvws_ctx_destroy(L->w[j].ctx);
            }
            delete L;
            return nullptr;
        }
    }
    for (int i = 0; i < 2; ++i) L->w[i].th = std::thread(lag_run, L, i);
    return L;
}

int hvws_lagged_step(hvws_lagged* L, uint8_t* d_rx, uint64_t rx_len, const hvws_segment* segs,
                     const websocket_parser* carry_in, uint32_t nseg) {
    if (!L || (!segs && nseg)) return HVWS_EINVAL;
    {
        std::lock_guard<std::mutex> ol(L->om);
        if (L->err != HVWS_OK) return L->err;
    }
    const uint64_t seq = L->next_seq++;
    const int i = (int)(seq & 1u);
    lag_idle(L, i);   // that worker's step two back has returned (at most two chains in flight)
    lag_worker& W = L->w[i];
    {
        std::lock_guard<std::mutex> lk(W.m);
        W.rx = d_rx;
        W.len = rx_len;
        W.segs.assign(segs, segs + nseg);
        W.has_carry = carry_in != nullptr;
        if (carry_in) W.carry.assign(carry_in, carry_in + nseg);
        W.seq = seq;
        W.has_job = true;
    }
    W.cv.notify_all();
    std::lock_guard<std::mutex> ol(L->om);
    return L->err;
}

int hvws_lagged_sync(hvws_lagged* L) {
    if (!L) return HVWS_EINVAL;
    for (int i = 0; i < 2; ++i) lag_idle(L, i);
    for (int i = 0; i < 2; ++i) {
        if (hipSetDevice(L->device) != hipSuccess || hipStreamSynchronize(hvws::ctx_stream(L->w[i].ctx)) != hipSuccess ||
            hipStreamSynchronize(hvws::ctx_scan_stream(L->w[i].ctx)) != hipSuccess)
            lag_fail(L, HVWS_EHIP, "hipStreamSynchronize (lagged)");
    }
    std::lock_guard<std::mutex> ol(L->om);
    return L->err;
}

hvws_ctx* hvws_lagged_context(hvws_lagged* L, int i) { return L && (i == 0 || i == 1) ? L->w[i].ctx : nullptr; }

const char* hvws_lagged_error(hvws_lagged* L) {
    if (!L) return "";
    std::lock_guard<std::mutex> ol(L->om);
    return L->err_msg.c_str();
}

void hvws_lagged_free(hvws_lagged* L) {
    if (!L) return;
    hvws_lagged_sync(L);
    for (int i = 0; i < 2; ++i) {
        {
            std::lock_guard<std::mutex> lk(L->w[i].m);
            L->w[i].quit = true;
        }
        L->w[i].cv.notify_all();
        L->w[i].th.join();
    }
    for (int i = 0; i < 2; ++i) {
        hipEventDestroy(L->w[i].done_ev);
        hvws_ctx_destroy(L->w[i].ctx);
    }
    delete L;
}

}  // extern "C"

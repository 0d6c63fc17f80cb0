// vram_probe.hip -- design probe (not product code) for the resident
// worker's request path: can the host write requests and read bytes straight
// into device memory (fine-grained VRAM through the PCIe BAR), so the worker
// polls its own HBM instead of host memory across PCIe, and stages a read from
// HBM instead of pulling it over the link?  Measures ping-pong round trips
// (host posts seq, the worker answers done = seq in pinned host memory) and
// the same with an 8 KiB read carried each way:
//   A  mailbox + data in pinned host memory (the round-3 worker)
//   B  mailbox + data in fine-grained device memory written by the host
// Every wait in the kernel is bounded (2 s without a request ends it).
//   hipcc --offload-arch=gfx950 -O2 scripts/probe/vram_probe.hip -o build/vram_probe
#include <hip/hip_runtime.h>
#include <setjmp.h>
#include <signal.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <vector>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

struct box_t {
    uint64_t seq, len, pad[6];
    uint64_t done, pad2[7];
};

// the worker: one workgroup of 256 threads
__global__ void k_pong(box_t* req, box_t* ans, uint8_t* din, uint8_t* dout, uint64_t n) {
    __shared__ uint64_t s_seq, s_len;
    __shared__ uint32_t s_quit;
    const uint32_t tid = threadIdx.x;
    uint64_t last = 0;
    for (uint64_t i = 0; i < n; ++i) {
        if (tid == 0) {
            const uint64_t t0 = wall_clock64();
            uint64_t s;
            uint32_t quit = 0;
            for (;;) {
                s = __hip_atomic_load(&req->seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                if (s != last) break;
                if (wall_clock64() - t0 > 200000000ull) {   // 2 s
                    quit = 1;
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
            s_seq = s;
            s_len = __hip_atomic_load(&req->len, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            s_quit = quit;
        }
        __syncthreads();
        if (s_quit) return;
        const uint64_t L = s_len;
        for (uint64_t c = (uint64_t)tid * 16; c < L; c += 256 * 16) {
            const u32x4 v = *reinterpret_cast<const u32x4*>(din + c);
            *reinterpret_cast<u32x4*>(dout + c) = v ^ u32x4{0x5A5A5A5Au, 0x5A5A5A5Au, 0x5A5A5A5Au, 0x5A5A5A5Au};
        }
        __threadfence_system();
        __syncthreads();
        last = s_seq;
        if (tid == 0) __hip_atomic_store(&ans->done, last, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

#define CK(x)                                                                  \
    do {                                                                       \
        hipError_t e_ = (x);                                                   \
        if (e_ != hipSuccess) {                                                \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));            \
            exit(1);                                                           \
        }                                                                      \
    } while (0)

static sigjmp_buf g_jb;
static void on_segv(int) { siglongjmp(g_jb, 1); }

// true when the host can store to and load from p
static bool host_can_touch(void* p) {
    struct sigaction sa = {}, old_segv = {}, old_bus = {};
    sa.sa_handler = on_segv;
    sigemptyset(&sa.sa_mask);
    sigaction(SIGSEGV, &sa, &old_segv);
    sigaction(SIGBUS, &sa, &old_bus);
    bool ok = false;
    if (sigsetjmp(g_jb, 1) == 0) {
        volatile uint64_t* q = reinterpret_cast<volatile uint64_t*>(p);
        q[0] = 0x1234;
        ok = q[0] == 0x1234;
    }
    sigaction(SIGSEGV, &old_segv, nullptr);
    sigaction(SIGBUS, &old_bus, nullptr);
    return ok;
}

static void run(const char* name, box_t* req_h, box_t* req_d, uint8_t* din_h, uint8_t* din_d, box_t* ans_h,
                box_t* ans_d, uint8_t* dout_h, uint8_t* dout_d, uint64_t len, int pings) {
    std::vector<uint8_t> src(len), dst(len);
    for (uint64_t i = 0; i < len; ++i) src[i] = (uint8_t)(i * 7 + 1);
    memset(ans_h, 0, sizeof(box_t));
    *(volatile uint64_t*)&req_h->seq = 0;
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    hipLaunchKernelGGL(k_pong, dim3(1), dim3(256), 0, st, req_d, ans_d, din_d, dout_d, (uint64_t)pings);
    CK(hipGetLastError());
    std::vector<double> us;
    int bad = 0;
    for (int i = 1; i <= pings; ++i) {
        const auto t0 = std::chrono::steady_clock::now();
        if (len) memcpy(din_h, src.data(), len);
        *(volatile uint64_t*)&req_h->len = len;
        __atomic_store_n(&req_h->seq, (uint64_t)i, __ATOMIC_RELEASE);
        while (__atomic_load_n(&ans_h->done, __ATOMIC_ACQUIRE) != (uint64_t)i) {
            if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(3)) {
                fprintf(stderr, "%s: no answer\n", name);
                exit(2);
            }
        }
        if (len) memcpy(dst.data(), dout_h, len);
        us.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
        if (len && (dst[0] != (src[0] ^ 0x5A) || dst[len - 1] != (src[len - 1] ^ 0x5A))) ++bad;
    }
    CK(hipStreamSynchronize(st));
    CK(hipStreamDestroy(st));
    std::sort(us.begin(), us.end());
    printf("{\"mode\": \"%s\", \"bytes\": %llu, \"pings\": %d, \"median_us\": %.2f, \"p10_us\": %.2f, \"p90_us\": %.2f, "
           "\"bad\": %d}\n",
           name, (unsigned long long)len, pings, us[us.size() / 2], us[us.size() / 10], us[us.size() * 9 / 10], bad);
    fflush(stdout);
}

int main() {
    CK(hipSetDevice(0));
    const uint64_t N = 64 << 10;
    // pinned host: mailbox (coherent), data in and out
    box_t *hreq, *hans;
    uint8_t *hin, *hout;
    CK(hipHostMalloc((void**)&hreq, sizeof(box_t), hipHostMallocCoherent));
    CK(hipHostMalloc((void**)&hans, sizeof(box_t), hipHostMallocCoherent));
    CK(hipHostMalloc((void**)&hin, N, 0));
    CK(hipHostMalloc((void**)&hout, N, 0));
    box_t *dreq_h, *dans_h;
    uint8_t *din_h, *dout_h;
    CK(hipHostGetDevicePointer((void**)&dreq_h, hreq, 0));
    CK(hipHostGetDevicePointer((void**)&dans_h, hans, 0));
    CK(hipHostGetDevicePointer((void**)&din_h, hin, 0));
    CK(hipHostGetDevicePointer((void**)&dout_h, hout, 0));
    for (uint64_t len : {0ull, 8192ull}) run("A_pinned_host", hreq, dreq_h, hin, din_h, hans, dans_h, hout, dout_h, len, 3000);
    // fine-grained device memory: can the host reach it?
    for (unsigned flags : {(unsigned)hipDeviceMallocFinegrained, (unsigned)hipDeviceMallocUncached}) {
        box_t* vreq = nullptr;
        uint8_t* vin = nullptr;
        if (hipExtMallocWithFlags((void**)&vreq, 4096, flags) != hipSuccess ||
            hipExtMallocWithFlags((void**)&vin, N, flags) != hipSuccess) {
            printf("{\"flags\": %u, \"alloc\": false}\n", flags);
            continue;
        }
        const bool touch = host_can_touch(vreq) && host_can_touch(vin);
        printf("{\"flags\": %u, \"alloc\": true, \"host_access\": %s}\n", flags, touch ? "true" : "false");
        fflush(stdout);
        if (touch) {
            // host write bandwidth into it (8 KiB memcpy)
            std::vector<uint8_t> src(8192, 3);
            const auto t0 = std::chrono::steady_clock::now();
            for (int i = 0; i < 2000; ++i) memcpy(vin, src.data(), 8192);
            const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() / 2000;
            printf("{\"flags\": %u, \"host_memcpy_8KiB_us\": %.2f}\n", flags, us);
            for (uint64_t len : {0ull, 8192ull})
                run(flags == hipDeviceMallocFinegrained ? "B_vram_finegrained" : "B_vram_uncached", vreq, vreq, vin, vin,
                    hans, dans_h, hout, dout_h, len, 3000);
        }
        CK(hipFree(vreq));
        CK(hipFree(vin));
    }
    return 0;
}

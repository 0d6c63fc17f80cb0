// query_probe.hip -- design probe (not product code): can hipStreamQuery
// report a stream idle while the kernel last launched on it is still
// running?  Round 3's k_door park trusted exactly that (alive == 0 plus
// hipStreamQuery == hipSuccess meant "the worker has ended", and the stream
// was then destroyed and the mailbox freed); two of four bench runs with
// that rule hung in the next leg.
//
// k_linger mimics the worker's exit: thread 0 clears `alive` (system scope),
// then stays for `linger` ticks of the 100 MHz clock while bumping a
// heartbeat, then stores `exited = epoch` as its last write and returns.  The
// host waits for alive == 0 and then polls hipStreamQuery, recording whether
// it ever answered hipSuccess while `exited` still lagged (the kernel still
// running) -- on a CU-masked stream (the worker's) and on an ordinary one.
//   hipcc --offload-arch=gfx950 -O2 scripts/probe/query_probe.hip -o build/query_probe
//   build/query_probe [rounds]   -> one JSON line per (stream kind, linger)
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <chrono>
#include <vector>

struct box_t {
    uint64_t alive, exited, beat, pad[5];
};

__global__ void k_linger(box_t* b, uint64_t linger, uint64_t epoch) {
    if (threadIdx.x != 0) return;
    __hip_atomic_store(&b->alive, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __threadfence_system();
    const uint64_t t0 = wall_clock64();
    uint64_t n = 0;
    while (wall_clock64() - t0 < linger) {
        __hip_atomic_store(&b->beat, ++n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __builtin_amdgcn_s_sleep(8);
    }
    __threadfence_system();
    __hip_atomic_store(&b->exited, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                        \
            exit(1);                                                                       \
        }                                                                                  \
    } while (0)

int main(int argc, char** argv) {
    const int rounds = argc > 1 ? atoi(argv[1]) : 300;
    CK(hipSetDevice(0));
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    std::vector<uint32_t> mask((size_t)(prop.multiProcessorCount + 31) / 32, 0u);
    for (int i = 0; i < prop.multiProcessorCount; ++i) mask[(size_t)i / 32] |= 1u << (i % 32);
    hipStream_t masked, plain;
    CK(hipExtStreamCreateWithCUMask(&masked, (uint32_t)mask.size(), mask.data()));
    CK(hipStreamCreateWithFlags(&plain, hipStreamNonBlocking));
    box_t* hb = nullptr;
    CK(hipHostMalloc((void**)&hb, sizeof(box_t), hipHostMallocCoherent));
    box_t* db = nullptr;
    CK(hipHostGetDevicePointer((void**)&db, hb, 0));
    uint64_t epoch = 0;
    const uint64_t lingers[] = {0, 1000, 10000};   // ticks: 0, 10 us, 100 us
    for (int kind = 0; kind < 2; ++kind) {
        hipStream_t st = kind == 0 ? masked : plain;
        for (uint64_t linger : lingers) {
            int early = 0, queries = 0;
            double worst_us = 0;
            for (int r = 0; r < rounds; ++r) {
                __atomic_store_n(&hb->alive, 1ull, __ATOMIC_RELEASE);
                ++epoch;
                hipLaunchKernelGGL(k_linger, dim3(1), dim3(64), 0, st, db, linger, epoch);
                CK(hipGetLastError());
                const auto t0 = std::chrono::steady_clock::now();
                while (__atomic_load_n(&hb->alive, __ATOMIC_ACQUIRE) != 0) {
                    if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(5)) {
                        fprintf(stderr, "kernel never started\n");
                        return 2;
                    }
                }
                for (;;) {
                    const hipError_t q = hipStreamQuery(st);
                    ++queries;
                    const uint64_t ex = __atomic_load_n(&hb->exited, __ATOMIC_ACQUIRE);
                    if (q == hipSuccess) {
                        if (ex != epoch) {   // idle by the query, not yet ended by the kernel's own word
                            ++early;
                            const auto t1 = std::chrono::steady_clock::now();
                            while (__atomic_load_n(&hb->exited, __ATOMIC_ACQUIRE) != epoch) {
                            }
                            const double us =
                                std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t1).count();
                            if (us > worst_us) worst_us = us;
                        }
                        break;
                    }
                    if (q != hipErrorNotReady) {
                        fprintf(stderr, "query: %s\n", hipGetErrorString(q));
                        return 3;
                    }
                }
                CK(hipStreamSynchronize(st));
            }
            printf("{\"stream\": \"%s\", \"linger_us\": %.1f, \"rounds\": %d, \"queries\": %d, "
                   "\"idle_before_exit\": %d, \"worst_lag_us\": %.2f}\n",
                   kind == 0 ? "cu_masked" : "plain", linger / 100.0, rounds, queries, early, worst_us);
            fflush(stdout);
        }
    }
    CK(hipStreamDestroy(masked));
    CK(hipStreamDestroy(plain));
    CK(hipHostFree(hb));
    return 0;
}

// membench2.hip -- design probe (not product code): geometry sweep of the
// in-place 16-B-per-lane XOR stream (k_unmask's access pattern) on MI355X.
// Variants interleaved round by round in one process (cdna guide rule 24).
//   build/membench2 <GiB> [rounds]
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <functional>
#include <string>
#include <vector>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

#define CK(x)                                                          \
    do {                                                               \
        hipError_t err_ = (x);                                         \
        if (err_ != hipSuccess) {                                      \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(err_));  \
            exit(1);                                                   \
        }                                                              \
    } while (0)

// SWZ 0: tile = blockIdx; 1: XCD-contiguous tile ranges (blocks b, b+8, ...
// share an XCD and walk adjacent tiles)
template <int T, int U, int SWZ>
__global__ __launch_bounds__(T) void k_inplace(u32x4* d, uint64_t n16, uint64_t ntiles, uint32_t pat) {
    uint64_t t = blockIdx.x;
    if (SWZ == 1) {
        const uint64_t q = ntiles / 8, r = ntiles % 8, x = t % 8, i = t / 8;
        t = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + i;
    }
    const uint64_t base = t * T * U;
    u32x4 v[U];
#pragma unroll
    for (int i = 0; i < U; ++i) {
        uint64_t c = base + (uint64_t)i * T + threadIdx.x;
        if (c < n16) v[i] = __builtin_nontemporal_load(d + c);
    }
#pragma unroll
    for (int i = 0; i < U; ++i) {
        uint64_t c = base + (uint64_t)i * T + threadIdx.x;
        if (c < n16) __builtin_nontemporal_store(v[i] ^ pat, d + c);
    }
}


// Same, with the bounds check hoisted to the tile (all loads back to back).
template <int T, int U, int SWZ, bool NT>
__global__ __launch_bounds__(T) void k_inplace2(u32x4* d, uint64_t n16, uint64_t ntiles, uint32_t pat) {
    uint64_t t = blockIdx.x;
    if (SWZ == 1) {
        const uint64_t q = ntiles / 8, r = ntiles % 8, x = t % 8, i = t / 8;
        t = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + i;
    }
    const uint64_t base = t * T * U;
    u32x4 v[U];
    if (base + (uint64_t)T * U <= n16) {
#pragma unroll
        for (int i = 0; i < U; ++i) {
            const u32x4* p = d + base + (uint64_t)i * T + threadIdx.x;
            v[i] = NT ? __builtin_nontemporal_load(p) : *p;
        }
#pragma unroll
        for (int i = 0; i < U; ++i) {
            u32x4* p = d + base + (uint64_t)i * T + threadIdx.x;
            if (NT) __builtin_nontemporal_store(v[i] ^ pat, p);
            else *p = v[i] ^ pat;
        }
    } else {
        for (int i = 0; i < U; ++i) {
            uint64_t c = base + (uint64_t)i * T + threadIdx.x;
            if (c < n16) d[c] = d[c] ^ pat;
        }
    }
}

// Each wave owns a contiguous (64*16*U)-byte run (wave-contiguous tiles).
template <int T, int U>
__global__ __launch_bounds__(T) void k_wavecontig(u32x4* d, uint64_t n16, uint32_t pat) {
    const uint64_t wave = (uint64_t)blockIdx.x * (T / 64) + threadIdx.x / 64;
    const uint64_t base = wave * 64 * U;
    const uint32_t lane = threadIdx.x & 63;
    u32x4 v[U];
#pragma unroll
    for (int i = 0; i < U; ++i) {
        uint64_t c = base + (uint64_t)i * 64 + lane;
        if (c < n16) v[i] = __builtin_nontemporal_load(d + c);
    }
#pragma unroll
    for (int i = 0; i < U; ++i) {
        uint64_t c = base + (uint64_t)i * 64 + lane;
        if (c < n16) __builtin_nontemporal_store(v[i] ^ pat, d + c);
    }
}

struct variant {
    std::string name;
    std::function<void()> run;
    std::vector<double> gbs;
};

int main(int argc, char** argv) {
    double gib = argc > 1 ? atof(argv[1]) : 16.0;
    int rounds = argc > 2 ? atoi(argv[2]) : 5;
    uint64_t bytes = (uint64_t)(gib * (1ull << 30)) & ~4095ull;
    uint64_t n16 = bytes / 16;
    u32x4* d;
    CK(hipMalloc(&d, bytes));
    CK(hipMemset(d, 1, bytes));
    std::vector<variant> vs;
#define INPL(T, U, S)                                                                                  \
    vs.push_back({"inplace T=" #T " U=" #U " swz=" #S, [&] {                                           \
                      uint64_t nt = (n16 + T * U - 1) / (T * U);                                       \
                      hipLaunchKernelGGL((k_inplace<T, U, S>), dim3((unsigned)nt), dim3(T), 0, 0, d, n16, nt, \
                                         0x5a5a5a5au);                                                 \
                  }, {}});
#define WAVEC(T, U)                                                                                    \
    vs.push_back({"wavecontig T=" #T " U=" #U, [&] {                                                   \
                      uint64_t nw = (n16 + 64 * U - 1) / (64 * U);                                     \
                      hipLaunchKernelGGL((k_wavecontig<T, U>), dim3((unsigned)((nw + T / 64 - 1) / (T / 64))), \
                                         dim3(T), 0, 0, d, n16, 0x5a5a5a5au);                          \
                  }, {}});
#define INPL2(T, U, S, NT)                                                                             \
    vs.push_back({"hoisted T=" #T " U=" #U " swz=" #S " nt=" #NT, [&] {                                  \
                      uint64_t nt = (n16 + T * U - 1) / (T * U);                                       \
                      hipLaunchKernelGGL((k_inplace2<T, U, S, NT>), dim3((unsigned)nt), dim3(T), 0, 0, d, n16, nt, \
                                         0x5a5a5a5au);                                                 \
                  }, {}});
    const char* set = getenv("MB_SET") ? getenv("MB_SET") : "a";
    if (set[0] == 'a') {
        INPL(64, 1, 0) INPL(64, 4, 0) INPL(128, 1, 0) INPL(128, 2, 0) INPL(256, 1, 0) INPL(256, 1, 1)
        INPL(512, 1, 0) INPL(512, 1, 1) INPL(1024, 1, 0) INPL(1024, 1, 1)
        INPL2(64, 4, 0, true) INPL2(64, 4, 1, true) INPL2(128, 2, 0, true) INPL2(128, 2, 1, true)
        INPL2(256, 1, 0, false) INPL2(64, 8, 0, true) INPL2(64, 16, 1, true)
        INPL(256, 2, 0) INPL2(256, 8, 1, true)
    } else {
        INPL(64, 1, 0) INPL(64, 4, 0) INPL(128, 2, 0) INPL(128, 2, 1) INPL(256, 2, 0)
        INPL2(64, 4, 0, true) INPL2(64, 4, 1, true) INPL2(64, 8, 1, true) INPL2(128, 2, 0, true)
        INPL2(128, 2, 1, true) INPL2(256, 8, 1, true)
    }
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (auto& v : vs) v.run();
    CK(hipDeviceSynchronize());
    for (int r = 0; r < rounds; ++r) {
        for (auto& v : vs) {
            CK(hipEventRecord(a));
            v.run();
            CK(hipEventRecord(b));
            CK(hipEventSynchronize(b));
            float ms;
            CK(hipEventElapsedTime(&ms, a, b));
            v.gbs.push_back(2.0 * bytes / (ms * 1e-3) / 1e9);
        }
    }
    printf("buffer %.2f GiB, %d rounds\n", bytes / double(1ull << 30), rounds);
    for (auto& v : vs) {
        std::sort(v.gbs.begin(), v.gbs.end());
        printf("%-30s median %7.1f  best %7.1f  worst %7.1f GB/s\n", v.name.c_str(), v.gbs[v.gbs.size() / 2],
               v.gbs.back(), v.gbs.front());
    }
    return 0;
}

// membench4.hip -- design probe (not product code): in-place 16-B XOR stream
// variants against k_unmask's geometry (256 threads x 4 chunks, XCD-contiguous
// tiles, nontemporal loads and stores), interleaved round by round.
//   membench4 <GiB> [rounds]
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

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

__device__ __forceinline__ uint64_t xcd_tile(uint64_t b, uint64_t ntiles) {
    const uint64_t q = ntiles >> 3, r = ntiles & 7u, x = b & 7u, i = b >> 3;
    return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + i;
}

// ORD 0: XCD-contiguous (k_unmask); 1: linear; 2: XCD-contiguous over two
// halves, alternate blocks of an XCD in the lower and upper half; 3: XCD order
// with the tile index bit-reversed inside 64-tile groups
template <int ORD>
__device__ __forceinline__ uint64_t tile_of(uint64_t b, uint64_t nt) {
    if constexpr (ORD == 0) return xcd_tile(b, nt);
    else if constexpr (ORD == 1) return b;
    else if constexpr (ORD == 2) {
        const uint64_t h = nt / 2;
        const uint64_t t = xcd_tile(b >> 1, h);
        return (b & 1) ? h + t : t;
    } else {
        const uint64_t t = xcd_tile(b, nt);
        const uint64_t g = t & ~63ull;
        const uint32_t r = __builtin_bitreverse32((uint32_t)(t & 63u)) >> 26;
        return g + r < nt ? g + r : t;
    }
}

template <int T, int U, int ORD>
__global__ __launch_bounds__(T) void k_ip(u32x4* d, uint64_t ntiles, uint32_t pat) {
    const uint64_t t = tile_of<ORD>(blockIdx.x, ntiles);
    u32x4* b = d + t * T * U;
    u32x4 v[U];
#pragma unroll
    for (int i = 0; i < U; ++i) v[i] = __builtin_nontemporal_load(b + i * T + threadIdx.x);
#pragma unroll
    for (int i = 0; i < U; ++i) __builtin_nontemporal_store(v[i] ^ pat, b + i * T + threadIdx.x);
}

// each block: two tiles half a buffer apart, all loads first
template <int T, int U>
__global__ __launch_bounds__(T) void k_ip2(u32x4* d, uint64_t ntiles, uint32_t pat) {
    const uint64_t h = ntiles / 2;
    const uint64_t t = xcd_tile(blockIdx.x, h);
    u32x4* a = d + t * T * U;
    u32x4* b = d + (t + h) * T * U;
    u32x4 v[U], w[U];
#pragma unroll
    for (int i = 0; i < U; ++i) v[i] = __builtin_nontemporal_load(a + i * T + threadIdx.x);
#pragma unroll
    for (int i = 0; i < U; ++i) w[i] = __builtin_nontemporal_load(b + i * T + threadIdx.x);
#pragma unroll
    for (int i = 0; i < U; ++i) __builtin_nontemporal_store(v[i] ^ pat, a + i * T + threadIdx.x);
#pragma unroll
    for (int i = 0; i < U; ++i) __builtin_nontemporal_store(w[i] ^ pat, b + i * T + threadIdx.x);
}

// lane-contiguous: each lane owns U consecutive 16-B chunks (64 B per lane)
template <int T, int U>
__global__ __launch_bounds__(T) void k_ipc(u32x4* d, uint64_t ntiles, uint32_t pat) {
    const uint64_t t = xcd_tile(blockIdx.x, ntiles);
    u32x4* b = d + t * T * U + threadIdx.x * U;
    u32x4 v[U];
#pragma unroll
    for (int i = 0; i < U; ++i) v[i] = __builtin_nontemporal_load(b + i);
#pragma unroll
    for (int i = 0; i < U; ++i) __builtin_nontemporal_store(v[i] ^ pat, b + i);
}

// wave-wise: each wave owns a 4 KiB contiguous piece (U x 1 KiB rows)
template <int T, int U>
__global__ __launch_bounds__(T) void k_ipw(u32x4* d, uint64_t ntiles, uint32_t pat) {
    const uint64_t t = xcd_tile(blockIdx.x, ntiles);
    const uint32_t w = threadIdx.x >> 6, l = threadIdx.x & 63u;
    u32x4* b = d + t * T * U + (uint64_t)w * 64 * U + l;
    u32x4 v[U];
#pragma unroll
    for (int i = 0; i < U; ++i) v[i] = __builtin_nontemporal_load(b + i * 64);
#pragma unroll
    for (int i = 0; i < U; ++i) __builtin_nontemporal_store(v[i] ^ pat, b + i * 64);
}

template <int T, int U>
__global__ __launch_bounds__(T) void k_cp(const u32x4* s, u32x4* d, uint64_t ntiles, uint32_t pat) {
    const uint64_t t = xcd_tile(blockIdx.x, ntiles);
    const u32x4* a = s + t * T * U;
    u32x4* b = d + t * T * U;
    u32x4 v[U];
#pragma unroll
    for (int i = 0; i < U; ++i) v[i] = __builtin_nontemporal_load(a + i * T + threadIdx.x);
#pragma unroll
    for (int i = 0; i < U; ++i) __builtin_nontemporal_store(v[i] ^ pat, b + i * T + threadIdx.x);
}

struct variant {
    std::string name;
    std::function<void()> run;
    std::vector<double> gbs;
};

int main(int argc, char** argv) {
    const double gib = argc > 1 ? atof(argv[1]) : 32.0;
    const int rounds = argc > 2 ? atoi(argv[2]) : 7;
    const uint64_t bytes = (uint64_t)(gib * (1ull << 30)) & ~((1ull << 21) - 1);
    const uint64_t n16 = bytes / 16;
    u32x4 *a, *b;
    CK(hipMalloc(&a, bytes));
    CK(hipMalloc(&b, bytes));
    CK(hipMemset(a, 1, bytes));
    CK(hipMemset(b, 2, bytes));
    std::vector<variant> vs;
#define IP(NAME, K, T, U)                                                                                  \
    vs.push_back({NAME, [&] {                                                                               \
                      const uint64_t nt = n16 / (T * U);                                                    \
                      hipLaunchKernelGGL(K, dim3((unsigned)nt), dim3(T), 0, 0, a, nt, 0x5a5a5a5au);         \
                  }, {}});
    IP("inplace xcd T256 U4 (k_unmask)", (k_ip<256, 4, 0>), 256, 4)
    IP("inplace xcd T256 U2", (k_ip<256, 2, 0>), 256, 2)
    IP("inplace xcd T128 U4", (k_ip<128, 4, 0>), 128, 4)
    IP("inplace xcd T512 U4", (k_ip<512, 4, 0>), 512, 4)
    IP("inplace xcd T1024 U2", (k_ip<1024, 2, 0>), 1024, 2)
    IP("inplace halves T256 U4", (k_ip<256, 4, 2>), 256, 4)
    IP("inplace bitrev64 T256 U4", (k_ip<256, 4, 3>), 256, 4)
    IP("inplace lane-contig T256 U4", (k_ipc<256, 4>), 256, 4)
    IP("inplace wave-contig T256 U4", (k_ipw<256, 4>), 256, 4)
    vs.push_back({"inplace 2 tiles/block half apart T256 U2", [&] {
                      const uint64_t nt = n16 / 512;
                      hipLaunchKernelGGL((k_ip2<256, 2>), dim3((unsigned)(nt / 2)), dim3(256), 0, 0, a, nt, 0x5a5a5a5au);
                  }, {}});
    vs.push_back({"inplace 2 tiles/block half apart T256 U4", [&] {
                      const uint64_t nt = n16 / 1024;
                      hipLaunchKernelGGL((k_ip2<256, 4>), dim3((unsigned)(nt / 2)), dim3(256), 0, 0, a, nt, 0x5a5a5a5au);
                  }, {}});
    vs.push_back({"copy xcd T256 U4", [&] {
                      const uint64_t nt = n16 / 1024;
                      hipLaunchKernelGGL((k_cp<256, 4>), dim3((unsigned)nt), dim3(256), 0, 0, a, b, nt, 0x5a5a5a5au);
                  }, {}});
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (auto& v : vs) v.run();
    CK(hipDeviceSynchronize());
    for (int r = 0; r < rounds; ++r) {
        for (auto& v : vs) {
            CK(hipEventRecord(e0));
            v.run();
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            v.gbs.push_back(2.0 * bytes / (ms * 1e-3) / 1e9);
        }
        fprintf(stderr, "round %d done\n", r);
    }
    printf("buffer %.2f GiB, %d rounds\n", bytes / double(1ull << 30), rounds);
    for (auto& v : vs) {
        std::sort(v.gbs.begin(), v.gbs.end());
        printf("%-44s median %7.1f  best %7.1f  worst %7.1f GB/s\n", v.name.c_str(), v.gbs[v.gbs.size() / 2],
               v.gbs.back(), v.gbs.front());
    }
    return 0;
}

// membench.hip -- design probe (not product code): HBM streaming variants on
// MI355X for the in-place unmask's access pattern.  Prints GB/s (read+write
// bytes / time) per variant; used to pick k_unmask's geometry.
//   hipcc --offload-arch=gfx950 -O3 scripts/membench.hip -o build/membench && build/membench [GiB]
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <vector>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

#define CK(x)                                                                         \
    do {                                                                              \
        hipError_t err_ = (x);                                                           \
        if (err_ != hipSuccess) {                                                     \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(err_));                  \
            exit(1);                                                                  \
        }                                                                             \
    } while (0)

template <bool NT>
__device__ __forceinline__ u32x4 ld(const u32x4* p) {
    if (NT) return __builtin_nontemporal_load(p);
    return *p;
}
template <bool NT>
__device__ __forceinline__ void st(u32x4* p, u32x4 v) {
    if (NT) __builtin_nontemporal_store(v, p);
    else *p = v;
}

// one tile per workgroup, in place
template <int T, int U, bool NT>
__global__ __launch_bounds__(T) void k_tile(u32x4* d, uint64_t n16, uint32_t pat) {
    const uint64_t base = (uint64_t)blockIdx.x * T * U;
    u32x4 v[U];
#pragma unroll
    for (int i = 0; i < U; ++i) {
        uint64_t c = base + (uint64_t)i * T + threadIdx.x;
        if (c < n16) v[i] = ld<NT>(d + c);
    }
#pragma unroll
    for (int i = 0; i < U; ++i) {
        uint64_t c = base + (uint64_t)i * T + threadIdx.x;
        if (c < n16) st<NT>(d + c, v[i] ^ pat);
    }
}

// persistent grid-stride over tiles, in place
template <int T, int U, bool NT>
__global__ __launch_bounds__(T) void k_persist(u32x4* d, uint64_t n16, uint32_t pat) {
    const uint64_t ntiles = (n16 + (uint64_t)T * U - 1) / ((uint64_t)T * U);
    for (uint64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
        const uint64_t base = t * T * U;
        u32x4 v[U];
#pragma unroll
        for (int i = 0; i < U; ++i) {
            uint64_t c = base + (uint64_t)i * T + threadIdx.x;
            if (c < n16) v[i] = ld<NT>(d + c);
        }
#pragma unroll
        for (int i = 0; i < U; ++i) {
            uint64_t c = base + (uint64_t)i * T + threadIdx.x;
            if (c < n16) st<NT>(d + c, v[i] ^ pat);
        }
    }
}

// copy A -> B, one tile per workgroup
template <int T, int U, bool NT>
__global__ __launch_bounds__(T) void k_copy(const u32x4* a, u32x4* b, uint64_t n16) {
    const uint64_t base = (uint64_t)blockIdx.x * T * U;
    u32x4 v[U];
#pragma unroll
    for (int i = 0; i < U; ++i) {
        uint64_t c = base + (uint64_t)i * T + threadIdx.x;
        if (c < n16) v[i] = ld<NT>(a + c);
    }
#pragma unroll
    for (int i = 0; i < U; ++i) {
        uint64_t c = base + (uint64_t)i * T + threadIdx.x;
        if (c < n16) st<NT>(b + c, v[i]);
    }
}

template <int T, int U>
__global__ __launch_bounds__(T) void k_read(const u32x4* d, uint64_t n16, uint32_t* sink) {
    const uint64_t base = (uint64_t)blockIdx.x * T * U;
    u32x4 acc = {0, 0, 0, 0};
#pragma unroll
    for (int i = 0; i < U; ++i) {
        uint64_t c = base + (uint64_t)i * T + threadIdx.x;
        if (c < n16) acc ^= __builtin_nontemporal_load(d + c);
    }
    if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) sink[0] = 1;
}

template <int T, int U>
__global__ __launch_bounds__(T) void k_write(u32x4* d, uint64_t n16, uint32_t pat) {
    const uint64_t base = (uint64_t)blockIdx.x * T * U;
#pragma unroll
    for (int i = 0; i < U; ++i) {
        uint64_t c = base + (uint64_t)i * T + threadIdx.x;
        if (c < n16) __builtin_nontemporal_store(u32x4{pat, pat, pat, pat}, d + c);
    }
}

struct res {
    const char* name;
    double best, med;
};

template <typename F>
res timeit(const char* name, double bytes, F launch) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    launch();
    CK(hipDeviceSynchronize());
    std::vector<double> v;
    for (int r = 0; r < 7; ++r) {
        CK(hipEventRecord(a));
        launch();
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        v.push_back(bytes / (ms * 1e-3) / 1e9);
    }
    std::sort(v.begin(), v.end());
    res r = {name, v.back(), v[v.size() / 2]};
    printf("%-34s best %8.1f GB/s  median %8.1f GB/s\n", name, r.best, r.med);
    fflush(stdout);
    return r;
}

#define TILE_V(T, U, NT)                                                                              \
    timeit("tile T=" #T " U=" #U " nt=" #NT, 2.0 * bytes, [&] {                                     \
        hipLaunchKernelGGL((k_tile<T, U, NT>), dim3((unsigned)((n16 + T * U - 1) / (T * U))), dim3(T), 0, 0, \
                           d, n16, 0x5a5a5a5au);                                                      \
    })
#define PERS_V(T, U, NT, G)                                                                           \
    timeit("persist T=" #T " U=" #U " nt=" #NT " G=" #G, 2.0 * bytes, [&] {                         \
        hipLaunchKernelGGL((k_persist<T, U, NT>), dim3(G), dim3(T), 0, 0, d, n16, 0x5a5a5a5au);     \
    })

int main(int argc, char** argv) {
    double gib = argc > 1 ? atof(argv[1]) : 16.0;
    uint64_t bytes = (uint64_t)(gib * (1ull << 30));
    bytes &= ~4095ull;
    uint64_t n16 = bytes / 16;
    u32x4* d;
    u32x4* e;
    uint32_t* sink;
    CK(hipMalloc(&d, bytes));
    CK(hipMalloc(&e, bytes));
    CK(hipMalloc(&sink, 64));
    CK(hipMemset(d, 1, bytes));
    CK(hipMemset(e, 2, bytes));
    printf("buffer %.1f GiB\n", bytes / double(1ull << 30));
    TILE_V(256, 4, true);
    TILE_V(256, 8, true);
    TILE_V(256, 8, false);
    TILE_V(256, 16, true);
    TILE_V(256, 16, false);
    TILE_V(512, 8, true);
    TILE_V(512, 8, false);
    TILE_V(1024, 4, true);
    TILE_V(1024, 8, false);
    PERS_V(256, 8, true, 2048);
    PERS_V(256, 8, false, 2048);
    PERS_V(256, 16, false, 1024);
    PERS_V(512, 8, false, 1024);
    PERS_V(256, 8, false, 4096);
    timeit("copy T=256 U=8 nt=1", 2.0 * bytes, [&] {
        hipLaunchKernelGGL((k_copy<256, 8, true>), dim3((unsigned)((n16 + 2047) / 2048)), dim3(256), 0, 0, d, e, n16);
    });
    timeit("copy T=256 U=8 nt=0", 2.0 * bytes, [&] {
        hipLaunchKernelGGL((k_copy<256, 8, false>), dim3((unsigned)((n16 + 2047) / 2048)), dim3(256), 0, 0, d, e, n16);
    });
    timeit("read T=256 U=8", 1.0 * bytes, [&] {
        hipLaunchKernelGGL((k_read<256, 8>), dim3((unsigned)((n16 + 2047) / 2048)), dim3(256), 0, 0, d, n16, sink);
    });
    timeit("write T=256 U=8", 1.0 * bytes, [&] {
        hipLaunchKernelGGL((k_write<256, 8>), dim3((unsigned)((n16 + 2047) / 2048)), dim3(256), 0, 0, d, n16, 7u);
    });
    timeit("hipMemcpyDtoD", 2.0 * bytes, [&] { CK(hipMemcpyAsync(e, d, bytes, hipMemcpyDeviceToDevice, 0)); });
    // host link
    void* h;
    uint64_t hb = 1ull << 30;
    CK(hipHostMalloc(&h, hb, hipHostMallocDefault));
    memset(h, 3, hb);
    timeit("H2D pinned 1 GiB", (double)hb, [&] { CK(hipMemcpyAsync(d, h, hb, hipMemcpyHostToDevice, 0)); });
    timeit("D2H pinned 1 GiB", (double)hb, [&] { CK(hipMemcpyAsync(h, d, hb, hipMemcpyDeviceToHost, 0)); });
    hipStream_t s1, s2;
    CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    void* h2;
    CK(hipHostMalloc(&h2, hb, hipHostMallocDefault));
    timeit("H2D+D2H concurrent (sum)", 2.0 * hb, [&] {
        CK(hipMemcpyAsync(d, h, hb, hipMemcpyHostToDevice, s1));
        CK(hipMemcpyAsync(h2, e, hb, hipMemcpyDeviceToHost, s2));
        CK(hipStreamSynchronize(s1));
        CK(hipStreamSynchronize(s2));
    });
    return 0;
}

// membench3.hip -- design probe (not product code): why does an out-of-place
// copy (k_build) run faster than the in-place read+write stream (k_unmask)?
// Same geometry (256 threads x U 16-B chunks per lane), variants interleaved
// round by round in one process: in place vs copy, tile order, cache-policy
// bits of the loads/stores (gfx950 CPol: sc0 = 1, nt = 2, sc1 = 16), and a
// persistent software-pipelined in-place loop.
//   membench3 <GiB> [rounds]
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

// LP/SP: 0 plain, 1 nontemporal builtin, else buffer op with aux = LP/SP - 2.
// `b` is the block-uniform tile base (the buffer descriptor must be scalar),
// `i` the lane's 16-B index inside the tile.
template <int LP>
__device__ __forceinline__ u32x4 ld(const u32x4* b, uint32_t i) {
    if constexpr (LP == 0) return b[i];
    else if constexpr (LP == 1) return __builtin_nontemporal_load(b + i);
    else {
        __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)b, 0, 0x7FFFFFFF, 0x00020000);
        return __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(r, i * 16, 0, LP - 2));
    }
}
template <int SP>
__device__ __forceinline__ void st(u32x4* b, uint32_t i, u32x4 v) {
    if constexpr (SP == 0) b[i] = v;
    else if constexpr (SP == 1) __builtin_nontemporal_store(v, b + i);
    else {
        __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)b, 0, 0x7FFFFFFF, 0x00020000);
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned int, v), r, i * 16, 0, SP - 2);
    }
}

// in place (dst == src) or copy; tile order XCD-contiguous (SWZ) or linear
template <int T, int U, bool SWZ, int LP, int SP>
__global__ __launch_bounds__(T) void k_rw(const u32x4* src, u32x4* dst, uint64_t ntiles, uint32_t pat) {
    const uint64_t t = SWZ ? xcd_tile(blockIdx.x, ntiles) : blockIdx.x;
    const uint64_t base = t * T * U;
    u32x4 v[U];
#pragma unroll
    for (int i = 0; i < U; ++i) v[i] = ld<LP>(src + base, i * T + threadIdx.x);
#pragma unroll
    for (int i = 0; i < U; ++i) st<SP>(dst + base, i * T + threadIdx.x, v[i] ^ pat);
}

// persistent in place: each block walks a contiguous range of tiles; the next
// tile's loads are issued before the current tile's stores
template <int T, int U>
__global__ __launch_bounds__(T) void k_pipe(u32x4* d, uint64_t ntiles, uint32_t pat) {
    const uint64_t per = (ntiles + gridDim.x - 1) / gridDim.x;
    const uint64_t b = xcd_tile(blockIdx.x, gridDim.x);
    const uint64_t t0 = b * per, t1 = t0 + per < ntiles ? t0 + per : ntiles;
    if (t0 >= t1) return;
    u32x4 v[U], w[U];
#pragma unroll
    for (int i = 0; i < U; ++i) v[i] = __builtin_nontemporal_load(d + t0 * T * U + (uint64_t)i * T + threadIdx.x);
    for (uint64_t t = t0; t < t1; ++t) {
        const bool more = t + 1 < t1;
        if (more) {
#pragma unroll
            for (int i = 0; i < U; ++i)
                w[i] = __builtin_nontemporal_load(d + (t + 1) * T * U + (uint64_t)i * T + threadIdx.x);
        }
#pragma unroll
        for (int i = 0; i < U; ++i) __builtin_nontemporal_store(v[i] ^ pat, d + t * T * U + (uint64_t)i * T + threadIdx.x);
#pragma unroll
        for (int i = 0; i < U; ++i) v[i] = w[i];
    }
}

template <int T, int U>
__global__ __launch_bounds__(T) void k_rd(const u32x4* d, uint64_t ntiles, uint32_t* sink) {
    const uint64_t t = xcd_tile(blockIdx.x, ntiles);
    u32x4 acc = {0, 0, 0, 0};
#pragma unroll
    for (int i = 0; i < U; ++i) acc ^= __builtin_nontemporal_load(d + t * T * U + (uint64_t)i * T + threadIdx.x);
    if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) sink[0] = 1;
}

template <int T, int U, int SP>
__global__ __launch_bounds__(T) void k_wr(u32x4* d, uint64_t ntiles, uint32_t pat) {
    const uint64_t t = xcd_tile(blockIdx.x, ntiles);
#pragma unroll
    for (int i = 0; i < U; ++i) st<SP>(d + t * T * U, i * T + threadIdx.x, u32x4{pat, pat, pat, pat});
}

struct variant {
    std::string name;
    double bytes_mult;
    std::function<void()> run;
    std::vector<double> gbs;
};

int main(int argc, char** argv) {
    const double gib = argc > 1 ? atof(argv[1]) : 16.0;
    const int rounds = argc > 2 ? atoi(argv[2]) : 5;
    const uint64_t bytes = (uint64_t)(gib * (1ull << 30)) & ~((1ull << 20) - 1);
    const uint64_t n16 = bytes / 16;
    u32x4 *a, *b;
    uint32_t* sink;
    CK(hipMalloc(&a, bytes));
    CK(hipMalloc(&b, bytes));
    CK(hipMalloc(&sink, 64));
    CK(hipMemset(a, 1, bytes));
    CK(hipMemset(b, 2, bytes));
    std::vector<variant> vs;
#define RW(NAME, T, U, S, LP, SP, DST)                                                                   \
    vs.push_back({NAME, 2.0, [&] {                                                                        \
                      const uint64_t nt = n16 / (T * U);                                                  \
                      hipLaunchKernelGGL((k_rw<T, U, S, LP, SP>), dim3((unsigned)nt), dim3(T), 0, 0, a, DST, nt, \
                                         0x5a5a5a5au);                                                    \
                  }, {}});
    RW("inplace xcd nt/nt U4 (k_unmask)", 256, 4, true, 1, 1, a)
    RW("copy    xcd nt/nt U4", 256, 4, true, 1, 1, b)
    RW("copy    lin nt/nt U2 (k_build)", 256, 2, false, 1, 1, b)
    RW("inplace lin nt/nt U2", 256, 2, false, 1, 1, a)
    RW("inplace lin nt/nt U4", 256, 4, false, 1, 1, a)
    RW("copy    lin nt/nt U4", 256, 4, false, 1, 1, b)
    RW("inplace xcd plain/nt U4", 256, 4, true, 0, 1, a)
    RW("inplace xcd nt/plain U4", 256, 4, true, 1, 0, a)
    RW("inplace xcd plain/plain U4", 256, 4, true, 0, 0, a)
    RW("inplace xcd nt/sc1 U4", 256, 4, true, 1, 2 + 16, a)
    RW("inplace xcd nt/sc0sc1 U4", 256, 4, true, 1, 2 + 17, a)
    RW("inplace xcd nt/sc1nt U4", 256, 4, true, 1, 2 + 18, a)
    RW("inplace xcd sc1/nt U4", 256, 4, true, 2 + 16, 1, a)
    RW("inplace xcd buf-nt/buf-nt U4", 256, 4, true, 2 + 2, 2 + 2, a)
    RW("inplace xcd nt/nt U8", 256, 8, true, 1, 1, a)
    RW("copy    xcd nt/sc1 U4", 256, 4, true, 1, 2 + 16, b)
    vs.push_back({"inplace persistent pipelined U4 G=2048", 2.0, [&] {
                      hipLaunchKernelGGL((k_pipe<256, 4>), dim3(2048), dim3(256), 0, 0, a, n16 / 1024, 0x5a5a5a5au);
                  }, {}});
    vs.push_back({"inplace persistent pipelined U2 G=4096", 2.0, [&] {
                      hipLaunchKernelGGL((k_pipe<256, 2>), dim3(4096), dim3(256), 0, 0, a, n16 / 512, 0x5a5a5a5au);
                  }, {}});
    vs.push_back({"read only xcd nt U4", 1.0, [&] {
                      hipLaunchKernelGGL((k_rd<256, 4>), dim3((unsigned)(n16 / 1024)), dim3(256), 0, 0, a, n16 / 1024, sink);
                  }, {}});
    vs.push_back({"write only xcd nt U4", 1.0, [&] {
                      hipLaunchKernelGGL((k_wr<256, 4, 1>), dim3((unsigned)(n16 / 1024)), dim3(256), 0, 0, b, n16 / 1024,
                                         7u);
                  }, {}});
    vs.push_back({"write only xcd sc1 U4", 1.0, [&] {
                      hipLaunchKernelGGL((k_wr<256, 4, 2 + 16>), dim3((unsigned)(n16 / 1024)), dim3(256), 0, 0, b,
                                         n16 / 1024, 7u);
                  }, {}});
    vs.push_back({"write only xcd plain U4", 1.0, [&] {
                      hipLaunchKernelGGL((k_wr<256, 4, 0>), dim3((unsigned)(n16 / 1024)), dim3(256), 0, 0, b, n16 / 1024,
                                         7u);
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
            v.gbs.push_back(v.bytes_mult * bytes / (ms * 1e-3) / 1e9);
        }
        fprintf(stderr, "round %d done\n", r);
    }
    printf("buffer %.2f GiB, %d rounds\n", bytes / double(1ull << 30), rounds);
    for (auto& v : vs) {
        std::sort(v.gbs.begin(), v.gbs.end());
        printf("%-40s median %7.1f  best %7.1f  worst %7.1f GB/s\n", v.name.c_str(), v.gbs[v.gbs.size() / 2],
               v.gbs.back(), v.gbs.front());
    }
    return 0;
}

// dispatch_probe.hip -- design probe (not product code): when does the
// hardware dispatch a kernel queued on a second stream while a large grid
// (66 K workgroups, like k_unmask at config 2) runs on the first?  Each kernel
// records its first-workgroup start and last-workgroup end with the 100 MHz
// wall clock; times are printed in us relative to the first big grid's start.
//   dispatch_probe [GiB]
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <unistd.h>

#include <vector>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

#define CK(x)                                                         \
    do {                                                              \
        hipError_t err_ = (x);                                        \
        if (err_ != hipSuccess) {                                     \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(err_)); \
            exit(1);                                                  \
        }                                                             \
    } while (0)

struct span {
    unsigned long long t0, t1;
};

__device__ __forceinline__ void mark_begin(span* s) {
    if (threadIdx.x == 0) atomicMin(&s->t0, (unsigned long long)wall_clock64());
}
__device__ __forceinline__ void mark_end(span* s) {
    __syncthreads();
    if (threadIdx.x == 0) atomicMax(&s->t1, (unsigned long long)wall_clock64());
}

__device__ __forceinline__ uint64_t xcd_tile(uint64_t b, uint64_t ntiles) {
    const uint64_t q = ntiles >> 3, r = ntiles & 7u, x = b & 7u, i = b >> 3;
    return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + i;
}

// Per-workgroup stamps for the big grids (same-address atomics from 66 K
// workgroups would serialise and slow the grid itself down ~4x).
// Only the first block, every 512th and the last 256 take stamps: the wall
// clock read itself costs enough to slow a 66 K-workgroup grid down.
__device__ __forceinline__ bool stamped() {
    return blockIdx.x % 512u == 0 || blockIdx.x + 256u >= gridDim.x;
}
__device__ __forceinline__ void stamp_begin(span* s) {
    if (threadIdx.x == 0 && stamped()) s[blockIdx.x].t0 = wall_clock64();
}
__device__ __forceinline__ void stamp_end(span* s) {
    if (!stamped()) return;
    __syncthreads();
    if (threadIdx.x == 0) s[blockIdx.x].t1 = wall_clock64();
}

// k_unmask-shaped in-place stream: 256 threads x 4 x 16 B per tile.
template <bool STAMP>
__global__ __launch_bounds__(256) void k_big_t(u32x4* dv, uint64_t ntiles, span* s) {
    if (STAMP) stamp_begin(s);
    // byte addressing (as k_stream_xor): the u32x4-pointer form of this loop
    // compiled to 64-bit VGPR address chains and ran at half the rate
    uint8_t* d = reinterpret_cast<uint8_t*>(dv);
    const uint64_t base = xcd_tile(blockIdx.x, ntiles) * 16384u;
    u32x4 v[4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
        v[i] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(d + base + ((uint64_t)i * 256 + threadIdx.x) * 16u));
#pragma unroll
    for (int i = 0; i < 4; ++i)
        __builtin_nontemporal_store(v[i] ^ 0x5A5A5A5Au,
                                    reinterpret_cast<u32x4*>(d + base + ((uint64_t)i * 256 + threadIdx.x) * 16u));
    if (STAMP) stamp_end(s);
}

// Variants of the big grid: linear tile order, and byte addressing as
// k_stream_xor does.
template <int MODE>
__global__ __launch_bounds__(256) void k_big_v(uint8_t* d, uint64_t ntiles, uint32_t pat) {
    const uint64_t t = MODE == 1 ? (uint64_t)blockIdx.x : xcd_tile(blockIdx.x, ntiles);
    const uint64_t base = t * 16384u;
    u32x4 v[4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
        v[i] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(d + base + ((uint64_t)i * 256 + threadIdx.x) * 16u));
#pragma unroll
    for (int i = 0; i < 4; ++i)
        __builtin_nontemporal_store(v[i] ^ u32x4{pat, pat, pat, pat},
                                    reinterpret_cast<u32x4*>(d + base + ((uint64_t)i * 256 + threadIdx.x) * 16u));
}

// Persistent variant: `grid` workgroups loop over the tiles.
__global__ __launch_bounds__(256) void k_big_persistent(u32x4* d, uint64_t ntiles, span* s) {
    stamp_begin(s);
    uint8_t* db = reinterpret_cast<uint8_t*>(d);
    for (uint64_t i = blockIdx.x; i < ntiles; i += gridDim.x) {   // gridDim a multiple of 8: XCD order kept
        const uint64_t base = xcd_tile(i, ntiles) * 16384u;
        u32x4 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u)
            v[u] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(db + base + ((uint64_t)u * 256 + threadIdx.x) * 16u));
#pragma unroll
        for (int u = 0; u < 4; ++u)
            __builtin_nontemporal_store(v[u] ^ 0x5A5A5A5Au,
                                        reinterpret_cast<u32x4*>(db + base + ((uint64_t)u * 256 + threadIdx.x) * 16u));
    }
    stamp_end(s);
}

// A small kernel standing in for one step of a scan chain: spins `us`.
__global__ __launch_bounds__(256) void k_probe(span* s, uint32_t us) {
    mark_begin(s);
    const unsigned long long t = wall_clock64();
    while (wall_clock64() - t < (unsigned long long)us * 100ull) __builtin_amdgcn_s_sleep(2);
    mark_end(s);
}

static void reset(span* h, int n) {
    for (int i = 0; i < n; ++i) h[i] = span{~0ull, 0ull};
}

int main(int argc, char** argv) {
    const double gib = argc > 1 ? atof(argv[1]) : 1.0;
    const uint64_t bytes = (uint64_t)(gib * (1ull << 30)) & ~16383ull;
    const uint64_t ntiles = bytes / 16384;
    u32x4* d;
    CK(hipMalloc(&d, bytes));
    CK(hipMemset(d, 1, bytes));
    span* h = (span*)malloc(64 * sizeof(span));
    span* dv;   // device memory: probe spans (atomics to host memory would go over PCIe)
    CK(hipMalloc(&dv, 64 * sizeof(span)));
    span *bigv[2], *bigh[2];   // per-workgroup stamps of the two big grids
    for (int i = 0; i < 2; ++i) {
        CK(hipMalloc(&bigv[i], ntiles * sizeof(span)));
        bigh[i] = (span*)malloc(ntiles * sizeof(span));
    }
    int least = 0, greatest = 0;
    CK(hipDeviceGetStreamPriorityRange(&least, &greatest));
    hipStream_t A, Bn, Bh;
    CK(hipStreamCreateWithFlags(&A, hipStreamNonBlocking));
    CK(hipStreamCreateWithPriority(&Bn, hipStreamNonBlocking, least));
    CK(hipStreamCreateWithPriority(&Bh, hipStreamNonBlocking, greatest));
    int ncu = 0;
    CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
    printf("buffer %.2f GiB, %llu tiles, %d CUs, priorities least %d greatest %d\n", gib,
           (unsigned long long)ntiles, ncu, least, greatest);
    // warm up
    for (int i = 0; i < 600; ++i) hipLaunchKernelGGL(k_big_t<false>, dim3(ntiles), dim3(256), 0, A, d, ntiles, bigv[0]);   // ~0.3 s: clocks up
    hipLaunchKernelGGL(k_probe, dim3(1), dim3(64), 0, Bn, dv + 61, 1u);
    CK(hipDeviceSynchronize());

    {   // the big grid alone, with and without stamps (hipEvent timing)
        hipEvent_t e0, e1;
        CK(hipEventCreate(&e0));
        CK(hipEventCreate(&e1));
        for (int stamp = 0; stamp < 2; ++stamp) {
            float best = 1e9f;
            for (int r = 0; r < 5; ++r) {
                CK(hipEventRecord(e0, A));
                if (stamp) hipLaunchKernelGGL(k_big_t<true>, dim3(ntiles), dim3(256), 0, A, d, ntiles, bigv[0]);
                else hipLaunchKernelGGL(k_big_t<false>, dim3(ntiles), dim3(256), 0, A, d, ntiles, bigv[0]);
                CK(hipEventRecord(e1, A));
                CK(hipEventSynchronize(e1));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                best = ms < best ? ms : best;
            }
            printf("big grid alone, stamps %d: %.1f us (%.0f GB/s in place)\n", stamp, best * 1e3, 2.0 * bytes / (best * 1e-3) / 1e9);
        }
        for (int mode = 0; mode < 2; ++mode) {
            float best = 1e9f;
            for (int r = 0; r < 5; ++r) {
                CK(hipEventRecord(e0, A));
                if (mode) hipLaunchKernelGGL(k_big_v<1>, dim3(ntiles), dim3(256), 0, A, (uint8_t*)d, ntiles, 0x5A5A5A5Au);
                else hipLaunchKernelGGL(k_big_v<0>, dim3(ntiles), dim3(256), 0, A, (uint8_t*)d, ntiles, 0x5A5A5A5Au);
                CK(hipEventRecord(e1, A));
                CK(hipEventSynchronize(e1));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                best = ms < best ? ms : best;
            }
            printf("big grid variant %s: %.1f us (%.0f GB/s in place)\n", mode ? "linear" : "xcd, byte addressing", best * 1e3, 2.0 * bytes / (best * 1e-3) / 1e9);
        }
    }
    // Pipeline emulation (hvws_step_resident's pattern): per step, a chain of
    // `chain` scan kernels on B (waits for its table set's free event), the
    // host waits for the chain's 5th kernel (the check), the big grid on A
    // waits for the chain's end event; set free event recorded after the big grid.
    for (int variant = 0; variant < 10; ++variant) {
        const bool high = variant & 1, setwait = variant < 2 || variant >= 4;
        const bool wide = variant >= 4;   // chain kernels shaped like the engine's: 1024 x 256 threads
        // variants 6-9: the big grid persistent, 6 or 7 workgroups per CU (wave slots left free)
        const int pers = variant >= 8 ? 7 : (variant >= 6 ? 6 : 0);
        hipStream_t B = high ? Bh : Bn;
        const int nstep = 6, chain = 7;
        hipEvent_t scan_done[nstep], check[nstep], freev[2];
        for (int k = 0; k < nstep; ++k) {
            CK(hipEventCreateWithFlags(&scan_done[k], hipEventDisableTiming));
            CK(hipEventCreateWithFlags(&check[k], hipEventDisableTiming));
        }
        for (auto& e : freev) {
            CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
            CK(hipEventRecord(e, A));
        }
        CK(hipDeviceSynchronize());
        reset(h, 64);
        CK(hipMemcpy(dv, h, 64 * sizeof(span), hipMemcpyHostToDevice));
        span* bigs;
        CK(hipMalloc(&bigs, nstep * ntiles * sizeof(span)));
        for (int k = 0; k < nstep; ++k) {
            if (setwait) CK(hipStreamWaitEvent(B, freev[k & 1], 0));
            for (int p = 0; p < chain; ++p) {
                hipLaunchKernelGGL(k_probe, dim3(wide ? 1024 : (p == 6 ? 64 : 16)), dim3(wide ? 256 : 64), 0, B,
                                   dv + k * 8 + p, p == 6 ? 50u : 5u);
                if (p == 4) CK(hipEventRecord(check[k], B));
            }
            CK(hipEventRecord(scan_done[k], B));
            CK(hipStreamWaitEvent(A, scan_done[k], 0));
            if (pers)
                hipLaunchKernelGGL(k_big_persistent, dim3(ncu * pers), dim3(256), 0, A, d, ntiles, bigs + k * ntiles);
            else
                hipLaunchKernelGGL(k_big_t<true>, dim3(ntiles), dim3(256), 0, A, d, ntiles, bigs + k * ntiles);
            CK(hipEventRecord(freev[k & 1], A));
            CK(hipEventSynchronize(check[k]));
        }
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(h, dv, 64 * sizeof(span), hipMemcpyDeviceToHost));
        std::vector<span> bh(nstep * ntiles);
        CK(hipMemcpy(bh.data(), bigs, nstep * ntiles * sizeof(span), hipMemcpyDeviceToHost));
        CK(hipFree(bigs));
        unsigned long long z = h[0].t0;
        printf("pipeline emulation, %s prio, %s set-free wait, chain kernels %s, big grid %s:\n", high ? "high" : "normal",
               setwait ? "with" : "without", wide ? "1024 x 256" : "16-64 x 64",
               pers == 0 ? "one workgroup per tile" : (pers == 6 ? "persistent 6/CU" : "persistent 7/CU"));
        for (int k = 0; k < nstep; ++k) {
            span b{~0ull, 0ull};
            const uint64_t gk = pers ? (uint64_t)ncu * pers : ntiles;
            for (uint64_t i = 0; i < gk; ++i) {
                if (!(i % 512u == 0 || i + 256u >= gk)) continue;
                const span& x = bh[k * ntiles + i];
                b.t0 = x.t0 < b.t0 ? x.t0 : b.t0;
                b.t1 = x.t1 > b.t1 ? x.t1 : b.t1;
            }
            printf("  step %d: scan [%8.1f .. %8.1f] kernels", k, (double)(long long)(h[k * 8].t0 - z) / 100.0,
                   (double)(long long)(h[k * 8 + 6].t1 - z) / 100.0);
            for (int p = 0; p < chain; ++p) printf(" %.1f", (double)(long long)(h[k * 8 + p].t0 - z) / 100.0);
            printf("  big [%8.1f .. %8.1f]\n", (double)(long long)(b.t0 - z) / 100.0, (double)(long long)(b.t1 - z) / 100.0);
        }
    }

    struct scen {
        const char* name;
        bool high;
        int nprobe;          // probes queued on B (a chain)
        uint32_t probe_wg;   // workgroups per probe
        uint32_t probe_us;
        int persistent_wg_per_cu;   // 0 = ordinary grid
        int delay_us;        // host sleep between the big launches and the probes
    };
    const scen S[] = {
        {"1 probe, normal prio", false, 1, 1, 20, 0, 50},
        {"1 probe, high prio", true, 1, 1, 20, 0, 50},
        {"chain of 6 probes, normal prio", false, 6, 1, 5, 0, 50},
        {"chain of 6 probes, high prio", true, 6, 1, 5, 0, 50},
        {"256-WG probe (persistent scan), high prio", true, 1, 256, 60, 0, 50},
        {"chain of 6, big grid persistent 6 WG/CU", false, 6, 1, 5, 6, 50},
        {"chain of 6, big grid persistent 7 WG/CU", false, 6, 1, 5, 7, 50},
        {"chain of 6 queued before the big grids", false, 6, 1, 5, 0, -1},
    };
    for (const scen& sc : S) {
        for (int rep = 0; rep < 3; ++rep) {
            reset(h, 16);
            CK(hipMemcpy(dv, h, 16 * sizeof(span), hipMemcpyHostToDevice));
            hipStream_t B = sc.high ? Bh : Bn;
            const uint32_t grid = sc.persistent_wg_per_cu ? (uint32_t)(ncu * sc.persistent_wg_per_cu) : (uint32_t)ntiles;
            auto big = [&](int slot) {
                if (sc.persistent_wg_per_cu)
                    hipLaunchKernelGGL(k_big_persistent, dim3(grid), dim3(256), 0, A, d, ntiles, bigv[slot]);
                else
                    hipLaunchKernelGGL(k_big_t<true>, dim3(grid), dim3(256), 0, A, d, ntiles, bigv[slot]);
            };
            auto probes = [&]() {
                for (int p = 0; p < sc.nprobe; ++p)
                    hipLaunchKernelGGL(k_probe, dim3(sc.probe_wg), dim3(64), 0, B, dv + 2 + p, sc.probe_us);
            };
            if (sc.delay_us < 0) probes();
            big(0);
            big(1);
            if (sc.delay_us >= 0) {
                usleep(sc.delay_us);
                probes();
            }
            CK(hipDeviceSynchronize());
            CK(hipMemcpy(h, dv, 16 * sizeof(span), hipMemcpyDeviceToHost));
            for (int i = 0; i < 2; ++i) {
                CK(hipMemcpy(bigh[i], bigv[i], grid * sizeof(span), hipMemcpyDeviceToHost));
                h[i] = span{~0ull, 0ull};
                for (uint32_t b = 0; b < grid; ++b) {
                    if (!(b % 512u == 0 || b + 256u >= grid)) continue;
                    h[i].t0 = bigh[i][b].t0 < h[i].t0 ? bigh[i][b].t0 : h[i].t0;
                    h[i].t1 = bigh[i][b].t1 > h[i].t1 ? bigh[i][b].t1 : h[i].t1;
                }
            }
            const unsigned long long z = h[0].t0;
            auto us = [&](unsigned long long t) { return (double)((long long)(t - z)) / 100.0; };
            printf("%-44s rep %d: big1 [%7.1f %7.1f] big2 [%7.1f %7.1f] probes", sc.name, rep, us(h[0].t0), us(h[0].t1),
                   us(h[1].t0), us(h[1].t1));
            for (int p = 0; p < sc.nprobe; ++p) printf(" [%.1f %.1f]", us(h[2 + p].t0), us(h[2 + p].t1));
            printf("\n");
        }
    }
    return 0;
}

// stage_probe.hip -- design probe (not product code) for the resident
// worker's staging and store phases: how long does one workgroup of 256
// threads take to bring an 8 KiB read into LDS, by memory kind and load form,
// and to send 8 KiB back to pinned host memory (stores + system fence)?
// Each iteration starts with a system-scope acquire fence, as the worker's
// request does.  Times are 100 MHz realtime ticks, medians over iterations.
//   hipcc --offload-arch=gfx950 -O2 scripts/probe/stage_probe.hip -o build/stage_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr int kIters = 400;
constexpr uint64_t kBytes = 8192;

// mode: 0 plain 16-B loads, every thread 2 chunks; 1 nontemporal loads;
// 2 one wave loads all 512 chunks (8 per lane); 3 plain loads, then stores to
// dst + system fence (store phase timed separately); 4 nontemporal stores
__global__ __launch_bounds__(256) void k_stage(const uint8_t* __restrict__ src, uint64_t stride, uint64_t span,
                                               uint8_t* __restrict__ dst, int mode, uint64_t* __restrict__ out) {
    __shared__ u32x4 lds[kBytes / 16];
    __shared__ uint64_t t[3];
    const uint32_t tid = threadIdx.x;
    for (int it = 0; it < kIters; ++it) {
        const uint8_t* s = src + (uint64_t)it * stride % span;
        if (tid == 0) {
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
            t[0] = wall_clock64();
        }
        __syncthreads();
        if (mode == 2) {
            if (tid < 64) {
                u32x4 v[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) v[u] = reinterpret_cast<const u32x4*>(s)[u * 64 + tid];
#pragma unroll
                for (int u = 0; u < 8; ++u) lds[u * 64 + tid] = v[u];
            }
        } else if (mode == 1) {
            u32x4 v[2];
#pragma unroll
            for (int u = 0; u < 2; ++u) v[u] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(s) + u * 256 + tid);
#pragma unroll
            for (int u = 0; u < 2; ++u) lds[u * 256 + tid] = v[u];
        } else {
            u32x4 v[2];
#pragma unroll
            for (int u = 0; u < 2; ++u) v[u] = reinterpret_cast<const u32x4*>(s)[u * 256 + tid];
#pragma unroll
            for (int u = 0; u < 2; ++u) lds[u * 256 + tid] = v[u];
        }
        __syncthreads();
        if (tid == 0) t[1] = wall_clock64();
        if (mode >= 3) {
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                u32x4* q = reinterpret_cast<u32x4*>(dst) + u * 256 + tid;
                if (mode == 4)
                    __builtin_nontemporal_store(lds[u * 256 + tid], q);
                else
                    *q = lds[u * 256 + tid];
            }
            __threadfence_system();
        }
        __syncthreads();
        if (tid == 0) {
            t[2] = wall_clock64();
            out[it * 2] = t[1] - t[0];
            out[it * 2 + 1] = t[2] - t[1];
        }
        __syncthreads();
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

static double med(std::vector<uint64_t> v) {
    std::sort(v.begin(), v.end());
    return v[v.size() / 2] * 0.01;   // ticks of 10 ns -> us
}

static void run(const char* kind, const uint8_t* src, uint64_t stride, uint64_t span, uint8_t* dst, int mode,
                uint64_t* d_out, uint64_t* h_out) {
    hipLaunchKernelGGL(k_stage, dim3(1), dim3(256), 0, 0, src, stride, span, dst, mode, d_out);
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(h_out, d_out, kIters * 2 * sizeof(uint64_t), hipMemcpyDeviceToHost));
    std::vector<uint64_t> a, b;
    for (int i = kIters / 10; i < kIters; ++i) {
        a.push_back(h_out[i * 2]);
        b.push_back(h_out[i * 2 + 1]);
    }
    printf("{\"src\": \"%s\", \"mode\": %d, \"stage_us\": %.2f, \"store_us\": %.2f}\n", kind, mode, med(a), med(b));
    fflush(stdout);
}

int main() {
    CK(hipSetDevice(0));
    uint64_t *d_out, *h_out = (uint64_t*)malloc(kIters * 2 * sizeof(uint64_t));
    CK(hipMalloc((void**)&d_out, kIters * 2 * sizeof(uint64_t)));
    uint8_t *fg, *cg, *ph, *ph_d, *oh, *oh_d, *ofg;
    CK(hipExtMallocWithFlags((void**)&fg, 1 << 20, hipDeviceMallocFinegrained));
    CK(hipMalloc((void**)&cg, 256ull << 20));
    CK(hipMemset(cg, 1, 256ull << 20));
    CK(hipHostMalloc((void**)&ph, 1 << 20, 0));
    CK(hipHostGetDevicePointer((void**)&ph_d, ph, 0));
    CK(hipHostMalloc((void**)&oh, 1 << 20, 0));
    CK(hipHostGetDevicePointer((void**)&oh_d, oh, 0));
    CK(hipExtMallocWithFlags((void**)&ofg, 1 << 20, hipDeviceMallocFinegrained));
    for (int mode : {0, 1, 2}) {
        run("vram_finegrained_same", fg, 0, 1 << 20, oh_d, mode, d_out, h_out);
        run("vram_finegrained_rot", fg, 8192, 1 << 20, oh_d, mode, d_out, h_out);
        run("vram_coarse_rot256M", cg, 1 << 20, 256ull << 20, oh_d, mode, d_out, h_out);
        run("vram_coarse_same", cg, 0, 256ull << 20, oh_d, mode, d_out, h_out);
        run("pinned_host", ph_d, 0, 1 << 20, oh_d, mode, d_out, h_out);
    }
    for (int mode : {3, 4}) {
        run("vram_finegrained_same->pinned_host", fg, 0, 1 << 20, oh_d, mode, d_out, h_out);
        run("vram_finegrained_same->vram_finegrained", fg, 0, 1 << 20, ofg, mode, d_out, h_out);
    }
    return 0;
}

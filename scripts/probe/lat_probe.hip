// Probe (diagnostics, not product code): latencies of the primitives the
// resident worker's read is made of, on one workgroup of an idle MI355X --
// dependent LDS loads, an s_barrier of 4 waves, a wave-local fence, the
// realtime-clock read, a system-scope fence after stores to pinned host
// memory, a fine-grained device-memory load (the mailbox poll), a dependent
// chain of 32-bit VALU ops and of 64-bit ones, and the acquire / release
// fences alone (profiles/r6_raw/door/README.md).  Cycles from s_memtime.
//   hipcc --offload-arch=gfx950 -O3 scripts/probe/lat_probe.hip -o scripts/probe/lat_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>
#include <utility>

#define CK(x)                                                                       \
    do {                                                                            \
        hipError_t e_ = (x);                                                        \
        if (e_ != hipSuccess) {                                                     \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                 \
            return 2;                                                               \
        }                                                                           \
    } while (0)

constexpr int N = 256;
constexpr int T = 16;   // tests

__global__ __launch_bounds__(256) void k_lat(uint64_t* out, const uint32_t* fg, uint32_t* host, uint32_t seed) {
    __shared__ uint32_t lds[4096];
    const uint32_t tid = threadIdx.x;
    for (uint32_t i = tid; i < 4096; i += 256) lds[i] = (i * 7u + 1u) & 4095u;
    __syncthreads();
    uint64_t t0, t1;
    uint32_t x = seed & 4095u;
    // 0: dependent LDS loads (pointer chase), wave 0
    t0 = clock64();
    for (int i = 0; i < N; ++i) x = lds[x];
    t1 = clock64();
    if (tid == 0) out[0] = (t1 - t0) / N;
    // 1: dependent 32-bit VALU chain (mad + xor + shift)
    uint32_t v = x + tid;
    t0 = clock64();
    for (int i = 0; i < N; ++i) v = ((v * 2654435761u) ^ (v >> 7)) + 0x9e3779b9u;
    t1 = clock64();
    if (tid == 0) out[1] = (t1 - t0) / N / 3;
    // 2: dependent 64-bit chain (shift, or, add)
    uint64_t w = v;
    t0 = clock64();
    for (int i = 0; i < N; ++i) w = ((w << 13) | (w >> 51)) + 0x9e3779b97f4a7c15ull;
    t1 = clock64();
    if (tid == 0) out[2] = (t1 - t0) / N / 3;
    // 3: s_barrier (4 waves)
    __syncthreads();
    t0 = clock64();
    for (int i = 0; i < N; ++i) __syncthreads();
    t1 = clock64();
    if (tid == 0) out[3] = (t1 - t0) / N;
    // 4: realtime clock read, waited for
    t0 = clock64();
    uint64_t r = 0;
    for (int i = 0; i < N; ++i) r += wall_clock64();
    t1 = clock64();
    if (tid == 0) out[4] = (t1 - t0) / N;
    // 5: fine-grained device-memory load, dependent (the mailbox poll)
    uint32_t y = 0;
    t0 = clock64();
    for (int i = 0; i < 32; ++i) y = __hip_atomic_load(&fg[y & 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    t1 = clock64();
    if (tid == 0) out[5] = (t1 - t0) / 32;
    // 6: store 16 B per thread to pinned host memory + system fence + barrier
    t0 = clock64();
    for (int i = 0; i < 32; ++i) {
        host[(i * 256 + tid) & 8191] = (uint32_t)(r + y + i);
        __threadfence_system();
        __syncthreads();
    }
    t1 = clock64();
    if (tid == 0) out[6] = (t1 - t0) / 32;
    // 7: LDS write then dependent read of another lane's word (wave barrier)
    uint32_t z = tid;
    t0 = clock64();
    for (int i = 0; i < N; ++i) {
        lds[tid] = z;
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        z = lds[(tid + 1) & 63u] + 1u;
    }
    t1 = clock64();
    if (tid == 0) out[7] = (t1 - t0) / N;
    // 8: ballot + readlane chain
    uint32_t b = tid;
    t0 = clock64();
    for (int i = 0; i < N; ++i) {
        const unsigned long long m = __ballot((b & 1u) != 0);
        b = (uint32_t)__builtin_amdgcn_readlane((int)b, (int)(m & 63u)) + tid;
    }
    t1 = clock64();
    if (tid == 0) out[8] = (t1 - t0) / N;
    // 9: a divergent 3-way branch on a uniform LDS value (door_size's shape)
    uint32_t q = x & 127u, acc = 0;
    t0 = clock64();
    for (int i = 0; i < N; ++i) {
        const uint32_t len7 = lds[q] & 127u;
        if (len7 < 126) acc += len7 + 2;
        else if (len7 == 126) acc += lds[q + 1] + 4;
        else acc += lds[q + 2] + 10;
        q = (q + acc) & 2047u;
    }
    t1 = clock64();
    if (tid == 0) out[9] = (t1 - t0) / N;
    // 10: clock frequency: s_memtime ticks per 100 MHz tick over ~20 us
    const uint64_t w0 = wall_clock64(), c0 = clock64();
    while (wall_clock64() - w0 < 2000) {
    }
    const uint64_t w1 = wall_clock64(), c1 = clock64();
    if (tid == 0) out[10] = (c1 - c0) * 100 / (w1 - w0);   // MHz
    // 11: system-scope acquire fence (buffer_inv sc0 sc1), thread 0 alone
    if (tid == 0) {
        t0 = clock64();
        for (int i = 0; i < 32; ++i) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
        t1 = clock64();
        out[11] = (t1 - t0) / 32;
        // 12: agent-scope acquire
        t0 = clock64();
        for (int i = 0; i < 32; ++i) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        t1 = clock64();
        out[12] = (t1 - t0) / 32;
        // 13: system-scope release with nothing dirty (buffer_wbl2 sc0 sc1)
        t0 = clock64();
        for (int i = 0; i < 32; ++i) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
        t1 = clock64();
        out[13] = (t1 - t0) / 32;
        // 14: one 16-B store to pinned host memory, then a system release
        t0 = clock64();
        for (int i = 0; i < 32; ++i) {
            host[i * 64] = (uint32_t)i;
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
        }
        t1 = clock64();
        out[14] = (t1 - t0) / 32;
    }
    if (tid == 0) out[15] = x + v + (uint32_t)w + y + z + b + acc + (uint32_t)r;
}


// Instruction-cache probe: a straight-line block of NI distinct VALU ops
// (each with its own 32-bit literal: 8 bytes, so NI * 8 bytes of code) timed
// the first time this dispatch runs it, again at once, and again after ~50 us
// of polling fine-grained memory with s_sleep, as the resident worker idles.
constexpr int NI = 2048;
template <uint32_t K>
__device__ __forceinline__ void add_lit(uint32_t& v) {
    asm volatile("v_add_u32 %0, %1, %0" : "+v"(v) : "i"(K));
}
template <size_t... I>
__device__ __forceinline__ uint32_t icache_block(uint32_t v, std::index_sequence<I...>) {
    (add_lit<(uint32_t)(I * 2654435761u + 0x10001u)>(v), ...);
    return v;
}
__global__ __launch_bounds__(64) void k_icache(uint64_t* out, const uint32_t* fg, uint32_t seed) {
    uint32_t v = seed + threadIdx.x;
    uint64_t t0 = clock64();
    v = icache_block(v, std::make_index_sequence<NI>{});
    uint64_t t1 = clock64();
    v = icache_block(v, std::make_index_sequence<NI>{});
    uint64_t t2 = clock64();
    const uint64_t w0 = wall_clock64();
    uint32_t y = 0;
    while (wall_clock64() - w0 < 5000) {
        y += __hip_atomic_load(&fg[y & 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __builtin_amdgcn_s_sleep(2);
    }
    uint64_t t3 = clock64();
    v = icache_block(v + y, std::make_index_sequence<NI>{});
    uint64_t t4 = clock64();
    if (threadIdx.x == 0) {
        out[0] = t1 - t0;
        out[1] = t2 - t1;
        out[2] = t4 - t3;
        out[3] = v;
    }
}

int main() {
    uint64_t* d_out;
    uint32_t *fg, *host;
    CK(hipMalloc(&d_out, T * 8));
    CK(hipExtMallocWithFlags((void**)&fg, 64, hipDeviceMallocFinegrained));
    CK(hipHostMalloc((void**)&host, 8192 * 4, 0));
    CK(hipMemset(fg, 0, 64));
    for (int rep = 0; rep < 3; ++rep) {
        hipLaunchKernelGGL(k_lat, dim3(1), dim3(256), 0, 0, d_out, fg, host, 17u + rep);
        CK(hipDeviceSynchronize());
    }
    uint64_t o[T];
    CK(hipMemcpy(o, d_out, sizeof o, hipMemcpyDeviceToHost));
    uint64_t ic[3][4];
    for (int rep = 0; rep < 3; ++rep) {
        hipLaunchKernelGGL(k_icache, dim3(1), dim3(64), 0, 0, d_out, fg, 5u + rep);
        CK(hipDeviceSynchronize());
        CK(hipMemcpy(ic[rep], d_out, sizeof ic[rep], hipMemcpyDeviceToHost));
    }
    printf("{\"icache_block_instructions\": %d, \"icache_block_bytes\": %d, \"cycles_first\": [%llu, %llu, %llu], "
           "\"cycles_again\": [%llu, %llu, %llu], \"cycles_after_50us_idle\": [%llu, %llu, %llu]}\n",
           NI, NI * 8, (unsigned long long)ic[0][0], (unsigned long long)ic[1][0], (unsigned long long)ic[2][0],
           (unsigned long long)ic[0][1], (unsigned long long)ic[1][1], (unsigned long long)ic[2][1],
           (unsigned long long)ic[0][2], (unsigned long long)ic[1][2], (unsigned long long)ic[2][2]);
    printf("{\"lds_dep_load_cycles\": %llu, \"valu32_dep_cycles\": %llu, \"valu64_dep_cycles\": %llu, "
           "\"barrier_4waves_cycles\": %llu, \"realtime_read_cycles\": %llu, \"finegrained_vram_load_cycles\": %llu, "
           "\"host_store_fence_sys_barrier_cycles\": %llu, \"lds_write_read_wave_cycles\": %llu, "
           "\"ballot_readlane_cycles\": %llu, \"branchy_size_step_cycles\": %llu, \"shader_MHz\": %llu, "
           "\"acquire_system_cycles\": %llu, \"acquire_agent_cycles\": %llu, \"release_system_clean_cycles\": %llu, "
           "\"store_host_release_system_cycles\": %llu}\n",
           (unsigned long long)o[0], (unsigned long long)o[1], (unsigned long long)o[2], (unsigned long long)o[3],
           (unsigned long long)o[4], (unsigned long long)o[5], (unsigned long long)o[6], (unsigned long long)o[7],
           (unsigned long long)o[8], (unsigned long long)o[9], (unsigned long long)o[10], (unsigned long long)o[11],
           (unsigned long long)o[12], (unsigned long long)o[13], (unsigned long long)o[14]);
    return 0;
}

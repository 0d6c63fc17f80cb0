// Probe (diagnostics, not product code): does a process that ends with a
// CU-masked stream alive crash at exit under rocprofv3, with no hvws code at
// all?  One tiny kernel on the stream, a sync, then exit.
//   hipcc --offload-arch=gfx950 -O2 scripts/probe/cumask_exit.hip -o scripts/probe/cumask_exit
//   cumask_exit 0   CU-masked stream, left alive at exit
//   cumask_exit 1   CU-masked stream, destroyed before exit
//   cumask_exit 2   ordinary stream, left alive at exit
//   cumask_exit 3   CU-masked stream, left alive, no kernel ever launched on it
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

__global__ void k_touch(unsigned* p) {
    if (threadIdx.x == 0) p[0] += 1u;
}

#define CK(x)                                                                          \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                    \
            return 2;                                                                  \
        }                                                                              \
    } while (0)

int main(int argc, char** argv) {
    const int mode = argc > 1 ? atoi(argv[1]) : 0;
    hipDeviceProp_t prop;
    CK(hipGetDeviceProperties(&prop, 0));
    std::vector<uint32_t> mask((size_t)(prop.multiProcessorCount + 31) / 32, 0u);
    for (int i = 0; i < prop.multiProcessorCount; ++i) mask[(size_t)i / 32] |= 1u << (i % 32);
    hipStream_t s = nullptr;
    if (mode == 2) CK(hipStreamCreate(&s));
    else CK(hipExtStreamCreateWithCUMask(&s, (uint32_t)mask.size(), mask.data()));
    unsigned* d = nullptr;
    CK(hipMalloc(&d, 64));
    CK(hipMemsetAsync(d, 0, 64, s));
    if (mode != 3) hipLaunchKernelGGL(k_touch, dim3(1), dim3(64), 0, s, d);
    CK(hipStreamSynchronize(s));
    if (mode == 1) CK(hipStreamDestroy(s));
    printf("[cumask_exit] mode %d done, exiting\n", mode);
    fflush(stdout);
    return 0;
}

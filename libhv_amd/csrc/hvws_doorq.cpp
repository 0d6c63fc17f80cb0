// hvws_doorq.cpp -- the resident worker's own HSA queue.
//
// The worker (k_door) is a kernel that stays on the device between calls, so
// it needs a hardware queue nothing else is queued behind.  Rounds 3-5 got
// one from the HIP runtime as a CU-masked stream.  Such a stream could not be
// destroyed safely (after hipStreamDestroy of one, the process's next
// ordinary hipStreamDestroy blocked for good: the r4k / r4n hangs, reproduced
// in round 5), so it was kept alive to the end of the process -- and a
// process ending with one alive crashed at exit under rocprofv3: the
// profiler's finalizer waited on a signal of that queue after the HSA runtime
// had been torn down (librocprofiler-sdk -> hsa_signal_wait on an unmapped
// signal page; gpurun_out/kt_r6a.log, symbolised in profiles/r6_raw/exit_crash).
// Destroying the stream at exit removed the crash (r6d) but is the destroy
// that hung processes in rounds 3-4.
//
// So the worker's queue is ours: an HSA queue created with hsa_queue_create
// on the device's agent, k_door dispatched on it as one AQL kernel-dispatch
// packet per launch (the kernel object of k_door as the HIP runtime loaded it,
// found through the AMD loader extension), the packet's completion signal
// telling when the launch has ended, and hsa_queue_destroy once it has -- on
// a context's release (the queue goes to a per-device pool) and at exit (every
// idle queue).  The HIP runtime never sees this queue.
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <hsa/hsa_ven_amd_loader.h>

#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "hvws.h"
#include "hvws_internal.h"

namespace hvws {

namespace {

thread_local char t_why[256] = "";

int fail(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
int fail(int code, const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(t_why, sizeof t_why, fmt, ap);
    va_end(ap);
    return code;
}

struct door_kernel {
    bool tried = false, ok = false;
    hsa_agent_t agent{};
    uint64_t object = 0;
    uint32_t group_static = 0, priv = 0, kernarg = 0;
    uint32_t queue_min = 0;
};

std::mutex g_dk_m;
std::vector<door_kernel> g_dk;   // per HIP device

struct sym_find {
    door_kernel* k;
    bool found;
};

hsa_status_t sym_cb(hsa_executable_t, hsa_executable_symbol_t s, void* data) {
    auto* f = static_cast<sym_find*>(data);
    hsa_symbol_kind_t kind;
    if (hsa_executable_symbol_get_info(s, HSA_EXECUTABLE_SYMBOL_INFO_TYPE, &kind) != HSA_STATUS_SUCCESS ||
        kind != HSA_SYMBOL_KIND_KERNEL)
        return HSA_STATUS_SUCCESS;
    uint32_t len = 0;
    if (hsa_executable_symbol_get_info(s, HSA_EXECUTABLE_SYMBOL_INFO_NAME_LENGTH, &len) != HSA_STATUS_SUCCESS)
        return HSA_STATUS_SUCCESS;
    std::string name(len, '\0');
    if (hsa_executable_symbol_get_info(s, HSA_EXECUTABLE_SYMBOL_INFO_NAME, name.data()) != HSA_STATUS_SUCCESS)
        return HSA_STATUS_SUCCESS;
    if (name.rfind(door_kernel_symbol_prefix(), 0) != 0) return HSA_STATUS_SUCCESS;
    door_kernel& k = *f->k;
    if (hsa_executable_symbol_get_info(s, HSA_EXECUTABLE_SYMBOL_INFO_AGENT, &k.agent) != HSA_STATUS_SUCCESS ||
        hsa_executable_symbol_get_info(s, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_OBJECT, &k.object) != HSA_STATUS_SUCCESS ||
        hsa_executable_symbol_get_info(s, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_GROUP_SEGMENT_SIZE, &k.group_static) !=
            HSA_STATUS_SUCCESS ||
        hsa_executable_symbol_get_info(s, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_PRIVATE_SEGMENT_SIZE, &k.priv) !=
            HSA_STATUS_SUCCESS ||
        hsa_executable_symbol_get_info(s, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_KERNARG_SEGMENT_SIZE, &k.kernarg) !=
            HSA_STATUS_SUCCESS)
        return HSA_STATUS_SUCCESS;
    f->found = true;
    return HSA_STATUS_INFO_BREAK;
}

// k_door as loaded for HIP device `device`: the loader extension names the
// executable holding a device symbol of its code object (door_anchor), whose
// kernel symbols give k_door's descriptor and the agent it was loaded for.
int find_door_kernel(int device, door_kernel& k) {
    void* anchor = nullptr;
    if (hipError_t e = hipSetDevice(device); e != hipSuccess) return fail(HVWS_EHIP, "hipSetDevice: %s", hipGetErrorString(e));
    if (hipError_t e = door_anchor(&anchor); e != hipSuccess)
        return fail(HVWS_EHIP, "k_door: code object not loaded: %s", hipGetErrorString(e));
    hsa_ven_amd_loader_1_01_pfn_t ld;
    if (hsa_system_get_major_extension_table(HSA_EXTENSION_AMD_LOADER, 1, sizeof(ld), &ld) != HSA_STATUS_SUCCESS)
        return fail(HVWS_EHIP, "k_door: no HSA loader extension");
    hsa_executable_t exe;
    if (ld.hsa_ven_amd_loader_query_executable(anchor, &exe) != HSA_STATUS_SUCCESS)
        return fail(HVWS_EHIP, "k_door: code object of the worker not found");
    sym_find f{&k, false};
    hsa_executable_iterate_symbols(exe, sym_cb, &f);
    if (!f.found) return fail(HVWS_EHIP, "k_door: kernel symbol not found in its code object");
    if (hsa_agent_get_info(k.agent, HSA_AGENT_INFO_QUEUE_MIN_SIZE, &k.queue_min) != HSA_STATUS_SUCCESS)
        k.queue_min = 64;
    return HVWS_OK;
}

void queue_error_cb(hsa_status_t status, hsa_queue_t*, void* data) {
    auto* q = static_cast<door_queue*>(data);
    q->error.store((int)status, std::memory_order_release);
}

}  // namespace

int door_queue_create(int device, door_queue** out) {
    *out = nullptr;
    door_kernel k;
    {
        std::lock_guard<std::mutex> lk(g_dk_m);
        if ((int)g_dk.size() <= device) g_dk.resize((size_t)device + 1);
        door_kernel& e = g_dk[(size_t)device];
        if (!e.tried) {
            e.tried = true;
            e.ok = find_door_kernel(device, e) == HVWS_OK;
            if (!e.ok) return HVWS_EHIP;   // t_why says why
        }
        if (!e.ok) return fail(HVWS_EHIP, "k_door: the worker kernel is not available on device %d", device);
        k = e;
    }
    auto* q = new door_queue();
    q->device = device;
    q->agent = k.agent;
    q->object = k.object;
    q->group = k.group_static + (uint32_t)(kDoorMax + 32);   // static LDS + k_door's dynamic area
    q->priv = k.priv;
    q->kernarg_size = k.kernarg;
    const uint32_t size = k.queue_min > 64 ? k.queue_min : 64;
    if (hsa_queue_create(k.agent, size, HSA_QUEUE_TYPE_SINGLE, queue_error_cb, q, UINT32_MAX, UINT32_MAX, &q->q) !=
        HSA_STATUS_SUCCESS) {
        delete q;
        return fail(HVWS_EHIP, "k_door: hsa_queue_create failed");
    }
    if (hsa_signal_create(0, 0, nullptr, &q->done) != HSA_STATUS_SUCCESS) {
        hsa_queue_destroy(q->q);
        delete q;
        return fail(HVWS_EHIP, "k_door: hsa_signal_create failed");
    }
    // kernel arguments in pinned host memory the device reads at dispatch
    // (one launch in flight per queue: a relaunch waits for the last to end)
    if (hipHostMalloc(&q->kernarg, 256, hipHostMallocCoherent | hipHostMallocMapped) != hipSuccess) {
        (void)hipGetLastError();
        hsa_signal_destroy(q->done);
        hsa_queue_destroy(q->q);
        delete q;
        return fail(HVWS_EHIP, "k_door: kernel argument area");
    }
    void* dev = nullptr;
    if (hipHostGetDevicePointer(&dev, q->kernarg, 0) != hipSuccess) {
        (void)hipGetLastError();
        dev = q->kernarg;
    }
    q->kernarg_dev = dev;
    *out = q;
    return HVWS_OK;
}

int door_queue_launch(door_queue* q, const void* args, uint32_t nargs) {
    if (nargs > 256 || nargs < q->kernarg_size) return fail(HVWS_EINVAL, "k_door: kernel arguments %u bytes", nargs);
    if (!door_queue_idle(q)) return fail(HVWS_EHIP, "k_door: a launch is still running on the worker queue");
    memcpy(q->kernarg, args, nargs);
    hsa_signal_store_screlease(q->done, 1);
    hsa_queue_t* hq = q->q;
    const uint64_t idx = hsa_queue_add_write_index_scacq_screl(hq, 1);
    while (idx - hsa_queue_load_read_index_scacquire(hq) >= hq->size) __builtin_ia32_pause();
    auto* pkt = static_cast<hsa_kernel_dispatch_packet_t*>(hq->base_address) + (idx & (hq->size - 1));
    pkt->workgroup_size_x = (uint16_t)kDoorThreads;
    pkt->workgroup_size_y = 1;
    pkt->workgroup_size_z = 1;
    pkt->reserved0 = 0;
    pkt->grid_size_x = kDoorThreads;
    pkt->grid_size_y = 1;
    pkt->grid_size_z = 1;
    pkt->private_segment_size = q->priv;
    pkt->group_segment_size = q->group;
    pkt->kernel_object = q->object;
    pkt->kernarg_address = q->kernarg_dev;
    pkt->reserved2 = 0;
    pkt->completion_signal = q->done;
    const uint16_t header = (uint16_t)((HSA_PACKET_TYPE_KERNEL_DISPATCH << HSA_PACKET_HEADER_TYPE) |
                                       (1u << HSA_PACKET_HEADER_BARRIER) |
                                       (HSA_FENCE_SCOPE_SYSTEM << HSA_PACKET_HEADER_SCACQUIRE_FENCE_SCOPE) |
                                       (HSA_FENCE_SCOPE_SYSTEM << HSA_PACKET_HEADER_SCRELEASE_FENCE_SCOPE));
    const uint16_t setup = (uint16_t)(1u << HSA_KERNEL_DISPATCH_PACKET_SETUP_DIMENSIONS);
    __atomic_store_n(reinterpret_cast<uint32_t*>(pkt), (uint32_t)header | ((uint32_t)setup << 16), __ATOMIC_RELEASE);
    hsa_signal_store_screlease(hq->doorbell_signal, (hsa_signal_value_t)idx);
    return HVWS_OK;
}

const char* door_queue_why() { return t_why; }

bool door_queue_idle(door_queue* q) { return hsa_signal_load_scacquire(q->done) == 0; }

int door_queue_error(door_queue* q) { return q->error.load(std::memory_order_acquire); }

void door_queue_destroy(door_queue* q) {
    if (!q) return;
    hsa_queue_destroy(q->q);
    hsa_signal_destroy(q->done);
    q->q = nullptr;
    // the kernel argument area: pinned host memory, freed only when HIP calls
    // are allowed (not at process exit); a queue destroyed at exit leaks it
    if (q->kernarg && !q->at_exit) hipHostFree(q->kernarg);
    delete q;
}

}  // namespace hvws

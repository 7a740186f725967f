// AQL dispatch on queues of libocm's own (see ocm/aql.h).
#include "ocm/aql.h"

#include <hip/hip_runtime_api.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <time.h>
#include <unistd.h>

#include <cstdio>
#include <cstring>
#include <mutex>

// The gfx950 device code object of xfer.hip, embedded by the build (aql_devcode.S).
extern "C" const char ocm_devcode_begin[];
extern "C" const char ocm_devcode_end[];

namespace ocm {
namespace {

struct AqlState {
    std::mutex mu;
    bool tried = false;
    int device = -1;
    const char *why = "not opened";
    hsa_agent_t gpu{}, cpu{};
    hsa_amd_memory_pool_t kernarg_pool{};
    bool have_pool = false;
    hsa_code_object_reader_t reader{};
    hsa_executable_t exe{};
};

AqlState &A() {
    static AqlState *s = new AqlState();  // never destroyed: queues may outlive static destructors
    return *s;
}

struct Find {
    uint32_t bdf = 0, domain = 0;
    hsa_agent_t gpu{}, cpu{};
    bool found = false;
};

hsa_status_t find_agent(hsa_agent_t a, void *p) {
    Find *f = static_cast<Find *>(p);
    hsa_device_type_t t;
    if (hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t) != HSA_STATUS_SUCCESS) return HSA_STATUS_SUCCESS;
    if (t == HSA_DEVICE_TYPE_CPU && !f->cpu.handle) f->cpu = a;
    if (t == HSA_DEVICE_TYPE_GPU && !f->found) {
        uint32_t bdf = 0, dom = 0;
        if (hsa_agent_get_info(a, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_BDFID, &bdf) == HSA_STATUS_SUCCESS &&
            hsa_agent_get_info(a, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_DOMAIN, &dom) == HSA_STATUS_SUCCESS &&
            bdf == f->bdf && dom == f->domain) {
            f->gpu = a;
            f->found = true;
        }
    }
    return HSA_STATUS_SUCCESS;
}

hsa_status_t find_kernarg_pool(hsa_amd_memory_pool_t pool, void *p) {
    AqlState *s = static_cast<AqlState *>(p);
    hsa_amd_segment_t seg;
    uint32_t flags = 0;
    if (hsa_amd_memory_pool_get_info(pool, HSA_AMD_MEMORY_POOL_INFO_SEGMENT, &seg) != HSA_STATUS_SUCCESS ||
        seg != HSA_AMD_SEGMENT_GLOBAL ||
        hsa_amd_memory_pool_get_info(pool, HSA_AMD_MEMORY_POOL_INFO_GLOBAL_FLAGS, &flags) != HSA_STATUS_SUCCESS)
        return HSA_STATUS_SUCCESS;
    if ((flags & HSA_AMD_MEMORY_POOL_GLOBAL_FLAG_KERNARG_INIT) && !s->have_pool) {
        s->kernarg_pool = pool;
        s->have_pool = true;
    }
    return HSA_STATUS_SUCCESS;
}

constexpr size_t kKernargSlot = 2048;

uint64_t mono_ns() {
    timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (uint64_t)ts.tv_sec * 1000000000ull + (uint64_t)ts.tv_nsec;
}

int open_locked(AqlState &s, int hip_device) {
    int bus = 0, dev = 0, dom = 0;
    if (hipDeviceGetAttribute(&bus, hipDeviceAttributePciBusId, hip_device) != hipSuccess ||
        hipDeviceGetAttribute(&dev, hipDeviceAttributePciDeviceId, hip_device) != hipSuccess ||
        hipDeviceGetAttribute(&dom, hipDeviceAttributePciDomainID, hip_device) != hipSuccess) {
        (void)hipGetLastError();
        s.why = "no PCI location for the HIP device";
        return -1;
    }
    if (hsa_init() != HSA_STATUS_SUCCESS) {
        s.why = "hsa_init failed";
        return -1;
    }
    Find f;
    f.bdf = ((uint32_t)bus << 8) | ((uint32_t)dev << 3);
    f.domain = (uint32_t)dom;
    if (hsa_iterate_agents(find_agent, &f) != HSA_STATUS_SUCCESS || !f.found || !f.cpu.handle) {
        s.why = "no HSA agent at the HIP device's PCI location";
        return -1;
    }
    s.gpu = f.gpu;
    s.cpu = f.cpu;
    if (hsa_amd_agent_iterate_memory_pools(s.cpu, find_kernarg_pool, &s) != HSA_STATUS_SUCCESS || !s.have_pool) {
        s.why = "no kernarg memory pool";
        return -1;
    }
    const size_t n = (size_t)(ocm_devcode_end - ocm_devcode_begin);
    if (n < 64 || std::memcmp(ocm_devcode_begin, "\x7f" "ELF", 4) != 0) {
        s.why = "no embedded device code object";
        return -1;
    }
    if (hsa_code_object_reader_create_from_memory(ocm_devcode_begin, n, &s.reader) != HSA_STATUS_SUCCESS) {
        s.why = "code object reader";
        return -1;
    }
    if (hsa_executable_create_alt(HSA_PROFILE_FULL, HSA_DEFAULT_FLOAT_ROUNDING_MODE_DEFAULT, nullptr, &s.exe) !=
        HSA_STATUS_SUCCESS) {
        (void)hsa_code_object_reader_destroy(s.reader);
        s.why = "creating an HSA executable";
        return -1;
    }
    if (hsa_executable_load_agent_code_object(s.exe, s.gpu, s.reader, nullptr, nullptr) != HSA_STATUS_SUCCESS ||
        hsa_executable_freeze(s.exe, nullptr) != HSA_STATUS_SUCCESS) {
        (void)hsa_executable_destroy(s.exe);
        (void)hsa_code_object_reader_destroy(s.reader);
        s.why = "loading the embedded code object (not gfx950?)";
        return -1;
    }
    s.device = hip_device;
    s.why = nullptr;
    return 0;
}

}  // namespace

int aql_open(int hip_device, const char **why) {
    AqlState &s = A();
    std::lock_guard<std::mutex> g(s.mu);
    if (!s.tried) {
        s.tried = true;
        (void)open_locked(s, hip_device);
    }
    if (s.why == nullptr && s.device != hip_device) {
        if (why) *why = "the AQL path serves one device per process";
        return -1;
    }
    if (why) *why = s.why;
    return s.why == nullptr ? 0 : -1;
}

int aql_kernel(const char *symbol, AqlKernel *k) {
    AqlState &s = A();
    if (s.why != nullptr) return -1;
    char name[160];
    if (std::snprintf(name, sizeof(name), "%s.kd", symbol) >= (int)sizeof(name)) return -1;
    hsa_executable_symbol_t sym;
    if (hsa_executable_get_symbol_by_name(s.exe, name, &s.gpu, &sym) != HSA_STATUS_SUCCESS) return -1;
    if (hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_OBJECT, &k->object) != HSA_STATUS_SUCCESS ||
        hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_KERNARG_SEGMENT_SIZE, &k->kernarg_bytes) !=
            HSA_STATUS_SUCCESS ||
        hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_GROUP_SEGMENT_SIZE, &k->group_bytes) !=
            HSA_STATUS_SUCCESS ||
        hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_PRIVATE_SEGMENT_SIZE, &k->private_bytes) !=
            HSA_STATUS_SUCCESS)
        return -1;
    return 0;
}

int aql_lane_create(AqlLane *l, bool high_priority) {
    AqlState &s = A();
    if (s.why != nullptr) return -1;
    hsa_queue_t *q = nullptr;
    // 64 packets: a lane never has more than one dispatch in flight.
    if (hsa_queue_create(s.gpu, 64, HSA_QUEUE_TYPE_MULTI, nullptr, nullptr, UINT32_MAX, UINT32_MAX, &q) !=
        HSA_STATUS_SUCCESS)
        return -1;
    if (high_priority) (void)hsa_amd_queue_set_priority(q, HSA_AMD_QUEUE_PRIORITY_HIGH);
    hsa_signal_t sig;
    if (hsa_signal_create(0, 0, nullptr, &sig) != HSA_STATUS_SUCCESS) {
        (void)hsa_queue_destroy(q);
        return -1;
    }
    // Kernel arguments in the runtime's kernarg pool (coherent host memory), or with
    // OCM_AQL_KERNARG=wc in write-combined host memory (no snoop of the CPU's caches on
    // the kernel's first loads; the host fences before the doorbell). Measured equal:
    // a relaunch costs 11.5 us after 100 us idle and 16.6-17.8 us after 1 ms either way
    // (profiles/idle_gap_r04_kernarg.json), the GPU's wake-up, not the argument fetch.
    void *ka = nullptr;
    bool wc = false;
    const char *km = std::getenv("OCM_AQL_KERNARG");
    if (km && std::strcmp(km, "wc") == 0) {
        if (hipHostMalloc(&ka, 2 * kKernargSlot, hipHostMallocWriteCombined | hipHostMallocMapped) == hipSuccess) {
            wc = true;
        } else {
            (void)hipGetLastError();
            ka = nullptr;
        }
    }
    if (!wc && (hsa_amd_memory_pool_allocate(s.kernarg_pool, 2 * kKernargSlot, 0, &ka) != HSA_STATUS_SUCCESS ||
                hsa_amd_agents_allow_access(1, &s.gpu, nullptr, ka) != HSA_STATUS_SUCCESS)) {
        if (ka) (void)hsa_amd_memory_pool_free(ka);
        (void)hsa_signal_destroy(sig);
        (void)hsa_queue_destroy(q);
        return -1;
    }
    l->queue = q;
    l->signal = sig.handle;
    l->kernarg = ka;
    l->kernarg_wc = wc;
    l->busy = false;
    return 0;
}

void aql_lane_destroy(AqlLane *l) {
    if (!l->queue) return;
    if (l->kernarg_wc)
        (void)hipHostFree(l->kernarg);
    else
        (void)hsa_amd_memory_pool_free(l->kernarg);
    (void)hsa_signal_destroy(hsa_signal_t{l->signal});
    (void)hsa_queue_destroy(static_cast<hsa_queue_t *>(l->queue));
    *l = AqlLane{};
}

int aql_dispatch(AqlLane *l, const AqlKernel &k, const void *args, size_t nargs, unsigned blocks, unsigned threads,
                 bool overlap, bool barrier) {
    hsa_queue_t *q = static_cast<hsa_queue_t *>(l->queue);
    const size_t hidden = (nargs + 7) & ~size_t(7);
    // COv5 hidden arguments read by the kernel: block count x/y/z at +0, group
    // size x/y/z at +12, remainders at +18, global offsets at +40, dims at +64.
    if (!q || blocks == 0 || threads == 0 || threads > 1024 || k.kernarg_bytes > kKernargSlot ||
        nargs > k.kernarg_bytes || (k.kernarg_bytes > nargs && hidden + 66 > k.kernarg_bytes))
        return -1;
    hsa_signal_t sig{l->signal};
    if (l->busy && !aql_lane_idle(l)) {
        // one dispatch still running: only when asked, and never a third
        if (!overlap || hsa_signal_load_scacquire(sig) > 1) return -1;
    }
    l->slot ^= 1u;
    char *ka = static_cast<char *>(l->kernarg) + (size_t)l->slot * kKernargSlot;
    std::memset(ka, 0, k.kernarg_bytes);
    std::memcpy(ka, args, nargs);
    if (k.kernarg_bytes > nargs) {
        const uint32_t bc[3] = {blocks, 1, 1};
        const uint16_t gs[3] = {(uint16_t)threads, 1, 1};
        const uint16_t dims = 1;
        std::memcpy(ka + hidden, bc, sizeof(bc));
        std::memcpy(ka + hidden + 12, gs, sizeof(gs));
        std::memcpy(ka + hidden + 64, &dims, sizeof(dims));
    }
    // write-combined kernargs leave the CPU's buffers before the packet names them
    if (l->kernarg_wc) __builtin_ia32_sfence();
    hsa_signal_add_relaxed(sig, 1);
    const uint64_t idx = hsa_queue_add_write_index_screlease(q, 1);
    const uint64_t t0 = mono_ns();
    while (idx - hsa_queue_load_read_index_scacquire(q) >= q->size) {
        if (mono_ns() - t0 > 1000000000ull) return -1;  // one in flight per lane: never expected
    }
    auto *p = static_cast<hsa_kernel_dispatch_packet_t *>(q->base_address) + (idx & (q->size - 1));
    p->workgroup_size_x = (uint16_t)threads;
    p->workgroup_size_y = 1;
    p->workgroup_size_z = 1;
    p->reserved0 = 0;
    p->grid_size_x = blocks * threads;
    p->grid_size_y = 1;
    p->grid_size_z = 1;
    p->private_segment_size = k.private_bytes;
    p->group_segment_size = k.group_bytes;
    p->kernel_object = k.object;
    p->kernarg_address = ka;
    p->reserved2 = 0;
    p->completion_signal = sig;
    // system-scope acquire at the start and release at the end, as HIP's own launches
    const uint16_t header = (HSA_PACKET_TYPE_KERNEL_DISPATCH << HSA_PACKET_HEADER_TYPE) |
                            ((barrier ? 1 : 0) << HSA_PACKET_HEADER_BARRIER) |
                            (HSA_FENCE_SCOPE_SYSTEM << HSA_PACKET_HEADER_SCACQUIRE_FENCE_SCOPE) |
                            (HSA_FENCE_SCOPE_SYSTEM << HSA_PACKET_HEADER_SCRELEASE_FENCE_SCOPE);
    const uint16_t setup = 1 << HSA_KERNEL_DISPATCH_PACKET_SETUP_DIMENSIONS;
    __atomic_store_n(reinterpret_cast<uint32_t *>(p), (uint32_t)header | ((uint32_t)setup << 16), __ATOMIC_RELEASE);
    hsa_signal_store_screlease(q->doorbell_signal, (hsa_signal_value_t)idx);
    l->busy = true;
    return 0;
}

bool aql_lane_idle(AqlLane *l) {
    if (!l->busy) return true;
    if (hsa_signal_load_scacquire(hsa_signal_t{l->signal}) != 0) return false;
    l->busy = false;
    return true;
}

long aql_lane_inflight(AqlLane *l) {
    if (!l->busy) return 0;
    const long v = (long)hsa_signal_load_scacquire(hsa_signal_t{l->signal});
    if (v == 0) l->busy = false;
    return v;
}

int aql_lane_wait(AqlLane *l, uint64_t timeout_ns) {
    const uint64_t t0 = mono_ns();
    for (unsigned i = 0; !aql_lane_idle(l); i++) {
        if (mono_ns() - t0 > timeout_ns) return -1;
        if (i > 1000) usleep(20);
    }
    return 0;
}

}  // namespace ocm

// Probe: dispatching a kernel on a user-mode AQL queue of our own (HSA runtime,
// no HIP stream) instead of hipLaunchKernelGGL, for the resident copy service.
//   hip_flag_us      hipLaunchKernelGGL of a kernel that stores a host-coherent flag;
//                    the host spins on the flag (launch + dispatch latency)
//   hsa_flag_us      the same kernel, from this process's code object loaded into an
//                    HSA executable, dispatched by writing one AQL packet and ringing the
//                    queue's doorbell
//   hip_launch_cpu_us / hsa_dispatch_cpu_us   host time of the launch call alone
//   sync_while_hsa_resident_us   hipDeviceSynchronize() while a persistent kernel runs
//                    on the AQL queue (HIP does not know the queue: it must not wait)
//   sync_while_hip_resident_us   the same with the persistent kernel on a HIP stream
//                    (waits for the kernel; the host stops it after ~5 ms)
//   interop_bad      words wrong after an AQL-dispatched kernel fills hipMalloc'd memory
// Every spin is bounded (1 s) and every persistent kernel leaves on a host stop word
// or after 200 ms of GPU time.
//
//   hsa_dispatch_probe <code object of this file (device only)>
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <thread>
#include <vector>

using clk = std::chrono::steady_clock;

extern "C" __global__ __launch_bounds__(256) void probe_flag_kernel(unsigned long long *flag, unsigned long long v) {
    if (threadIdx.x == 0 && blockIdx.x == 0) __hip_atomic_store(flag, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

extern "C" __global__ __launch_bounds__(256) void probe_fill_kernel(unsigned *p, unsigned long long n, unsigned nblocks) {
    for (unsigned long long i = (unsigned long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (unsigned long long)nblocks * 256)
        p[i] = (unsigned)(i * 2654435761u);
}

// Leaves on *stop != 0 or after max_ticks of s_memrealtime (100 MHz).
extern "C" __global__ __launch_bounds__(256) void probe_persist_kernel(const unsigned long long *stop,
                                                                       unsigned long long *alive,
                                                                       unsigned long long max_ticks) {
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0 && blockIdx.x == 0) __hip_atomic_store(alive, 1ull, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    for (;;) {
        unsigned long long s = 0;
        if (threadIdx.x == 0) s = __hip_atomic_load(stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        s = __shfl(s, 0);
        if (s || __builtin_amdgcn_s_memrealtime() - t0 > max_ticks) break;
        __builtin_amdgcn_s_sleep(8);
    }
    if (threadIdx.x == 0 && blockIdx.x == 0) __hip_atomic_store(alive, 2ull, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

#define CHK(x)                                                                                 \
    do {                                                                                       \
        hsa_status_t st_ = (x);                                                                \
        if (st_ != HSA_STATUS_SUCCESS) {                                                       \
            const char *m_ = nullptr;                                                          \
            hsa_status_string(st_, &m_);                                                       \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, m_ ? m_ : "?");    \
            return 1;                                                                          \
        }                                                                                      \
    } while (0)

struct Ctx {
    hsa_agent_t gpu{}, cpu{};
    uint32_t want_bdf = 0;
    bool found = false;
    hsa_amd_memory_pool_t kernarg_pool{};
    bool have_pool = false;
};

static hsa_status_t agent_cb(hsa_agent_t a, void *p) {
    Ctx *c = static_cast<Ctx *>(p);
    hsa_device_type_t t;
    if (hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t) != HSA_STATUS_SUCCESS) return HSA_STATUS_SUCCESS;
    if (t == HSA_DEVICE_TYPE_CPU && !c->cpu.handle) c->cpu = a;
    if (t == HSA_DEVICE_TYPE_GPU && !c->found) {
        uint32_t bdf = 0;
        if (hsa_agent_get_info(a, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_BDFID, &bdf) == HSA_STATUS_SUCCESS &&
            bdf == c->want_bdf) {
            c->gpu = a;
            c->found = true;
        }
    }
    return HSA_STATUS_SUCCESS;
}

static hsa_status_t pool_cb(hsa_amd_memory_pool_t pool, void *p) {
    Ctx *c = static_cast<Ctx *>(p);
    hsa_amd_segment_t seg;
    if (hsa_amd_memory_pool_get_info(pool, HSA_AMD_MEMORY_POOL_INFO_SEGMENT, &seg) != HSA_STATUS_SUCCESS ||
        seg != HSA_AMD_SEGMENT_GLOBAL)
        return HSA_STATUS_SUCCESS;
    uint32_t flags = 0;
    if (hsa_amd_memory_pool_get_info(pool, HSA_AMD_MEMORY_POOL_INFO_GLOBAL_FLAGS, &flags) != HSA_STATUS_SUCCESS)
        return HSA_STATUS_SUCCESS;
    if ((flags & HSA_AMD_MEMORY_POOL_GLOBAL_FLAG_KERNARG_INIT) && !c->have_pool) {
        c->kernarg_pool = pool;
        c->have_pool = true;
    }
    return HSA_STATUS_SUCCESS;
}

struct Kern {
    uint64_t object = 0;
    uint32_t kernarg = 0, group = 0, priv = 0;
};

static int get_kernel(hsa_executable_t ex, hsa_agent_t gpu, const char *name, Kern &k) {
    hsa_executable_symbol_t sym;
    char full[128];
    std::snprintf(full, sizeof(full), "%s.kd", name);
    CHK(hsa_executable_get_symbol_by_name(ex, full, &gpu, &sym));
    CHK(hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_OBJECT, &k.object));
    CHK(hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_KERNARG_SEGMENT_SIZE, &k.kernarg));
    CHK(hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_GROUP_SEGMENT_SIZE, &k.group));
    CHK(hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_PRIVATE_SEGMENT_SIZE, &k.priv));
    return 0;
}

// One AQL dispatch of `blocks` x 256 threads. `args` (explicit arguments, `nargs` bytes)
// go to `ka` followed by the hidden block count / group size the code object reads.
static void dispatch(hsa_queue_t *q, const Kern &k, void *ka, const void *args, size_t nargs, unsigned blocks,
                     hsa_signal_t done) {
    std::memset(ka, 0, k.kernarg);
    std::memcpy(ka, args, nargs);
    const size_t h = (nargs + 7) & ~size_t(7);
    if (h + 64 <= k.kernarg) {
        uint32_t bc[3] = {blocks, 1, 1};
        uint16_t gs[3] = {256, 1, 1};
        std::memcpy(static_cast<char *>(ka) + h, bc, sizeof(bc));
        std::memcpy(static_cast<char *>(ka) + h + 12, gs, sizeof(gs));
        uint16_t dims = 1;
        std::memcpy(static_cast<char *>(ka) + h + 64, &dims, sizeof(dims));
    }
    const uint64_t idx = hsa_queue_add_write_index_screlease(q, 1);
    while (idx - hsa_queue_load_read_index_scacquire(q) >= q->size) {
    }
    auto *p = reinterpret_cast<hsa_kernel_dispatch_packet_t *>(q->base_address) + (idx & (q->size - 1));
    p->workgroup_size_x = 256;
    p->workgroup_size_y = 1;
    p->workgroup_size_z = 1;
    p->reserved0 = 0;
    p->grid_size_x = blocks * 256u;
    p->grid_size_y = 1;
    p->grid_size_z = 1;
    p->private_segment_size = k.priv;
    p->group_segment_size = k.group;
    p->kernel_object = k.object;
    p->kernarg_address = ka;
    p->reserved2 = 0;
    p->completion_signal = done;
    const uint16_t header = (HSA_PACKET_TYPE_KERNEL_DISPATCH << HSA_PACKET_HEADER_TYPE) |
                            (HSA_FENCE_SCOPE_SYSTEM << HSA_PACKET_HEADER_SCACQUIRE_FENCE_SCOPE) |
                            (HSA_FENCE_SCOPE_SYSTEM << HSA_PACKET_HEADER_SCRELEASE_FENCE_SCOPE);
    const uint16_t setup = 1 << HSA_KERNEL_DISPATCH_PACKET_SETUP_DIMENSIONS;
    __atomic_store_n(reinterpret_cast<uint32_t *>(p), (uint32_t)header | ((uint32_t)setup << 16), __ATOMIC_RELEASE);
    hsa_signal_store_screlease(q->doorbell_signal, (hsa_signal_value_t)idx);
}

static double p50(std::vector<double> v) {
    std::sort(v.begin(), v.end());
    return v.empty() ? -1 : v[v.size() / 2] * 1e6;
}

static bool spin_until(const unsigned long long *f, unsigned long long v) {
    const auto a = clk::now();
    while (__atomic_load_n(f, __ATOMIC_ACQUIRE) != v)
        if (std::chrono::duration<double>(clk::now() - a).count() > 1.0) return false;
    return true;
}

int main(int argc, char **argv) {
    if (argc < 2) {
        std::fprintf(stderr, "usage: %s <device code object>\n", argv[0]);
        return 2;
    }
    std::vector<char> co;
    {
        FILE *f = std::fopen(argv[1], "rb");
        if (!f) {
            std::perror(argv[1]);
            return 2;
        }
        char buf[65536];
        size_t n;
        while ((n = std::fread(buf, 1, sizeof(buf), f)) > 0) co.insert(co.end(), buf, buf + n);
        std::fclose(f);
    }
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, 0) != hipSuccess) return 1;
    hipStream_t st;
    if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess) return 1;
    unsigned long long *flags = nullptr;
    if (hipHostMalloc((void **)&flags, 4096, hipHostMallocCoherent | hipHostMallocMapped) != hipSuccess) return 1;
    std::memset(flags, 0, 4096);

    CHK(hsa_init());
    Ctx c;
    c.want_bdf = ((uint32_t)prop.pciBusID << 8) | ((uint32_t)prop.pciDeviceID << 3);
    CHK(hsa_iterate_agents(agent_cb, &c));
    if (!c.found || !c.cpu.handle) {
        std::fprintf(stderr, "no HSA GPU agent with BDF %#x\n", c.want_bdf);
        return 1;
    }
    CHK(hsa_amd_agent_iterate_memory_pools(c.cpu, pool_cb, &c));
    if (!c.have_pool) {
        std::fprintf(stderr, "no kernarg pool\n");
        return 1;
    }
    hsa_code_object_reader_t rd;
    CHK(hsa_code_object_reader_create_from_memory(co.data(), co.size(), &rd));
    hsa_executable_t ex;
    CHK(hsa_executable_create_alt(HSA_PROFILE_FULL, HSA_DEFAULT_FLOAT_ROUNDING_MODE_DEFAULT, nullptr, &ex));
    CHK(hsa_executable_load_agent_code_object(ex, c.gpu, rd, nullptr, nullptr));
    CHK(hsa_executable_freeze(ex, nullptr));
    Kern kflag, kfill, kpers;
    if (get_kernel(ex, c.gpu, "probe_flag_kernel", kflag) || get_kernel(ex, c.gpu, "probe_fill_kernel", kfill) ||
        get_kernel(ex, c.gpu, "probe_persist_kernel", kpers))
        return 1;
    hsa_queue_t *q = nullptr;
    CHK(hsa_queue_create(c.gpu, 64, HSA_QUEUE_TYPE_MULTI, nullptr, nullptr, UINT32_MAX, UINT32_MAX, &q));
    (void)hsa_amd_queue_set_priority(q, HSA_AMD_QUEUE_PRIORITY_HIGH);
    void *ka = nullptr;
    CHK(hsa_amd_memory_pool_allocate(c.kernarg_pool, 4096, 0, &ka));
    CHK(hsa_amd_agents_allow_access(1, &c.gpu, nullptr, ka));
    hsa_signal_t sig;
    CHK(hsa_signal_create(1, 0, nullptr, &sig));
    auto wait_sig = [&]() {
        return hsa_signal_wait_scacquire(sig, HSA_SIGNAL_CONDITION_LT, 1, 1000000000ull, HSA_WAIT_STATE_ACTIVE) == 0;
    };

    const int n = 2000;
    int fails = 0;
    std::vector<double> t_hip, t_hsa, c_hip, c_hsa;
    // ---- HIP launch + flag ----
    for (int i = 0; i < n + 50; i++) {
        const unsigned long long v = 100000 + i;
        const auto a = clk::now();
        hipLaunchKernelGGL(probe_flag_kernel, dim3(1), dim3(256), 0, st, flags, v);
        const auto b = clk::now();
        fails += !spin_until(flags, v);
        const auto e = clk::now();
        if (i >= 50) {
            t_hip.push_back(std::chrono::duration<double>(e - a).count());
            c_hip.push_back(std::chrono::duration<double>(b - a).count());
        }
        (void)hipStreamSynchronize(st);
    }
    // ---- AQL dispatch + flag ----
    for (int i = 0; i < n + 50; i++) {
        const unsigned long long v = 200000 + i;
        struct {
            unsigned long long *f;
            unsigned long long v;
        } args{flags, v};
        hsa_signal_store_relaxed(sig, 1);
        const auto a = clk::now();
        dispatch(q, kflag, ka, &args, sizeof(args), 1, sig);
        const auto b = clk::now();
        fails += !spin_until(flags, v);
        const auto e = clk::now();
        if (i >= 50) {
            t_hsa.push_back(std::chrono::duration<double>(e - a).count());
            c_hsa.push_back(std::chrono::duration<double>(b - a).count());
        }
        fails += !wait_sig();  // the kernarg buffer is reused: wait for the kernel's end
    }
    // ---- interop: an AQL kernel fills hipMalloc'd memory ----
    const unsigned long long words = 1 << 22;
    unsigned *dbuf = nullptr;
    if (hipMalloc((void **)&dbuf, words * 4) != hipSuccess) return 1;
    if (hipMemset(dbuf, 0, words * 4) != hipSuccess || hipDeviceSynchronize() != hipSuccess) return 1;
    {
        struct {
            unsigned *p;
            unsigned long long n;
            unsigned nb;
        } args{dbuf, words, 1024};
        hsa_signal_store_relaxed(sig, 1);
        dispatch(q, kfill, ka, &args, sizeof(args), 1024, sig);
        fails += !wait_sig();
    }
    std::vector<unsigned> host(words);
    if (hipMemcpy(host.data(), dbuf, words * 4, hipMemcpyDeviceToHost) != hipSuccess) return 1;
    unsigned long long bad = 0;
    for (unsigned long long i = 0; i < words; i++) bad += host[i] != (unsigned)(i * 2654435761u);
    // ---- device sync while a persistent kernel is resident ----
    // stop word in `stopw` (coherent or write-combined host memory); returns the device
    // sync time and, in *stop_us, the time from the host's stop store to the kernel's exit flag
    unsigned long long *wc = nullptr;
    if (hipHostMalloc((void **)&wc, 4096, hipHostMallocWriteCombined | hipHostMallocMapped) != hipSuccess) return 1;
    wc[0] = 0;
    auto persist_sync = [&](bool on_hsa, unsigned long long *stopw, double *stop_us) -> double {
        __atomic_store_n(stopw, 0ull, __ATOMIC_RELEASE);
        flags[48] = 0;  // alive: 1 running, 2 left
        struct {
            const unsigned long long *stop;
            unsigned long long *alive;
            unsigned long long max_ticks;
        } args{stopw, flags + 48, 100ull * 200000};  // 200 ms
        hsa_signal_store_relaxed(sig, 1);
        if (on_hsa)
            dispatch(q, kpers, ka, &args, sizeof(args), 4, sig);
        else
            hipLaunchKernelGGL(probe_persist_kernel, dim3(4), dim3(256), 0, st, stopw, flags + 48, 100ull * 200000);
        if (!spin_until(flags + 48, 1)) return -1;
        clk::time_point ts;
        std::thread stopper([&]() {
            std::this_thread::sleep_for(std::chrono::milliseconds(5));
            ts = clk::now();
            __atomic_store_n(stopw, 1ull, __ATOMIC_RELEASE);
            __builtin_ia32_sfence();
        });
        const auto a = clk::now();
        (void)hipDeviceSynchronize();
        const double t = std::chrono::duration<double>(clk::now() - a).count();
        stopper.join();
        fails += !spin_until(flags + 48, 2);
        *stop_us = std::chrono::duration<double>(clk::now() - ts).count() * 1e6;
        if (on_hsa) fails += !wait_sig();
        (void)hipDeviceSynchronize();
        return t * 1e6;
    };
    double stop_hsa = 0, stop_hip = 0, stop_wc = 0;
    const double s_hsa = persist_sync(true, flags + 32, &stop_hsa);
    const double s_hip = persist_sync(false, flags + 32, &stop_hip);
    double s_wc = persist_sync(true, wc, &stop_wc);
    std::printf("{\"hip_flag_us\": %.2f, \"hsa_flag_us\": %.2f, \"hip_launch_cpu_us\": %.2f, \"hsa_dispatch_cpu_us\": %.2f, "
                "\"sync_while_hsa_resident_us\": %.1f, \"sync_while_hip_resident_us\": %.1f, \"sync_hsa_wc_us\": %.1f, "
                "\"stop_seen_us\": [%.1f, %.1f, %.1f], \"interop_bad\": %llu, "
                "\"kernarg_bytes\": [%u, %u, %u], \"fails\": %d}\n",
                p50(t_hip), p50(t_hsa), p50(c_hip), p50(c_hsa), s_hsa, s_hip, s_wc, stop_hsa, stop_hip, stop_wc, bad, kflag.kernarg, kfill.kernarg,
                kpers.kernarg, fails);
    (void)hsa_signal_destroy(sig);
    (void)hsa_amd_memory_pool_free(ka);
    (void)hsa_queue_destroy(q);
    (void)hsa_executable_destroy(ex);
    (void)hsa_code_object_reader_destroy(rd);
    (void)hsa_shut_down();
    (void)hipFree(dbuf);
    (void)hipHostFree(flags);
    (void)hipHostFree(wc);
    return (fails || bad) ? 1 : 0;
}


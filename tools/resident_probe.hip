// Probe library (ctypes, tools/resident_cost_probe.py): one persistent workgroup
// resident on its own stream while the caller runs other GPU work, to see which
// footprint of a resident poller delays a full-GPU GEMM. The workgroup polls a
// host flag and leaves when it is set, or after 2 s of GPU time.
//   ocmp_start(threads, heavy): threads 64 or 256; heavy keeps ~100 VGPRs live
//   ocmp_stop(): set the flag, wait for the kernel
#include <hip/hip_runtime.h>

namespace {

__global__ __launch_bounds__(256) void resident_light(const volatile unsigned long long *stop) {
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    for (;;) {
        unsigned long long s = 0;
        if (threadIdx.x == 0) s = __hip_atomic_load(stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        s = __shfl(s, 0);
        if (s || __builtin_amdgcn_s_memrealtime() - t0 > 200000000ull) break;
        __builtin_amdgcn_s_sleep(24);
    }
}

// ~100 live VGPRs across the loop (a 48 x float4 register array the compiler cannot fold).
__global__ __launch_bounds__(256) void resident_heavy(const volatile unsigned long long *stop, float4 *sink) {
    float4 r[48];
    for (int i = 0; i < 48; i++) r[i] = make_float4(threadIdx.x + i, i, 1.0f * i, 2.0f);
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    for (;;) {
        unsigned long long s = 0;
        if (threadIdx.x == 0) s = __hip_atomic_load(stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        s = __shfl(s, 0);
        if (s || __builtin_amdgcn_s_memrealtime() - t0 > 200000000ull) break;
        for (int i = 0; i < 48; i++) r[i].x += r[(i + 1) % 48].y + r[(i + 7) % 48].z;
        __builtin_amdgcn_s_sleep(24);
    }
    float4 acc = make_float4(0, 0, 0, 0);
    for (int i = 0; i < 48; i++) acc.x += r[i].x + r[i].y + r[i].z + r[i].w;
    if (acc.x == -1.0f) sink[threadIdx.x] = acc;
}

hipStream_t g_stream = nullptr;
unsigned long long *g_flag = nullptr;
float4 *g_sink = nullptr;

}  // namespace

extern "C" int ocmp_start(int threads, int heavy) {
    // a priority of its own: HIP pools hardware queues per priority, so the resident
    // kernel never sits in front of the caller's work on a shared queue
    int lo = 0, hi = 0;
    if (!g_stream && (hipDeviceGetStreamPriorityRange(&lo, &hi) != hipSuccess ||
                      hipStreamCreateWithPriority(&g_stream, hipStreamNonBlocking, hi) != hipSuccess))
        return -1;
    if (!g_flag && hipHostMalloc(reinterpret_cast<void **>(&g_flag), 4096, hipHostMallocCoherent | hipHostMallocMapped) !=
                       hipSuccess)
        return -1;
    if (!g_sink && hipMalloc(reinterpret_cast<void **>(&g_sink), 256 * sizeof(float4)) != hipSuccess) return -1;
    if (threads != 64 && threads != 256) return -1;
    __atomic_store_n(g_flag, 0ull, __ATOMIC_RELEASE);
    if (heavy)
        hipLaunchKernelGGL(resident_heavy, dim3(1), dim3(threads), 0, g_stream, g_flag, g_sink);
    else
        hipLaunchKernelGGL(resident_light, dim3(1), dim3(threads), 0, g_stream, g_flag);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

extern "C" int ocmp_stop() {
    if (!g_flag) return 0;
    __atomic_store_n(g_flag, 1ull, __ATOMIC_RELEASE);
    return hipStreamSynchronize(g_stream) == hipSuccess ? 0 : -1;
}

// Probe: where the ~13 us of a blocking launch-path op goes on MI355X.
//   launch_cpu   host time inside hipLaunchKernelGGL (kernarg + AQL packet + doorbell)
//   event_spin   launch + hipEventRecord + spin on hipEventQuery (libocm's OCM_SYNC_MODE=1)
//   stream_sync  launch + hipStreamSynchronize
//   flag_spin    launch of a kernel whose last act is a system-scope release store of a
//                host-coherent flag; the host spins on the flag (no runtime completion path):
//                launch + dispatch latency without the end-of-kernel signal
// Every host spin is bounded (1 s), and the kernels are trivial and finite.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <vector>

using clk = std::chrono::steady_clock;

__global__ __launch_bounds__(256) void empty_kernel(int *p) {
    if (threadIdx.x == 0 && blockIdx.x == 0 && p) p[0] = 1;
}

__global__ __launch_bounds__(256) void flag_kernel(unsigned long long *flags, unsigned long long v) {
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        __hip_atomic_store(&flags[0], v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(&flags[16], v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

static double p50(std::vector<double> v) {
    std::sort(v.begin(), v.end());
    return v[v.size() / 2] * 1e6;
}

int main() {
    hipStream_t st;
    if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess) return 1;
    hipEvent_t ev;
    if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) return 1;
    unsigned long long *flags = nullptr;
    if (hipHostMalloc((void **)&flags, 4096, hipHostMallocCoherent | hipHostMallocMapped) != hipSuccess) return 1;
    for (int i = 0; i < 32; i++) flags[i] = 0;
    const int n = 2000;
    std::vector<double> tl, te, ts, tf, t1;
    for (int i = 0; i < 50; i++) hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(256), 0, st, nullptr);
    if (hipStreamSynchronize(st) != hipSuccess) return 1;
    for (int i = 0; i < n; i++) {
        auto a = clk::now();
        hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(256), 0, st, nullptr);
        auto b = clk::now();
        (void)hipStreamSynchronize(st);
        tl.push_back(std::chrono::duration<double>(b - a).count());
    }
    for (int i = 0; i < n; i++) {
        auto a = clk::now();
        hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(256), 0, st, nullptr);
        (void)hipEventRecord(ev, st);
        while (hipEventQuery(ev) == hipErrorNotReady) {
        }
        te.push_back(std::chrono::duration<double>(clk::now() - a).count());
    }
    for (int i = 0; i < n; i++) {
        auto a = clk::now();
        hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(256), 0, st, nullptr);
        (void)hipStreamSynchronize(st);
        ts.push_back(std::chrono::duration<double>(clk::now() - a).count());
    }
    int fails = 0;
    for (int i = 0; i < n; i++) {
        const unsigned long long v = (unsigned long long)i + 1;
        auto a = clk::now();
        hipLaunchKernelGGL(flag_kernel, dim3(1), dim3(256), 0, st, flags, v);
        bool ok = true;
        while (__atomic_load_n(&flags[0], __ATOMIC_ACQUIRE) != v) {
            if (std::chrono::duration<double>(clk::now() - a).count() > 1.0) {
                ok = false;
                break;
            }
        }
        tf.push_back(std::chrono::duration<double>(clk::now() - a).count());
        fails += !ok;
        (void)hipStreamSynchronize(st);
    }
    std::printf("{\"launch_cpu_us\": %.2f, \"event_spin_us\": %.2f, \"stream_sync_us\": %.2f, \"flag_spin_us\": %.2f, "
                "\"fails\": %d}\n",
                p50(tl), p50(te), p50(ts), p50(tf), fails);
    (void)hipHostFree(flags);
    return fails ? 1 : 0;
}

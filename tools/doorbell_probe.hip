// Probe: round-trip latency of a persistent copy-service kernel fed through a
// host-pinned doorbell, vs a plain launch + stream sync of the same small copy.
// Every spin is bounded: the kernel exits on STOP, or after 2 s without work
// (s_memrealtime, 100 MHz); the host gives up after 1 s per op.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

struct Bell {
    unsigned long long seq;   // host -> device: next request id (STOP = ~0)
    unsigned long long bytes;
    unsigned long long pad[6];
    unsigned long long done;  // device -> host: last completed id
    unsigned long long pad2[7];
};

constexpr unsigned long long kStop = ~0ull;

__global__ __launch_bounds__(256) void service(Bell *b, const u32x4 *src, u32x4 *dst, unsigned long long *status) {
    __shared__ unsigned long long cmd[2];
    unsigned long long expect = 1;
    unsigned long long idle_start = __builtin_amdgcn_s_memrealtime();
    for (;;) {
        if (threadIdx.x == 0) {
            unsigned long long s;
            for (;;) {
                s = __hip_atomic_load(&b->seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                if (s == expect || s == kStop) break;
                if (__builtin_amdgcn_s_memrealtime() - idle_start > 200000000ull) {  // 2 s idle
                    s = kStop;
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
            cmd[0] = s;
            cmd[1] = __hip_atomic_load(&b->bytes, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        __syncthreads();
        const unsigned long long s = cmd[0], n = cmd[1];
        if (s == kStop) break;
        for (unsigned long long i = threadIdx.x; i < n / 16; i += blockDim.x) dst[i] = src[i];
        __threadfence_system();
        __syncthreads();
        if (threadIdx.x == 0) {
            __hip_atomic_store(&b->done, s, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
            idle_start = __builtin_amdgcn_s_memrealtime();
        }
        expect++;
        __syncthreads();
    }
    if (threadIdx.x == 0) *status = expect;
}

__global__ void plain_copy(const u32x4 *src, u32x4 *dst, unsigned long long n) {
    for (unsigned long long i = threadIdx.x; i < n / 16; i += blockDim.x) dst[i] = src[i];
}

int main() {
    const size_t n = 4096;
    u32x4 *src, *dst;
    unsigned long long *status;
    Bell *b;
    (void)hipMalloc(&src, 1 << 20);
    (void)hipMalloc(&dst, 1 << 20);
    (void)hipMalloc(&status, 8);
    (void)hipHostMalloc(&b, sizeof(Bell), hipHostMallocCoherent | hipHostMallocMapped);
    b->seq = 0;
    b->done = 0;
    b->bytes = n;
    hipStream_t s1, s2;
    (void)hipStreamCreateWithFlags(&s1, hipStreamNonBlocking);
    (void)hipStreamCreateWithFlags(&s2, hipStreamNonBlocking);
    std::vector<double> plain, bell;
    for (int i = 0; i < 2000; i++) {
        auto t0 = std::chrono::steady_clock::now();
        hipLaunchKernelGGL(plain_copy, dim3(1), dim3(256), 0, s2, src, dst, (unsigned long long)n);
        (void)hipStreamSynchronize(s2);
        plain.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
    }
    hipLaunchKernelGGL(service, dim3(1), dim3(256), 0, s1, b, src, dst, status);
    int fails = 0;
    for (unsigned long long i = 1; i <= 20000; i++) {
        auto t0 = std::chrono::steady_clock::now();
        __atomic_store_n(&b->seq, i, __ATOMIC_RELEASE);
        bool ok = false;
        for (;;) {
            if (__atomic_load_n(&b->done, __ATOMIC_ACQUIRE) == i) {
                ok = true;
                break;
            }
            if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(1)) break;
        }
        if (!ok) {
            fails++;
            break;
        }
        bell.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
    }
    __atomic_store_n(&b->seq, kStop, __ATOMIC_RELEASE);
    (void)hipStreamSynchronize(s1);
    std::sort(plain.begin(), plain.end());
    std::sort(bell.begin(), bell.end());
    auto pct = [](std::vector<double> &v, double q) { return v.empty() ? -1.0 : v[(size_t)(q * (v.size() - 1))]; };
    printf("{\"plain_launch_sync_p50_us\": %.2f, \"plain_p99_us\": %.2f, \"doorbell_p50_us\": %.2f, \"doorbell_p99_us\": %.2f, \"fails\": %d}\n",
           pct(plain, 0.5), pct(plain, 0.99), pct(bell, 0.5), pct(bell, 0.99), fails);
    return fails ? 1 : 0;
}

// Probe: host <-> resident-kernel ping-pong, the copy service's hand-off without the
// copy, to find which leg carries the per-process ~1.5 us small-op penalty
// (profiles/numa_mode_r04.json: the timing thread's core decides, the NUMA node
// does not). One workgroup, lane 0, polls the doorbell word and answers each value
// in the reply word; the host posts 1..N and spins for each answer.
//   pingpong_probe <cpu> <doorbell: wc|coh> <spin: plain|pause|flush> [none|get|put] [N]
// get / put: before answering, the wave copies 4 KiB from registered host memory to
// HBM (get) or back (put), as the copy service does for a 4 KiB op.
// The process pins itself to <cpu> before any HIP call. Bounded: the kernel leaves
// after N answers or 2 s of GPU time, whichever comes first.
#include <hip/hip_runtime.h>
#include <immintrin.h>
#include <sched.h>
#include <sys/mman.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

// data: 0 none; 1 "get" (4 KiB host -> HBM before answering); 2 "put" (HBM -> host)
__global__ __launch_bounds__(64) void responder(const unsigned long long *bell, unsigned long long *reply, unsigned n,
                                                int data, uint4 *host, uint4 *hbm) {
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    const int lane = threadIdx.x;
    for (unsigned long long want = 1; want <= n;) {
        const unsigned long long v = __hip_atomic_load(bell, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        if (v == want) {  // wave-uniform: every lane read the same word
            if (data) {
                const uint4 *src = data == 1 ? host : hbm;
                uint4 *dst = data == 1 ? hbm : host;
                uint4 r[4];
                for (int k = 0; k < 4; k++) r[k] = src[k * 64 + lane];
                for (int k = 0; k < 4; k++) dst[k * 64 + lane] = r[k];
                __threadfence_system();
            }
            if (lane == 0) __hip_atomic_store(reply, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
            want++;
            continue;
        }
        if (__builtin_amdgcn_s_memrealtime() - t0 > 200000000ull) break;  // 2 s
        __builtin_amdgcn_s_sleep(8);
    }
}

int main(int argc, char **argv) {
    if (argc < 4) {
        std::fprintf(stderr, "usage: %s <cpu> <wc|coh> <plain|pause|flush> [N]\n", argv[0]);
        return 2;
    }
    const int cpu = std::atoi(argv[1]);
    const bool wc = std::strcmp(argv[2], "wc") == 0;
    const int spin = std::strcmp(argv[3], "pause") == 0 ? 1 : std::strcmp(argv[3], "flush") == 0 ? 2 : 0;
    const int data = argc > 4 ? (std::strcmp(argv[4], "get") == 0 ? 1 : std::strcmp(argv[4], "put") == 0 ? 2 : 0) : 0;
    const unsigned n = argc > 5 ? (unsigned)std::atoi(argv[5]) : 3000;
    cpu_set_t set;
    CPU_ZERO(&set);
    CPU_SET(cpu, &set);
    if (sched_setaffinity(0, sizeof(set), &set) != 0) return 3;
    unsigned long long *bell = nullptr, *reply = nullptr;
    const unsigned bf = (wc ? hipHostMallocWriteCombined : hipHostMallocCoherent) | hipHostMallocMapped;
    if (hipHostMalloc(reinterpret_cast<void **>(&bell), 4096, bf) != hipSuccess ||
        hipHostMalloc(reinterpret_cast<void **>(&reply), 4096, hipHostMallocCoherent | hipHostMallocMapped) != hipSuccess)
        return 1;
    __atomic_store_n(bell, 0ull, __ATOMIC_RELEASE);
    __atomic_store_n(reply, 0ull, __ATOMIC_RELEASE);
    _mm_sfence();
    void *dbell = nullptr, *dreply = nullptr;
    if (hipHostGetDevicePointer(&dbell, bell, 0) != hipSuccess || hipHostGetDevicePointer(&dreply, reply, 0) != hipSuccess)
        return 1;
    // the data's host half as the host tier has it: shared memory registered mapped
    void *hdata = mmap(nullptr, 1 << 20, PROT_READ | PROT_WRITE, MAP_SHARED | MAP_ANONYMOUS, -1, 0);
    void *hdata_dev = nullptr, *ddata = nullptr;
    if (hdata == MAP_FAILED) return 1;
    std::memset(hdata, 1, 1 << 20);
    if (hipHostRegister(hdata, 1 << 20, hipHostRegisterMapped | hipHostRegisterPortable) != hipSuccess ||
        hipHostGetDevicePointer(&hdata_dev, hdata, 0) != hipSuccess || hipMalloc(&ddata, 1 << 20) != hipSuccess)
        return 1;
    hipStream_t st;
    if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess) return 1;
    hipLaunchKernelGGL(responder, dim3(1), dim3(64), 0, st, static_cast<const unsigned long long *>(dbell),
                       static_cast<unsigned long long *>(dreply), n, data, static_cast<uint4 *>(hdata_dev),
                       static_cast<uint4 *>(ddata));
    if (hipGetLastError() != hipSuccess) return 1;
    std::vector<double> rtt;
    rtt.reserve(n);
    bool ok = true;
    for (unsigned long long i = 1; i <= n && ok; i++) {
        const auto t0 = std::chrono::steady_clock::now();
        __atomic_store_n(bell, i, __ATOMIC_RELEASE);
        _mm_sfence();
        for (unsigned long long k = 0;; k++) {
            if (spin == 2) _mm_clflush(reply);
            if (__atomic_load_n(reply, __ATOMIC_ACQUIRE) == i) break;
            if (spin == 1) _mm_pause();
            if ((k & 0xFFFFF) == 0xFFFFF &&
                std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(500)) {
                ok = false;  // the responder left (its 2 s bound): stop
                break;
            }
        }
        rtt.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
    }
    __atomic_store_n(bell, ~0ull, __ATOMIC_RELEASE);
    _mm_sfence();
    if (hipStreamSynchronize(st) != hipSuccess) return 1;
    std::vector<double> t(rtt.begin() + std::min<size_t>(100, rtt.size()), rtt.end());
    std::sort(t.begin(), t.end());
    if (t.empty()) return 1;
    std::printf("{\"cpu\": %d, \"data\": %d, \"bell\": \"%s\", \"spin\": \"%s\", \"n\": %zu, \"rtt_us_p10\": %.2f, \"rtt_us_p50\": %.2f, "
                "\"rtt_us_p90\": %.2f, \"complete\": %s}\n",
                cpu, data, wc ? "wc" : "coh", argv[3], t.size(), t[t.size() / 10], t[t.size() / 2], t[t.size() * 9 / 10],
                ok ? "true" : "false");
    return ok ? 0 : 4;
}

// ocm_gpu_hog: hold all but a few CUs of the GPU for a bounded time.
//
// Test tool for the copy service's roster (ocm/xfer.h): a workgroup of this
// kernel declares the whole 160 KiB LDS of a CU, so each CU it lands on can run
// no other workgroup that needs LDS (the copy service's workgroups need 136 B).
// With (CUs - free) workgroups, only `free` CUs are left for another process's
// persistent service, which then cannot get its whole grid resident: its gang
// ops must complete with the members that did start.
//
//   ocm_gpu_hog [--free-cus N] [--ms T] [--device D]
//
// Prints "ready <resident workgroups> <grid>" once the grid is resident (or
// after 2 s with what is), then "done" when the kernel has left. Every
// workgroup leaves after T ms of s_memrealtime (100 MHz): the grid always drains.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>

namespace {

constexpr int kLdsWords = 163840 / 4;  // all of a CU's LDS

__global__ __launch_bounds__(64) void hog_kernel(unsigned long long ticks, unsigned *started, int *sink) {
    __shared__ int lds[kLdsWords];
    lds[threadIdx.x * 640] = (int)threadIdx.x;  // touch it: the allocation is what matters
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_fetch_add(started, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(127);
    if (lds[((threadIdx.x + 1) & 63) * 640] < 0) sink[threadIdx.x] = 1;  // never true; keeps the LDS live
}

int die(const char *what, hipError_t e) {
    std::fprintf(stderr, "ocm_gpu_hog: %s: %s\n", what, hipGetErrorString(e));
    return 1;
}

}  // namespace

int main(int argc, char **argv) {
    int free_cus = 4, ms = 3000, dev = 0;
    for (int i = 1; i + 1 < argc; i += 2) {
        if (!std::strcmp(argv[i], "--free-cus")) free_cus = std::atoi(argv[i + 1]);
        else if (!std::strcmp(argv[i], "--ms")) ms = std::atoi(argv[i + 1]);
        else if (!std::strcmp(argv[i], "--device")) dev = std::atoi(argv[i + 1]);
    }
    if (ms < 1 || ms > 60000 || free_cus < 0) {
        std::fprintf(stderr, "ocm_gpu_hog: --ms must be 1..60000, --free-cus >= 0\n");
        return 2;
    }
    hipError_t e = hipSetDevice(dev);
    if (e != hipSuccess) return die("hipSetDevice", e);
    int cus = 0;
    if ((e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev)) != hipSuccess)
        return die("CU count", e);
    const int grid = cus > free_cus ? cus - free_cus : 1;
    unsigned *started = nullptr;
    int *sink = nullptr;
    if ((e = hipHostMalloc(reinterpret_cast<void **>(&started), 128, hipHostMallocCoherent | hipHostMallocMapped)) !=
        hipSuccess)
        return die("hipHostMalloc", e);
    *started = 0;
    if ((e = hipMalloc(reinterpret_cast<void **>(&sink), 64 * sizeof(int))) != hipSuccess) return die("hipMalloc", e);
    hipStream_t st;
    if ((e = hipStreamCreateWithFlags(&st, hipStreamNonBlocking)) != hipSuccess) return die("stream", e);
    hipLaunchKernelGGL(hog_kernel, dim3(grid), dim3(64), 0, st, 100000ull * (unsigned long long)ms, started, sink);
    if ((e = hipGetLastError()) != hipSuccess) return die("launch", e);
    const auto t0 = std::chrono::steady_clock::now();
    unsigned in = 0;
    for (;;) {
        in = __atomic_load_n(started, __ATOMIC_ACQUIRE);
        if ((int)in >= grid || std::chrono::steady_clock::now() - t0 > std::chrono::seconds(2)) break;
        std::this_thread::sleep_for(std::chrono::microseconds(200));
    }
    std::printf("ready %u %d %d\n", in, grid, cus);
    std::fflush(stdout);
    if ((e = hipStreamSynchronize(st)) != hipSuccess) return die("kernel", e);
    std::printf("done\n");
    std::fflush(stdout);
    (void)hipStreamDestroy(st);
    (void)hipFree(sink);
    (void)hipHostFree(started);
    return 0;
}

// Probe: why does the persistent copy service read host-tier memory slower than a
// freshly launched kernel does (16 KiB get: ~6 us of GPU time in the service
// against 2.7 us in tools/pcie_copy_probe.hip)?
//
// One workgroup of 256 threads copies S bytes host -> device R times inside ONE
// launch, the way the resident service does between doorbells, and stamps each
// copy on the GPU clock (100 MHz). Variants of what runs between two copies:
//   acq_sys    fence(acquire, system) + s_waitcnt (the service's doorbell acquire)
//   acq_agent  fence(acquire, agent) + s_waitcnt
//   none       nothing (stale host lines may then be served from L2: timing only)
// and of the offset of the copied range in the host buffer (0 or 4096), plus a
// fresh launch per copy (the pcie_copy_probe shape) as the reference row.
// Every kernel is finite; the host checks the bytes of the last copy.
#include <hip/hip_runtime.h>
#include <sys/mman.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <vector>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

#define CHECK(x)                                                                      \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess) {                                                       \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            return 1;                                                                 \
        }                                                                             \
    } while (0)

constexpr int kThreads = 256;
constexpr int kUnroll = 8;

// the service's span copy (remainder form: every load before the first store)
__device__ __forceinline__ void copy_span(u32x4 *d, const u32x4 *s, uint64_t nv) {
    const int tid = threadIdx.x;
    uint64_t base = 0;
    for (; base + (uint64_t)kThreads * kUnroll <= nv; base += (uint64_t)kThreads * kUnroll) {
        u32x4 v[kUnroll];
#pragma unroll
        for (int k = 0; k < kUnroll; k++) v[k] = __builtin_nontemporal_load(s + base + (uint64_t)k * kThreads + tid);
#pragma unroll
        for (int k = 0; k < kUnroll; k++) d[base + (uint64_t)k * kThreads + tid] = v[k];
    }
    if (base < nv) {
        u32x4 v[kUnroll];
#pragma unroll
        for (int k = 0; k < kUnroll; k++) {
            const uint64_t i = base + (uint64_t)k * kThreads + tid;
            if (i < nv) v[k] = __builtin_nontemporal_load(s + i);
        }
#pragma unroll
        for (int k = 0; k < kUnroll; k++) {
            const uint64_t i = base + (uint64_t)k * kThreads + tid;
            if (i < nv) d[i] = v[k];
        }
    }
}

// Loads with cache-policy bits instead of an acquire: aux 16 = sc1, 17 = sc0 sc1.
template <int AUX>
__device__ __forceinline__ void copy_span_aux(u32x4 *d, const u32x4 *s, uint64_t nv) {
    const int tid = threadIdx.x;
    const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<u32x4 *>(s), 0, (int)(nv * 16), 0x00020000);
    for (uint32_t base = 0; base < nv; base += kThreads * kUnroll) {
        u32x4 v[kUnroll];
#pragma unroll
        for (int k = 0; k < kUnroll; k++) v[k] = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)((base + k * kThreads + tid) << 4), 0, AUX);
#pragma unroll
        for (int k = 0; k < kUnroll; k++)
            if (base + k * kThreads + tid < nv) d[base + k * kThreads + tid] = v[k];
    }
}

template <int MODE>  // 0 acq_sys, 1 acq_agent, 2 none, 3 sc1 loads, 4 sc0 sc1 loads (no acquire)
__global__ __launch_bounds__(kThreads) void loop_kernel(u32x4 *dst, const u32x4 *src, uint64_t nv, int reps,
                                                         unsigned long long *ts) {
    for (int r = 0; r < reps; r++) {
        if (MODE == 0) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
        if (MODE == 1) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
        if (MODE == 3)
            copy_span_aux<16>(dst, src, nv);
        else if (MODE == 4)
            copy_span_aux<17>(dst, src, nv);
        else
            copy_span(dst, src, nv);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
        if (threadIdx.x == 0) ts[r] = t1 - t0;
        __syncthreads();
    }
}

__global__ __launch_bounds__(kThreads) void once_kernel(u32x4 *dst, const u32x4 *src, uint64_t nv, unsigned long long *ts) {
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    copy_span(dst, src, nv);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) ts[0] = __builtin_amdgcn_s_memrealtime() - t0;
}

// argv[1]: host memory source: "anon" (default), "memfd" (the host tier's memfd
// slab), "memfd0"/"memfd1" (memfd with an MPOL_PREFERRED policy for NUMA node 0/1);
// argv[2]: "pool" to copy into a stream-ordered pool block (the library's local halves).
int main(int argc, char **argv) {
    const uint64_t host_bytes = 64ull << 20;
    const char *src_mode = argc > 1 ? argv[1] : "anon";
    void *host = MAP_FAILED;
    if (std::strncmp(src_mode, "memfd", 5) == 0) {
        const int fd = memfd_create("probe", MFD_CLOEXEC);
        if (fd < 0 || ftruncate(fd, (off_t)host_bytes) != 0) return 1;
        host = mmap(nullptr, host_bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
        if (host != MAP_FAILED && src_mode[5]) {
            unsigned long mask = 1ul << (src_mode[5] - '0');
            if (syscall(SYS_mbind, host, host_bytes, 1 /* MPOL_PREFERRED */, &mask, 64ul, 0u) != 0) return 1;
        }
    } else {
        host = mmap(nullptr, host_bytes, PROT_READ | PROT_WRITE, MAP_SHARED | MAP_ANONYMOUS, -1, 0);
    }
    if (host == MAP_FAILED) return 1;
    for (uint64_t i = 0; i < host_bytes / 4; i++) static_cast<unsigned *>(host)[i] = (unsigned)(i * 2654435761u);
    CHECK(hipHostRegister(host, host_bytes, hipHostRegisterMapped | hipHostRegisterPortable));
    void *hdev = nullptr;
    CHECK(hipHostGetDevicePointer(&hdev, host, 0));
    void *dev = nullptr;
    if (argc > 2 && std::strcmp(argv[2], "pool") == 0) {
        hipMemPool_t pool;
        hipMemPoolProps props = {};
        props.allocType = hipMemAllocationTypePinned;
        props.location.type = hipMemLocationTypeDevice;
        props.location.id = 0;
        CHECK(hipMemPoolCreate(&pool, &props));
        CHECK(hipMallocFromPoolAsync(&dev, 8 << 20, pool, 0));
        CHECK(hipStreamSynchronize(0));
    } else {
        CHECK(hipMalloc(&dev, 8 << 20));
    }
    unsigned long long *ts = nullptr;
    const int reps = 64;
    CHECK(hipMalloc((void **)&ts, reps * sizeof(unsigned long long)));
    std::vector<unsigned long long> h(reps);
    const char *names[] = {"acq_sys", "acq_agent", "none", "fresh", "sc1", "sc0sc1"};
    std::printf("{");
    bool first = true;
    for (uint64_t off : {0ull, 4096ull, 1ull << 20}) {
        for (uint64_t s = 4096; s <= (256u << 10); s <<= 1) {
            for (int m = 0; m < 6; m++) {
                const u32x4 *src = reinterpret_cast<const u32x4 *>(static_cast<char *>(hdev) + off);
                u32x4 *dst = reinterpret_cast<u32x4 *>(static_cast<char *>(dev) + off);
                const uint64_t nv = s / 16;
                std::vector<double> t;
                if (m != 3) {
                    if (m == 4) hipLaunchKernelGGL(loop_kernel<3>, dim3(1), dim3(kThreads), 0, 0, dst, src, nv, reps, ts);
                    if (m == 5) hipLaunchKernelGGL(loop_kernel<4>, dim3(1), dim3(kThreads), 0, 0, dst, src, nv, reps, ts);
                    if (m == 0) hipLaunchKernelGGL(loop_kernel<0>, dim3(1), dim3(kThreads), 0, 0, dst, src, nv, reps, ts);
                    if (m == 1) hipLaunchKernelGGL(loop_kernel<1>, dim3(1), dim3(kThreads), 0, 0, dst, src, nv, reps, ts);
                    if (m == 2) hipLaunchKernelGGL(loop_kernel<2>, dim3(1), dim3(kThreads), 0, 0, dst, src, nv, reps, ts);
                    CHECK(hipGetLastError());
                    CHECK(hipDeviceSynchronize());
                    CHECK(hipMemcpy(h.data(), ts, reps * sizeof(unsigned long long), hipMemcpyDeviceToHost));
                    for (int r = 4; r < reps; r++) t.push_back(h[r] / 100.0);
                } else {
                    for (int r = 0; r < 24; r++) {
                        hipLaunchKernelGGL(once_kernel, dim3(1), dim3(kThreads), 0, 0, dst, src, nv, ts);
                        CHECK(hipGetLastError());
                        CHECK(hipDeviceSynchronize());
                        CHECK(hipMemcpy(h.data(), ts, sizeof(unsigned long long), hipMemcpyDeviceToHost));
                        if (r >= 4) t.push_back(h[0] / 100.0);
                    }
                }
                std::vector<char> back(s);
                CHECK(hipMemcpy(back.data(), dst, s, hipMemcpyDeviceToHost));
                if (std::memcmp(back.data(), static_cast<char *>(host) + off, s) != 0) {
                    std::fprintf(stderr, "MISMATCH off %llu size %llu %s\n", (unsigned long long)off,
                                 (unsigned long long)s, names[m]);
                    return 1;
                }
                std::sort(t.begin(), t.end());
                std::printf("%s\"%s/off%llu/%llu\": [%.2f, %.2f]", first ? "" : ", ", names[m],
                            (unsigned long long)off, (unsigned long long)s, t[0], t[t.size() / 2]);
                first = false;
                std::fflush(stdout);
            }
        }
    }
    std::printf("}\n");
    CHECK(hipHostUnregister(host));
    munmap(host, host_bytes);
    return 0;
}

// Probe: GPU read latency of host memory by allocation kind, the question being whether
// the host tier's slabs (memfd, hipHostRegister'ed as mapped, i.e. fine-grained) could
// be read faster as another kind. One workgroup; lane 0 times 200 dependent
// system-scope loads, each from a new 4 KiB page, with s_memrealtime (100 MHz).
// Each kind is measured twice: after a GPU kernel wrote the buffer (no CPU cache holds
// its lines, as for data a put left) and after a CPU memset (lines dirty in CPU caches).
// A third pass reads one line over and over (a poller's pattern); then 1-64 workgroups
// poll at once, all in one line, a line each or a page each.
// Prints one JSON object of medians in ns. Bounded: 200 loads per launch, 8 MiB buffers.
#include <hip/hip_runtime.h>
#include <sys/mman.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <vector>

constexpr int kIters = 200;
constexpr size_t kStride = 4096 / 8;  // in words
constexpr size_t kBytes = (size_t)(kIters + 8) * 4096;

__global__ void gpu_fill(unsigned long long *p, size_t words) {
    for (size_t i = blockIdx.x * blockDim.x + threadIdx.x; i < words; i += (size_t)gridDim.x * blockDim.x) p[i] = 0;
    __threadfence_system();
}

// stride 0: every load reads the same line, as a poller of one record does
__global__ __launch_bounds__(64) void chase(const unsigned long long *p, unsigned long long *out, size_t stride) {
    if (threadIdx.x != 0) return;
    unsigned long long v = 0;
    for (int i = 0; i < kIters; i++) {
        const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
        v += __hip_atomic_load(p + (size_t)i * stride + (v & 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        out[i] = __builtin_amdgcn_s_memrealtime() - t0;
    }
    out[kIters] = v;
}

// N workgroups at once, lane 0 of each timing 200 dependent loads of its own word: all
// in one line (stride 0, as the copy service's gang pollers read one record), one line
// each (stride 16 words), or one page each (stride 512 words).
__global__ __launch_bounds__(64) void poll_many(const unsigned long long *p, unsigned long long *out, size_t stride) {
    if (threadIdx.x != 0) return;
    const unsigned long long *q = p + (size_t)blockIdx.x * stride + (stride ? 0 : (blockIdx.x & 7));
    unsigned long long v = 0, *o = out + (size_t)blockIdx.x * kIters;
    for (int i = 0; i < kIters; i++) {
        const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
        v += __hip_atomic_load(q + (v & 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        o[i] = __builtin_amdgcn_s_memrealtime() - t0 + (v & 0);
    }
}

static unsigned long long median_ns(unsigned long long *dev_out) {
    std::vector<unsigned long long> h(kIters + 1);
    if (hipMemcpy(h.data(), dev_out, (kIters + 1) * 8, hipMemcpyDeviceToHost) != hipSuccess) return 0;
    std::vector<unsigned long long> t(h.begin() + 8, h.begin() + kIters);  // the first loads warm the TLB
    std::sort(t.begin(), t.end());
    return t[t.size() / 2] * 10;
}

int main() {
    unsigned long long *out = nullptr;
    if (hipMalloc(reinterpret_cast<void **>(&out), (kIters + 1) * 8) != hipSuccess) return 1;
    struct Kind {
        const char *name;
        unsigned malloc_flags;   // hipHostMalloc, or 0 with register_flags
        unsigned register_flags;  // mmap + hipHostRegister
    } kinds[] = {
        {"hostmalloc_coherent", hipHostMallocMapped | hipHostMallocCoherent, 0},
        {"hostmalloc_noncoherent", hipHostMallocMapped | hipHostMallocNonCoherent, 0},
        {"hostmalloc_writecombined", hipHostMallocMapped | hipHostMallocWriteCombined, 0},
        {"register_mapped", 0, hipHostRegisterMapped | hipHostRegisterPortable},
        {"register_coarse", 0, hipHostRegisterMapped | hipHostRegisterPortable | hipExtHostRegisterCoarseGrained},
    };
    std::printf("{");
    bool first = true;
    for (const Kind &k : kinds) {
        void *h = nullptr;
        bool mapped = false;
        if (k.malloc_flags) {
            if (hipHostMalloc(&h, kBytes, k.malloc_flags) != hipSuccess) h = nullptr;
        } else {
            h = mmap(nullptr, kBytes, PROT_READ | PROT_WRITE, MAP_SHARED | MAP_ANONYMOUS, -1, 0);
            if (h == MAP_FAILED) h = nullptr;
            if (h) {
                std::memset(h, 0, kBytes);
                mapped = true;
                if (hipHostRegister(h, kBytes, k.register_flags) != hipSuccess) {
                    (void)hipGetLastError();
                    munmap(h, kBytes);
                    h = nullptr;
                }
            }
        }
        unsigned long long gpu_last = 0, cpu_last = 0, same_line = 0;
        if (h) {
            void *d = nullptr;
            if (hipHostGetDevicePointer(&d, h, 0) == hipSuccess) {
                unsigned long long *dp = static_cast<unsigned long long *>(d);
                hipLaunchKernelGGL(gpu_fill, dim3(64), dim3(256), 0, nullptr, dp, kBytes / 8);
                hipLaunchKernelGGL(chase, dim3(1), dim3(64), 0, nullptr, dp, out, kStride);
                if (hipDeviceSynchronize() == hipSuccess) gpu_last = median_ns(out);
                std::memset(h, 0, kBytes);
                hipLaunchKernelGGL(chase, dim3(1), dim3(64), 0, nullptr, dp, out, kStride);
                if (hipDeviceSynchronize() == hipSuccess) cpu_last = median_ns(out);
                hipLaunchKernelGGL(chase, dim3(1), dim3(64), 0, nullptr, dp, out, (size_t)0);
                if (hipDeviceSynchronize() == hipSuccess) same_line = median_ns(out);
            }
            if (mapped) {
                (void)hipHostUnregister(h);
                munmap(h, kBytes);
            } else {
                (void)hipHostFree(h);
            }
        }
        std::printf("%s\"%s\": {\"gpu_written_ns_p50\": %llu, \"cpu_written_ns_p50\": %llu, \"same_line_ns_p50\": %llu}",
                    first ? "" : ", ", k.name, gpu_last, cpu_last, same_line);
        first = false;
    }
    // concurrent pollers, write-combined host memory (the request records' kind)
    void *wc = nullptr, *wcd = nullptr;
    unsigned long long *many = nullptr;
    if (hipHostMalloc(&wc, kBytes, hipHostMallocMapped | hipHostMallocWriteCombined) == hipSuccess &&
        hipHostGetDevicePointer(&wcd, wc, 0) == hipSuccess &&
        hipMalloc(reinterpret_cast<void **>(&many), (size_t)64 * kIters * 8) == hipSuccess) {
        std::memset(wc, 0, kBytes);
        const size_t strides[] = {0, 16, 512};
        const char *sname[] = {"same_line", "line_each", "page_each"};
        for (int si = 0; si < 3; si++) {
            std::printf(", \"pollers_%s\": {", sname[si]);
            const unsigned ns[] = {1, 4, 8, 16, 32, 64};
            for (int ni = 0; ni < 6; ni++) {
                hipLaunchKernelGGL(poll_many, dim3(ns[ni]), dim3(64), 0, nullptr,
                                   static_cast<const unsigned long long *>(wcd), many, strides[si]);
                unsigned long long med = 0;
                if (hipDeviceSynchronize() == hipSuccess) {
                    std::vector<unsigned long long> h((size_t)ns[ni] * kIters);
                    if (hipMemcpy(h.data(), many, h.size() * 8, hipMemcpyDeviceToHost) == hipSuccess) {
                        std::vector<unsigned long long> t;
                        for (unsigned b = 0; b < ns[ni]; b++)
                            for (int i = 8; i < kIters; i++) t.push_back(h[(size_t)b * kIters + i]);
                        std::sort(t.begin(), t.end());
                        med = t[t.size() / 2] * 10;
                    }
                }
                std::printf("%s\"%u\": %llu", ni ? ", " : "", ns[ni], med);
            }
            std::printf("}");
        }
    }
    std::printf("}\n");
    return 0;
}

// Probe: how fast can G workgroups move S bytes between HBM and registered host
// memory (the host tier) over PCIe, as seen on the GPU clock?
//
// The copy service (csrc/src/kernels/xfer.hip) copies 32 KiB tiles with 8 x 16 B
// loads then 8 x 16 B stores per lane. On gfx9-family parts vmcnt counts loads AND
// stores in issue order, so the loads of tile k+1 wait for the stores of tile k:
// over PCIe every tile costs a full write (put) or read (get) round trip. This
// probe times alternatives on the GPU's 100 MHz clock (first workgroup start to
// last workgroup end, after its stores drained and were released system-wide):
//   tile8     current: 32 KiB tiles grid-strided over the gang, 8 loads / 8 stores
//   deep16    one contiguous chunk per workgroup, 16 loads in flight per lane
//   deep32    same, 32 loads in flight per lane (128 VGPRs of data)
//   wave8     chunk per WAVE (not workgroup), 8 loads in flight per lane
// Host memory is mmap'ed and hipHostRegister'ed, as host-tier slabs are.
// Every kernel is finite; the host verifies the bytes of every configuration.
#include <hip/hip_runtime.h>
#include <sys/mman.h>

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

__device__ __forceinline__ unsigned long long now_ticks() { return __builtin_amdgcn_s_memrealtime(); }

__device__ __forceinline__ void stamp_end(unsigned long long *ts) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        __threadfence_system();
        ts[2 * blockIdx.x + 1] = now_ticks();
    }
}

// Vectors [v0, v1) of the transfer, `D` loads in flight per lane, `lanes` lanes from `lane`.
template <int D>
__device__ __forceinline__ void deep_copy(u32x4 *dst, const u32x4 *src, uint64_t v0, uint64_t v1, int lane, int lanes) {
    uint64_t i = v0;
    for (; i + (uint64_t)D * lanes <= v1; i += (uint64_t)D * lanes) {
        u32x4 r[D];
#pragma unroll
        for (int k = 0; k < D; k++) r[k] = __builtin_nontemporal_load(src + i + (uint64_t)k * lanes + lane);
#pragma unroll
        for (int k = 0; k < D; k++) dst[i + (uint64_t)k * lanes + lane] = r[k];
    }
    if (i < v1) {
        u32x4 r[D];
#pragma unroll
        for (int k = 0; k < D; k++) {
            const uint64_t j = i + (uint64_t)k * lanes + lane;
            if (j < v1) r[k] = __builtin_nontemporal_load(src + j);
        }
#pragma unroll
        for (int k = 0; k < D; k++) {
            const uint64_t j = i + (uint64_t)k * lanes + lane;
            if (j < v1) dst[j] = r[k];
        }
    }
}

template <int MODE>
__global__ __launch_bounds__(kThreads) void copy_kernel(u32x4 *dst, const u32x4 *src, uint64_t nv, unsigned long long *ts) {
    if (threadIdx.x == 0) ts[2 * blockIdx.x] = now_ticks();
    if constexpr (MODE == 0) {
        // tile8: 2048-vector (32 KiB) tiles, grid-strided
        const uint64_t ntiles = (nv + 2047) / 2048;
        for (uint64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
            const uint64_t a = t * 2048, b = std::min<uint64_t>(a + 2048, nv);
            deep_copy<8>(dst, src, a, b, threadIdx.x, kThreads);
        }
    } else if constexpr (MODE == 1 || MODE == 2) {
        const uint64_t per = (nv + gridDim.x - 1) / gridDim.x;
        const uint64_t a = std::min<uint64_t>((uint64_t)blockIdx.x * per, nv), b = std::min<uint64_t>(a + per, nv);
        if (MODE == 1)
            deep_copy<16>(dst, src, a, b, threadIdx.x, kThreads);
        else
            deep_copy<32>(dst, src, a, b, threadIdx.x, kThreads);
    } else {
        const int waves = gridDim.x * (kThreads / 64);
        const int w = blockIdx.x * (kThreads / 64) + (threadIdx.x >> 6);
        const uint64_t per = (nv + waves - 1) / waves;
        const uint64_t a = std::min<uint64_t>((uint64_t)w * per, nv), b = std::min<uint64_t>(a + per, nv);
        deep_copy<8>(dst, src, a, b, threadIdx.x & 63, 64);
    }
    stamp_end(ts);
}

template <int MODE>
static hipError_t launch(int grid, u32x4 *dst, const u32x4 *src, uint64_t nv, unsigned long long *ts, hipStream_t st) {
    hipLaunchKernelGGL(copy_kernel<MODE>, dim3(grid), dim3(kThreads), 0, st, dst, src, nv, ts);
    return hipGetLastError();
}

int main(int argc, char **argv) {
    const uint64_t max_bytes = 8ull << 20;
    const int reps = 30;
    void *host = mmap(nullptr, max_bytes, PROT_READ | PROT_WRITE, MAP_SHARED | MAP_ANONYMOUS, -1, 0);
    if (host == MAP_FAILED) return 1;
    std::memset(host, 0x5a, max_bytes);
    CHECK(hipHostRegister(host, max_bytes, hipHostRegisterMapped | hipHostRegisterPortable));
    void *hdev = nullptr;
    CHECK(hipHostGetDevicePointer(&hdev, host, 0));
    void *dev = nullptr;
    CHECK(hipMalloc(&dev, max_bytes));
    unsigned long long *ts = nullptr;
    CHECK(hipMalloc((void **)&ts, 2 * 1024 * sizeof(unsigned long long)));
    std::vector<unsigned long long> h_ts(2 * 1024);
    std::vector<unsigned> pattern(max_bytes / 4);
    for (size_t i = 0; i < pattern.size(); i++) pattern[i] = (unsigned)(i * 2654435761u);
    hipStream_t st;
    CHECK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    const char *modes[] = {"tile8", "deep16", "deep32", "wave8"};
    const int grids[] = {1, 2, 4, 8, 16, 32, 64};
    std::printf("{");
    bool first = true;
    for (int dir = 0; dir < 2; dir++) {  // 0 get (host -> dev), 1 put (dev -> host)
        for (uint64_t s = 4096; s <= max_bytes; s <<= 1) {
            for (int m = 0; m < 4; m++) {
                for (int g : grids) {
                    const uint64_t nv = s / 16;
                    if ((uint64_t)g * 64 > nv && g > 1) continue;  // less than one vector per lane
                    u32x4 *dst = (u32x4 *)(dir ? hdev : dev);
                    const u32x4 *src = (const u32x4 *)(dir ? dev : hdev);
                    // verify once
                    if (dir == 0) {
                        std::memcpy(host, pattern.data(), s);
                        CHECK(hipMemset(dev, 0, s));
                    } else {
                        CHECK(hipMemcpy(dev, pattern.data(), s, hipMemcpyHostToDevice));
                        std::memset(host, 0, s);
                    }
                    std::vector<double> t;
                    for (int r = 0; r < reps + 3; r++) {
                        hipError_t e = m == 0   ? launch<0>(g, dst, src, nv, ts, st)
                                       : m == 1 ? launch<1>(g, dst, src, nv, ts, st)
                                       : m == 2 ? launch<2>(g, dst, src, nv, ts, st)
                                                : launch<3>(g, dst, src, nv, ts, st);
                        CHECK(e);
                        CHECK(hipStreamSynchronize(st));
                        CHECK(hipMemcpy(h_ts.data(), ts, 2 * g * sizeof(unsigned long long), hipMemcpyDeviceToHost));
                        unsigned long long lo = ~0ull, hi = 0;
                        for (int b = 0; b < g; b++) {
                            lo = std::min(lo, h_ts[2 * b]);
                            hi = std::max(hi, h_ts[2 * b + 1]);
                        }
                        if (r >= 3) t.push_back((hi - lo) / 100.0);  // us
                        if (r == 0) {
                            std::vector<unsigned> back(s / 4);
                            if (dir == 0)
                                CHECK(hipMemcpy(back.data(), dev, s, hipMemcpyDeviceToHost));
                            else
                                std::memcpy(back.data(), host, s);
                            if (std::memcmp(back.data(), pattern.data(), s) != 0) {
                                std::fprintf(stderr, "MISMATCH dir %d size %llu mode %s grid %d\n", dir,
                                             (unsigned long long)s, modes[m], g);
                                return 1;
                            }
                        }
                    }
                    std::sort(t.begin(), t.end());
                    std::printf("%s\"%s/%llu/%s/g%d\": [%.2f, %.2f]", first ? "" : ", ", dir ? "put" : "get",
                                (unsigned long long)s, modes[m], g, t[0], t[t.size() / 2]);
                    first = false;
                    std::fflush(stdout);
                }
            }
        }
    }
    std::printf("}\n");
    (void)argc;
    (void)argv;
    CHECK(hipHostUnregister(host));
    munmap(host, max_bytes);
    return 0;
}

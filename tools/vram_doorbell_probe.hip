// Probe: where should the copy service's doorbell live?
//   host  : the request word in host-coherent pinned memory; the kernel polls
//           it across PCIe (the current design, ServiceSlot).
//   vram_fg / vram_uc : the request word in fine-grained / uncached device
//           memory that the CPU writes through the BAR; the kernel polls its
//           own HBM. Only if the runtime maps that memory for the CPU: each
//           mode first checks CPU access (a SIGSEGV/SIGBUS on the first touch
//           just marks the mode unavailable).
// The completion word stays in host memory (the CPU polls its own cache).
// Each op is a 4 KiB copy (and a 0-byte "null" op for pure signalling).
// Every spin is bounded: the kernel exits on STOP or after 2 s idle; the host
// gives up after 1 s per op and then stops the kernel.
#include <hip/hip_runtime.h>
#include <immintrin.h>
#include <setjmp.h>
#include <signal.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
constexpr unsigned long long kStop = ~0ull;

struct Req {  // written by the host
    unsigned long long seq;
    unsigned long long bytes;
    unsigned long long pad[14];
};
struct Done {  // written by the device
    unsigned long long done;
    unsigned long long pad[15];
};

// fence: 0 none, 1 agent-scope acquire, 2 system-scope acquire after the doorbell
// (a persistent kernel never gets the kernel-start cache invalidation).
__global__ __launch_bounds__(256) void service(Req *r, Done *d, const u32x4 *src, u32x4 *dst, int sleep_poll, int fence) {
    __shared__ unsigned long long cmd[2];
    unsigned long long expect = 1;
    unsigned long long idle_start = __builtin_amdgcn_s_memrealtime();
    for (;;) {
        if (threadIdx.x == 0) {
            unsigned long long s;
            for (;;) {
                s = __hip_atomic_load(&r->seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                if (s == expect || s == kStop) break;
                if (__builtin_amdgcn_s_memrealtime() - idle_start > 200000000ull) {
                    s = kStop;
                    break;
                }
                if (sleep_poll) __builtin_amdgcn_s_sleep(1);
            }
            cmd[0] = s;
            cmd[1] = __hip_atomic_load(&r->bytes, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        if (fence == 1) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        if (fence == 2) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
        __syncthreads();
        const unsigned long long s = cmd[0], n = cmd[1];
        if (s == kStop) break;
        for (unsigned long long i = threadIdx.x; i < n / 16; i += blockDim.x) dst[i] = src[i];
        __syncthreads();
        if (threadIdx.x == 0) {
            __threadfence_system();
            __hip_atomic_store(&d->done, s, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
            idle_start = __builtin_amdgcn_s_memrealtime();
        }
        expect++;
        __syncthreads();
    }
}

static sigjmp_buf g_jmp;
static void on_segv(int) { siglongjmp(g_jmp, 1); }

// CPU access check in this process: a SIGSEGV/SIGBUS on the first touch
// (memory not mapped for the CPU) jumps back here instead of killing us.
static bool cpu_can_touch(void *p) {
    struct sigaction sa = {}, old_segv, old_bus;
    sa.sa_handler = on_segv;
    sigemptyset(&sa.sa_mask);
    sigaction(SIGSEGV, &sa, &old_segv);
    sigaction(SIGBUS, &sa, &old_bus);
    bool ok = false;
    if (sigsetjmp(g_jmp, 1) == 0) {
        volatile unsigned long long *q = static_cast<volatile unsigned long long *>(p);
        q[0] = 0;
        (void)q[0];
        ok = true;
    }
    sigaction(SIGSEGV, &old_segv, nullptr);
    sigaction(SIGBUS, &old_bus, nullptr);
    return ok;
}

// Host write styles of a 128-byte request record (words 0 = seq and 1 = bytes
// are what the kernel reads; the rest stands in for the copy arguments).
__attribute__((target("avx2"))) static void write_avx(Req *r, const unsigned long long *rec) {
    for (int i = 0; i < 4; i++)
        _mm256_stream_si256(reinterpret_cast<__m256i *>(r) + i, _mm256_load_si256(reinterpret_cast<const __m256i *>(rec) + i));
}
__attribute__((target("avx512f"))) static void write_avx512(Req *r, const unsigned long long *rec) {
    for (int i = 0; i < 2; i++)
        _mm512_stream_si512(reinterpret_cast<__m512i *>(r) + i, _mm512_load_si512(reinterpret_cast<const __m512i *>(rec) + i));
}
static void write_words(Req *r, const unsigned long long *rec) {
    unsigned long long *q = reinterpret_cast<unsigned long long *>(r);
    for (int i = 15; i >= 1; i--) __atomic_store_n(q + i, rec[i], __ATOMIC_RELAXED);
    __atomic_store_n(q, rec[0], __ATOMIC_RELEASE);
}

static double pct(std::vector<double> &v, double q) {
    if (v.empty()) return -1.0;
    std::sort(v.begin(), v.end());
    return v[(size_t)(q * (v.size() - 1))];
}

int main() {
    u32x4 *src, *dst;
    Done *d;
    if (hipMalloc(&src, 1 << 20) != hipSuccess || hipMalloc(&dst, 1 << 20) != hipSuccess ||
        hipHostMalloc(&d, sizeof(Done), hipHostMallocCoherent | hipHostMallocMapped) != hipSuccess) {
        printf("{\"error\": \"alloc\"}\n");
        return 1;
    }
    hipStream_t st;
    (void)hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
    struct Mode {
        const char *name;
        unsigned flags;  // 0: host pinned
    } modes[] = {{"host", 0}, {"vram_fg", hipDeviceMallocFinegrained}, {"vram_uc", hipDeviceMallocUncached}};
    setvbuf(stderr, nullptr, _IONBF, 0);
    fprintf(stderr, "start\n");
    std::string out = "{";
    int rc = 0;
    for (auto &m : modes) {
        Req *r = nullptr;
        hipError_t e = m.flags ? hipExtMallocWithFlags(reinterpret_cast<void **>(&r), sizeof(Req), m.flags)
                               : hipHostMalloc(reinterpret_cast<void **>(&r), sizeof(Req), hipHostMallocCoherent | hipHostMallocMapped);
        char buf[512];
        if (e != hipSuccess) {
            (void)hipGetLastError();
            snprintf(buf, sizeof(buf), "\"%s\": {\"error\": \"%s\"}, ", m.name, hipGetErrorString(e));
            out += buf;
            continue;
        }
        fprintf(stderr, "%s: allocated %p\n", m.name, (void *)r);
        if (m.flags && !cpu_can_touch(r)) {
            snprintf(buf, sizeof(buf), "\"%s\": {\"error\": \"not CPU-accessible\"}, ", m.name);
            out += buf;
            (void)hipFree(r);
            continue;
        }
        for (int variant = 0; variant <= 6; variant++) {
            const int sleep_poll = variant == 1, fence = (variant == 2 || variant == 3) ? variant - 1 : 0;
            const int style = variant >= 4 ? variant - 3 : 0;  // 1 words, 2 avx, 3 avx512
            if (style == 2 && !__builtin_cpu_supports("avx2")) continue;
            if (style == 3 && !__builtin_cpu_supports("avx512f")) continue;
            std::memset((void *)d, 0, sizeof(Done));
            if (m.flags)
                (void)hipMemset(r, 0, sizeof(Req));
            else
                std::memset((void *)r, 0, sizeof(Req));
            (void)hipDeviceSynchronize();
            fprintf(stderr, "%s sleep%d: launching\n", m.name, sleep_poll);
            hipLaunchKernelGGL(service, dim3(1), dim3(256), 0, st, r, d, src, dst, sleep_poll, fence);
            std::vector<double> lat4k, lat0;
            int fails = 0;
            unsigned long long i = 1;
            for (; i <= 20000 && !fails; i++) {
                const unsigned long long bytes = (i & 1) ? 4096 : 0;
                auto t0 = std::chrono::steady_clock::now();
                alignas(64) unsigned long long rec[16] = {i, bytes};
                for (int k = 2; k < 16; k++) rec[k] = i * 31 + k;
                if (style == 0) {
                    __atomic_store_n(&r->bytes, bytes, __ATOMIC_RELAXED);
                    __atomic_store_n(&r->seq, i, __ATOMIC_RELEASE);
                } else if (style == 1) {
                    write_words(r, rec);
                } else if (style == 2) {
                    write_avx(r, rec);
                } else {
                    write_avx512(r, rec);
                }
                _mm_sfence();  // BAR mappings may be write-combined; NT stores need it anyway
                for (;;) {
                    if (__atomic_load_n(&d->done, __ATOMIC_ACQUIRE) == i) break;
                    if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(1)) {
                        fails++;
                        break;
                    }
                }
                const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
                if (i > 200) (bytes ? lat4k : lat0).push_back(us);
            }
            __atomic_store_n(&r->seq, kStop, __ATOMIC_RELEASE);
            if (m.flags) __builtin_ia32_sfence();
            fprintf(stderr, "%s sleep%d: %llu ops, %d fails; stopping\n", m.name, sleep_poll, i - 1, fails);
            (void)hipStreamSynchronize(st);
            fprintf(stderr, "%s sleep%d: stopped\n", m.name, sleep_poll);
            snprintf(buf, sizeof(buf),
                     "\"%s_sleep%d_fence%d_style%d\": {\"p50_4k_us\": %.2f, \"p99_4k_us\": %.2f, \"p50_null_us\": %.2f, "
                     "\"p99_null_us\": %.2f, \"fails\": %d}, ",
                     m.name, sleep_poll, fence, style, pct(lat4k, 0.5), pct(lat4k, 0.99), pct(lat0, 0.5), pct(lat0, 0.99), fails);
            out += buf;
            if (fails) rc = 1;
        }
        if (m.flags)
            (void)hipFree(r);
        else
            (void)hipHostFree(r);
    }
    out += "\"ok\": 1}";
    printf("%s\n", out.c_str());
    return rc;
}

// Host-gated ticks: how soon does work queued behind hipStreamWaitValue64 run
// after the host releases the gate, against launching the same work then?
// The question behind a tick design where the allgather is queued ahead and
// released by the host once its records are written (no seal kernel).
//   gate_probe [iters]   -> one JSON object on stdout (p50 / p90 us)
// Variants:
//   launch_flag    launch a one-lane kernel that stores k to pinned host memory; spin on it
//   gate_flag      the same kernel queued behind a wait on a signal-memory gate; host stores the gate
//   gate_gather    a 1-rank ncclAllGather of one tick slot (pinned send -> pinned recv) behind the
//                  gate; the host fills the send slot, releases the gate, spins on the recv copy
//   seal_gather    today's tick: a one-wave kernel copies the slot into HBM, then the allgather; the
//                  host spins on the recv copy (launches issued at t0)
// Result on MI355X (round 3): gate_flag works, but ncclAllGather queued behind the
// gate never returns to the caller: RCCL's enqueue blocks the host thread on the
// gated stream, so the thread that would release the gate never gets there. A
// host-gated allgather is not a usable tick design; the seal kernel stays.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <unistd.h>
#include <vector>

#define CK(x)                                                                  \
    do {                                                                       \
        hipError_t e_ = (x);                                                   \
        if (e_ != hipSuccess) {                                                \
            std::fprintf(stderr, "%s failed at %d: %s\n", #x, __LINE__, hipGetErrorString(e_)); \
            std::exit(1);                                                      \
        }                                                                      \
    } while (0)
#define NK(x)                                                                  \
    do {                                                                       \
        if ((x) != ncclSuccess) {                                              \
            std::fprintf(stderr, "%s failed at %d\n", #x, __LINE__);           \
            std::exit(1);                                                      \
        }                                                                      \
    } while (0)

constexpr size_t kSlot = 1376;  // sizeof(TickSlot)

__global__ void flag_kernel(unsigned long long *flag, unsigned long long v) {
    if (threadIdx.x == 0) __hip_atomic_store(flag, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ void seal_like_kernel(const unsigned long long *src, unsigned long long *dst, int words) {
    for (int i = threadIdx.x; i < words; i += 64)
        dst[i] = __hip_atomic_load(src + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

static double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static void spin_eq(volatile unsigned long long *p, unsigned long long v) {
    const double t0 = now_us();
    while (__atomic_load_n(p, __ATOMIC_ACQUIRE) != v) {
        if (now_us() - t0 > 2e6) {
            std::fprintf(stderr, "timed out waiting for %llu\n", v);
            std::_Exit(2);  // no runtime teardown behind a wait that never ends
        }
    }
}

struct Stat {
    double p50, p90;
};
static Stat stat(std::vector<double> t) {
    std::sort(t.begin(), t.end());
    return {t[t.size() / 2], t[t.size() * 9 / 10]};
}

int main(int argc, char **argv) {
    const int iters = argc > 1 ? std::atoi(argv[1]) : 300;
    CK(hipSetDevice(0));
    int can_wait = 0;
    CK(hipDeviceGetAttribute(&can_wait, hipDeviceAttributeCanUseStreamWaitValue, 0));
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    const unsigned fl = hipHostMallocMapped | hipHostMallocCoherent | hipHostMallocPortable;
    unsigned long long *flag, *send, *recv, *dslot;
    CK(hipHostMalloc(reinterpret_cast<void **>(&flag), 64, fl));
    CK(hipHostMalloc(reinterpret_cast<void **>(&send), kSlot, fl));
    CK(hipHostMalloc(reinterpret_cast<void **>(&recv), kSlot, fl));
    CK(hipMalloc(reinterpret_cast<void **>(&dslot), kSlot));
    std::memset(flag, 0, 64);
    std::memset(send, 0, kSlot);
    std::memset(recv, 0, kSlot);
    unsigned long long *gate = nullptr;
    if (can_wait) CK(hipExtMallocWithFlags(reinterpret_cast<void **>(&gate), 8, hipMallocSignalMemory));
    if (gate) *reinterpret_cast<volatile unsigned long long *>(gate) = 0;
    std::fprintf(stderr, "init: can_wait=%d gate=%p\n", can_wait, (void *)gate);
    ncclUniqueId id;
    NK(ncclGetUniqueId(&id));
    ncclComm_t comm;
    NK(ncclCommInitRank(&comm, 1, id, 0));
    unsigned long long k = 0;
    const int words = (int)(kSlot / 8);
    // warm everything up once
    hipLaunchKernelGGL(flag_kernel, dim3(1), dim3(64), 0, st, flag, ++k);
    NK(ncclAllGather(send, recv, kSlot, ncclUint8, comm, st));
    CK(hipStreamSynchronize(st));
    std::fprintf(stderr, "warm\n");

    std::vector<double> a, b, c, d;
    for (int i = 0; i < iters; i++) {
        // launch_flag
        const unsigned long long v1 = ++k;
        double t0 = now_us();
        hipLaunchKernelGGL(flag_kernel, dim3(1), dim3(64), 0, st, flag, v1);
        spin_eq(flag, v1);
        a.push_back(now_us() - t0);
        CK(hipStreamSynchronize(st));
        if (i == 0) std::fprintf(stderr, "launch_flag ok\n");
        if (gate) {
            // gate_flag
            const unsigned long long v2 = ++k;
            CK(hipStreamWaitValue64(st, gate, v2, hipStreamWaitValueGte, ~0ull));
            hipLaunchKernelGGL(flag_kernel, dim3(1), dim3(64), 0, st, flag, v2);
            std::this_thread::sleep_for(std::chrono::microseconds(200));
            t0 = now_us();
            __atomic_store_n(reinterpret_cast<volatile unsigned long long *>(gate), v2, __ATOMIC_RELEASE);
            spin_eq(flag, v2);
            b.push_back(now_us() - t0);
            CK(hipStreamSynchronize(st));
            if (i == 0) std::fprintf(stderr, "gate_flag ok\n");
            // gate_gather
            const unsigned long long v3 = ++k;
            CK(hipStreamWaitValue64(st, gate, v3, hipStreamWaitValueGte, ~0ull));
            NK(ncclAllGather(send, recv, kSlot, ncclUint8, comm, st));
            std::this_thread::sleep_for(std::chrono::microseconds(200));
            t0 = now_us();
            for (int w = 0; w < words; w++) send[w] = v3;
            __atomic_store_n(reinterpret_cast<volatile unsigned long long *>(gate), v3, __ATOMIC_RELEASE);
            spin_eq(recv + words - 1, v3);
            c.push_back(now_us() - t0);
            CK(hipStreamSynchronize(st));
            if (i == 0) std::fprintf(stderr, "gate_gather ok\n");
        }
        // seal_gather
        const unsigned long long v4 = ++k;
        t0 = now_us();
        for (int w = 0; w < words; w++) send[w] = v4;
        hipLaunchKernelGGL(seal_like_kernel, dim3(1), dim3(64), 0, st, send, dslot, words);
        NK(ncclAllGather(dslot, recv, kSlot, ncclUint8, comm, st));
        spin_eq(recv + words - 1, v4);
        d.push_back(now_us() - t0);
        CK(hipStreamSynchronize(st));
    }
    const Stat sa = stat(a), sd = stat(d);
    std::printf("{\"iters\": %d, \"can_wait_value\": %d, \"launch_flag\": [%.2f, %.2f], \"seal_gather\": [%.2f, %.2f]",
                iters, can_wait, sa.p50, sa.p90, sd.p50, sd.p90);
    if (gate) {
        const Stat sb = stat(b), sc = stat(c);
        std::printf(", \"gate_flag\": [%.2f, %.2f], \"gate_gather\": [%.2f, %.2f]", sb.p50, sb.p90, sc.p50, sc.p90);
    }
    std::printf(", \"unit\": \"us [p50, p90]\"}\n");
    NK(ncclCommDestroy(comm));
    return 0;
}

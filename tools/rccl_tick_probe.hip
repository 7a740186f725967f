// Floor of one control tick on RCCL: what a 1-rank ncclAllGather of one
// TickSlot (1352 B) costs end to end, against a bare kernel launch and a
// runtime copy, with the completion spin the tick thread uses. Also the
// back-to-back rate (64 queued ops, one sync) = the GPU-side cost alone.
//   rccl_tick_probe [iters]   -> one JSON object on stdout
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <string>
#include <vector>

#define CK(x)                                                                  \
    do {                                                                       \
        if ((x) != hipSuccess) {                                               \
            std::fprintf(stderr, "%s failed at %d\n", #x, __LINE__);           \
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

__global__ void empty_kernel() {}

static double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static void spin(hipStream_t s) {
    hipError_t e;
    while ((e = hipStreamQuery(s)) == hipErrorNotReady) {
    }
    CK(e);
}

static double median_us(int iters, const std::function<void()> &op) {
    std::vector<double> t;
    for (int i = 0; i < iters + 20; i++) {
        const double t0 = now_us();
        op();
        if (i >= 20) t.push_back(now_us() - t0);
    }
    std::sort(t.begin(), t.end());
    return t[t.size() / 2];
}

int main(int argc, char **argv) {
    const int iters = argc > 1 ? std::atoi(argv[1]) : 300;
    const size_t bytes = 1352;
    CK(hipSetDevice(0));
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    ncclUniqueId id;
    NK(ncclGetUniqueId(&id));
    ncclComm_t comm;
    NK(ncclCommInitRank(&comm, 1, id, 0));
    void *ds, *dr, *hs, *hr, *ms, *mr;
    CK(hipMalloc(&ds, bytes));
    CK(hipMalloc(&dr, bytes));
    CK(hipHostMalloc(&hs, bytes));
    CK(hipHostMalloc(&hr, bytes));
    CK(hipHostMalloc(&ms, bytes, hipHostMallocMapped | hipHostMallocCoherent));
    CK(hipHostMalloc(&mr, bytes, hipHostMallocMapped | hipHostMallocCoherent));
    std::string out = "{";
    auto add = [&](const char *k, double v) {
        char b[96];
        std::snprintf(b, sizeof(b), "%s\"%s\": %.2f", out.size() > 1 ? ", " : "", k, v);
        out += b;
    };
    add("kernel_launch_spin_us", median_us(iters, [&] {
            empty_kernel<<<1, 64, 0, st>>>();
            spin(st);
        }));
    add("memcpy_d2d_spin_us", median_us(iters, [&] {
            CK(hipMemcpyAsync(dr, ds, bytes, hipMemcpyDeviceToDevice, st));
            spin(st);
        }));
    add("allgather_dev_sync_us", median_us(iters, [&] {
            NK(ncclAllGather(ds, dr, bytes, ncclUint8, comm, st));
            CK(hipStreamSynchronize(st));
        }));
    add("allgather_dev_spin_us", median_us(iters, [&] {
            NK(ncclAllGather(ds, dr, bytes, ncclUint8, comm, st));
            spin(st);
        }));
    add("allgather_dev_h2d_d2h_spin_us", median_us(iters, [&] {
            CK(hipMemcpyAsync(ds, hs, bytes, hipMemcpyHostToDevice, st));
            NK(ncclAllGather(ds, dr, bytes, ncclUint8, comm, st));
            CK(hipMemcpyAsync(hr, dr, bytes, hipMemcpyDeviceToHost, st));
            spin(st);
        }));
    add("allgather_mapped_spin_us", median_us(iters, [&] {
            NK(ncclAllGather(ms, mr, bytes, ncclUint8, comm, st));
            spin(st);
        }));
    // graph replay of the device-buffer allgather
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
    NK(ncclAllGather(ds, dr, bytes, ncclUint8, comm, st));
    CK(hipStreamEndCapture(st, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    add("allgather_graph_dev_spin_us", median_us(iters, [&] {
            CK(hipGraphLaunch(ge, st));
            spin(st);
        }));
    // back-to-back: 64 queued, one sync -> GPU-side cost per op
    const double t0 = now_us();
    for (int r = 0; r < 10; r++) {
        for (int i = 0; i < 64; i++) NK(ncclAllGather(ds, dr, bytes, ncclUint8, comm, st));
        spin(st);
    }
    add("allgather_dev_back_to_back_us", (now_us() - t0) / 640.0);
    const double t1 = now_us();
    for (int r = 0; r < 10; r++) {
        for (int i = 0; i < 64; i++) empty_kernel<<<1, 64, 0, st>>>();
        spin(st);
    }
    add("kernel_back_to_back_us", (now_us() - t1) / 640.0);
    out += "}";
    std::printf("%s\n", out.c_str());
    (void)hipGraphExecDestroy(ge);
    (void)hipGraphDestroy(g);
    (void)ncclCommDestroy(comm);
    return 0;
}

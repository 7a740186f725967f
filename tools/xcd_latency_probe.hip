// Probe: latency of one load across PCIe (host-coherent memory, system scope) and of
// one load from HBM that misses the caches, seen from each XCD of the MI355X.
// 64 workgroups (round-robin over the 8 XCDs); lane 0 of each times 200 dependent
// loads with s_memrealtime (100 MHz) and reads its XCD from the XCC_ID hardware
// register. Prints per-XCD medians as JSON. Bounded: 200 loads per workgroup.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

constexpr int kBlocks = 64, kIters = 200;

__global__ __launch_bounds__(64) void xcd_latency(const unsigned long long *host, const unsigned long long *hbm,
                                                  unsigned long long *out) {
    if (threadIdx.x != 0) return;
    const unsigned xcc = __builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 20) & 0xFu;  // HW_REG_XCC_ID[3:0]
    unsigned long long ph[kIters], pd[kIters];
    unsigned long long v = 0;
    for (int i = 0; i < kIters; i++) {
        const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
        v += __hip_atomic_load(host + (v & 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        ph[i] = __builtin_amdgcn_s_memrealtime() - t0;
    }
    for (int i = 0; i < kIters; i++) {
        const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
        // a different line each time, system scope: not served by this CU's caches
        v += __hip_atomic_load(hbm + (size_t)(blockIdx.x * kIters + i) * 64 + (v & 1), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_SYSTEM);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        pd[i] = __builtin_amdgcn_s_memrealtime() - t0;
    }
    unsigned long long *o = out + blockIdx.x * (2 * kIters + 2);
    o[0] = xcc;
    o[1] = v;
    for (int i = 0; i < kIters; i++) {
        o[2 + i] = ph[i];
        o[2 + kIters + i] = pd[i];
    }
}

int main() {
    unsigned long long *host = nullptr, *hbm = nullptr, *out = nullptr;
    if (hipHostMalloc(reinterpret_cast<void **>(&host), 4096, hipHostMallocCoherent | hipHostMallocMapped) != hipSuccess)
        return 1;
    host[0] = 0;
    host[1] = 0;
    const size_t hbm_words = (size_t)kBlocks * kIters * 64 + 64;
    if (hipMalloc(reinterpret_cast<void **>(&hbm), hbm_words * 8) != hipSuccess ||
        hipMemset(hbm, 0, hbm_words * 8) != hipSuccess)
        return 1;
    const size_t out_words = (size_t)kBlocks * (2 * kIters + 2);
    if (hipMalloc(reinterpret_cast<void **>(&out), out_words * 8) != hipSuccess) return 1;
    hipLaunchKernelGGL(xcd_latency, dim3(kBlocks), dim3(64), 0, nullptr, host, hbm, out);
    if (hipDeviceSynchronize() != hipSuccess) return 1;
    std::vector<unsigned long long> h(out_words);
    if (hipMemcpy(h.data(), out, out_words * 8, hipMemcpyDeviceToHost) != hipSuccess) return 1;
    std::vector<std::vector<unsigned long long>> pcie(16), local(16);
    for (int b = 0; b < kBlocks; b++) {
        const unsigned long long *o = h.data() + (size_t)b * (2 * kIters + 2);
        const unsigned x = (unsigned)o[0] & 15u;
        for (int i = 10; i < kIters; i++) {  // the first loads warm the TLB
            pcie[x].push_back(o[2 + i]);
            local[x].push_back(o[2 + kIters + i]);
        }
    }
    std::printf("{");
    bool first = true;
    for (int x = 0; x < 16; x++) {
        if (pcie[x].empty()) continue;
        std::sort(pcie[x].begin(), pcie[x].end());
        std::sort(local[x].begin(), local[x].end());
        std::printf("%s\"xcd%d\": {\"pcie_load_ns_p50\": %llu, \"pcie_load_ns_p10\": %llu, \"hbm_load_ns_p50\": %llu}",
                    first ? "" : ", ", x, pcie[x][pcie[x].size() / 2] * 10, pcie[x][pcie[x].size() / 10] * 10,
                    local[x][local[x].size() / 2] * 10);
        first = false;
    }
    std::printf("}\n");
    return 0;
}

// Seal kernel of the RCCL tick transport (ocm/tick.h): runs in the tick's
// stream right before its ncclAllGather, so the records a tick carries are
// chosen when the tick executes, not when it was queued.
//
// One wave. The host appended records to a ring in pinned host memory and
// released `published` (x86 stores are ordered; sfence after). Lane 0 reads
// `published` at system scope, then every record word is read at system scope
// (sc0 sc1: never served from a cache line left by an earlier lap of the ring)
// and stored to the send slot in HBM. The collective that follows in the same
// stream reads the slot after this kernel ends.
#include <hip/hip_runtime.h>

#include "ocm/tick.h"

namespace ocm {
namespace {

__global__ __launch_bounds__(64) void tick_seal_kernel(const TickRing *ring, uint64_t *consumed, TickSlot *slot) {
    const int lane = threadIdx.x;
    const uint64_t c = *consumed;  // this stream's own counter: plain load
    const uint64_t pub = __hip_atomic_load(&ring->published, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    const uint64_t pending = pub > c ? pub - c : 0;
    const uint32_t n = pending < (uint64_t)kTickMsgs ? (uint32_t)pending : (uint32_t)kTickMsgs;
    constexpr int kWords = (int)(sizeof(TickRecord) / sizeof(uint64_t));  // 21
    for (int w = lane; w < (int)n * kWords; w += 64) {
        const int r = w / kWords, k = w % kWords;
        const uint64_t *src = reinterpret_cast<const uint64_t *>(&ring->rec[(c + (uint64_t)r) & (kTickRing - 1)]) + k;
        uint64_t *dst = reinterpret_cast<uint64_t *>(&slot->rec[r]) + k;
        *dst = __hip_atomic_load(src, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    if (lane == 0) {
        slot->count = n;
        slot->busy = pending > n ? 1u : 0u;
        slot->first = c;
        *consumed = c + n;
    }
}

__global__ __launch_bounds__(64) void tick_done_kernel(uint64_t *flag, uint64_t seq) {
    // Stream order: the collective before this kernel has finished and its
    // stores to the gathered slots are released at its end.
    if (threadIdx.x == 0) __hip_atomic_store(flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

}  // namespace

hipError_t tick_done_launch(uint64_t *flag, uint64_t seq, hipStream_t stream) {
    (void)hipGetLastError();  // report this launch, not an earlier call's error
    hipLaunchKernelGGL(tick_done_kernel, dim3(1), dim3(64), 0, stream, flag, seq);
    return hipGetLastError();
}

hipError_t tick_seal_launch(const TickRing *ring, uint64_t *consumed, TickSlot *slot, hipStream_t stream) {
    (void)hipGetLastError();  // report this launch, not an earlier call's error
    hipLaunchKernelGGL(tick_seal_kernel, dim3(1), dim3(64), 0, stream, ring, consumed, slot);
    return hipGetLastError();
}

}  // namespace ocm

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

#include <algorithm>
#include <cstdlib>
#include <cstring>

#include "ocm/tick.h"

namespace ocm {
namespace {

__device__ __forceinline__ uint64_t sys_load(const uint64_t *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Two round trips: `published` first, then the records it covers (OCM_TICK_SEAL_SPEC=0).
__device__ __forceinline__ uint64_t wave_xor64(uint64_t v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)v, off, 64);
        const uint32_t hi = (uint32_t)__shfl_xor((int)(uint32_t)(v >> 32), off, 64);
        v ^= ((uint64_t)hi << 32) | lo;
    }
    return v;
}

__global__ __launch_bounds__(64) void tick_seal2_kernel(const TickRing *ring, uint64_t *consumed, TickSlot *slot,
                                                       uint64_t tick, uint64_t *ctr) {
    const int lane = threadIdx.x;
    const uint64_t c = *consumed;  // this stream's own counter: plain load
    const uint64_t pub = sys_load(&ring->published);
    const uint64_t pending = pub > c ? pub - c : 0;
    const uint32_t n = pending < (uint64_t)kTickMsgs ? (uint32_t)pending : (uint32_t)kTickMsgs;
    for (int w = lane; w < (int)n * kTickRecordWords; w += 64) {
        const int r = w / kTickRecordWords, k = w % kTickRecordWords;
        const uint64_t *src = reinterpret_cast<const uint64_t *>(&ring->rec[(c + (uint64_t)r) & (kTickRing - 1)]) + k;
        uint64_t *dst = reinterpret_cast<uint64_t *>(&slot->rec[r]) + k;
        *dst = sys_load(src);
    }
    __syncthreads();  // the slot's records, written above, are hashed below
    uint64_t rt = 0;
    if ((uint32_t)lane < n) rt = tick_record_tag(reinterpret_cast<const uint64_t *>(&slot->rec[lane]), c + (uint64_t)lane);
    rt = wave_xor64(rt);
    if (lane == 0) {
        if (ctr) tick = *ctr + 1;  // graph-captured ticks number themselves
        const uint32_t busy = pending > n ? 1u : 0u;
        slot->count = n;
        slot->busy = busy;
        slot->first = c;
        slot->tick = tick;
        slot->tag = tick_slot_tag(n, busy, c, tick, rt);
        *consumed = c + n;
        if (ctr) *ctr = tick;
    }
}

// Speculative seal (one PCIe round trip instead of two): lanes 0..kTickMsgs-1
// each load record c + lane (21 words) and its tag, lane 63 loads `published`,
// all in flight together. A record whose tag does not match was read before the
// host finished it (it cannot be a published one then): every record the tick
// takes is read again after `published` is known, the two-round-trip path.
// Measured: the seal was 2.6 us of a ~9 us tick (profiles/rocprof_tick_kernels_r02.json).
// With `wait` (s_memrealtime ticks, 100 MHz) the read repeats while the ring
// holds nothing unsent, up to that long: a record the host posts just after the
// previous tick completed then rides this tick rather than the next one.
//
// `ctr` (graph-captured ticks, whose arguments are fixed at capture): the tick
// number is the device counter + 1, stored back by the seal (seals run in
// stream order, one at a time).
__global__ __launch_bounds__(64) void tick_seal_kernel(const TickRing *ring, uint64_t *consumed, TickSlot *slot,
                                                      uint64_t tick, uint64_t wait, uint64_t *ctr, const uint32_t *bell,
                                                      uint32_t *bell_seen) {
    const int lane = threadIdx.x;
    // Seals run one at a time (one stream, or two alternating streams ordered by an
    // event), but possibly on different queues: agent-scope (sc1) load and store.
    const uint64_t c = __hip_atomic_load(consumed, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    uint64_t w[kTickRecordWords];
    uint64_t tag = 0, pub = 0;
    const uint64_t j = c + (uint64_t)lane;
    const uint64_t *src = reinterpret_cast<const uint64_t *>(&ring->rec[j & (kTickRing - 1)]);
    uint64_t t_end = __builtin_amdgcn_s_memrealtime() + wait;
    if (bell) {
        // Idle tick: poll only `published` and the host-wide doorbell (two words over
        // PCIe, ~0.6 us apart) until one moves or the idle period ends, then read the
        // records once below. Polling the whole outbox for up to a millisecond would
        // pull ~1 GB/s over the GPU's PCIe link the whole time the mesh is idle.
        const uint32_t seen = __hip_atomic_load(bell_seen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        uint32_t rung = seen;
        for (;;) {
            uint64_t pub_l = 0;
            uint32_t bell_l = 0;
            if (lane == 63) pub_l = sys_load(&ring->published);
            if (lane == 62) bell_l = __hip_atomic_load(bell, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            pub = ((uint64_t)__builtin_amdgcn_readlane((int)(pub_l >> 32), 63) << 32) |
                  (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)pub_l, 63);
            rung = (uint32_t)__builtin_amdgcn_readlane((int)bell_l, 62);
            // Uniform exit: pub and the bell are read-lane broadcasts and the clock is scalar.
            if (pub > c || rung != seen || (int64_t)(__builtin_amdgcn_s_memrealtime() - t_end) >= 0) break;
            __builtin_amdgcn_s_sleep(16);
        }
        if (lane == 0) __hip_atomic_store(bell_seen, rung, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        wait = 0;  // one read of the outbox now
        t_end = 0;
    }
    for (;;) {
        uint64_t pub_l = 0;
        if (lane < kTickMsgs) {
#pragma unroll
            for (int k = 0; k < kTickRecordWords; k++) w[k] = sys_load(src + k);
            tag = sys_load(&ring->tag[j & (kTickRing - 1)]);
        }
        if (lane == 63) pub_l = sys_load(&ring->published);
        pub = ((uint64_t)__builtin_amdgcn_readlane((int)(pub_l >> 32), 63) << 32) |
              (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)pub_l, 63);
        // Uniform exit: pub is read-lane broadcast and the clock is scalar.
        if (pub > c || wait == 0 || (int64_t)(__builtin_amdgcn_s_memrealtime() - t_end) >= 0) break;
    }
    const uint64_t pending = pub > c ? pub - c : 0;
    const uint32_t n = pending < (uint64_t)kTickMsgs ? (uint32_t)pending : (uint32_t)kTickMsgs;
    const bool mine = (uint32_t)lane < n;
    const bool torn = mine && tick_record_tag(w, j) != tag;
    uint64_t rt = mine ? tag : 0;
    if (__builtin_amdgcn_ballot_w64(torn) != 0 && mine) {
#pragma unroll
        for (int k = 0; k < kTickRecordWords; k++) w[k] = sys_load(src + k);  // published: complete now
        rt = tick_record_tag(w, j);
    }
    if (mine) {
        uint64_t *dst = reinterpret_cast<uint64_t *>(&slot->rec[lane]);
#pragma unroll
        for (int k = 0; k < kTickRecordWords; k++) dst[k] = w[k];
    }
    rt = wave_xor64(rt);
    if (lane == 0) {
        if (ctr) tick = __hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1;
        const uint32_t busy = pending > n ? 1u : 0u;
        slot->count = n;
        slot->busy = busy;
        slot->first = c;
        slot->tick = tick;
        slot->tag = tick_slot_tag(n, busy, c, tick, rt);
        __hip_atomic_store(consumed, c + n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (ctr) __hip_atomic_store(ctr, tick, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
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

hipError_t tick_seal_launch(const TickRing *ring, uint64_t *consumed, TickSlot *slot, uint64_t tick, uint32_t wait_us,
                            hipStream_t stream, uint64_t *tick_ctr, const uint32_t *bell, uint32_t *bell_seen) {
    (void)hipGetLastError();  // report this launch, not an earlier call's error
    static const bool spec = [] {
        const char *v = std::getenv("OCM_TICK_SEAL_SPEC");
        return !(v && std::strcmp(v, "0") == 0);
    }();
    // s_memrealtime: 100 MHz; idle ticks wait up to 20 ms, busy ones a few us
    const uint64_t wait = (uint64_t)std::min<uint32_t>(wait_us, 20000) * 100;
    if (!bell_seen) bell = nullptr;
    if (spec || bell)
        hipLaunchKernelGGL(tick_seal_kernel, dim3(1), dim3(64), 0, stream, ring, consumed, slot, tick, wait, tick_ctr,
                           bell, bell_seen);
    else
        hipLaunchKernelGGL(tick_seal2_kernel, dim3(1), dim3(64), 0, stream, ring, consumed, slot, tick, tick_ctr);
    return hipGetLastError();
}

}  // namespace ocm

// Kernel dispatch on user-mode AQL queues owned by libocm (HSA runtime), next
// to HIP's streams.
//
// The resident copy service lives on such a queue. HIP does not know it, so a
// device-wide synchronize (hipDeviceSynchronize, torch.cuda.synchronize) never
// waits for the persistent kernel, and the service can stay resident across an
// application's compute phases instead of leaving after 50 us (the round-3
// design, which made every small op after an idle gap pay a relaunch). A
// dispatch is one 64-byte packet and a doorbell store: 0.04 us of host time
// against 2.2 us for hipLaunchKernelGGL (profiles/hsa_dispatch_probe_r04.json).
//
// The kernels come from a gfx950 device code object embedded in libocm at build
// time (the same xfer.hip source the HIP fat binary is built from), loaded into
// an HSA executable for the agent whose PCI location matches the HIP device.
#pragma once
#include <cstddef>
#include <cstdint>

namespace ocm {

struct AqlKernel {
    uint64_t object = 0;         // kernel descriptor address
    uint32_t kernarg_bytes = 0;  // explicit + hidden arguments
    uint32_t group_bytes = 0;    // static LDS
    uint32_t private_bytes = 0;  // scratch per work-item
};

// One queue, its completion signal (the dispatches still running: every
// dispatch adds one, the packet processor subtracts one when it completes) and
// two kernarg slots used in turn, so a dispatch may follow one that is still
// running (the packets carry no barrier bit: the second starts as soon as every
// workgroup of the first has been dispatched).
struct AqlLane {
    void *queue = nullptr;  // hsa_queue_t *
    uint64_t signal = 0;    // hsa_signal_t handle
    void *kernarg = nullptr;
    unsigned slot = 0;      // kernarg slot of the last dispatch
    bool busy = false;      // a dispatch was issued and not yet seen complete
    bool kernarg_wc = false;  // kernarg buffer in write-combined host memory (else the runtime's pool)
};

// Load the embedded code object for HIP device `hip_device` (idempotent per
// process). 0 on success; -1 with *why set when the HSA path is unusable.
int aql_open(int hip_device, const char **why);
// The kernel named `symbol` in the embedded code object (after aql_open).
int aql_kernel(const char *symbol, AqlKernel *k);
int aql_lane_create(AqlLane *l, bool high_priority);
void aql_lane_destroy(AqlLane *l);
// One 1-D dispatch of `blocks` x `threads`: `args` (the explicit kernel
// arguments, `nargs` bytes) followed by the hidden arguments the code object
// reads (block count, group size, grid dimensions). The lane must be idle unless
// `overlap`: then at most one dispatch may still run (its kernel must have read
// its arguments already), and the new one starts once all of its workgroups
// have been dispatched. `barrier`: the new one starts only once every earlier
// dispatch of the lane has completed (the packet's barrier bit).
int aql_dispatch(AqlLane *l, const AqlKernel &k, const void *args, size_t nargs, unsigned blocks, unsigned threads,
                 bool overlap = false, bool barrier = false);
// Whether the lane's dispatches have completed (a load of its signal).
bool aql_lane_idle(AqlLane *l);
// Dispatches of the lane still running.
long aql_lane_inflight(AqlLane *l);
// Wait up to timeout_ns for the lane's dispatch to complete. 0: idle.
int aql_lane_wait(AqlLane *l, uint64_t timeout_ns);

}  // namespace ocm

// Fused optimizer kernels that update parameters in place while their state
// lives in a remote (striped) oncilla allocation: the kernel reads and writes
// the state straight from peer HBM over xGMI (or the pinned host tier), with
// no staging copy. See csrc/src/kernels/optim.hip.
#pragma once

#include <hip/hip_runtime_api.h>

#include <cstdint>

#include "ocm/xfer.h"

namespace ocm {

struct AdamArgs {
    float *p;                        // parameters (this GPU), n elements, 16-byte aligned (bf16: 8-byte)
    const float *g;                  // gradients (this GPU), n elements, 16-byte aligned (bf16: 8-byte)
    char *ext[kXferMaxExtents];      // extent bases of the striped state space
    uint32_t n_ext;
    uint32_t unit_shift;             // log2(stripe unit) when n_ext > 1
    uint64_t m_off, v_off;           // byte offsets of element 0's exp_avg / exp_avg_sq (16-byte aligned)
    uint64_t n;                      // elements
    float b1, b2, eps, wd;           // betas, eps, L2 weight decay
    float step_size;                 // lr / (1 - b1^t)
    float inv_sqrt_bc2;              // 1 / sqrt(1 - b2^t)
    uint32_t bf16;                   // 1: p and g are bf16; fp32 master weights at w_off in the state
    uint64_t w_off;                  // byte offset of element 0's master weight (bf16 mode, 16-byte aligned)
    uint32_t decoupled;              // 1: AdamW (p *= decay before the step; wd unused)
    float decay;                     // 1 - lr * weight_decay (AdamW)
    uint32_t host_state;             // 1: the state is all in the pinned host tier (PCIe-bound launch shape)
    uint32_t host_span;              // (set by the launcher) bytes of the host extent the kernel may touch
};

// Many parameters in one launch: blockIdx.y picks the tensor (descriptors ride
// in the kernarg segment), blockIdx.x strides within it. The common fields
// (extents, hyper-parameters, bf16 / decoupled) come from `c`; its per-tensor
// fields are unused.
struct AdamTensor {
    void *p;                         // fp32 or bf16 parameters (alignment as in AdamArgs)
    const void *g;
    uint64_t n, w_off, m_off, v_off;
};
constexpr int kAdamMaxTensors = 32;
struct AdamMultiArgs {
    AdamArgs c;
    uint32_t count;
    AdamTensor t[kAdamMaxTensors];
};
static_assert(sizeof(AdamMultiArgs) < 4096, "kernarg segment limit");
hipError_t adam_remote_multi_launch(const AdamMultiArgs &a, hipStream_t stream);

// torch.optim.Adam's update (L2 weight decay, bias correction), or AdamW's
// (decoupled weight decay) with `decoupled`, one pass:
// reads p, g (local) and m, v (remote), writes p (local) and m, v (remote).
// bf16 mode: the update runs on the fp32 master weights (remote) and p gets
// their bf16 rounding (round to nearest even).
hipError_t adam_remote_launch(const AdamArgs &a, hipStream_t stream);

}  // namespace ocm

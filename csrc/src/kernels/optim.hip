// gfx950 fused Adam over remote optimizer state (see ocm/optim.h).
//
// Each lane owns 4 consecutive elements: 16-byte loads of p and g from local
// HBM and of exp_avg / exp_avg_sq from the state's extents (peer HBM over
// xGMI, or pinned host memory over PCIe), the update in registers, 16-byte
// stores back. A 16-byte vector never crosses a stripe unit (units are powers
// of two >= 16 and the offsets are 16-byte aligned), so the extent math runs
// once per vector. Lanes keep kVec (4) vectors in flight before the first use,
// which covers the xGMI round trip. The tail (n % 4) is done by lane 0 of
// the last workgroup, element by element.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>

#include "ocm/optim.h"

namespace ocm {

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kThreads = 256;

__device__ __forceinline__ char *state_ptr(const AdamArgs &a, uint64_t x) {
    if (a.n_ext == 1) return a.ext[0] + x;
    const uint64_t u = x >> a.unit_shift;
    const uint64_t mask = (1ull << a.unit_shift) - 1;
    if (u <= 0xFFFFFFFFull) {
        // Stripe over 3/5/6/7 peers: 64-bit division is a ~100-instruction
        // software routine on gfx950, 32-bit a handful (unit counts fit easily).
        const uint32_t u32 = (uint32_t)u, q = u32 / a.n_ext;
        return a.ext[u32 - q * a.n_ext] + (((uint64_t)q << a.unit_shift) | (x & mask));
    }
    return a.ext[u % a.n_ext] + (((u / a.n_ext) << a.unit_shift) | (x & mask));
}

__device__ __forceinline__ float adam1(float &p, float g, float &m, float &v, const AdamArgs &a) {
    if (a.decoupled)
        p = p * a.decay;  // AdamW: p *= 1 - lr * weight_decay, gradient untouched
    else if (a.wd != 0.f)
        g = g + a.wd * p;  // Adam: L2 term in the gradient
    m = m + (1.f - a.b1) * (g - m);  // torch: exp_avg.lerp_(grad, 1 - beta1)
    v = a.b2 * v + (1.f - a.b2) * g * g;
    const float denom = sqrtf(v) * a.inv_sqrt_bc2 + a.eps;
    p = p - a.step_size * (m / denom);
    return p;
}

template <int kVec>  // vectors per lane in flight per iteration
__global__ __launch_bounds__(kThreads) void adam_remote_kernel(AdamArgs a) {
    const uint64_t nvec = a.n >> 2;
    const uint64_t lanes = (uint64_t)gridDim.x * kThreads;
    const uint64_t tid = (uint64_t)blockIdx.x * kThreads + threadIdx.x;
    f32x4 *p4 = reinterpret_cast<f32x4 *>(a.p);
    const f32x4 *g4 = reinterpret_cast<const f32x4 *>(a.g);
    for (uint64_t base = tid; base < nvec; base += lanes * kVec) {
        f32x4 p[kVec], g[kVec], m[kVec], v[kVec];
        f32x4 *mp[kVec], *vp[kVec];
#pragma unroll
        for (int k = 0; k < kVec; k++) {
            const uint64_t i = base + (uint64_t)k * lanes;
            if (i < nvec) {
                mp[k] = reinterpret_cast<f32x4 *>(state_ptr(a, a.m_off + (i << 4)));
                vp[k] = reinterpret_cast<f32x4 *>(state_ptr(a, a.v_off + (i << 4)));
                m[k] = __builtin_nontemporal_load(mp[k]);
                v[k] = __builtin_nontemporal_load(vp[k]);
                p[k] = p4[i];
                g[k] = __builtin_nontemporal_load(g4 + i);
            }
        }
#pragma unroll
        for (int k = 0; k < kVec; k++) {
            const uint64_t i = base + (uint64_t)k * lanes;
            if (i < nvec) {
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    float pj = p[k][j], mj = m[k][j], vj = v[k][j];
                    adam1(pj, g[k][j], mj, vj, a);
                    p[k][j] = pj;
                    m[k][j] = mj;
                    v[k][j] = vj;
                }
                p4[i] = p[k];
                __builtin_nontemporal_store(m[k], mp[k]);
                __builtin_nontemporal_store(v[k], vp[k]);
            }
        }
    }
    if (blockIdx.x == gridDim.x - 1 && threadIdx.x == 0) {
        for (uint64_t i = nvec << 2; i < a.n; i++) {
            float *mq = reinterpret_cast<float *>(state_ptr(a, a.m_off + 4 * i));
            float *vq = reinterpret_cast<float *>(state_ptr(a, a.v_off + 4 * i));
            float pj = a.p[i], mj = *mq, vj = *vq;
            adam1(pj, a.g[i], mj, vj, a);
            a.p[i] = pj;
            *mq = mj;
            *vq = vj;
        }
    }
}

// ---- state in the pinned host tier, one extent (the N=1 case) ----
// PCIe, not HBM, bounds this: the state streams in and out over one x16 Gen5
// link at once. Buffer loads/stores on the extent (uniform base, 32-bit lane
// offsets) so the stores can carry sc1 (write-through), which streams into host
// memory faster than nontemporal or plain stores (profiles/pcie_stream_r03.json:
// 57.0 vs 55.5 GB/s), and a grid of its own (OCM_ADAM_HOST_GRID): PCIe reads
// want fewer streams than HBM.
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
constexpr int kAuxNT = 2, kAuxSC1 = 16;

template <int kVec>
__global__ __launch_bounds__(kThreads) void adam_host_kernel(AdamArgs a, uint32_t span) {
    const uint64_t nvec = a.n >> 2;
    const uint64_t lanes = (uint64_t)gridDim.x * kThreads;
    const uint64_t tid = (uint64_t)blockIdx.x * kThreads + threadIdx.x;
    f32x4 *p4 = reinterpret_cast<f32x4 *>(a.p);
    const f32x4 *g4 = reinterpret_cast<const f32x4 *>(a.g);
    // the extent holds [min(m_off, v_off), +span): both arrays addressed from its base
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(a.ext[0], 0, (int)span, 0x00020000);
    const uint32_t m0 = (uint32_t)a.m_off, v0 = (uint32_t)a.v_off;
    for (uint64_t base = tid; base < nvec; base += lanes * kVec) {
        f32x4 p[kVec], g[kVec], m[kVec], v[kVec];
#pragma unroll
        for (int k = 0; k < kVec; k++) {
            const uint64_t i = base + (uint64_t)k * lanes;
            const uint32_t o = (uint32_t)(i << 4);  // past-the-end lanes: dropped by the range check
            m[k] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(m0 + o), 0, kAuxNT));
            v[k] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(v0 + o), 0, kAuxNT));
            if (i < nvec) {
                p[k] = p4[i];
                g[k] = __builtin_nontemporal_load(g4 + i);
            }
        }
#pragma unroll
        for (int k = 0; k < kVec; k++) {
            const uint64_t i = base + (uint64_t)k * lanes;
            if (i < nvec) {
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    float pj = p[k][j], mj = m[k][j], vj = v[k][j];
                    adam1(pj, g[k][j], mj, vj, a);
                    p[k][j] = pj;
                    m[k][j] = mj;
                    v[k][j] = vj;
                }
                p4[i] = p[k];
                const uint32_t o = (uint32_t)(i << 4);
                __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, m[k]), rs, (int)(m0 + o), 0, kAuxSC1);
                __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v[k]), rs, (int)(v0 + o), 0, kAuxSC1);
            }
        }
    }
    if (blockIdx.x == gridDim.x - 1 && threadIdx.x == 0) {
        for (uint64_t i = nvec << 2; i < a.n; i++) {
            float *mq = reinterpret_cast<float *>(a.ext[0] + a.m_off + 4 * i);
            float *vq = reinterpret_cast<float *>(a.ext[0] + a.v_off + 4 * i);
            float pj = a.p[i], mj = *mq, vj = *vq;
            adam1(pj, a.g[i], mj, vj, a);
            a.p[i] = pj;
            *mq = mj;
            *vq = vj;
        }
    }
}

// ---- mixed precision: bf16 parameters and gradients here, fp32 master
// weights and moments in the remote half. Local footprint 4 bytes/parameter
// (bf16 p + g), remote 12; one pass updates the master, the moments and the
// bf16 copy (round to nearest even, like torch's .to(torch.bfloat16)).
typedef unsigned short u16x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float bf16_to_f32(unsigned short h) { return __uint_as_float((unsigned)h << 16); }

__device__ __forceinline__ unsigned short f32_to_bf16(float f) {
    unsigned u = __float_as_uint(f);
    if ((u & 0x7fffffffu) > 0x7f800000u) return (unsigned short)((u >> 16) | 0x40u);  // quiet NaN
    u += 0x7fffu + ((u >> 16) & 1u);
    return (unsigned short)(u >> 16);
}

template <int kVec>
__global__ __launch_bounds__(kThreads) void adam_remote_bf16_kernel(AdamArgs a) {
    const uint64_t nvec = a.n >> 2;
    const uint64_t lanes = (uint64_t)gridDim.x * kThreads;
    const uint64_t tid = (uint64_t)blockIdx.x * kThreads + threadIdx.x;
    u16x4 *p4 = reinterpret_cast<u16x4 *>(a.p);
    const u16x4 *g4 = reinterpret_cast<const u16x4 *>(a.g);
    for (uint64_t base = tid; base < nvec; base += lanes * kVec) {
        f32x4 w[kVec], m[kVec], v[kVec];
        u16x4 g[kVec];
        f32x4 *wp[kVec], *mp[kVec], *vp[kVec];
#pragma unroll
        for (int k = 0; k < kVec; k++) {
            const uint64_t i = base + (uint64_t)k * lanes;
            if (i < nvec) {
                wp[k] = reinterpret_cast<f32x4 *>(state_ptr(a, a.w_off + (i << 4)));
                mp[k] = reinterpret_cast<f32x4 *>(state_ptr(a, a.m_off + (i << 4)));
                vp[k] = reinterpret_cast<f32x4 *>(state_ptr(a, a.v_off + (i << 4)));
                w[k] = __builtin_nontemporal_load(wp[k]);
                m[k] = __builtin_nontemporal_load(mp[k]);
                v[k] = __builtin_nontemporal_load(vp[k]);
                g[k] = __builtin_nontemporal_load(g4 + i);
            }
        }
#pragma unroll
        for (int k = 0; k < kVec; k++) {
            const uint64_t i = base + (uint64_t)k * lanes;
            if (i < nvec) {
                u16x4 out;
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    float wj = w[k][j], mj = m[k][j], vj = v[k][j];
                    adam1(wj, bf16_to_f32(g[k][j]), mj, vj, a);
                    w[k][j] = wj;
                    m[k][j] = mj;
                    v[k][j] = vj;
                    out[j] = f32_to_bf16(wj);
                }
                p4[i] = out;
                __builtin_nontemporal_store(w[k], wp[k]);
                __builtin_nontemporal_store(m[k], mp[k]);
                __builtin_nontemporal_store(v[k], vp[k]);
            }
        }
    }
    if (blockIdx.x == gridDim.x - 1 && threadIdx.x == 0) {
        unsigned short *p16 = reinterpret_cast<unsigned short *>(a.p);
        const unsigned short *g16 = reinterpret_cast<const unsigned short *>(a.g);
        for (uint64_t i = nvec << 2; i < a.n; i++) {
            float *wq = reinterpret_cast<float *>(state_ptr(a, a.w_off + 4 * i));
            float *mq = reinterpret_cast<float *>(state_ptr(a, a.m_off + 4 * i));
            float *vq = reinterpret_cast<float *>(state_ptr(a, a.v_off + 4 * i));
            float wj = *wq, mj = *mq, vj = *vq;
            adam1(wj, bf16_to_f32(g16[i]), mj, vj, a);
            *wq = wj;
            *mq = mj;
            *vq = vj;
            p16[i] = f32_to_bf16(wj);
        }
    }
}

// One launch for up to kAdamMaxTensors parameters (see AdamMultiArgs).
// kHost: the state is one pinned host-tier extent whose offsets fit 32 bits:
// buffer loads, write-through (sc1) stores into host memory (see adam_host_kernel).
template <bool kBf16, bool kHost, int kV = 4>
__global__ __launch_bounds__(kThreads) void adam_multi_kernel(AdamMultiArgs a) {
    const AdamTensor &T = a.t[blockIdx.y];  // uniform: scalar loads from the kernarg segment
    const AdamArgs &c = a.c;
    const uint64_t nvec = T.n >> 2;
    const uint64_t lanes = (uint64_t)gridDim.x * kThreads;
    const uint64_t tid = (uint64_t)blockIdx.x * kThreads + threadIdx.x;
    __amdgpu_buffer_rsrc_t rs;
    if constexpr (kHost) rs = __builtin_amdgcn_make_buffer_rsrc(c.ext[0], 0, (int)c.host_span, 0x00020000);
    auto host_ld = [&](uint64_t off) {
        return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(uint32_t)off, 0, kAuxNT));
    };
    auto host_st = [&](uint64_t off, f32x4 x) {
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, x), rs, (int)(uint32_t)off, 0, kAuxSC1);
    };
    for (uint64_t base = tid; base < nvec; base += lanes * kV) {
        f32x4 w[kV], m[kV], v[kV], g[kV];
        f32x4 *wp[kV], *mp[kV], *vp[kV];
#pragma unroll
        for (int k = 0; k < kV; k++) {
            const uint64_t i = base + (uint64_t)k * lanes;
            if (i < nvec) {
                if constexpr (kHost) {
                    m[k] = host_ld(T.m_off + (i << 4));
                    v[k] = host_ld(T.v_off + (i << 4));
                } else {
                    mp[k] = reinterpret_cast<f32x4 *>(state_ptr(c, T.m_off + (i << 4)));
                    vp[k] = reinterpret_cast<f32x4 *>(state_ptr(c, T.v_off + (i << 4)));
                    m[k] = __builtin_nontemporal_load(mp[k]);
                    v[k] = __builtin_nontemporal_load(vp[k]);
                }
                if constexpr (kBf16) {
                    if constexpr (kHost) {
                        w[k] = host_ld(T.w_off + (i << 4));
                    } else {
                        wp[k] = reinterpret_cast<f32x4 *>(state_ptr(c, T.w_off + (i << 4)));
                        w[k] = __builtin_nontemporal_load(wp[k]);
                    }
                    const u16x4 gh = __builtin_nontemporal_load(reinterpret_cast<const u16x4 *>(T.g) + i);
#pragma unroll
                    for (int j = 0; j < 4; j++) g[k][j] = bf16_to_f32(gh[j]);
                } else {
                    w[k] = reinterpret_cast<const f32x4 *>(T.p)[i];
                    g[k] = __builtin_nontemporal_load(reinterpret_cast<const f32x4 *>(T.g) + i);
                }
            }
        }
#pragma unroll
        for (int k = 0; k < kV; k++) {
            const uint64_t i = base + (uint64_t)k * lanes;
            if (i < nvec) {
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    float wj = w[k][j], mj = m[k][j], vj = v[k][j];
                    adam1(wj, g[k][j], mj, vj, c);
                    w[k][j] = wj;
                    m[k][j] = mj;
                    v[k][j] = vj;
                }
                if constexpr (kBf16) {
                    u16x4 out;
#pragma unroll
                    for (int j = 0; j < 4; j++) out[j] = f32_to_bf16(w[k][j]);
                    reinterpret_cast<u16x4 *>(T.p)[i] = out;
                    if constexpr (kHost)
                        host_st(T.w_off + (i << 4), w[k]);
                    else
                        __builtin_nontemporal_store(w[k], wp[k]);
                } else {
                    reinterpret_cast<f32x4 *>(T.p)[i] = w[k];
                }
                if constexpr (kHost) {
                    host_st(T.m_off + (i << 4), m[k]);
                    host_st(T.v_off + (i << 4), v[k]);
                } else {
                    __builtin_nontemporal_store(m[k], mp[k]);
                    __builtin_nontemporal_store(v[k], vp[k]);
                }
            }
        }
    }
    if (blockIdx.x == gridDim.x - 1 && threadIdx.x == 0) {
        for (uint64_t i = nvec << 2; i < T.n; i++) {
            float *mq = reinterpret_cast<float *>(state_ptr(c, T.m_off + 4 * i));
            float *vq = reinterpret_cast<float *>(state_ptr(c, T.v_off + 4 * i));
            float mj = *mq, vj = *vq, wj, gj;
            if constexpr (kBf16) {
                wj = *reinterpret_cast<float *>(state_ptr(c, T.w_off + 4 * i));
                gj = bf16_to_f32(static_cast<const unsigned short *>(T.g)[i]);
            } else {
                wj = static_cast<float *>(T.p)[i];
                gj = static_cast<const float *>(T.g)[i];
            }
            adam1(wj, gj, mj, vj, c);
            *mq = mj;
            *vq = vj;
            if constexpr (kBf16) {
                *reinterpret_cast<float *>(state_ptr(c, T.w_off + 4 * i)) = wj;
                static_cast<unsigned short *>(T.p)[i] = f32_to_bf16(wj);
            } else {
                static_cast<float *>(T.p)[i] = wj;
            }
        }
    }
}

}  // namespace

static int env_int(const char *k, int dflt) {
    const char *v = std::getenv(k);
    return (v && *v) ? std::atoi(v) : dflt;
}

hipError_t adam_remote_launch(const AdamArgs &a, hipStream_t stream) {
    if (a.n == 0) return hipSuccess;
    if (a.n_ext < 1 || a.n_ext > (uint32_t)kXferMaxExtents) return hipErrorInvalidValue;
    if (a.n_ext > 1 && a.unit_shift < 4) return hipErrorInvalidValue;
    if (a.bf16 ? ((((uintptr_t)a.p | (uintptr_t)a.g) & 7u) || ((a.w_off | a.m_off | a.v_off) & 15u))
               : (((uintptr_t)a.p | (uintptr_t)a.g | a.m_off | a.v_off) & 15u))
        return hipErrorInvalidValue;
    // Measured (profiles/optim_offload_r01.json "adam_kernel_sweep"): 4 vectors
    // per lane and 2 workgroups per CU are the fastest on HBM state (1.40 ms for
    // 256 Mi params); 8 vectors per lane is 4x slower. Knobs kept for re-tuning.
    static const int vec = env_int("OCM_ADAM_VEC", 4);
    static const int per_cu = env_int("OCM_ADAM_BLOCKS_PER_CU", 2);
    const int v = vec == 2 ? 2 : 4;
    const uint64_t nvec = a.n >> 2;
    uint64_t want = (nvec + (uint64_t)kThreads * v - 1) / ((uint64_t)kThreads * v);
    if (want < 1) want = 1;
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
        cus = 256;
    const uint64_t cap = (uint64_t)cus * (uint64_t)(per_cu > 0 ? per_cu : 2);
    unsigned grid = (unsigned)(want < cap ? want : cap);
    static const int force_grid = env_int("OCM_ADAM_GRID", 0);
    if (force_grid > 0) grid = (unsigned)force_grid;
    // Host-tier state in one extent, both arrays within 4 GiB of its base: the PCIe
    // variant (OCM_ADAM_HOST=0 keeps the generic kernel).
    static const int host_kernel = env_int("OCM_ADAM_HOST", 1);
    // 128 workgroups: 91 GiB/s of state (both directions of the link at once) against
    // 82 for the HBM-tuned full-chip grid; 64-160 are equal, 192 and up lose
    // (profiles/adam_host_probe_r03.json).
    static const int host_grid = env_int("OCM_ADAM_HOST_GRID", 128);
    const uint64_t end = (a.m_off > a.v_off ? a.m_off : a.v_off) + (nvec << 4);
    if (!a.bf16 && a.host_state && host_kernel && a.n_ext == 1 && end < (1ull << 32)) {
        if (host_grid > 0 && force_grid <= 0) grid = (unsigned)std::min<uint64_t>((uint64_t)host_grid, want);
        if (v == 2)
            hipLaunchKernelGGL(adam_host_kernel<2>, dim3(grid), dim3(kThreads), 0, stream, a, (uint32_t)end);
        else
            hipLaunchKernelGGL(adam_host_kernel<4>, dim3(grid), dim3(kThreads), 0, stream, a, (uint32_t)end);
        return hipGetLastError();
    }
    if (a.bf16)
        hipLaunchKernelGGL(adam_remote_bf16_kernel<4>, dim3(grid), dim3(kThreads), 0, stream, a);
    else if (v == 2)
        hipLaunchKernelGGL(adam_remote_kernel<2>, dim3(grid), dim3(kThreads), 0, stream, a);
    else
        hipLaunchKernelGGL(adam_remote_kernel<4>, dim3(grid), dim3(kThreads), 0, stream, a);
    return hipGetLastError();
}

hipError_t adam_remote_multi_launch(const AdamMultiArgs &a, hipStream_t stream) {
    if (a.count == 0) return hipSuccess;
    if (a.count > (uint32_t)kAdamMaxTensors) return hipErrorInvalidValue;
    if (a.c.n_ext < 1 || a.c.n_ext > (uint32_t)kXferMaxExtents) return hipErrorInvalidValue;
    if (a.c.n_ext > 1 && a.c.unit_shift < 4) return hipErrorInvalidValue;
    uint64_t biggest = 0, total = 0;
    for (uint32_t k = 0; k < a.count; k++) {
        const AdamTensor &t = a.t[k];
        const uintptr_t pal = a.c.bf16 ? 7u : 15u;
        if ((((uintptr_t)t.p | (uintptr_t)t.g) & pal) || ((t.m_off | t.v_off | (a.c.bf16 ? t.w_off : 0)) & 15u))
            return hipErrorInvalidValue;
        if (t.n > biggest) biggest = t.n;
        total += t.n;
    }
    if (biggest == 0) return hipSuccess;
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
        cus = 256;
    // Blocks per tensor (uniform over blockIdx.y): the tuned total of 2 workgroups
    // per CU, shared in proportion to the biggest tensor's part of the work, so
    // equal tensors split it evenly and one big tensor among small ones gets
    // nearly all of it; the extra blocks of small tensors exit at once.
    uint64_t want = ((biggest >> 2) + (uint64_t)kThreads * 4 - 1) / ((uint64_t)kThreads * 4);
    if (want < 1) want = 1;
    uint64_t cap = (uint64_t)((double)cus * 2.0 * (double)biggest / (double)total + 0.999);
    if (cap < 1) cap = 1;
    unsigned gx = (unsigned)(want < cap ? want : cap);
    // Host-tier state in one extent whose every offset fits 32 bits: the PCIe variant
    // (c.host_span: the byte span of the extent the kernel may touch).
    static const int host_kernel = env_int("OCM_ADAM_HOST", 1);
    // 128 workgroups: 91 GiB/s of state (both directions of the link at once) against
    // 82 for the HBM-tuned full-chip grid; 64-160 are equal, 192 and up lose
    // (profiles/adam_host_probe_r03.json).
    static const int host_grid = env_int("OCM_ADAM_HOST_GRID", 128);
    static const int force_grid = env_int("OCM_ADAM_GRID", 0);
    uint64_t span = 0;
    for (uint32_t k = 0; k < a.count; k++) {
        const AdamTensor &t = a.t[k];
        const uint64_t bytes = (t.n & ~3ull) * 4;
        span = std::max(span, std::max(t.m_off, t.v_off) + bytes);
        if (a.c.bf16) span = std::max(span, t.w_off + bytes);
    }
    const bool host = a.c.host_state && host_kernel && a.c.n_ext == 1 && span < (1ull << 32);
    if (host && host_grid > 0) {
        // the host grid shared like the HBM one: in proportion to the biggest tensor's part
        const uint64_t hg = (uint64_t)((double)host_grid * (double)biggest / (double)total + 0.999);
        gx = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(hg, want));
    }
    if (force_grid > 0) gx = (unsigned)force_grid;
    if (host) {
        AdamMultiArgs h = a;
        h.c.host_span = (uint32_t)span;
        static const int host_vec = env_int("OCM_ADAM_HOST_VEC", 4);
        if (a.c.bf16)
            hipLaunchKernelGGL((adam_multi_kernel<true, true>), dim3(gx, a.count), dim3(kThreads), 0, stream, h);
        else if (host_vec == 2)
            hipLaunchKernelGGL((adam_multi_kernel<false, true, 2>), dim3(gx, a.count), dim3(kThreads), 0, stream, h);
        else if (host_vec == 8)
            hipLaunchKernelGGL((adam_multi_kernel<false, true, 8>), dim3(gx, a.count), dim3(kThreads), 0, stream, h);
        else
            hipLaunchKernelGGL((adam_multi_kernel<false, true>), dim3(gx, a.count), dim3(kThreads), 0, stream, h);
        return hipGetLastError();
    }
    if (a.c.bf16)
        hipLaunchKernelGGL((adam_multi_kernel<true, false>), dim3(gx, a.count), dim3(kThreads), 0, stream, a);
    else
        hipLaunchKernelGGL((adam_multi_kernel<false, false>), dim3(gx, a.count), dim3(kThreads), 0, stream, a);
    return hipGetLastError();
}

}  // namespace ocm

// gfx950 one-sided transfer kernels (put/get over xGMI, HBM and pinned host).
//
// See ocm/xfer.h for the contract. Two variants:
//   XFER_REG  register-staged: each lane keeps UNROLL 16-byte loads in flight,
//             then issues UNROLL 16-byte stores (nontemporal on the destination).
//   XFER_LDS  LDS-DMA staged: each wave streams its 8 KiB slice of a tile into a
//             wave-private LDS double buffer with global_load_lds_dwordx4 while
//             it drains the previous tile from LDS (ds_read_b128 + global store).
//             Wave-private buffers need no workgroup barrier; ordering is the
//             issuing wave's own counted vmcnt (guide: "Pipelining across barriers").
// Work decomposition: the striped address space is cut into tiles aligned to
// the tile size (a power of two <= stripe unit), so a tile never crosses a
// stripe unit and maps to one contiguous range on both sides. Workgroups
// grid-stride over tiles; per-tile extent/offset math runs once per workgroup.
// Reference parity: the one-sided data movers they replace are ib_read /
// ib_write (one signaled RDMA READ/WRITE work request, post_send src/rdma.c:47-92)
// and extoll_read / extoll_write (8 MiB chunks, 2 outstanding, extoll_rma2_transfer
// src/extoll.c:40-167).
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <cstring>

#include "ocm/xfer.h"

namespace ocm {

namespace {

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

constexpr int kThreads = 256;
constexpr int kUnroll = 8;                                    // 8 x 16 B in flight per lane
constexpr uint32_t kTileShift = 15;                           // 32 KiB tiles = 256 lanes x 16 B x 8
constexpr int kWaves = kThreads / 64;
constexpr int kWaveSlice = (1 << kTileShift) / kWaves;        // 8 KiB per wave per tile
constexpr int kChunksPerWave = kWaveSlice / 1024;             // 8 glds (1 KiB each) per wave per tile

template <bool NT>
__device__ __forceinline__ void store16(u32x4 *p, u32x4 v) {
    if constexpr (NT)
        __builtin_nontemporal_store(v, p);
    else
        *p = v;
}

__device__ __forceinline__ u32x4 load16(const u32x4 *p) { return __builtin_nontemporal_load(p); }

// Block-cooperative copy of n bytes (n <= one tile is the common case, any n works).
template <bool NT>
__device__ __forceinline__ void span_copy(char *__restrict__ dst, const char *__restrict__ src, uint64_t n) {
    const int tid = threadIdx.x;
    uint64_t head = (16u - ((uintptr_t)dst & 15u)) & 15u;
    if (head > n) head = n;
    if ((uint64_t)tid < head) dst[tid] = src[tid];
    dst += head;
    src += head;
    n -= head;
    if (((uintptr_t)src & 15u) == 0) {
        const uint64_t nv = n >> 4;
        const u32x4 *s = reinterpret_cast<const u32x4 *>(src);
        u32x4 *d = reinterpret_cast<u32x4 *>(dst);
        uint64_t base = 0;
        for (; base + (uint64_t)kThreads * kUnroll <= nv; base += (uint64_t)kThreads * kUnroll) {
            u32x4 v[kUnroll];
#pragma unroll
            for (int k = 0; k < kUnroll; k++) v[k] = load16(s + base + (uint64_t)k * kThreads + tid);
#pragma unroll
            for (int k = 0; k < kUnroll; k++) store16<NT>(d + base + (uint64_t)k * kThreads + tid, v[k]);
        }
        if (base < nv) {
            // Remainder (< kThreads x kUnroll vectors): every load issued before
            // the first store, so a partial tile costs one memory round trip,
            // not one per 4 KiB (a GET of host-tier memory pays PCIe latency each).
            u32x4 v[kUnroll];
#pragma unroll
            for (int k = 0; k < kUnroll; k++) {
                const uint64_t i = base + (uint64_t)k * kThreads + tid;
                if (i < nv) v[k] = load16(s + i);
            }
#pragma unroll
            for (int k = 0; k < kUnroll; k++) {
                const uint64_t i = base + (uint64_t)k * kThreads + tid;
                if (i < nv) store16<NT>(d + i, v[k]);
            }
        }
        const uint64_t tail = n & 15u;
        if ((uint64_t)tid < tail) dst[(nv << 4) + tid] = src[(nv << 4) + tid];
    } else {
        // Source and destination disagree mod 16: byte loop (rare; unaligned user offsets).
        for (uint64_t i = tid; i < n; i += kThreads) dst[i] = src[i];
    }
}

struct TileSpan {
    char *dst;
    const char *src;
    uint64_t n;
};

// Span of tile `ti` of a transfer of [rem_off, rem_off + len) in striped
// coordinates. `E` holds the extent bases (`E::ext[]`); it is read in place
// (kernarg segment or LDS): copying it to a local array would put the
// dynamically indexed array in scratch.
template <class E>
__device__ __forceinline__ TileSpan tile_span_of(const E &x, uint32_t n_ext, uint32_t unit_shift, uint32_t tile_shift,
                                                 char *lin, uint64_t rem_off, uint64_t len, uint32_t put, uint64_t ti,
                                                 uint64_t first_tile) {
    const uint64_t tile = 1ull << tile_shift;
    const uint64_t r0 = rem_off, r1 = rem_off + len;
    const uint64_t lo = first_tile + (ti << tile_shift);
    const uint64_t ts = lo > r0 ? lo : r0;
    const uint64_t te = (lo + tile) < r1 ? (lo + tile) : r1;
    char *rp;
    if (n_ext == 1) {
        rp = x.ext[0] + ts;
    } else {
        // Stripe unit u of the address space lives on extent u % n at (u / n) * unit.
        const uint64_t unit_mask = (1ull << unit_shift) - 1;
        const uint32_t u = (uint32_t)(ts >> unit_shift);
        const uint32_t e = u % n_ext;
        const uint64_t eoff = ((uint64_t)(u / n_ext) << unit_shift) | (ts & unit_mask);
        rp = x.ext[e] + eoff;
    }
    char *lp = lin + (ts - r0);
    TileSpan s;
    s.dst = put ? rp : lp;
    s.src = put ? lp : rp;
    s.n = te - ts;
    return s;
}

__device__ __forceinline__ TileSpan tile_span(const XferArgs &a, uint64_t ti, uint64_t first_tile) {
    return tile_span_of(a, a.n_ext, a.unit_shift, a.tile_shift, a.lin, a.rem_off, a.len, a.put, ti, first_tile);
}

// Drain every wave's stores into L2, join the workgroup, then ONE system-scope
// fence per workgroup writes them back and makes them visible to the host,
// DMA engines and other kernels (guide: scoped release after a barrier).
__device__ __forceinline__ void block_release_system() {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) __threadfence_system();
}

// Kernel-published completion (see XferDone): the last workgroup to count in
// re-arms the counter and releases the host flag.
__device__ __forceinline__ void xfer_publish(const XferDone &d) {
    if (!d.flag) return;  // kernel argument: uniform
    block_release_system();
    if (threadIdx.x == 0) {
        const unsigned old = __hip_atomic_fetch_add(d.cnt, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
        if (old == gridDim.x - 1) {
            __hip_atomic_store(d.cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(d.flag, d.val, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
}

template <bool NT>
__global__ __launch_bounds__(kThreads) void xfer_reg_kernel(XferArgs a, XferDone d) {
    const uint64_t tile_mask = (1ull << a.tile_shift) - 1;
    const uint64_t first = a.rem_off & ~tile_mask;
    const uint64_t ntiles = (((a.rem_off + a.len + tile_mask) & ~tile_mask) - first) >> a.tile_shift;
    for (uint64_t ti = blockIdx.x; ti < ntiles; ti += gridDim.x) {
        TileSpan s = tile_span(a, ti, first);
        span_copy<NT>(s.dst, s.src, s.n);
    }
    xfer_publish(d);
}

// ---- LDS-DMA variant ----
typedef __attribute__((address_space(3))) void lds_void;
typedef const __attribute__((address_space(1))) void glob_void;

__device__ __forceinline__ bool full_aligned(const TileSpan &s) {
    return s.n == (1ull << kTileShift) && (((uintptr_t)s.dst | (uintptr_t)s.src) & 15u) == 0;
}

// Issue this wave's 8 x 1 KiB LDS-DMA loads of a full tile into `buf`.
__device__ __forceinline__ void stage_tile(const char *src, char *buf, int wave, int lane) {
    const char *g = src + (size_t)wave * kWaveSlice + (size_t)lane * 16;
    char *l = buf + (size_t)wave * kWaveSlice;  // wave-uniform LDS base; lane offset is implicit
#pragma unroll
    for (int c = 0; c < kChunksPerWave; c++)
        __builtin_amdgcn_global_load_lds((glob_void *)(g + c * 1024), (lds_void *)(l + c * 1024), 16, 0, 0);
}

template <bool NT>
__device__ __forceinline__ void drain_tile(char *dst, const char *buf, int wave, int lane) {
    const char *l = buf + (size_t)wave * kWaveSlice + (size_t)lane * 16;
    char *g = dst + (size_t)wave * kWaveSlice + (size_t)lane * 16;
    u32x4 v[kChunksPerWave];
#pragma unroll
    for (int c = 0; c < kChunksPerWave; c++) v[c] = *reinterpret_cast<const u32x4 *>(l + c * 1024);
#pragma unroll
    for (int c = 0; c < kChunksPerWave; c++) store16<NT>(reinterpret_cast<u32x4 *>(g + c * 1024), v[c]);
}

// Body of the LDS-DMA kernel: this workgroup's tiles ti, ti + grid, ...
template <bool NT>
__device__ __forceinline__ void lds_stream(const XferArgs &a, char *lds, int wave, int lane, uint64_t ti,
                                           uint64_t first, uint64_t ntiles) {
    TileSpan cur = tile_span(a, ti, first);
    bool cur_staged = full_aligned(cur);
    if (cur_staged) stage_tile(cur.src, lds, wave, lane);
    int slot = 0;
    for (;;) {
        const uint64_t nt = ti + gridDim.x;
        TileSpan nxt;
        bool nxt_staged = false;
        if (nt < ntiles) {
            nxt = tile_span(a, nt, first);
            nxt_staged = full_aligned(nxt);
            if (nxt_staged) stage_tile(nxt.src, lds + (slot ^ 1) * (1 << kTileShift), wave, lane);
        }
        if (cur_staged) {
            // Retire this wave's loads of `cur`, leaving the next tile's 8 in flight.
            if (nxt_staged)
                asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
            else
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            drain_tile<NT>(cur.dst, lds + slot * (1 << kTileShift), wave, lane);
        } else {
            span_copy<NT>(cur.dst, cur.src, cur.n);
        }
        if (nt >= ntiles) break;
        ti = nt;
        cur = nxt;
        cur_staged = nxt_staged;
        slot ^= 1;
    }
}

template <bool NT>
__global__ __launch_bounds__(kThreads) void xfer_lds_kernel(XferArgs a, XferDone d) {
    // One LDS array (guide: a second __shared__ object can de-pipeline glds).
    __shared__ __attribute__((aligned(16))) char lds[2 * (1 << kTileShift)];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint64_t tile_mask = (1ull << a.tile_shift) - 1;
    const uint64_t first = a.rem_off & ~tile_mask;
    const uint64_t ntiles = (((a.rem_off + a.len + tile_mask) & ~tile_mask) - first) >> a.tile_shift;
    uint64_t ti = blockIdx.x;
    if (ti < ntiles) lds_stream<NT>(a, lds, wave, lane, ti, first, ntiles);  // grid <= ntiles: always true
    xfer_publish(d);
}

int env_int(const char *k, int dflt) {
    const char *v = std::getenv(k);
    return (v && *v) ? std::atoi(v) : dflt;
}

int g_num_cus = 0;

int num_cus() {
    if (g_num_cus) return g_num_cus;
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) == hipSuccess && hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && n > 0)
        g_num_cus = n;
    else
        g_num_cus = 256;
    return g_num_cus;
}

}  // namespace

XferTuning xfer_tuning_from_env() {
    XferTuning t;
    const char *v = std::getenv("OCM_XFER_VARIANT");
    if (v && (!std::strcmp(v, "lds") || !std::strcmp(v, "2"))) t.variant = XFER_LDS;
    if (v && (!std::strcmp(v, "reg") || !std::strcmp(v, "1"))) t.variant = XFER_REG;
    t.max_blocks = env_int("OCM_XFER_BLOCKS", 0);
    t.nontemporal = env_int("OCM_XFER_NT", 1) != 0;
    return t;
}

hipError_t xfer_normalize(XferArgs &a) {
    if (a.n_ext < 1 || a.n_ext > (uint32_t)kXferMaxExtents) return hipErrorInvalidValue;
    a.tile_shift = kTileShift;
    if (a.n_ext > 1) {
        if (a.unit_shift < 4) return hipErrorInvalidValue;
        if (a.unit_shift < kTileShift) a.tile_shift = a.unit_shift;  // tile must not cross a stripe unit
    }
    return hipSuccess;
}

hipError_t xfer_launch(const XferArgs &in, const XferTuning &t, hipStream_t stream, const XferDone *done) {
    if (in.len == 0) return hipSuccess;
    XferArgs a = in;
    if (xfer_normalize(a) != hipSuccess) return hipErrorInvalidValue;
    const uint64_t tile_mask = (1ull << a.tile_shift) - 1;
    const uint64_t ntiles = (((a.rem_off + a.len + tile_mask) & ~tile_mask) - (a.rem_off & ~tile_mask)) >> a.tile_shift;
    int variant = t.variant;
    if (variant == XFER_AUTO) variant = XFER_REG;
    if (a.tile_shift != kTileShift) variant = XFER_REG;  // LDS path is built for 32 KiB tiles
    // Grid caps from the round-1 sweep (profiles/ksweep_r01.json): LDS-DMA
    // peaks at 4 blocks per CU (2 resident, 64 KiB LDS each), the register
    // path at 2 per CU; never more blocks than tiles.
    int cap = t.max_blocks > 0 ? t.max_blocks : num_cus() * (variant == XFER_LDS ? 4 : 2);
    const unsigned grid = (unsigned)(ntiles < (uint64_t)cap ? ntiles : (uint64_t)cap);
    const XferDone d = done ? *done : XferDone{};
    if (variant == XFER_LDS) {
        if (t.nontemporal)
            hipLaunchKernelGGL(xfer_lds_kernel<true>, dim3(grid), dim3(kThreads), 0, stream, a, d);
        else
            hipLaunchKernelGGL(xfer_lds_kernel<false>, dim3(grid), dim3(kThreads), 0, stream, a, d);
    } else {
        if (t.nontemporal)
            hipLaunchKernelGGL(xfer_reg_kernel<true>, dim3(grid), dim3(kThreads), 0, stream, a, d);
        else
            hipLaunchKernelGGL(xfer_reg_kernel<false>, dim3(grid), dim3(kThreads), 0, stream, a, d);
    }
    return hipGetLastError();
}

hipError_t xfer_copy(void *dst, const void *src, uint64_t bytes, const XferTuning &t, hipStream_t stream) {
    XferArgs a;
    std::memset(&a, 0, sizeof(a));
    a.lin = const_cast<char *>(static_cast<const char *>(src));
    a.ext[0] = static_cast<char *>(dst);
    a.rem_off = 0;
    a.len = bytes;
    a.n_ext = 1;
    a.put = 1;
    return xfer_launch(a, t, stream);
}

// ---- batched one-sided ops ----

namespace {

constexpr uint32_t kBatchTileShift = 12;  // 4 KiB per wave-tile: 64 lanes x 16 B x 4 in flight
constexpr int kBatchUnroll = 4;

// One wave copies n bytes (n <= one wave-tile in the common case; any n works).
template <bool NT>
__device__ __forceinline__ void wave_copy(char *__restrict__ dst, const char *__restrict__ src, uint64_t n, int lane) {
    uint64_t head = (16u - ((uintptr_t)dst & 15u)) & 15u;
    if (head > n) head = n;
    if ((uint64_t)lane < head) dst[lane] = src[lane];
    dst += head;
    src += head;
    n -= head;
    if (((uintptr_t)src & 15u) == 0) {
        const uint64_t nv = n >> 4;
        const u32x4 *s = reinterpret_cast<const u32x4 *>(src);
        u32x4 *d = reinterpret_cast<u32x4 *>(dst);
        uint64_t i = lane;
        for (; i + (kBatchUnroll - 1) * 64 < nv; i += kBatchUnroll * 64) {
            u32x4 v[kBatchUnroll];
#pragma unroll
            for (int k = 0; k < kBatchUnroll; k++) v[k] = load16(s + i + k * 64);
#pragma unroll
            for (int k = 0; k < kBatchUnroll; k++) store16<NT>(d + i + k * 64, v[k]);
        }
        for (; i < nv; i += 64) store16<NT>(d + i, load16(s + i));
        const uint64_t tail = n & 15u;
        if ((uint64_t)lane < tail) dst[(nv << 4) + lane] = src[(nv << 4) + lane];
    } else {
        for (uint64_t i = lane; i < n; i += 64) dst[i] = src[i];
    }
}

template <bool NT>
__global__ __launch_bounds__(kThreads) void xfer_batch_kernel(XferBatchArgs a) {
    const int lane = threadIdx.x & 63;
    // wave index, made scalar: everything below is wave-uniform
    const uint32_t w = __builtin_amdgcn_readfirstlane(blockIdx.x * kWaves + (threadIdx.x >> 6));
    const uint64_t waves = (uint64_t)a.grid * kWaves;
    const uint64_t per = (a.total_tiles + waves - 1) / waves;
    uint64_t t = (uint64_t)w * per;
    const uint64_t t1 = t + per < a.total_tiles ? t + per : a.total_tiles;
    if (t >= t1) return;
    const bool inl = a.n_ops <= (uint32_t)kXferInlineOps;
    const XferBatchOp *ops = inl ? a.inline_ops : a.ops;
    uint32_t i = inl ? 0u : a.wave_op[w];
    const uint64_t tile_mask = (1ull << a.tile_shift) - 1;
    for (; t < t1; t++) {
        while (i + 1 < a.n_ops && ops[i + 1].first_tile <= t) i++;
        const XferBatchOp &op = ops[i];
        char *lin = a.abs_lin ? reinterpret_cast<char *>(static_cast<uintptr_t>(op.lin_off)) : a.lin + op.lin_off;
        TileSpan sp = tile_span_of(a, a.n_ext, a.unit_shift, a.tile_shift, lin, op.rem_off, op.len, op.put,
                                   t - op.first_tile, op.rem_off & ~tile_mask);
        wave_copy<NT>(sp.dst, sp.src, sp.n, lane);
    }
}

}  // namespace

uint32_t xfer_batch_tile_shift(uint32_t n_ext, uint32_t unit_shift) {
    return (n_ext > 1 && unit_shift < kBatchTileShift) ? unit_shift : kBatchTileShift;
}

uint64_t xfer_batch_plan(XferBatchOp *ops, uint32_t n, uint32_t tile_shift) {
    const uint64_t mask = (1ull << tile_shift) - 1;
    uint64_t total = 0;
    for (uint32_t i = 0; i < n; i++) {
        ops[i].first_tile = total;
        if (ops[i].len)
            total += (((ops[i].rem_off + ops[i].len + mask) & ~mask) - (ops[i].rem_off & ~mask)) >> tile_shift;
    }
    return total;
}

uint32_t xfer_batch_grid(uint64_t total_tiles) {
    // One wave per tile until the chip holds 8 workgroups (32 waves) per CU.
    const uint64_t want = (total_tiles + kWaves - 1) / kWaves;
    const uint64_t cap = (uint64_t)num_cus() * 8;
    return (uint32_t)(want < cap ? (want ? want : 1) : cap);
}

void xfer_batch_wave_ops(const XferBatchOp *ops, uint32_t n, uint64_t total_tiles, uint32_t grid, uint32_t *out) {
    const uint64_t waves = (uint64_t)grid * kWaves;
    const uint64_t per = (total_tiles + waves - 1) / waves;
    uint32_t i = 0;
    for (uint64_t w = 0; w < waves; w++) {
        const uint64_t t = w * per;
        while (i + 1 < n && ops[i + 1].first_tile <= t) i++;
        out[w] = i;
    }
}

hipError_t xfer_batch_launch(const XferBatchArgs &a, const XferTuning &t, hipStream_t stream) {
    if (a.total_tiles == 0 || a.n_ops == 0) return hipSuccess;
    if (a.n_ext < 1 || a.n_ext > (uint32_t)kXferMaxExtents || a.grid == 0) return hipErrorInvalidValue;
    if (a.n_ops > (uint32_t)kXferInlineOps && (!a.ops || !a.wave_op)) return hipErrorInvalidValue;
    if (t.nontemporal)
        hipLaunchKernelGGL(xfer_batch_kernel<true>, dim3(a.grid), dim3(kThreads), 0, stream, a);
    else
        hipLaunchKernelGGL(xfer_batch_kernel<false>, dim3(a.grid), dim3(kThreads), 0, stream, a);
    return hipGetLastError();
}

// ---- persistent copy service ----

namespace {

__host__ __device__ __forceinline__ unsigned long long service_mix(unsigned long long h, unsigned long long w) {
    h ^= w + 0x9E3779B97F4A7C15ull + (h << 6) + (h >> 2);
    h *= 0xBF58476D1CE4E5B9ull;
    return h ^ (h >> 31);
}

__device__ __forceinline__ unsigned long long readlane64(unsigned long long w, int lane) {
    const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)w, lane);
    const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(w >> 32), lane);
    return ((unsigned long long)hi << 32) | lo;
}

__device__ __forceinline__ uint64_t service_tiles(const XferArgs &a) {
    const uint64_t tile_mask = (1ull << a.tile_shift) - 1;
    return (((a.rem_off + a.len + tile_mask) & ~tile_mask) - (a.rem_off & ~tile_mask)) >> a.tile_shift;
}

// Tiles first, first + stride, ... of the request in `sh` (args at sh + 2).
__device__ __forceinline__ void service_copy(const unsigned long long *sh, uint64_t first, uint64_t stride) {
    const XferArgs &a = *reinterpret_cast<const XferArgs *>(sh + 2);  // read in place (no scratch copy)
    const uint64_t ntiles = service_tiles(a);
    const uint64_t base = a.rem_off & ~((1ull << a.tile_shift) - 1);
    for (uint64_t ti = first; ti < ntiles; ti += stride) {
        TileSpan sp = tile_span(a, ti, base);
        span_copy<false>(sp.dst, sp.src, sp.n);
    }
}

// Gang completion: each taking-part workgroup releases its bytes, then counts
// itself in; the last of `active` publishes `done`.
__device__ __forceinline__ void service_gang_done(ServiceSlot *slot, ServiceBox *box, unsigned long long s,
                                                  unsigned long long active) {
    block_release_system();
    if (threadIdx.x == 0) {
        const unsigned long long old =
            __hip_atomic_fetch_add(&box->cnt, 1ull, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
        if (old == active - 1) __hip_atomic_store(&slot->done, s, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

__global__ __launch_bounds__(kThreads) void service_kernel(const ServiceReq *rq, ServiceSlot *slot, ServiceBox *box,
                                                           unsigned long long first_seq,
                                                           unsigned long long idle_ticks, unsigned solo_tiles,
                                                           unsigned hbm_bell) {
    __shared__ __attribute__((aligned(16))) unsigned long long sh[16];
    const int tid = threadIdx.x;
    if (blockIdx.x != 0) {
        // Gang member: wait for workgroup 0 to publish a large request in the box.
        // Thread 0 takes a consistent snapshot {seq, active, args}: if seq moved
        // while it read, that request completed without this workgroup (it was
        // not taking part), so the newer one is taken instead.
        unsigned long long last = 0;
        for (;;) {
            if (tid == 0) {
                unsigned long long v = 0, act = 0;
                for (;;) {
                    v = __hip_atomic_load(&box->seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    if (v == last || v == 0) {
                        __builtin_amdgcn_s_sleep(4);
                        continue;
                    }
                    if (v == kServiceStop) break;
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // box contents, and no stale cached data
                    act = __hip_atomic_load(&box->active, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    if (blockIdx.x < act)
                        for (int i = 0; i < kServiceArgWords; i++)
                            sh[2 + i] = __hip_atomic_load(&box->args[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");  // the reads above before the re-check
                    if (__hip_atomic_load(&box->seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == v) break;
                }
                sh[0] = v;
                sh[1] = act;
            }
            __syncthreads();
            const unsigned long long v = sh[0], active = sh[1];
            if (v == kServiceStop) break;
            if (blockIdx.x < active) {  // block-uniform: workgroups past `active` sit this one out
                service_copy(sh, blockIdx.x, active);
                service_gang_done(slot, box, v, active);
            }
            last = v;
            __syncthreads();  // sh is rewritten by the next request
        }
        return;
    }
    unsigned long long expect = first_seq;
    unsigned long long idle_start = __builtin_amdgcn_s_memrealtime();
    unsigned long long ticks_sum = __hip_atomic_load(&slot->gpu_ticks, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    const unsigned long long *req = reinterpret_cast<const unsigned long long *>(rq);
    for (;;) {
        if (tid < 64) {
            // One wave reads the whole request record per poll (lanes 0..15).
            // A record in this GPU's HBM is polled through its seq word alone
            // (one lane, cheap local reads) and read whole once seq moved.
            unsigned long long w = 0, s;
            for (;;) {
                if (hbm_bell) {
                    unsigned long long q = 0;
                    if (tid == 0) q = __hip_atomic_load(req + 15, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                    q = readlane64(q, 0);
                    if (q != expect && q != kServiceStop) {
                        if (__builtin_amdgcn_s_memrealtime() - idle_start > idle_ticks) {
                            s = kServiceStop;
                            break;
                        }
                        __builtin_amdgcn_s_sleep(1);
                        continue;
                    }
                }
                if (tid < 16) w = __hip_atomic_load(req + tid, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                s = readlane64(w, 15);
                if (s == kServiceStop) break;
                if (s == expect) {
                    unsigned long long h = service_mix(0, s);
#pragma unroll
                    for (int i = 0; i < kServiceArgWords; i++) h = service_mix(h, readlane64(w, i));
                    if (h == readlane64(w, 14)) break;
                    continue;  // seq landed before the args: read the record again
                }
                if (__builtin_amdgcn_s_memrealtime() - idle_start > idle_ticks) {
                    s = kServiceStop;
                    break;
                }
                __builtin_amdgcn_s_sleep(8);  // ~0.2 us between PCIe polls
            }
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // order the data loads after the doorbell
            if (tid < kServiceArgWords) sh[2 + tid] = w;  // args -> sh[2..]
            if (tid == 0) sh[0] = s;
        }
        __syncthreads();
        const unsigned long long s = sh[0];
        if (s == kServiceStop) break;
        const unsigned long long t_seen = __builtin_amdgcn_s_memrealtime();
        const uint64_t ntiles = service_tiles(*reinterpret_cast<const XferArgs *>(sh + 2));
        if (gridDim.x > 1 && ntiles > solo_tiles) {
            const unsigned long long active = ntiles < gridDim.x ? ntiles : gridDim.x;
            if (tid < kServiceArgWords) box->args[tid] = sh[2 + tid];
            if (tid == 0) {
                __hip_atomic_store(&box->active, active, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __hip_atomic_store(&box->cnt, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            __syncthreads();
            if (tid == 0) __hip_atomic_store(&box->seq, s, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
            service_copy(sh, 0, active);
            service_gang_done(slot, box, s, active);  // gpu_ticks: until workgroup 0's share is out
        } else {
            service_copy(sh, 0, 1);
            // Make the bytes visible to the host, other kernels and DMA (system scope).
            block_release_system();
            if (tid == 0) __hip_atomic_store(&slot->done, s, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        idle_start = __builtin_amdgcn_s_memrealtime();  // every lane: the idle test must stay wave-uniform
        // Diagnostic, after `done` so it never delays it: a running sum in a
        // register, published with a plain store (no PCIe atomic round trip).
        ticks_sum += idle_start - t_seen;
        if (tid == 0) __hip_atomic_store(&slot->gpu_ticks, ticks_sum, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        expect++;
        __syncthreads();  // sh is rewritten by the next poll
    }
    if (tid == 0) {
        __hip_atomic_store(&box->seq, kServiceStop, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&slot->exited, expect, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

}  // namespace

void service_post(ServiceReq *req, const XferArgs &a, unsigned long long seq) {
    unsigned long long w[14] = {};
    std::memcpy(w, &a, sizeof(a));
    unsigned long long h = service_mix(0, seq);
    for (int i = 0; i < kServiceArgWords; i++) h = service_mix(h, w[i]);
    // Line 0 (args 0..7) first and fenced, then line 1 (args 8..13, sum, seq):
    // write-combining may flush a BAR-mapped record's lines in any order, and a
    // poll that saw seq ahead of its args would fail the hash and cost another
    // round trip. Host memory keeps x86 store order anyway.
    for (int i = 0; i < 8; i++) __atomic_store_n(&req->args[i], w[i], __ATOMIC_RELAXED);
    __builtin_ia32_sfence();
    for (int i = 8; i < 14; i++) __atomic_store_n(&req->args[i], w[i], __ATOMIC_RELAXED);
    __atomic_store_n(&req->sum, h, __ATOMIC_RELAXED);
    __atomic_store_n(&req->seq, seq, __ATOMIC_RELEASE);
    __builtin_ia32_sfence();  // drain write-combining buffers now
}

void service_store_seq(ServiceReq *req, unsigned long long seq) {
    __atomic_store_n(&req->seq, seq, __ATOMIC_RELEASE);
    __builtin_ia32_sfence();
}

hipError_t service_launch(ServiceReq *req, ServiceSlot *slot, ServiceBox *box, unsigned long long first_seq,
                          unsigned long long idle_ticks, unsigned blocks, unsigned solo_tiles, bool hbm_bell,
                          hipStream_t stream) {
    if (!req || !slot || !box || blocks == 0) return hipErrorInvalidValue;
    hipError_t e = hipMemsetAsync(box, 0, sizeof(ServiceBox), stream);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(service_kernel, dim3(blocks), dim3(kThreads), 0, stream, req, slot, box, first_seq, idle_ticks,
                       solo_tiles, hbm_bell ? 1u : 0u);
    return hipGetLastError();
}
// ---- verification patterns (benchmarks and tests check data without a host round trip) ----

__device__ __host__ __forceinline__ uint32_t pattern_word(uint64_t i, uint32_t seed) {
    uint64_t x = (i + 1) * 0x9E3779B97F4A7C15ull ^ ((uint64_t)seed << 32 | seed);
    x ^= x >> 31;
    x *= 0xBF58476D1CE4E5B9ull;
    x ^= x >> 29;
    return (uint32_t)x;
}

namespace {

__global__ __launch_bounds__(kThreads) void fill_kernel(uint32_t *p, uint64_t words, uint64_t first, uint32_t seed) {
    for (uint64_t i = (uint64_t)blockIdx.x * kThreads + threadIdx.x; i < words; i += (uint64_t)gridDim.x * kThreads)
        p[i] = pattern_word(first + i, seed);
}

__global__ __launch_bounds__(kThreads) void check_kernel(const uint32_t *p, uint64_t words, uint64_t first, uint32_t seed,
                                                         unsigned long long *bad) {
    unsigned long long local = 0;
    for (uint64_t i = (uint64_t)blockIdx.x * kThreads + threadIdx.x; i < words; i += (uint64_t)gridDim.x * kThreads)
        local += p[i] != pattern_word(first + i, seed);
    if (local) atomicAdd(bad, local);
}

}  // namespace

hipError_t pattern_fill(void *p, uint64_t words, uint64_t first_word, uint32_t seed, hipStream_t stream) {
    if (!words) return hipSuccess;
    const uint64_t want = (words + kThreads - 1) / kThreads;
    const unsigned grid = (unsigned)(want < 4096 ? want : 4096);
    hipLaunchKernelGGL(fill_kernel, dim3(grid), dim3(kThreads), 0, stream, static_cast<uint32_t *>(p), words, first_word, seed);
    return hipGetLastError();
}

hipError_t pattern_check(const void *p, uint64_t words, uint64_t first_word, uint32_t seed, unsigned long long *bad_dev,
                         hipStream_t stream) {
    if (!words) return hipSuccess;
    const uint64_t want = (words + kThreads - 1) / kThreads;
    const unsigned grid = (unsigned)(want < 4096 ? want : 4096);
    hipLaunchKernelGGL(check_kernel, dim3(grid), dim3(kThreads), 0, stream, static_cast<const uint32_t *>(p), words,
                       first_word, seed, bad_dev);
    return hipGetLastError();
}

uint32_t pattern_word_host(uint64_t i, uint32_t seed) { return pattern_word(i, seed); }

}  // namespace ocm

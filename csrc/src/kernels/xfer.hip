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

// Store flavours of the copy loops:
//   ST_PLAIN  plain stores (cached in the XCD's L2);
//   ST_NT     nontemporal stores (streaming; still released by a fence);
//   ST_WT     write-through (sc1) stores: the bytes leave L2 for memory as they
//             are stored, so a drain (s_waitcnt vmcnt(0)) of every storing wave
//             is all a hand-off needs - no buffer_wbl2 release fence
//             (guide: Guideline 16 R1; MI355X_MICROARCH.md visibility table);
//             the loads of such a span are sc1 as well.
enum StoreKind : int { ST_PLAIN = 0, ST_NT = 1, ST_WT = 2 };

__device__ __forceinline__ u32x4 load16(const u32x4 *p) { return __builtin_nontemporal_load(p); }

// Buffer descriptor over [base, base + bytes), built from wave-uniform values
// (every caller passes a workgroup-uniform span). Buffer accesses are range
// checked in hardware: a load past the end returns 0 without touching memory
// and a store past the end is dropped, so a partial tile needs no per-lane
// branches. (Branches around loads made the compiler put an s_waitcnt vmcnt(0)
// in front of each one inside the service loop: a partial host-tier tile then
// paid one PCIe round trip per 4 KiB.)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t span_rsrc(const void *base, uint32_t bytes) {
    const uint64_t b = reinterpret_cast<uint64_t>(base);
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)b);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(b >> 32));
    const uint32_t n = __builtin_amdgcn_readfirstlane(bytes);
    return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void *>(((uint64_t)hi << 32) | lo), 0, (int)n, 0x00020000);
}

// cache-policy bits of buffer accesses on gfx950: nt = 2, sc1 = 16
constexpr int kAuxNT = 2, kAuxSC1 = 16;

template <int ST>
constexpr int store_aux() {
    return ST == ST_WT ? kAuxSC1 : ST == ST_NT ? kAuxNT : 0;
}
// ST_WT spans are loaded sc1 too: such loads bypass the CU's L1 and read host /
// peer memory from memory rather than from stale L2 copies (measured:
// profiles/svc_copy_probe_r02.json), so the persistent service needs no acquire.
template <int ST>
constexpr int load_aux() {
    return ST == ST_WT ? kAuxSC1 : kAuxNT;
}

template <int ST>
__device__ __forceinline__ char load_byte(const char *p) {
    if constexpr (ST == ST_WT)
        return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // sc1, like the vectors
    else
        return *p;
}

template <int ST>
__device__ __forceinline__ void store_byte(char *p, char v) {
    if constexpr (ST == ST_WT)
        __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // sc1
    else
        *p = v;
}

// Plain / nt store of one vector through a pointer (LDS drain, batch waves).
template <int ST>
__device__ __forceinline__ void store16(u32x4 *p, u32x4 v) {
    if constexpr (ST == ST_NT)
        __builtin_nontemporal_store(v, p);
    else
        *p = v;
}

// Block-cooperative copy of n bytes (n <= one tile is the common case; spans
// of 2 GiB or more, which no caller makes, take a byte loop).
template <int ST>
__device__ __forceinline__ void span_copy(char *__restrict__ dst, const char *__restrict__ src, uint64_t n) {
    const int tid = threadIdx.x;
    uint64_t head = (16u - ((uintptr_t)dst & 15u)) & 15u;
    if (head > n) head = n;
    if ((uint64_t)tid < head) store_byte<ST>(dst + tid, load_byte<ST>(src + tid));
    dst += head;
    src += head;
    n -= head;
    if (((uintptr_t)src & 15u) == 0 && n < (1ull << 31)) {
        const uint32_t nv = (uint32_t)(n >> 4);
        const __amdgpu_buffer_rsrc_t rs = span_rsrc(src, nv << 4);
        const __amdgpu_buffer_rsrc_t rd = span_rsrc(dst, nv << 4);
        // every load of a round in flight before its first store; past-the-end
        // lanes of the last round are dropped by the range check
        for (uint32_t base = 0; base < nv; base += kThreads * kUnroll) {
            u32x4 v[kUnroll];
#pragma unroll
            for (int k = 0; k < kUnroll; k++)
                v[k] = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)((base + k * kThreads + tid) << 4), 0,
                                                             load_aux<ST>());
#pragma unroll
            for (int k = 0; k < kUnroll; k++)
                __builtin_amdgcn_raw_buffer_store_b128(v[k], rd, (int)((base + k * kThreads + tid) << 4), 0,
                                                       store_aux<ST>());
        }
        const uint64_t tail = n & 15u;
        if ((uint64_t)tid < tail) store_byte<ST>(dst + ((uint64_t)nv << 4) + tid, load_byte<ST>(src + ((uint64_t)nv << 4) + tid));
    } else {
        // Source and destination disagree mod 16: byte loop (rare; unaligned user offsets).
        for (uint64_t i = tid; i < n; i += kThreads) store_byte<ST>(dst + i, load_byte<ST>(src + i));
    }
}

struct TileSpan {
    char *dst;
    const char *src;
    uint64_t n;
};

// Two tile spans with all their loads in flight before the first store: a
// workgroup that copies two tiles from a far source (host tier over PCIe, peer
// HBM over xGMI) pays one read round trip instead of two. Each span is at most
// one tile, i.e. one round of kThreads x kUnroll vectors. Spans whose source and
// destination disagree mod 16 (unaligned user offsets) go one after the other.
template <int ST>
__device__ __forceinline__ void span_copy2(const TileSpan &a, const TileSpan &b) {
    const bool vec = (((uintptr_t)a.src ^ (uintptr_t)a.dst) & 15u) == 0 &&
                     (((uintptr_t)b.src ^ (uintptr_t)b.dst) & 15u) == 0 &&
                     a.n <= (uint64_t)kThreads * kUnroll * 16 && b.n <= (uint64_t)kThreads * kUnroll * 16;
    if (!vec) {
        span_copy<ST>(a.dst, a.src, a.n);
        span_copy<ST>(b.dst, b.src, b.n);
        return;
    }
    const int tid = threadIdx.x;
    // byte heads up to 16-byte alignment (same offset mod 16 on both sides)
    const uint64_t ha = ((16u - ((uintptr_t)a.dst & 15u)) & 15u) < a.n ? ((16u - ((uintptr_t)a.dst & 15u)) & 15u) : a.n;
    const uint64_t hb = ((16u - ((uintptr_t)b.dst & 15u)) & 15u) < b.n ? ((16u - ((uintptr_t)b.dst & 15u)) & 15u) : b.n;
    if ((uint64_t)tid < ha) store_byte<ST>(a.dst + tid, load_byte<ST>(a.src + tid));
    if ((uint64_t)tid < hb) store_byte<ST>(b.dst + tid, load_byte<ST>(b.src + tid));
    const uint32_t nva = (uint32_t)((a.n - ha) >> 4), nvb = (uint32_t)((b.n - hb) >> 4);
    const __amdgpu_buffer_rsrc_t rsa = span_rsrc(a.src + ha, nva << 4), rda = span_rsrc(a.dst + ha, nva << 4);
    const __amdgpu_buffer_rsrc_t rsb = span_rsrc(b.src + hb, nvb << 4), rdb = span_rsrc(b.dst + hb, nvb << 4);
    u32x4 va[kUnroll], vb[kUnroll];
#pragma unroll
    for (int k = 0; k < kUnroll; k++)
        va[k] = __builtin_amdgcn_raw_buffer_load_b128(rsa, (int)((k * kThreads + tid) << 4), 0, load_aux<ST>());
#pragma unroll
    for (int k = 0; k < kUnroll; k++)
        vb[k] = __builtin_amdgcn_raw_buffer_load_b128(rsb, (int)((k * kThreads + tid) << 4), 0, load_aux<ST>());
#pragma unroll
    for (int k = 0; k < kUnroll; k++)
        __builtin_amdgcn_raw_buffer_store_b128(va[k], rda, (int)((k * kThreads + tid) << 4), 0, store_aux<ST>());
#pragma unroll
    for (int k = 0; k < kUnroll; k++)
        __builtin_amdgcn_raw_buffer_store_b128(vb[k], rdb, (int)((k * kThreads + tid) << 4), 0, store_aux<ST>());
    const uint64_t ta = (a.n - ha) & 15u, tb = (b.n - hb) & 15u;
    const uint64_t oa = ha + ((uint64_t)nva << 4), ob = hb + ((uint64_t)nvb << 4);
    if ((uint64_t)tid < ta) store_byte<ST>(a.dst + oa + tid, load_byte<ST>(a.src + oa + tid));
    if ((uint64_t)tid < tb) store_byte<ST>(b.dst + ob + tid, load_byte<ST>(b.src + ob + tid));
}

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

template <int ST>
__global__ __launch_bounds__(kThreads) void xfer_reg_kernel(XferArgs a, XferDone d) {
    const uint64_t tile_mask = (1ull << a.tile_shift) - 1;
    const uint64_t first = a.rem_off & ~tile_mask;
    const uint64_t ntiles = (((a.rem_off + a.len + tile_mask) & ~tile_mask) - first) >> a.tile_shift;
    for (uint64_t ti = blockIdx.x; ti < ntiles; ti += gridDim.x) {
        TileSpan s = tile_span(a, ti, first);
        span_copy<ST>(s.dst, s.src, s.n);
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
    for (int c = 0; c < kChunksPerWave; c++)
        store16<NT ? ST_NT : ST_PLAIN>(reinterpret_cast<u32x4 *>(g + c * 1024), v[c]);
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
            span_copy<NT ? ST_NT : ST_PLAIN>(cur.dst, cur.src, cur.n);
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

// ---- PCIe streaming variant (host-tier extents) ----
// Large ops between this GPU's HBM and the pinned host tier are bound by PCIe,
// not by the CUs, and the 32 KiB-tile register kernel on a full-chip grid
// stays at 54-55 GB/s. Measured over shapes (tools/pcie_stream_probe.hip,
// profiles/pcie_stream_r03.json, 256 MiB, against hipMemcpyAsync at 56.8-57.1):
//   get (host -> HBM): 2 loads in flight per lane and 128 workgroups reach
//       57.4 GB/s; cache bits of either side change nothing; full-chip grids
//       lose up to 2 GB/s (too many streams scatter the read window);
//   put (HBM -> host): write-through (sc1) stores are the whole difference,
//       57.0 against 55.5 GB/s with plain or nontemporal stores, flat from 48
//       to 256 workgroups.
// So: 8 KiB tiles (256 lanes x 16 B x 2), grid-strided over a small grid, and
// sc1 stores when the destination is the host tier.
constexpr int kPcieUnroll = 2;
constexpr uint32_t kPcieTileShift = 13;  // 256 x 16 B x kPcieUnroll
constexpr unsigned kPcieBlocksDefault = 128;

template <int LA, int SA>
__device__ __forceinline__ void span_copy_pcie(char *__restrict__ dst, const char *__restrict__ src, uint64_t n) {
    const int tid = threadIdx.x;
    uint64_t head = (16u - ((uintptr_t)dst & 15u)) & 15u;
    if (head > n) head = n;
    if ((uint64_t)tid < head) dst[tid] = src[tid];
    dst += head;
    src += head;
    n -= head;
    if (((uintptr_t)src & 15u) == 0) {
        const uint32_t nv = (uint32_t)(n >> 4);  // a span is at most one tile
        const __amdgpu_buffer_rsrc_t rs = span_rsrc(src, nv << 4);
        const __amdgpu_buffer_rsrc_t rd = span_rsrc(dst, nv << 4);
        for (uint32_t base = 0; base < nv; base += kThreads * kPcieUnroll) {
            u32x4 v[kPcieUnroll];
#pragma unroll
            for (int k = 0; k < kPcieUnroll; k++)
                v[k] = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)((base + k * kThreads + tid) << 4), 0, LA);
#pragma unroll
            for (int k = 0; k < kPcieUnroll; k++)
                __builtin_amdgcn_raw_buffer_store_b128(v[k], rd, (int)((base + k * kThreads + tid) << 4), 0, SA);
        }
        const uint64_t tail = n & 15u;
        if ((uint64_t)tid < tail) dst[((uint64_t)nv << 4) + tid] = src[((uint64_t)nv << 4) + tid];
    } else {
        for (uint64_t i = tid; i < n; i += kThreads) dst[i] = src[i];
    }
}

// SA: store bits (kAuxSC1 when the destination is the host tier).
template <int SA>
__global__ __launch_bounds__(kThreads) void xfer_pcie_kernel(XferArgs a, XferDone d) {
    const uint64_t tile_mask = (1ull << a.tile_shift) - 1;
    const uint64_t first = a.rem_off & ~tile_mask;
    const uint64_t ntiles = (((a.rem_off + a.len + tile_mask) & ~tile_mask) - first) >> a.tile_shift;
    for (uint64_t ti = blockIdx.x; ti < ntiles; ti += gridDim.x) {
        TileSpan s = tile_span(a, ti, first);
        span_copy_pcie<kAuxNT, SA>(s.dst, s.src, s.n);
    }
    xfer_publish(d);
}

// ---- push-based get ----
// Launched on an owner's GPU: tiles of the extents in `mask` only (the other
// owners' launches take the rest); loads from this GPU's HBM, nontemporal
// stores into the app's buffer on another GPU over xGMI.
__global__ __launch_bounds__(kThreads) void xfer_push_kernel(XferArgs a, uint32_t mask) {
    const uint64_t tile_mask = (1ull << a.tile_shift) - 1;
    const uint64_t first = a.rem_off & ~tile_mask;
    const uint64_t ntiles = (((a.rem_off + a.len + tile_mask) & ~tile_mask) - first) >> a.tile_shift;
    const uint64_t r0 = a.rem_off;
    for (uint64_t ti = blockIdx.x; ti < ntiles; ti += gridDim.x) {
        if (a.n_ext > 1) {
            const uint64_t lo = first + (ti << a.tile_shift);
            const uint64_t ts = lo > r0 ? lo : r0;
            const uint32_t e = (uint32_t)(ts >> a.unit_shift) % a.n_ext;
            if (!((mask >> e) & 1u)) continue;  // workgroup-uniform
        }
        TileSpan s = tile_span(a, ti, first);
        span_copy<ST_NT>(s.dst, s.src, s.n);
    }
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
    if (v && (!std::strcmp(v, "pcie") || !std::strcmp(v, "4"))) t.variant = XFER_PCIE;
    if (v && (!std::strcmp(v, "push") || !std::strcmp(v, "5"))) t.variant = XFER_PUSH;
    t.max_blocks = env_int("OCM_XFER_BLOCKS", 0);
    t.nontemporal = env_int("OCM_XFER_NT", 1) != 0;
    t.write_through = env_int("OCM_XFER_NT", 1) == 2;  // 2: sc1 loads and stores (register kernel)
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
    const XferDone d0 = done ? *done : XferDone{};
    if (variant == XFER_PCIE) {
        if (a.tile_shift > kPcieTileShift) a.tile_shift = kPcieTileShift;
        const uint64_t mask = (1ull << a.tile_shift) - 1;
        const uint64_t tiles = (((a.rem_off + a.len + mask) & ~mask) - (a.rem_off & ~mask)) >> a.tile_shift;
        const uint64_t cap = t.max_blocks > 0 ? (uint64_t)t.max_blocks : (uint64_t)kPcieBlocksDefault;
        const unsigned g = (unsigned)(tiles < cap ? tiles : cap);
        // sc1 (write-through) stores into the host tier, plain ones into HBM
        if (a.put && t.nontemporal)
            hipLaunchKernelGGL(xfer_pcie_kernel<kAuxSC1>, dim3(g), dim3(kThreads), 0, stream, a, d0);
        else
            hipLaunchKernelGGL(xfer_pcie_kernel<0>, dim3(g), dim3(kThreads), 0, stream, a, d0);
        return hipGetLastError();
    }
    if (a.tile_shift != kTileShift) variant = XFER_REG;  // LDS path is built for 32 KiB tiles
    // Grid caps from the round-1 sweep (profiles/ksweep_r01.json): LDS-DMA
    // peaks at 4 blocks per CU (2 resident, 64 KiB LDS each), the register
    // path at 2 per CU; never more blocks than tiles.
    int cap = t.max_blocks > 0 ? t.max_blocks : num_cus() * (variant == XFER_LDS ? 4 : 2);
    const unsigned grid = (unsigned)(ntiles < (uint64_t)cap ? ntiles : (uint64_t)cap);
    const XferDone d = d0;
    if (variant == XFER_LDS) {
        if (t.nontemporal)
            hipLaunchKernelGGL(xfer_lds_kernel<true>, dim3(grid), dim3(kThreads), 0, stream, a, d);
        else
            hipLaunchKernelGGL(xfer_lds_kernel<false>, dim3(grid), dim3(kThreads), 0, stream, a, d);
    } else {
        if (t.write_through)
            hipLaunchKernelGGL(xfer_reg_kernel<ST_WT>, dim3(grid), dim3(kThreads), 0, stream, a, d);
        else if (t.nontemporal)
            hipLaunchKernelGGL(xfer_reg_kernel<ST_NT>, dim3(grid), dim3(kThreads), 0, stream, a, d);
        else
            hipLaunchKernelGGL(xfer_reg_kernel<ST_PLAIN>, dim3(grid), dim3(kThreads), 0, stream, a, d);
    }
    return hipGetLastError();
}

hipError_t xfer_push_launch(const XferArgs &in, uint32_t ext_mask, int max_blocks, hipStream_t stream) {
    if (in.len == 0 || ext_mask == 0) return hipSuccess;
    XferArgs a = in;
    if (a.put || xfer_normalize(a) != hipSuccess) return hipErrorInvalidValue;
    const uint64_t mask = (1ull << a.tile_shift) - 1;
    const uint64_t tiles = (((a.rem_off + a.len + mask) & ~mask) - (a.rem_off & ~mask)) >> a.tile_shift;
    const uint32_t mine = (uint32_t)__builtin_popcount(ext_mask & ((1u << a.n_ext) - 1));
    const uint64_t own = a.n_ext > 1 ? (tiles * mine + a.n_ext - 1) / a.n_ext : tiles;
    const uint64_t cap = max_blocks > 0 ? (uint64_t)max_blocks : (uint64_t)num_cus() * 2;
    const unsigned g = (unsigned)(own < cap ? (own ? own : 1) : cap);
    hipLaunchKernelGGL(xfer_push_kernel, dim3(g), dim3(kThreads), 0, stream, a, ext_mask);
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
// ST: the store kind (ST_NT / ST_PLAIN; ST_WT for puts into the host tier).
template <int ST>
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
            for (int k = 0; k < kBatchUnroll; k++) store16<ST>(d + i + k * 64, v[k]);
        }
        for (; i < nv; i += 64) store16<ST>(d + i, load16(s + i));
        const uint64_t tail = n & 15u;
        if ((uint64_t)lane < tail) dst[(nv << 4) + lane] = src[(nv << 4) + lane];
    } else {
        for (uint64_t i = lane; i < n; i += 64) dst[i] = src[i];
    }
}

// HOST: the host-tier shape: puts store write-through (sc1) into the pinned
// host extents, as the PCIe streaming kernel does (57.0 vs 55.5 GB/s).
template <bool NT, bool HOST = false>
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
        if (HOST && op.put)
            wave_copy<ST_WT>(sp.dst, sp.src, sp.n, lane);
        else
            wave_copy<NT ? ST_NT : ST_PLAIN>(sp.dst, sp.src, sp.n, lane);
    }
}

}  // namespace

// Host-tier batches store puts write-through (OCM_BATCH_HOST_SC1=0: the generic kernel).
static bool host_sc1() {
    static const bool on = env_int("OCM_BATCH_HOST_SC1", 1) != 0;
    return on;
}

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

uint32_t xfer_batch_grid(uint64_t total_tiles, bool host_tier) {
    // One wave per tile until the chip holds 8 workgroups (32 waves) per CU.
    const uint64_t want = (total_tiles + kWaves - 1) / kWaves;
    // Host tier: 128 workgroups and write-through puts; 4096-block KV swaps 48.0-48.1 /
    // 48.8-49.9 GiB/s out/in against 46.8-46.9 / 47.5-48.1 with the HBM shape
    // (profiles/kv_swap_host_r03.json; the PCIe ceiling is ~53).
    static const int host_grid = env_int("OCM_BATCH_HOST_GRID", 128);
    const uint64_t cap = host_tier && host_grid > 0 ? (uint64_t)host_grid : (uint64_t)num_cus() * 8;
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
    if (a.host_tier && host_sc1())
        hipLaunchKernelGGL((xfer_batch_kernel<true, true>), dim3(a.grid), dim3(kThreads), 0, stream, a);
    else if (t.nontemporal)
        hipLaunchKernelGGL(xfer_batch_kernel<true>, dim3(a.grid), dim3(kThreads), 0, stream, a);
    else
        hipLaunchKernelGGL(xfer_batch_kernel<false>, dim3(a.grid), dim3(kThreads), 0, stream, a);
    return hipGetLastError();
}

hipError_t xfer_batch_graph_node(hipGraph_t graph, hipGraphNode_t dep, const XferBatchArgs &a, const XferTuning &t,
                                 hipGraphNode_t *node) {
    const size_t ndep = dep ? 1 : 0;
    if (a.total_tiles == 0 || a.n_ops == 0) return hipGraphAddEmptyNode(node, graph, dep ? &dep : nullptr, ndep);
    if (a.n_ext < 1 || a.n_ext > (uint32_t)kXferMaxExtents || a.grid == 0) return hipErrorInvalidValue;
    if (a.n_ops > (uint32_t)kXferInlineOps && (!a.ops || !a.wave_op)) return hipErrorInvalidValue;
    // Parameters by address: `a` must outlive the graph (the plan's stage
    // storage), whether or not the runtime copies them into the node.
    void *params[] = {const_cast<XferBatchArgs *>(&a)};
    hipKernelNodeParams kp;
    std::memset(&kp, 0, sizeof(kp));
    kp.func = (a.host_tier && host_sc1()) ? reinterpret_cast<void *>(&xfer_batch_kernel<true, true>)
              : t.nontemporal             ? reinterpret_cast<void *>(&xfer_batch_kernel<true>)
                                          : reinterpret_cast<void *>(&xfer_batch_kernel<false>);
    kp.gridDim = dim3(a.grid);
    kp.blockDim = dim3(kThreads);
    kp.sharedMemBytes = 0;
    kp.kernelParams = params;
    kp.extra = nullptr;
    return hipGraphAddKernelNode(node, graph, dep ? &dep : nullptr, ndep, &kp);
}

// ---- persistent copy service ----

namespace {

__host__ __device__ __forceinline__ unsigned long long service_mix(unsigned long long h, unsigned long long w) {
    h ^= w + 0x9E3779B97F4A7C15ull + (h << 6) + (h >> 2);
    h *= 0xBF58476D1CE4E5B9ull;
    return h ^ (h >> 31);
}

// Hash of a request record's seq and words 0..kServiceReqGang (args, gang word).
__host__ __device__ __forceinline__ unsigned long long service_sum(unsigned long long seq, const unsigned long long *w) {
    unsigned long long h = service_mix(0, seq);
    for (int i = 0; i <= kServiceReqGang; i++) h = service_mix(h, w[i]);
    return h;
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
template <int ST>
__device__ __forceinline__ void service_copy(const unsigned long long *sh, uint64_t first, uint64_t stride) {
    const XferArgs &a = *reinterpret_cast<const XferArgs *>(sh + 2);  // read in place (no scratch copy)
    const uint64_t ntiles = service_tiles(a);
    const uint64_t base = a.rem_off & ~((1ull << a.tile_shift) - 1);
    // tiles two at a time: both tiles' loads in flight at once (span_copy2)
    uint64_t ti = first;
    for (; ti + stride < ntiles; ti += 2 * stride) span_copy2<ST>(tile_span(a, ti, base), tile_span(a, ti + stride, base));
    if (ti < ntiles) {
        TileSpan sp = tile_span(a, ti, base);
        span_copy<ST>(sp.dst, sp.src, sp.n);
    }
}

__device__ __forceinline__ void service_stamp(ServiceBox *box, unsigned proto, unsigned id, int k) {
    if ((proto & kServiceProtoTrace) && threadIdx.x == 0 && id < (unsigned)kServiceTraceWgs)
        __hip_atomic_store(&box->trace[id][k], __builtin_amdgcn_s_memrealtime(), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
}

// Copy member `id`'s share of the request in `sh` and make it visible
// system-wide; the member that completes the request publishes `done`.
__device__ __forceinline__ void service_serve(const unsigned long long *sh, unsigned long long s, ServiceSlot *slot,
                                              ServiceBox *box, unsigned proto, unsigned id) {
    const unsigned long long gang = sh[1];
    const unsigned long long active = gang & 0xFFFFull, target = (gang >> 16) & kServiceGangTargetMask;
    if (id >= active) return;  // block-uniform: members past `active` sit this one out
    // STRICT requests (extents in another GPU's HBM) take the fenced hand-off even
    // under the WT protocol: sc1 accesses keep this GPU's caches coherent with host
    // memory and its own HBM, but a resident instance may hold L2 lines of peer
    // memory from an earlier request, and nothing else invalidates them.
    const bool strict = (gang & kServiceGangStrict) != 0;
    const bool wt = (proto & kServiceProtoWT) && (!strict || (proto & kServiceProtoStrictWT));
    service_stamp(box, proto, id, 1);
    if (wt) {
        if (strict) {  // STRICTWT: drop stale L2 lines of peer memory before the sc1 (L2-served) loads
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        service_copy<ST_WT>(sh, id, active);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // EVERY storing wave drains its sc1 stores
        __syncthreads();
    } else {
        if (proto & kServiceProtoWT) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // the poll skipped it
        service_copy<ST_PLAIN>(sh, id, active);
        block_release_system();
    }
    service_stamp(box, proto, id, 2);
    if (threadIdx.x == 0 && service_wg_done(proto, active)) {
        // WGDONE: this member's own completion word; the host waits for all of them.
        if (wt)
            __hip_atomic_store(&slot->wg_done[id], s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        else
            __hip_atomic_store(&slot->wg_done[id], s, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    } else if (threadIdx.x == 0) {
        bool last = active == 1;
        if (!last) {
            const unsigned long long old =
                wt ? __hip_atomic_fetch_add(&box->cnt, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                   : __hip_atomic_fetch_add(&box->cnt, 1ull, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
            last = old == target - 1;
        }
        if (last) {
            if (wt)
                __hip_atomic_store(&slot->done, s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);  // after the drain
            else
                __hip_atomic_store(&slot->done, s, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
    service_stamp(box, proto, id, 3);
}

// Whether every member named by the last request workgroup 0 served (seq
// `last`, gang word `gang`) has finished it. Wave 0 of workgroup 0, all lanes.
__device__ __forceinline__ bool service_last_complete(ServiceSlot *slot, ServiceBox *box, unsigned proto,
                                                      unsigned long long last, unsigned long long gang) {
    const unsigned long long active = gang & 0xFFFFull, target = (gang >> 16) & kServiceGangTargetMask;
    if (active <= 1) return true;  // workgroup 0 served it alone
    const unsigned lane = threadIdx.x & 63u;
    bool ok = true;
    if (service_wg_done(proto, active)) {
        for (unsigned long long i = lane; i < active; i += 64)
            ok &= __hip_atomic_load(&slot->wg_done[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) == last;
    } else {
        ok = __hip_atomic_load(&box->cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= target;
    }
    return __builtin_amdgcn_ballot_w64(!ok) == 0;
}

// Workgroup 0 polls the host request record across PCIe; for a gang request it
// relays the record, as read (the host's hash included), to the gang through
// device memory with one 16-lane write-through store, before anything else.
// The gang polls that device copy: 32 workgroups polling the host record
// directly cost every op 3-4 us (profiles/svc_v3_direct_r02.json), and a relay
// that re-hashed and fenced first cost the gang ~2 us (profiles/svc_trace_r02.json).
// GANGREC (grq != nullptr): gang requests sit in their own host record, which
// members 0..direct_wgs-1 poll themselves; workgroup 0 reads both records in
// one load (lanes 0..15 the small-op record, 16..31 the gang record) and
// relays only gangs wider than direct_wgs to the others. 16 direct pollers
// cost small ops nothing measurable; 32 cost them ~1 us
// (profiles/svc_direct_gang_ab_r02.json).
// Members are numbered in check-in order; member 0 (the first workgroup to
// start) is "workgroup 0" of the protocol above and publishes how many have
// checked in (the roster, see ocm/xfer.h): lane 32 of its poll reads the
// check-in counter until the whole grid is in.
}  // namespace

// The copy service. extern "C": libocm also dispatches it by name from the device
// code object embedded in the library, on an AQL queue of its own (ocm/aql.h).
extern "C" __global__ __launch_bounds__(kThreads) void ocm_service_kernel(ServiceKernelArgs ka) {
    const ServiceReq *rq = ka.req, *grq = ka.gang_req;
    ServiceSlot *slot = ka.slot;
    ServiceBox *box = ka.box;
    const unsigned long long first_seq = ka.first_seq, idle_ticks = ka.idle_ticks, checkin_base = ka.checkin_base;
    const unsigned long long degraded_idle_ticks = ka.degraded_idle_ticks, lone_ticks = ka.lone_ticks;
    const unsigned proto = ka.proto, direct_wgs = ka.direct_wgs, epoch = ka.epoch, grid = ka.blocks;
    __shared__ __attribute__((aligned(16))) unsigned long long sh[16];
    __shared__ unsigned sh_id;
    const int tid = threadIdx.x;
    // Member ids in check-in order. The first workgroup to start is workgroup 0 of
    // the protocol (the lead), whichever block it is: the dispatcher spreads blocks
    // over the XCDs, and block 0's XCD may have no room while others do (measured
    // under tests/test_gpu_service.py's CU hog: block 0 waited for the hog to end).
    // The counter only grows across instances (the box is not cleared between
    // launches): tickets of this instance start at checkin_base.
    if (tid == 0)
        sh_id = (unsigned)(__hip_atomic_fetch_add(&box->checkin, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) -
                           checkin_base);
    __syncthreads();
    const unsigned id = __builtin_amdgcn_readfirstlane(sh_id);  // this workgroup's member id
    const bool lead = id == 0;
    const bool direct = grq != nullptr && id < direct_wgs;  // polls the host gang record itself
    const unsigned long long relay_above = grq != nullptr ? direct_wgs : 1;  // gangs wider than this are relayed
    // COPIES: direct member i polls copy i of the gang record (the lead, member 0, copy 0)
    const ServiceReq *gmine = grq + ((proto & kServiceProtoCopies) && direct ? id : 0u);
    const unsigned long long *req = reinterpret_cast<const unsigned long long *>(
        lead ? static_cast<const void *>(rq) : direct ? static_cast<const void *>(gmine) : static_cast<const void *>(box->rec));
    const unsigned long long *greq = reinterpret_cast<const unsigned long long *>(grq);
    unsigned long long last = first_seq - 1;  // requests carry strictly increasing seqs
    unsigned long long last_gang = 0;          // gang word of request `last` (workgroup 0's idle-exit test)
    unsigned long long roster = 0;             // members published so far (workgroup 0)
    unsigned long long idle_start = __builtin_amdgcn_s_memrealtime();
    // The host launches an instance only for a request it is about to post, and it
    // may first wait for the roster: no idle exit before the first request (with a
    // 1 us idle window the lead left before every post, and host and kernel
    // relaunched each other until the op timed out), unless none comes in 20 ms.
    const unsigned long long started = idle_start;
    bool served = false;
    bool lone = false;        // the lead alone: the members have left (lone_ticks)
    bool superseded = false;  // the lead saw a newer instance: it leaves without touching the slot
    // The last gang request was already seen complete by an earlier idle check. The idle
    // window runs from the lead's own share, and a PCIe-bound gang op of 8-16 MiB ends up
    // to ~50 us later on its slowest member: leaving at the first check that finds it
    // complete raced the host's next post (12-15 % of those ops relaunched,
    // profiles/bench_n1_r04_final_b.json). A gang op gets one more window from then.
    bool gang_drained = false;
    // This instance's own sum (the host folds each instance's into its total when it
    // starts the next): no read across PCIe before the first poll.
    unsigned long long ticks_sum = 0;
    if (lead && tid == 0) {
        // where the lead runs (diagnostic; a posted write, nothing waits for it): 1 + its XCD
        // (HW_REG_XCC_ID[3:0]) in bits 0..7, its HW_REG_HW_ID (CU, shader array, engine) above
        const unsigned long long xcc = __builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 20) & 0xFu;
        const unsigned long long hwid = (unsigned)__builtin_amdgcn_s_getreg((31 << 11) | (0 << 6) | 4);
        __hip_atomic_store(&slot->lead_xcd, service_tag(epoch, (1ull + xcc) | (hwid << 8)), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
    }
    for (;;) {
        int base = 0;  // first lane of the record being served (wave-uniform)
        if (tid < 64) {
            // One load instruction per poll: lanes 0..15 read the whole record
            // (args, gang word, sum, seq); a seq whose hash checks out is whole.
            unsigned long long w = 0, s;
            for (;;) {
                const bool count = lead && !lone && roster < grid;  // wave-uniform
                if (tid < 16)
                    w = (lead || direct) ? __hip_atomic_load(req + tid, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)
                                         : __hip_atomic_load(req + tid, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                else if (direct && lead && !lone && tid < 32)
                    w = __hip_atomic_load(greq + (tid - 16), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                else if (!lead && tid == 16)
                    w = __hip_atomic_load(&box->stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // the lead left
                else if (count && tid == 32)
                    w = __hip_atomic_load(&box->checkin, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                else if (lone && tid == 48)
                    w = __hip_atomic_load(&slot->epoch_now, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                if (count) {
                    const unsigned long long r = readlane64(w, 32) - checkin_base;  // check-ins, the lead's included
                    if (r > roster) {  // members counted here are running: requests may name them
                        if (tid == 0)
                            __hip_atomic_store(&slot->roster, service_tag(epoch, r), __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_SYSTEM);
                        roster = r;
                    }
                }
                base = 0;
                s = readlane64(w, 15);
                if (!lead && readlane64(w, 16) == first_seq) {  // the lead of THIS instance left
                    s = kServiceStop;
                    break;
                }
                if (lone && (readlane64(w, 48) & kServiceGangEpochMask) != epoch) {  // replaced by a full instance
                    s = kServiceStop;
                    superseded = true;
                    break;
                }
                if (direct && lead && !lone) {
                    const unsigned long long s2 = readlane64(w, 31);  // the gang record's seq
                    if (s2 == kServiceStop) {  // the host parked it
                        s = kServiceStop;
                        break;
                    }
                    if (s2 > last && s2 != 0) {
                        s = s2;  // the host posts one request at a time: at most one record is new
                        base = 16;
                    }
                }
                if (s == kServiceStop) break;
                if (s > last) {
                    unsigned long long h = service_mix(0, s);
#pragma unroll
                    for (int i = 0; i <= kServiceReqGang; i++) h = service_mix(h, readlane64(w, base + i));
                    if (h != readlane64(w, base + 14)) continue;  // seq landed before the rest: read it again
                    // Whole. A member of an earlier instance (started late) leaves a newer one's
                    // request alone; a lead that sees one has been replaced and leaves. A lone
                    // lead takes no gang request (its members are gone: the host starts a
                    // full instance for it).
                    const unsigned long long g = readlane64(w, base + kServiceReqGang);
                    const bool mine = ((g >> kServiceGangEpochShift) & kServiceGangEpochMask) == epoch;
                    if (lead && !mine) {
                        s = kServiceStop;
                        superseded = true;
                        break;
                    }
                    if (mine && !(lone && (g & 0xFFFFull) > 1)) break;
                }
                // While part of the grid has not started (the roster is short) it waits
                // longer (degraded_idle_ticks): the kernel cannot complete before those
                // workgroups get CUs and leave anyway, so leaving early would release a
                // device-wide sync no sooner, and every relaunch would need another
                // stream while they wait (the pool is small).
                if (lead &&
                    __builtin_amdgcn_s_memrealtime() - idle_start >
                        (lone ? lone_ticks : roster >= grid ? idle_ticks : degraded_idle_ticks) &&
                    (served || __builtin_amdgcn_s_memrealtime() - started > 2000000ull)) {
                    // Leave only once every member the last request named is done
                    // with it: a member that saw the STOP first would never serve it.
                    const bool complete = service_last_complete(slot, box, proto, last, last_gang);
                    if (complete && (gang_drained || (last_gang & 0xFFFFull) <= 1 || !served)) {
                        // Only an instance whose whole grid has started goes lone: one with
                        // workgroups still waiting for a CU leaves whole, as its lane drains
                        // only once they have started (and left at once), and the full
                        // instance that would replace a lone lead needs a drained lane.
                        if (lone || lone_ticks == 0 || roster < grid) {
                            s = kServiceStop;
                            break;
                        }
                        // The members leave; the lead stays alone and says so (the host
                        // then sizes no gang on this instance).
                        lone = true;
                        if (tid == 0) {
                            __hip_atomic_store(&box->stop, first_seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                            __hip_atomic_store(&slot->lone, service_tag(epoch, last + 1), __ATOMIC_RELEASE,
                                               __HIP_MEMORY_SCOPE_SYSTEM);
                        }
                    } else if (complete) {
                        gang_drained = true;  // complete only now: the host gets a whole window to post
                    }
                    idle_start = __builtin_amdgcn_s_memrealtime();
                }
                if (lone)
                    __builtin_amdgcn_s_sleep(24);  // ~0.6 us: one PCIe read of the record per poll
                else if (lead || direct)
                    __builtin_amdgcn_s_sleep(8);  // ~0.2 us between PCIe polls
                else
                    __builtin_amdgcn_s_sleep(1);
            }
            if (lead && s != kServiceStop && (readlane64(w, base + kServiceReqGang) & 0xFFFFull) > relay_above &&
                tid >= base && tid < base + 16)
                __hip_atomic_store(&box->rec[tid - base], w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // relay, sc1
            // Data loads are sc1 (ST_WT protocol): they bypass this CU's L1 and are
            // not served from stale L2 copies of host or peer memory, so no acquire
            // fence is needed; the plain protocol keeps the system-scope acquire.
            if (!(proto & kServiceProtoWT)) {
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
            const int r = tid - base;  // this lane's word of the served record
            if (r >= 0 && r <= kServiceReqGang) sh[r == kServiceReqGang ? 1 : 2 + r] = w;  // args -> sh[2..], gang -> sh[1]
            if (tid == 0) sh[0] = s;
        }
        __syncthreads();
        const unsigned long long s = sh[0];
        if (s == kServiceStop) break;
        const unsigned long long t_seen = __builtin_amdgcn_s_memrealtime();
        service_stamp(box, proto, id, 0);
        service_serve(sh, s, slot, box, proto, id);
        last = s;
        last_gang = sh[1];
        served = true;
        gang_drained = false;
        idle_start = __builtin_amdgcn_s_memrealtime();  // every lane: the idle test must stay wave-uniform
        if (lead) {
            // Diagnostic, after `done` so it never delays it: a running sum in a
            // register, published with a plain store (no PCIe atomic round trip).
            ticks_sum += idle_start - t_seen;
            if (tid == 0) __hip_atomic_store(&slot->gpu_ticks, ticks_sum, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        __syncthreads();  // sh is rewritten by the next poll
    }
    if (lead && tid == 0) {
        // Every member leaves when it sees this instance's first seq here (an
        // earlier instance's value never matches, so the box needs no clearing).
        __hip_atomic_store(&box->stop, first_seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (!superseded)
            __hip_atomic_store(&slot->exited, service_tag(epoch, last + 1), __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// Zero a lane's gang box on the lane's own AQL queue (one workgroup), ahead of an
// instance dispatched with the barrier bit: no host memset and stream sync.
extern "C" __global__ __launch_bounds__(kThreads) void ocm_service_box_clear(ServiceBox *box) {
    unsigned long long *w = reinterpret_cast<unsigned long long *>(box);
    for (unsigned i = threadIdx.x; i < sizeof(ServiceBox) / 8; i += kThreads) w[i] = 0ull;
}

uint32_t service_gang_size(const XferArgs &a, unsigned blocks, unsigned solo_tiles) {
    const uint64_t tile_mask = (1ull << a.tile_shift) - 1;
    const uint64_t ntiles = (((a.rem_off + a.len + tile_mask) & ~tile_mask) - (a.rem_off & ~tile_mask)) >> a.tile_shift;
    if (blocks <= 1 || ntiles <= solo_tiles) return 1;
    return (uint32_t)(ntiles < blocks ? ntiles : blocks);
}

void service_post(ServiceReq *req, const XferArgs &a, unsigned long long gang, unsigned long long seq,
                  unsigned copies) {
    unsigned long long w[kServiceReqGang + 1] = {};
    std::memcpy(w, &a, sizeof(a));
    w[kServiceReqGang] = gang;
    const unsigned long long h = service_sum(seq, w);
    // Line 0 (words 0..7) of every copy first and fenced, then line 1 (words 8..13,
    // sum, seq): a poll that saw seq ahead of the rest fails the hash and reads again.
    // The last copy first: copy 0 is the lead's.
    for (unsigned c = copies; c-- > 0;)
        for (int i = 0; i < 8; i++) __atomic_store_n(&req[c].args[i], w[i], __ATOMIC_RELAXED);
    __builtin_ia32_sfence();
    for (unsigned c = copies; c-- > 0;) {
        for (int i = 8; i <= kServiceReqGang; i++) __atomic_store_n(&req[c].args[i], w[i], __ATOMIC_RELAXED);
        __atomic_store_n(&req[c].sum, h, __ATOMIC_RELAXED);
        __atomic_store_n(&req[c].seq, seq, __ATOMIC_RELEASE);
    }
    __builtin_ia32_sfence();
}

void service_store_seq(ServiceReq *req, unsigned long long seq, unsigned copies) {
    for (unsigned c = 0; c < copies; c++) __atomic_store_n(&req[c].seq, seq, __ATOMIC_RELEASE);
    __builtin_ia32_sfence();
}

hipError_t service_launch(const ServiceKernelArgs &args, unsigned blocks, bool reset_box, hipStream_t stream) {
    if (!args.req || !args.slot || !args.box || blocks == 0 || blocks != args.blocks || args.first_seq == 0 ||
        (args.gang_req && args.direct_wgs == 0) || args.epoch > kServiceGangEpochMask)
        return hipErrorInvalidValue;
    if (reset_box) {
        hipError_t e = hipMemsetAsync(args.box, 0, sizeof(ServiceBox), stream);
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(ocm_service_kernel, dim3(blocks), dim3(kThreads), 0, stream, args);
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

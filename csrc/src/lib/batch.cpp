// libocm batched one-sided ops (ocm_copy_onesided_batch), stream interop
// (ocm_stream_wait/signal) and transfer plans (ocm_plan_*: fixed batch
// schedules captured into a HIP graph and replayed).
#include "internal.h"

using namespace ocm;
using namespace ocmlib;

// Launch geometry of a batch on `a` for the descriptors in `v` (first_tile filled in).
static void plan_batch_args(lib_alloc *a, std::vector<XferBatchOp> &v, bool abs_lin, XferBatchArgs *args) {
    std::memset(args, 0, sizeof(*args));
    args->lin = abs_lin ? nullptr : static_cast<char *>(a->local);
    args->abs_lin = abs_lin ? 1 : 0;
    for (size_t i = 0; i < a->ext.size(); i++) args->ext[i] = a->ext[i].dptr;
    args->n_ext = (uint32_t)a->ext.size();
    args->unit_shift = args->n_ext > 1 ? (uint32_t)log2_exact(a->stripe_unit) : 0;
    args->tile_shift = xfer_batch_tile_shift(args->n_ext, args->unit_shift);
    args->n_ops = (uint32_t)v.size();
    args->total_tiles = xfer_batch_plan(v.data(), (uint32_t)v.size(), args->tile_shift);
    args->host_tier = (!a->any_gpu && !a->any_net) ? 1u : 0u;
    args->grid = args->total_tiles ? xfer_batch_grid(args->total_tiles, args->host_tier != 0) : 0;
    if (v.size() <= (size_t)kXferInlineOps) std::memcpy(args->inline_ops, v.data(), v.size() * sizeof(XferBatchOp));
}

// Batch launch arguments for `ops` on `a` (descriptors in `v`; inline ones copied into args).
static void build_batch_args(lib_alloc *a, const struct ocm_params *ops, int n_ops, XferBatchArgs *args,
                             std::vector<XferBatchOp> *v) {
    v->assign((size_t)n_ops, XferBatchOp{});
    for (int i = 0; i < n_ops; i++) {
        (*v)[i].lin_off = ops[i].src_offset;
        (*v)[i].rem_off = ops[i].dest_offset;
        (*v)[i].len = ops[i].bytes;
        (*v)[i].put = ops[i].op_flag != 0;
    }
    plan_batch_args(a, *v, false, args);
}

// Bounds of every op against the pair (as ocm_copy_onesided). Adds the bytes to *moved.
static int check_batch_ops(lib_alloc *a, const struct ocm_params *ops, int n_ops, uint64_t *moved) {
    for (int i = 0; i < n_ops; i++) {
        const ocm_params &p = ops[i];
        if (p.src_offset > a->local_bytes || p.bytes > a->local_bytes - p.src_offset)
            OCM_FAIL(-1, "batch op %d: local range [%llu,+%llu) exceeds %zu bytes", i,
                     (unsigned long long)p.src_offset, (unsigned long long)p.bytes, a->local_bytes);
        if (p.dest_offset > a->remote_bytes || p.bytes > a->remote_bytes - p.dest_offset)
            OCM_FAIL(-1, "batch op %d: remote range [%llu,+%llu) exceeds %zu bytes", i,
                     (unsigned long long)p.dest_offset, (unsigned long long)p.bytes, a->remote_bytes);
        *moved += p.bytes;
    }
    return 0;
}

// One kernel can serve this pair: device local half, every extent device-accessible.
static bool batch_device_path(const lib_alloc *a) {
    const State &s = S();
    return s.device >= 0 && a->loc == LOC_DEVICE && a->all_dev_ok && !a->any_net &&
           (a->ext.size() == 1 || log2_exact(a->stripe_unit) >= 4);
}

namespace ocmlib {

// Upload (large lists), launch and complete one batch on `a`. `args` from plan_batch_args.
int run_batch(lib_alloc *a, XferBatchArgs &args, std::vector<XferBatchOp> &v, bool async) {
    State &s = S();
    DeviceGuard guard(s.device);
    if (!async && wait_alloc(a) != 0) return -1;
    hipStream_t st = async ? lane_stream(a) : s.stream;
    if (honor_dep(a, st, false) != 0) return -1;
    hipError_t err = hipSuccess;
    const size_t n_ops = v.size();
    if (n_ops > (size_t)kXferInlineOps) {
        // descriptors, then the per-wave starting ops, in one upload
        const size_t dbytes = v.size() * sizeof(XferBatchOp);
        const size_t need = dbytes + (size_t)args.grid * 4 * sizeof(uint32_t);
        if (a->batch_up && hipEventSynchronize(a->batch_up) != hipSuccess)  // staging free again
            OCM_FAIL(-1, "batch staging wait failed");
        if (a->batch_cap < need) {
            if (a->batch_dev) (void)hipFreeAsync(a->batch_dev, st);
            if (a->batch_host) (void)hipHostFree(a->batch_host);
            a->batch_dev = a->batch_host = nullptr;
            a->batch_cap = 0;
            const size_t cap = std::max<size_t>(need, 64 << 10);
            err = local_pool() ? hipMallocFromPoolAsync(&a->batch_dev, cap, s.pool, st) : hipMallocAsync(&a->batch_dev, cap, st);
            if (err == hipSuccess) err = hipHostMalloc(&a->batch_host, cap, hipHostMallocDefault);
            if (err == hipSuccess && !a->batch_up) err = hipEventCreateWithFlags(&a->batch_up, hipEventDisableTiming);
            if (err != hipSuccess) {
                (void)hipGetLastError();
                OCM_FAIL(-1, "batch descriptors: %s", hipGetErrorString(err));
            }
            a->batch_cap = cap;
        }
        char *up = static_cast<char *>(a->batch_host);
        std::memcpy(up, v.data(), dbytes);
        xfer_batch_wave_ops(v.data(), (uint32_t)n_ops, args.total_tiles, args.grid, reinterpret_cast<uint32_t *>(up + dbytes));
        // Pinned source: a real async DMA; batch_up tells the next batch when `up` is free.
        err = hipMemcpyAsync(a->batch_dev, up, need, hipMemcpyHostToDevice, st);
        if (err == hipSuccess) err = hipEventRecord(a->batch_up, st);
        if (err != hipSuccess) OCM_FAIL(-1, "batch descriptor upload: %s", hipGetErrorString(err));
        args.ops = static_cast<const XferBatchOp *>(a->batch_dev);
        args.wave_op = reinterpret_cast<const uint32_t *>(static_cast<char *>(a->batch_dev) + dbytes);
    }
    before_launch();
    err = xfer_batch_launch(args, s.tuning, st);
    if (err != hipSuccess) OCM_FAIL(-1, "batch launch failed: %s", hipGetErrorString(err));
    s.ctr.n_batch_launches++;
    if (async) {
        if (st != s.stream && a->ev) {
            err = hipEventRecord(a->ev, st);
            if (err != hipSuccess) OCM_FAIL(-1, "event record failed: %s", hipGetErrorString(err));
            a->async_pending = true;
            return 0;
        }
    }
    return sync_stream();
}

// Remote -> remote copies: every op's linear side is an absolute device address
// (a source extent), written into `dst`'s remote half by one launch.
int batch_put_abs(lib_alloc *dst, std::vector<XferBatchOp> &v) {
    if (v.empty()) return 0;
    XferBatchArgs args;
    plan_batch_args(dst, v, true, &args);
    if (args.total_tiles == 0) return 0;
    return run_batch(dst, args, v, false);
}

}  // namespace ocmlib

extern "C" {

static int batch_impl(ocm_alloc_t a, const struct ocm_params *ops, int n_ops, int flags, uint64_t *moved);

// Batch launch arguments for `ops` on `a` (descriptors in `v`; inline ones copied into args).
int ocm_copy_onesided_batch(ocm_alloc_t a, const struct ocm_params *ops, int n_ops, int flags) {
    TraceRange tr("ocm_batch");
    const uint64_t t0 = now_ns();
    uint64_t moved = 0;
    int rc = batch_impl(a, ops, n_ops, flags, &moved);
    const uint64_t t1 = now_ns();
    if (rc == 0) {
        OpCounters &c = S().ctr;
        c.n_batch++;
        c.n_batch_ops += (uint64_t)n_ops;
        c.bytes_batch += moved;
        c.ns_batch += t1 - t0;
    }
    trace_op("batch", moved, t0, t1, rc);
    return rc;
}

static int batch_impl(ocm_alloc_t a, const struct ocm_params *ops, int n_ops, int flags, uint64_t *moved) {
    State &s = S();
    std::lock_guard<std::recursive_mutex> lk(s.mu);
    if (!a || (!ops && n_ops)) OCM_FAIL(-1, "ocm_copy_onesided_batch: NULL argument");
    if (!s.allocs.count(a)) OCM_FAIL(-1, "ocm_copy_onesided_batch: unknown allocation");
    if (!a->remote) OCM_FAIL(-1, "batched one-sided copies need a remote pair (kind %d)", (int)a->kind);
    if (n_ops < 0) OCM_FAIL(-1, "ocm_copy_onesided_batch: n_ops < 0");
    const bool async = (flags & OCM_BATCH_ASYNC) != 0;
    if (check_batch_ops(a, ops, n_ops, moved) != 0) return -1;
    if (n_ops == 0) return 0;
    if (!batch_device_path(a)) {
        // No device-side path (CPU app, network tier, host local half): op by op, in order.
        for (int i = 0; i < n_ops; i++)
            if (xfer(a, ops[i].op_flag != 0, static_cast<char *>(a->local) + ops[i].src_offset, a->loc,
                     ops[i].dest_offset, ops[i].bytes, async) != 0)
                return -1;
        return 0;
    }
    DeviceGuard guard(s.device);
    XferBatchArgs args;
    std::vector<XferBatchOp> v;
    build_batch_args(a, ops, n_ops, &args, &v);
    if (args.total_tiles == 0) return 0;  // only empty ops
    return run_batch(a, args, v, async);
}

int ocm_stream_wait(ocm_alloc_t a, void *stream) {
    State &s = S();
    std::lock_guard<std::recursive_mutex> lk(s.mu);
    if (!a || !s.allocs.count(a)) OCM_FAIL(-1, "ocm_stream_wait: unknown allocation");
    if (s.device < 0) return 0;  // CPU app: every op is synchronous already
    DeviceGuard g(s.device);
    if (!a->dep_ev && hipEventCreateWithFlags(&a->dep_ev, hipEventDisableTiming) != hipSuccess) {
        (void)hipGetLastError();
        a->dep_ev = nullptr;
        OCM_FAIL(-1, "ocm_stream_wait: no event");
    }
    hipError_t e = hipEventRecord(a->dep_ev, static_cast<hipStream_t>(stream));
    if (e != hipSuccess) OCM_FAIL(-1, "ocm_stream_wait: %s", hipGetErrorString(e));
    a->dep_pending = true;
    return 0;
}

int ocm_stream_signal(ocm_alloc_t a, void *stream) {
    State &s = S();
    std::lock_guard<std::recursive_mutex> lk(s.mu);
    if (!a || !s.allocs.count(a)) OCM_FAIL(-1, "ocm_stream_signal: unknown allocation");
    if (s.device < 0 || !a->async_pending || !a->ev) return 0;  // nothing queued: already complete
    DeviceGuard g(s.device);
    hipError_t e = hipStreamWaitEvent(static_cast<hipStream_t>(stream), a->ev, 0);
    if (e != hipSuccess) OCM_FAIL(-1, "ocm_stream_signal: %s", hipGetErrorString(e));
    return 0;
}

// ---------------- transfer plans (hipGraph replay of fixed batch schedules) ----------------

ocm_plan_t ocm_plan_create(void) {
    State &s = S();
    std::lock_guard<std::recursive_mutex> lk(s.mu);
    if (!s.inited) {
        set_last_error("ocm_plan_create: ocm_init first");
        return nullptr;
    }
    if (s.device < 0) {
        set_last_error("ocm_plan_create: plans replay on a GPU; this process has none");
        return nullptr;
    }
    return new ocm_plan();
}

static void plan_drop_graph(ocm_plan *p) {
    if (p->exec) (void)hipGraphExecDestroy(p->exec);
    if (p->graph) (void)hipGraphDestroy(p->graph);
    p->exec = nullptr;
    p->graph = nullptr;
}

int ocm_plan_add(ocm_plan_t p, ocm_alloc_t a, const struct ocm_params *ops, int n_ops) {
    State &s = S();
    std::lock_guard<std::recursive_mutex> lk(s.mu);
    if (!p || !a || (!ops && n_ops) || n_ops < 0) OCM_FAIL(-1, "ocm_plan_add: bad argument");
    if (!s.allocs.count(a) || !a->remote) OCM_FAIL(-1, "ocm_plan_add: not a live remote pair");
    if (!batch_device_path(a)) OCM_FAIL(-1, "ocm_plan_add: this pair has no device-side path (plans need one)");
    uint64_t moved = 0;
    if (check_batch_ops(a, ops, n_ops, &moved) != 0) return -1;
    if (n_ops == 0) return 0;
    DeviceGuard g(s.device);
    ocm_plan::Stage st;
    st.a = a;
    std::vector<XferBatchOp> v;
    build_batch_args(a, ops, n_ops, &st.args, &v);
    if (st.args.total_tiles == 0) return 0;
    if (n_ops > kXferInlineOps) {
        const size_t dbytes = v.size() * sizeof(XferBatchOp);
        const size_t need = dbytes + (size_t)st.args.grid * 4 * sizeof(uint32_t);
        std::vector<char> up(need);
        std::memcpy(up.data(), v.data(), dbytes);
        xfer_batch_wave_ops(v.data(), (uint32_t)n_ops, st.args.total_tiles, st.args.grid,
                            reinterpret_cast<uint32_t *>(up.data() + dbytes));
        hipError_t e = hipMalloc(&st.dev, need);
        if (e == hipSuccess) e = hipMemcpy(st.dev, up.data(), need, hipMemcpyHostToDevice);
        if (e != hipSuccess) {
            (void)hipGetLastError();
            if (st.dev) (void)hipFree(st.dev);
            OCM_FAIL(-1, "ocm_plan_add: descriptor upload: %s", hipGetErrorString(e));
        }
        st.args.ops = static_cast<const XferBatchOp *>(st.dev);
        st.args.wave_op = reinterpret_cast<const uint32_t *>(static_cast<char *>(st.dev) + dbytes);
    }
    p->stages.push_back(st);
    p->bytes += moved;
    p->n_ops += (uint64_t)n_ops;
    a->plans++;
    plan_drop_graph(p);  // rebuilt at the next launch (the stages may have moved)
    return 0;
}

int ocm_plan_launch(ocm_plan_t p, void *stream) {
    State &s = S();
    std::lock_guard<std::recursive_mutex> lk(s.mu);
    TraceRange tr("ocm_plan_launch");
    const uint64_t t0 = now_ns();
    if (!p) OCM_FAIL(-1, "ocm_plan_launch: NULL plan");
    if (p->stages.empty()) return 0;
    DeviceGuard g(s.device);
    hipError_t e = hipSuccess;
    if (!p->exec) {
        // Build the stage chain as a graph once (explicit kernel nodes, no stream
        // capture: a capture would fail if another thread synchronized the device
        // meanwhile, tools/gpu_fuzz.py --threads); every later launch is one
        // hipGraphLaunch.
        hipGraph_t graph = nullptr;
        e = hipGraphCreate(&graph, 0);
        hipGraphNode_t prev = nullptr;
        for (size_t i = 0; e == hipSuccess && i < p->stages.size(); i++) {
            hipGraphNode_t node = nullptr;
            e = xfer_batch_graph_node(graph, prev, p->stages[i].args, s.tuning, &node);
            prev = node;
        }
        if (e == hipSuccess) e = hipGraphInstantiate(&p->exec, graph, nullptr, nullptr, 0);
        if (e != hipSuccess) {
            (void)hipGetLastError();
            if (graph) (void)hipGraphDestroy(graph);
            p->exec = nullptr;
            OCM_FAIL(-1, "ocm_plan_launch: graph build: %s", hipGetErrorString(e));
        }
        p->graph = graph;
    }
    hipStream_t st = stream ? static_cast<hipStream_t>(stream) : s.stream;
    // Order after the allocations' own queued work and ocm_stream_wait dependencies.
    for (auto &sg : p->stages) {
        lib_alloc *a = sg.a;
        if (a->async_pending && a->ev) (void)hipStreamWaitEvent(st, a->ev, 0);
        if (honor_dep(a, st, false) != 0) return -1;
    }
    before_launch();
    e = hipGraphLaunch(p->exec, st);
    if (e != hipSuccess) OCM_FAIL(-1, "ocm_plan_launch: %s", hipGetErrorString(e));
    int rc = stream ? 0 : sync_stream();
    const uint64_t t1 = now_ns();
    if (rc == 0) {
        OpCounters &c = s.ctr;
        c.n_batch++;
        c.n_batch_ops += p->n_ops;
        c.bytes_batch += p->bytes;
        c.ns_batch += t1 - t0;
    }
    trace_op("plan", p->bytes, t0, t1, rc);
    return rc;
}

int ocm_plan_destroy(ocm_plan_t p) {
    State &s = S();
    std::lock_guard<std::recursive_mutex> lk(s.mu);
    if (!p) return -1;
    DeviceGuard g(s.device);
    plan_drop_graph(p);
    for (auto &st : p->stages) {
        if (st.dev) (void)hipFree(st.dev);  // synchronizing free: replays have finished
        if (s.allocs.count(st.a) && st.a->plans > 0) st.a->plans--;
    }
    delete p;
    return 0;
}


}  // extern "C"

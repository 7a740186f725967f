// libocm: the application library behind oncillamem.h.
//
// Parity with reference src/lib.c (struct lib_alloc, ocm_init/tini/alloc/free,
// accessors, ocm_copy, ocm_copy_onesided). MI355X design:
//   * control: one mailbox RPC to the local ocmd (seq-matched; a bounded poll
//     for the reply, then a blocking wait), multi-record replies for striped pairs;
//   * registration: remote HBM extents are imported once per slab with
//     hipIpcOpenMemHandle (lazy peer access) and cached; host-tier extents are
//     mmap'ed from the owner's memfd and hipHostRegister'ed (device-mapped);
//   * data: one-sided put/get run the gfx950 transfer kernel (ocm/xfer.h) on a
//     per-process non-blocking stream; host-tier legs use the DMA engines
//     (hipMemcpyAsync); completion = stream sync, or ocm_wait() for the async form.
// Reference defects deliberately not reproduced: inverted ocm_is_remote
// (src/lib.c:461), NULL deref before check in ocm_free (:357-359), stub
// copy_in/out (:491-499), swapped GPU->RMA offsets (:654).
#include <cmath>

#include "internal.h"
#include "ocm/affinity.h"
#include "ocm/optim.h"

using namespace ocm;
using namespace ocmlib;

// ================================================================ C API

extern "C" {

int ocm_init(void) {
    State &s = S();
    std::lock_guard<std::recursive_mutex> lk(s.mu);
    if (s.inited) return 0;
    s.pid = getpid();
    s.ns = pmsg_namespace();
    const char *dr = std::getenv("OCM_DAEMON_RANK");
    const char *lr = std::getenv("LOCAL_RANK");
    s.daemon_rank = dr && *dr ? std::atoi(dr) : (lr && *lr ? std::atoi(lr) : 0);
    s.daemon_mbox = daemon_mailbox_name(s.daemon_rank, s.ns);
    s.rpc_timeout_ms = env_int("OCM_RPC_TIMEOUT_MS", 60000);
    s.rpc_spin_ns = (uint64_t)std::max(0, env_int("OCM_RPC_SPIN_US", 50)) * 1000;
    s.net_streams = std::max(1, std::min(env_int("OCM_NET_STREAMS", 4), 64));
    if (const char *ns = std::getenv("OCM_NET_SPLIT_MIN")) s.net_split_min = std::max(4096ull, std::strtoull(ns, nullptr, 0));
    const int connect_ms = env_int("OCM_CONNECT_TIMEOUT_MS", 10000);
    // Connect to the daemon mailbox, retrying while it starts (reference: 10 x 10 ms).
    long deadline = now_ms() + connect_ms;
    if (s.chan.connect(s.daemon_mbox, connect_ms) != 0)
        OCM_FAIL(-1, "no ocmd mailbox @%s (is the daemon running?)", s.daemon_mbox.c_str());
    // Shared-memory fast path of the mailbox (ocm/shmlink.h), offered with CONNECT.
    // Every CONNECT offers a fresh link: the daemon attaches each offer anew, with
    // its ring counts at zero, so a retried CONNECT must not reuse a link whose
    // counts have moved on.
    const bool want_link = env_int("OCM_SHM_LINK", 1) != 0;
    Msg reply;
    for (;;) {
        if (want_link && s.link.create() != 0) OCM_WARN("no shared-memory link (%s); mailbox only", strerror(errno));
        Msg c = new_msg(MSG_CONNECT);
        if (rpc(c, &reply, std::max(1000, connect_ms)) != 0) {
            s.chan.close();
            s.link.close();
            return -1;
        }
        if (s.link.ok() && !s.last_via_link) {
            // The daemon answered on the socket: it did not take the link (it found it
            // unusable, or does not take links at all). Requests stay on the socket.
            OCM_INFO("ocmd declined the shared-memory link; using the mailbox socket");
            s.link.close();
        }
        if (reply.err != EAGAIN) break;
        if (now_ms() > deadline) {
            s.chan.close();
            s.link.close();
            OCM_FAIL(-1, "daemon mesh not ready after %d ms", connect_ms);
        }
        usleep(20000);  // mesh still joining
    }
    s.daemon = reply.u.node;
    // Pick the GPU this process copies on: OCM_GPU, else the daemon's GPU.
    int ndev = 0;
    if (!std::getenv("OCM_NO_GPU") && hipGetDeviceCount(&ndev) != hipSuccess) {
        (void)hipGetLastError();
        ndev = 0;
    }
    const char *g = std::getenv("OCM_GPU");
    int dev = g && *g ? std::atoi(g) : s.daemon.gpu;
    if (dev < 0 && ndev > 0 && s.daemon.gpu >= 0) dev = 0;
    s.device = (ndev > 0 && dev >= 0 && dev < ndev) ? dev : -1;
    s.peers_enabled = 0;
    if (s.device >= 0) {
        DeviceGuard guard(s.device);
        if (hipStreamCreateWithFlags(&s.stream, hipStreamNonBlocking) != hipSuccess) {
            (void)hipGetLastError();
            OCM_FAIL(-1, "cannot create HIP stream on device %d", s.device);
        }
        if (hipEventCreateWithFlags(&s.done, hipEventDisableTiming) != hipSuccess) {
            (void)hipGetLastError();
            s.done = nullptr;
        }
        // Map every peer MI355X now: remote extents are read/written by kernels
        // on this device over xGMI (imports also request lazy peer access).
        for (int p = 0; p < ndev; p++) {
            int can = 0;
            if (p == s.device || hipDeviceCanAccessPeer(&can, s.device, p) != hipSuccess || !can) continue;
            hipError_t pe = hipDeviceEnablePeerAccess(p, 0);
            if (pe != hipSuccess && pe != hipErrorPeerAccessAlreadyEnabled)
                OCM_WARN("peer access %d -> %d: %s", s.device, p, hipGetErrorString(pe));
            else
                s.peers_enabled++;
            (void)hipGetLastError();
        }
    }
    if (s.device >= 0) {
        // This thread next to the GPU, on the L3 complex its daemon uses (ocm/affinity.h).
        char bus[64] = {0};
        DeviceGuard guard(s.device);
        if (hipDeviceGetPCIBusId(bus, sizeof(bus), s.device) == hipSuccess)
            (void)pin_near_gpu(bus, s.device, PinRole::App, s.daemon_rank);
        else
            (void)hipGetLastError();
    }
    s.sync_mode = env_int("OCM_SYNC_MODE", 1);
    s.n_lanes = env_int("OCM_ASYNC_LANES", 4);
    if (const char *k = std::getenv("OCM_PINNED_KEEP")) s.pinned_keep = std::strtoull(k, nullptr, 0);
    if (const char *k = std::getenv("OCM_LOCAL_CACHE")) s.dev_cache_cap = std::strtoull(k, nullptr, 0);
    const char *sm = std::getenv("OCM_SERVICE_MAX");
    s.svc_max = sm && *sm ? std::strtoull(sm, nullptr, 0) : kServiceMaxDefault;
    const char *smh = std::getenv("OCM_SERVICE_MAX_HOST");  // unset: follows an explicit OCM_SERVICE_MAX
    s.svc_max_host = smh && *smh ? std::strtoull(smh, nullptr, 0) : (sm && *sm ? s.svc_max : kServiceMaxHostDefault);
    s.svc_blocks = (unsigned)std::max(1, std::min(env_int("OCM_SERVICE_BLOCKS", kServiceBlocksDefault), 1024));
    s.svc_solo_tiles = (unsigned)std::max(0, env_int("OCM_SERVICE_SOLO_TILES", kServiceSoloTilesDefault));
    s.svc_solo_tiles_host_get = (unsigned)std::max(0, env_int("OCM_SERVICE_SOLO_TILES_HOST_GET", 1));
    s.svc_proto = (unsigned)env_int("OCM_SERVICE_PROTO", (int)kServiceProtoDefault) & kServiceProtoMask;
    // OCM_SERVICE_STRICT=1 (measurements, tests): every request takes the STRICT
    // (peer-HBM) hand-off, so its cost shows on a one-GPU box
    s.svc_force_strict = env_int("OCM_SERVICE_STRICT", 0) != 0;
    if (const char *v = std::getenv("OCM_SERVICE_MAX_LOCAL"); v && *v) s.svc_max_local = std::strtoull(v, nullptr, 0);
    s.svc_gang_host = (unsigned)std::max(1, std::min(env_int("OCM_SERVICE_GANG_HOST", (int)s.svc_gang_host), 1024));
    s.svc_direct = (unsigned)std::max(1, std::min(env_int("OCM_SERVICE_DIRECT", kServiceDirectDefault), 1024));
    if (s.svc_direct > (unsigned)kServiceGangCopiesMax) s.svc_proto &= ~kServiceProtoCopies;  // one page of copies
    if (const char *v = std::getenv("OCM_SERVICE_DIRECT_MAX_HOST"); v && *v) s.svc_direct_max_host = std::strtoull(v, nullptr, 0);
    if (const char *v = std::getenv("OCM_SERVICE_DIRECT_MAX_HBM"); v && *v) s.svc_direct_max_hbm = std::strtoull(v, nullptr, 0);
    s.svc_host_tile_shift_get = (unsigned)std::max(0, env_int("OCM_SERVICE_HOST_TILE_SHIFT_GET", (int)s.svc_host_tile_shift_get));
    s.svc_host_tile_shift_put = (unsigned)std::max(0, env_int("OCM_SERVICE_HOST_TILE_SHIFT_PUT", (int)s.svc_host_tile_shift_put));
    if (const char *v = std::getenv("OCM_SERVICE_HOST_TILE_MAX"); v && *v) s.svc_host_tile_max = std::strtoull(v, nullptr, 0);
    if (const char *v = std::getenv("OCM_SERVICE_HOST_TILE_MIN"); v && *v) s.svc_host_tile_min = std::strtoull(v, nullptr, 0);
    if (const char *v = std::getenv("OCM_SERVICE_HOST_GET_NARROW_MIN"); v && *v)
        s.svc_host_get_narrow_min = std::strtoull(v, nullptr, 0);
    s.svc_host_get_width = (unsigned)std::max(1, std::min(env_int("OCM_SERVICE_HOST_GET_WIDTH", 12), 1024));
    s.launch_flags = env_int("OCM_LAUNCH_FLAG", 1) != 0;
    s.svc_park_kernel = env_int("OCM_SERVICE_PARK_KERNEL", 0) != 0;
    s.svc_idle_ticks = 100ull * (unsigned long long)std::max(1, env_int("OCM_SERVICE_IDLE_US", kServiceIdleUsDefault));  // 100 MHz clock
    s.svc_roster_wait_ns = 1000ull * (unsigned long long)std::max(0, env_int("OCM_SERVICE_ROSTER_WAIT_US", 200));
    s.svc_timeout_ns = 1000000ull * (unsigned long long)std::max(1, env_int("OCM_SERVICE_TIMEOUT_MS", 10000));
    s.svc_drain_ns = 1000000ull * (unsigned long long)std::max(1, env_int("OCM_SERVICE_DRAIN_MS", 10000));
    s.svc_box_reset_always = env_int("OCM_SERVICE_BOX_RESET", 0) != 0;
    s.svc_lanes_max = (unsigned)std::max(1, std::min(env_int("OCM_SERVICE_STREAMS", 4), 16));
    s.svc_relaunch_query = env_int("OCM_SERVICE_RELAUNCH_QUERY", 0) != 0;
    s.svc_degraded_idle_ticks = 100ull * (unsigned long long)std::max(1, env_int("OCM_SERVICE_DEGRADED_IDLE_US", 5000));
    {
        const char *v = std::getenv("OCM_SERVICE_QUEUE");  // State outlives ocm_tini: set it on every init
        s.svc_queue_aql = !(v && std::strcmp(v, "hip") == 0);
    }
    s.svc_lone_ticks = 100ull * (unsigned long long)std::max(0, env_int("OCM_SERVICE_LONE_US", kServiceLoneUsDefault));
    const char *lfm = std::getenv("OCM_LAUNCH_FLAG_MAX");
    s.launch_flag_max = lfm && *lfm ? std::strtoull(lfm, nullptr, 0) : kLaunchFlagMaxDefault;
    s.tuning = xfer_tuning_from_env();
    const char *he = std::getenv("OCM_HOST_ENGINE");
    s.host_engine_kernel = !(he && !std::strcmp(he, "sdma"));  // the PCIe streaming kernel unless asked for SDMA
    if (he && !std::strcmp(he, "sdma")) s.host_kernel_max = 0;
    if (const char *hk = std::getenv("OCM_HOST_KERNEL_MAX")) s.host_kernel_max = std::strtoull(hk, nullptr, 0);
    s.inited = true;
    OCM_LOG("attached to ocmd rank %d (gpu %d, %u nodes), copying on device %d", s.daemon_rank, s.daemon.gpu,
            s.daemon.num_nodes, s.device);
    return 0;
}

// An application that exits without ocm_tini may leave the copy service's lone
// lead resident on the library's AQL queue: tell it to leave (a store to the
// host record; nothing waits, the process is going away).
__attribute__((destructor)) static void ocm_lib_exit() {
    State &s = S();
    if (s.svc && s.svc_req) {
        service_store_seq(s.svc_req, kServiceStop);
        if (s.svc_greq) service_store_seq(s.svc_greq, kServiceStop, s.svc_greq_copies);
    }
}

int ocm_tini(void) {
    State &s = S();
    std::lock_guard<std::recursive_mutex> lk(s.mu);
    if (!s.inited) return -1;
    service_stop();  // no copy-service instance may outlive the mappings below
    std::vector<lib_alloc *> left(s.allocs.begin(), s.allocs.end());
    for (auto *a : left) ocm_free(a);
    Msg d = new_msg(MSG_DISCONNECT);
    s.chan.send(&d, kMsgBytes, 1000);
    push_release();
    for (auto &kv : s.imports) {
        Mapping &m = kv.second;
        for (auto &v : m.dev_views) {
            DeviceGuard gv(v.first);
            (void)hipIpcCloseMemHandle(v.second);
        }
        m.dev_views.clear();
        DeviceGuard g(s.device);
        if (kv.first.tier == TIER_GPU && m.dbase) (void)hipIpcCloseMemHandle(m.dbase);
        if (m.registered) (void)hipHostUnregister(m.hbase);
        if (m.hbase) munmap(m.hbase, m.bytes);
    }
    s.imports.clear();
    net_close_all();
    close_fd_chans();
    for (auto st : s.lanes) {
        DeviceGuard g(s.device);
        (void)hipStreamSynchronize(st);
        (void)hipStreamDestroy(st);
    }
    s.lanes.clear();
    s.next_lane = 0;
    if (s.lane_flags) {
        DeviceGuard g(s.device);
        (void)hipHostFree(s.lane_flags);
        (void)hipFree(s.lane_cnt);
        s.lane_flags = nullptr;
        s.lane_cnt = nullptr;
        s.lane_flag_seq.clear();
    }
    release_dev_cache();
    if (s.pattern_bad) {
        DeviceGuard g(s.device);
        (void)hipFree(s.pattern_bad);
        s.pattern_bad = nullptr;
    }
    if (s.stream) {
        DeviceGuard g(s.device);
        (void)hipStreamSynchronize(s.stream);
        (void)hipStreamDestroy(s.stream);
        s.stream = nullptr;
    }
    if (s.pool) {
        DeviceGuard g(s.device);
        (void)hipMemPoolDestroy(s.pool);
        s.pool = nullptr;
    }
    s.pool_tried = false;
    if (s.pinned) s.pinned->release_all();
    s.chan.close();
    s.link.close();
    s.inited = false;
    trace_flush("app");
    return 0;
}

ocm_alloc_t ocm_alloc(ocm_alloc_param_t p) { return ocm_alloc_ex(p, nullptr); }

static ocm_alloc_t alloc_impl(ocm_alloc_param_t p, const struct ocm_alloc_ex_params *ex);

ocm_alloc_t ocm_alloc_ex(ocm_alloc_param_t p, const struct ocm_alloc_ex_params *ex) {
    TraceRange tr("ocm_alloc");
    const uint64_t t0 = now_ns();
    ocm_alloc_t a = alloc_impl(p, ex);
    const uint64_t t1 = now_ns();
    State &s = S();
    if (a) {
        s.ctr.n_alloc++;
        s.ctr.ns_alloc += t1 - t0;
    }
    trace_op("alloc", p ? (p->rem_alloc_bytes ? p->rem_alloc_bytes : p->local_alloc_bytes) : 0, t0, t1, a ? 0 : -1);
    return a;
}

static ocm_alloc_t alloc_impl(ocm_alloc_param_t p, const struct ocm_alloc_ex_params *ex) {
    State &s = S();
    std::lock_guard<std::recursive_mutex> lk(s.mu);
    if (!s.inited) OCM_FAIL(nullptr, "ocm_alloc before ocm_init");
    if (!p) OCM_FAIL(nullptr, "ocm_alloc: NULL parameters");
    enum ocm_kind kind = p->kind;
    if (kind == OCM_LOCAL_RMA || kind == OCM_LOCAL_RDMA) kind = OCM_LOCAL_HOST;
    if (kind < OCM_LOCAL_HOST || kind > OCM_REMOTE_GPU) OCM_FAIL(nullptr, "ocm_alloc: invalid kind %d", (int)p->kind);
    const bool pair = is_pair(kind);
    if (kind == OCM_LOCAL_GPU && s.device < 0) OCM_FAIL(nullptr, "OCM_LOCAL_GPU requested but no GPU is available");
    const uint64_t req_bytes = pair ? p->rem_alloc_bytes : p->local_alloc_bytes;
    if (req_bytes == 0) OCM_FAIL(nullptr, "ocm_alloc: zero-byte request");

    Msg m = new_msg(MSG_REQ_ALLOC);
    m.u.req.orig_rank = s.daemon_rank;
    m.u.req.remote_rank = ex ? ex->remote_rank : -1;
    m.u.req.bytes = req_bytes;
    m.u.req.kind = (uint32_t)kind;
    m.u.req.flags = ex ? ex->flags : 0;
    if (s.device < 0) m.u.req.flags |= OCM_ALLOC_HOST_TIER;  // a CPU-only app cannot map HBM
    m.u.req.stripe_width = ex ? ex->stripe_width : 0;
    m.u.req.stripe_unit = ex ? ex->stripe_unit : 0;
    m.u.req.tier = (m.u.req.flags & OCM_ALLOC_HOST_TIER) ? TIER_HOST : TIER_GPU;
    m.u.req.app_pid = s.pid;
    if (m.u.req.stripe_unit && log2_exact(m.u.req.stripe_unit) < 12)
        OCM_FAIL(nullptr, "stripe unit must be a power of two >= 4 KiB");
    Msg r;
    if (rpc(m, &r, s.rpc_timeout_ms) != 0) return nullptr;
    if (r.type != MSG_RELEASE_APP) OCM_FAIL(nullptr, "unexpected reply %s", msg_type_str(r.type));
    if (r.err) OCM_FAIL(nullptr, "ocm_alloc of %llu bytes failed: %s", (unsigned long long)req_bytes, strerror(r.err));

    auto *a = new lib_alloc();
    a->kind = kind;
    a->alloc_id = r.u.region.alloc_id;
    if (pair) {
        a->remote = true;
        a->remote_bytes = r.u.region.bytes;
        a->stripe_unit = r.u.region.stripe_unit;
        const int n = r.u.region.n_extents;
        a->ext.resize(n);
        bool ok = n >= 1 && n <= kMaxExtents;
        for (int i = 0; ok && i < n; i++) {
            Msg e;
            if (recv_seq(&e, r.seq, MSG_EXTENT, s.rpc_timeout_ms) != 0) {
                ok = false;
                break;
            }
            const int idx = e.u.region.extent_idx;
            if (idx >= n) {
                ok = false;
                break;
            }
            a->ext[idx].r = e.u.region;
        }
        for (int i = 0; ok && i < n; i++) ok = import_extent(a->ext[i]) == 0;
        if (ok) {
            a->all_gpu = a->any_gpu = false;
            bool all = true;
            for (auto &e : a->ext) {
                all &= e.r.tier == TIER_GPU;
                a->any_gpu |= e.r.tier == TIER_GPU;
            }
            a->all_gpu = all;
            a->all_dev_ok = true;
            for (auto &e : a->ext) {
                a->all_dev_ok &= e.dev_ok;
                a->any_net |= e.net;
                if (e.net) a->all_gpu = false;
            }
            a->any_gpu = a->any_gpu && !a->any_net;
            a->same_gpu = a->all_gpu && s.device >= 0;
            for (auto &e : a->ext) a->same_gpu &= e.r.owner_gpu == s.device;
            a->any_peer = false;
            for (auto &e : a->ext) a->any_peer |= !e.net && e.r.tier == TIER_GPU && e.r.owner_gpu != s.device;
            Loc want = kind == OCM_REMOTE_GPU ? LOC_DEVICE : LOC_PINNED;
            ok = alloc_local_half(a, p->local_alloc_bytes, want) == 0;
        }
        if (!ok) {
            std::string why = last_error();
            for (auto &e : a->ext)
                if (e.dptr || e.hptr) release_extent(e, false);
            Msg f = new_msg(MSG_REQ_FREE);
            f.u.req.alloc_id = a->alloc_id;
            Msg fr;
            rpc(f, &fr, s.rpc_timeout_ms);
            free_local_half(a);
            delete a;
            set_last_error("%s", why.c_str());
            return nullptr;
        }
    } else {
        Loc want = kind == OCM_LOCAL_GPU ? LOC_DEVICE : LOC_HOST;
        if (alloc_local_half(a, p->local_alloc_bytes, want) != 0) {
            std::string why = last_error();
            Msg f = new_msg(MSG_REQ_FREE);
            f.u.req.alloc_id = a->alloc_id;
            Msg fr;
            rpc(f, &fr, s.rpc_timeout_ms);
            delete a;
            set_last_error("%s", why.c_str());
            return nullptr;
        }
    }
    if ((m.u.req.flags & OCM_ALLOC_ZERO) && a->local) {
        if (a->loc == LOC_DEVICE) {
            DeviceGuard g(s.device);
            (void)hipMemsetAsync(a->local, 0, a->local_bytes, s.stream);
            sync_stream();
        } else {
            std::memset(a->local, 0, a->local_bytes);
        }
    }
    s.allocs.insert(a);
    return a;
}

static int free_impl(ocm_alloc_t a);

int ocm_free(ocm_alloc_t a) {
    TraceRange tr("ocm_free");
    const uint64_t t0 = now_ns();
    int rc = free_impl(a);
    const uint64_t t1 = now_ns();
    S().ctr.n_free += rc == 0;
    S().ctr.ns_free += t1 - t0;
    trace_op("free", 0, t0, t1, rc);
    return rc;
}

static int free_impl(ocm_alloc_t a) {
    State &s = S();
    std::lock_guard<std::recursive_mutex> lk(s.mu);
    if (!a || !s.allocs.count(a)) OCM_FAIL(-1, "ocm_free: unknown allocation");
    if (a->plans) OCM_FAIL(-1, "ocm_free: allocation is used by %d plan stage(s); destroy the plans first", a->plans);
    wait_alloc(a);
    if (a->batch_dev || a->batch_host) {
        DeviceGuard g(s.device);
        if (a->batch_up) (void)hipEventSynchronize(a->batch_up);
        if (a->batch_dev) (void)hipFreeAsync(a->batch_dev, s.stream);
        if (a->batch_host) (void)hipHostFree(a->batch_host);
        if (a->batch_up) (void)hipEventDestroy(a->batch_up);
        a->batch_dev = a->batch_host = nullptr;
        a->batch_up = nullptr;
    }
    if (a->ev) {
        DeviceGuard g(s.device);
        (void)hipEventDestroy(a->ev);
        a->ev = nullptr;
    }
    if (a->dep_ev) {
        DeviceGuard g(s.device);
        (void)hipEventDestroy(a->dep_ev);
        a->dep_ev = nullptr;
    }
    // Unmap dedicated remote slabs before the owner frees them.
    for (auto &e : a->ext) release_extent(e, false);
    free_local_half(a);
    Msg f = new_msg(MSG_REQ_FREE);
    f.u.req.alloc_id = a->alloc_id;
    f.u.req.n_extents = (int32_t)a->ext.size();
    Msg r;
    int rc = rpc(f, &r, s.rpc_timeout_ms);
    s.allocs.erase(a);
    delete a;
    if (rc != 0) return -1;
    if (r.err) OCM_FAIL(-1, "ocm_free: %s", strerror(r.err));
    return 0;
}

int ocm_localbuf(ocm_alloc_t a, void **buf, size_t *len) {
    if (!a || !buf || !len) return -1;
    *buf = a->local;
    *len = a->local_bytes;
    return 0;
}

bool ocm_is_remote(ocm_alloc_t a) { return a && a->remote; }

enum ocm_kind ocm_alloc_kind(ocm_alloc_t a) { return a ? a->kind : (enum ocm_kind)0; }

int ocm_remote_sz(ocm_alloc_t a, size_t *len) {
    if (!a || !len || !a->remote) return -1;  // no remote buffer for local kinds
    *len = a->remote_bytes;
    return 0;
}

static int onesided_impl(ocm_alloc_t a, ocm_param_t p, bool async);

static int ocm_copy_onesided_impl(ocm_alloc_t a, ocm_param_t p, bool async) {
    const bool put = p && p->op_flag != 0;
    TraceRange tr(put ? "ocm_put" : "ocm_get");
    const uint64_t t0 = now_ns();
    int rc = onesided_impl(a, p, async);
    const uint64_t t1 = now_ns();
    if (rc == 0 && p) {
        OpCounters &c = S().ctr;
        (put ? c.n_put : c.n_get)++;
        (put ? c.bytes_put : c.bytes_get) += p->bytes;
        (put ? c.ns_put : c.ns_get) += t1 - t0;
    }
    trace_op(put ? "put" : "get", p ? p->bytes : 0, t0, t1, rc);
    return rc;
}

static int onesided_impl(ocm_alloc_t a, ocm_param_t p, bool async) {
    State &s = S();
    hipEvent_t wait_ev = nullptr;
    XferDone wait_done_flag;
    {
        std::lock_guard<std::recursive_mutex> lk(s.mu);
        if (!a || !p) OCM_FAIL(-1, "ocm_copy_onesided: NULL argument");
        if (!s.allocs.count(a)) OCM_FAIL(-1, "ocm_copy_onesided: unknown allocation");
        if (!a->remote) OCM_FAIL(-1, "one-sided copy needs a remote pair (kind %d)", (int)a->kind);
        // Bounds (reference src/rdma.c:55-59, src/lib.c:679): the local side is
        // src_offset, the remote side dest_offset, for both directions (overflow-safe).
        if (p->src_offset > a->local_bytes || p->bytes > a->local_bytes - p->src_offset)
            OCM_FAIL(-1, "one-sided copy: local range [%llu,+%llu) exceeds %zu bytes",
                     (unsigned long long)p->src_offset, (unsigned long long)p->bytes, a->local_bytes);
        if (p->dest_offset > a->remote_bytes || p->bytes > a->remote_bytes - p->dest_offset)
            OCM_FAIL(-1, "one-sided copy: remote range [%llu,+%llu) exceeds %zu bytes",
                     (unsigned long long)p->dest_offset, (unsigned long long)p->bytes, a->remote_bytes);
        char *lin = static_cast<char *>(a->local) + p->src_offset;
        const bool put = p->op_flag != 0;
        // Large blocking ops: launch on the allocation's lane under the lock, wait
        // outside it, so other threads' ops proceed meanwhile. Small ones keep the
        // copy service (no launch) and the network tier its own blocking path.
        const bool service = a->loc == LOC_DEVICE && a->all_dev_ok && p->bytes <= s.svc_limit(a);
        if (async || s.device < 0 || service || a->any_net)
            return xfer(a, put, lin, a->loc, p->dest_offset, p->bytes, async);
        if (xfer(a, put, lin, a->loc, p->dest_offset, p->bytes, true, &wait_done_flag) != 0) return -1;
        if (!a->async_pending || !a->ev) return 0;  // it completed inside xfer
        wait_ev = a->ev;
    }
    DeviceGuard g(s.device);
    // The kernel publishes its own completion (~6 us before the runtime's event).
    if (wait_done_flag.flag) return wait_done(wait_done_flag, wait_ev);
    return wait_event(wait_ev);
}

int ocm_copy_onesided(ocm_alloc_t a, ocm_param_t p) { return ocm_copy_onesided_impl(a, p, false); }
int ocm_copy_onesided_async(ocm_alloc_t a, ocm_param_t p) { return ocm_copy_onesided_impl(a, p, true); }

int ocm_wait(ocm_alloc_t a) {
    State &s = S();
    std::lock_guard<std::recursive_mutex> lk(s.mu);
    if (a) {
        if (!s.allocs.count(a)) OCM_FAIL(-1, "ocm_wait: unknown allocation");
        return wait_alloc(a);
    }
    int rc = 0;  // NULL: every allocation
    for (auto *x : s.allocs) rc |= wait_alloc(x);
    return rc | sync_stream();
}

static bool range_ok(uint64_t off, uint64_t n, uint64_t cap) { return off <= cap && n <= cap - off; }

static int copy_impl(ocm_alloc_t dst, ocm_alloc_t src, ocm_param_t p);

int ocm_copy(ocm_alloc_t dst, ocm_alloc_t src, ocm_param_t p) {
    TraceRange tr("ocm_copy");
    const uint64_t t0 = now_ns();
    int rc = copy_impl(dst, src, p);
    const uint64_t t1 = now_ns();
    if (rc == 0 && p) {
        S().ctr.n_copy++;
        S().ctr.bytes_copy += p->bytes;
    }
    trace_op("copy", p ? p->bytes : 0, t0, t1, rc);
    return rc;
}

static int copy_impl(ocm_alloc_t dst, ocm_alloc_t src, ocm_param_t p) {
    State &s = S();
    std::lock_guard<std::recursive_mutex> lk(s.mu);
    if (!dst || !src || !p) OCM_FAIL(-1, "ocm_copy: NULL argument");
    if (wait_alloc(dst) != 0 || wait_alloc(src) != 0) return -1;  // their queued async ops come first
    // A read (op_flag == 0) is the write with the roles swapped (reference src/lib.c:511-515).
    struct ocm_params q = *p;
    if (!q.op_flag) {
        std::swap(dst, src);
        q.op_flag = 1;
    }
    const uint64_t n = q.bytes;
    if (!src->remote && !dst->remote) {
        if (!range_ok(q.src_offset, n, src->local_bytes) || !range_ok(q.dest_offset, n, dst->local_bytes))
            OCM_FAIL(-1, "ocm_copy: range out of bounds");
        return copy_local(static_cast<char *>(dst->local) + q.dest_offset, dst->loc,
                          static_cast<char *>(src->local) + q.src_offset, src->loc, n);
    }
    if (!src->remote && dst->remote) {
        // Stage into dst's local half, then one-sided write local[src_offset_2] -> remote[dest_offset_2].
        if (!range_ok(q.src_offset, n, src->local_bytes) || !range_ok(q.dest_offset, n, dst->local_bytes) ||
            !range_ok(q.src_offset_2, n, dst->local_bytes) || !range_ok(q.dest_offset_2, n, dst->remote_bytes))
            OCM_FAIL(-1, "ocm_copy: range out of bounds");
        if (copy_local(static_cast<char *>(dst->local) + q.dest_offset, dst->loc,
                       static_cast<char *>(src->local) + q.src_offset, src->loc, n) != 0)
            return -1;
        return xfer(dst, true, static_cast<char *>(dst->local) + q.src_offset_2, dst->loc, q.dest_offset_2, n, false);
    }
    if (src->remote && !dst->remote) {
        // One-sided read remote[dest_offset_2] -> src local[src_offset_2], then unstage.
        if (!range_ok(q.src_offset_2, n, src->local_bytes) || !range_ok(q.dest_offset_2, n, src->remote_bytes) ||
            !range_ok(q.src_offset, n, src->local_bytes) || !range_ok(q.dest_offset, n, dst->local_bytes))
            OCM_FAIL(-1, "ocm_copy: range out of bounds");
        if (xfer(src, false, static_cast<char *>(src->local) + q.src_offset_2, src->loc, q.dest_offset_2, n, false) != 0)
            return -1;
        return copy_local(static_cast<char *>(dst->local) + q.dest_offset, dst->loc,
                          static_cast<char *>(src->local) + q.src_offset, src->loc, n);
    }
    // remote -> remote (not supported by the reference): direct, no staging.
    if (!range_ok(q.src_offset, n, src->remote_bytes) || !range_ok(q.dest_offset, n, dst->remote_bytes))
        OCM_FAIL(-1, "ocm_copy: range out of bounds");
    if (src->any_net || dst->any_net) {
        // A side on another node: bounce through host memory, 64 MiB at a time.
        const uint64_t chunk = std::min<uint64_t>(n, 64ull << 20);
        std::vector<char> tmp(chunk);
        for (uint64_t done = 0; done < n;) {
            const uint64_t k = std::min(chunk, n - done);
            if (xfer(src, false, tmp.data(), LOC_HOST, q.src_offset + done, k, false) != 0) return -1;
            if (xfer(dst, true, tmp.data(), LOC_HOST, q.dest_offset + done, k, false) != 0) return -1;
            done += k;
        }
        return 0;
    }
    std::vector<Seg> ss;
    segments(src, q.src_offset, n, ss);
    const bool one_launch = s.device >= 0 && src->all_dev_ok && dst->all_dev_ok &&
                            (dst->ext.size() == 1 || log2_exact(dst->stripe_unit) >= 4);
    if (one_launch) {
        // Every source segment is a device address: one batched launch writes them all.
        std::vector<XferBatchOp> v(ss.size());
        for (size_t i = 0; i < ss.size(); i++) {
            const Seg &g = ss[i];
            v[i].lin_off = reinterpret_cast<uintptr_t>(src->ext[g.ext].dptr + g.ext_off);
            v[i].rem_off = q.dest_offset + g.lin_off;
            v[i].len = g.len;
            v[i].put = 1;
        }
        return batch_put_abs(dst, v);
    }
    for (auto &g : ss) {
        const Extent &e = src->ext[g.ext];
        char *sp = (s.device >= 0 ? e.dptr : e.hptr) + g.ext_off;
        Loc sl = (s.device >= 0 && (e.r.tier == TIER_GPU || e.dptr != e.hptr)) ? LOC_DEVICE : LOC_HOST;
        if (s.device >= 0 && sl == LOC_DEVICE) {
            if (xfer(dst, true, sp, LOC_DEVICE, q.dest_offset + g.lin_off, g.len, false) != 0) return -1;
        } else {
            if (xfer(dst, true, sp, LOC_HOST, q.dest_offset + g.lin_off, g.len, false) != 0) return -1;
        }
    }
    return 0;
}

int ocm_copy_in(ocm_alloc_t dst, void *src) {
    State &s = S();
    std::lock_guard<std::recursive_mutex> lk(s.mu);
    if (!dst || !src) OCM_FAIL(-1, "ocm_copy_in: NULL argument");
    if (wait_alloc(dst) != 0) return -1;
    const Loc sl = pointer_loc(src);
    if (dst->remote) return xfer(dst, true, static_cast<char *>(src), sl, 0, dst->remote_bytes, false);
    return copy_local(dst->local, dst->loc, src, sl, dst->local_bytes);
}

int ocm_copy_out(void *dst, ocm_alloc_t src) {
    State &s = S();
    std::lock_guard<std::recursive_mutex> lk(s.mu);
    if (!dst || !src) OCM_FAIL(-1, "ocm_copy_out: NULL argument");
    if (wait_alloc(src) != 0) return -1;
    const Loc dl = pointer_loc(dst);
    if (src->remote) return xfer(src, false, static_cast<char *>(dst), dl, 0, src->remote_bytes, false);
    return copy_local(dst, dl, src->local, src->loc, src->local_bytes);
}

int ocm_remote_info(ocm_alloc_t a, struct ocm_remote_info *info) {
    if (!a || !info) return -1;
    std::memset(info, 0, sizeof(*info));
    info->alloc_id = a->alloc_id;
    info->remote_bytes = a->remote_bytes;
    info->stripe_unit = a->stripe_unit;
    info->n_extents = (uint32_t)a->ext.size();
    for (size_t i = 0; i < a->ext.size() && i < OCM_MAX_EXTENTS; i++) {
        info->tier[i] = a->ext[i].r.tier;
        info->owner_rank[i] = a->ext[i].r.owner_rank;
        info->owner_gpu[i] = a->ext[i].r.owner_gpu;
        info->extent_bytes[i] = a->ext[i].r.bytes;
        if (a->ext[i].net) info->net_mask |= 1u << i;
    }
    return a->remote ? 0 : -1;
}

// Raw 64-byte handle of extent i (tests: the network tier's capability checks).
int ocm_x_extent_handle(ocm_alloc_t a, int i, uint8_t *out) {
    if (!a || !out || i < 0 || (size_t)i >= a->ext.size()) return -1;
    std::memcpy(out, a->ext[(size_t)i].r.handle, kHandleBytes);
    return 0;
}

// Layout of the app's shared-memory link (ocm/shmlink.h), for tests that drive a
// link by hand: {mapped bytes, req_taken, rsp_taken, daemon_polling, app_waiting,
// req[0], rsp[0], slot bytes, seq offset in a slot, slots, magic}.
void ocm_x_link_layout(uint64_t out[11]) {
    out[0] = ((uint64_t)sizeof(ShmLinkLayout) + 4095) & ~4095ull;
    out[1] = offsetof(ShmLinkLayout, req_taken);
    out[2] = offsetof(ShmLinkLayout, rsp_taken);
    out[3] = offsetof(ShmLinkLayout, daemon_polling);
    out[4] = offsetof(ShmLinkLayout, app_waiting);
    out[5] = offsetof(ShmLinkLayout, req);
    out[6] = offsetof(ShmLinkLayout, rsp);
    out[7] = sizeof(ShmLinkSlot);
    out[8] = offsetof(ShmLinkSlot, seq);
    out[9] = kShmLinkSlots;
    out[10] = kShmLinkMagic;
}

// xGMI self-diagnosis of this process: {device, peers with access enabled,
// other GPUs' HBM slabs imported, such imports refused, push-get launches}.
void ocm_x_xgmi_diag(uint64_t out[5]) {
    State &s = S();
    std::lock_guard<std::recursive_mutex> lk(s.mu);
    out[0] = (uint64_t)(int64_t)s.device;
    out[1] = (uint64_t)s.peers_enabled;
    out[2] = s.ipc_peer_imports;
    out[3] = s.ipc_peer_failures;
    out[4] = s.push_launches;
}

// Where extent i lives inside its owner's slab: {offset in the slab, extent
// bytes, slab bytes, owner GPU (-1: host tier)}. With ocm_x_extent_handle, a
// process on the OWNER's GPU can map the same bytes (tests: owner-side kernels).
int ocm_x_extent_region(ocm_alloc_t a, int i, uint64_t out[4]) {
    if (!a || !out || i < 0 || (size_t)i >= a->ext.size()) return -1;
    const Region &r = a->ext[(size_t)i].r;
    out[0] = r.offset;
    out[1] = r.bytes;
    out[2] = r.slab_bytes;
    out[3] = (uint64_t)(int64_t)r.owner_gpu;
    return 0;
}

// Owner-side helpers that need no ocm_init (a verifier process on the owner's
// GPU): open an exported HBM slab on `device`, and fill / check the word
// pattern there with the same gfx950 kernels on that device's null stream.
int ocm_x_ipc_open(int device, const uint8_t *handle, void **out) {
    if (!handle || !out || hipSetDevice(device) != hipSuccess) return -1;
    hipIpcMemHandle_t h;
    std::memcpy(&h, handle, sizeof(h));
    if (hipIpcOpenMemHandle(out, h, hipIpcMemLazyEnablePeerAccess) != hipSuccess) {
        (void)hipGetLastError();
        return -1;
    }
    return 0;
}

int ocm_x_ipc_close(int device, void *p) {
    if (hipSetDevice(device) != hipSuccess) return -1;
    return hipIpcCloseMemHandle(p) == hipSuccess ? 0 : -1;
}

long long ocm_x_pattern_dev(int device, void *p, uint64_t words, uint64_t first, uint32_t seed, int check) {
    if (!p || hipSetDevice(device) != hipSuccess) return -1;
    unsigned long long *bad_dev = nullptr, bad = 0;
    hipError_t e = hipSuccess;
    if (check) {
        e = hipMalloc(reinterpret_cast<void **>(&bad_dev), sizeof(bad));
        if (e == hipSuccess) e = hipMemset(bad_dev, 0, sizeof(bad));
        if (e == hipSuccess) e = pattern_check(p, words, first, seed, bad_dev, nullptr);
        if (e == hipSuccess) e = hipMemcpy(&bad, bad_dev, sizeof(bad), hipMemcpyDeviceToHost);
        if (bad_dev) (void)hipFree(bad_dev);
    } else {
        e = pattern_fill(p, words, first, seed, nullptr);
        if (e == hipSuccess) e = hipDeviceSynchronize();
    }
    if (e != hipSuccess) {
        (void)hipGetLastError();
        return -1;
    }
    return (long long)bad;
}

void *ocm_remotebuf(ocm_alloc_t a) {
    if (!a || a->ext.size() != 1 || a->ext[0].net) return nullptr;
    return S().device >= 0 ? a->ext[0].dptr : a->ext[0].hptr;
}

int ocm_stats(int rank, struct ocm_daemon_stats *out) {
    State &s = S();
    std::lock_guard<std::recursive_mutex> lk(s.mu);
    if (!s.inited || !out) return -1;
    Msg m = new_msg(MSG_STATS);
    m.u.req.remote_rank = rank;
    Msg r;
    if (rpc(m, &r, s.rpc_timeout_ms) != 0) return -1;
    if (r.err) OCM_FAIL(-1, "stats from rank %d: %s", rank, strerror(r.err));
    const NodeConfig &c = r.u.node;
    std::memset(out, 0, sizeof(*out));
    out->rank = c.rank;
    out->gpu = c.gpu;
    out->num_nodes = (int32_t)c.num_nodes;
    out->num_apps = (int32_t)c.num_apps;
    out->gpu_capacity = c.gpu_capacity;
    out->gpu_used = c.gpu_used;
    out->host_capacity = c.host_capacity;
    out->host_used = c.host_used;
    out->n_alloc = c.n_alloc;
    out->n_free = c.n_free;
    out->n_reclaimed = c.n_reclaimed;
    out->n_spilled = c.n_spilled;
    out->n_slabs = c.n_slabs;
    out->ctrl_ticks = c.ticks;
    out->n_leases = c.n_leases;
    out->lease_allocs = c.lease_allocs;
    out->xgmi_peers = c.xgmi_peers;
    out->min_hops = c.min_hops;
    out->max_hops = c.max_hops;
    out->ctrl_transport = c.ctrl;
    return 0;
}

int ocm_rank(void) { return S().inited ? S().daemon_rank : -1; }
int ocm_num_nodes(void) { return S().inited ? (int)S().daemon.num_nodes : -1; }
int ocm_device(void) { return S().inited ? S().device : -1; }
const char *ocm_last_error(void) { return last_error(); }

// ---------------- internal hooks for tests and benchmarks (not part of the ABI) ----------------

// Per-process operation counters (see ocm/trace.h): 17 x uint64.
void ocm_x_counters(uint64_t out[21]) {
    const OpCounters &c = S().ctr;
    const uint64_t v[21] = {c.n_put,  c.n_get,    c.bytes_put, c.bytes_get,   c.n_alloc,     c.n_free,
                            c.n_copy, c.bytes_copy, c.ns_put,  c.ns_get,      c.ns_alloc,    c.ns_free,
                            c.n_batch, c.n_batch_ops, c.bytes_batch, c.ns_batch, c.n_batch_launches,
                            c.n_slab_fd, c.n_slab_path, c.n_link_rpc, c.n_link_wake};
    std::memcpy(out, v, sizeof(v));
}

// Fused Adam over optimizer state kept in the remote half of `a` (see
// ocm/optim.h): p/g are this GPU's parameters and gradients (n floats),
// exp_avg / exp_avg_sq of element 0 sit at byte offsets m_off / v_off of the
// remote half. hp = {b1, b2, eps, weight_decay, step_size, 1/sqrt(bias_correction2),
// adamw_decay}: adamw_decay = 1 - lr * weight_decay selects AdamW (decoupled decay;
// weight_decay then unused), NaN selects Adam with the L2 term.
// Queued on `stream` (e.g. torch's current stream); no host wait.
static int adam_common(ocm_alloc_t a, void *p, const void *g, uint64_t n, uint64_t w_off, uint64_t m_off,
                       uint64_t v_off, const float hp[7], void *stream, bool bf16);

int ocm_x_adam(ocm_alloc_t a, float *p, const float *g, uint64_t n, uint64_t m_off, uint64_t v_off,
               const float hp[7], void *stream) {
    return adam_common(a, p, g, n, 0, m_off, v_off, hp, stream, false);
}

// Mixed precision: p / g are bf16 on this GPU, the fp32 master weights sit at
// byte offset w_off of the remote half next to the moments.
int ocm_x_adam_bf16(ocm_alloc_t a, void *p, const void *g, uint64_t n, uint64_t w_off, uint64_t m_off,
                    uint64_t v_off, const float hp[7], void *stream) {
    return adam_common(a, p, g, n, w_off, m_off, v_off, hp, stream, true);
}

// Many parameters per launch (32 per kernel, descriptors in the kernarg
// segment): p[i] / g[i] of n[i] elements, state at w_off[i] (bf16 only),
// m_off[i], v_off[i] of the remote half. Same hp as ocm_x_adam.
int ocm_x_adam_multi(ocm_alloc_t a, int count, void *const *p, const void *const *g, const uint64_t *n,
                     const uint64_t *w_off, const uint64_t *m_off, const uint64_t *v_off, const float hp[7],
                     int bf16, void *stream) {
    State &s = S();
    if (!a || count < 0 || (count && (!p || !g || !n || !m_off || !v_off || (bf16 && !w_off))) || !hp)
        OCM_FAIL(-1, "ocm_x_adam_multi: null argument");
    if (s.device < 0) OCM_FAIL(-1, "ocm_x_adam_multi needs a GPU");
    if (!is_pair(a->kind) || a->ext.empty() || !a->all_dev_ok || a->ext.size() > (size_t)kXferMaxExtents)
        OCM_FAIL(-1, "ocm_x_adam_multi needs a remote half this GPU can address");
    const uint64_t rb = a->remote_bytes;
    auto fits = [rb](uint64_t off, uint64_t len) { return off <= rb && len <= rb - off; };
    AdamMultiArgs x;
    std::memset(&x, 0, sizeof(x));
    for (size_t i = 0; i < a->ext.size(); i++) x.c.ext[i] = a->ext[i].dptr;
    x.c.n_ext = (uint32_t)a->ext.size();
    if (x.c.n_ext > 1) {
        const int sh = log2_exact(a->stripe_unit);
        if (sh < 4) OCM_FAIL(-1, "ocm_x_adam_multi: stripe unit unusable");
        x.c.unit_shift = (uint32_t)sh;
    }
    x.c.b1 = hp[0];
    x.c.b2 = hp[1];
    x.c.eps = hp[2];
    x.c.wd = hp[3];
    x.c.step_size = hp[4];
    x.c.inv_sqrt_bc2 = hp[5];
    x.c.decoupled = std::isnan(hp[6]) ? 0u : 1u;  // NaN: L2 Adam; else AdamW's weight multiplier
    x.c.decay = hp[6];
    x.c.host_state = (!a->any_gpu && !a->any_net) ? 1u : 0u;
    x.c.bf16 = bf16 ? 1u : 0u;
    // Every tensor is checked before the first launch: a bad one never leaves
    // some parameters a step ahead of the others.
    for (int i = 0; i < count; i++) {
        if (!p[i] || !g[i]) OCM_FAIL(-1, "ocm_x_adam_multi: tensor %d has no data", i);
        if (n[i] > (UINT64_MAX >> 3) || !fits(m_off[i], 4 * n[i]) || !fits(v_off[i], 4 * n[i]) ||
            (bf16 && !fits(w_off[i], 4 * n[i])))
            OCM_FAIL(-1, "ocm_x_adam_multi: tensor %d state range exceeds the remote half", i);
    }
    std::lock_guard<std::recursive_mutex> lk(s.mu);
    if (wait_alloc(a) != 0) return -1;
    DeviceGuard dg(s.device);
    before_launch();
    for (int k0 = 0; k0 < count; k0 += kAdamMaxTensors) {
        x.count = (uint32_t)std::min(count - k0, kAdamMaxTensors);
        for (uint32_t j = 0; j < x.count; j++) {
            const int i = k0 + (int)j;
            x.t[j] = AdamTensor{p[i], g[i], n[i], bf16 ? w_off[i] : 0, m_off[i], v_off[i]};
        }
        const hipError_t e = adam_remote_multi_launch(x, static_cast<hipStream_t>(stream));
        if (e != hipSuccess) OCM_FAIL(-1, "ocm_x_adam_multi launch: %s", hipGetErrorString(e));
    }
    return 0;
}

static int adam_common(ocm_alloc_t a, void *p, const void *g, uint64_t n, uint64_t w_off, uint64_t m_off,
                       uint64_t v_off, const float hp[7], void *stream, bool bf16) {
    State &s = S();
    if (!a || !p || !g || !hp) OCM_FAIL(-1, "ocm_x_adam: null argument");
    if (s.device < 0) OCM_FAIL(-1, "ocm_x_adam needs a GPU");
    if (!is_pair(a->kind) || a->ext.empty() || !a->all_dev_ok)
        OCM_FAIL(-1, "ocm_x_adam needs a remote half this GPU can address (HBM or host tier, not another node)");
    if (n > (UINT64_MAX >> 3) || m_off > a->remote_bytes || 4 * n > a->remote_bytes - m_off ||
        v_off > a->remote_bytes || 4 * n > a->remote_bytes - v_off ||
        (bf16 && (w_off > a->remote_bytes || 4 * n > a->remote_bytes - w_off)))
        OCM_FAIL(-1, "ocm_x_adam: state range exceeds the remote half (%zu bytes)", a->remote_bytes);
    if (a->ext.size() > (size_t)kXferMaxExtents) OCM_FAIL(-1, "ocm_x_adam: too many extents");
    AdamArgs x;
    std::memset(&x, 0, sizeof(x));
    x.p = static_cast<float *>(p);
    x.g = static_cast<const float *>(g);
    x.bf16 = bf16 ? 1u : 0u;
    x.w_off = w_off;
    for (size_t i = 0; i < a->ext.size(); i++) x.ext[i] = a->ext[i].dptr;
    x.n_ext = (uint32_t)a->ext.size();
    if (x.n_ext > 1) {
        const int sh = log2_exact(a->stripe_unit);
        if (sh < 4) OCM_FAIL(-1, "ocm_x_adam: stripe unit %llu unusable", (unsigned long long)a->stripe_unit);
        x.unit_shift = (uint32_t)sh;
    }
    x.m_off = m_off;
    x.v_off = v_off;
    x.n = n;
    x.b1 = hp[0];
    x.b2 = hp[1];
    x.eps = hp[2];
    x.wd = hp[3];
    x.step_size = hp[4];
    x.inv_sqrt_bc2 = hp[5];
    x.decoupled = std::isnan(hp[6]) ? 0u : 1u;
    x.decay = hp[6];
    x.host_state = (!a->any_gpu && !a->any_net) ? 1u : 0u;
    std::lock_guard<std::recursive_mutex> lk(s.mu);
    if (wait_alloc(a) != 0) return -1;  // queued async ops on this allocation come first
    DeviceGuard dg(s.device);
    before_launch();
    const hipError_t e = adam_remote_launch(x, static_cast<hipStream_t>(stream));
    if (e != hipSuccess) OCM_FAIL(-1, "ocm_x_adam launch: %s", hipGetErrorString(e));
    return 0;
}

// Park the resident copy service now. A device-wide synchronize
// (hipDeviceSynchronize, torch.cuda.synchronize) waits for every stream,
// including the service's persistent kernel, which otherwise leaves by itself
// after OCM_SERVICE_IDLE_US (50 us) without work; the next small op relaunches it.
// Optional: only callers that cannot afford those microseconds need it.
void ocm_x_quiesce(void) {
    State &s = S();
    std::lock_guard<std::recursive_mutex> lk(s.mu);
    service_park();
}

// The local daemon's tick control transport statistics (TickStatsWire as 16
// words: ticks, own records, latency sum / max ns, periods, period sum ns,
// start() calls, their sum / max ns, transport | ticks_per_start << 32, then the
// hop breakdown: wait sum ns, exec sum ns, deliver sum ns, deliveries, idle ticks,
// TCP wake-ups sent).
int ocm_x_tick_stats(uint64_t out[16]) {
    State &s = S();
    std::lock_guard<std::recursive_mutex> lk(s.mu);
    if (!s.inited || !out) return -1;
    Msg m = new_msg(MSG_TICK_STATS);
    Msg r;
    if (rpc(m, &r, s.rpc_timeout_ms) != 0) return -1;
    TickStatsWire st;
    std::memcpy(&st, r.u.raw, sizeof(st));
    const uint64_t v[16] = {st.ticks, st.own_records, st.lat_sum_ns, st.lat_max_ns, st.periods, st.period_sum_ns,
                            st.starts, st.start_sum_ns, st.start_max_ns,
                            (uint64_t)st.transport | ((uint64_t)st.ticks_per_start << 32),
                            st.wait_sum_ns, st.exec_sum_ns, st.deliver_sum_ns, st.deliver_n, st.lazy_ticks,
                            st.tcp_wakes};
    std::memcpy(out, v, sizeof(v));
    return 0;
}

// Copy-service diagnostics: {ops, ns posting requests, ns waiting for done,
// GPU ticks (100 MHz) from doorbell seen to done published, relaunches after an
// idle exit}. The doorbell record stays in host memory (a BAR-mapped HBM record
// measured slower: profiles/svc_doorbell_hbm_ab_r02.json).
void ocm_x_service_stats(uint64_t out[5]) {
    State &s = S();
    std::lock_guard<std::recursive_mutex> lk(s.mu);
    out[0] = s.svc_ops;
    out[1] = s.svc_ns_post;
    out[2] = s.svc_ns_wait;
    out[3] = s.svc_gpu_ticks_done + (s.svc ? __atomic_load_n(&s.svc->gpu_ticks, __ATOMIC_ACQUIRE) : 0);
    out[4] = s.svc_relaunches;  // instances started because the previous one left idle
}

// Copy-service health: {gang ops sized below their wanted width because fewer
// members were resident, instances that left with the posted op unfinished,
// ops abandoned after OCM_SERVICE_TIMEOUT_MS (drained, then redone by a launch),
// 1 if an instance could not be drained (service off, op failed), the smallest
// roster a gang op was sized to (0: none yet), the current instance's roster,
// relaunches after an idle exit, and the host ns they took (reap + launch), then
// over every start: ns choosing a lane, ns in the launch call, starts}.
// Then: 1 if the lanes are AQL queues of the library's own (0: HIP streams),
// gang ops that replaced a lone lead with a full instance, 1 if the running
// instance's lead is alone (its members left), and the lanes created.
// Then the longest wait for a lane to drain (ns) and where it happened
// (1 lane pick at a start, 2 park, 3 shutdown, 4 abort, 5 re-post after an exit),
// the instances dispatched beside a previous lead that had not left yet, and 1
// while an instance is resident (started and not yet left), and 1 + the XCD of
// the running instance's lead (0: unknown).
void ocm_x_service_health(uint64_t out[19]) {
    State &s = S();
    std::lock_guard<std::recursive_mutex> lk(s.mu);
    const bool run = s.svc && s.svc_running;
    out[0] = s.svc_degraded;
    out[1] = s.svc_incomplete_exits;
    out[2] = s.svc_aborts;
    out[3] = s.svc_wedged ? 1 : 0;
    out[4] = s.svc_roster_min == ~0ull ? 0 : s.svc_roster_min;
    out[5] = run ? service_untag(s.svc_epoch, __atomic_load_n(&s.svc->roster, __ATOMIC_ACQUIRE)) : 0;
    out[6] = s.svc_relaunches;
    out[7] = s.svc_ns_relaunch;
    out[8] = s.svc_ns_pick;
    out[9] = s.svc_ns_launch;
    out[10] = s.svc_epoch_starts;
    out[11] = s.svc_aql ? 1 : 0;
    out[12] = s.svc_promotions;
    out[13] = (run && service_untag(s.svc_epoch, __atomic_load_n(&s.svc->lone, __ATOMIC_ACQUIRE)) != 0) ? 1 : 0;
    out[14] = s.svc_drain_max_ns;
    out[15] = s.svc_drain_max_site;
    out[16] = s.svc_overlaps;
    out[17] = (run && service_untag(s.svc_epoch, __atomic_load_n(&s.svc->exited, __ATOMIC_ACQUIRE)) == 0) ? 1 : 0;
    out[18] = run ? service_untag(s.svc_epoch, __atomic_load_n(&s.svc->lead_xcd, __ATOMIC_ACQUIRE)) : 0;
}

// Copy-service phase stamps of the last request (OCM_SERVICE_PROTO with the
// TRACE bit): 4 GPU-clock words per workgroup for the first n workgroups.
int ocm_x_service_trace(uint64_t *out, int n_wgs) {
    State &s = S();
    std::lock_guard<std::recursive_mutex> lk(s.mu);
    if (!s.svc_box || n_wgs < 1 || n_wgs > kServiceTraceWgs) return -1;
    DeviceGuard g(s.device);
    if (hipMemcpy(out, s.svc_box->trace, (size_t)n_wgs * 4 * sizeof(uint64_t), hipMemcpyDeviceToHost) != hipSuccess) {
        (void)hipGetLastError();
        return -1;
    }
    return 0;
}

// Host addresses behind the copy service's hand-off (diagnostics: which NUMA node
// holds them): the request record pages, the status slot, and extent 0's host
// mapping of `a` (0 where there is none).
int ocm_x_service_pages(ocm_alloc_t a, uint64_t out[3]) {
    State &s = S();
    std::lock_guard<std::recursive_mutex> lk(s.mu);
    out[0] = reinterpret_cast<uint64_t>(s.svc_rec_pages);
    out[1] = reinterpret_cast<uint64_t>(s.svc);
    out[2] = (a && !a->ext.empty()) ? reinterpret_cast<uint64_t>(a->ext[0].hptr) : 0;
    return s.svc ? 0 : -1;
}

// Transfer tuning at runtime (benchmarks): variant 0 auto / 1 reg / 2 lds,
// blocks 0 = per-path default, nt = nontemporal destination stores.
void ocm_x_set_tuning(int variant, int blocks, int nt) {
    State &s = S();
    std::lock_guard<std::recursive_mutex> lk(s.mu);
    s.tuning.variant = variant;
    s.tuning.max_blocks = blocks;
    s.tuning.nontemporal = nt != 0;
    s.tuning.write_through = nt == 2;
    s.dir_tuning[0] = s.dir_tuning[1] = XferTuning{};
}

// Per-direction override of one-sided kernel ops (dir 0 get, 1 put), e.g. the
// winner of an autotune over the xGMI links; variant 0 clears it.
int ocm_x_set_tuning_dir(int dir, int variant, int blocks, int nt) {
    if (dir != 0 && dir != 1) return -1;
    if (variant < XFER_AUTO || variant > XFER_PUSH || blocks < 0) return -1;
    State &s = S();
    std::lock_guard<std::recursive_mutex> lk(s.mu);
    XferTuning t;
    t.variant = variant;
    t.max_blocks = blocks;
    t.nontemporal = nt != 0;
    t.write_through = nt == 2;  // 2: sc1 loads and stores (register kernel)
    s.dir_tuning[dir] = t;
    return 0;
}

// Link type (hipExtLinkType) and hop count between two devices; -1 on error.
int ocm_x_link_info(int dev, int peer, uint32_t *type, uint32_t *hops) {
    if (hipExtGetLinkTypeAndHopCount(dev, peer, type, hops) != hipSuccess) {
        (void)hipGetLastError();
        return -1;
    }
    return 0;
}

void ocm_x_layout(uint64_t out[8]) {
    out[0] = sizeof(Msg);
    out[1] = sizeof(struct ocm_params);
    out[2] = sizeof(struct ocm_alloc_params);
    out[3] = offsetof(Msg, u);
    out[4] = sizeof(Region);
    out[5] = sizeof(NodeConfig);
    out[6] = sizeof(AllocReq);
    out[7] = kHandleBytes;
}

// Striped transfer between raw device pointers on `device` (kernel numerics tests).
int ocm_x_xfer(int device, void *lin, void **ext, int n_ext, uint64_t unit, uint64_t rem_off, uint64_t len, int put,
               int variant, int blocks, int sync) {
    if (n_ext < 1 || n_ext > kXferMaxExtents) return -1;
    DeviceGuard g(device);
    XferArgs x;
    std::memset(&x, 0, sizeof(x));
    x.lin = static_cast<char *>(lin);
    for (int i = 0; i < n_ext; i++) x.ext[i] = static_cast<char *>(ext[i]);
    x.n_ext = (uint32_t)n_ext;
    x.rem_off = rem_off;
    x.len = len;
    x.put = (uint32_t)put;
    if (n_ext > 1) {
        int sh = log2_exact(unit);
        if (sh < 4) return -1;
        x.unit_shift = (uint32_t)sh;
    }
    XferTuning t = xfer_tuning_from_env();
    if (variant) t.variant = variant;
    if (blocks) t.max_blocks = blocks;
    if (t.variant == XFER_PUSH && !put) {
        // the push-get kernel, every extent in the mask (numerics tests); the
        // same kernel a push get launches on each owner's GPU
        const uint32_t all = (uint32_t)((1ull << n_ext) - 1);
        if (xfer_push_launch(x, all, blocks, nullptr) != hipSuccess) return -1;
    } else if (xfer_launch(x, t, nullptr) != hipSuccess) {
        return -1;
    }
    if (!sync) return 0;  // caller orders it on the null stream
    return hipDeviceSynchronize() == hipSuccess ? 0 : -1;
}

// Batched transfer between raw device pointers (kernel numerics tests / PMC
// profiles without daemons). ops: n x {lin_off, rem_off, len, put} (u64 each).
// Returns 0, or -1 on bad arguments; iters > 1 repeats the launch (profiling).
int ocm_x_batch(int device, void *lin, void **ext, int n_ext, uint64_t unit, const uint64_t *ops, int n_ops, int iters) {
    if (n_ext < 1 || n_ext > kXferMaxExtents || n_ops < 1 || !ops) return -1;
    DeviceGuard g(device);
    XferBatchArgs args;
    std::memset(&args, 0, sizeof(args));
    args.lin = static_cast<char *>(lin);
    for (int i = 0; i < n_ext; i++) args.ext[i] = static_cast<char *>(ext[i]);
    args.n_ext = (uint32_t)n_ext;
    if (n_ext > 1) {
        const int sh = log2_exact(unit);
        if (sh < 4) return -1;
        args.unit_shift = (uint32_t)sh;
    }
    args.tile_shift = xfer_batch_tile_shift(args.n_ext, args.unit_shift);
    std::vector<XferBatchOp> v((size_t)n_ops);
    for (int i = 0; i < n_ops; i++) {
        v[i].lin_off = ops[4 * i];
        v[i].rem_off = ops[4 * i + 1];
        v[i].len = ops[4 * i + 2];
        v[i].put = ops[4 * i + 3] != 0;
    }
    args.n_ops = (uint32_t)n_ops;
    args.total_tiles = xfer_batch_plan(v.data(), (uint32_t)n_ops, args.tile_shift);
    if (!args.total_tiles) return 0;
    args.grid = xfer_batch_grid(args.total_tiles);
    void *dev = nullptr;
    if (n_ops <= kXferInlineOps) {
        std::memcpy(args.inline_ops, v.data(), v.size() * sizeof(XferBatchOp));
    } else {
        const size_t dbytes = v.size() * sizeof(XferBatchOp), need = dbytes + (size_t)args.grid * 16;
        std::vector<char> up(need);
        std::memcpy(up.data(), v.data(), dbytes);
        xfer_batch_wave_ops(v.data(), (uint32_t)n_ops, args.total_tiles, args.grid,
                            reinterpret_cast<uint32_t *>(up.data() + dbytes));
        if (hipMalloc(&dev, need) != hipSuccess || hipMemcpy(dev, up.data(), need, hipMemcpyHostToDevice) != hipSuccess)
            return -1;
        args.ops = static_cast<const XferBatchOp *>(dev);
        args.wave_op = reinterpret_cast<const uint32_t *>(static_cast<char *>(dev) + dbytes);
    }
    XferTuning t = xfer_tuning_from_env();
    int rc = 0;
    for (int k = 0; k < std::max(1, iters) && rc == 0; k++)
        rc = xfer_batch_launch(args, t, nullptr) == hipSuccess ? 0 : -1;
    if (hipDeviceSynchronize() != hipSuccess) rc = -1;
    if (dev) (void)hipFree(dev);
    return rc;
}

// Time `iters` back-to-back device copies (seconds per copy, event-timed).
double ocm_x_time_device_copy(int device, void *dst, const void *src, uint64_t bytes, int variant, int blocks,
                              int nt, int iters) {
    DeviceGuard g(device);
    XferTuning t;
    t.variant = variant;
    t.max_blocks = blocks;
    t.nontemporal = nt != 0;
    t.write_through = nt == 2;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)xfer_copy(dst, src, bytes, t, nullptr);  // warm
    (void)hipEventRecord(e0, nullptr);
    for (int i = 0; i < iters; i++) (void)xfer_copy(dst, src, bytes, t, nullptr);
    (void)hipEventRecord(e1, nullptr);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    return (double)ms / 1e3 / (iters > 0 ? iters : 1);
}

// Wall-clock seconds per blocking one-sided op, measured inside the library
// (no Python in the loop): the sweep primitive of bench.py.
// Per-sample wall time (seconds) of ocm_alloc_ex and the matching ocm_free,
// timed in C so callers (bench.py) report the API's latency, not their FFI's.
// Returns the number of samples taken (< samples on the first failure).
int ocm_x_alloc_latency(ocm_alloc_param_t ap, const struct ocm_alloc_ex_params *ex, int samples, double *alloc_s,
                        double *free_s) {
    for (int i = 0; i < samples; i++) {
        struct timespec t0, t1, t2;
        clock_gettime(CLOCK_MONOTONIC, &t0);
        ocm_alloc_t a = ocm_alloc_ex(ap, ex);
        clock_gettime(CLOCK_MONOTONIC, &t1);
        if (!a) return i;
        const int rc = ocm_free(a);
        clock_gettime(CLOCK_MONOTONIC, &t2);
        if (rc != 0) return i;
        alloc_s[i] = (double)(t1.tv_sec - t0.tv_sec) + (double)(t1.tv_nsec - t0.tv_nsec) * 1e-9;
        free_s[i] = (double)(t2.tv_sec - t1.tv_sec) + (double)(t2.tv_nsec - t1.tv_nsec) * 1e-9;
    }
    return samples;
}

double ocm_x_time_onesided(ocm_alloc_t a, ocm_param_t p, int iters) {
    struct timespec t0, t1;
    clock_gettime(CLOCK_MONOTONIC, &t0);
    for (int i = 0; i < iters; i++)
        if (ocm_copy_onesided(a, p) != 0) return -1.0;
    clock_gettime(CLOCK_MONOTONIC, &t1);
    double dt = (double)(t1.tv_sec - t0.tv_sec) + (double)(t1.tv_nsec - t0.tv_nsec) * 1e-9;
    return dt / (iters > 0 ? iters : 1);
}

// Per-op samples of a blocking one-sided op, each timed on its own: up to
// `iters` ops, stopping early once `cap_ns` have passed (at least `min_iters`
// ops). Before each op the calling thread stays busy for `gap_ns` without
// touching the library (an application computing between small ops), so the
// samples include whatever an idle gap costs the next op (the copy service's
// idle exit and relaunch). out[i] = seconds of op i; *relaunches = copy-service
// relaunches during the run. Returns the number of samples, -1 on an op failure.
int ocm_x_time_onesided_samples(ocm_alloc_t a, ocm_param_t p, int iters, int min_iters, uint64_t gap_ns,
                                uint64_t cap_ns, double *out, uint64_t *relaunches) {
    auto ns = []() {
        struct timespec t;
        clock_gettime(CLOCK_MONOTONIC, &t);
        return (uint64_t)t.tv_sec * 1000000000ull + (uint64_t)t.tv_nsec;
    };
    uint64_t r0 = 0;
    {
        std::lock_guard<std::recursive_mutex> lk(S().mu);
        r0 = S().svc_relaunches;
    }
    const uint64_t start = ns();
    int n = 0;
    for (; n < iters; n++) {
        if (n >= min_iters && ns() - start > cap_ns) break;
        if (gap_ns) {
            const uint64_t g0 = ns();
            while (ns() - g0 < gap_ns) __builtin_ia32_pause();
        }
        const uint64_t t0 = ns();
        if (ocm_copy_onesided(a, p) != 0) return -1;
        out[n] = (double)(ns() - t0) * 1e-9;
    }
    if (relaunches) {
        std::lock_guard<std::recursive_mutex> lk(S().mu);
        *relaunches = S().svc_relaunches - r0;
    }
    return n;
}

// Fill / check the deterministic word pattern on device or host memory.
// `words` 32-bit words starting at pattern index `first`; returns mismatches (check) or 0 / -1.
long long ocm_x_pattern(void *p, uint64_t words, uint64_t first, uint32_t seed, int check) {
    State &s = S();
    Loc l = pointer_loc(p);
    if (s.device < 0 || l == LOC_HOST) {
        uint32_t *w = static_cast<uint32_t *>(p);
        long long bad = 0;
        for (uint64_t i = 0; i < words; i++) {
            if (check)
                bad += w[i] != pattern_word_host(first + i, seed);
            else
                w[i] = pattern_word_host(first + i, seed);
        }
        return bad;
    }
    std::lock_guard<std::recursive_mutex> lk(s.mu);  // the library stream and its event are shared
    DeviceGuard g(s.device);
    if (!check) {
        if (pattern_fill(p, words, first, seed, s.stream) != hipSuccess) return -1;
        return sync_stream() == 0 ? 0 : -1;
    }
    // One counter kept for the process: hipFree synchronizes the whole device,
    // which would also wait for the resident copy service's idle exit.
    if (!s.pattern_bad && hipMalloc(reinterpret_cast<void **>(&s.pattern_bad), sizeof(unsigned long long)) != hipSuccess) {
        s.pattern_bad = nullptr;
        return -1;
    }
    unsigned long long bad = 0;
    (void)hipMemsetAsync(s.pattern_bad, 0, sizeof(bad), s.stream);
    hipError_t e = pattern_check(p, words, first, seed, s.pattern_bad, s.stream);
    if (e == hipSuccess) e = hipMemcpyAsync(&bad, s.pattern_bad, sizeof(bad), hipMemcpyDeviceToHost, s.stream);
    int rc = sync_stream();
    return (e == hipSuccess && rc == 0) ? (long long)bad : -1;
}

// ---- PyTorch pluggable allocator: tensors in disaggregated memory ----
// torch.cuda.memory.CUDAPluggableAllocator(libocm.so, "ocm_torch_alloc",
// "ocm_torch_free") behind a torch.cuda.MemPool (oncilla_amd.torch_pool): each
// block torch's caching allocator asks for is the remote half of a pair with
// no local half, one extent (a tensor needs contiguous addresses), in another
// daemon's HBM (or its pinned host tier) and addressed in place over xGMI.
// torch caches the blocks; a block comes back here only when torch releases it.
}  // extern "C"

namespace {
struct TorchPool {
    std::mutex mu;
    std::map<void *, ocm_alloc_t> live;
    struct ocm_alloc_ex_params ex = {-1, 0, 1, 0, 0};  // any owner, single extent
    uint64_t bytes = 0;
};
TorchPool &torch_pool() {
    static TorchPool *p = new TorchPool();  // never destroyed: torch may free at exit
    return *p;
}
}  // namespace

extern "C" {

// remote_rank -1: rank0 places; flags: enum ocm_alloc_flags (e.g. OCM_ALLOC_HOST_TIER).
void ocm_x_torch_pool_config(int remote_rank, uint32_t flags) {
    TorchPool &tp = torch_pool();
    std::lock_guard<std::mutex> lk(tp.mu);
    tp.ex.remote_rank = remote_rank;
    tp.ex.flags = flags & ~(uint32_t)OCM_ALLOC_STRIPE;  // one extent: contiguous addresses
    tp.ex.stripe_width = 1;
}

void *ocm_torch_alloc(ssize_t size, int device, void *stream) {
    (void)stream;  // the memory is ready when the owner answers; torch orders its reuse
    State &s = S();
    if (size <= 0 || !s.inited || s.device < 0 || device != s.device) return nullptr;  // torch reports the OOM
    TorchPool &tp = torch_pool();
    struct ocm_alloc_ex_params ex;
    {
        std::lock_guard<std::mutex> lk(tp.mu);
        ex = tp.ex;
    }
    struct ocm_alloc_params p = {0, (uint64_t)size, OCM_REMOTE_GPU};
    ocm_alloc_t a = ocm_alloc_ex(&p, &ex);
    if (!a) return nullptr;
    void *ptr = ocm_remotebuf(a);
    if (!ptr) {
        ocm_free(a);
        return nullptr;
    }
    std::lock_guard<std::mutex> lk(tp.mu);
    tp.live[ptr] = a;
    tp.bytes += (uint64_t)size;
    return ptr;
}

void ocm_torch_free(void *ptr, ssize_t size, int device, void *stream) {
    (void)device;
    (void)stream;
    TorchPool &tp = torch_pool();
    ocm_alloc_t a = nullptr;
    {
        std::lock_guard<std::mutex> lk(tp.mu);
        auto it = tp.live.find(ptr);
        if (it == tp.live.end()) return;
        a = it->second;
        tp.live.erase(it);
        tp.bytes -= std::min<uint64_t>(tp.bytes, (uint64_t)(size > 0 ? size : 0));
    }
    State &s = S();
    if (!s.inited) return;
    {
        // hipFree semantics: kernels still reading or writing the block finish
        // before its bytes go back to the owner (which may hand them out again).
        // Park the copy service first and hold the lock across the sync, so no
        // other thread relaunches it in between and the wait stays bounded.
        std::lock_guard<std::recursive_mutex> lk(s.mu);
        service_park();
        DeviceGuard g(s.device);
        if (hipDeviceSynchronize() != hipSuccess) (void)hipGetLastError();
    }
    ocm_free(a);
}

// {blocks held by torch, their bytes}
void ocm_x_torch_pool_stats(uint64_t out[2]) {
    TorchPool &tp = torch_pool();
    std::lock_guard<std::mutex> lk(tp.mu);
    out[0] = tp.live.size();
    out[1] = tp.bytes;
}

}  // extern "C"

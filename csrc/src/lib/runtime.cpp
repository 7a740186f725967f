// libocm process state, mailbox RPC to the local ocmd, the import cache of
// remote extents (hipIpcOpenMemHandle / memfd + hipHostRegister), and the
// local halves of allocations (stream-ordered pool, pinned host, malloc).
// Reference parity: ocm_init / ocm_tini src/lib.c:97-165, the local half of
// ocm_alloc src/lib.c:174-344 (malloc / cudaMalloc / ib_new+ib_connect there).
#include "internal.h"

namespace ocmlib {

State &S() {
    static State *s = new State();  // never destroyed: safe at process exit
    return *s;
}

int env_int(const char *k, int dflt) {
    const char *v = std::getenv(k);
    return (v && *v) ? std::atoi(v) : dflt;
}


long now_ms() {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec * 1000L + ts.tv_nsec / 1000000L;
}

Msg new_msg(uint32_t type) {
    Msg m;
    std::memset(&m, 0, sizeof(m));
    m.type = type;
    m.status = MSG_REQUEST;
    m.pid = S().pid;
    m.rank = S().daemon_rank;
    m.src_rank = -1;
    return m;
}

// The next record from the daemon: the shared-memory link first (ocm/shmlink.h),
// then the socket (everything when there is no link; wake-ups, which are
// skipped, when there is one). Polls for `spin_ns`, then sleeps in poll(2) on
// the socket until `deadline_ms`. Returns 1, 0 on timeout, -1 on error.
static int recv_record(Msg *m, long deadline_ms, uint64_t spin_ns) {
    State &s = S();
    const bool link = s.link.ok();
    const uint64_t t0 = now_ns();
    s.last_via_link = false;
    for (unsigned i = 0;; i++) {
        if (link && s.link.take_reply(m)) return s.last_via_link = true, 1;
        // With a link the socket carries only wake-ups: look at it now and then.
        if (!link || (i & 63) == 0) {
            const int rc = s.chan.recv(m, kMsgBytes, 0);
            if (rc < 0) return -1;
            if (rc == 1 && m->type != MSG_WAKE) return 1;
        }
        if (now_ns() - t0 >= spin_ns) break;
        // The daemon may be the other hardware thread of this core: leave it the pipeline.
        if (link) __builtin_ia32_pause();
    }
    for (;;) {
        const long left = deadline_ms - now_ms();
        if (left <= 0) return 0;
        if (link) {
            s.link.set_app_waiting(true);  // from here the daemon wakes us; look once more
            if (s.link.replies_pending()) {
                s.link.set_app_waiting(false);
                if (s.link.take_reply(m)) return s.last_via_link = true, 1;
                continue;
            }
        }
        const int rc = s.chan.recv(m, kMsgBytes, (int)std::min<long>(left, 1000));
        if (link) {
            s.link.set_app_waiting(false);
            if (rc >= 0 && (rc == 0 || m->type == MSG_WAKE)) {
                if (s.link.take_reply(m)) return s.last_via_link = true, 1;
                continue;
            }
        }
        if (rc < 0) return -1;
        if (rc == 1 && m->type != MSG_WAKE) return 1;
    }
}

// Send a request and wait for the reply carrying the same seq.
int rpc(Msg &req, Msg *reply, int timeout_ms) {
    State &s = S();
    req.seq = ++s.seq;
    int sent = 0;
    if (req.type == MSG_CONNECT && s.link.ok()) {
        // Offer the shared-memory link with the CONNECT (SCM_RIGHTS).
        sent = mbox_send_fd(s.chan.fd(), &req, kMsgBytes, s.link.fd(), timeout_ms);
    } else if (s.link.ok() && req.type != MSG_CONNECT && req.type != MSG_SLAB_FD && s.link.post_request(req)) {
        sent = 1;
        s.ctr.n_link_rpc++;
        if (s.link.request_needs_wake()) {  // the daemon sleeps: a wake-up on the socket
            Msg w = new_msg(MSG_WAKE);
            sent = s.chan.send(&w, kMsgBytes, timeout_ms);
            s.ctr.n_link_wake++;
        }
    } else {
        sent = s.chan.send(&req, kMsgBytes, timeout_ms);
    }
    if (sent != 1) OCM_FAIL(-1, "mailbox send to daemon failed");
    // A reply usually lands within a few microseconds: poll for it (bounded,
    // OCM_RPC_SPIN_US) before sleeping, which adds a wake-up.
    const long deadline = now_ms() + timeout_ms;
    uint64_t spin = s.rpc_spin_ns;
    for (;;) {
        const int rc = recv_record(reply, deadline, spin);
        spin = 0;
        if (rc < 0) return -1;
        if (rc == 0) OCM_FAIL(-1, "daemon did not answer %s within %d ms", msg_type_str(req.type), timeout_ms);
        if (reply->seq == req.seq && reply->type != MSG_EXTENT) return 0;
        OCM_LOG("dropping stale reply %s seq %llu", msg_type_str(reply->type), (unsigned long long)reply->seq);
    }
}

int recv_seq(Msg *m, uint64_t seq, uint32_t type, int timeout_ms) {
    const long deadline = now_ms() + timeout_ms;
    for (;;) {
        const int rc = recv_record(m, deadline, S().rpc_spin_ns);
        if (rc < 0) return -1;
        if (rc == 0) OCM_FAIL(-1, "timed out waiting for %s", msg_type_str(type));
        if (m->seq == seq && m->type == type) return 0;
    }
}

bool is_pair(enum ocm_kind k) { return k == OCM_REMOTE_GPU || k == OCM_REMOTE_RDMA || k == OCM_REMOTE_RMA; }

// ---------------------------------------------------------------- import cache

// Ask the owner daemon for host-tier slab `slab_id`'s memfd over its mailbox
// (a side connection per owner, kept open). -1 when it cannot be had.
int slab_fd_from_owner(int owner, uint32_t slab_id) {
    State &s = S();
    auto it = s.fd_chans.find(owner);
    if (it == s.fd_chans.end()) {
        const int fd = mbox_connect(daemon_mailbox_name(owner, s.ns), 2000);
        if (fd < 0) return -1;
        it = s.fd_chans.emplace(owner, fd).first;
    }
    Msg q = new_msg(MSG_SLAB_FD);
    q.seq = ++s.seq;
    q.u.region.owner_rank = owner;
    q.u.region.slab_id = slab_id;
    q.u.region.tier = TIER_HOST;
    Msg r;
    int got = -1;
    if (mbox_send(it->second, &q, kMsgBytes, 5000) != 1 || mbox_recv_fd(it->second, &r, kMsgBytes, &got, 5000) != 1 ||
        r.seq != q.seq || r.type != MSG_SLAB_FD || r.err) {
        if (got >= 0) close(got);
        close(it->second);
        s.fd_chans.erase(it);  // the stream may be out of step: reconnect next time
        return -1;
    }
    return got;
}

void close_fd_chans() {
    State &s = S();
    for (auto &kv : s.fd_chans) close(kv.second);
    s.fd_chans.clear();
}

namespace {
void close_views(Mapping &m) {
    for (auto &kv : m.dev_views) {
        DeviceGuard g(kv.first);
        (void)hipIpcCloseMemHandle(kv.second);
    }
    m.dev_views.clear();
}
}  // namespace

int import_extent(Extent &e) {
    State &s = S();
    const Region &r = e.r;
    if (r.flags & REGION_NET) {
        std::string host;
        int port = 0;
        uint64_t tok = 0, grant = 0;
        if (!parse_net_handle(r.handle, &host, &port, &tok, &grant)) OCM_FAIL(-1, "bad network-tier handle");
        e.net = true;
        e.dev_ok = false;
        e.ep = host + ":" + std::to_string(port);
        e.net_token = tok;
        e.net_grant = grant;
        return 0;
    }
    SlabKey key{r.owner_rank, r.tier, r.slab_id};
    auto it = s.imports.find(key);
    if (it != s.imports.end() && std::memcmp(it->second.handle, r.handle, kHandleBytes) != 0) {
        // Same id, different export: the owner restarted. Drop the stale mapping.
        Mapping &m = it->second;
        if (!m.dev_views.empty()) {
            push_release();
            close_views(m);
        }
        if (r.tier == TIER_GPU && m.dbase) (void)hipIpcCloseMemHandle(m.dbase);
        if (m.registered) (void)hipHostUnregister(m.hbase);
        if (m.hbase) munmap(m.hbase, m.bytes);
        s.imports.erase(it);
        it = s.imports.end();
    }
    if (it == s.imports.end()) {
        Mapping m;
        m.bytes = r.slab_bytes;
        m.dedicated = (r.flags & REGION_DEDICATED) != 0;
        std::memcpy(m.handle, r.handle, kHandleBytes);
        if (r.tier == TIER_GPU) {
            if (s.device < 0) OCM_FAIL(-1, "remote HBM extent but this process has no GPU");
            DeviceGuard g(s.device);
            hipIpcMemHandle_t h;
            std::memcpy(&h, r.handle, sizeof(h));
            void *p = nullptr;
            // (the lazy-peer-access flag is mandatory: 0 is rejected as an invalid argument)
            hipError_t err = hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess);
            if (err != hipSuccess) {
                if (r.owner_gpu != s.device) s.ipc_peer_failures++;
                OCM_FAIL(-1, "hipIpcOpenMemHandle(owner %d slab %u): %s", r.owner_rank, r.slab_id, hipGetErrorString(err));
            }
            if (r.owner_gpu != s.device) s.ipc_peer_imports++;  // another GPU's HBM, reached over xGMI
            m.dbase = static_cast<char *>(p);
        } else {
            // The owner hands us the slab's memfd (SCM_RIGHTS); the /proc path in
            // the handle is the fallback (it needs ptrace access to the owner).
            int fd = slab_fd_from_owner(r.owner_rank, r.slab_id);
            if (fd >= 0) {
                s.ctr.n_slab_fd++;
            } else {
                char path[kHandleBytes + 1];
                std::memcpy(path, r.handle, kHandleBytes);
                path[kHandleBytes] = 0;
                fd = open(path, O_RDWR | O_CLOEXEC);
                if (fd < 0) OCM_FAIL(-1, "host-tier slab %u of rank %d: no fd from its owner, and open(%s): %s", r.slab_id,
                                     r.owner_rank, path, strerror(errno));
                s.ctr.n_slab_path++;
            }
            void *p = mmap(nullptr, r.slab_bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
            close(fd);
            if (p == MAP_FAILED) OCM_FAIL(-1, "mmap host-tier slab: %s", strerror(errno));
            m.hbase = static_cast<char *>(p);
            m.dbase = m.hbase;
            if (s.device >= 0) {
                DeviceGuard g(s.device);
                hipError_t err = hipHostRegister(p, r.slab_bytes, hipHostRegisterMapped | hipHostRegisterPortable);
                if (err == hipSuccess) {
                    void *dp = nullptr;
                    if (hipHostGetDevicePointer(&dp, p, 0) == hipSuccess) m.dbase = static_cast<char *>(dp);
                    m.registered = true;
                } else {
                    (void)hipGetLastError();
                    OCM_WARN("hipHostRegister of host-tier slab failed: %s (DMA from pageable memory)", hipGetErrorString(err));
                }
            }
        }
        it = s.imports.emplace(key, m).first;
    }
    it->second.refs++;
    e.dev_ok = r.tier == TIER_GPU || it->second.registered;
    e.dptr = it->second.dbase + r.offset;
    e.hptr = it->second.hbase ? it->second.hbase + r.offset : nullptr;
    return 0;
}

char *extent_view(const Extent &e, int dev) {
    State &s = S();
    if (e.net || e.r.tier != TIER_GPU) return nullptr;
    if (dev == s.device) return e.dptr;
    auto it = s.imports.find(SlabKey{e.r.owner_rank, e.r.tier, e.r.slab_id});
    if (it == s.imports.end()) return nullptr;
    Mapping &m = it->second;
    auto v = m.dev_views.find(dev);
    if (v == m.dev_views.end()) {
        // A second import of the slab, by this process's context on `dev`: HIP allows
        // one open per device context, and it maps the slab into that device's
        // address space (the first import mapped it for s.device only).
        DeviceGuard g(dev);
        hipIpcMemHandle_t h;
        std::memcpy(&h, m.handle, sizeof(h));
        void *p = nullptr;
        const hipError_t err = hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess);
        if (err != hipSuccess) {
            (void)hipGetLastError();
            OCM_FAIL(nullptr, "hipIpcOpenMemHandle on device %d (owner %d slab %u): %s", dev, e.r.owner_rank,
                     e.r.slab_id, hipGetErrorString(err));
        }
        v = m.dev_views.emplace(dev, static_cast<char *>(p)).first;
    }
    return v->second + e.r.offset;
}

void release_extent(const Extent &e, bool force) {
    State &s = S();
    if (e.net) return;
    SlabKey key{e.r.owner_rank, e.r.tier, e.r.slab_id};
    auto it = s.imports.find(key);
    if (it == s.imports.end()) return;
    Mapping &m = it->second;
    if (--m.refs > 0 && !force) return;
    if (!m.dedicated && !force) return;  // shared slabs stay mapped for reuse
    if (!m.dev_views.empty()) {
        push_release();  // no push launch may still read a view we close
        close_views(m);
    }
    DeviceGuard g(s.device);
    if (e.r.tier == TIER_GPU && m.dbase) (void)hipIpcCloseMemHandle(m.dbase);
    if (m.registered) (void)hipHostUnregister(m.hbase);
    if (m.hbase) munmap(m.hbase, m.bytes);
    s.imports.erase(it);
}

Loc pointer_loc(const void *p) {
    State &s = S();
    if (s.device < 0 || !p) return LOC_HOST;
    hipPointerAttribute_t at;
    if (hipPointerGetAttributes(&at, p) != hipSuccess) {
        (void)hipGetLastError();
        return LOC_HOST;
    }
    if (at.type == hipMemoryTypeDevice) return LOC_DEVICE;
    if (at.type == hipMemoryTypeHost) return LOC_PINNED;
    return LOC_HOST;
}

hipMemPool_t local_pool() {
    State &s = S();
    if (s.pool_tried) return s.pool;
    s.pool_tried = true;
    if (s.device < 0 || !env_int("OCM_LOCAL_POOL", 1)) return nullptr;
    DeviceGuard g(s.device);
    hipMemPoolProps props;
    std::memset(&props, 0, sizeof(props));
    props.allocType = hipMemAllocationTypePinned;
    props.handleTypes = hipMemHandleTypeNone;
    props.location.type = hipMemLocationTypeDevice;
    props.location.id = s.device;
    if (hipMemPoolCreate(&s.pool, &props) != hipSuccess) {
        (void)hipGetLastError();
        OCM_WARN("hipMemPoolCreate on device %d failed; local halves use hipMalloc", s.device);
        s.pool = nullptr;
        return nullptr;
    }
    if (const char *k = std::getenv("OCM_LOCAL_POOL_KEEP")) s.pool_keep = std::strtoull(k, nullptr, 0);
    uint64_t keep = s.pool_keep;
    (void)hipMemPoolSetAttribute(s.pool, hipMemPoolAttrReleaseThreshold, &keep);
    // Peers read/write the local half too (SDMA from peer engines, torch on another GPU).
    int ndev = 0;
    (void)hipGetDeviceCount(&ndev);
    for (int p = 0; p < ndev; p++) {
        int can = 0;
        if (p == s.device || hipDeviceCanAccessPeer(&can, p, s.device) != hipSuccess || !can) continue;
        hipMemAccessDesc d;
        d.location.type = hipMemLocationTypeDevice;
        d.location.id = p;
        d.flags = hipMemAccessFlagsProtReadWrite;
        if (hipMemPoolSetAccess(s.pool, &d, 1) != hipSuccess) (void)hipGetLastError();
    }
    return s.pool;
}

// ---------------------------------------------------------------- pinned arena

namespace {
constexpr uint64_t kPinnedChunk = 64ull << 20;
constexpr uint64_t kPinnedAlign = 2ull << 20;
PinnedArena &pinned_arena() {
    State &s = S();
    if (!s.pinned) s.pinned = new PinnedArena();
    return *s.pinned;
}
}  // namespace

void *PinnedArena::alloc(size_t bytes) {
    State &s = S();
    if (bytes == 0) return nullptr;
    const bool big = bytes >= kPinnedChunk / 2;
    if (!big) {
        for (auto &kv : chunks_) {
            Chunk &c = kv.second;
            uint64_t off = 0;
            if (!c.dedicated && c.ra.alloc(bytes, 4096, &off)) return c.base + off;
        }
    } else {
        // A cached dedicated chunk of about this size (up to 2x) is reused as a whole.
        Chunk *best = nullptr;
        for (auto &kv : chunks_) {
            Chunk &c = kv.second;
            if (c.dedicated && c.ra.empty() && c.bytes >= bytes && c.bytes <= 2 * bytes &&
                (!best || c.bytes < best->bytes))
                best = &c;
        }
        uint64_t off = 0;
        if (best && best->ra.alloc(bytes, 4096, &off)) return best->base + off;
    }
    const uint64_t size = big ? (bytes + kPinnedAlign - 1) & ~(kPinnedAlign - 1) : kPinnedChunk;
    void *p = nullptr;
    DeviceGuard g(s.device);
    if (hipHostMalloc(&p, size, hipHostMallocDefault) != hipSuccess) {
        (void)hipGetLastError();
        trim();  // give idle chunks back and try once more
        if (hipHostMalloc(&p, size, hipHostMallocDefault) != hipSuccess) {
            (void)hipGetLastError();
            return nullptr;
        }
    }
    Chunk &c = chunks_[reinterpret_cast<uintptr_t>(p)];
    c.base = static_cast<char *>(p);
    c.bytes = size;
    c.dedicated = big;
    c.ra.reset(size);
    pinned_ += size;
    uint64_t off = 0;
    c.ra.alloc(bytes, 4096, &off);
    return c.base + off;
}

bool PinnedArena::free(void *ptr) {
    const uintptr_t v = reinterpret_cast<uintptr_t>(ptr);
    auto it = chunks_.upper_bound(v);
    if (it == chunks_.begin()) return false;
    --it;
    Chunk &c = it->second;
    if (v >= it->first + c.bytes) return false;
    if (!c.ra.free(v - it->first)) return false;
    if (c.ra.empty()) trim();
    return true;
}

void PinnedArena::trim() {
    State &s = S();
    // Unpin idle chunks beyond the keep budget (largest first).
    uint64_t idle = 0;
    for (auto &kv : chunks_) idle += kv.second.ra.empty() ? kv.second.bytes : 0;
    while (idle > s.pinned_keep) {
        auto victim = chunks_.end();
        for (auto it = chunks_.begin(); it != chunks_.end(); ++it)
            if (it->second.ra.empty() && (victim == chunks_.end() || it->second.bytes > victim->second.bytes)) victim = it;
        if (victim == chunks_.end()) break;
        DeviceGuard g(s.device);
        (void)hipHostFree(victim->second.base);
        idle -= victim->second.bytes;
        pinned_ -= victim->second.bytes;
        chunks_.erase(victim);
    }
}

void PinnedArena::release_all() {
    State &s = S();
    DeviceGuard g(s.device);
    for (auto &kv : chunks_) (void)hipHostFree(kv.second.base);
    chunks_.clear();
    pinned_ = 0;
}

int free_local_half(lib_alloc *a) {
    State &s = S();
    if (!a->local) return 0;
    if (a->pooled) {
        // The library's own ops on the block are done (ocm_free waited for them):
        // keep it for an exact-size reuse, or return it to the pool, ordered after
        // every transfer queued on s.stream.
        const uint64_t kMaxCachedBlock = 256ull << 20;
        if (a->local_bytes <= kMaxCachedBlock && s.dev_cache_bytes + a->local_bytes <= s.dev_cache_cap) {
            s.dev_cache.emplace(a->local_bytes, a->local);
            s.dev_cache_bytes += a->local_bytes;
        } else {
            DeviceGuard g(s.device);
            if (hipFreeAsync(a->local, s.stream) != hipSuccess) (void)hipGetLastError();
        }
        a->pooled = false;
    } else if (a->loc == LOC_DEVICE) {
        DeviceGuard g(s.device);
        (void)hipFree(a->local);
    } else if (a->loc == LOC_PINNED) {
        if (!pinned_arena().free(a->local)) {
            DeviceGuard g(s.device);
            (void)hipHostFree(a->local);
        }
    } else {
        std::free(a->local);
    }
    a->local = nullptr;
    return 0;
}

// Return every cached block to the pool (ocm_tini, before the pool goes).
void release_dev_cache() {
    State &s = S();
    if (s.dev_cache.empty()) return;
    DeviceGuard g(s.device);
    for (auto &kv : s.dev_cache)
        if (hipFreeAsync(kv.second, s.stream) != hipSuccess) (void)hipGetLastError();
    s.dev_cache.clear();
    s.dev_cache_bytes = 0;
    (void)hipStreamSynchronize(s.stream);
}

int alloc_local_half(lib_alloc *a, size_t bytes, Loc want) {
    State &s = S();
    a->local_bytes = bytes;
    if (bytes == 0) return 0;
    if (want != LOC_HOST && s.device < 0) want = LOC_HOST;
    if (want == LOC_DEVICE && local_pool()) {
        auto hit = s.dev_cache.find(bytes);
        if (hit != s.dev_cache.end()) {
            a->local = hit->second;
            s.dev_cache_bytes -= bytes;
            s.dev_cache.erase(hit);
            a->pooled = true;
            a->loc = want;
            return 0;
        }
        DeviceGuard g(s.device);
        hipError_t e = hipMallocFromPoolAsync(&a->local, bytes, s.pool, s.stream);
        // The app may touch the buffer from any stream as soon as ocm_alloc returns:
        // the block's earlier user must be done. Blocking ops leave s.stream idle, so
        // a query (no wait) settles it; otherwise wait for the stream.
        if (e == hipSuccess) {
            e = hipStreamQuery(s.stream);
            if (e == hipErrorNotReady) e = hipStreamSynchronize(s.stream);
        }
        if (e != hipSuccess) {
            (void)hipGetLastError();
            OCM_FAIL(-1, "pool allocation of %zu bytes for local half: %s", bytes, hipGetErrorString(e));
        }
        a->pooled = true;
    } else if (want == LOC_DEVICE) {
        DeviceGuard g(s.device);
        hipError_t e = hipMalloc(&a->local, bytes);
        if (e != hipSuccess) {
            (void)hipGetLastError();
            OCM_FAIL(-1, "hipMalloc(%zu) for local half: %s", bytes, hipGetErrorString(e));
        }
    } else if (want == LOC_PINNED) {
        a->local = pinned_arena().alloc(bytes);
        if (!a->local) OCM_FAIL(-1, "pinned host memory for a %zu-byte local half", bytes);
    } else {
        if (posix_memalign(&a->local, 4096, bytes) != 0) OCM_FAIL(-1, "host allocation of %zu bytes failed", bytes);
    }
    a->loc = want;
    return 0;
}


}  // namespace ocmlib

// libocm copy engine: striped segments, per-allocation lanes and events, the
// resident copy service, one-sided transfers (gfx950 kernels / DMA / CPU)
// and process-local copies.
// Reference parity: ocm_copy src/lib.c:501-665 and ocm_copy_onesided
// src/lib.c:669-723, whose RDMA/RMA legs (ib_read/ib_write over post_send,
// src/rdma.c:47-92,241-302; extoll_read/extoll_write over extoll_rma2_transfer,
// src/extoll.c:40-167,286-310, 8 MiB x 2 outstanding) become
// gfx950 kernel launches or the resident copy service here.
#include "internal.h"

namespace ocmlib {

// ---------------------------------------------------------------- copy engine


// Split [rem_off, rem_off+len) of a striped buffer into contiguous pieces.
void segments(const lib_alloc *a, uint64_t rem_off, uint64_t len, std::vector<Seg> &out) {
    out.clear();
    const int n = (int)a->ext.size();
    if (n == 1 || a->stripe_unit == 0) {
        out.push_back({0, rem_off, 0, len});
        return;
    }
    const uint64_t unit = a->stripe_unit;
    uint64_t pos = rem_off, done = 0;
    while (done < len) {
        const uint64_t u = pos / unit, within = pos % unit;
        const uint64_t take = std::min(unit - within, len - done);
        out.push_back({(int)(u % n), (u / n) * unit + within, done, take});
        pos += take;
        done += take;
    }
}


int wait_event(hipEvent_t ev) {
    State &s = S();
    hipError_t e = hipSuccess;
    if (s.sync_mode == 1) {
        while ((e = hipEventQuery(ev)) == hipErrorNotReady) {
        }
    } else {
        e = hipEventSynchronize(ev);
    }
    if (e != hipSuccess) OCM_FAIL(-1, "event wait: %s", hipGetErrorString(e));
    return 0;
}

// ocm_stream_wait dependency: order it before work on `st` (nullptr: the
// copy service, which has no stream, so wait on the host).
int honor_dep(lib_alloc *a, hipStream_t st, bool host_wait) {
    if (!a->dep_pending) return 0;
    a->dep_pending = false;
    hipError_t e = host_wait ? hipEventSynchronize(a->dep_ev) : hipStreamWaitEvent(st, a->dep_ev, 0);
    if (e != hipSuccess) OCM_FAIL(-1, "stream dependency: %s", hipGetErrorString(e));
    return 0;
}

// Completion of `a`'s queued async ops (its lane up to the recorded event).
int wait_alloc(lib_alloc *a) {
    State &s = S();
    if (!a || !a->async_pending) return 0;
    a->async_pending = false;
    if (!a->ev) return 0;
    DeviceGuard g(s.device);
    return wait_event(a->ev);
}

hipStream_t lane_stream(lib_alloc *a) {
    State &s = S();
    if (a->lane < 0) {
        if (s.lanes.empty()) {
            DeviceGuard g(s.device);
            for (int i = 0; i < std::max(1, s.n_lanes); i++) {
                hipStream_t st = nullptr;
                if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess) {
                    (void)hipGetLastError();
                    break;
                }
                s.lanes.push_back(st);
            }
        }
        if (s.lanes.empty()) return s.stream;
        if (!s.lane_flags && s.launch_flags) {
            DeviceGuard g(s.device);
            const size_t nl = s.lanes.size();
            if (hipHostMalloc(reinterpret_cast<void **>(&s.lane_flags), nl * 128,
                              hipHostMallocCoherent | hipHostMallocMapped) != hipSuccess ||
                hipMalloc(reinterpret_cast<void **>(&s.lane_cnt), nl * 128) != hipSuccess ||
                hipMemset(s.lane_cnt, 0, nl * 128) != hipSuccess) {
                (void)hipGetLastError();
                s.launch_flags = false;  // events only
            } else {
                std::memset(s.lane_flags, 0, nl * 128);
                s.lane_flag_seq.assign(nl, 0);
            }
        }
        a->lane = s.next_lane++ % (int)s.lanes.size();
    }
    if (!a->ev) {
        DeviceGuard g(s.device);
        if (hipEventCreateWithFlags(&a->ev, hipEventDisableTiming) != hipSuccess) {
            (void)hipGetLastError();
            a->ev = nullptr;
            return s.stream;
        }
    }
    return s.lanes[a->lane];
}

int sync_stream() {
    State &s = S();
    if (!s.stream) return 0;
    DeviceGuard g(s.device);
    hipError_t e = hipSuccess;
    if (s.sync_mode == 0 || !s.done) {
        e = hipStreamSynchronize(s.stream);
    } else {
        e = hipEventRecord(s.done, s.stream);
        if (e == hipSuccess && s.sync_mode == 1) {
            // Spin: lowest completion latency for small one-sided ops.
            while ((e = hipEventQuery(s.done)) == hipErrorNotReady) {
            }
        } else if (e == hipSuccess) {
            e = hipEventSynchronize(s.done);
        }
    }
    if (e != hipSuccess) OCM_FAIL(-1, "stream sync: %s", hipGetErrorString(e));
    return 0;
}

// ---- persistent copy service ----
// Instances run on lanes: an AQL queue of the library's own (ocm/aql.h; HIP does
// not know it, so a device-wide synchronize never waits for the service and the
// lead may stay resident alone between bursts, OCM_SERVICE_LONE_US) or, when that
// is unavailable or OCM_SERVICE_QUEUE=hip, a HIP stream of the service's priority
// (then the whole instance leaves after OCM_SERVICE_IDLE_US).

static bool lane_idle(State::SvcLane &l) {
    if (l.aql) return aql_lane_idle(&l.q);
    const hipError_t e = hipStreamQuery(l.stream);
    (void)hipGetLastError();
    return e == hipSuccess;
}

// Wait until every workgroup of the lane's last instance has left. 0: drained;
// -1: not within timeout_ns. `site` names the caller in the health counters
// (the longest drain and where it happened).
enum DrainSite : unsigned { kDrainStart = 1, kDrainPark, kDrainStop, kDrainAbort, kDrainRepost };
static int lane_drain_timed(State::SvcLane &l, uint64_t timeout_ns) {
    if (l.aql) return aql_lane_wait(&l.q, timeout_ns);
    const uint64_t t0 = now_ns();
    hipError_t e;
    while ((e = hipStreamQuery(l.stream)) == hipErrorNotReady) {
        if (now_ns() - t0 > timeout_ns) return -1;
        usleep(20);
    }
    (void)hipGetLastError();
    return 0;
}
static int lane_drain(State::SvcLane &l, uint64_t timeout_ns, DrainSite site) {
    State &s = S();
    const uint64_t t0 = now_ns();
    const int rc = lane_drain_timed(l, timeout_ns);
    const uint64_t dt = now_ns() - t0;
    if (dt > s.svc_drain_max_ns) {
        s.svc_drain_max_ns = dt;
        s.svc_drain_max_site = site;
    }
    return rc;
}

// The current instance's tagged status words (ocm/xfer.h): 0 unless it wrote them.
static unsigned long long svc_word(const unsigned long long *w) {
    return service_untag(S().svc_epoch, __atomic_load_n(w, __ATOMIC_ACQUIRE));
}

// A new lane: an AQL queue or a stream of the service's priority, and a gang box. -1 on failure.
static int service_new_lane() {
    State &s = S();
    State::SvcLane l;
    if (s.svc_aql) {
        if (aql_lane_create(&l.q, true) != 0) return -1;
        l.aql = true;
    } else {
        hipError_t e = s.svc_prio_ok ? hipStreamCreateWithPriority(&l.stream, hipStreamNonBlocking, s.svc_stream_prio)
                                     : hipStreamCreateWithFlags(&l.stream, hipStreamNonBlocking);
        if (e != hipSuccess) {
            (void)hipGetLastError();
            return -1;
        }
    }
    if (hipMalloc(reinterpret_cast<void **>(&l.box), sizeof(ServiceBox)) != hipSuccess) {
        (void)hipGetLastError();
        if (l.aql)
            aql_lane_destroy(&l.q);
        else
            (void)hipStreamDestroy(l.stream);
        return -1;
    }
    l.dirty = true;  // fresh device memory: its first launch clears it
    s.svc_lanes.push_back(l);
    return (int)s.svc_lanes.size() - 1;
}

int service_start(unsigned long long first_seq) {
    State &s = S();
    DeviceGuard g(s.device);
    if (!s.svc) {
        if (hipHostMalloc(reinterpret_cast<void **>(&s.svc), sizeof(ServiceSlot),
                          hipHostMallocCoherent | hipHostMallocMapped) != hipSuccess) {
            (void)hipGetLastError();
            s.svc = nullptr;
            s.svc_max = 0;
            OCM_FAIL(-1, "copy service: no coherent host memory");
        }
        std::memset(s.svc, 0, sizeof(ServiceSlot));
        s.svc_req = &s.svc->req;
        // The library's own AQL queue when the embedded code object loads for this
        // device; otherwise HIP streams (and no lone lead: a device-wide synchronize
        // would wait for it).
        s.svc_aql = false;
        if (s.svc_queue_aql) {
            const char *why = nullptr;
            if (aql_open(s.device, &why) != 0)
                OCM_INFO("copy service on HIP streams: AQL queue unavailable (%s)", why ? why : "?");
            else if (aql_kernel(kServiceKernelSymbol, &s.svc_kernel) != 0 ||
                     s.svc_kernel.kernarg_bytes < sizeof(ServiceKernelArgs))
                OCM_INFO("copy service on HIP streams: no usable %s in the embedded code object", kServiceKernelSymbol);
            else
                s.svc_aql = true;
            // OCM_SERVICE_CLEAR_KERNEL=0: clear gang boxes with a host memset (A/B)
            if (s.svc_aql && (env_int("OCM_SERVICE_CLEAR_KERNEL", 1) == 0 ||
                              aql_kernel(kServiceBoxClearSymbol, &s.svc_clear_kernel) != 0))
                s.svc_clear_kernel = AqlKernel{};
        }
        if (!s.svc_aql) s.svc_lone_ticks = 0;
        // Streams of their own priority: HIP shares its few hardware queues
        // (GPU_MAX_HW_QUEUES) among a process's streams, and a launch on a stream
        // that shares the service's queue waits behind the persistent kernel until
        // its idle exit (2 ms per large op in bench.py with torch's streams around, when
        // the idle exit was 2 ms).
        // Queues are pooled per priority, so the service's is not shared with the
        // normal-priority streams of the library and the application.
        int lo = 0, hi = 0;
        s.svc_prio_ok = hipDeviceGetStreamPriorityRange(&lo, &hi) == hipSuccess && lo != hi;
        (void)hipGetLastError();
        s.svc_stream_prio = env_int("OCM_SERVICE_STREAM_PRIO", hi);
        if (service_new_lane() < 0 && s.svc_aql) {
            OCM_INFO("copy service on HIP streams: no AQL queue could be created");
            s.svc_aql = false;
            s.svc_lone_ticks = 0;
            service_new_lane();
        }
        if (s.svc_lanes.empty() && s.svc_prio_ok) {
            s.svc_prio_ok = false;
            s.svc_shared_queue = true;  // launches park the service first (see xfer)
            service_new_lane();
        }
        if (s.svc_lanes.empty()) {
            s.svc_max = 0;
            OCM_FAIL(-1, "copy service: no stream or device mailbox");
        }
        s.svc_lane = 0;
        const bool gangrec = (s.svc_proto & kServiceProtoGangRec) && s.svc_blocks > 1;
        const bool wc = (s.svc_proto & kServiceProtoWCReq) != 0;
        if (gangrec || wc) {
            // page 0: the small-op record when write-combined; page 1: the gang record
            const unsigned flags = (wc ? hipHostMallocWriteCombined : hipHostMallocCoherent) | hipHostMallocMapped;
            if (hipHostMalloc(reinterpret_cast<void **>(&s.svc_rec_pages), 8192, flags) != hipSuccess) {
                (void)hipGetLastError();
                s.svc_rec_pages = nullptr;  // one coherent record, relay protocol
                OCM_WARN("copy service: no %s record pages; using one coherent record and the relay protocol",
                         wc ? "write-combined" : "gang");
            } else {
                for (int i = 0; i < 8192 / 8; i++) __atomic_store_n(reinterpret_cast<unsigned long long *>(s.svc_rec_pages) + i, 0ull, __ATOMIC_RELAXED);
                __builtin_ia32_sfence();
                if (wc) s.svc_req = reinterpret_cast<ServiceReq *>(s.svc_rec_pages);
                if (gangrec) {
                    s.svc_greq = reinterpret_cast<ServiceReq *>(s.svc_rec_pages + 4096);
                    s.svc_greq_copies = (s.svc_proto & kServiceProtoCopies)
                                            ? std::max(1u, std::min(std::min(s.svc_direct, s.svc_blocks),
                                                                    (unsigned)kServiceGangCopiesMax))
                                            : 1u;
                }
            }
        }
    }
    if (s.svc_wedged) OCM_FAIL(-1, "copy service: a previous instance could not be drained");
    // A lane whose last instance has drained: the current one normally (its last
    // instance's workgroups leave microseconds after its lead), another drained one,
    // a new one, or - every lane still holding workgroups that found no CU, or a
    // lone lead that has not yet seen it was replaced - wait for the current.
    // HIP lanes: when the last instance had its whole grid resident (its roster is
    // still in the slot), its workgroups leave right behind its lead: stay on its
    // lane without a runtime query (stream order starts the new instance after them;
    // they ignore the new epoch meanwhile). A stream query costs ~10 us of host
    // time; an AQL lane's is one load of its completion signal.
    // AQL lanes: when the last instance had its whole grid resident (a lone lead
    // included: only such an instance goes lone), the new one goes on the same
    // queue right away, beside a lead that has not left yet (it leaves on the new
    // epoch; the packet starts once the old one's workgroups have all been
    // dispatched, which they have): no new queue, no wait.
    const uint64_t tq = now_ns();
    int pick = -1;
    bool overlap = false;
    const int n = (int)s.svc_lanes.size();
    const bool whole = s.svc_lane >= 0 && svc_word(&s.svc->roster) >= s.svc_blocks;
    if (whole && !s.svc_aql && !s.svc_relaunch_query) pick = s.svc_lane;
    if (whole && s.svc_aql && !s.svc_lanes[(size_t)s.svc_lane].dirty && !s.svc_box_reset_always &&
        s.svc_lanes[(size_t)s.svc_lane].gang_total <= (1ull << 30)) {  // a box clear would make a third dispatch
        const long run = aql_lane_inflight(&s.svc_lanes[(size_t)s.svc_lane].q);
        if (run <= 1) {
            pick = s.svc_lane;
            overlap = run == 1;
        }
    }
    for (int k = 0; k < n && pick < 0; k++) {
        const int i = (s.svc_lane + k) % n;
        if (lane_idle(s.svc_lanes[(size_t)i])) pick = i;
    }
    if (pick < 0 && (unsigned)n < s.svc_lanes_max) pick = service_new_lane();
    if (pick < 0) {
        pick = s.svc_lane;
        if (s.svc_lanes[(size_t)pick].aql) {
            // a lone lead on it leaves once it sees the new epoch
            __atomic_store_n(&s.svc->epoch_now, (unsigned long long)((s.svc_epoch + 1) & (unsigned)kServiceGangEpochMask),
                             __ATOMIC_RELEASE);
            __builtin_ia32_sfence();
        }
        if (lane_drain(s.svc_lanes[(size_t)pick], s.svc_drain_ns, kDrainStart) != 0) {
            s.svc_wedged = true;
            s.svc_max = 0;
            OCM_FAIL(-1, "copy service: no lane drained within OCM_SERVICE_DRAIN_MS");
        }
    }
    s.svc_lane = pick;
    State::SvcLane &l = s.svc_lanes[(size_t)pick];
    s.svc_stream = l.stream;
    s.svc_box = l.box;
    s.svc_epoch = (s.svc_epoch + 1) & (unsigned)kServiceGangEpochMask;
    // the last instance's GPU time (diagnostic) joins the total; a lead that is still
    // leaving serves nothing more, so it writes no more ticks
    s.svc_gpu_ticks_done += __atomic_exchange_n(&s.svc->gpu_ticks, 0ull, __ATOMIC_ACQ_REL);
    __atomic_store_n(&s.svc->exited, 0ull, __ATOMIC_RELEASE);
    __atomic_store_n(&s.svc->roster, 0ull, __ATOMIC_RELEASE);  // the new lead publishes its own
    __atomic_store_n(&s.svc->lone, 0ull, __ATOMIC_RELEASE);
    // A lone lead of an earlier instance (another lane) leaves when it sees this.
    __atomic_store_n(&s.svc->epoch_now, (unsigned long long)s.svc_epoch, __ATOMIC_RELEASE);
    service_store_seq(s.svc_req, 0ull);  // clear a STOP left by a parked instance
    if (s.svc_greq) service_store_seq(s.svc_greq, 0ull, s.svc_greq_copies);
    // the gang counter mirror stays below the 31-bit target field (ocm/xfer.h)
    const bool reset = l.dirty || s.svc_box_reset_always || l.gang_total > (1ull << 30);
    if (reset) {
        l.gang_total = 0;  // the launch zeroes the device counters
        l.checkins = 0;
    }
    ServiceKernelArgs ka;
    std::memset(&ka, 0, sizeof(ka));
    ka.req = s.svc_req;
    ka.gang_req = s.svc_greq;
    ka.slot = s.svc;
    ka.box = l.box;
    ka.first_seq = first_seq;
    ka.idle_ticks = s.svc_idle_ticks;
    ka.proto = s.svc_proto;
    ka.direct_wgs = std::min(s.svc_direct, s.svc_blocks);
    ka.checkin_base = l.checkins;
    ka.epoch = s.svc_epoch;
    ka.blocks = s.svc_blocks;
    ka.degraded_idle_ticks = s.svc_degraded_idle_ticks;
    ka.lone_ticks = l.aql ? s.svc_lone_ticks : 0;
    const uint64_t tl = now_ns();
    s.svc_ns_pick += tl - tq;
    if (l.aql) {
        // The box is cleared first: on the lane itself, the instance behind it with the
        // barrier bit (the queue is not a HIP stream); a host memset if that kernel is missing.
        bool barrier = false;
        if (reset && s.svc_clear_kernel.object && !overlap) {
            ServiceBox *bx = l.box;
            if (aql_dispatch(&l.q, s.svc_clear_kernel, &bx, sizeof(bx), 1, 256) != 0) {
                s.svc_max = 0;
                OCM_FAIL(-1, "copy service: gang box clear dispatch failed");
            }
            barrier = overlap = true;
        } else if (reset && (hipMemsetAsync(l.box, 0, sizeof(ServiceBox), s.stream) != hipSuccess ||
                             hipStreamSynchronize(s.stream) != hipSuccess)) {
            (void)hipGetLastError();
            s.svc_max = 0;
            OCM_FAIL(-1, "copy service: clearing the gang box failed");
        }
        if (aql_dispatch(&l.q, s.svc_kernel, &ka, sizeof(ka), s.svc_blocks, 256, overlap, barrier) != 0) {
            s.svc_max = 0;
            OCM_FAIL(-1, "copy service dispatch failed");
        }
        if (overlap && !barrier) s.svc_overlaps++;
    } else if (service_launch(ka, s.svc_blocks, reset, l.stream) != hipSuccess) {
        (void)hipGetLastError();
        s.svc_max = 0;
        OCM_FAIL(-1, "copy service launch failed");
    }
    s.svc_ns_launch += now_ns() - tl;
    s.svc_epoch_starts++;
    l.dirty = false;
    l.checkins += s.svc_blocks;  // every workgroup takes one ticket before the instance drains
    s.svc_running = true;
    s.svc_launch_ns = now_ns();
    return 0;
}

// Without a stream priority of its own (svc_shared_queue) the service may share
// a hardware queue with the library's launch streams, and a launch queued behind
// the persistent kernel would wait for its idle exit: park it first. Application
// kernels on such a queue still wait up to OCM_SERVICE_IDLE_US.
void before_launch() {
    State &s = S();
    if (s.svc_shared_queue) service_park();
}

// Park the resident kernel: its doorbell polls cross PCIe and slow down
// large DMA-engine transfers (measured: 53 -> 34 GiB/s on host-tier sweeps).
void service_park() {
    State &s = S();
    if (!s.svc || !s.svc_running) return;
    DeviceGuard g(s.device);
    service_store_seq(s.svc_req, kServiceStop);
    if (s.svc_greq) service_store_seq(s.svc_greq, kServiceStop, s.svc_greq_copies);
    State::SvcLane &l = s.svc_lanes[(size_t)s.svc_lane];
    if (l.aql) {
        if (lane_drain(l, s.svc_drain_ns, kDrainPark) != 0) {
            s.svc_wedged = true;
            s.svc_max = 0;
            OCM_WARN("copy service did not leave on STOP within OCM_SERVICE_DRAIN_MS; the service is off");
        }
    } else {
        (void)hipStreamSynchronize(l.stream);
    }
    s.svc_running = false;
}

void service_stop() {
    State &s = S();
    if (!s.svc) return;
    DeviceGuard g(s.device);
    service_store_seq(s.svc_req, kServiceStop);
    if (s.svc_greq) service_store_seq(s.svc_greq, kServiceStop, s.svc_greq_copies);
    s.svc_running = false;
    for (State::SvcLane &l : s.svc_lanes) {  // every lane drained before its box goes
        if (l.aql) {
            if (lane_drain(l, s.svc_drain_ns, kDrainStop) != 0) {
                // never free what a kernel that did not leave may still touch
                OCM_WARN("copy service: a lane did not drain at shutdown; its queue and box are leaked");
                continue;
            }
            aql_lane_destroy(&l.q);
        } else {
            (void)hipStreamSynchronize(l.stream);
            (void)hipStreamDestroy(l.stream);
        }
        if (l.box) (void)hipFree(l.box);
    }
    s.svc_lanes.clear();
    s.svc_lane = -1;
    s.svc_req = nullptr;
    if (s.svc_rec_pages) (void)hipHostFree(s.svc_rec_pages);
    s.svc_rec_pages = nullptr;
    s.svc_greq = nullptr;
    (void)hipHostFree(s.svc);
    s.svc = nullptr;
    s.svc_box = nullptr;
    s.svc_stream = nullptr;
}

// Members of the running instance a gang may name (ocm/xfer.h roster): right
// after a launch wait up to svc_roster_wait_ns for `want` of them to check in,
// then settle for the ones that did (at least workgroup 0).
static unsigned service_roster(unsigned want) {
    State &s = S();
    unsigned long long r = svc_word(&s.svc->roster);
    while (r < want && now_ns() - s.svc_launch_ns < s.svc_roster_wait_ns) {
        __builtin_ia32_pause();
        r = svc_word(&s.svc->roster);
    }
    if (r < 1) r = 1;
    if (r < want) s.svc_degraded++;
    if (r < s.svc_roster_min) s.svc_roster_min = r;
    return (unsigned)std::min<unsigned long long>(r, want);
}

// Give up on the instance holding request `seq`: STOP on both records, then wait
// (bounded) until the kernel has left, so no member can still run the request
// when the op is redone by a launch. -1: drained; -2: it would not drain.
static int service_abort(unsigned long long seq, unsigned long long active, const char *why) {
    State &s = S();
    DeviceGuard g(s.device);
    unsigned long long wg_in = 0;
    for (unsigned long long i = 0; i < active && i < (unsigned long long)kServiceWgDoneMax; i++)
        wg_in += __atomic_load_n(&s.svc->wg_done[i], __ATOMIC_ACQUIRE) == seq;
    const unsigned long long ex = svc_word(&s.svc->exited);
    const unsigned long long roster = svc_word(&s.svc->roster);
    service_store_seq(s.svc_req, kServiceStop);
    if (s.svc_greq) service_store_seq(s.svc_greq, kServiceStop, s.svc_greq_copies);
    s.svc_aborts++;
    if (lane_drain(s.svc_lanes[(size_t)s.svc_lane], s.svc_drain_ns, kDrainAbort) != 0) {
        s.svc_wedged = true;
        s.svc_max = 0;
        OCM_FAIL(-2, "copy service %s (seq %llu, %llu members, %llu done words, roster %llu, exited %llu) "
                     "and did not leave on STOP: not redoing the op",
                 why, seq, active, wg_in, roster, ex);
    }
    s.svc_running = false;
    if (s.svc_lane >= 0) s.svc_lanes[(size_t)s.svc_lane].dirty = true;
    OCM_FAIL(-1, "copy service %s (seq %llu, %llu members, %llu done words, roster %llu, exited %llu); drained",
             why, seq, active, wg_in, roster, ex);
}

// Run one normalized transfer through the resident kernel and wait for it.
int service_xfer(XferArgs x, unsigned solo_tiles, bool hbm, bool strict) {
    State &s = S();
    if (xfer_normalize(x) != hipSuccess) OCM_FAIL(-1, "invalid transfer");
    if (!hbm && x.len >= s.svc_host_tile_min && x.len <= s.svc_host_tile_max) {
        const unsigned sh = x.put ? s.svc_host_tile_shift_put : s.svc_host_tile_shift_get;
        if (sh >= 12 && sh < x.tile_shift) x.tile_shift = sh;
    }
    unsigned long long seq = ++s.svc_seq;
    const uint64_t t_enter = now_ns();
    bool relaunched = false;
    if (s.svc_running && svc_word(&s.svc->exited) != 0) {
        // The instance left on its idle timeout (OCM_SERVICE_IDLE_US), its last request
        // complete: start the next one right away instead of posting to nobody. No wait
        // for its stream: the next instance takes a drained lane, and a workgroup of the
        // old one still polling (or starting late) leaves requests of a newer epoch alone.
        s.svc_running = false;
        s.svc_relaunches++;
        relaunched = true;
    }
    if (!s.svc_running) {
        if (service_start(seq) != 0) return -1;
        if (relaunched) s.svc_ns_relaunch += now_ns() - t_enter;
    }
    // The host sizes the gang and the completion count every workgroup agrees on:
    // up to the direct pollers (no relay) for ops they copy fast enough, and never
    // wider than the members already running (the roster).
    const bool direct = s.svc_greq && x.len <= (hbm ? s.svc_direct_max_hbm : s.svc_direct_max_host);
    unsigned long long active = 1;
    bool wgdone = false;
    ServiceReq *rq = s.svc_req;
    unsigned long long gang = 0;
    auto size_and_post = [&]() -> int {
        unsigned width = direct ? std::min(s.svc_direct, s.svc_blocks)
                                : (hbm ? s.svc_blocks : std::min(s.svc_gang_host, s.svc_blocks));
        if (!hbm && !x.put && x.len >= s.svc_host_get_narrow_min) width = std::min(width, s.svc_host_get_width);
        if (service_gang_size(x, width, solo_tiles) > 1) {
            // A lone lead takes no gang: a full instance replaces it (the lead leaves
            // on the new epoch by itself; it holds no request of ours).
            if (svc_word(&s.svc->lone) != 0) {
                s.svc_promotions++;
                if (service_start(seq) != 0) return -1;
            }
            width = service_roster(width);
        }
        active = service_gang_size(x, width, solo_tiles);
        wgdone = service_wg_done(s.svc_proto, active);
        unsigned long long target = 0;
        if (active > 1 && !wgdone) {  // WGDONE gangs leave the counter alone
            State::SvcLane &l = s.svc_lanes[(size_t)s.svc_lane];
            l.gang_total += active;
            target = l.gang_total;
        }
        gang = active | (target << 16) | ((unsigned long long)s.svc_epoch << kServiceGangEpochShift) |
               (strict ? kServiceGangStrict : 0ull);
        // GANGREC: gang requests go to the record the whole gang polls.
        rq = (active > 1 && s.svc_greq) ? s.svc_greq : s.svc_req;
        service_post(rq, x, gang, seq, rq == s.svc_greq ? s.svc_greq_copies : 1u);
        return 0;
    };
    // Completed: `done` (a solo op or the gang's last member), or under WGDONE
    // every member's own word.
    auto finished = [&]() {
        if (!wgdone) return __atomic_load_n(&s.svc->done, __ATOMIC_ACQUIRE) == seq;
        for (unsigned long long i = active; i-- > 0;)
            if (__atomic_load_n(&s.svc->wg_done[i], __ATOMIC_ACQUIRE) != seq) return false;
        return true;
    };
    const uint64_t t0 = now_ns();
    if (size_and_post() != 0) return -1;
    const uint64_t t_posted = now_ns();
    for (unsigned spins = 1;; spins++) {
        if (finished()) {
            s.svc_ops++;
            s.svc_ns_post += t_posted - t0;
            s.svc_ns_wait += now_ns() - t_posted;
            return 0;
        }
        if ((spins & 1023) == 0) {
            // The kernel leaves after idle_ticks without work, and only once the
            // last request it took is complete. If it left before taking this one
            // (exited <= seq), start a new instance for it. exited > seq with the
            // op unfinished is not expected (workgroup 0 waits for its members):
            // counted, and handled the same way, since after the drain no member
            // of the old instance is left to finish it. The same when the members
            // of the instance left (a lone lead) before this gang request: the lead
            // is told to leave too, and the op goes to a new instance.
            const unsigned long long ex = svc_word(&s.svc->exited);
            const unsigned long long ln = active > 1 ? svc_word(&s.svc->lone) : 0;
            if (ex || (ln && ln <= seq)) {
                DeviceGuard g(s.device);
                if (!ex) {
                    service_store_seq(s.svc_req, kServiceStop);
                    if (s.svc_greq) service_store_seq(s.svc_greq, kServiceStop, s.svc_greq_copies);
                }
                if (lane_drain(s.svc_lanes[(size_t)s.svc_lane], s.svc_drain_ns, kDrainRepost) != 0)
                    return service_abort(seq, active, "left part of a request behind and did not drain");
                s.svc_running = false;
                s.svc_relaunches++;
                if (finished()) {
                    s.svc_ops++;
                    return 0;
                }
                if (ex > seq) s.svc_incomplete_exits++;
                // Members may have counted part of the request in: start from a clean box.
                s.svc_lanes[(size_t)s.svc_lane].dirty = true;
                // Re-post under a fresh seq. Direct gang members of the instance that
                // left may have served part of this request and stored its seq in their
                // WGDONE words; under the old seq those stale words would count as the
                // new instance's members finishing, and the op would return while some
                // of them were still copying (a later write to the local half then raced
                // the copy: tests/test_gpu_service.py::test_service_direct_and_relayed_gangs_interleave).
                seq = ++s.svc_seq;
                if (service_start(seq) != 0) return -1;
                if (size_and_post() != 0) return -1;  // sized to the new instance's roster; start cleared the doorbell
            }
            if (now_ns() - t0 > s.svc_timeout_ns) return service_abort(seq, active, "did not complete a transfer in time");
        }
    }
}

// One-sided transfer between the linear buffer `lin` (location `lloc`) and the
// remote half of `a` at striped offset `rem_off`.
int wait_done(const XferDone &d, hipEvent_t ev) {
    for (unsigned spins = 1;; spins++) {
        if ((long long)(__atomic_load_n(d.flag, __ATOMIC_ACQUIRE) - d.val) >= 0) return 0;
        if ((spins & 4095) == 0) {
            // Backstop: the runtime saw the kernel end (the flag is then set, or
            // the kernel had nothing to publish); errors surface here too.
            const hipError_t e = hipEventQuery(ev);
            if (e == hipSuccess) return 0;
            if (e != hipErrorNotReady) OCM_FAIL(-1, "event wait: %s", hipGetErrorString(e));
        }
    }
}

int xfer(lib_alloc *a, bool put, char *lin, Loc lloc, uint64_t rem_off, uint64_t len, bool async, XferDone *done) {
    State &s = S();
    if (done) *done = XferDone{};
    if (len == 0) return 0;
    if (a->any_net) {
        // Another node: stream every piece through its owner's data server (blocking).
        std::vector<Seg> segs;
        segments(a, rem_off, len, segs);
        if (wait_alloc(a) != 0) return -1;
        if (honor_dep(a, nullptr, true) != 0) return -1;
        for (auto &g : segs) {
            const Extent &e = a->ext[g.ext];
            if (e.net) {
                if (net_piece(e, put, lin + g.lin_off, lloc, g.ext_off, g.len) != 0) return -1;
                continue;
            }
            // mixed placement: this piece is on this node
            char *r = (lloc == LOC_DEVICE || e.r.tier == TIER_GPU) ? e.dptr : e.hptr;
            r += g.ext_off;
            if (s.device < 0 || (lloc != LOC_DEVICE && e.r.tier != TIER_GPU)) {
                std::memcpy(put ? r : lin + g.lin_off, put ? lin + g.lin_off : r, g.len);
            } else {
                DeviceGuard dg(s.device);
                if ((put ? hipMemcpyAsync(r, lin + g.lin_off, g.len, hipMemcpyDefault, s.stream)
                         : hipMemcpyAsync(lin + g.lin_off, r, g.len, hipMemcpyDefault, s.stream)) != hipSuccess)
                    OCM_FAIL(-1, "transfer launch failed");
                if (sync_stream() != 0) return -1;
            }
        }
        return 0;
    }
    std::vector<Seg> segs;
    if (s.device < 0) {
        segments(a, rem_off, len, segs);
        for (auto &g : segs) {
            char *r = a->ext[g.ext].hptr + g.ext_off;
            if (put)
                std::memcpy(r, lin + g.lin_off, g.len);
            else
                std::memcpy(lin + g.lin_off, r, g.len);
        }
        return 0;
    }
    DeviceGuard guard(s.device);
    const bool lin_dev = lloc == LOC_DEVICE;
    // Every extent kind goes through the repo's own kernels: HBM extents the
    // register / LDS-DMA kernels, host-tier extents the PCIe streaming kernel
    // (57.0-57.4 GB/s, at or above the runtime's copy at 56.8-57.1:
    // profiles/pcie_stream_r03.json). OCM_HOST_ENGINE=sdma keeps the runtime's
    // copy engines for host-tier pairs as a measured baseline.
    const XferTuning &dt = s.dir_tuning[put ? 1 : 0];
    const bool dma_pick = (dt.variant != XFER_AUTO ? dt.variant : s.tuning.variant) == XFER_DMA;
    const bool use_kernel =
        lin_dev && !dma_pick && (a->any_gpu || s.host_engine_kernel || len <= s.host_kernel_max);
    hipError_t err = hipSuccess;
    // Small blocking ops go to the resident copy service (no launch, no stream sync).
    if (lin_dev && a->all_dev_ok && !async && len <= s.svc_limit(a) && !dma_pick) {
        XferArgs x;
        std::memset(&x, 0, sizeof(x));
        x.lin = lin;
        for (size_t i = 0; i < a->ext.size(); i++) x.ext[i] = a->ext[i].dptr;
        x.n_ext = (uint32_t)a->ext.size();
        x.rem_off = rem_off;
        x.len = len;
        x.put = put ? 1 : 0;
        if (x.n_ext > 1) x.unit_shift = (uint32_t)log2_exact(a->stripe_unit);
        if (wait_alloc(a) != 0) return -1;  // keep program order with queued async ops
        if (honor_dep(a, nullptr, true) != 0) return -1;
        // Gets from the host tier are bound by PCIe read round trips: two tiles
        // already go faster on two workgroups (64 KiB: 7.7 vs 8.4 us); puts and
        // HBM owners keep small requests on workgroup 0 (profiles/svc_v4_r02.json).
        const unsigned solo = (!put && !a->any_gpu) ? std::min(s.svc_solo_tiles, s.svc_solo_tiles_host_get)
                                                    : s.svc_solo_tiles;
        const int rc = service_xfer(x, solo, a->any_gpu, a->any_peer || s.svc_force_strict);
        if (rc == 0) return 0;
        // -2: an instance may still hold the request; a launch now would race it.
        if (rc == -2) return -1;
        // -1: nothing holds the request any more (never launched, or drained after STOP).
        OCM_WARN("copy service failed (%s); falling back to launches", last_error());
        s.svc_max = 0;
    }
    // Async ops queue on the allocation's lane; blocking ops on the library stream
    // after the allocation's queued async work.
    if (!async && wait_alloc(a) != 0) return -1;
    hipStream_t st = async ? lane_stream(a) : s.stream;
    if (honor_dep(a, st, false) != 0) return -1;
    const XferTuning &getdt = s.dir_tuning[0];
    if (use_kernel && !put && a->all_gpu && !a->any_net &&
        (getdt.variant != XFER_AUTO ? getdt.variant : s.tuning.variant) == XFER_PUSH) {
        before_launch();
        if (push_get(a, lin, rem_off, len, st, async) != 0) return -1;
        if (async) {
            if (st != s.stream && a->ev) {
                err = hipEventRecord(a->ev, st);
                if (err != hipSuccess) OCM_FAIL(-1, "event record failed: %s", hipGetErrorString(err));
            } else if (a->ev == nullptr && sync_stream() != 0) {
                return -1;
            }
            a->async_pending = a->ev != nullptr;
        }
        return 0;
    }
    if (use_kernel) {
        // No resident poller during a large copy over PCIe (its doorbell reads share
        // the link) or when asked (A/B); without a queue of its own the service
        // would also hold this launch until its idle exit.
        if ((s.svc_park_kernel || !a->any_gpu) && len > s.svc_limit(a)) service_park();
        before_launch();
        XferArgs x;
        std::memset(&x, 0, sizeof(x));
        x.lin = lin;
        for (size_t i = 0; i < a->ext.size(); i++) x.ext[i] = a->ext[i].dptr;
        x.n_ext = (uint32_t)a->ext.size();
        x.rem_off = rem_off;
        x.len = len;
        x.put = put ? 1 : 0;
        if (x.n_ext > 1) {
            int sh = log2_exact(a->stripe_unit);
            if (sh < 0) OCM_FAIL(-1, "stripe unit %llu is not a power of two", (unsigned long long)a->stripe_unit);
            x.unit_shift = (uint32_t)sh;
        }
        XferTuning t = s.dir_tuning[put ? 1 : 0].variant != XFER_AUTO ? s.dir_tuning[put ? 1 : 0] : s.tuning;
        if (t.variant == XFER_AUTO) {
            // Measured (profiles/ksweep_r01.json): LDS-DMA staging wins HBM->HBM
            // copies up to ~256 MiB on the same GPU; everything else (peer HBM
            // over xGMI, host-mapped memory, huge copies) uses the register path.
            bool same_gpu = lloc == LOC_DEVICE;
            for (auto &e : a->ext) same_gpu &= e.r.tier == TIER_GPU && e.r.owner_gpu == s.device;
            t.variant = !a->any_gpu ? XFER_PCIE : (same_gpu && len <= (256ull << 20)) ? XFER_LDS : XFER_REG;
        }
        XferDone dn;
        if (done && async && len <= s.launch_flag_max && s.launch_flags && s.lane_flags && st != s.stream &&
            a->lane >= 0 && a->ev) {
            dn.flag = s.lane_flags + (size_t)a->lane * 16;
            dn.cnt = s.lane_cnt + (size_t)a->lane * 32;
            dn.val = ++s.lane_flag_seq[(size_t)a->lane];
        }
        err = xfer_launch(x, t, st, dn.flag ? &dn : nullptr);
        if (err == hipSuccess && done) *done = dn;
    } else {
        service_park();
        segments(a, rem_off, len, segs);
        // Pieces between a host-resident local half and the host tier are copied
        // by this thread right away: first let the work they must follow finish
        // (an ocm_stream_wait dependency and earlier async ops, both queued on st).
        bool cpu_piece = false;
        for (auto &g : segs) cpu_piece |= lloc != LOC_DEVICE && a->ext[g.ext].r.tier != TIER_GPU;
        if (cpu_piece && (err = hipStreamSynchronize(st)) != hipSuccess)
            OCM_FAIL(-1, "ordering a host copy after queued work: %s", hipGetErrorString(err));
        for (auto &g : segs) {
            const Extent &e = a->ext[g.ext];
            char *r = (lloc == LOC_DEVICE || e.r.tier == TIER_GPU) ? e.dptr : e.hptr;
            r += g.ext_off;
            if (lloc != LOC_DEVICE && e.r.tier != TIER_GPU) {
                // host <-> host tier: the CPU is the fastest engine.
                if (put)
                    std::memcpy(r, lin + g.lin_off, g.len);
                else
                    std::memcpy(lin + g.lin_off, r, g.len);
                continue;
            }
            err = put ? hipMemcpyAsync(r, lin + g.lin_off, g.len, hipMemcpyDefault, st)
                      : hipMemcpyAsync(lin + g.lin_off, r, g.len, hipMemcpyDefault, st);
            if (err != hipSuccess) break;
        }
    }
    if (err != hipSuccess) OCM_FAIL(-1, "transfer launch failed: %s", hipGetErrorString(err));
    if (async) {
        if (st != s.stream && a->ev) {
            err = hipEventRecord(a->ev, st);
            if (err != hipSuccess) OCM_FAIL(-1, "event record failed: %s", hipGetErrorString(err));
        } else if (a->ev == nullptr && sync_stream() != 0) {
            return -1;  // no lane available: complete it now
        }
        a->async_pending = a->ev != nullptr;
        return 0;
    }
    return sync_stream();
}

// ---- push-based get (XFER_PUSH) ----
// RDMA READ vs WRITE (reference src/rdma.c:240-263): over xGMI a remote write is
// usually cheaper than a remote read, so a get can be turned into pushes. For
// every owner GPU d of the pair's extents, this process launches a kernel on d
// (a stream of its own there) that reads d's extents from d's HBM and stores
// them into the local half over xGMI. The owner's CPU and daemon take no part.
// Needs: the slab mapped on d (extent_view: a second IPC open by d's context),
// peer access d -> this GPU and, for a pool-allocated local half, pool access
// for d (local_pool() grants it to every peer at creation).

void push_release() {
    State &s = S();
    for (auto &kv : s.push) {
        DeviceGuard g(kv.first);
        if (kv.second.stream) (void)hipStreamSynchronize(kv.second.stream);
    }
}

static PushDev *push_dev(int d) {
    State &s = S();
    PushDev &p = s.push[d];
    if (p.ready) return &p;
    DeviceGuard g(d);
    if (d != s.device) {
        int can = 0;
        if (hipDeviceCanAccessPeer(&can, d, s.device) != hipSuccess || !can)
            OCM_FAIL(nullptr, "push get: GPU %d cannot reach GPU %d", d, s.device);
        const hipError_t pe = hipDeviceEnablePeerAccess(s.device, 0);
        if (pe != hipSuccess && pe != hipErrorPeerAccessAlreadyEnabled)
            OCM_FAIL(nullptr, "push get: peer access %d -> %d: %s", d, s.device, hipGetErrorString(pe));
        (void)hipGetLastError();
    }
    if (!p.stream && hipStreamCreateWithFlags(&p.stream, hipStreamNonBlocking) != hipSuccess)
        OCM_FAIL(nullptr, "push get: no stream on GPU %d", d);
    if (!p.done && hipEventCreateWithFlags(&p.done, hipEventDisableTiming) != hipSuccess)
        OCM_FAIL(nullptr, "push get: no event on GPU %d", d);
    p.ready = true;
    return &p;
}

int push_get(lib_alloc *a, char *lin, uint64_t rem_off, uint64_t len, hipStream_t st, bool async) {
    State &s = S();
    if (!a->all_gpu || a->any_net) OCM_FAIL(-1, "push get needs every extent in a GPU's HBM");
    std::map<int, uint32_t> owners;  // device -> extent mask
    for (size_t i = 0; i < a->ext.size(); i++) {
        const int d = a->ext[i].r.owner_gpu;
        if (d < 0) OCM_FAIL(-1, "push get: extent %zu has no owner GPU", i);
        owners[d] |= 1u << i;
    }
    DeviceGuard g(s.device);
    if (!s.push_order && hipEventCreateWithFlags(&s.push_order, hipEventDisableTiming) != hipSuccess)
        OCM_FAIL(-1, "push get: no event");
    if (hipEventRecord(s.push_order, st) != hipSuccess) OCM_FAIL(-1, "push get: ordering event");
    std::vector<PushDev *> used;
    for (auto &kv : owners) {
        const int d = kv.first;
        PushDev *p = push_dev(d);
        if (!p) return -1;
        XferArgs x;
        std::memset(&x, 0, sizeof(x));
        x.lin = lin;  // the local half: peer-accessible from d (peer access + pool access)
        for (size_t i = 0; i < a->ext.size(); i++) {
            if (!((kv.second >> i) & 1u)) continue;
            x.ext[i] = extent_view(a->ext[i], d);
            if (!x.ext[i]) return -1;
        }
        x.n_ext = (uint32_t)a->ext.size();
        x.rem_off = rem_off;
        x.len = len;
        x.put = 0;
        if (x.n_ext > 1) x.unit_shift = (uint32_t)log2_exact(a->stripe_unit);
        DeviceGuard gd(d);
        hipError_t e = hipStreamWaitEvent(p->stream, s.push_order, 0);  // after the work queued before this op
        if (e == hipSuccess) e = xfer_push_launch(x, kv.second, s.dir_tuning[0].max_blocks, p->stream);
        if (e == hipSuccess) e = hipEventRecord(p->done, p->stream);
        if (e != hipSuccess) OCM_FAIL(-1, "push get on GPU %d: %s", d, hipGetErrorString(e));
        used.push_back(p);
        s.push_launches++;
    }
    for (PushDev *p : used) {
        const hipError_t e = async ? hipStreamWaitEvent(st, p->done, 0) : hipEventSynchronize(p->done);
        if (e != hipSuccess) OCM_FAIL(-1, "push get completion: %s", hipGetErrorString(e));
    }
    return 0;
}

// Copy between two process-local buffers.
int copy_local(void *dst, Loc dl, const void *src, Loc sl, size_t n) {
    State &s = S();
    if (n == 0) return 0;
    if (dl != LOC_DEVICE && sl != LOC_DEVICE) {
        std::memcpy(dst, src, n);
        return 0;
    }
    DeviceGuard g(s.device);
    hipError_t e;
    before_launch();
    if (dl == LOC_DEVICE && sl == LOC_DEVICE) {
        XferTuning t = s.tuning;
        if (t.variant == XFER_AUTO) t.variant = n <= (256ull << 20) ? XFER_LDS : XFER_REG;
        e = xfer_copy(dst, src, n, t, s.stream);
    } else
    {
        e = hipMemcpyAsync(dst, src, n, hipMemcpyDefault, s.stream);
    }
    if (e != hipSuccess) OCM_FAIL(-1, "local copy failed: %s", hipGetErrorString(e));
    return sync_stream();
}


}  // namespace ocmlib

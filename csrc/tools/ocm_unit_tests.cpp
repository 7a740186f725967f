// Native unit tests (no daemon, no GPU): wire layout, nodefile, range
// allocator, governor placement policies, stripe geometry, host-tier arena,
// tick slot tags and the tick transport's state machine over a 1-rank socket
// collective (plain and batched).
// Prints one line per test and exits non-zero on the first failure.
#include <sys/mman.h>
#include <unistd.h>

#include <cerrno>
#include <chrono>
#include <cstdlib>
#include <thread>
#include <cstdio>
#include <cstring>
#include <functional>
#include <random>
#include <set>
#include <string>
#include <vector>

#include "oncillamem.h"
#include "ocm/arena.h"
#include "ocm/governor.h"
#include "ocm/msg.h"
#include "ocm/nodefile.h"
#include "ocm/range_alloc.h"
#include "ocm/shmlink.h"
#include "ocm/siphash.h"
#include "ocm/tick.h"

using namespace ocm;

static int g_fail = 0;
#define CHECK(c)                                                        \
    do {                                                                \
        if (!(c)) {                                                     \
            fprintf(stderr, "  CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
            g_fail++;                                                   \
            return;                                                     \
        }                                                               \
    } while (0)

static void t_layout() {
    CHECK(sizeof(Msg) == 160);
    CHECK(sizeof(struct ocm_params) == 48);
    CHECK(sizeof(struct ocm_alloc_params) == 24);
    CHECK(OCM_LOCAL_HOST == 1 && OCM_REMOTE_GPU == 7 && OCM_REMOTE_RDMA == 5);
    CHECK(std::string(msg_type_str(MSG_DO_ALLOC)) == "MSG_DO_ALLOC");
}

static void t_nodefile() {
    NodeFile nf;
    std::string err;
    const char *ref = "#rank dns ethernet_ip ocm_port rdmacm_port\n"
                      "0 shiva.cc 143.215.131.65 12345 67890\n"
                      "1 ifrit.cc 143.215.131.185 12345 67890\n";
    CHECK(parse_nodefile_text(ref, &nf, &err) == 0);
    CHECK(nf.size() == 2 && nf.nodes[1].dns == "ifrit.cc" && nf.nodes[1].ocm_port == 12345);
    CHECK(nf.nodes[0].data_port == 67890 && nf.nodes[0].gpu == -1);
    const char *rma = "#rank dns ethernet_ip ocm_port\n0 peac14 192.168.1.114 12345\n1 peac15 192.168.1.115 12345\n";
    CHECK(parse_nodefile_text(rma, &nf, &err) == 0 && nf.size() == 2);
    const char *gpu = "0 n 127.0.0.1 5000 0 gpu=3\n1 n 127.0.0.1 5001 0 4  # comment\n";
    CHECK(parse_nodefile_text(gpu, &nf, &err) == 0 && nf.nodes[0].gpu == 3 && nf.nodes[1].gpu == 4);
    CHECK(resolve_rank(nf, 1, &err) == 1);
    CHECK(resolve_rank(nf, 5, &err) == -1);
    CHECK(parse_nodefile_text("0 a b notaport\n", &nf, &err) == -1);
    CHECK(parse_nodefile_text("0 a b 1\n0 a b 2\n", &nf, &err) == -1);  // duplicate rank
    CHECK(parse_nodefile_text("1 a b 1\n", &nf, &err) == -1);            // not dense
    CHECK(parse_nodefile_text("# only comments\n", &nf, &err) == -1);
}

static void t_range_alloc() {
    RangeAllocator ra(1 << 20);
    uint64_t a, b, c;
    CHECK(ra.alloc(1000, 4096, &a) && a == 0);
    CHECK(ra.alloc(5000, 4096, &b) && b == 4096);
    CHECK(ra.alloc(4096, 4096, &c) && c % 4096 == 0);
    CHECK(!ra.alloc(2 << 20, 4096, &a));
    CHECK(ra.free(b) && !ra.free(b));
    CHECK(ra.free(0) && ra.free(c));
    CHECK(ra.used() == 0 && ra.num_free_ranges() == 1 && ra.largest_free() == (1u << 20));
    // random churn keeps accounting exact and ranges disjoint
    std::mt19937 g(7);
    std::vector<std::pair<uint64_t, uint64_t>> live;
    uint64_t used = 0;
    for (int i = 0; i < 5000; i++) {
        if (live.empty() || g() % 3) {
            uint64_t n = 1 + g() % 20000, off;
            if (ra.alloc(n, 256, &off)) {
                for (auto &l : live) CHECK(off + n <= l.first || l.first + l.second <= off);
                live.push_back({off, n});
                used += n;
            }
        } else {
            size_t k = g() % live.size();
            CHECK(ra.free(live[k].first));
            used -= live[k].second;
            live.erase(live.begin() + (long)k);
        }
        CHECK(ra.used() == used);
    }
    for (auto &l : live) CHECK(ra.free(l.first));
    CHECK(ra.used() == 0 && ra.num_free_ranges() == 1);
}

static NodeConfig cfg(int rank, uint64_t gpu, uint64_t host) {
    NodeConfig c;
    std::memset(&c, 0, sizeof(c));
    c.rank = rank;
    c.gpu = gpu ? rank : -1;
    c.gpu_capacity = gpu;
    c.host_capacity = host;
    return c;
}

static void t_governor() {
    const uint64_t G = 1ull << 30;
    {  // ring: (orig + 1) % N, the reference policy
        Governor gov(4, Policy::Ring, 1 << 20);
        for (int r = 0; r < 4; r++) gov.add_node(cfg(r, 8 * G, G));
        PlaceRequest pr;
        pr.orig_rank = 3;
        pr.bytes = G;
        Placement p = gov.place(pr);
        CHECK(p.err == 0 && p.extents.size() == 1 && p.extents[0].owner == 0 && p.extents[0].tier == TIER_GPU);
        pr.remote_rank = 2;  // explicit owner honoured
        p = gov.place(pr);
        CHECK(p.extents[0].owner == 2);
        CHECK(gov.node(2).gpu_reserved == G);
        CHECK(gov.release(p.alloc_id) && gov.node(2).gpu_reserved == 0);
        CHECK(!gov.release(p.alloc_id));
    }
    {  // spill to the host tier when HBM is exhausted, then ENOMEM
        Governor gov(2, Policy::Ring, 1 << 20);
        gov.add_node(cfg(0, 2 * G, 4 * G));
        gov.add_node(cfg(1, 2 * G, 1 * G));
        PlaceRequest pr;
        pr.orig_rank = 0;
        pr.bytes = 2 * G;
        Placement a = gov.place(pr);
        CHECK(a.err == 0 && a.extents[0].owner == 1 && a.extents[0].tier == TIER_GPU);
        Placement b = gov.place(pr);  // rank1 full -> rank0 HBM? (fallback peers exclude origin) -> host tier
        CHECK(b.err == 0 && b.extents[0].tier == TIER_HOST && b.extents[0].spilled);
        CHECK(gov.spilled_count() == 1);
        pr.flags = OCM_ALLOC_NO_SPILL;
        Placement c = gov.place(pr);
        CHECK(c.err == ENOMEM);
        pr.flags = 0;
        pr.bytes = 100 * G;
        CHECK(gov.place(pr).err == ENOMEM);
    }
    {  // stripe over every peer, extents sum to the request
        Governor gov(8, Policy::Stripe, 1 << 20);
        for (int r = 0; r < 8; r++) gov.add_node(cfg(r, 8 * G, G));
        PlaceRequest pr;
        pr.orig_rank = 5;
        pr.bytes = 3 * G + 12345;
        Placement p = gov.place(pr);
        CHECK(p.err == 0 && p.extents.size() == 7 && p.stripe_unit == (1u << 20));
        uint64_t sum = 0;
        std::set<int> owners;
        for (auto &e : p.extents) {
            sum += e.bytes;
            owners.insert(e.owner);
            CHECK(e.owner != 5);
        }
        CHECK(sum == pr.bytes && owners.size() == 7);
        pr.bytes = 2 << 20;  // smaller than 7 units: only 2 extents
        CHECK(gov.place(pr).extents.size() == 2);
        pr.stripe_width = 3;
        pr.bytes = G;
        CHECK(gov.place(pr).extents.size() == 3);
    }
    {  // single node: remote requests land in the host tier
        Governor gov(1, Policy::Ring, 1 << 20);
        gov.add_node(cfg(0, 8 * G, G));
        PlaceRequest pr;
        pr.orig_rank = 0;
        pr.bytes = 1 << 20;
        Placement p = gov.place(pr);
        CHECK(p.err == 0 && p.extents[0].owner == 0 && p.extents[0].tier == TIER_HOST);
        pr.flags = OCM_ALLOC_LOOPBACK;
        p = gov.place(pr);
        CHECK(p.extents[0].owner == 0 && p.extents[0].tier == TIER_GPU);
    }
    {  // least loaded + dead nodes are skipped + re-placement
        Governor gov(3, Policy::LeastLoaded, 1 << 20);
        gov.add_node(cfg(0, 8 * G, G));
        gov.add_node(cfg(1, 2 * G, G));
        gov.add_node(cfg(2, 6 * G, G));
        PlaceRequest pr;
        pr.orig_rank = 0;
        pr.bytes = G;
        Placement p = gov.place(pr);
        CHECK(p.extents[0].owner == 2);
        gov.mark_dead(2);
        p = gov.place(pr);
        CHECK(p.extents[0].owner == 1);
        PlacedExtent e;
        CHECK(gov.replace_extent(p.alloc_id, 0, 1, &e) && e.owner != 1);
        CHECK(gov.allocations_from(0).size() == 2);
    }
}

static void t_governor_hosts() {
    const uint64_t G = 1ull << 30;
    Governor gov(4, Policy::Stripe, 1 << 20);
    for (int r = 0; r < 4; r++) {
        NodeConfig c = cfg(r, 8 * G, G);
        std::snprintf(c.host, sizeof(c.host), "%s", r < 2 ? "nodeA" : "nodeB");
        gov.add_node(c);
    }
    PlaceRequest pr;
    pr.orig_rank = 0;
    pr.bytes = 64 << 20;
    Placement p = gov.place(pr);
    CHECK(p.err == 0 && p.extents.size() == 1 && p.extents[0].owner == 1);  // only the same-host peer
    pr.orig_rank = 3;
    p = gov.place(pr);
    CHECK(p.err == 0 && p.extents.size() == 1 && p.extents[0].owner == 2);
    CHECK(!p.extents[0].net);
    pr.remote_rank = 0;  // explicit owner on the other host: network tier
    p = gov.place(pr);
    CHECK(p.err == 0 && p.extents[0].owner == 0 && p.extents[0].net);
    // one daemon per host (the reference layout): ring to the next node
    Governor g2(2, Policy::Ring, 1 << 20);
    for (int r = 0; r < 2; r++) {
        NodeConfig c = cfg(r, 8 * G, G);
        std::snprintf(c.host, sizeof(c.host), "host%d", r);
        g2.add_node(c);
    }
    PlaceRequest q;
    q.orig_rank = 1;
    q.bytes = 1 << 20;
    p = g2.place(q);
    CHECK(p.err == 0 && p.extents[0].owner == 0 && p.extents[0].net && p.extents[0].tier == TIER_GPU);
}

static void t_governor_checkpoint() {
    const uint64_t G = 1ull << 30;
    Governor gov(3, Policy::Ring, 1 << 20);
    for (int r = 0; r < 3; r++) gov.add_node(cfg(r, 4 * G, G), 100 + r);
    PlaceRequest pr;
    pr.orig_rank = 1;
    pr.bytes = G;
    Placement a = gov.place(pr), b = gov.place(pr);
    CHECK(a.err == 0 && b.err == 0 && a.extents[0].owner == 2 && b.extents[0].owner == 2);
    const std::string snap = gov.checkpoint();
    std::string err;
    // a truncated file is refused, not half-loaded
    Governor bad(3, Policy::Ring, 1 << 20);
    CHECK(bad.restore(snap.substr(0, snap.size() - 4), &err) < 0);
    CHECK(bad.restore("garbage", &err) < 0);
    // resume: rank 2 rejoins with the same boot id and confirms only `a`
    Governor g2(3, Policy::Ring, 1 << 20);
    CHECK(g2.restore(snap, &err) == 2);
    g2.add_node(cfg(0, 4 * G, G), 999);  // rank0 restarted
    g2.add_node(cfg(1, 4 * G, G), 101);
    g2.add_node(cfg(2, 4 * G, G), 102);
    CHECK(g2.node(2).gpu_reserved == 0);  // nothing held until confirmed
    Region r{};
    r.alloc_id = a.alloc_id;
    r.bytes = G;
    r.orig_rank = 1;
    r.tier = TIER_GPU;
    r.n_extents = 1;
    g2.confirm_extent(2, r, 77);
    CHECK(g2.node(2).gpu_reserved == G);
    CHECK(g2.end_reconcile(2) == 1);  // b was freed while rank0 was away
    CHECK(g2.find(a.alloc_id) && !g2.find(b.alloc_id));
    // new ids continue after the restored ones
    Placement c = g2.place(pr);
    CHECK(c.err == 0 && c.alloc_id > b.alloc_id && g2.node(2).gpu_reserved == 2 * G);
    CHECK(g2.release(a.alloc_id) && g2.node(2).gpu_reserved == G);
    // an owner that comes back as a new process lost its memory
    g2.add_node(cfg(2, 4 * G, G), 555);
    CHECK(!g2.find(c.alloc_id) && g2.node(2).gpu_reserved == 0);
}

static void t_stripe_geometry() {
    for (uint64_t total : {1ull, 4095ull, 4096ull, 1000000ull, (3ull << 20) + 7}) {
        for (int n = 1; n <= 8; n++) {
            uint64_t sum = 0;
            for (int i = 0; i < n; i++) sum += stripe_extent_bytes(total, 4096, n, i);
            CHECK(sum == total);
        }
    }
    CHECK(stripe_extent_bytes(10000, 4096, 2, 0) == 4096 + (10000 - 8192));
    CHECK(stripe_extent_bytes(10000, 4096, 2, 1) == 4096);
}

static void t_arena_host() {
    ArenaConfig ac;
    ac.gpu = -1;
    ac.host_capacity = 64ull << 20;
    ac.slab_bytes = 16ull << 20;
    Arena ar(ac);
    Region r1, r2, r3;
    std::memset(&r1, 0, sizeof(r1));
    std::memset(&r2, 0, sizeof(r2));
    std::memset(&r3, 0, sizeof(r3));
    CHECK(ar.alloc(TIER_HOST, 1 << 20, &r1) == 0);
    CHECK(ar.alloc(TIER_HOST, 1 << 20, &r2) == 0);
    CHECK(r1.slab_id == r2.slab_id && r1.offset != r2.offset);
    CHECK(ar.alloc(TIER_GPU, 1 << 20, &r3) != 0);  // no GPU tier on a CPU daemon
    CHECK(ar.alloc(TIER_HOST, 12ull << 20, &r3) == 0 && (r3.flags & REGION_DEDICATED));
    CHECK(ar.used(TIER_HOST) == (14ull << 20));
    CHECK(ar.alloc(TIER_HOST, 60ull << 20, &r3) == ENOMEM);
    // the exported handle is a path another process can open
    char path[65] = {0};
    std::memcpy(path, r1.handle, 64);
    CHECK(std::string(path).find("/proc/") == 0 && access(path, R_OK | W_OK) == 0);
    std::memset(ar.resolve(r1.slab_id, r1.offset), 0xab, 1 << 20);
    CHECK(ar.free(r1.slab_id, r1.offset) == 0 && ar.free(r1.slab_id, r1.offset) == ENOENT);
    CHECK(ar.free(r2.slab_id, r2.offset) == 0);
}

// xGMI topology: rank0 places on the nearest peer GPU (hops from the origin's
// GPU), ring order among equals; stripes take the nearest peers first.
static void t_governor_topology() {
    const uint64_t G = 1ull << 30;
    auto links = [](int rank, std::vector<int> h) {
        NodeLinks l;
        std::memset(&l, 0, sizeof(l));
        l.rank = rank;
        l.gpu = rank;
        l.n = (uint32_t)h.size();
        std::memset(l.hops, kHopsUnknown, sizeof(l.hops));
        for (size_t i = 0; i < h.size(); i++) l.hops[i] = h[i] < 0 ? kHopsUnknown : (uint8_t)h[i];
        return l;
    };
    {  // ring from rank 0: (0+1) % 4 would be rank 1 (2 hops); rank 2 is 1 hop away
        Governor gov(4, Policy::Ring, 1 << 20);
        for (int r = 0; r < 4; r++) gov.add_node(cfg(r, 8 * G, G));
        gov.set_links(links(0, {-1, 2, 1, 2}));
        CHECK(gov.hops(0, 2) == 1 && gov.hops(0, 1) == 2 && gov.hops(1, 0) == kHopsUnknown);
        PlaceRequest pr;
        pr.orig_rank = 0;
        pr.bytes = G;
        Placement p = gov.place(pr);
        CHECK(p.err == 0 && p.extents[0].owner == 2);
        pr.orig_rank = 1;  // no table for rank 1: reference ring order
        CHECK(gov.place(pr).extents[0].owner == 2);
    }
    {  // least loaded: equal free capacity -> the 1-hop peer; more free space still wins
        Governor gov(4, Policy::LeastLoaded, 1 << 20);
        for (int r = 0; r < 4; r++) gov.add_node(cfg(r, 8 * G, G));
        gov.set_links(links(0, {-1, 3, 3, 1}));
        PlaceRequest pr;
        pr.orig_rank = 0;
        pr.bytes = G;
        CHECK(gov.place(pr).extents[0].owner == 3);
        CHECK(gov.place(pr).extents[0].owner == 1);  // rank 3 now has less free HBM
    }
    {  // stripe width 2 takes the two nearest peers
        Governor gov(5, Policy::Stripe, 1 << 20);
        for (int r = 0; r < 5; r++) gov.add_node(cfg(r, 8 * G, G));
        gov.set_links(links(0, {-1, 2, 2, 1, 1}));
        PlaceRequest pr;
        pr.orig_rank = 0;
        pr.bytes = 8 << 20;
        pr.stripe_width = 2;
        Placement p = gov.place(pr);
        std::set<int> owners;
        for (auto &e : p.extents) owners.insert(e.owner);
        CHECK(p.err == 0 && owners == std::set<int>({3, 4}));
    }
}

// SipHash-2-4 reference vectors (key 00..0f; messages "" and 00..0e), and the
// HELLO record fits the 160 B wire format.
static void t_siphash() {
    const SipKey k{0x0706050403020100ull, 0x0f0e0d0c0b0a0908ull};
    uint8_t m[15];
    for (int i = 0; i < 15; i++) m[i] = (uint8_t)i;
    CHECK(siphash24(k, m, 0) == 0x726fdb47dd0e0e31ull);
    CHECK(siphash24(k, m, 15) == 0xa129ca6149be45e5ull);
    const SipKey a = sip_derive_key("ns\x1fsecret"), b = sip_derive_key("ns\x1fsecreT");
    CHECK((a.k0 != b.k0 || a.k1 != b.k1) && a.k0 != a.k1);
    CHECK(offsetof(Msg, u.hello.mac) == 32 + 24);
}

// The app <-> daemon shared-memory link (ocm/shmlink.h): order across ring
// wrap-around, full rings, the wake-up flags, and what a hostile app can write
// (forged slot numbers, a bogus count of replies taken, a wrong magic).
static void t_shmlink() {
    ShmLink app, dmn;
    CHECK(app.create() == 0);
    CHECK(dmn.attach(dup(app.fd())) == 0);
    const size_t bytes = (sizeof(ShmLinkLayout) + 4095) & ~size_t(4095);
    auto *raw = static_cast<ShmLinkLayout *>(mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_SHARED, app.fd(), 0));
    CHECK(raw != MAP_FAILED);
    auto rec = [](uint64_t i) {
        Msg m;
        std::memset(&m, 0, sizeof(m));
        m.type = MSG_PING;
        m.seq = i;
        m.u.raw[0] = (uint8_t)(i * 7);
        return m;
    };
    // requests in bursts of 1..64 with wrap-around, taken in order
    uint64_t posted = 0, taken = 0;
    std::mt19937 rng(5);
    for (int round = 0; round < 50; round++) {
        const int burst = 1 + (int)(rng() % kShmLinkSlots);
        for (int k = 0; k < burst; k++) CHECK(app.post_request(rec(++posted)));
        CHECK(dmn.requests_pending());
        Msg m;
        while (dmn.take_request(&m)) {
            ++taken;
            CHECK(m.seq == taken && m.u.raw[0] == (uint8_t)(taken * 7));
        }
        CHECK(taken == posted && !dmn.requests_pending());
    }
    // a full request ring refuses the next record until one is taken
    for (uint32_t k = 0; k < kShmLinkSlots; k++) CHECK(app.post_request(rec(++posted)));
    CHECK(!app.post_request(rec(posted + 1)));
    Msg m;
    CHECK(dmn.take_request(&m) && m.seq == ++taken);
    CHECK(app.post_request(rec(++posted)));
    while (dmn.take_request(&m)) CHECK(m.seq == ++taken);
    CHECK(taken == posted);
    // replies: the same, and a bogus count of replies taken reads as a full ring
    for (uint64_t i = 1; i <= 200; i++) {
        CHECK(dmn.post_reply(rec(i)));
        CHECK(app.replies_pending() && app.take_reply(&m) && m.seq == i);
    }
    raw->rsp_taken.store(1ull << 40);
    int ok = 0;
    while (ok < 1000 && dmn.post_reply(rec(1000 + ok))) ok++;
    CHECK(ok <= (int)kShmLinkSlots);  // never more than one ring's worth past the app
    // a forged slot number ahead of the daemon's count is not a record
    const uint64_t next = taken + 1;
    raw->req[(next - 1) % kShmLinkSlots].seq.store(next + 5);
    CHECK(!dmn.requests_pending() && !dmn.take_request(&m));
    // the wake-up flags (Dekker): a sleeping daemon must be woken, an awake one not
    dmn.set_daemon_polling(false);
    CHECK(app.request_needs_wake());
    dmn.set_daemon_polling(true);
    CHECK(!app.request_needs_wake());
    app.set_app_waiting(true);
    CHECK(dmn.reply_needs_wake());
    app.set_app_waiting(false);
    CHECK(!dmn.reply_needs_wake());
    // a sealed memfd of the right size without the magic is refused
    raw->magic = 0;
    ShmLink bad;
    CHECK(bad.attach(dup(app.fd())) != 0);
    munmap(static_cast<void *>(raw), bytes);
}

// Sealed tick slots: whole only for their own tick, with every record and
// header field as sealed (tick_slot_whole is what completion detection and the
// socket stand-in trust).
static void t_tick_tags() {
    TickSlot s;
    std::memset(&s, 0, sizeof(s));
    s.count = 3;
    s.busy = 1;
    s.first = 40;
    for (int r = 0; r < 3; r++) {
        s.rec[r].dest = r;
        s.rec[r].msg.type = MSG_DO_ALLOC;
        s.rec[r].msg.seq = 100 + (uint64_t)r;
    }
    tick_slot_seal_tag(&s, 7);
    CHECK(tick_slot_whole(s, 7));
    CHECK(!tick_slot_whole(s, 8));  // a slot left from another tick
    TickSlot t = s;
    t.rec[1].msg.seq ^= 1;  // a record torn or changed after sealing
    CHECK(!tick_slot_whole(t, 7));
    t = s;
    t.first = 41;  // the sender's progress changed
    CHECK(!tick_slot_whole(t, 7));
    t = s;
    t.count = kTickMsgs + 1;
    CHECK(!tick_slot_whole(t, 7));
    TickSlot e;  // an empty sealed slot is whole too
    std::memset(&e, 0, sizeof(e));
    tick_slot_seal_tag(&e, 1);
    CHECK(tick_slot_whole(e, 1));
    // record tags depend on the ring index
    const uint64_t *w = reinterpret_cast<const uint64_t *>(&s.rec[0]);
    CHECK(tick_record_tag(w, 5) != tick_record_tag(w, 6));
}

// The transport over a 1-rank socket collective with the sealed outbox (the CPU
// stand-in for the RCCL seal kernel): records to ourselves come back in order,
// and with OCM_TICK_SOCKET_BATCH the transport queues ticks K at a time and
// stops on a multiple of K.
static void tick_roundtrip(int batch, bool sealed = true) {
    setenv("OCM_TICK_SOCKET_SEAL", sealed ? "1" : "0", 1);
    if (batch > 1)
        setenv("OCM_TICK_SOCKET_BATCH", std::to_string(batch).c_str(), 1);
    else
        unsetenv("OCM_TICK_SOCKET_BATCH");
    const std::string ns = "ut" + std::to_string(getpid()) + "_" + std::to_string(batch) + (sealed ? "s" : "h");
    TickTransport tt(0, 1, [ns](std::string *err, const std::atomic<bool> *cancel) {
        return make_socket_collective(ns, 0, 1, sizeof(TickSlot), err, cancel);
    });
    tt.start();
    const auto t0 = std::chrono::steady_clock::now();
    auto elapsed_ms = [&] {
        return std::chrono::duration_cast<std::chrono::milliseconds>(std::chrono::steady_clock::now() - t0).count();
    };
    while (!tt.up() && !tt.failed() && elapsed_ms() < 5000) std::this_thread::sleep_for(std::chrono::milliseconds(1));
    CHECK(tt.up());
    constexpr int kN = 300;  // more than the outbox ring holds at once (kTickRing records)
    for (int i = 0; i < kN; i++) {
        Msg m;
        std::memset(&m, 0, sizeof(m));
        m.type = MSG_STATS;
        m.seq = (uint64_t)i;
        CHECK(tt.post(0, m));
    }
    std::vector<uint64_t> got;
    while ((int)got.size() < kN && !tt.failed() && elapsed_ms() < 10000) {
        for (const Msg &m : tt.drain()) got.push_back(m.seq);
        std::this_thread::sleep_for(std::chrono::microseconds(200));
    }
    CHECK((int)got.size() == kN);
    for (int i = 0; i < kN; i++) CHECK(got[(size_t)i] == (uint64_t)i);
    // idle again after the burst: every queued tick has completed
    uint64_t last = tt.ticks();
    for (int k = 0; k < 200; k++) {
        std::this_thread::sleep_for(std::chrono::milliseconds(5));
        const uint64_t now = tt.ticks();
        if (now == last) break;
        last = now;
    }
    CHECK(last > 0 && last % (uint64_t)batch == 0);
    TickStatsWire st;
    tt.stats(&st);
    CHECK(st.own_records == (uint64_t)kN && st.lat_sum_ns > 0 && st.starts > 0);
    CHECK(st.ticks_per_start == (uint32_t)batch);
    tt.stop();
    CHECK(!tt.failed());
    unsetenv("OCM_TICK_SOCKET_SEAL");
    unsetenv("OCM_TICK_SOCKET_BATCH");
}

static void t_tick_transport() { tick_roundtrip(1); }
static void t_tick_transport_batched() { tick_roundtrip(4); }
static void t_tick_transport_host_filled() { tick_roundtrip(1, false); }

int main(int argc, char **argv) {
    if (argc > 1 && std::strcmp(argv[1], "--nodefile") == 0) {
        // ocm_unit_tests --nodefile F...: parse each with the daemon's parser
        int bad = 0;
        for (int i = 2; i < argc; i++) {
            NodeFile nf;
            std::string err;
            if (parse_nodefile(argv[i], &nf, &err) != 0) {
                printf("FAIL %s: %s\n", argv[i], err.c_str());
                bad++;
            } else {
                printf("OK %s: %zu daemons\n", argv[i], nf.nodes.size());
            }
        }
        return bad ? 1 : 0;
    }
    struct T {
        const char *name;
        std::function<void()> fn;
    } tests[] = {{"layout", t_layout},           {"nodefile", t_nodefile}, {"range_alloc", t_range_alloc},
                 {"governor", t_governor},       {"governor_hosts", t_governor_hosts},
                 {"governor_topology", t_governor_topology},
                 {"governor_checkpoint", t_governor_checkpoint},
                 {"stripe_geometry", t_stripe_geometry},
                 {"arena_host", t_arena_host},   {"siphash", t_siphash},
                 {"shmlink", t_shmlink},         {"tick_tags", t_tick_tags},
                 {"tick_transport", t_tick_transport},
                 {"tick_transport_batched", t_tick_transport_batched},
                 {"tick_transport_host_filled", t_tick_transport_host_filled}};
    for (auto &t : tests) {
        int before = g_fail;
        t.fn();
        printf("%s %s\n", g_fail == before ? "PASS" : "FAIL", t.name);
    }
    return g_fail ? 1 : 0;
}

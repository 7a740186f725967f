// Shared-memory fast path of an app's mailbox (app <-> its local ocmd).
//
// The mailbox (ocm/pmsg.h) costs a system call per record on each side, plus an
// epoll wake-up in the daemon and a poll in the app: 2.5-3 us for a remote
// ocm_alloc round trip on MI355X hosts, most of it kernel entry and exit. The
// reference paid a 500 us mailbox poll here (src/main.c:112-126).
//
// A ShmLink is one memfd the app creates at ocm_init, seals against resizing
// (F_SEAL_SHRINK/GROW/SEAL, so the daemon's mapping can never fault), and passes
// to its daemon with MSG_CONNECT (SCM_RIGHTS). It holds two single-producer /
// single-consumer rings of 160-byte records: requests app -> daemon, replies
// daemon -> app. Records, ordering and semantics are exactly those of the
// mailbox; only the transport changes. The socket stays for the connection's
// lifetime (EOF still tells the daemon that the app died) and carries the
// wake-ups:
//   * the daemon polls its links while it is awake (its post-activity spin);
//     before it sleeps it clears `daemon_polling`, fences and looks once more.
//     An app that posts a request, fences and finds the flag clear sends
//     MSG_WAKE on the socket (Dekker: one of the two always sees the other);
//   * an app spins on the reply ring for OCM_RPC_SPIN_US, then sets
//     `app_waiting`, fences, looks once more and sleeps in poll(2) on the
//     socket; a daemon that posts a reply and finds the flag set sends MSG_WAKE.
// Slots carry their own sequence number (written last, with release), so a
// consumer polls the slot it expects next instead of a shared head counter,
// and each side keeps its own counters privately: a round trip moves the two
// records' cache lines and little else (bench.py remote alloc p50 0.75-0.81 us
// with the app on either NUMA node, against 0.85-1.06 us with shared head/tail
// counters and 2.6 us over the socket alone; profiles/alloc_link_numa_r03.json).
// The consumer publishes how many records it took, which the producer reads
// only when its own count says the ring may be full.
// The daemon copies every record out of the shared ring before it looks at it
// (the app may rewrite the ring at any time) and trusts the connection's
// SO_PEERCRED pid, not the record's, as on the socket path.
#pragma once
#include <atomic>
#include <cstddef>
#include <cstdint>

#include "ocm/msg.h"

namespace ocm {

constexpr uint32_t kShmLinkSlots = 64;  // power of two
constexpr uint32_t kShmLinkMagic = 0x324d434fu;  // "OCM2"

struct alignas(64) ShmLinkSlot {
    Msg msg;
    uint8_t pad[64 - (sizeof(Msg) + 8) % 64];
    std::atomic<uint64_t> seq;  // n (1-based) once record n is whole in this slot
};
static_assert(sizeof(ShmLinkSlot) % 64 == 0, "slots are whole cache lines");

struct ShmLinkLayout {
    alignas(64) uint32_t magic;
    uint32_t slots;
    alignas(64) std::atomic<uint64_t> req_taken;       // daemon: requests taken (flow control only)
    alignas(64) std::atomic<uint64_t> rsp_taken;       // app: replies taken (flow control only)
    alignas(64) std::atomic<uint32_t> daemon_polling;  // the daemon looks at the link without a wake-up
    alignas(64) std::atomic<uint32_t> app_waiting;     // the app sleeps on the socket: wake it
    ShmLinkSlot req[kShmLinkSlots];
    ShmLinkSlot rsp[kShmLinkSlots];
};
static_assert(std::atomic<uint64_t>::is_always_lock_free, "ring counters must be lock-free across processes");

class ShmLink {
public:
    ShmLink() = default;
    ~ShmLink() { close(); }
    ShmLink(const ShmLink &) = delete;
    ShmLink &operator=(const ShmLink &) = delete;

    // App: a fresh sealed memfd with the layout, mapped. Returns 0; fd() passes it.
    int create();
    // Daemon: map an app's link. Refuses a descriptor that is not a sealed memfd
    // of exactly the layout's size. Takes ownership of `fd` either way.
    int attach(int fd);
    void close();
    bool ok() const { return l_ != nullptr; }
    int fd() const { return fd_; }

    // App side.
    bool post_request(const Msg &m);  // false: ring full (use the socket)
    bool take_reply(Msg *m);
    // Daemon side.
    bool take_request(Msg *m);        // a copy, taken out of the shared ring first
    bool post_reply(const Msg &m);    // false: ring full (keep it and retry)

    // The wake-up protocol (see the header comment). Each returns whether the
    // caller must send MSG_WAKE on the socket.
    bool request_needs_wake();        // app, after post_request
    bool reply_needs_wake();          // daemon, after post_reply
    void set_daemon_polling(bool on);
    bool requests_pending();          // daemon, after set_daemon_polling(false): look once more
    void set_app_waiting(bool on);
    bool replies_pending();           // app, after set_app_waiting(true)

private:
    bool post(ShmLinkSlot *ring, std::atomic<uint64_t> &peer_taken, const Msg &m);
    bool take(ShmLinkSlot *ring, std::atomic<uint64_t> &taken, Msg *m);
    ShmLinkLayout *l_ = nullptr;
    int fd_ = -1;
    uint64_t sent_ = 0;        // records this side posted
    uint64_t got_ = 0;         // records this side took
    uint64_t peer_taken_ = 0;  // the peer's last published count of records taken (cached)
};

}  // namespace ocm

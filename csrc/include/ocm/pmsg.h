// Process mailboxes (app <-> local daemon control plane).
//
// Parity with reference inc/pmsg.h:31-51 / src/pmsg.c: fixed-size records,
// one mailbox per process, attach-then-send, cleanup of stale mailboxes.
// Transport: AF_UNIX SOCK_SEQPACKET in the abstract namespace instead of POSIX
// message queues. Measured reason: on the MI355X pool the app user runs with
// RLIMIT_MSGQUEUE = 0 (`ulimit -q` 0), so every mq_open fails with EMFILE; the
// same holds in most containers. Seqpacket sockets keep record boundaries,
// block in the kernel (no EAGAIN spin as in reference src/pmsg.c:135-151),
// sit in an epoll set, report the peer's pid via SO_PEERCRED (an app cannot
// impersonate another pid) and deliver EOF when the peer process dies (crash
// reclaim without polling). Abstract names need no filesystem and vanish with
// their owner, so there are no stale mailboxes to clean up.
//   daemon endpoint: "@ocm_<ns>_d<rank>"   app endpoint (pmsg C API only): "@ocm_<ns>_p<pid>"
#pragma once
#include <sys/types.h>

#include <cstddef>
#include <map>
#include <string>
#include <vector>

namespace ocm {

std::string pmsg_namespace();                                   // OCM_NS or "default"
std::string daemon_mailbox_name(int rank, const std::string &ns);
std::string app_mailbox_name(pid_t pid, const std::string &ns);

// Listening endpoint (non-blocking). Returns fd or -1.
int mbox_listen(const std::string &name, int backlog = 256);
// Accept one pending connection (non-blocking), fills the peer pid. -1 when none.
int mbox_accept(int listen_fd, pid_t *peer_pid);
// Connect to a listening endpoint, retrying for `timeout_ms`. Returns fd or -1.
int mbox_connect(const std::string &name, int timeout_ms);
// Peer pid of a connected mailbox socket (SO_PEERCRED), -1 on error.
pid_t mbox_peer_pid(int fd);
int mbox_peer_uid(int fd);  // SO_PEERCRED uid, -1 on error
// One record. timeout_ms < 0 blocks, 0 polls. Returns 1 ok, 0 timeout / would
// block, -1 error or peer closed.
int mbox_send(int fd, const void *msg, size_t size, int timeout_ms);
int mbox_recv(int fd, void *msg, size_t size, int timeout_ms);
// The same with one file descriptor attached (SCM_RIGHTS): the capability
// transfer of a host-tier slab (memfd) from its owner daemon to an app.
// mbox_recv_fd sets *passed to the received fd, or -1 when none came.
int mbox_send_fd(int fd, const void *msg, size_t size, int pass_fd, int timeout_ms);
int mbox_recv_fd(int fd, void *msg, size_t size, int *passed, int timeout_ms);

// Client-side channel to one daemon (what libocm uses).
class Channel {
public:
    ~Channel() { close(); }
    int connect(const std::string &name, int timeout_ms);
    void close();
    int fd() const { return fd_; }
    bool connected() const { return fd_ >= 0; }
    int send(const void *msg, size_t size, int timeout_ms) { return mbox_send(fd_, msg, size, timeout_ms); }
    int recv(void *msg, size_t size, int timeout_ms) { return mbox_recv(fd_, msg, size, timeout_ms); }

private:
    int fd_ = -1;
};

// Stale-mailbox cleanup. Abstract sockets disappear with their owner, so this
// only reports whether `name` is still served by a live process.
bool mbox_alive(const std::string &name);
int pmsg_cleanup(const std::string &ns);

}  // namespace ocm

// ---- reference-shaped C interface (inc/pmsg.h:31-51), used by tools/tests ----
extern "C" {
int pmsg_init(size_t pmsg_size);
int pmsg_open(pid_t self_pid);   // PMSG_DAEMON_PID(rank) opens a daemon mailbox
int pmsg_close(void);
int pmsg_attach(pid_t to_pid);
int pmsg_detach(pid_t to_pid);
int pmsg_send(pid_t to_pid, void *msg);
int pmsg_recv(void *msg, bool block);
int pmsg_cleanup_all(void);
int pmsg_pending(void);
}
#define PMSG_DAEMON_PID(rank) (-1 - (rank))

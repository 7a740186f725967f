// Process mailboxes over POSIX message queues (app <-> local daemon).
//
// Parity with reference inc/pmsg.h:31-51 / src/pmsg.c: every process owns one
// receive-only mailbox, "attaches" to others to send, messages have one fixed
// size, and stale mailboxes can be cleaned up. Differences by design:
//   * names are namespaced so 8 per-GPU daemons (and concurrent test meshes)
//     share one host: /ocm_<ns>_d<rank> (daemon), /ocm_<ns>_p<pid> (app);
//   * receives block in the kernel (mq_timedreceive) instead of spinning on
//     EAGAIN (reference src/pmsg.c:135-151), and the daemon side exposes the
//     queue descriptor so it can sit in an epoll set;
//   * sends from the daemon are non-blocking so a stalled app can never wedge
//     the event loop (the caller keeps a backlog and waits for EPOLLOUT).
#pragma once
#include <mqueue.h>
#include <sys/types.h>

#include <string>
#include <unordered_map>

namespace ocm {

std::string pmsg_namespace();                       // OCM_NS or "default"
std::string daemon_mailbox_name(int rank, const std::string &ns);
std::string app_mailbox_name(pid_t pid, const std::string &ns);

class Mailbox {
public:
    Mailbox() = default;
    ~Mailbox();
    Mailbox(const Mailbox &) = delete;
    Mailbox &operator=(const Mailbox &) = delete;

    // Create (O_EXCL) and open our own receive queue. `replace` unlinks a stale
    // queue of the same name first (daemon restart after a crash).
    int open_self(const std::string &name, size_t msg_size, long depth, bool replace);
    void close_self(bool unlink_queue = true);
    int fd() const { return static_cast<int>(rx_); }
    const std::string &name() const { return name_; }

    // Receive one message. timeout_ms < 0 blocks, 0 polls.
    // Returns 1 = got one, 0 = timeout / empty, -1 = error.
    int recv(void *msg, int timeout_ms);
    long pending() const;

    // Sending side.
    int attach(const std::string &peer, bool nonblocking);
    void detach(const std::string &peer);
    // Returns 1 sent, 0 would block (non-blocking peer queue full), -1 error.
    int send(const std::string &peer, const void *msg, int timeout_ms = -1);
    int peer_fd(const std::string &peer) const;

private:
    mqd_t rx_ = (mqd_t)-1;
    std::string name_;
    size_t msg_size_ = 0;
    std::unordered_map<std::string, mqd_t> tx_;
};

// Unlink every mailbox of namespace `ns` whose owner process is gone
// (reference pmsg_cleanup unlinked /ocm_mq_2../ocm_mq_<pid_max> blindly).
int pmsg_cleanup(const std::string &ns);

}  // namespace ocm

// ---- reference-shaped C interface (inc/pmsg.h:31-51), used by tools/tests ----
extern "C" {
int pmsg_init(size_t pmsg_size);
int pmsg_open(pid_t self_pid);   // PMSG_DAEMON_PID (-1 - rank) opens a daemon mailbox
int pmsg_close(void);
int pmsg_attach(pid_t to_pid);
int pmsg_detach(pid_t to_pid);
int pmsg_send(pid_t to_pid, void *msg);
int pmsg_recv(void *msg, bool block);
int pmsg_cleanup_all(void);
int pmsg_pending(void);
}
#define PMSG_DAEMON_PID(rank) (-1 - (rank))

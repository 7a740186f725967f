// TCP helpers for the daemon mesh.
//
// Parity with reference src/sock.c (connect/localbind/accept/put/get). The
// reference opened one TCP connection per RPC (src/mem.c:62-111); the mesh here
// keeps one persistent, non-blocking, TCP_NODELAY connection per daemon pair
// and frames fixed 160-byte records over it.
#pragma once
#include <cstddef>
#include <cstdint>
#include <string>
#include <vector>

namespace ocm {

int tcp_listen(const std::string &bind_ip, int port, int backlog);
// Blocking connect with retries until `timeout_ms` elapses; returns fd or -1.
int tcp_connect(const std::string &host, int port, int timeout_ms);
int tcp_accept(int listen_fd);
int set_nonblocking(int fd, bool on);
void tune_socket(int fd);
// Blocking full-length I/O: 1 ok, 0 peer closed, -1 error.
int send_all(int fd, const void *buf, size_t len);
int recv_all(int fd, void *buf, size_t len);

// Non-blocking framed connection for the event loop.
struct Conn {
    int fd = -1;
    int peer_rank = -1;
    std::vector<uint8_t> rx;   // partial record
    std::vector<uint8_t> tx;   // unsent bytes
    size_t tx_off = 0;
    bool want_write = false;
};

// Read as many complete records as are available; appends them to `out`.
// Returns 0 ok, -1 on error or EOF (connection must be dropped).
int conn_read_records(Conn &c, size_t rec, std::vector<std::vector<uint8_t>> &out);
// Queue and try to flush; returns 0 ok, -1 error. Sets want_write if bytes remain.
int conn_write(Conn &c, const void *buf, size_t len);
int conn_flush(Conn &c);

}  // namespace ocm

// Network tier: remote memory on ANOTHER node.
//
// The reference's primary use case was one-sided access to memory on another
// host over InfiniBand verbs / EXTOLL RMA (reference src/rdma.c, src/extoll.c).
// Within a node our data plane maps owner memory directly (IPC over xGMI,
// memfd for the host tier); across nodes there is no such mapping, so the
// owner daemon runs a data server and the app streams one-sided PUT/GET
// records to it over TCP. The owner's CPU moves the bytes (like EXTOLL's
// notification-driven transfers), HBM owners stage through pinned buffers.
// Extents reached this way carry REGION_NET and "net:<ip>:<port>:<token>" as handle.
#pragma once
#include <atomic>
#include <memory>
#include <cstdint>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace ocm {

constexpr uint32_t kNetMagic = 0x4f434e44;  // "OCND"
enum NetOp : uint32_t { NET_PUT = 1, NET_GET = 2, NET_PING = 3 };

struct NetReq {
    uint32_t magic;
    uint32_t op;
    uint32_t slab_id;
    uint32_t tier;
    uint64_t offset;  // absolute offset inside the slab
    uint64_t len;
};
struct NetResp {
    uint32_t magic;
    int32_t err;
    uint64_t len;
};
static_assert(sizeof(NetReq) == 32 && sizeof(NetResp) == 16, "net wire layout");

constexpr size_t kNetChunk = 4u << 20;  // staging chunk for HBM owners / device-side apps

class Arena;

class DataServer {
public:
    // `token`: a connection must send these 8 bytes first (apps learn it from
    // the net: handle their own daemon hands them).
    DataServer(Arena *arena, int gpu, uint64_t token);
    ~DataServer();
    int start(const std::string &bind_ip);  // ephemeral port
    int port() const { return port_; }
    void stop();

private:
    void accept_loop();
    void serve(int fd);
    Arena *arena_;
    int gpu_;
    uint64_t token_;
    int listen_fd_ = -1, port_ = 0;
    std::atomic<bool> stop_{false};
    std::thread acceptor_;
    struct Worker {
        std::thread th;
        std::shared_ptr<std::atomic<bool>> done;
    };
    void reap();  // join workers whose connection ended (under mu_)
    std::mutex mu_;
    std::vector<Worker> workers_;
    std::vector<int> conns_;
    static constexpr size_t kMaxConns = 1024;
};

// "net:<ip>:<port>:<token hex>"
bool parse_net_handle(const uint8_t *handle, std::string *ip, int *port, uint64_t *token);

}  // namespace ocm

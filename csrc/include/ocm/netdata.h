// Network tier: remote memory on ANOTHER node.
//
// The reference's primary use case was one-sided access to memory on another
// host over InfiniBand verbs / EXTOLL RMA (reference src/rdma.c, src/extoll.c).
// Within a node our data plane maps owner memory directly (IPC over xGMI,
// memfd for the host tier); across nodes there is no such mapping, so the
// owner daemon runs a data server and the app streams one-sided PUT/GET
// records to it over TCP. The owner's CPU moves the bytes (like EXTOLL's
// notification-driven transfers), HBM owners stage through pinned buffers.
// Extents reached this way carry REGION_NET and
// "net:<ip>:<port>:<conn token>:<grant>" as handle. The grant is a random
// 64-bit capability for ONE extent: every request names it, and the server
// bounds the request by that extent (reference parity: the rkey of an RDMA
// memory region, src/rdma.h:37-41, which only opened the registered buffer).
#pragma once
#include <atomic>
#include <memory>
#include <cstdint>
#include <map>
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
    uint64_t grant;   // the extent's capability (from its net: handle)
    uint64_t offset;  // offset inside the extent
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
    int start(const std::string &bind_ip, int port = 0);  // port 0: ephemeral
    int port() const { return port_; }
    void stop();
    // Open extent [offset, offset+bytes) of `slab_id` to network requests;
    // returns its grant (random, nonzero).
    uint64_t grant(uint32_t slab_id, uint64_t offset, uint64_t bytes);
    // Close a grant. true: no request is using it, the caller frees the extent
    // now. false: requests are in flight; the last one to finish frees the
    // extent in the arena (so a free never pulls memory from under a copy).
    bool revoke(uint64_t grant);
    size_t grants() const;

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
    struct Grant {
        uint32_t slab_id = 0;
        uint64_t offset = 0, bytes = 0;
        int busy = 0;          // requests using it now
        bool revoked = false;  // freed by the owner; the last request frees the extent
    };
    // Resolve a request against its grant and pin the grant; false: unknown /
    // revoked / out of bounds (err set).
    bool acquire(const NetReq &q, void **mem, uint32_t *tier, int *err);
    void release(uint64_t grant);
    mutable std::mutex mu_;
    std::map<uint64_t, Grant> grants_;
    std::vector<Worker> workers_;
    std::vector<int> conns_;
    static constexpr size_t kMaxConns = 1024;
};

// "net:<ip>:<port>:<conn token hex>:<grant hex>"
bool parse_net_handle(const uint8_t *handle, std::string *ip, int *port, uint64_t *token, uint64_t *grant);
// Format one; false when it does not fit the 64-byte handle.
bool format_net_handle(uint8_t *handle, const std::string &ip, int port, uint64_t token, uint64_t grant);

}  // namespace ocm

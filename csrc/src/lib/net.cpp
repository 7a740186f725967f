// libocm network-tier client: one-sided PUT/GET records streamed to the owner
// daemon's data server (ocm/netdata.h) over cached TCP connections.
//
// Reference parity: the one-sided verbs to another host (src/rdma.c:46-85
// ib_read/ib_write; src/extoll.c:40-173, which pipelined 8 MiB chunks with 2
// in flight). Here a large op is cut into `net_streams` contiguous parts, each
// moved on its own connection (its own server worker thread on the owner), so
// several cores and flows drive the link at once; device-side local memory is
// staged through a pinned buffer per connection.
#include <thread>

#include "internal.h"

namespace ocmlib {

// ---- network tier client ----

namespace {

std::string conn_key(const std::string &ep, int stream) { return ep + "#" + std::to_string(stream); }

// Connection `stream` to `ep` (created on first use). Caller holds the library lock.
NetConn *net_conn(const std::string &ep, uint64_t token, int stream) {
    State &s = S();
    const std::string key = conn_key(ep, stream);
    auto it = s.net_conns.find(key);
    if (it != s.net_conns.end()) return &it->second;
    const size_t colon = ep.rfind(':');
    int fd = tcp_connect(ep.substr(0, colon), std::atoi(ep.c_str() + colon + 1), 10000);
    if (fd < 0) {
        set_last_error("cannot reach data server %s", ep.c_str());
        return nullptr;
    }
    if (send_all(fd, &token, sizeof(token)) != 1) {
        close(fd);
        set_last_error("data server %s refused the connection", ep.c_str());
        return nullptr;
    }
    NetConn c;
    c.fd = fd;
    return &(s.net_conns[key] = c);
}

void net_close(NetConn &c) {
    if (c.fd >= 0) close(c.fd);
    c.fd = -1;
    if (c.stage) {
        State &s = S();
        DeviceGuard g(s.device);
        (void)hipHostFree(c.stage);
        c.stage = nullptr;
    }
}

// Blocking PUT/GET of one contiguous part on one connection. Runs on the
// calling thread or a helper thread: touches only `c` and the caller's buffers.
int net_part(NetConn &c, const Extent &e, bool put, char *lin, bool dev, int device, uint64_t ext_off,
             uint64_t len) {
    NetReq q{kNetMagic, put ? (uint32_t)NET_PUT : (uint32_t)NET_GET, e.net_grant, ext_off, len};
    if (send_all(c.fd, &q, sizeof(q)) != 1) return -1;
    DeviceGuard g(dev ? device : -1);
    NetResp r;
    if (put) {
        for (uint64_t done = 0; done < len;) {
            const size_t n = (size_t)std::min<uint64_t>(kNetChunk, len - done);
            const char *src = lin + done;
            if (dev) {
                if (hipMemcpy(c.stage, lin + done, n, hipMemcpyDeviceToHost) != hipSuccess) return -1;
                src = static_cast<const char *>(c.stage);
            }
            if (send_all(c.fd, src, n) != 1) return -1;
            done += n;
        }
        if (recv_all(c.fd, &r, sizeof(r)) != 1 || r.magic != kNetMagic) return -1;
        return r.err ? -(int)r.err - 1000 : 0;
    }
    if (recv_all(c.fd, &r, sizeof(r)) != 1 || r.magic != kNetMagic) return -1;
    if (r.err) return -(int)r.err - 1000;
    for (uint64_t done = 0; done < len;) {
        const size_t n = (size_t)std::min<uint64_t>(kNetChunk, len - done);
        char *dst = dev ? static_cast<char *>(c.stage) : lin + done;
        if (recv_all(c.fd, dst, n) != 1) return -1;
        if (dev && hipMemcpy(lin + done, c.stage, n, hipMemcpyHostToDevice) != hipSuccess) return -1;
        done += n;
    }
    return 0;
}

}  // namespace

void net_drop(const std::string &ep) {
    State &s = S();
    for (auto it = s.net_conns.begin(); it != s.net_conns.end();) {
        if (it->first.compare(0, ep.size() + 1, ep + "#") == 0) {
            net_close(it->second);
            it = s.net_conns.erase(it);
        } else {
            ++it;
        }
    }
}

void net_close_all() {
    State &s = S();
    for (auto &kv : s.net_conns) net_close(kv.second);
    s.net_conns.clear();
}

// Blocking one-sided PUT/GET of one contiguous piece of a network extent.
int net_piece(const Extent &e, bool put, char *lin, Loc lloc, uint64_t ext_off, uint64_t len) {
    State &s = S();
    const bool dev = lloc == LOC_DEVICE;
    // Parts: one per stream, each at least net_split_min bytes, 64 KiB aligned.
    int k = 1;
    if (s.net_streams > 1 && len >= 2 * s.net_split_min)
        k = (int)std::min<uint64_t>((uint64_t)s.net_streams, len / s.net_split_min);
    std::vector<NetConn *> conns((size_t)k);
    for (int i = 0; i < k; i++) {
        conns[(size_t)i] = net_conn(e.ep, e.net_token, i);
        if (!conns[(size_t)i]) return -1;
        if (dev && !conns[(size_t)i]->stage) {
            DeviceGuard g(s.device);
            if (hipHostMalloc(&conns[(size_t)i]->stage, kNetChunk, hipHostMallocDefault) != hipSuccess) {
                (void)hipGetLastError();
                conns[(size_t)i]->stage = nullptr;
                OCM_FAIL(-1, "no pinned staging buffer for the network tier");
            }
        }
    }
    const uint64_t per = ((len / (uint64_t)k) + 0xFFFF) & ~0xFFFFull;
    std::vector<int> rc((size_t)k, 0);
    std::vector<std::thread> helpers;
    for (int i = 1; i < k; i++) {
        const uint64_t off = per * (uint64_t)i;
        if (off >= len) break;
        const uint64_t n = std::min(per, len - off);
        helpers.emplace_back([&, i, off, n] {
            rc[(size_t)i] = net_part(*conns[(size_t)i], e, put, lin + off, dev, s.device, ext_off + off, n);
        });
    }
    rc[0] = net_part(*conns[0], e, put, lin, dev, s.device, ext_off, std::min(per, len));
    for (auto &t : helpers) t.join();
    for (int i = 0; i < k; i++) {
        if (rc[(size_t)i] == 0) continue;
        net_drop(e.ep);  // the byte streams may be out of step: start over on fresh connections
        if (rc[(size_t)i] <= -1000) OCM_FAIL(-1, "remote %s refused: %s", put ? "PUT" : "GET", strerror(-rc[(size_t)i] - 1000));
        OCM_FAIL(-1, "network tier %s with %s failed", put ? "PUT" : "GET", e.ep.c_str());
    }
    return 0;
}

}  // namespace ocmlib

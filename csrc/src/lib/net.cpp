// libocm network-tier client: one-sided PUT/GET records streamed to the owner
// daemon's data server (ocm/netdata.h) over one cached TCP connection per
// owner, device memory staged through a pinned buffer.
#include "internal.h"

namespace ocmlib {

// ---- network tier client ----

int net_conn(const std::string &ep, uint64_t token) {
    State &s = S();
    auto it = s.net_conns.find(ep);
    if (it != s.net_conns.end()) return it->second;
    const size_t colon = ep.rfind(':');
    int fd = tcp_connect(ep.substr(0, colon), std::atoi(ep.c_str() + colon + 1), 10000);
    if (fd < 0) OCM_FAIL(-1, "cannot reach data server %s", ep.c_str());
    if (send_all(fd, &token, sizeof(token)) != 1) {
        close(fd);
        OCM_FAIL(-1, "data server %s refused the connection", ep.c_str());
    }
    s.net_conns[ep] = fd;
    return fd;
}

void net_drop(const std::string &ep) {
    State &s = S();
    auto it = s.net_conns.find(ep);
    if (it == s.net_conns.end()) return;
    close(it->second);
    s.net_conns.erase(it);
}

// Blocking one-sided PUT/GET of one contiguous piece over TCP. Device-side
// local memory is staged through a pinned buffer, kNetChunk at a time.
int net_piece(const Extent &e, bool put, char *lin, Loc lloc, uint64_t ext_off, uint64_t len) {
    State &s = S();
    int fd = net_conn(e.ep, e.net_token);
    if (fd < 0) return -1;
    NetReq q{kNetMagic, put ? (uint32_t)NET_PUT : (uint32_t)NET_GET, e.r.slab_id, e.r.tier, e.r.offset + ext_off, len};
    const bool dev = lloc == LOC_DEVICE;
    if (dev && !s.net_stage) {
        DeviceGuard g(s.device);
        if (hipHostMalloc(&s.net_stage, kNetChunk, hipHostMallocDefault) != hipSuccess) {
            (void)hipGetLastError();
            s.net_stage = nullptr;
            OCM_FAIL(-1, "no pinned staging buffer for the network tier");
        }
    }
    auto fail = [&](const char *what) {
        net_drop(e.ep);
        set_last_error("network tier %s with %s failed", what, e.ep.c_str());
        return -1;
    };
    if (send_all(fd, &q, sizeof(q)) != 1) return fail("request");
    NetResp r;
    if (put) {
        for (uint64_t done = 0; done < len;) {
            const size_t n = (size_t)std::min<uint64_t>(kNetChunk, len - done);
            const char *src = lin + done;
            if (dev) {
                DeviceGuard g(s.device);
                if (hipMemcpy(s.net_stage, lin + done, n, hipMemcpyDeviceToHost) != hipSuccess) return fail("staging");
                src = static_cast<const char *>(s.net_stage);
            }
            if (send_all(fd, src, n) != 1) return fail("payload");
            done += n;
        }
        if (recv_all(fd, &r, sizeof(r)) != 1 || r.magic != kNetMagic) return fail("response");
        if (r.err) OCM_FAIL(-1, "remote PUT refused: %s", strerror(r.err));
        return 0;
    }
    if (recv_all(fd, &r, sizeof(r)) != 1 || r.magic != kNetMagic) return fail("response");
    if (r.err) OCM_FAIL(-1, "remote GET refused: %s", strerror(r.err));
    for (uint64_t done = 0; done < len;) {
        const size_t n = (size_t)std::min<uint64_t>(kNetChunk, len - done);
        char *dst = dev ? static_cast<char *>(s.net_stage) : lin + done;
        if (recv_all(fd, dst, n) != 1) return fail("payload");
        if (dev) {
            DeviceGuard g(s.device);
            if (hipMemcpy(lin + done, s.net_stage, n, hipMemcpyHostToDevice) != hipSuccess) return fail("staging");
        }
        done += n;
    }
    return 0;
}


}  // namespace ocmlib

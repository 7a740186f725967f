// Network-tier handle text, shared by ocmd (formats it at DO_ALLOC) and libocm
// (parses it at import): "net:<ip>:<port>:<conn token>:<grant>" (ocm/netdata.h).
#include <cstdio>
#include <cstring>

#include "ocm/msg.h"
#include "ocm/netdata.h"

namespace ocm {

bool parse_net_handle(const uint8_t *handle, std::string *ip, int *port, uint64_t *token, uint64_t *grant) {
    char buf[65] = {0};
    std::memcpy(buf, handle, 64);
    char host[64] = {0};
    int p = 0;
    unsigned long long t = 0, g = 0;
    if (std::sscanf(buf, "net:%63[^:]:%d:%llx:%llx", host, &p, &t, &g) != 4 || p <= 0 || g == 0) return false;
    *ip = host;
    *port = p;
    *token = t;
    *grant = g;
    return true;
}

bool format_net_handle(uint8_t *handle, const std::string &ip, int port, uint64_t token, uint64_t grant) {
    char buf[kHandleBytes + 1];
    const int n = std::snprintf(buf, sizeof(buf), "net:%s:%d:%llx:%llx", ip.c_str(), port, (unsigned long long)token,
                                (unsigned long long)grant);
    if (n <= 0 || n >= (int)kHandleBytes) return false;  // keep a NUL inside the handle
    std::memset(handle, 0, kHandleBytes);
    std::memcpy(handle, buf, (size_t)n);
    return true;
}

}  // namespace ocm

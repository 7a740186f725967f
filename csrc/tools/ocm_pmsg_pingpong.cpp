// Mailbox ping-pong (reference test/pmsg_daemon.c + test/pmsg_client.c):
//   ocm_pmsg_pingpong server <rank>            echo server on a daemon mailbox
//   ocm_pmsg_pingpong client <rank> <count>    send `count` pings, print p50/p99 RTT
// The client sends MSG_SHUTDOWN at the end so the server exits.
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "ocm/msg.h"
#include "ocm/pmsg.h"

using namespace ocm;

int main(int argc, char **argv) {
    if (argc < 3) {
        fprintf(stderr, "usage: %s server <rank> | client <rank> <count>\n", argv[0]);
        return 2;
    }
    const std::string ns = pmsg_namespace();
    const int rank = std::atoi(argv[2]);
    Mailbox box;
    if (!std::strcmp(argv[1], "server")) {
        if (box.open_self(daemon_mailbox_name(rank, ns), kMsgBytes, 8, true) != 0) return 1;
        printf("ready\n");
        fflush(stdout);
        Msg m;
        for (;;) {
            if (box.recv(&m, 30000) != 1) return 1;
            if (m.type == MSG_SHUTDOWN) break;
            std::string peer = app_mailbox_name(m.pid, ns);
            if (box.attach(peer, false) != 0) return 1;
            m.status = MSG_RESPONSE;
            box.send(peer, &m, 5000);
        }
        box.close_self(true);
        return 0;
    }
    const int count = argc > 3 ? std::atoi(argv[3]) : 1000;
    if (box.open_self(app_mailbox_name(getpid(), ns), kMsgBytes, 8, true) != 0) return 1;
    const std::string d = daemon_mailbox_name(rank, ns);
    for (int i = 0; box.attach(d, false) != 0; i++) {
        if (i > 500) return 1;
        usleep(10000);
    }
    std::vector<double> rtt;
    Msg m, r;
    std::memset(&m, 0, sizeof(m));
    m.type = MSG_PING;
    m.pid = getpid();
    for (int i = 0; i < count; i++) {
        m.seq = (uint64_t)i + 1;
        auto t0 = std::chrono::steady_clock::now();
        if (box.send(d, &m, 5000) != 1 || box.recv(&r, 5000) != 1 || r.seq != m.seq || r.status != MSG_RESPONSE) {
            fprintf(stderr, "ping %d failed\n", i);
            return 1;
        }
        rtt.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
    }
    m.type = MSG_SHUTDOWN;
    box.send(d, &m, 5000);
    std::sort(rtt.begin(), rtt.end());
    printf("{\"count\": %d, \"p50_us\": %.2f, \"p99_us\": %.2f}\n", count, rtt[rtt.size() / 2],
           rtt[std::min(rtt.size() - 1, rtt.size() * 99 / 100)]);
    box.close_self(true);
    return 0;
}

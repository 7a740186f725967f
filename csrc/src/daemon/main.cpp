// ocmd entry point: `ocmd <nodefile> [options]` (reference: `oncillamem <nodefile>`,
// src/main.c:187-224). Start one per GPU; rank0 is the master and must be
// reachable within --join-timeout-ms by the others.
#include <cstdio>
#include <string>

#include "ocm/daemon.h"
#include "ocm/log.h"

int main(int argc, char **argv) {
    ocm::DaemonConfig cfg;
    std::string err;
    const int rc = ocm::parse_daemon_args(argc, argv, &cfg, &err);
    if (rc > 0) {  // --help
        std::printf("%s\n", err.c_str());
        return 0;
    }
    if (rc != 0) {
        std::fprintf(stderr, "%s\n", err.c_str());
        return 2;
    }
    ocm::Daemon d(cfg);
    return d.run();
}

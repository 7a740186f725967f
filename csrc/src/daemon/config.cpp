// ocmd command line and OCM_* environment (DaemonConfig).
#include "ocm/daemon.h"

#include <fcntl.h>
#include <hip/hip_runtime_api.h>
#include <signal.h>
#include <sys/epoll.h>
#include <sys/signalfd.h>
#include <sys/syscall.h>
#include <time.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>

#include "../../include/oncillamem.h"
#include "ocm/log.h"
#include "ocm/trace.h"
#include "util.h"

namespace ocm {
using namespace dm;

static const char *kUsage =
    "usage: ocmd <nodefile> [options]            (one daemon per GPU; rank 0 is the master)\n"
    "  --rank R                 this daemon's nodefile line (default: OCM_RANK / LOCAL_RANK / hostname)\n"
    "  --gpu G|none             device ordinal (default: gpu= column, else rank % visible GPUs)\n"
    "  --ns NS                  mailbox namespace, several meshes per host      [OCM_NS]\n"
    "  --policy P               ring | least_loaded | stripe | loopback        [OCM_PLACEMENT]\n"
    "  --stripe-unit B          default stripe unit (power of two)             [OCM_STRIPE_UNIT]\n"
    "  --slab-bytes B           HBM slab size (default 4G)                       [OCM_SLAB_BYTES]\n"
    "  --gpu-capacity B         HBM this daemon may hand out (default 75% free) [OCM_GPU_CAPACITY]\n"
    "  --host-capacity B        host-tier bytes (default 25% MemAvailable)      [OCM_HOST_CAPACITY]\n"
    "  --ctrl auto|tcp|rccl|socket  daemon<->daemon record transport (auto: RCCL when every\n"
    "                           rank has a GPU of its own, else TCP)            [OCM_CTRL]\n"
    "  --lease-bytes B          capacity lease chunk (0 = off, default 1G)      [OCM_LEASE_BYTES]\n"
    "  --state-file PATH        rank0 directory checkpoint (resume)            [OCM_STATE_FILE]\n"
    "  --host-alias NAME        node name to report (emulate several nodes)    [OCM_HOST_ALIAS]\n"
    "  --bind IP                listen address (default 0.0.0.0)\n"
    "  --join-timeout-ms MS     how long to wait for rank0\n"
    "  --ready-file PATH        written once the mesh is complete\n"
    "  --watch-pid PID          exit when this process exits\n"
    "  --zero                   zero memory on allocation                      [OCM_ZERO_ON_ALLOC]\n"
    "  --spin-us US             poll without sleeping for US after activity (default 50, 0 = off) [OCM_DAEMON_SPIN_US]\n"
    "sizes accept K/M/G/T suffixes; OCM_MESH_KEY sets the mesh authentication secret";

int parse_daemon_args(int argc, char **argv, DaemonConfig *cfg, std::string *err) {
    auto env = [](const char *k) -> const char * {
        const char *v = std::getenv(k);
        return (v && *v) ? v : nullptr;
    };
    if (const char *v = env("OCM_NODEFILE")) cfg->nodefile = v;
    if (const char *v = env("OCM_PLACEMENT")) cfg->policy = parse_policy(v, cfg->policy);
    if (const char *v = env("OCM_STRIPE_UNIT")) cfg->stripe_unit = parse_bytes(v);
    if (const char *v = env("OCM_SLAB_BYTES")) cfg->slab_bytes = parse_bytes(v);
    if (const char *v = env("OCM_GPU_CAPACITY")) cfg->gpu_capacity = parse_bytes(v);
    if (const char *v = env("OCM_HOST_CAPACITY")) cfg->host_capacity = parse_bytes(v);
    if (const char *v = env("OCM_GPU_FRACTION")) cfg->gpu_fraction = std::atof(v);
    if (const char *v = env("OCM_HOST_FRACTION")) cfg->host_fraction = std::atof(v);
    if (env("OCM_ZERO_ON_ALLOC")) cfg->zero_on_alloc = true;
    if (env("OCM_NO_GPU")) cfg->gpu = -1;
    if (const char *v = env("OCM_CTRL")) cfg->ctrl = v;
    if (const char *v = env("OCM_LEASE_BYTES")) cfg->lease_bytes = parse_bytes(v);
    if (const char *v = env("OCM_LEASE_AFTER")) cfg->lease_after = std::atoi(v);
    if (env("OCM_LEASE_HOST")) cfg->lease_host = true;
    if (const char *v = env("OCM_LEASE_IDLE_MS")) cfg->lease_idle_ms = std::atoi(v);
    if (const char *v = env("OCM_HOST_ALIAS")) cfg->host_alias = v;
    if (const char *v = env("OCM_STATE_FILE")) cfg->state_file = v;
    if (const char *v = env("OCM_MESH_KEY")) cfg->mesh_key = v;
    if (const char *v = env("OCM_STATE_INTERVAL_MS")) cfg->state_interval_ms = std::atoi(v);
    if (const char *v = env("OCM_DAEMON_SPIN_US")) cfg->spin_us = std::atoi(v);
    for (int i = 1; i < argc; i++) {
        std::string a = argv[i];
        if (a == "-h" || a == "--help") {
            *err = kUsage;
            return 1;
        }
        auto val = [&](std::string *out) {
            if (i + 1 >= argc) {
                *err = "missing value for " + a;
                return false;
            }
            *out = argv[++i];
            return true;
        };
        std::string v;
        if (a == "--rank") {
            if (!val(&v)) return -1;
            cfg->rank = std::atoi(v.c_str());
        } else if (a == "--gpu") {
            if (!val(&v)) return -1;
            cfg->gpu = (v == "none" || v == "cpu") ? -1 : std::atoi(v.c_str());
        } else if (a == "--ns") {
            if (!val(&cfg->ns)) return -1;
        } else if (a == "--policy") {
            if (!val(&v)) return -1;
            cfg->policy = parse_policy(v, cfg->policy);
        } else if (a == "--stripe-unit") {
            if (!val(&v)) return -1;
            cfg->stripe_unit = parse_bytes(v);
        } else if (a == "--slab-bytes") {
            if (!val(&v)) return -1;
            cfg->slab_bytes = parse_bytes(v);
        } else if (a == "--gpu-capacity") {
            if (!val(&v)) return -1;
            cfg->gpu_capacity = parse_bytes(v);
        } else if (a == "--host-capacity") {
            if (!val(&v)) return -1;
            cfg->host_capacity = parse_bytes(v);
        } else if (a == "--join-timeout-ms") {
            if (!val(&v)) return -1;
            cfg->join_timeout_ms = std::atoi(v.c_str());
        } else if (a == "--ready-file") {
            if (!val(&cfg->ready_file)) return -1;
        } else if (a == "--bind") {
            if (!val(&cfg->bind_ip)) return -1;
        } else if (a == "--ctrl") {
            if (!val(&cfg->ctrl)) return -1;
            if (cfg->ctrl != "auto" && cfg->ctrl != "tcp" && cfg->ctrl != "rccl" && cfg->ctrl != "socket") {
                *err = "--ctrl must be auto, tcp, rccl or socket";
                return -1;
            }
        } else if (a == "--host-alias") {
            if (!val(&cfg->host_alias)) return -1;
        } else if (a == "--state-file") {
            if (!val(&cfg->state_file)) return -1;
        } else if (a == "--lease-bytes") {
            if (!val(&v)) return -1;
            cfg->lease_bytes = parse_bytes(v);
        } else if (a == "--watch-pid") {
            if (!val(&v)) return -1;
            cfg->watch_pid = std::atoi(v.c_str());
        } else if (a == "--zero") {
            cfg->zero_on_alloc = true;
        } else if (a == "--spin-us") {
            if (!val(&v)) return -1;
            cfg->spin_us = std::atoi(v.c_str());
        } else if (!a.empty() && a[0] == '-') {
            *err = "unknown option " + a;
            return -1;
        } else {
            cfg->nodefile = a;
        }
    }
    if (cfg->nodefile.empty()) {
        *err = kUsage;
        return -1;
    }
    if (cfg->ns.empty()) cfg->ns = pmsg_namespace();
    return 0;
}

Daemon::Daemon(const DaemonConfig &cfg) : cfg_(cfg) {}

Daemon::~Daemon() { shutdown(); }


}  // namespace ocm

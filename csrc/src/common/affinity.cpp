// CPU placement next to a GPU (see ocm/affinity.h).
#include "ocm/affinity.h"

#include <sched.h>

#include <algorithm>
#include <cctype>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>

#include "ocm/log.h"

namespace ocm {

namespace {

bool read_line(const std::string &path, std::string *out) {
    FILE *f = std::fopen(path.c_str(), "r");
    if (!f) return false;
    char buf[4096];
    const bool ok = std::fgets(buf, sizeof(buf), f) != nullptr;
    std::fclose(f);
    if (!ok) return false;
    *out = buf;
    while (!out->empty() && std::isspace((unsigned char)out->back())) out->pop_back();
    return true;
}

// "0-63,128-191" -> {0..63, 128..191}
std::vector<int> parse_cpulist(const std::string &s) {
    std::vector<int> out;
    size_t i = 0;
    while (i < s.size()) {
        size_t j = s.find(',', i);
        if (j == std::string::npos) j = s.size();
        const std::string part = s.substr(i, j - i);
        int a = 0, b = 0;
        if (std::sscanf(part.c_str(), "%d-%d", &a, &b) == 2) {
            for (int c = a; c <= b && c - a < 65536; c++) out.push_back(c);
        } else if (std::sscanf(part.c_str(), "%d", &a) == 1) {
            out.push_back(a);
        }
        i = j + 1;
    }
    return out;
}

}  // namespace

int pci_numa_node(const std::string &bus_id) {
    std::string bus = bus_id;
    for (char &c : bus) c = (char)std::tolower((unsigned char)c);
    std::string v;
    if (!read_line("/sys/bus/pci/devices/" + bus + "/numa_node", &v)) return -1;
    return std::atoi(v.c_str());
}

std::vector<int> ccd_cpus(int node, int slot) {
    std::string list;
    if (node < 0 || !read_line("/sys/devices/system/node/node" + std::to_string(node) + "/cpulist", &list)) return {};
    // group the node's CPUs by L3 instance
    std::map<int, std::vector<int>> by_l3;
    for (int c : parse_cpulist(list)) {
        std::string id;
        if (!read_line("/sys/devices/system/cpu/cpu" + std::to_string(c) + "/cache/index3/id", &id)) return {};
        by_l3[std::atoi(id.c_str())].push_back(c);
    }
    if (by_l3.empty()) return {};
    std::vector<std::vector<int>> groups;
    for (auto &kv : by_l3) groups.push_back(kv.second);
    std::sort(groups.begin(), groups.end(),
              [](const std::vector<int> &a, const std::vector<int> &b) { return a.front() < b.front(); });
    return groups[(size_t)(slot < 0 ? 0 : slot) % groups.size()];
}

int pin_thread(const std::vector<int> &cpus) {
    cpu_set_t cur;
    CPU_ZERO(&cur);
    if (sched_getaffinity(0, sizeof(cur), &cur) != 0) return 0;
    cpu_set_t want;
    CPU_ZERO(&want);
    int n = 0;
    for (int c : cpus)
        if (c >= 0 && c < CPU_SETSIZE && CPU_ISSET(c, &cur)) {
            CPU_SET(c, &want);
            n++;
        }
    if (n == 0) return 0;
    if (sched_setaffinity(0, sizeof(want), &want) != 0) return 0;
    return n;
}

std::vector<int> thread_cpus() {
    cpu_set_t cur;
    CPU_ZERO(&cur);
    std::vector<int> out;
    if (sched_getaffinity(0, sizeof(cur), &cur) != 0) return out;
    for (int c = 0; c < CPU_SETSIZE; c++)
        if (CPU_ISSET(c, &cur)) out.push_back(c);
    return out;
}

int set_thread_cpus(const std::vector<int> &cpus) {
    cpu_set_t want;
    CPU_ZERO(&want);
    int n = 0;
    for (int c : cpus)
        if (c >= 0 && c < CPU_SETSIZE) {
            CPU_SET(c, &want);
            n++;
        }
    if (n == 0) return -1;
    return sched_setaffinity(0, sizeof(want), &want) == 0 ? 0 : -1;
}

std::vector<int> core_siblings(int cpu) {
    std::string list;
    if (!read_line("/sys/devices/system/cpu/cpu" + std::to_string(cpu) + "/topology/thread_siblings_list", &list))
        return {cpu};
    return parse_cpulist(list);
}

std::vector<int> near_gpu_cpus(const std::string &bus_id, int gpu_ordinal, PinRole role, int daemon_rank) {
    const char *e = std::getenv("OCM_PIN");
    const bool whole_ccd = e && std::strcmp(e, "ccd") == 0;  // everyone on the whole complex
    const int node = pci_numa_node(bus_id);
    std::vector<int> ccd = ccd_cpus(node, gpu_ordinal);
    if (ccd.empty()) return {};
    // Physical cores of the complex (the first hardware thread of each).
    std::vector<int> cores;
    for (int c : ccd) {
        const std::vector<int> sib = core_siblings(c);
        if (!sib.empty() && *std::min_element(sib.begin(), sib.end()) == c) cores.push_back(c);
    }
    if (cores.empty()) cores = ccd;
    // The daemon's event loop gets a core of the complex to itself (one hardware
    // thread; several daemons of one GPU take successive cores by rank); its apps
    // get every other core, so none shares a core or its SMT sibling with it.
    const int dcore = cores[(size_t)(daemon_rank < 0 ? 0 : daemon_rank) % cores.size()];
    const std::vector<int> dsib = core_siblings(dcore);
    std::vector<int> cpus;
    if (whole_ccd) {
        cpus = ccd;
    } else if (role == PinRole::Daemon) {
        cpus.push_back(dcore);
    } else {
        for (int c : ccd)
            if (std::find(dsib.begin(), dsib.end(), c) == dsib.end()) cpus.push_back(c);
        if (cpus.empty()) cpus = ccd;
    }
    return cpus;
}

std::vector<int> pin_near_gpu(const std::string &bus_id, int gpu_ordinal, PinRole role, int daemon_rank) {
    const char *e = std::getenv("OCM_PIN");
    if (e && std::strcmp(e, "0") == 0) return {};
    // Apps opt in: their calling thread's mask would be inherited by everything
    // the application starts later.
    if (role == PinRole::App && (!e || !*e)) return {};
    std::vector<int> cpus = near_gpu_cpus(bus_id, gpu_ordinal, role, daemon_rank);
    if (cpus.empty()) return {};
    const int node = pci_numa_node(bus_id);
    const int n = pin_thread(cpus);
    if (n == 0) return {};
    OCM_LOG("%s: pinned to %d CPU(s) from %d (NUMA node %d of GPU %s)", role == PinRole::Daemon ? "ocmd" : "libocm", n,
            cpus.front(), node, bus_id.c_str());
    return cpus;
}

}  // namespace ocm

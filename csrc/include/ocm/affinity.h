// CPU placement next to a GPU.
//
// A blocking one-sided op and a control RPC are round trips between the app's
// thread, the GPU (doorbell / completion words in host memory) and the
// daemon's thread (mailbox). Their latency depends on where those threads
// run: on the GPU's socket (its PCIe root) and sharing one L3 complex (CCD), a
// cache line moves between them in tens of ns instead of hundreds. The daemon
// of GPU g and the apps that copy on GPU g both restrict themselves to the
// same CCD of g's NUMA node (chosen by g's ordinal, so the GPUs of one node get
// different CCDs), the daemon to a core of its own; OCM_PIN=0 turns it off
// (apps opt in with OCM_PIN=1: see pin_near_gpu). No reference counterpart: the
// reference's daemon and apps ran wherever the scheduler put them.
#pragma once
#include <string>
#include <vector>

namespace ocm {

// NUMA node of a PCI device ("0000:0a:00.0", any case); -1 if unknown.
int pci_numa_node(const std::string &bus_id);

// Every hardware thread of one L3 complex of `node`: complex `slot` modulo the
// node's complexes, ordered by their lowest CPU. Empty if sysfs is unreadable.
std::vector<int> ccd_cpus(int node, int slot);

// Restrict the calling thread to `cpus` intersected with its allowed set.
// Returns the number of CPUs it may now run on (0: unchanged, nothing in common).
int pin_thread(const std::vector<int> &cpus);

// The CPUs the calling thread may run on now (empty if unknown).
std::vector<int> thread_cpus();
// Set the calling thread's mask to exactly `cpus` (e.g. restore a saved mask
// for a thread that must not share the pinned event loop's core). 0 on success.
int set_thread_cpus(const std::vector<int> &cpus);

// Hardware threads sharing `cpu`'s core (itself included).
std::vector<int> core_siblings(int cpu);

// Daemon (unless OCM_PIN=0): the event loop of daemon `daemon_rank` on one core
// of the GPU's L3 complex (one hardware thread; core = rank modulo the complex's
// cores). App (only when OCM_PIN is set, e.g. OCM_PIN=1): the calling thread on
// the complex's other cores. Apps are not pinned by default, because the mask
// of the calling thread (usually the application's main thread) is inherited by
// every thread and process it creates later (intra-op pools, data loaders).
// Returns the CPUs pinned to (empty: not pinned); logs the choice under OCM_VERBOSE.
enum class PinRole { Daemon, App };
std::vector<int> pin_near_gpu(const std::string &bus_id, int gpu_ordinal, PinRole role, int daemon_rank);
// The CPUs pin_near_gpu would pick for `role` (App: the complex's cores other than
// the daemon's), without pinning anything; empty if the topology is unknown.
std::vector<int> near_gpu_cpus(const std::string &bus_id, int gpu_ordinal, PinRole role, int daemon_rank);

}  // namespace ocm

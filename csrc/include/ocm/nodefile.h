// Cluster membership: the nodefile.
//
// Parity with reference src/nodefile.c:30-116 / inc/nodefile.h:19-39: one line
// per daemon, `#` comments, columns `rank dns ethernet_ip ocm_port [rdmacm_port]`.
// Extended for one daemon per GPU: an optional trailing `gpu=<ordinal>` column
// (or a bare sixth integer). Because 8 daemons share one hostname, the own rank
// comes from --rank / OCM_RANK; the reference's "dns == gethostname()" match is
// still used when exactly one line matches.
#pragma once
#include <string>
#include <vector>

namespace ocm {

struct NodeEntry {
    int rank = -1;
    std::string dns;
    std::string ip;
    int ocm_port = 0;
    int data_port = 0;  // reference rdmacm_port column; unused by the xGMI data plane
    int gpu = -1;       // -1: daemon chooses (rank % visible GPUs, or CPU-only)
};

struct NodeFile {
    std::vector<NodeEntry> nodes;  // indexed by rank
    int size() const { return static_cast<int>(nodes.size()); }
};

// Returns 0 on success; on failure returns -1 and fills `err`.
int parse_nodefile(const std::string &path, NodeFile *out, std::string *err);
int parse_nodefile_text(const std::string &text, NodeFile *out, std::string *err);
// Resolve own rank: explicit (>=0) wins, else OCM_RANK, else a unique dns match.
int resolve_rank(const NodeFile &nf, int explicit_rank, std::string *err);

}  // namespace ocm

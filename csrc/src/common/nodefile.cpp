#include "ocm/nodefile.h"

#include <unistd.h>

#include <climits>
#include <cstdlib>
#include <fstream>
#include <sstream>

namespace ocm {

static bool parse_int(const std::string &s, int *v) {
    if (s.empty()) return false;
    char *end = nullptr;
    long x = std::strtol(s.c_str(), &end, 10);
    if (*end != '\0' || x < INT_MIN || x > INT_MAX) return false;
    *v = (int)x;
    return true;
}

int parse_nodefile_text(const std::string &text, NodeFile *out, std::string *err) {
    std::istringstream in(text);
    std::string line;
    std::vector<NodeEntry> entries;
    int lineno = 0;
    while (std::getline(in, line)) {
        lineno++;
        size_t hash = line.find('#');
        if (hash != std::string::npos) line.resize(hash);
        std::istringstream ls(line);
        std::vector<std::string> tok;
        for (std::string t; ls >> t;) tok.push_back(t);
        if (tok.empty()) continue;
        if (tok.size() < 4) {
            if (err) *err = "line " + std::to_string(lineno) + ": need `rank dns ip ocm_port`";
            return -1;
        }
        NodeEntry e;
        if (!parse_int(tok[0], &e.rank) || e.rank < 0) {
            if (err) *err = "line " + std::to_string(lineno) + ": bad rank '" + tok[0] + "'";
            return -1;
        }
        e.dns = tok[1];
        e.ip = tok[2];
        if (!parse_int(tok[3], &e.ocm_port) || e.ocm_port <= 0 || e.ocm_port > 65535) {
            if (err) *err = "line " + std::to_string(lineno) + ": bad ocm_port '" + tok[3] + "'";
            return -1;
        }
        for (size_t i = 4; i < tok.size(); i++) {
            const std::string &t = tok[i];
            int v = 0;
            if (t.compare(0, 4, "gpu=") == 0) {
                if (!parse_int(t.substr(4), &e.gpu)) {
                    if (err) *err = "line " + std::to_string(lineno) + ": bad gpu column '" + t + "'";
                    return -1;
                }
            } else if (parse_int(t, &v)) {
                // 5th column: rdmacm/data port (reference). 6th: gpu ordinal.
                if (i == 4)
                    e.data_port = v;
                else if (i == 5)
                    e.gpu = v;
            } else {
                if (err) *err = "line " + std::to_string(lineno) + ": unknown column '" + t + "'";
                return -1;
            }
        }
        entries.push_back(e);
    }
    if (entries.empty()) {
        if (err) *err = "nodefile has no entries";
        return -1;
    }
    NodeFile nf;
    nf.nodes.resize(entries.size());
    std::vector<bool> seen(entries.size(), false);
    for (const auto &e : entries) {
        if (e.rank >= (int)entries.size() || seen[e.rank]) {
            if (err) *err = "ranks must be unique and dense 0..N-1 (rank " + std::to_string(e.rank) + ")";
            return -1;
        }
        seen[e.rank] = true;
        nf.nodes[e.rank] = e;
    }
    *out = nf;
    return 0;
}

int parse_nodefile(const std::string &path, NodeFile *out, std::string *err) {
    std::ifstream f(path);
    if (!f) {
        if (err) *err = "cannot open nodefile " + path;
        return -1;
    }
    std::stringstream ss;
    ss << f.rdbuf();
    return parse_nodefile_text(ss.str(), out, err);
}

int resolve_rank(const NodeFile &nf, int explicit_rank, std::string *err) {
    int r = explicit_rank;
    if (r < 0) {
        const char *env = std::getenv("OCM_RANK");
        if (env && *env) r = std::atoi(env);
    }
    if (r >= 0) {
        if (r >= nf.size()) {
            if (err) *err = "rank " + std::to_string(r) + " not in nodefile";
            return -1;
        }
        return r;
    }
    char host[256] = {0};
    gethostname(host, sizeof(host) - 1);
    int match = -1, count = 0;
    for (const auto &e : nf.nodes) {
        if (e.dns == host) {
            match = e.rank;
            count++;
        }
    }
    if (count == 1) return match;
    if (err)
        *err = count == 0 ? std::string("hostname '") + host + "' not in nodefile; pass --rank"
                          : std::string("hostname '") + host + "' appears several times; pass --rank";
    return -1;
}

}  // namespace ocm

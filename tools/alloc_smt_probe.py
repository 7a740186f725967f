#!/usr/bin/env python3
"""Remote/local ocm_alloc p50 with the app's calling thread pinned (after its
daemon is up) to: the SMT sibling of the daemon's event-loop core, another core
of the same complex, or left unpinned. Only the calling thread moves, so the
daemon and the runtime's helper threads keep their own CPUs.

  python3 tools/alloc_smt_probe.py --repeat 3 --out x.json
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

from oncilla_amd import api  # noqa: E402
from oncilla_amd.models import workloads as wl  # noqa: E402
from oncilla_amd.parallel.mesh import Mesh  # noqa: E402


def loop_core(pid):
    line = [x for x in open(f"/proc/{pid}/status") if x.startswith("Cpus_allowed_list")][0]
    return int(line.split()[1].split(",")[0].split("-")[0])


def siblings(cpu):
    out = set()
    for part in open(f"/sys/devices/system/cpu/cpu{cpu}/topology/thread_siblings_list").read().strip().split(","):
        lo, _, hi = part.partition("-")
        out.update(range(int(lo), int(hi or lo) + 1))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--repeat", type=int, default=3)
    ap.add_argument("--samples", type=int, default=300)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    orig = os.sched_getaffinity(0)
    res = {}
    with Mesh(1, gpus=[0]) as m, api.Client(daemon_rank=0, gpu=0, ns=m.ns) as c:
        d = loop_core(m.daemons[0].proc.pid)
        sib = sorted(siblings(d) - {d})
        other = d + 2 if (d + 2) in orig else sorted(orig - siblings(d))[0]
        places = {"unpinned": orig, "daemon_sibling": set(sib[:1]) if sib else orig, "other_core": {other}}
        for r in range(a.repeat):
            for name, cpus in places.items():
                os.sched_setaffinity(0, cpus)
                try:
                    rem = wl.alloc_latency(c, api.OCM_REMOTE_GPU, a.samples, local_bytes=4096, remote_bytes=1 << 20)
                    loc = wl.alloc_latency(c, api.OCM_LOCAL_HOST, a.samples, local_bytes=4096)
                finally:
                    os.sched_setaffinity(0, orig)
                res[f"{name}#{r}"] = {"cpu": sorted(cpus)[0] if len(cpus) == 1 else "any",
                                      "alloc_p50_us": round(rem["alloc_p50_us"], 2),
                                      "alloc_p99_us": round(rem["alloc_p99_us"], 2),
                                      "local_alloc_p50_us": round(loc["alloc_p50_us"], 2)}
                print(name, res[f"{name}#{r}"], flush=True)
    doc = {"what": "ocm_alloc p50 (remote: 1 daemon, host-tier pair; local: malloc kind) with the app's calling "
                   f"thread on the SMT sibling of the daemon's event-loop core (cpu {d}), on another core, or unpinned",
           "result": res}
    if a.out:
        with open(a.out, "w") as f:
            json.dump(doc, f, indent=1)


if __name__ == "__main__":
    main()

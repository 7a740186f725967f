"""Does the CPU the application thread spins on set small-op latency? After ocm_init
(OCM_PIN=1: the GPU's L3 complex minus the daemon's core), pin this thread to each
allowed hardware thread in turn and time 200 back-to-back 4 KiB gets and puts per
tier, three passes over the CPUs. Prints the p50 per CPU.

    python tools/cpu_placement_probe.py [--out ...]
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="")
    ap.add_argument("--passes", type=int, default=3)
    a = ap.parse_args()
    os.environ.setdefault("OCM_PIN", "1")
    from oncilla_amd import api
    from oncilla_amd.models import workloads as wl
    from oncilla_amd.parallel.mesh import Mesh

    res = {}
    with Mesh(1, gpus=[0]) as m:
        with api.Client(daemon_rank=0, gpu=0, ns=m.ns) as c:
            allowed = sorted(os.sched_getaffinity(0))
            pairs = {t: c.alloc(api.OCM_REMOTE_GPU, local_bytes=4096, remote_bytes=4096, flags=f)
                     for t, f in (("host", api.OCM_ALLOC_HOST_TIER), ("hbm", api.OCM_ALLOC_LOOPBACK))}
            for _ in range(a.passes):
                for cpu in allowed:
                    os.sched_setaffinity(0, {cpu})
                    for t, p in pairs.items():
                        p.time_onesided(0, 4096, 20)
                        g, _ = p.time_onesided_samples(0, 4096, 200, cap_s=0.2)
                        u, _ = p.time_onesided_samples(1, 4096, 200, cap_s=0.2)
                        res.setdefault(f"{t}/cpu{cpu}", []).append(
                            (round(wl.percentile(g, 50) * 1e6, 2), round(wl.percentile(u, 50) * 1e6, 2)))
            os.sched_setaffinity(0, set(allowed))
            for p in pairs.values():
                p.free()
    print(json.dumps({"allowed": allowed, "per_cpu": res}), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump({"allowed": allowed, "per_cpu": res}, f, indent=1)


if __name__ == "__main__":
    main()

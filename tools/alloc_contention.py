"""Remote ocm_alloc latency with K apps allocating at once, each on its own
daemon of a K-daemon mesh whose daemons all sit on GPU 0 (the shared-GPU
rehearsal of the N-GPU bench).

Separates the two things the rehearsal shares that an 8-GPU node does not:
  gpu_apps: every app holds GPU 0 (local halves from its stream-ordered pool)
  cpu_apps: the apps run CPU-only (OCM_NO_GPU=1, pinned-host local halves)
against 1 app alone. Alloc/free loops timed inside libocm (2000 samples).

    python tools/alloc_contention.py [--apps 1,2,4] [--out FILE]
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

from oncilla_amd.parallel.mesh import Mesh  # noqa: E402


def child(rank: int, ns: str, gpu_app: bool, samples: int) -> None:
    from oncilla_amd import api
    from oncilla_amd.models import workloads as wl

    if not gpu_app:
        os.environ["OCM_NO_GPU"] = "1"
    with api.Client(daemon_rank=rank, gpu=0 if gpu_app else None, ns=ns) as c:
        kind = api.OCM_REMOTE_GPU if gpu_app else api.OCM_REMOTE_RDMA
        lat = wl.alloc_latency(c, kind, samples, local_bytes=64 << 10, remote_bytes=1 << 20)
        lat["lease_allocs"] = c.stats()["lease_allocs"]
    print(json.dumps(lat), flush=True)


def run(k: int, gpu_apps: bool, samples: int) -> dict:
    with Mesh(k, gpus=[0] * k, policy="stripe") as m:
        procs = [subprocess.Popen([sys.executable, os.path.abspath(__file__), "--child", str(r), "--ns", m.ns,
                                   "--samples", str(samples)] + (["--gpu-app"] if gpu_apps else []),
                                  stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True) for r in range(k)]
        out = []
        for p in procs:
            so, se = p.communicate(timeout=240)
            if p.returncode != 0:
                raise SystemExit(f"child failed: {so[-400:]} {se[-800:]}\n{m.logs()}")
            out.append(json.loads(so.strip().splitlines()[-1]))
        return {"alloc_p50_per_app": [round(o["alloc_p50_us"], 2) for o in out],
                "free_p50_per_app": [round(o["free_p50_us"], 2) for o in out],
                "lease_allocs_per_app": [o["lease_allocs"] for o in out]}


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--apps", default="1,2,4")
    ap.add_argument("--out", default=None)
    ap.add_argument("--samples", type=int, default=2000)
    ap.add_argument("--child", type=int, default=None, help=argparse.SUPPRESS)
    ap.add_argument("--ns", default=None, help=argparse.SUPPRESS)
    ap.add_argument("--gpu-app", action="store_true", help=argparse.SUPPRESS)
    args = ap.parse_args()
    if args.child is not None:
        child(args.child, args.ns, args.gpu_app, args.samples)
        return
    res = {}
    for mode in ("gpu_apps", "cpu_apps"):
        for k in [int(x) for x in args.apps.split(",")]:
            key = f"{mode}_{k}"
            res[key] = run(k, mode == "gpu_apps", args.samples)
            print(key, json.dumps(res[key]), flush=True)
    line = json.dumps(res)
    if args.out:
        with open(args.out, "w") as f:
            f.write(line + "\n")
    print(line)


if __name__ == "__main__":
    main()

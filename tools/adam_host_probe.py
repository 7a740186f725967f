#!/usr/bin/env python3
"""Fused remote Adam with its state in the pinned host tier (the N=1 bench's
fused_remote_adam extra): ms per step and state GiB/s (exp_avg + exp_avg_sq read
and written, over PCIe) for kernel variants and launch shapes, each in a fresh
process (the kernels read their knobs once).

  python3 tools/adam_host_probe.py --configs generic,host,host_g128,... --out x.json
"""
import argparse
import json
import os
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CONFIGS = {
    "generic": {"OCM_ADAM_HOST": "0"},
    "host": {"OCM_ADAM_HOST": "1"},
    "host_g64": {"OCM_ADAM_HOST": "1", "OCM_ADAM_HOST_GRID": "64"},
    "host_g128": {"OCM_ADAM_HOST": "1", "OCM_ADAM_HOST_GRID": "128"},
    "host_g256": {"OCM_ADAM_HOST": "1", "OCM_ADAM_HOST_GRID": "256"},
    "host_g96": {"OCM_ADAM_HOST": "1", "OCM_ADAM_HOST_GRID": "96"},
    "host_g160": {"OCM_ADAM_HOST": "1", "OCM_ADAM_HOST_GRID": "160"},
    "host_g192": {"OCM_ADAM_HOST": "1", "OCM_ADAM_HOST_GRID": "192"},
    "host_g128_v2": {"OCM_ADAM_HOST": "1", "OCM_ADAM_HOST_GRID": "128", "OCM_ADAM_HOST_VEC": "2"},
    "host_g256_v2": {"OCM_ADAM_HOST": "1", "OCM_ADAM_HOST_GRID": "256", "OCM_ADAM_HOST_VEC": "2"},
    "host_g64_v8": {"OCM_ADAM_HOST": "1", "OCM_ADAM_HOST_GRID": "64", "OCM_ADAM_HOST_VEC": "8"},
    "host_g128_v8": {"OCM_ADAM_HOST": "1", "OCM_ADAM_HOST_GRID": "128", "OCM_ADAM_HOST_VEC": "8"},
    "generic_g128": {"OCM_ADAM_HOST": "0", "OCM_ADAM_GRID": "128"},
    "generic_g256": {"OCM_ADAM_HOST": "0", "OCM_ADAM_GRID": "256"},
}


def child(elems: int, steps: int):
    sys.path.insert(0, REPO)
    import torch

    from oncilla_amd import api
    from oncilla_amd.models import OffloadedAdam
    from oncilla_amd.parallel.mesh import Mesh

    with Mesh(1, gpus=[0]) as m, api.Client(daemon_rank=0, gpu=0, ns=m.ns) as c:
        p = torch.zeros(elems, device="cuda:0").requires_grad_()
        p.grad = torch.randn(elems, device="cuda:0")
        opt = OffloadedAdam([p], c, lr=1e-3, flags=api.OCM_ALLOC_HOST_TIER)
        try:
            tiers = {e["tier"] for e in opt.allocs[0].remote_info()["extents"]}
            for _ in range(2):
                opt.step()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(steps):
                opt.step()
            torch.cuda.synchronize()
            s = (time.perf_counter() - t0) / steps
        finally:
            opt.close()
    print(json.dumps({"ms_per_step": round(s * 1e3, 3), "state_GiBps": round(16 * elems / s / (1 << 30), 2),
                      "tiers": sorted(tiers)}))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default=",".join(CONFIGS))
    ap.add_argument("--elems", type=int, default=64 << 20)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--repeat", type=int, default=2)
    ap.add_argument("--out", default=None)
    ap.add_argument("--child", action="store_true")
    a = ap.parse_args()
    if a.child:
        child(a.elems, a.steps)
        return
    out = {}
    for r in range(a.repeat):
        for name in a.configs.split(","):
            env = dict(os.environ, **CONFIGS[name])
            p = subprocess.run([sys.executable, __file__, "--child", "--elems", str(a.elems), "--steps", str(a.steps)],
                               env=env, capture_output=True, text=True, timeout=300)
            key = name if a.repeat == 1 else f"{name}#{r}"
            try:
                out[key] = json.loads(p.stdout.strip().splitlines()[-1])
            except (IndexError, ValueError):
                out[key] = {"error": (p.stderr or p.stdout)[-400:]}
            print(key, out[key], flush=True)
    doc = {"what": "tools/adam_host_probe.py: OffloadedAdam fused step, fp32 params, moments in the pinned host tier "
                   "(1 daemon, 1 GPU); state_GiBps counts exp_avg + exp_avg_sq read and written per step",
           "elems": a.elems, "result": out}
    if a.out:
        with open(a.out, "w") as f:
            json.dump(doc, f, indent=1)


if __name__ == "__main__":
    main()

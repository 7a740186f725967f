"""Which HIP runtime does libocm run on, and does it matter for latency?

PyTorch's ROCm wheel bundles its own libamdhip64.so.7 / libhsa-runtime64.so.1
(same SONAMEs as /opt/rocm's). Whichever is loaded first serves the whole
process: `import torch` first puts libocm on torch's bundled runtime; loading
libocm first puts torch on /opt/rocm's. This probe measures remote ocm_alloc /
ocm_free latency and 4 KiB put/get in one mode per process:
  torch_first   import torch, then libocm (what bench.py did in round 1)
  ocm_first     libocm (-> /opt/rocm runtime), then import torch
  no_torch      libocm only

    python tools/runtime_probe.py [--out FILE]
"""
from __future__ import annotations

import argparse
import json
import os
import re
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def child(mode: str) -> None:
    if mode == "torch_first":
        import torch  # noqa: F401
    from oncilla_amd import api

    api.load()
    if mode == "ocm_first":
        import torch  # noqa: F401
    from oncilla_amd.models import workloads as wl
    from oncilla_amd.parallel.mesh import Mesh

    maps = open("/proc/self/maps").read()
    hip = sorted(set(re.findall(r"\S*libamdhip64\S*", maps)))
    out = {"hip_runtime": hip}
    with Mesh(1, gpus=[0]) as m:
        with api.Client(daemon_rank=0, gpu=0, ns=m.ns) as c:
            lat = wl.alloc_latency(c, api.OCM_REMOTE_GPU, 2000, local_bytes=64 << 10, remote_bytes=1 << 20)
            out["alloc_p50_us"] = round(lat["alloc_p50_us"], 2)
            out["free_p50_us"] = round(lat["free_p50_us"], 2)
            loc = wl.alloc_latency(c, api.OCM_LOCAL_HOST, 2000, local_bytes=1 << 20)
            out["local_alloc_p50_us"] = round(loc["alloc_p50_us"], 2)
            a = c.alloc(api.OCM_REMOTE_GPU, local_bytes=1 << 20, remote_bytes=1 << 20)
            a.time_onesided(1, 4096, 50)
            out["put4k_us"] = round(min(a.time_onesided(1, 4096, 500) for _ in range(3)) * 1e6, 2)
            out["get4k_us"] = round(min(a.time_onesided(0, 4096, 500) for _ in range(3)) * 1e6, 2)
            a.free()
    print(json.dumps(out))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--child", default=None)
    ap.add_argument("--out", default=None)
    ap.add_argument("--modes", default="torch_first,ocm_first,no_torch")
    ap.add_argument("--repeat", type=int, default=2)
    args = ap.parse_args()
    if args.child:
        child(args.child)
        return
    res = {}
    for rep in range(args.repeat):
        for mode in args.modes.split(","):
            r = subprocess.run([sys.executable, os.path.abspath(__file__), "--child", mode], capture_output=True,
                               text=True, timeout=300)
            key = f"{mode}#{rep}"
            res[key] = json.loads(r.stdout.strip().splitlines()[-1]) if r.returncode == 0 else {
                "error": (r.stdout + r.stderr)[-600:]}
            print(key, json.dumps(res[key]), flush=True)
    if args.out:
        with open(args.out, "w") as f:
            f.write(json.dumps(res) + "\n")


if __name__ == "__main__":
    main()

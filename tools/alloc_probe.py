"""ocm_alloc / ocm_free latency of GPU kinds vs local-half size, with the local
half from the stream-ordered pool (OCM_LOCAL_POOL=1, default) or hipMalloc.

    python tools/alloc_probe.py [--samples N] [--out gpurun_out/alloc_probe.json]

Starts a 2-daemon mesh on GPU 0 (rank1's HBM is the remote half), then runs
each mode in a child process so the pool setting is fresh.
"""
import argparse
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

SIZES = [4096, 1 << 20, 64 << 20, 1 << 30]


def child(ns: str, samples: int) -> None:
    from oncilla_amd import api
    from oncilla_amd.models import workloads as wl

    out = {}
    with api.Client(daemon_rank=0, gpu=0, ns=ns) as c:
        for kind, name in ((api.OCM_LOCAL_GPU, "local_gpu"), (api.OCM_REMOTE_GPU, "remote_gpu"),
                           (api.OCM_REMOTE_RDMA, "remote_rdma_pinned_local")):
            for s in SIZES:
                remote = s if kind != api.OCM_LOCAL_GPU else 0
                r = wl.alloc_latency(c, kind, samples, local_bytes=s, remote_bytes=remote)
                out[f"{name}_{s}"] = {k: round(v, 2) if isinstance(v, float) else v for k, v in r.items()}
    print(json.dumps(out))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--samples", type=int, default=50)
    ap.add_argument("--out", default="")
    ap.add_argument("--child", default="")
    args = ap.parse_args()
    if args.child:
        child(args.child, args.samples)
        return
    from oncilla_amd.parallel import Mesh

    res = {}
    with Mesh(2, gpus=[0, 0]) as m:
        for mode in ("1", "0"):
            env = dict(m.client_env(0), OCM_LOCAL_POOL=mode)
            p = subprocess.run([sys.executable, __file__, "--child", m.ns, "--samples", str(args.samples)],
                               env=env, capture_output=True, text=True, timeout=600)
            if p.returncode != 0:
                raise SystemExit(p.stderr)
            res["pool" if mode == "1" else "hipmalloc"] = json.loads(p.stdout.strip().splitlines()[-1])
    txt = json.dumps(res, indent=1)
    print(txt)
    if args.out:
        os.makedirs(os.path.dirname(args.out) or ".", exist_ok=True)
        with open(args.out, "w") as f:
            f.write(txt + "\n")


if __name__ == "__main__":
    main()

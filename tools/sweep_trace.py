#!/usr/bin/env python3
"""Per-op wall time of bench.py's R/W sweep order (get then put of every size),
to find ops that pay more in the sweep than in a repeated-op loop.

    python tools/sweep_trace.py [--remote loopback|host] [--steps 3]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from oncilla_amd import api  # noqa: E402
from oncilla_amd.models import workloads as wl  # noqa: E402
from oncilla_amd.parallel.mesh import Mesh  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--remote", default="loopback", choices=["loopback", "host"])
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--max-bytes", type=int, default=1 << 30)
    ap.add_argument("--torch", action="store_true", help="initialise torch's CUDA context first, as bench.py does")
    ap.add_argument("--verify", action="store_true", help="fill/put/get/check first, as bench.py does")
    args = ap.parse_args()
    if args.torch:
        import torch

        torch.cuda.synchronize(0)
    flags = api.OCM_ALLOC_LOOPBACK if args.remote == "loopback" else api.OCM_ALLOC_HOST_TIER
    with Mesh(1, gpus=[0]) as m, api.Client(daemon_rank=0, gpu=0, ns=m.ns) as c:
        n = 2 * args.max_bytes + 1
        a = c.alloc(api.OCM_REMOTE_GPU, local_bytes=n, remote_bytes=n, flags=flags)
        sizes = wl.sweep_sizes(4096, args.max_bytes)
        if args.verify:
            a.fill(seed=1234, nbytes=args.max_bytes)
            a.put(0, 0, args.max_bytes)
            a.fill(seed=0, nbytes=args.max_bytes)
            a.get(0, 0, args.max_bytes)
            assert a.check(seed=1234, nbytes=args.max_bytes) == 0
        wl.rw_sweep_step(a, sizes)
        steps = []
        for _ in range(args.steps):
            rec, t_step = [], time.perf_counter()
            for s in sizes:
                for op, f in (("get", a.get), ("put", a.put)):
                    t0 = time.perf_counter()
                    f(0, 0, s)
                    rec.append((op, s, round((time.perf_counter() - t0) * 1e6, 2)))
            steps.append({"step_ms": round((time.perf_counter() - t_step) * 1e3, 3), "ops": rec})
        char = wl.characterize(a, sizes)
        a.free()
    out = {"remote": args.remote, "steps": steps,
           "char_us": {str(s): (round(v["get_s"] * 1e6, 2), round(v["put_s"] * 1e6, 2)) for s, v in char.items()}}
    print(json.dumps(out))


if __name__ == "__main__":
    main()

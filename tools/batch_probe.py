"""Scatter/gather throughput: N small one-sided gets (random remote pieces) as
one ocm_copy_onesided_batch vs N blocking ocm_copy_onesided calls.

    python tools/batch_probe.py [--out gpurun_out/batch_probe.json]

Runs a 4-daemon mesh on GPU 0 (remote half striped over 3 owners' HBM) and a
1-daemon mesh (remote half in the pinned host tier).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

from oncilla_amd import api  # noqa: E402
from oncilla_amd.parallel import Mesh  # noqa: E402


def measure(a, nbytes, piece, count, reps=5):
    rng = np.random.default_rng(piece)
    slots = nbytes // piece
    ops = [(0, i * piece, int(s) * piece, piece) for i, s in enumerate(rng.choice(slots, size=count, replace=False))]
    prepared = api.batch_ops(ops)  # time the call, not the Python list conversion
    a.batch(prepared)  # warm
    t = []
    for _ in range(reps):
        t0 = time.perf_counter()
        a.batch(prepared)
        t.append(time.perf_counter() - t0)
    batch_s = float(np.median(t))
    plan_s = None
    if a._c.device >= 0:
        with a._c.plan() as plan:  # the same list as a captured graph: no per-call planning/upload
            plan.add(a, prepared)
            plan.launch()
            tp = []
            for _ in range(reps):
                t0 = time.perf_counter()
                plan.launch()
                tp.append(time.perf_counter() - t0)
            plan_s = float(np.median(tp))
    loop_ops = ops[: min(count, 2000)]
    for f, lo, ro, n in loop_ops[:10]:
        a.get(lo, ro, n)
    t0 = time.perf_counter()
    for f, lo, ro, n in loop_ops:
        a.get(lo, ro, n)
    loop_s = (time.perf_counter() - t0) / len(loop_ops) * count
    moved = piece * count
    return {"piece": piece, "count": count, "batch_us": round(batch_s * 1e6, 1), "loop_us": round(loop_s * 1e6, 1),
            "batch_GiBps": round(moved / batch_s / 2**30, 2), "loop_GiBps": round(moved / loop_s / 2**30, 3),
            "speedup": round(loop_s / batch_s, 1),
            "plan_us": round(plan_s * 1e6, 1) if plan_s else None,
            "plan_GiBps": round(moved / plan_s / 2**30, 2) if plan_s else None}


def run(mesh_n, label, out):
    with Mesh(mesh_n, gpus=[0] * mesh_n, policy="stripe") as m:
        with api.Client(daemon_rank=0, gpu=0, ns=m.ns) as c:
            n = 256 << 20
            a = c.alloc(api.OCM_REMOTE_GPU, local_bytes=n, remote_bytes=n, stripe_unit=1 << 20)
            rows = []
            for piece, count in ((64, 4096), (4096, 256), (4096, 4096), (65536, 1024), (4096, 32768)):
                rows.append(measure(a, n, piece, count))
                print(label, rows[-1], flush=True)
            a.free()
    out[label] = rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    out = {}
    run(4, "hbm_striped3", out)
    run(1, "host_tier", out)
    if args.out:
        os.makedirs(os.path.dirname(args.out) or ".", exist_ok=True)
        with open(args.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()

"""OffloadedAdam step time vs torch.optim.Adam with resident moments.

A flat set of fp32 parameters (default 256 Mi elements = 1 GiB, so 2 GiB of
moments) with fixed random gradients. Configurations:
  torch_resident: torch.optim.Adam (foreach), moments in this GPU's HBM; torch_fused_resident: fused=True
  ocm_*_fused:    OffloadedAdam mode="fused": one gfx950 kernel per parameter reads/writes the
                  moments in place in remote memory (no staging)
  ocm_hbm:        OffloadedAdam, moments in another daemon's HBM (IPC; on a 1-GPU box
                  the daemon shares the GPU, standing in for a peer over xGMI)
  ocm_host:       OffloadedAdam, moments in the pinned host tier (PCIe)
Each is warmed up, then timed over --steps steps with one device sync at the end.

    python tools/optim_offload_probe.py [--elems N] [--chunk N] [--steps K] [--out FILE]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main() -> None:
    import torch

    from oncilla_amd import api
    from oncilla_amd.models import OffloadedAdam
    from oncilla_amd.parallel.mesh import Mesh

    ap = argparse.ArgumentParser()
    ap.add_argument("--elems", type=int, default=256 << 20)
    ap.add_argument("--chunk", default="16777216,67108864")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--out", default=None)
    ap.add_argument("--fused-hbm-only", action="store_true", help="only the fused kernel on HBM state (tuning sweeps)")
    args = ap.parse_args()
    dev = "cuda:0"
    n_params = 4
    per = args.elems // n_params
    params = [torch.zeros(per, device=dev).requires_grad_() for _ in range(n_params)]
    for p in params:
        p.grad = torch.randn(per, device=dev)

    def timed(step_fn):
        for _ in range(2):
            step_fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            step_fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / args.steps

    res = {"elems": args.elems, "moment_bytes": 8 * args.elems, "steps": args.steps}
    for name, kw in (() if args.fused_hbm_only else (("torch_resident_ms", {}), ("torch_fused_resident_ms", {"fused": True}))):
        try:
            opt = torch.optim.Adam(params, lr=1e-3, **kw)
            res[name] = round(timed(opt.step) * 1e3, 3)
        except Exception as e:  # noqa: BLE001 - recorded
            res[name] = repr(e)[:120]
        opt = None
        torch.cuda.empty_cache()
    print(json.dumps(res), flush=True)
    with Mesh(2, gpus=[0, 0]) as m:
        with api.Client(daemon_rank=0, gpu=0, ns=m.ns) as c:
            for name, flags in (("ocm_hbm", 0),) + ((("ocm_host", api.OCM_ALLOC_HOST_TIER),) if not args.fused_hbm_only else ()):
                for chunk in [0] + ([int(x) for x in args.chunk.split(",")] if not args.fused_hbm_only else []):
                    mode = "fused" if chunk == 0 else "staged"
                    o = OffloadedAdam(params, c, lr=1e-3, chunk_elems=chunk or 1, flags=flags, mode=mode)
                    tier = o.allocs[0].remote_info()["extents"][0]["tier"]
                    t = timed(o.step)
                    o.close()
                    key = f"{name}_fused_ms" if chunk == 0 else f"{name}_chunk{chunk >> 20}Mi_ms"
                    res[key] = round(t * 1e3, 3)
                    # bytes through the data plane per step: every moment read and written once
                    res[key.replace("_ms", "_GiBps")] = round(2 * 8 * args.elems / t / (1 << 30), 2)
                    res[f"{name}_tier"] = {1: "host", 2: "hbm"}[tier]
                    print(key, res[key], flush=True)
            if not args.fused_hbm_only:
                # mixed precision: bf16 params / grads here, fp32 master + moments remote (3 GiB)
                p16 = [p.detach().to(torch.bfloat16).requires_grad_() for p in params]
                for q, p in zip(p16, params):
                    q.grad = p.grad.to(torch.bfloat16)
                o = OffloadedAdam(p16, c, lr=1e-3)
                t = timed(o.step)
                o.close()
                res["ocm_hbm_fused_bf16_ms"] = round(t * 1e3, 3)
                res["ocm_hbm_fused_bf16_local_bytes_per_param"] = 4
                print("ocm_hbm_fused_bf16_ms", res["ocm_hbm_fused_bf16_ms"], flush=True)
                del p16
    line = json.dumps(res)
    if args.out:
        with open(args.out, "w") as f:
            f.write(line + "\n")
    print(line)


if __name__ == "__main__":
    main()

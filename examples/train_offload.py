"""Training with the optimizer state in disaggregated memory.

A small MLP regression trained with models.OffloadedAdam: the Adam moments (and,
with --bf16, the fp32 master weights) live in the HBM of other daemons' GPUs,
striped over them (on a one-GPU box the daemons share GPU 0), and one fused
gfx950 kernel per parameter updates them in place. Without a GPU the staged path
runs on the CPU with the state in the daemons' host tier.

    python examples/train_offload.py [--gpu 0] [--bf16] [--steps 200]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from oncilla_amd import api  # noqa: E402
from oncilla_amd.models import OffloadedAdam  # noqa: E402
from oncilla_amd.parallel import Mesh  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpu", type=int, default=None)
    ap.add_argument("--bf16", action="store_true")
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--daemons", type=int, default=3)
    args = ap.parse_args()
    on_gpu = args.gpu is not None
    dev = f"cuda:{args.gpu}" if on_gpu else "cpu"
    dtype = torch.bfloat16 if args.bf16 else torch.float32
    torch.manual_seed(0)
    model = torch.nn.Sequential(torch.nn.Linear(64, 256), torch.nn.GELU(), torch.nn.Linear(256, 1)).to(dev, dtype)
    teacher = torch.nn.Sequential(torch.nn.Linear(64, 32), torch.nn.Tanh(), torch.nn.Linear(32, 1)).to(dev)
    gpus = [args.gpu] * args.daemons if on_gpu else None
    with Mesh(args.daemons, gpus=gpus, policy="stripe") as mesh:
        with api.Client(daemon_rank=0, gpu=args.gpu, ns=mesh.ns) as c:
            opt = OffloadedAdam(model.parameters(), c, lr=3e-3)
            tiers = sorted({e["tier"] for e in opt.allocs[0].remote_info()["extents"]})
            first = last = None
            for step in range(args.steps):
                x = torch.randn(256, 64, device=dev)
                with torch.no_grad():
                    y = teacher(x)
                loss = torch.nn.functional.mse_loss(model(x.to(dtype)).float(), y)
                opt.zero_grad()
                loss.backward()
                opt.step()
                if step == 0:
                    first = loss.item()
                last = loss.item()
            opt.close()
    where = "+".join({1: "host tier", 2: "peer HBM"}[t] for t in tiers)
    print(f"{args.steps} steps, mode={opt.mode}, {dtype}, optimizer state in {where}: "
          f"loss {first:.4f} -> {last:.4f}")
    if not last < 0.5 * first:
        raise SystemExit("loss did not go down")


if __name__ == "__main__":
    main()

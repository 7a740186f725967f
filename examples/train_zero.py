"""Data-parallel training, sharded optimizer (ZeRO-1) with offloaded state.

Run one process per GPU (or CPU rank):

    torchrun --nproc-per-node 2 --master-addr 127.0.0.1 examples/train_zero.py [--cpu]

Every rank starts the ocmd daemon of its GPU; the daemons form one mesh. Each
rank trains the same MLP on its own batches with parallel.ShardedOffloadedAdam:
gradients are reduce-scattered (RCCL, or gloo with --cpu), each rank updates its
shard with the state in other ranks' memory (fused remote-Adam kernel on a GPU),
and the shards are all-gathered. Every rank also replays the whole job in one
process with torch.optim.Adam (all ranks' batches, averaged gradients) and
checks that the parameters agree.
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from oncilla_amd import api  # noqa: E402
from oncilla_amd.parallel.mesh import Mesh, free_ports  # noqa: E402
from oncilla_amd.parallel.zero import ShardedOffloadedAdam  # noqa: E402


def make_model(dev):
    torch.manual_seed(1)
    return torch.nn.Sequential(torch.nn.Linear(32, 97), torch.nn.Tanh(), torch.nn.Linear(97, 3)).to(dev)


def batch(step, r, dev):
    g = torch.Generator().manual_seed(1000 * step + r)
    x = torch.randn(64, 32, generator=g)
    y = torch.randn(64, 3, generator=g)
    return x.to(dev), y.to(dev)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cpu", action="store_true")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--share-gpu", action="store_true", help="all ranks on GPU 0 (rehearsal on a 1-GPU box)")
    args = ap.parse_args()
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    local = int(os.environ.get("LOCAL_RANK", "0"))
    gpu = None if args.cpu else (0 if args.share_gpu else local)
    if args.cpu:
        os.environ["OCM_NO_GPU"] = "1"
    dev = "cpu" if args.cpu else f"cuda:{gpu}"
    if not args.cpu:
        torch.cuda.set_device(gpu)
    # RCCL takes one rank per GPU; the shared-GPU rehearsal runs its collectives on gloo
    dist.init_process_group("gloo" if (args.cpu or args.share_gpu) else "nccl")

    def gather(obj):
        out = [None] * world
        dist.all_gather_object(out, obj)
        return out

    # one ocmd per rank, one mesh (rank 0 picks the ports)
    import secrets

    ports, key = gather((free_ports(world), secrets.token_hex(16)) if rank == 0 else None)[0]
    ns = f"zero{os.environ.get('MASTER_PORT', '0')}_{ports[0]}"
    workdir = os.path.join("/tmp", f"ocm_{ns}")
    os.makedirs(workdir, exist_ok=True)
    gpus = gather(gpu) if gpu is not None else [None] * world
    mesh = Mesh(world, gpus=gpus, ns=ns, policy="stripe", workdir=workdir, ports=ports, ranks=[rank],
                key=key).start(timeout=120)
    dist.barrier()
    ok = False
    try:
        with api.Client(daemon_rank=rank, gpu=gpu, ns=ns) as c:
            model = make_model(dev)
            ref = make_model(dev)
            opt = ShardedOffloadedAdam(model.parameters(), c, lr=1e-2, weight_decay=0.01)
            ref_opt = torch.optim.Adam(ref.parameters(), lr=1e-2, weight_decay=0.01)
            tiers = sorted({e["tier"] for e in opt.opt.allocs[0].remote_info()["extents"]})
            for step in range(args.steps):
                x, y = batch(step, rank, dev)
                opt.zero_grad()
                torch.nn.functional.mse_loss(model(x), y).backward()
                opt.step()
                ref_opt.zero_grad()
                loss = sum(torch.nn.functional.mse_loss(ref(*batch(step, r, dev)[:1]), batch(step, r, dev)[1])
                           for r in range(world)) / world
                loss.backward()
                ref_opt.step()
            opt.close()
            worst = max((a - b).abs().max().item() for a, b in zip(model.parameters(), ref.parameters()))
            ok = worst < 1e-5
            if rank == 0:
                where = "+".join({1: "host tier", 2: "peer HBM"}[t] for t in tiers)
                print(f"{world} ranks, {args.steps} steps, state shards in {where}, mode={opt.opt.mode}: "
                      f"max |param - single-process Adam| = {worst:.2e}", flush=True)
        dist.barrier()
    finally:
        mesh.stop()
        dist.destroy_process_group()
    if not ok:
        raise SystemExit(f"rank {rank}: parameters diverge from the single-process reference")


if __name__ == "__main__":
    main()

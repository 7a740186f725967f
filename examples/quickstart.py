"""Quick tour of the Python API on a self-started mesh.

    python examples/quickstart.py            # CPU-only daemons (works anywhere)
    python examples/quickstart.py --gpu 0    # daemons and the app on MI355X #0

1. start a 3-daemon mesh (rank0 = directory); 2. allocate a remote pair,
striped over the two peers; 3. one-sided put/get with a data check;
4. a batched scatter/gather list in one call; 5. stats and free.
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from oncilla_amd import api  # noqa: E402
from oncilla_amd.parallel import Mesh  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpu", type=int, default=None)
    args = ap.parse_args()
    if args.gpu is None:
        os.environ["OCM_NO_GPU"] = "1"
    gpus = [args.gpu] * 3 if args.gpu is not None else None
    kind = api.OCM_REMOTE_GPU if args.gpu is not None else api.OCM_REMOTE_RDMA
    with Mesh(3, gpus=gpus, policy="stripe") as mesh:
        with api.Client(daemon_rank=0, gpu=args.gpu, ns=mesh.ns) as c:
            n = 8 << 20
            a = c.alloc(kind, local_bytes=n, remote_bytes=n, stripe_unit=1 << 20)
            owners = [e["owner_rank"] for e in a.remote_info()["extents"]]
            a.fill(seed=1)                 # deterministic pattern in the local half
            a.put(0, 0, n)                 # local -> remote (striped over `owners`)
            a.fill(seed=0)
            a.get(0, 0, n)                 # remote -> local
            assert a.check(seed=1) == 0
            print(f"{n >> 20} MiB round trip, striped over ranks {owners}")
            # scatter/gather: 64 gets of 4 KiB from random remote pages, one call
            ops = [(0, i * 4096, ((i * 37) % 2048) * 4096, 4096) for i in range(64)]
            a.batch(ops)
            print("batched 64 gets in one launch; counters:", {k: v for k, v in api.counters().items() if "batch" in k})
            for r in range(3):
                st = c.stats(r)
                print(f"rank {r}: host_used={st['host_used'] >> 20} MiB gpu_used={st['gpu_used'] >> 20} MiB")
            a.free()


if __name__ == "__main__":
    main()

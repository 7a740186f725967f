"""Model weights in another GPU's HBM: a torch model built inside a
`RemoteMemPool` keeps its parameters in a peer daemon's HBM (reached over
xGMI), and its forward pass reads them in place. No copies, and the local GPU's
HBM stays free for activations. On a one-GPU box every daemon shares GPU 0,
so the "peer" HBM is local (a same-GPU stand-in).

    python examples/remote_weights.py [--daemons 2]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from oncilla_amd import api  # noqa: E402
from oncilla_amd.parallel import Mesh  # noqa: E402
from oncilla_amd.torch_pool import RemoteMemPool  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--daemons", type=int, default=2)
    args = ap.parse_args()
    ndev = torch.cuda.device_count()
    gpus = [r % ndev for r in range(args.daemons)]  # one per GPU when the node has them
    with Mesh(args.daemons, gpus=gpus) as mesh:
        with api.Client(daemon_rank=0, gpu=0, ns=mesh.ns) as c:
            torch.manual_seed(0)
            local = torch.nn.Sequential(torch.nn.Linear(2048, 8192), torch.nn.GELU(), torch.nn.Linear(8192, 2048))
            local = local.to("cuda:0", torch.bfloat16)
            pool = RemoteMemPool(c, remote_rank=1)
            with pool:  # parameters allocated here live in rank 1's HBM
                remote = torch.nn.Sequential(torch.nn.Linear(2048, 8192), torch.nn.GELU(),
                                             torch.nn.Linear(8192, 2048)).to("cuda:0", torch.bfloat16)
                remote.load_state_dict(local.state_dict())
            x = torch.randn(64, 2048, device="cuda:0", dtype=torch.bfloat16)
            with torch.no_grad():
                same = torch.equal(remote(x), local(x))
            st = RemoteMemPool.stats()
            print(f"weights in rank {1}'s HBM (gpu {gpus[1]}): {st['bytes'] >> 20} MiB in {st['blocks']} blocks; "
                  f"forward matches the local copy: {same}")
            assert same
            del remote, pool


if __name__ == "__main__":
    main()

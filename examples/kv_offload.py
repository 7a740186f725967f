"""Paged KV-cache offload on an MI355X: swap KV blocks of idle sequences to a
pool in other GPUs' HBM (or the pinned host tier on a single-daemon node) and
back, each swap list being one batched launch ordered against torch's stream.

    python examples/kv_offload.py [--daemons 4]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from oncilla_amd import api  # noqa: E402
from oncilla_amd.models import PagedKVOffload  # noqa: E402
from oncilla_amd.parallel import Mesh  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--daemons", type=int, default=4)
    args = ap.parse_args()
    with Mesh(args.daemons, gpus=[0] * args.daemons, policy="stripe") as mesh:
        with api.Client(daemon_rank=0, gpu=0, ns=mesh.ns) as c:
            # 256 GPU blocks of (K/V, 16 tokens, 8 heads, 128 dims) fp16 = 64 KiB; pool of 2048 blocks
            kv = PagedKVOffload(c, 256, 2048, (2, 16, 8, 128), dtype=torch.float16)
            kv.gpu_cache.normal_()
            before = kv.gpu_cache[:64].clone()
            kv.swap_out([(g, 1000 + g) for g in range(64)])     # 64 blocks out (coalesced: 1 op)
            kv.gpu_cache[:64].zero_()                            # blocks reused by other sequences
            kv.swap_in([(1000 + g, g) for g in range(64)])      # ... and back before the next step
            assert torch.equal(kv.gpu_cache[:64], before)        # torch's stream waited for the copies
            print("64 KV blocks swapped out and back; pool on", sorted({e["owner_rank"] for e in kv.alloc.remote_info()["extents"]}))
            kv.close()


if __name__ == "__main__":
    main()

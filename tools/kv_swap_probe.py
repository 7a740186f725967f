"""KV-cache block swap: one batched launch (PagedKVOffload) vs the usual
per-block copy loop (torch `copy_(non_blocking=True)` per block).

    python tools/kv_swap_probe.py [--out gpurun_out/kv_swap_probe.json]

Pools: pinned host (1 daemon: host tier; baseline: pinned CPU tensor) and HBM
(4 daemons on GPU 0 striped; baseline: a device tensor on the same GPU).
"""
import argparse
import json
import os
import random
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

from oncilla_amd import api  # noqa: E402
from oncilla_amd.models import PagedKVOffload  # noqa: E402
from oncilla_amd.parallel import Mesh  # noqa: E402

BLOCK = (2, 16, 8, 128)  # K+V, 16 tokens, 8 kv heads, head dim 128, fp16 = 64 KiB


def timeit(fn, reps=7):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    return sorted(ts)[len(ts) // 2]


def case(label, n_daemons, n_gpu_blocks, n_pool_blocks, n_swap, pool_device):
    rng = random.Random(0)
    with Mesh(n_daemons, gpus=[0] * n_daemons, policy="stripe") as m:
        with api.Client(daemon_rank=0, gpu=0, ns=m.ns) as c:
            kv = PagedKVOffload(c, n_gpu_blocks, n_pool_blocks, BLOCK)
            kv.gpu_cache.normal_()
            pairs = list(zip(rng.sample(range(n_gpu_blocks), n_swap), rng.sample(range(n_pool_blocks), n_swap)))
            out_np = np.array(pairs, dtype=np.int64)
            in_np = out_np[:, ::-1].copy()
            t_out = timeit(lambda: kv.swap_out(out_np, async_=True))
            t_in = timeit(lambda: kv.swap_in(in_np, async_=True))
            # baseline: one copy per block
            pool = torch.empty((n_pool_blocks, *BLOCK), dtype=torch.float16, device=pool_device,
                               pin_memory=(pool_device == "cpu"))
            cache = kv.gpu_cache
            b_out = timeit(lambda: [pool[p].copy_(cache[g], non_blocking=True) for g, p in pairs])
            b_in = timeit(lambda: [cache[g].copy_(pool[p], non_blocking=True) for g, p in pairs])
            kv.close()
    nbytes = n_swap * kv.block_bytes
    row = {"case": label, "blocks": n_swap, "block_KiB": kv.block_bytes >> 10,
           "swap_out_us": round(t_out * 1e6, 1), "swap_in_us": round(t_in * 1e6, 1),
           "baseline_out_us": round(b_out * 1e6, 1), "baseline_in_us": round(b_in * 1e6, 1),
           "swap_out_GiBps": round(nbytes / t_out / 2**30, 1), "swap_in_GiBps": round(nbytes / t_in / 2**30, 1),
           "baseline_out_GiBps": round(nbytes / b_out / 2**30, 1), "baseline_in_GiBps": round(nbytes / b_in / 2**30, 1)}
    print(row, flush=True)
    return row


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="")
    ap.add_argument("--host-only", action="store_true", help="the host-tier pool cases only (and a 4096-block swap)")
    args = ap.parse_args()
    if args.host_only:
        rows = [case("host_tier_pool", 1, 4096, 8192, n, "cpu") for n in (256, 1024, 4096)]
    else:
        rows = [case("host_tier_pool", 1, 1024, 4096, 256, "cpu"),
                case("host_tier_pool", 1, 1024, 4096, 1024, "cpu"),
                case("hbm_pool_striped3", 4, 1024, 4096, 256, "cuda:0"),
                case("hbm_pool_striped3", 4, 1024, 4096, 1024, "cuda:0")]
    if args.out:
        os.makedirs(os.path.dirname(args.out) or ".", exist_ok=True)
        with open(args.out, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()

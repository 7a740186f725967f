"""Paged KV-cache offload (oncilla_amd.models.PagedKVOffload): swap lists run as
one batched one-sided launch; checked against a plain torch model of the pool."""
import random

import pytest
import torch

from oncilla_amd import api
from oncilla_amd.models import PagedKVOffload, coalesce


def test_coalesce_runs():
    assert coalesce([(3, 10), (1, 8), (2, 9), (7, 0), (8, 2)]) == [(1, 8, 3), (7, 0, 1), (8, 2, 1)]
    assert coalesce([]) == []


def _exercise(kv, rounds, seed, device):
    rng = random.Random(seed)
    g = torch.Generator(device="cpu").manual_seed(seed)
    pool_model = {}
    for r in range(rounds):
        fresh = torch.randn((kv.num_gpu_blocks, *kv.block_shape), generator=g).to(kv.dtype).to(device)
        kv.gpu_cache.copy_(fresh)  # written by torch on its stream; swap_out must see it
        k = rng.randint(1, kv.num_gpu_blocks)
        gpu_ids = rng.sample(range(kv.num_gpu_blocks), k)
        pool_ids = rng.sample(range(kv.num_pool_blocks), k)
        if r % 2 == 0:  # consecutive runs get coalesced
            base = rng.randrange(0, kv.num_pool_blocks - k + 1)
            pool_ids = list(range(base, base + k))
            gpu_ids = sorted(gpu_ids)
        kv.swap_out(list(zip(gpu_ids, pool_ids)), async_=bool(r % 3))
        for gi, pi in zip(gpu_ids, pool_ids):
            pool_model[pi] = fresh[gi].clone()
        kv.gpu_cache.zero_()
        known = list(pool_model)
        back = rng.sample(known, min(len(known), kv.num_gpu_blocks))
        dst = rng.sample(range(kv.num_gpu_blocks), len(back))
        kv.swap_in(list(zip(back, dst)), async_=bool(r % 2))
        # torch reads on its stream right away: swap_in made it wait for the copies
        for pi, gi in zip(back, dst):
            assert torch.equal(kv.gpu_cache[gi], pool_model[pi]), (r, pi, gi)
    kv.wait()


def test_kv_offload_cpu(mesh_factory, monkeypatch):
    monkeypatch.setenv("OCM_NO_GPU", "1")
    m = mesh_factory(3, policy="stripe")
    with api.Client(daemon_rank=0, ns=m.ns) as c:
        kv = PagedKVOffload(c, 12, 40, (2, 4, 8), dtype=torch.float32, kind=api.OCM_REMOTE_RDMA, stripe_unit=4096)
        _exercise(kv, 6, seed=3, device="cpu")
        with pytest.raises(IndexError):
            kv.swap_out([(12, 0)])
        kv.close()


@pytest.mark.gpu
@pytest.mark.parametrize("n_daemons", [1, 4])  # 1: pool in the pinned host tier; 4: striped over 3 peers' HBM
def test_kv_offload_gpu(mesh_factory, n_daemons):
    m = mesh_factory(n_daemons, gpus=[0] * n_daemons, policy="stripe")
    with api.Client(daemon_rank=0, gpu=0, ns=m.ns) as c:
        kv = PagedKVOffload(c, 64, 256, (2, 16, 8, 64), dtype=torch.float16)  # 32 KiB blocks
        side = torch.cuda.Stream()
        with torch.cuda.stream(side):  # torch work on a non-default stream
            _exercise(kv, 8, seed=n_daemons, device="cuda:0")
        torch.cuda.synchronize()
        kv.close()

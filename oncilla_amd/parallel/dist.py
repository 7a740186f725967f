"""torch.distributed glue for multi-GPU runs: one process per MI355X.

The benchmark and multi-rank tests run one app process per GPU under
`torch.distributed.run` (RCCL backend "nccl" on ROCm, gloo on CPU). Every rank
starts the ocmd daemon of its own GPU; the daemon mesh itself does not depend
on torch — this module only coordinates the app processes (port exchange,
barriers, max-over-ranks timing reductions).
"""
from __future__ import annotations

import os
from dataclasses import dataclass
from typing import Optional


@dataclass
class DistInfo:
    rank: int = 0
    world: int = 1
    local_rank: int = 0
    backend: Optional[str] = None

    @property
    def is_dist(self) -> bool:
        return self.world > 1


def env_info() -> DistInfo:
    return DistInfo(
        rank=int(os.environ.get("RANK", "0")),
        world=int(os.environ.get("WORLD_SIZE", "1")),
        local_rank=int(os.environ.get("LOCAL_RANK", "0")),
    )


def init(use_gpu: bool) -> DistInfo:
    info = env_info()
    if info.world > 1:
        import torch
        import torch.distributed as dist

        info.backend = "nccl" if use_gpu else "gloo"
        if use_gpu:
            torch.cuda.set_device(info.local_rank)
            dist.init_process_group(info.backend, device_id=torch.device("cuda", info.local_rank))
        else:
            dist.init_process_group(info.backend)
    return info


def _device(use_gpu: bool, info: DistInfo):
    import torch

    return torch.device("cuda", info.local_rank) if use_gpu else torch.device("cpu")


def barrier(info: DistInfo, use_gpu: bool) -> None:
    if info.is_dist:
        import torch.distributed as dist

        if use_gpu:
            dist.barrier(device_ids=[info.local_rank])
        else:
            dist.barrier()


def all_gather_ints(info: DistInfo, values: list[int], use_gpu: bool) -> list[list[int]]:
    if not info.is_dist:
        return [list(values)]
    import torch
    import torch.distributed as dist

    t = torch.tensor(values, dtype=torch.int64, device=_device(use_gpu, info))
    out = [torch.zeros_like(t) for _ in range(info.world)]
    dist.all_gather(out, t)
    return [o.cpu().tolist() for o in out]


def reduce_max(info: DistInfo, values: list[float], use_gpu: bool) -> list[float]:
    if not info.is_dist:
        return list(values)
    import torch
    import torch.distributed as dist

    t = torch.tensor(values, dtype=torch.float64, device=_device(use_gpu, info))
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return t.cpu().tolist()


def reduce_sum(info: DistInfo, values: list[float], use_gpu: bool) -> list[float]:
    if not info.is_dist:
        return list(values)
    import torch
    import torch.distributed as dist

    t = torch.tensor(values, dtype=torch.float64, device=_device(use_gpu, info))
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return t.cpu().tolist()


def finish(info: DistInfo) -> None:
    if info.is_dist:
        import torch.distributed as dist

        dist.destroy_process_group()

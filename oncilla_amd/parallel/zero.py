"""Data parallel training with a sharded optimizer whose state is offloaded.

One process per MI355X under torch.distributed (RCCL, or gloo on CPU). The
model's parameters are re-pointed into one flat fp32 buffer per rank. Each step:

  1. the flat gradient is reduce-scattered (averaged), so rank r holds the
     gradient of its 1/N shard of the parameters (ZeRO stage 1);
  2. rank r updates its shard with models.OffloadedAdam / OffloadedAdamW, whose
     state lives in disaggregated memory (peer HBM over xGMI or the host tier)
     and, on a GPU, is updated in place by the fused remote-Adam kernel;
  3. the updated shards are all-gathered back into every rank's flat buffer.

So per GPU the optimizer takes neither the full state (as plain DP does) nor a
1/N slice of HBM (as ZeRO does): it takes none, only the remote half's owners
do. Collectives are bucket-free here: one reduce-scatter and one all-gather of
the whole flat buffer per step, the large transfers xGMI rings handle best.
"""
from __future__ import annotations

from typing import Iterable

from .. import api


def flatten_params(params: Iterable, device=None):
    """Move every parameter into one contiguous fp32 buffer (params become views of
    it) and return (flat, [(param, offset, numel)])."""
    import torch

    params = [p for p in params if p.requires_grad]
    bad = sorted({str(p.dtype) for p in params if p.dtype != torch.float32})
    if bad:
        # re-pointing p.data at an fp32 buffer would silently change the model's dtype
        raise TypeError(f"flatten_params takes float32 parameters only (got {', '.join(bad)})")
    total = sum(p.numel() for p in params)
    device = device or params[0].device
    flat = torch.empty(total, dtype=torch.float32, device=device)
    layout, off = [], 0
    for p in params:
        n = p.numel()
        flat[off:off + n].copy_(p.data.reshape(-1))
        p.data = flat[off:off + n].view_as(p)
        layout.append((p, off, n))
        off += n
    return flat, layout


class ShardedOffloadedAdam:
    def __init__(self, params: Iterable, client: api.Client, group=None, adamw: bool = False, **adam_kw):
        import torch
        import torch.distributed as dist

        from ..models.optim_offload import OffloadedAdam, OffloadedAdamW

        self.dist = dist
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.flat, self.layout = flatten_params(params)
        self.total = self.flat.numel()
        # pad to a multiple of 4 * world elements so shards are equal and 16-byte aligned
        q = 4 * self.world
        self.padded = (self.total + q - 1) // q * q
        if self.padded != self.total:
            grown = torch.zeros(self.padded, dtype=self.flat.dtype, device=self.flat.device)
            grown[:self.total].copy_(self.flat)
            for p, off, n in self.layout:
                p.data = grown[off:off + n].view_as(p)
            self.flat = grown
        self.shard_n = self.padded // self.world
        lo = self.rank * self.shard_n
        self.shard = torch.nn.Parameter(self.flat[lo:lo + self.shard_n], requires_grad=True)
        self.flat_grad = torch.zeros_like(self.flat)
        cls = OffloadedAdamW if adamw else OffloadedAdam
        self.opt = cls([self.shard], client, **adam_kw)
        self.backend = dist.get_backend(group)

    def _gather_grads(self) -> None:
        for p, off, n in self.layout:
            if p.grad is None:
                self.flat_grad[off:off + n].zero_()
            else:
                self.flat_grad[off:off + n].copy_(p.grad.reshape(-1))

    def step(self) -> None:
        import torch

        dist = self.dist
        self._gather_grads()
        lo = self.rank * self.shard_n
        if self.backend == "gloo":  # no reduce_scatter on gloo: all-reduce (on the host), keep the shard
            fg = self.flat_grad.cpu()
            dist.all_reduce(fg, group=self.group)
            g = (fg[lo:lo + self.shard_n] / self.world).to(self.flat.device)
        else:
            g = torch.empty(self.shard_n, dtype=self.flat.dtype, device=self.flat.device)
            dist.reduce_scatter_tensor(g, self.flat_grad, op=dist.ReduceOp.AVG, group=self.group)
        self.shard.grad = g.contiguous()
        self.opt.step()
        shard = self.flat[lo:lo + self.shard_n]
        if self.backend == "gloo":
            mine = shard.cpu()
            parts = [torch.empty_like(mine) for _ in range(self.world)]
            dist.all_gather(parts, mine, group=self.group)
            self.flat.copy_(torch.cat(parts).to(self.flat.device))
        else:
            dist.all_gather_into_tensor(self.flat, shard.clone(), group=self.group)

    def zero_grad(self) -> None:
        for p, _, _ in self.layout:
            p.grad = None

    def close(self) -> None:
        self.opt.close()

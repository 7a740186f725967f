"""Paged KV-cache offload onto disaggregated memory (a serving workload).

LLM serving keeps the KV cache in fixed-size blocks on the GPU. When memory runs
short, blocks of idle sequences are swapped out to a larger pool and swapped back
in before their next step. The usual implementation issues one memcpy per block.
Here the GPU cache is the *local half* of one oncilla remote pair, and the
offload pool is its *remote half*. The pool can be HBM striped over the node's
other MI355X (xGMI), the pinned host tier, or another node. A whole swap list
becomes ONE batched one-sided launch (ocm_copy_onesided_batch), with runs of
consecutive blocks coalesced into single ops.

Streams: swap_out waits for work already queued on torch's current stream (the
kernels that wrote the cache). After an async swap_in, that stream waits for the
copies, so later attention kernels see the blocks without a host sync.
"""
from __future__ import annotations

import math
from typing import Iterable, Sequence

import numpy as np

from .. import api


def coalesce_array(pairs) -> "np.ndarray":
    """(k, 2) [src, dst] block pairs -> (r, 3) [src, dst, count] runs where both sides are consecutive."""
    a = np.asarray(pairs, dtype=np.int64).reshape(-1, 2)
    if a.shape[0] == 0:
        return np.zeros((0, 3), dtype=np.int64)
    a = a[np.argsort(a[:, 0], kind="stable")]
    brk = np.ones(a.shape[0], dtype=bool)
    brk[1:] = (np.diff(a[:, 0]) != 1) | (np.diff(a[:, 1]) != 1)
    starts = np.flatnonzero(brk)
    counts = np.diff(np.append(starts, a.shape[0]))
    return np.stack([a[starts, 0], a[starts, 1], counts], axis=1)


def coalesce(pairs: Iterable[tuple[int, int]]) -> list[tuple[int, int, int]]:
    """[(src, dst)] block pairs -> [(src, dst, count)] runs where both sides are consecutive."""
    return [tuple(int(v) for v in r) for r in coalesce_array(list(pairs))]


class PagedKVOffload:
    """GPU KV-cache blocks (local half) + an offload pool of blocks (remote half)."""

    def __init__(self, client: api.Client, num_gpu_blocks: int, num_pool_blocks: int, block_shape: Sequence[int],
                 dtype=None, kind: int = api.OCM_REMOTE_GPU, flags: int = api.OCM_ALLOC_STRIPE, stripe_unit: int = 0,
                 remote_rank: int = -1):
        import torch

        self.dtype = dtype or torch.float16
        self.block_shape = tuple(block_shape)
        elem = torch.empty((), dtype=self.dtype).element_size()
        self.block_bytes = int(math.prod(self.block_shape)) * elem
        self.num_gpu_blocks = num_gpu_blocks
        self.num_pool_blocks = num_pool_blocks
        self.alloc = client.alloc(kind, local_bytes=num_gpu_blocks * self.block_bytes,
                                  remote_bytes=num_pool_blocks * self.block_bytes, remote_rank=remote_rank,
                                  flags=flags, stripe_unit=stripe_unit)
        # The cache the model reads and writes: a zero-copy view of the local half.
        self.gpu_cache = self.alloc.local_tensor(self.dtype)[: num_gpu_blocks * self.block_bytes // elem].view(
            num_gpu_blocks, *self.block_shape)

    def _ops(self, pairs, put: bool) -> api.BatchOps:
        runs = coalesce_array(pairs if isinstance(pairs, np.ndarray) else list(pairs))
        g, p = (runs[:, 0], runs[:, 1]) if put else (runs[:, 1], runs[:, 0])  # (gpu block, pool block)
        n = runs[:, 2]
        if len(n) and ((g < 0).any() or (g + n > self.num_gpu_blocks).any() or (p < 0).any()
                       or (p + n > self.num_pool_blocks).any()):
            raise IndexError("block run out of range")
        bb = self.block_bytes
        ops = np.stack([np.full_like(n, 1 if put else 0), g * bb, p * bb, n * bb], axis=1)
        return api.batch_ops(ops)

    def swap_out(self, gpu_to_pool: Iterable[tuple[int, int]], async_: bool = True) -> int:
        """Copy GPU blocks to pool blocks. Returns the number of batched ops issued."""
        ops = self._ops(gpu_to_pool, put=True)
        self.alloc.stream_wait()  # after the kernels that produced the blocks
        self.alloc.batch(ops, async_=async_)
        if async_:
            self.alloc.stream_signal()  # and before anything that overwrites them
        return ops.n

    def swap_in(self, pool_to_gpu: Iterable[tuple[int, int]], async_: bool = True) -> int:
        """Copy pool blocks into GPU blocks; torch's current stream waits for them."""
        ops = self._ops(pool_to_gpu, put=False)
        self.alloc.stream_wait()  # do not overwrite blocks still being read
        self.alloc.batch(ops, async_=async_)
        if async_:
            self.alloc.stream_signal()
        return ops.n

    def wait(self) -> None:
        self.alloc.wait()

    def close(self) -> None:
        self.alloc.free()

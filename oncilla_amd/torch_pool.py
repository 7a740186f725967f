"""PyTorch tensors in disaggregated memory.

`RemoteMemPool` is a `torch.cuda.MemPool` whose backing allocator is libocm
(`ocm_torch_alloc` / `ocm_torch_free`, a `CUDAPluggableAllocator`). Each block
that torch's caching allocator requests becomes the remote half of an oncilla
pair with no local half, placed in another daemon's HBM (reached over xGMI) or
its pinned host tier. Kernels then address it in place. Tensors created inside
`with pool:` live there. torch caches and splits the blocks as it does for
device memory, and hands a block back only when it releases it.

    with api.Client(daemon_rank=0, gpu=0) as c:
        pool = RemoteMemPool(c)                      # rank0 places; or remote_rank=3
        with pool:
            kv = torch.empty(n, device="cuda")       # lives in a peer GPU's HBM
        out = attn(q, kv)                            # read over xGMI, no copy

The pool serves the client's device only, and one pool configuration is active
per process (the placement is a library setting). A tensor needs contiguous
addresses, so blocks are never striped. `use_on_oom` is passed to torch (retry
an out-of-memory allocation in this pool); it is not exercised by the tests:
torch's per-process memory cap, the one way to force an OOM cheaply, also
bounds that retry.

Beyond the reference: it had no framework integration. The
closest reference path is OCM_REMOTE_* memory used through ocm_copy
(src/lib.c:501-723).
"""
from __future__ import annotations

import ctypes
from typing import Optional

from . import api
from .utils.paths import lib_path


_ALLOCATOR = None


def _allocator():
    """The pluggable allocator, created once and kept for the life of the process:
    every MemPool built on it calls back into it until torch has released the
    pool's last block, which can be after the pool object is gone."""
    global _ALLOCATOR
    if _ALLOCATOR is None:
        import torch

        # the same file the ctypes binding loaded: one library, one state
        _ALLOCATOR = torch.cuda.memory.CUDAPluggableAllocator(lib_path(), "ocm_torch_alloc", "ocm_torch_free")
    return _ALLOCATOR


class RemoteMemPool:
    def __init__(self, client: api.Client, remote_rank: int = -1, host_tier: bool = False, use_on_oom: bool = False):
        import torch

        if client.device < 0:
            raise ValueError("RemoteMemPool needs a GPU client")
        self.client = client
        self.device = client.device
        flags = api.OCM_ALLOC_HOST_TIER if host_tier else 0
        client.lib.ocm_x_torch_pool_config(int(remote_rank), flags)
        self.pool = torch.cuda.MemPool(_allocator().allocator(), use_on_oom=use_on_oom)
        self._ctx = None

    def __enter__(self) -> "RemoteMemPool":
        import torch

        self._ctx = torch.cuda.use_mem_pool(self.pool, device=self.device)
        self._ctx.__enter__()
        return self

    def __exit__(self, *exc) -> None:
        ctx, self._ctx = self._ctx, None
        ctx.__exit__(*exc)

    @staticmethod
    def stats() -> dict:
        """Blocks libocm currently holds for torch, and their bytes."""
        out = (ctypes.c_uint64 * 2)()
        api.load().ocm_x_torch_pool_stats(out)
        return {"blocks": int(out[0]), "bytes": int(out[1])}

"""Adam with its moments in disaggregated memory (a training workload).

Adam keeps two fp32 moments per parameter: 8 bytes per parameter on top of the
weights, which is what runs a large model out of HBM first. Here the moments live
in the *remote half* of oncilla allocations: HBM striped over the node's other
MI355X (xGMI), the pinned host tier (PCIe), or another node. The GPU holds only
two staging slots of `chunk_elems` moments each.

A step walks the flat parameter space in chunks. Chunk k uses slot k % 2, and
each slot is its own allocation, so it has its own copy lane and event:

    slot X = allocs[k % 2]
    torch stream waits for X's lane (the get of chunk k)       X.stream_signal()
    Adam update of chunk k on the torch stream (views of X)
    X's lane waits for that update                              X.stream_wait()
    put chunk k back; get chunk k + 2 into the same slot        async, in order on X's lane

So the get of chunk k + 1 (slot k + 1 % 2, other lane) overlaps the update of chunk
k, and the write-back of chunk k overlaps the update of chunk k + 1. Nothing waits
on the host inside a step.

mode="fused" (default on a GPU) skips the staging altogether: one gfx950 kernel
per parameter (ocm_x_adam, csrc/src/kernels/optim.hip) reads p and g from local
HBM and exp_avg / exp_avg_sq straight from the remote half (peer HBM over xGMI or
the pinned host tier), updates in registers and writes everything back: one pass,
no copies, no extra local HBM traffic. bfloat16 parameters keep fp32 master
weights next to the moments in remote memory (mixed precision: 4 bytes per
parameter stay local, bf16 p and g; 12 go remote). mode="staged" is the path above (CPU
processes, and state on another node, which a kernel cannot address).

The update is torch.optim.Adam's (L2 weight decay, bias correction; reference
behaviour: torch/optim/adam.py single-tensor path), so results match it to
float32 rounding (tests/test_optim_offload.py). The reference runtime has no
training workloads; this is a use of the API beyond it.
"""
from __future__ import annotations

import math
from typing import Iterable

from .. import api


class OffloadedAdam:
    """Adam (or AdamW with decoupled=True) with its state in disaggregated memory; see the module docstring."""

    def __init__(self, params: Iterable, client: api.Client, lr: float = 1e-3, betas=(0.9, 0.999),
                 eps: float = 1e-8, weight_decay: float = 0.0, chunk_elems: int = 16 << 20, flags: int = 0,
                 mode: str = "auto", stripe_unit: int = 0, decoupled: bool = False):
        import torch

        self.params = [p for p in params if p.requires_grad]
        if not self.params:
            raise ValueError("no parameters to optimize")
        self.bf16 = all(p.dtype == torch.bfloat16 for p in self.params)
        for p in self.params:
            if p.dtype not in (torch.float32, torch.bfloat16) or not p.is_contiguous():
                raise ValueError("OffloadedAdam takes contiguous float32 or bfloat16 parameters")
        if not self.bf16 and any(p.dtype != torch.float32 for p in self.params):
            raise ValueError("mixed float32 / bfloat16 parameter lists are not supported")
        self.lr, self.betas, self.eps, self.weight_decay = lr, betas, eps, weight_decay
        self.decoupled = decoupled  # AdamW (torch.optim.AdamW): decay the weights, not the gradient
        self.t = 0
        self.total = sum(p.numel() for p in self.params)
        self.C = max(1, min(int(chunk_elems), self.total))
        self.nchunks = (self.total + self.C - 1) // self.C
        self.slot_bytes = 8 * self.C  # [m (C floats) | v (C floats)]
        on_gpu = client.device >= 0
        kind = api.OCM_REMOTE_GPU if on_gpu else api.OCM_REMOTE_RDMA
        self.mode = ("fused" if on_gpu else "staged") if mode == "auto" else mode
        if self.mode not in ("fused", "staged"):
            raise ValueError(f"mode {mode!r}")
        if self.bf16 and self.mode == "staged":
            # the staged path has no fp32 master weights: small updates would round away in bf16
            raise ValueError("bfloat16 parameters need mode='fused' on a GPU client (fp32 master weights "
                             "in remote memory)")
        if self.mode == "fused":
            if not on_gpu:
                raise ValueError("mode='fused' needs a GPU client")
            self._init_fused(client, kind, flags, stripe_unit)
            return
        self.allocs = []
        for parity in range(min(2, self.nchunks)):
            n_mine = (self.nchunks - parity + 1) // 2
            self.allocs.append(client.alloc(kind, local_bytes=self.slot_bytes, remote_bytes=n_mine * self.slot_bytes,
                                            flags=flags, stripe_unit=stripe_unit))
        self.slots = [a.local_tensor(torch.float32) for a in self.allocs]
        # chunk k -> [(param, lo, hi, offset in chunk)]
        self.segments = []
        bounds, start = [], 0
        for p in self.params:
            bounds.append((p, start, start + p.numel()))
            start += p.numel()
        for k in range(self.nchunks):
            c0, c1 = k * self.C, min((k + 1) * self.C, self.total)
            segs = [(p, max(c0, b0) - b0, min(c1, b1) - b0, max(c0, b0) - c0) for p, b0, b1 in bounds
                    if b0 < c1 and b1 > c0]
            self.segments.append(segs)
        # zero moments in the remote halves
        for s in self.slots:
            s.zero_()
        if on_gpu:
            torch.cuda.synchronize(client.device)
        for k in range(self.nchunks):
            self.allocs[k % 2].put(0, (k // 2) * self.slot_bytes, self.chunk_bytes(k))

    # ---- fused mode: state addressed in place by the update kernel ----
    _PAD = 64  # elements: every parameter's state starts 256-byte aligned

    def _init_fused(self, client, kind, flags, stripe_unit) -> None:
        import torch

        self.starts, pos = [], 0
        for p in self.params:
            self.starts.append(pos)
            pos += (p.numel() + self._PAD - 1) // self._PAD * self._PAD
        self.padded = pos
        # [exp_avg | exp_avg_sq] (padded), and for bf16 parameters [.. | fp32 master weights]
        self.arrays = 3 if self.bf16 else 2
        remote = 4 * self.arrays * self.padded
        self.stage = min(remote, 64 << 20)
        self.allocs = [client.alloc(kind, local_bytes=self.stage, remote_bytes=remote, flags=flags,
                                    stripe_unit=stripe_unit)]
        a = self.allocs[0]
        a.local_tensor(torch.uint8).zero_()
        torch.cuda.current_stream(client.device).synchronize()
        for off in range(0, remote, self.stage):
            a.put(0, off, min(self.stage, remote - off))
        if self.bf16:
            # master weights start as the fp32 value of the bf16 parameters
            buf = a.local_tensor(torch.float32)
            step = self.stage // 4
            for p, start in zip(self.params, self.starts):
                flat = p.data.view(-1)
                for e0 in range(0, p.numel(), step):
                    e1 = min(p.numel(), e0 + step)
                    buf[:e1 - e0].copy_(flat[e0:e1].float())
                    torch.cuda.current_stream(client.device).synchronize()  # the copy, before the put reads buf
                    a.put(0, 4 * (2 * self.padded + start + e0), 4 * (e1 - e0))

    def _step_fused(self) -> None:
        b1, b2 = self.betas
        hp = (b1, b2, self.eps, self.weight_decay, self.lr / (1 - b1 ** self.t), 1 / math.sqrt(1 - b2 ** self.t),
              (1 - self.lr * self.weight_decay) if self.decoupled else math.nan)  # NaN: L2 Adam
        ps, gs, mo, vo, wo = [], [], [], [], []
        for p, start in zip(self.params, self.starts):
            if p.grad is None:
                continue
            ps.append(p.data)
            gs.append(p.grad if p.grad.is_contiguous() else p.grad.contiguous())
            mo.append(4 * start)
            vo.append(4 * (self.padded + start))
            wo.append(4 * (2 * self.padded + start))
        # every parameter in ceil(n / 32) launches (descriptors in the kernel arguments)
        self.allocs[0].adam_multi(ps, gs, mo, vo, hp, w_offs=wo if self.bf16 else None)

    def chunk_bytes(self, k: int) -> int:
        """Bytes of chunk k's record: its m half in full, then v up to the chunk's length."""
        n = min(self.C, self.total - k * self.C)
        return 4 * self.C + 4 * n

    def _get(self, k: int) -> None:
        self.allocs[k % 2].get(0, (k // 2) * self.slot_bytes, self.chunk_bytes(k), async_=True)

    def _put(self, k: int) -> None:
        self.allocs[k % 2].put(0, (k // 2) * self.slot_bytes, self.chunk_bytes(k), async_=True)

    def _update(self, k: int) -> None:
        b1, b2 = self.betas
        bc1 = 1 - b1 ** self.t
        bc2 = 1 - b2 ** self.t
        step_size = self.lr / bc1
        slot = self.slots[k % 2]
        for p, lo, hi, off in self.segments[k]:
            if p.grad is None:
                continue
            n = hi - lo
            pv = p.data.view(-1)[lo:hi]
            g = p.grad.view(-1)[lo:hi]
            if self.decoupled:
                pv.mul_(1 - self.lr * self.weight_decay)
            elif self.weight_decay:
                g = g.add(pv, alpha=self.weight_decay)
            m = slot[off:off + n]
            v = slot[self.C + off:self.C + off + n]
            m.mul_(b1).add_(g, alpha=1 - b1)
            v.mul_(b2).addcmul_(g, g, value=1 - b2)
            denom = (v.sqrt() / math.sqrt(bc2)).add_(self.eps)
            pv.addcdiv_(m, denom, value=-step_size)

    def step(self) -> None:
        """One Adam step over every parameter; queued on torch's current stream (GPU) without a host wait."""
        self.t += 1
        if self.mode == "fused":
            self._step_fused()
            return
        # Prefetch chunks 0 and 1. Each slot's lane already orders these gets after
        # the previous step's write-back of that slot, which waited for its update;
        # nothing here waits for backward, so the prefetch can overlap it.
        for k in range(min(2, self.nchunks)):
            self._get(k)
        for k in range(self.nchunks):
            x = self.allocs[k % 2]
            x.stream_signal()   # torch waits for chunk k's moments
            self._update(k)
            x.stream_wait()     # the write-back waits for the update
            self._put(k)
            if k + 2 < self.nchunks:
                self._get(k + 2)

    def zero_grad(self, set_to_none: bool = True) -> None:
        for p in self.params:
            if set_to_none:
                p.grad = None
            elif p.grad is not None:
                p.grad.zero_()

    def synchronize(self) -> None:
        """Wait on the host for every queued write-back (fused mode: for the update kernels)."""
        if self.mode == "fused":
            import torch

            # the update kernels run on torch's current stream (the copy service's
            # persistent kernel is on a stream of its own and is not waited for)
            torch.cuda.current_stream(self.params[0].device).synchronize()
        for a in self.allocs:
            a.wait()

    def _read_fused(self, base: int, n: int):
        import torch

        a, t = self.allocs[0], torch.empty(n, dtype=torch.float32)
        for e0 in range(0, n, self.stage // 4):
            e1 = min(n, e0 + self.stage // 4)
            a.get(0, base + 4 * e0, 4 * (e1 - e0))
            t[e0:e1] = a.local_tensor(torch.float32)[:e1 - e0].cpu()
        return t

    def master(self, param_index: int):
        """fp32 master weights of a bfloat16 parameter (fused mode), gathered from remote memory."""
        if not self.bf16:
            raise ValueError("master weights exist for bfloat16 parameters only")
        self.synchronize()
        p = self.params[param_index]
        return self._read_fused(4 * (2 * self.padded + self.starts[param_index]), p.numel()).view(p.shape)

    def moments(self, param_index: int):
        """(exp_avg, exp_avg_sq) of one parameter, gathered from remote memory (tests, checkpoints)."""
        import torch

        self.synchronize()
        p = self.params[param_index]
        if self.mode == "fused":
            n, s0 = p.numel(), self.starts[param_index]
            return (self._read_fused(4 * s0, n).view(p.shape), self._read_fused(4 * (self.padded + s0), n).view(p.shape))
        start = sum(q.numel() for q in self.params[:param_index])
        m = torch.empty(p.numel(), dtype=torch.float32)
        v = torch.empty(p.numel(), dtype=torch.float32)
        for k in range(start // self.C, (start + p.numel() - 1) // self.C + 1):
            self.allocs[k % 2].get(0, (k // 2) * self.slot_bytes, self.chunk_bytes(k))
            slot = self.slots[k % 2].cpu()
            for q, lo, hi, off in self.segments[k]:
                if q is p:
                    m[lo:hi] = slot[off:off + hi - lo]
                    v[lo:hi] = slot[self.C + off:self.C + off + hi - lo]
        return m.view_as(p), v.view_as(p)

    def close(self) -> None:
        self.synchronize()
        for a in self.allocs:
            a.free()
        self.allocs = []


class OffloadedAdamW(OffloadedAdam):
    """torch.optim.AdamW semantics (decoupled weight decay, default 1e-2) with offloaded state."""

    def __init__(self, params, client, lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8,
                 weight_decay: float = 1e-2, **kw):
        super().__init__(params, client, lr=lr, betas=betas, eps=eps, weight_decay=weight_decay, decoupled=True, **kw)

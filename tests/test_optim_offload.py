"""OffloadedAdam (oncilla_amd.models.OffloadedAdam): Adam moments in the remote
half of oncilla allocations, streamed through two staging slots per step; the
parameters and moments must match torch.optim.Adam (fp32 oracle)."""
import pytest
import torch

from oncilla_amd import api
from oncilla_amd.models import OffloadedAdam


def _model(device, seed=0):
    g = torch.Generator().manual_seed(seed)
    shapes = [(37, 11), (5,), (64, 33), (1,), (300,)]  # 407 + 5 + 2112 + 1 + 300 elements
    return [torch.randn(s, generator=g).to(device).requires_grad_() for s in shapes]


def _grads(params, step, device):
    g = torch.Generator().manual_seed(100 + step)
    for p in params:
        p.grad = torch.randn(p.shape, generator=g).to(device)


def _run(client, device, chunk, weight_decay, steps=4):
    ref = _model(device)
    mine = [p.detach().clone().requires_grad_() for p in ref]
    opt_ref = torch.optim.Adam(ref, lr=1e-2, betas=(0.8, 0.95), eps=1e-6, weight_decay=weight_decay)
    opt = OffloadedAdam(mine, client, lr=1e-2, betas=(0.8, 0.95), eps=1e-6, weight_decay=weight_decay,
                        chunk_elems=chunk)
    try:
        for s in range(steps):
            _grads(ref, s, device)
            _grads(mine, s, device)
            opt_ref.step()
            opt.step()
            if s == 1:  # parameters agree mid-run without an explicit host wait (stream order)
                for a, b in zip(ref, mine):
                    torch.testing.assert_close(b.detach().cpu(), a.detach().cpu(), rtol=1e-5, atol=1e-6)
        opt.synchronize()
        for i, (a, b) in enumerate(zip(ref, mine)):
            torch.testing.assert_close(b.detach().cpu(), a.detach().cpu(), rtol=1e-5, atol=1e-6)
            m, v = opt.moments(i)
            st = opt_ref.state[a]
            torch.testing.assert_close(m, st["exp_avg"].cpu(), rtol=1e-5, atol=1e-7)
            torch.testing.assert_close(v, st["exp_avg_sq"].cpu(), rtol=1e-5, atol=1e-8)
        return opt.nchunks
    finally:
        opt.close()


@pytest.mark.parametrize("chunk,wd", [(500, 0.0), (1 << 20, 0.01), (97, 0.0)])
def test_offloaded_adam_matches_torch_cpu(mesh_factory, chunk, wd, monkeypatch):
    monkeypatch.setenv("OCM_NO_GPU", "1")
    m = mesh_factory(2)
    with api.Client(daemon_rank=0, ns=m.ns) as c:
        n = _run(c, "cpu", chunk, wd)
        assert n == (2825 + chunk - 1) // chunk  # chunks span parameter boundaries


@pytest.mark.gpu
@pytest.mark.parametrize("chunk", [500, 4096])
def test_offloaded_adam_matches_torch_gpu(mesh_factory, chunk):
    m = mesh_factory(2, gpus=[0, 0])
    with api.Client(daemon_rank=0, gpu=0, ns=m.ns) as c:
        n = _run(c, "cuda:0", chunk, 0.01, steps=5)
        assert n >= 1

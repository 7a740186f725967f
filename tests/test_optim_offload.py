"""OffloadedAdam (oncilla_amd.models.OffloadedAdam): Adam moments in the remote
half of oncilla allocations, streamed through two staging slots per step; the
parameters and moments must match torch.optim.Adam (fp32 oracle)."""
import pytest
import torch

from oncilla_amd import api
from oncilla_amd.models import OffloadedAdam, OffloadedAdamW


def _model(device, seed=0):
    g = torch.Generator().manual_seed(seed)
    shapes = [(37, 11), (5,), (64, 33), (1,), (300,)]  # 407 + 5 + 2112 + 1 + 300 elements
    return [torch.randn(s, generator=g).to(device).requires_grad_() for s in shapes]


def _grads(params, step, device):
    g = torch.Generator().manual_seed(100 + step)
    for p in params:
        p.grad = torch.randn(p.shape, generator=g).to(device=device, dtype=p.dtype)


def _run(client, device, chunk, weight_decay, steps=4, adamw=False, **kw):
    ref = _model(device)
    mine = [p.detach().clone().requires_grad_() for p in ref]
    ref_cls, cls = (torch.optim.AdamW, OffloadedAdamW) if adamw else (torch.optim.Adam, OffloadedAdam)
    opt_ref = ref_cls(ref, lr=1e-2, betas=(0.8, 0.95), eps=1e-6, weight_decay=weight_decay)
    opt = cls(mine, client, lr=1e-2, betas=(0.8, 0.95), eps=1e-6, weight_decay=weight_decay, chunk_elems=chunk, **kw)
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
            torch.testing.assert_close(v, st["exp_avg_sq"].cpu(), rtol=1e-4, atol=1e-6)
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


def test_offloaded_adamw_matches_torch_cpu(mesh_factory, monkeypatch):
    monkeypatch.setenv("OCM_NO_GPU", "1")
    m = mesh_factory(2)
    with api.Client(daemon_rank=0, ns=m.ns) as c:
        _run(c, "cpu", 700, 0.1, adamw=True)


@pytest.mark.gpu
@pytest.mark.parametrize("mode,chunk,adamw", [("staged", 500, False), ("staged", 4096, False), ("fused", 0, False),
                                              ("fused", 0, True), ("staged", 700, True)])
def test_offloaded_adam_matches_torch_gpu(mesh_factory, mode, chunk, adamw):
    m = mesh_factory(2, gpus=[0, 0])
    with api.Client(daemon_rank=0, gpu=0, ns=m.ns) as c:
        n = _run(c, "cuda:0", chunk or 1 << 20, 0.05 if adamw else 0.01, steps=5, mode=mode, adamw=adamw)
        assert n >= 1


@pytest.mark.gpu
@pytest.mark.parametrize("flags", [api.OCM_ALLOC_STRIPE, api.OCM_ALLOC_HOST_TIER])
def test_fused_adam_on_striped_and_host_tier_state(mesh_factory, flags):
    """The fused kernel addresses state striped over three owners (4 KiB units,
    so every parameter's moments cross extents) and state in the pinned host tier."""
    m = mesh_factory(4, gpus=[0, 0, 0, 0], policy="stripe")
    with api.Client(daemon_rank=0, gpu=0, ns=m.ns) as c:
        kw = {"stripe_unit": 4096} if flags == api.OCM_ALLOC_STRIPE else {}
        ref = _model("cuda:0", seed=3)
        mine = [p.detach().clone().requires_grad_() for p in ref]
        opt_ref = torch.optim.Adam(ref, lr=5e-3, weight_decay=0.1)
        opt = OffloadedAdam(mine, c, lr=5e-3, weight_decay=0.1, mode="fused", flags=flags, **kw)
        try:
            ext = opt.allocs[0].remote_info()["extents"]
            if flags == api.OCM_ALLOC_STRIPE:
                assert len(ext) == 3
            else:
                assert {e["tier"] for e in ext} == {1}
            for s in range(3):
                _grads(ref, s, "cuda:0")
                _grads(mine, s, "cuda:0")
                opt_ref.step()
                opt.step()
            opt.synchronize()
            for i, (a, b) in enumerate(zip(ref, mine)):
                torch.testing.assert_close(b.detach().cpu(), a.detach().cpu(), rtol=1e-5, atol=1e-6)
                mm, vv = opt.moments(i)
                torch.testing.assert_close(mm, opt_ref.state[a]["exp_avg"].cpu(), rtol=1e-5, atol=1e-7)
                torch.testing.assert_close(vv, opt_ref.state[a]["exp_avg_sq"].cpu(), rtol=1e-4, atol=1e-6)
        finally:
            opt.close()


@pytest.mark.gpu
@pytest.mark.parametrize("flags", [0, api.OCM_ALLOC_HOST_TIER])
def test_fused_adam_bf16_params_with_remote_fp32_master(mesh_factory, flags):
    """Mixed precision: bf16 parameters and gradients on the GPU, fp32 master
    weights and moments in another daemon's HBM. Oracle: torch.optim.Adam on
    fp32 copies fed the same (bf16-valued) gradients; parameters = master
    rounded to bf16."""
    m = mesh_factory(2, gpus=[0, 0])
    with api.Client(daemon_rank=0, gpu=0, ns=m.ns) as c:
        master_ref = _model("cuda:0", seed=5)
        mine = [p.detach().to(torch.bfloat16).requires_grad_() for p in master_ref]
        # the oracle starts from the same (bf16-representable) values
        with torch.no_grad():
            for r, q in zip(master_ref, mine):
                r.copy_(q.float())
        opt_ref = torch.optim.Adam(master_ref, lr=3e-3, weight_decay=0.01)
        opt = OffloadedAdam(mine, c, lr=3e-3, weight_decay=0.01, flags=flags)
        try:
            assert opt.mode == "fused" and opt.bf16
            if flags:  # the PCIe variant of the kernel (host-tier state)
                assert {e["tier"] for e in opt.allocs[0].remote_info()["extents"]} == {1}
            for s in range(4):
                _grads(mine, s, "cuda:0")
                for q in mine:
                    q.grad = q.grad.to(torch.bfloat16)
                for r, q in zip(master_ref, mine):
                    r.grad = q.grad.float()
                opt_ref.step()
                opt.step()
            opt.synchronize()
            for i, (r, q) in enumerate(zip(master_ref, mine)):
                torch.testing.assert_close(opt.master(i), r.detach().cpu(), rtol=1e-5, atol=1e-6)
                torch.testing.assert_close(q.detach().cpu(), r.detach().to(torch.bfloat16).cpu())
                mm, vv = opt.moments(i)
                torch.testing.assert_close(mm, opt_ref.state[r]["exp_avg"].cpu(), rtol=1e-5, atol=1e-7)
                torch.testing.assert_close(vv, opt_ref.state[r]["exp_avg_sq"].cpu(), rtol=1e-4, atol=1e-6)
        finally:
            opt.close()


@pytest.mark.gpu
@pytest.mark.parametrize("flags", [0, api.OCM_ALLOC_HOST_TIER])
def test_fused_adamw_many_tensors_and_missing_grads(mesh_factory, flags):
    """More than one launch's worth of parameters (32 descriptors per launch),
    large and tiny tensors mixed, some without a gradient (skipped, like torch),
    and AdamW with lr * weight_decay == 1 (decay multiplier 0: the weights are
    fully decayed, which an in-band 0 = 'no AdamW' flag used to turn into L2 Adam)."""
    m = mesh_factory(2, gpus=[0, 0])
    g = torch.Generator().manual_seed(9)
    shapes = [(1 << 16,) if i % 7 == 0 else (int(torch.randint(1, 300, (1,), generator=g)),) for i in range(45)]
    with api.Client(daemon_rank=0, gpu=0, ns=m.ns) as c:
        for lr, wd in ((1e-2, 0.05), (0.5, 2.0)):
            ref = [torch.randn(s, generator=g).to("cuda:0").requires_grad_() for s in shapes]
            mine = [p.detach().clone().requires_grad_() for p in ref]
            opt_ref = torch.optim.AdamW(ref, lr=lr, weight_decay=wd)
            opt = OffloadedAdamW(mine, c, lr=lr, weight_decay=wd, mode="fused", flags=flags)
            try:
                for s in range(3):
                    gg = torch.Generator().manual_seed(200 + s)
                    for i, (a, b) in enumerate(zip(ref, mine)):
                        if i % 5 == 3:
                            a.grad = b.grad = None
                            continue
                        a.grad = torch.randn(a.shape, generator=gg).to("cuda:0")
                        b.grad = a.grad.clone()
                    opt_ref.step()
                    opt.step()
                opt.synchronize()
                for a, b in zip(ref, mine):
                    torch.testing.assert_close(b.detach().cpu(), a.detach().cpu(), rtol=1e-5, atol=1e-6)
            finally:
                opt.close()


@pytest.mark.gpu
def test_fused_adam_rejects_bad_tensor_before_any_launch(mesh_factory):
    """A state range outside the remote half anywhere in the list fails the whole
    call before the first launch: no parameter moves."""
    m = mesh_factory(2, gpus=[0, 0])
    with api.Client(daemon_rank=0, gpu=0, ns=m.ns) as c:
        a = c.alloc(api.OCM_REMOTE_GPU, local_bytes=4096, remote_bytes=64 * 40 * 8)
        ps = [torch.zeros(64, device="cuda:0") for _ in range(40)]
        gs = [torch.ones(64, device="cuda:0") for _ in range(40)]
        mo = [4 * 64 * i for i in range(40)]
        vo = [4 * 64 * (40 + i) for i in range(40)]
        vo[37] = 64 * 40 * 8  # past the end, in the second launch's chunk
        hp = (0.9, 0.999, 1e-8, 0.0, 1e-3, 1.0, float("nan"))
        with pytest.raises(api.OcmError):
            a.adam_multi(ps, gs, mo, vo, hp)
        torch.cuda.synchronize()
        assert all(int(p.count_nonzero()) == 0 for p in ps)
        a.free()


def test_staged_mode_refuses_bf16_after_auto_resolution(mesh_factory, monkeypatch):
    monkeypatch.setenv("OCM_NO_GPU", "1")
    m = mesh_factory(1)
    with api.Client(daemon_rank=0, ns=m.ns) as c:
        p = torch.zeros(16, dtype=torch.bfloat16, requires_grad=True)
        with pytest.raises(ValueError, match="fused"):
            OffloadedAdam([p], c)  # mode='auto' resolves to staged on a CPU client


def test_flatten_params_keeps_dtypes_honest():
    from oncilla_amd.parallel.zero import flatten_params

    with pytest.raises(TypeError):
        flatten_params([torch.zeros(4, dtype=torch.bfloat16, requires_grad=True)])
    p = torch.ones(3, requires_grad=True)
    flat, layout = flatten_params([p])
    assert p.dtype == torch.float32 and flat.numel() == 3 and layout[0][1:] == (0, 3)


@pytest.mark.gpu
@pytest.mark.parametrize("flags", [0, api.OCM_ALLOC_HOST_TIER])
def test_single_tensor_adam_matches_torch(mesh_factory, flags):
    """Allocation.adam (ocm_x_adam, one launch for one tensor) with the moments in
    another daemon's HBM or in the pinned host tier (the PCIe variant of the
    kernel), a length that leaves a 3-element tail, against torch.optim.Adam."""
    import math

    m = mesh_factory(2, gpus=[0, 0])
    n = (1 << 20) + 3
    vec = (n + 3) // 4 * 4
    m_off, v_off = 0, 4 * vec
    rbytes = 8 * vec
    with api.Client(daemon_rank=0, gpu=0, ns=m.ns) as c:
        a = c.alloc(api.OCM_REMOTE_GPU, local_bytes=rbytes, remote_bytes=rbytes, flags=flags)
        try:
            if flags:
                assert {e["tier"] for e in a.remote_info()["extents"]} == {1}
            a.local_tensor(torch.float32).zero_()
            a.put(0, 0, rbytes)
            g0 = torch.Generator().manual_seed(21)
            ref = torch.randn(n, generator=g0).to("cuda:0").requires_grad_()
            mine = ref.detach().clone()
            lr, b1, b2, eps, wd = 2e-3, 0.9, 0.999, 1e-8, 0.05
            opt_ref = torch.optim.Adam([ref], lr=lr, betas=(b1, b2), eps=eps, weight_decay=wd)
            for t in range(1, 4):
                g = torch.randn(n, generator=torch.Generator().manual_seed(100 + t)).to("cuda:0")
                ref.grad = g.clone()
                opt_ref.step()
                a.adam(mine, g, m_off, v_off, (b1, b2, eps, wd, lr / (1 - b1 ** t), 1 / math.sqrt(1 - b2 ** t)))
            torch.cuda.synchronize()
            torch.testing.assert_close(mine.cpu(), ref.detach().cpu(), rtol=1e-5, atol=1e-6)
            a.get(0, 0, rbytes)
            loc = a.local_tensor(torch.float32).cpu()
            torch.testing.assert_close(loc[:n], opt_ref.state[ref]["exp_avg"].cpu(), rtol=1e-5, atol=1e-7)
            torch.testing.assert_close(loc[vec:vec + n], opt_ref.state[ref]["exp_avg_sq"].cpu(), rtol=1e-4, atol=1e-6)
        finally:
            a.free()

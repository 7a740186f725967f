"""ocm_copy_onesided_batch: many one-sided ops (puts and gets mixed) in one call.

On a GPU the whole list runs as ONE gfx950 kernel launch (descriptors in the
kernarg segment up to 48 ops, in a device table above). Without a device
path (CPU app) the ops run one by one. Both are checked against a NumPy model
of the local and remote halves, with random, unaligned, disjoint ranges.
"""
import numpy as np
import pytest
import torch

from oncilla_amd import api


def _disjoint(rng, space, n, max_len):
    """n disjoint [off, off+len) ranges inside [0, space), in random order."""
    lens = rng.integers(1, max_len + 1, size=n)
    slack = space - int(lens.sum())
    assert slack >= 0
    gaps = rng.multinomial(slack, np.ones(n + 1) / (n + 1))[:n]
    order = rng.permutation(n)
    offs = np.empty(n, dtype=np.int64)
    pos = 0
    for k, i in enumerate(order):
        pos += int(gaps[k])
        offs[i] = pos
        pos += int(lens[i])
    return offs, lens


def run_batch_check(a, nbytes, n_ops, max_len, seed, async_=False):
    rng = np.random.default_rng(seed)
    loc = a.local_tensor(torch.uint8)
    dev = loc.device
    init = rng.integers(0, 256, size=nbytes, dtype=np.uint8)
    loc.copy_(torch.from_numpy(init).to(dev))
    if dev.type == "cuda":
        torch.cuda.synchronize()
    a.put(0, 0, nbytes)  # known remote state
    remote = init.copy()
    fresh = rng.integers(0, 256, size=nbytes, dtype=np.uint8)
    loc.copy_(torch.from_numpy(fresh).to(dev))
    if dev.type == "cuda":
        torch.cuda.synchronize()
    local = fresh.copy()
    loffs, lens = _disjoint(rng, nbytes, n_ops, max_len)
    # remote ranges: same lengths, independent placement
    rl = rng.permutation(n_ops)
    space = nbytes - int(lens.sum())
    gaps = rng.multinomial(space, np.ones(n_ops + 1) / (n_ops + 1))[:n_ops]
    roffs = np.empty(n_ops, dtype=np.int64)
    pos = 0
    for k, i in enumerate(rl):
        pos += int(gaps[k])
        roffs[i] = pos
        pos += int(lens[i])
    flags = rng.integers(0, 2, size=n_ops)
    ops = []
    for i in range(n_ops):
        lo, ro, n, f = int(loffs[i]), int(roffs[i]), int(lens[i]), int(flags[i])
        ops.append((f, lo, ro, n))
    # model (disjoint ranges: order-independent)
    new_local, new_remote = local.copy(), remote.copy()
    for f, lo, ro, n in ops:
        if f:
            new_remote[ro:ro + n] = local[lo:lo + n]
        else:
            new_local[lo:lo + n] = remote[ro:ro + n]
    a.batch(ops, async_=async_)
    if async_:
        a.wait()
    got_local = a.local_tensor(torch.uint8).cpu().numpy()
    assert np.array_equal(got_local, new_local), "local half differs from the model"
    a.get(0, 0, nbytes)
    got_remote = a.local_tensor(torch.uint8).cpu().numpy()
    assert np.array_equal(got_remote, new_remote), "remote half differs from the model"


@pytest.fixture
def cpu_app(monkeypatch):
    monkeypatch.setenv("OCM_NO_GPU", "1")


def test_batch_fallback_cpu(mesh_factory, cpu_app):
    m = mesh_factory(3, policy="stripe")
    with api.Client(daemon_rank=0, ns=m.ns) as c:
        n = 1 << 20
        a = c.alloc(api.OCM_REMOTE_RDMA, local_bytes=n, remote_bytes=n, stripe_unit=64 << 10)
        assert len(a.remote_info()["extents"]) == 2
        before = api.counters()
        run_batch_check(a, n, 200, 3000, seed=1)
        after = api.counters()
        assert after["n_batch"] == before["n_batch"] + 1 and after["n_batch_ops"] == before["n_batch_ops"] + 200
        a.batch([])  # empty list is a no-op
        with pytest.raises(api.OcmError):
            a.batch([(1, n - 10, 0, 20)])  # local range out of bounds
        a.free()


@pytest.mark.gpu
@pytest.mark.parametrize("unit,n_ops,max_len,async_", [
    (64 << 10, 1, 70000, False),        # one op spanning stripe units
    (64 << 10, 40, 20000, False),       # inline descriptors
    (4 << 10, 48, 9000, True),          # 4 KiB stripe unit -> 4 KiB tiles, async
    (64 << 10, 1500, 600, False),       # device descriptor table, tiny ops
    (1 << 20, 3000, 2500, True),        # many ops, async
])
def test_batch_kernel_gpu(mesh_factory, unit, n_ops, max_len, async_):
    m = mesh_factory(4, gpus=[0, 0, 0, 0], policy="stripe")
    with api.Client(daemon_rank=0, gpu=0, ns=m.ns) as c:
        n = 16 << 20
        a = c.alloc(api.OCM_REMOTE_GPU, local_bytes=n, remote_bytes=n, stripe_unit=unit)
        assert len(a.remote_info()["extents"]) == 3
        before = api.counters()
        run_batch_check(a, n, n_ops, max_len, seed=n_ops + unit, async_=async_)
        assert api.counters()["n_batch_ops"] == before["n_batch_ops"] + n_ops
        a.free()


@pytest.mark.gpu
@pytest.mark.parametrize("n_ops,max_len,async_", [(300, 5000, False), (40, 70000, True), (3000, 2500, True)])
def test_batch_host_tier_gpu(mesh_factory, n_ops, max_len, async_):
    # single daemon: the remote half is the pinned host tier, still one kernel (mapped
    # host memory): the host-tier launch shape with write-through puts
    m = mesh_factory(1, gpus=[0])
    with api.Client(daemon_rank=0, gpu=0, ns=m.ns) as c:
        n = 4 << 20
        a = c.alloc(api.OCM_REMOTE_GPU, local_bytes=n, remote_bytes=n)
        assert a.remote_info()["extents"][0]["tier"] == api.OCM_TIER_HOST
        run_batch_check(a, n, n_ops, max_len, seed=7 + n_ops, async_=async_)
        a.free()


def test_plan_needs_gpu(mesh_factory, cpu_app):
    m = mesh_factory(1)
    with api.Client(daemon_rank=0, ns=m.ns) as c:
        with pytest.raises(api.OcmError):
            c.plan()


@pytest.mark.gpu
def test_plan_graph_replay(mesh_factory):
    # Two pairs, a 3-stage schedule (gather from A, scatter to B, a large-list
    # stage on A) captured once and replayed with fresh data each time.
    m = mesh_factory(4, gpus=[0, 0, 0, 0], policy="stripe")
    with api.Client(daemon_rank=0, gpu=0, ns=m.ns) as c:
        n = 8 << 20
        A = c.alloc(api.OCM_REMOTE_GPU, local_bytes=n, remote_bytes=n, stripe_unit=64 << 10)
        B = c.alloc(api.OCM_REMOTE_GPU, local_bytes=n, remote_bytes=n, stripe_unit=64 << 10)
        rng = np.random.default_rng(11)
        piece = 4096
        slots = n // piece
        gather = [(0, i * piece, int(r) * piece, piece) for i, r in enumerate(rng.choice(slots, 40, replace=False))]
        scatter = [(1, i * piece, int(r) * piece, piece) for i, r in enumerate(rng.choice(slots, 40, replace=False))]
        big = [(1, (100 + i) * piece, int(r) * piece, piece) for i, r in enumerate(rng.choice(slots, 900, replace=False))]
        plan = c.plan().add(A, gather).add(B, scatter).add(A, big)
        for rep in range(3):
            a_rem = rng.integers(0, 256, n, dtype=np.uint8)
            A.local_tensor(torch.uint8).copy_(torch.from_numpy(a_rem).cuda())
            torch.cuda.synchronize()
            A.put(0, 0, n)
            a_loc = rng.integers(0, 256, n, dtype=np.uint8)
            b_loc = rng.integers(0, 256, n, dtype=np.uint8)
            A.local_tensor(torch.uint8).copy_(torch.from_numpy(a_loc).cuda())
            B.local_tensor(torch.uint8).copy_(torch.from_numpy(b_loc).cuda())
            torch.cuda.synchronize()
            B.put(0, 0, n)
            b_rem = b_loc.copy()
            # model
            for _, lo, ro, k in gather:
                a_loc[lo:lo + k] = a_rem[ro:ro + k]
            for _, lo, ro, k in scatter:
                b_rem[ro:ro + k] = b_loc[lo:lo + k]
            for _, lo, ro, k in big:
                a_rem[ro:ro + k] = a_loc[lo:lo + k]
            if rep == 1:
                s = torch.cuda.Stream()
                plan.launch(s)
                s.synchronize()
            else:
                plan.launch()
            assert np.array_equal(A.local_tensor(torch.uint8).cpu().numpy(), a_loc), rep
            A.get(0, 0, n)
            assert np.array_equal(A.local_tensor(torch.uint8).cpu().numpy(), a_rem), rep
            B.get(0, 0, n)
            assert np.array_equal(B.local_tensor(torch.uint8).cpu().numpy(), b_rem), rep
        with pytest.raises(api.OcmError):
            A.free()  # still used by the plan
        plan.close()
        A.free()
        B.free()

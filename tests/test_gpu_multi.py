"""One daemon per PHYSICAL MI355X: the data path over xGMI.

Every other GPU test puts all daemons on device 0 (same-GPU IPC stand-in).
These tests need >= 2 visible GPUs and skip cleanly on the 1-GPU pool; they
are the ones that exercise cross-device hipIpcOpenMemHandle, peer access,
stores into peer HBM and the RCCL control plane between real ranks.

Reference parity: the 2-node one-sided R/W path, test/ocm_test.c:323-425 over
src/rdma.c:240-263 (ib_read / ib_write), with the remote buffer on another GPU
instead of another host.
"""
import pytest
import torch

from oncilla_amd import api

from conftest import gpu_count

NDEV = gpu_count()
pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(NDEV < 2, reason=f"needs >= 2 MI355X (this box has {NDEV})")]


def _roundtrip(a, n, seed, loff=0, roff=0):
    a.fill(seed=seed, offset=loff, nbytes=n)
    a.put(loff, roff, n)
    a.fill(seed=0, offset=loff, nbytes=n)
    a.get(loff, roff, n)
    return a.check(seed=seed, offset=loff, nbytes=n)


def test_remote_pair_owned_by_another_gpu(mesh_factory):
    """App on GPU 0, remote half in rank 1's HBM on GPU 1: IPC import across
    devices, peer access, put/get through the gfx950 kernel over xGMI."""
    m = mesh_factory(2, gpus=[0, 1])
    with api.Client(daemon_rank=0, gpu=0, ns=m.ns) as c:
        n = 256 << 20
        a = c.alloc(api.OCM_REMOTE_GPU, local_bytes=n, remote_bytes=n, remote_rank=1)
        ext = a.remote_info()["extents"]
        assert len(ext) == 1 and ext[0]["owner_rank"] == 1 and ext[0]["owner_gpu"] == 1
        assert ext[0]["tier"] == api.OCM_TIER_GPU
        assert _roundtrip(a, n, seed=3) == 0
        assert _roundtrip(a, (1 << 20) + 12, seed=4, loff=8, roff=4096 + 4) == 0  # unaligned
        # the bytes really live on GPU 1: a torch view on the app's device reads them
        rt = a.remote_tensor(torch.int32)
        assert rt.device.index == 0
        link = api.link_info(0, 1)
        assert link["hops"] >= 1
        st = c.stats(0)  # the daemon's xGMI table reached rank0's placement and the stats
        assert st["xgmi_peers"] >= 1 and st["min_hops"] >= 1
        assert c.stats(1)["gpu_used"] >= n
        a.free()
        assert c.stats(1)["gpu_used"] == 0


def test_stripe_over_every_peer_gpu(mesh_factory):
    """A striped pair over all other GPUs (every xGMI link of GPU 0), verified."""
    m = mesh_factory(NDEV, gpus=list(range(NDEV)), policy="stripe")
    with api.Client(daemon_rank=0, gpu=0, ns=m.ns) as c:
        n = (NDEV - 1) * (64 << 20) + 4096
        a = c.alloc(api.OCM_REMOTE_GPU, local_bytes=n, remote_bytes=n, flags=api.OCM_ALLOC_STRIPE)
        ext = a.remote_info()["extents"]
        assert len(ext) == NDEV - 1
        assert sorted(e["owner_gpu"] for e in ext) == list(range(1, NDEV))
        assert _roundtrip(a, n, seed=11) == 0
        assert _roundtrip(a, 3 << 20, seed=12, loff=4096, roff=(1 << 20) - 256) == 0  # crosses stripe units
        a.free()


@pytest.mark.parametrize("proto", ["15", "47"])
@pytest.mark.parametrize("size", [4096, 65536, 1 << 20, 4 << 20])
def test_copy_service_small_ops_on_peer_hbm(mesh_factory, monkeypatch, size, proto):
    """Blocking small ops ride the resident copy service; on peer HBM its
    stores cross xGMI. Many back-to-back ops, each verified. proto 47 adds
    STRICTWT: the peer-HBM hand-off copies write-through behind its acquire
    instead of releasing with an L2 writeback (profiles/svc_strict_cost_r03.json)."""
    monkeypatch.setenv("OCM_SERVICE_PROTO", proto)
    m = mesh_factory(2, gpus=[0, 1])
    with api.Client(daemon_rank=0, gpu=0, ns=m.ns) as c:
        a = c.alloc(api.OCM_REMOTE_GPU, local_bytes=8 << 20, remote_bytes=8 << 20, remote_rank=1)
        for i in range(16):
            off = (i * 4096 * 3) % ((8 << 20) - size)
            assert _roundtrip(a, size, seed=100 + i, roff=off) == 0, i
        svc = api.service_stats()
        assert svc["ops"] > 0
        a.free()


OWNER_SIZES = [4096, 256 << 10, 4 << 20, 16 << 20, 256 << 20]  # service (<= 4 MiB on peer HBM), then launches


def owner_round_trips(c, owner_rank, size, rounds=3):
    """a kernel on the OWNER's GPU verifies what the app put
    (copy service for small ops, launches above), and writes what the app's next
    get must return, with idle exits of the service in between."""
    import time

    from oncilla_amd.utils.owner_side import OwnerView

    a = c.alloc(api.OCM_REMOTE_GPU, local_bytes=size, remote_bytes=size, remote_rank=owner_rank)
    try:
        with OwnerView(a) as v:
            for r in range(rounds):
                a.fill(seed=500 + r, nbytes=size)
                a.put(0, 0, size)
                assert v.check(seed=500 + r, nbytes=size) == 0, f"owner GPU misses the app's put ({size} B, round {r})"
                v.fill(seed=700 + r, nbytes=size)  # the owner's kernel rewrites the extent
                a.get(0, 0, size)  # a resident service may hold lines of the old bytes: STRICT hand-off
                assert a.check(seed=700 + r, nbytes=size) == 0, f"app get misses the owner's writes ({size} B, round {r})"
                if r == 1:
                    time.sleep(0.002)  # past the service's idle exit: the next op relaunches it
    finally:
        a.free()


@pytest.mark.parametrize("size", OWNER_SIZES)
def test_owner_gpu_sees_app_puts_and_app_gets_see_owner_writes(mesh_factory, size):
    m = mesh_factory(2, gpus=[0, 1])
    with api.Client(daemon_rank=0, gpu=0, ns=m.ns) as c:
        owner_round_trips(c, 1, size)


def test_fused_adam_with_state_in_peer_hbm(mesh_factory):
    """The fused remote-Adam kernel reads and writes the moments in another
    GPU's HBM over xGMI; results match torch.optim.Adam."""
    from oncilla_amd.models import OffloadedAdam

    m = mesh_factory(2, gpus=[0, 1])
    with api.Client(daemon_rank=0, gpu=0, ns=m.ns) as c:
        g = torch.Generator().manual_seed(0)
        ref = [torch.randn(s, generator=g).to("cuda:0").requires_grad_() for s in [(257, 33), (4096,), (3,)]]
        mine = [p.detach().clone().requires_grad_() for p in ref]
        opt_ref = torch.optim.Adam(ref, lr=1e-2, weight_decay=0.01)
        opt = OffloadedAdam(mine, c, lr=1e-2, weight_decay=0.01, mode="fused")
        try:
            assert all(e["owner_gpu"] == 1 for e in opt.allocs[0].remote_info()["extents"])
            for s in range(3):
                gg = torch.Generator().manual_seed(50 + s)
                for a, b in zip(ref, mine):
                    a.grad = torch.randn(a.shape, generator=gg).to("cuda:0")
                    b.grad = a.grad.clone()
                opt_ref.step()
                opt.step()
            opt.synchronize()
            for i, (a, b) in enumerate(zip(ref, mine)):
                torch.testing.assert_close(b.detach().cpu(), a.detach().cpu(), rtol=1e-5, atol=1e-6)
                mm, vv = opt.moments(i)
                torch.testing.assert_close(mm, opt_ref.state[a]["exp_avg"].cpu(), rtol=1e-5, atol=1e-7)
        finally:
            opt.close()


@pytest.mark.parametrize("graph", ["0", "8"])
def test_rccl_control_plane_between_gpus(mesh_factory, graph):
    """--ctrl rccl: the daemons' control records ride ncclAllGather ticks over
    xGMI (one rank per GPU). Leases off, so every allocation takes the full
    REQ_ALLOC -> DO_ALLOC -> reply path through the ticks. graph=8: the ticks
    are queued as replays of captured graphs of 8 (OCM_TICK_GRAPH)."""
    k = min(NDEV, 4)
    m = mesh_factory(k, gpus=list(range(k)), extra_args=["--ctrl", "rccl"],
                     env={"OCM_LEASE_BYTES": "0", "OCM_TICK_GRAPH": graph})
    with api.Client(daemon_rank=0, gpu=0, ns=m.ns) as c:
        for i in range(20):
            a = c.alloc(api.OCM_REMOTE_GPU, local_bytes=1 << 20, remote_bytes=1 << 20, remote_rank=1 + i % (k - 1))
            assert _roundtrip(a, 1 << 20, seed=200 + i) == 0
            a.free()
        assert c.stats(0)["ctrl_ticks"] > 0, m.logs()
        assert "falling back to TCP" not in m.logs()
    if graph != "0":
        assert m.logs().count("ticks per captured graph") == k, m.logs()


def test_host_tier_of_another_gpus_daemon(mesh_factory):
    """Rank 1's pinned host tier (its GPU's NUMA node), mapped by an app on GPU 0."""
    m = mesh_factory(2, gpus=[0, 1])
    with api.Client(daemon_rank=0, gpu=0, ns=m.ns) as c:
        n = 32 << 20
        a = c.alloc(api.OCM_REMOTE_GPU, local_bytes=n, remote_bytes=n, remote_rank=1, flags=api.OCM_ALLOC_HOST_TIER)
        assert a.remote_info()["extents"][0]["tier"] == api.OCM_TIER_HOST
        assert _roundtrip(a, n, seed=31) == 0
        a.free()


def test_bench_on_real_gpus():
    """The driver's scaling launch on EVERY GPU of this box at the driver's config
    (1 GiB max transfer): one rank and one daemon per physical GPU, striped over
    every peer, autotune over xGMI, the per-peer table with link types, the
    self-diagnosis fields (xgmi, peer access / IPC import per rank, control
    transport per rank) and the control-plane extra with RCCL ticks."""
    import json
    import os
    import subprocess
    import sys

    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    k = min(NDEV, 8)
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(k),
                        "--master-addr", "127.0.0.1", "--master-port", "29671", os.path.join(repo, "bench.py"),
                        "--gpus", str(k), "--steps", "1", "--warmup", "1", "--max-bytes", str(1 << 30),
                        "--alloc-samples", "50", "--no-characterize"],
                       capture_output=True, text=True, timeout=900, cwd="/tmp")
    assert r.returncode == 0, r.stderr[-4000:]
    res = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert res["n_gpus"] == k and res["value"] > 0 and res["config"]["remote_tier"] == "hbm", res
    assert res["xgmi"] is True and "fallback" not in res, res
    diag = res["ranks"]
    assert len(diag) == k and all(d["peer_access"] == k - 1 and d["ipc_imports"] >= k - 1 for d in diag), diag
    assert res["config"]["extents_per_pair"] == k - 1
    peers = res["peers_from_rank0"]
    assert sorted(peers) == [str(p) for p in range(1, k)], peers
    for p, row in peers.items():
        assert row["owner_gpu"] == int(p) and row["put_GiBps"] > 0 and row["link"] is not None, row
    cp = res["control_plane"]
    assert cp["tcp"]["alloc_p50_us"] > 0 and cp["rccl"]["ticks_rank0"] > 0, cp
    # the RCCL control plane stands on its own (idle ticks, no TCP wake-ups)
    assert cp["rccl"]["transport_up_all_ranks"] and cp["rccl"]["tcp_wakes_all_ranks"] == 0, cp
    # a clean run - no library warning on any rank (a copy-service
    # fallback, a tick transport leaving for TCP, a refused IPC import ...)
    assert res["service_clean"] is True, res["ranks"]
    warns = [l for l in (r.stdout + r.stderr).splitlines() if "[ocm W" in l or "[ocm E" in l]
    assert not warns, warns[:20]


def test_torch_tensors_in_another_gpus_hbm(mesh_factory):
    """RemoteMemPool with the owner on GPU 1: a matmul on GPU 0 reads its operand
    over xGMI, in place."""
    from oncilla_amd.torch_pool import RemoteMemPool

    m = mesh_factory(2, gpus=[0, 1])
    with api.Client(daemon_rank=0, gpu=0, ns=m.ns) as c:
        pool = RemoteMemPool(c, remote_rank=1)
        with pool:
            w = torch.full((2048, 2048), 0.5, device="cuda:0")
        assert c.stats(1)["gpu_used"] >= 16 << 20
        x = torch.ones((64, 2048), device="cuda:0")
        assert torch.equal(x @ w, torch.full((64, 2048), 1024.0, device="cuda:0"))
        del w, pool

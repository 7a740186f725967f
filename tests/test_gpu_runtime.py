"""The runtime on a real MI355X: daemons owning HBM, IPC import into the app,
put/get through the gfx950 kernel, multi-daemon meshes sharing one GPU, the
graft smoke and the benchmark contract."""
import json
import os
import subprocess
import sys
import time

import pytest
import torch

from oncilla_amd import api

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_native_library_is_the_path(native):
    from oncilla_amd.utils.paths import lib_path

    api.load()
    maps = open(f"/proc/{os.getpid()}/maps").read()
    assert os.path.realpath(lib_path()) in maps


@pytest.mark.parametrize("args", [["1", "4", "8", "2"], ["1", "4", "8", "5"], ["1", "4", "8", "3"], ["2", "8", "8"],
                                  ["3", "4", "8"], ["4", "2", "3", "16"], ["5", "8", "16"]])
def test_ocm_test_single_gpu_daemon(mesh_factory, tool, native, args):
    m = mesh_factory(1, gpus=[0])
    rc, out = tool([f"{native}/ocm_test", *args], env=dict(m.client_env(0), OCM_GPU="0"))
    assert rc == 0, out + m.logs()


def test_remote_hbm_across_processes(mesh_factory):
    # two daemons on the same MI355X: rank1's HBM is "remote" for an app on rank0
    m = mesh_factory(2, gpus=[0, 0])
    with api.Client(daemon_rank=0, gpu=0, ns=m.ns) as c:
        n = 64 << 20
        a = c.alloc(api.OCM_REMOTE_GPU, local_bytes=n, remote_bytes=n)
        info = a.remote_info()
        assert info["extents"][0]["owner_rank"] == 1 and info["extents"][0]["tier"] == api.OCM_TIER_GPU
        a.fill(seed=5)
        a.put(0, 0, n)
        a.fill(seed=0)
        a.get(0, 0, n)
        assert a.check(seed=5) == 0
        st = c.stats(1)
        assert st["gpu_used"] == n and st["gpu"] == 0
        a.free()
        assert c.stats(1)["gpu_used"] == 0


def test_striped_hbm_over_three_owners(mesh_factory):
    m = mesh_factory(4, gpus=[0, 0, 0, 0], policy="stripe")
    with api.Client(daemon_rank=0, gpu=0, ns=m.ns) as c:
        n = (96 << 20) + 4096
        a = c.alloc(api.OCM_REMOTE_GPU, local_bytes=n, remote_bytes=n)
        info = a.remote_info()
        assert len(info["extents"]) == 3 and all(e["tier"] == api.OCM_TIER_GPU for e in info["extents"])
        a.fill(seed=9)
        a.put(0, 0, n)
        a.fill(seed=0)
        a.get(0, 0, n)
        assert a.check(seed=9) == 0
        # async put/get + wait
        a.fill(seed=10)
        a.put(0, 0, n, async_=True)
        a.wait()
        a.fill(seed=0)
        a.get(0, 0, n, async_=True)
        a.wait()
        assert a.check(seed=10) == 0
        a.free()


def test_host_tier_pair_and_copy_in_out(mesh_factory):
    m = mesh_factory(1, gpus=[0])
    with api.Client(daemon_rank=0, gpu=0, ns=m.ns) as c:
        n = 16 << 20
        a = c.alloc(api.OCM_REMOTE_GPU, local_bytes=n, remote_bytes=n)
        assert a.remote_info()["extents"][0]["tier"] == api.OCM_TIER_HOST
        src = torch.randint(0, 256, (n,), dtype=torch.uint8, device="cuda:0")
        dst = torch.zeros_like(src)
        a.copy_in(src.data_ptr())
        a.copy_out(dst.data_ptr())
        torch.cuda.synchronize()
        assert torch.equal(src, dst)
        hsrc = src.cpu()
        hdst = torch.zeros_like(hsrc)
        a.copy_in(hsrc.data_ptr())
        a.copy_out(hdst.data_ptr())
        assert torch.equal(hsrc, hdst)
        a.free()


def test_graft_smoke():
    r = subprocess.run([sys.executable, os.path.join(REPO, "__graft_entry__.py"), "smoke"], capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "smoke OK" in r.stdout


def test_bench_gpu_small():
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--steps", "2", "--warmup", "1", "--max-bytes",
                        str(64 << 20), "--alloc-samples", "50"], capture_output=True, text=True, timeout=600,
                       cwd="/tmp")
    assert r.returncode == 0, r.stderr[-4000:]
    res = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert res["config"]["device"] == "gpu" and res["value"] > 0


def test_bench_two_ranks_sharing_one_gpu():
    """The driver's N>1 launch shape (torch.distributed.run, one ocmd per rank,
    striped remote halves, setup-time autotune, the all-rank gathers) on one
    GPU: both ranks and both daemons share GPU 0 (OCM_BENCH_SHARE_GPU)."""
    env = dict(os.environ, OCM_BENCH_SHARE_GPU="1")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", "29641", os.path.join(REPO, "bench.py"),
                        "--gpus", "2", "--steps", "1", "--warmup", "1", "--max-bytes", str(32 << 20),
                        "--alloc-samples", "50", "--no-characterize", "--no-hw-baseline"],
                       capture_output=True, text=True, timeout=300, cwd="/tmp", env=env)
    assert r.returncode == 0, r.stderr[-4000:]
    res = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert res["n_gpus"] == 2 and res["value"] > 0 and res["config"]["remote_tier"] == "hbm", res
    assert res["autotune"]["ranks"] == 2 and res["autotune"]["put"] in res["autotune"]["GiBps"], res["autotune"]
    # per-peer table and the control-plane extra (RCCL cannot put two ranks on one GPU:
    # its entry records an error or a TCP fallback, the TCP entry must be measured)
    assert res["peers_from_rank0"]["1"]["put_GiBps"] > 0, res["peers_from_rank0"]
    assert res["control_plane"]["tcp"]["alloc_p50_us"] > 0, res["control_plane"]
    assert "rccl" in res["control_plane"], res["control_plane"]
    if os.path.isdir(os.path.join(REPO, "gpurun_out")):
        with open(os.path.join(REPO, "gpurun_out", "bench_share2.json"), "w") as f:
            json.dump(res, f)


@pytest.mark.parametrize("policy", ["ring", "stripe"])
def test_copy_service_small_ops(mesh_factory, policy):
    """Small blocking put/get run on the resident copy service; interleave them
    with launch-path transfers and fills so stale caches would show."""
    import time

    m = mesh_factory(4, gpus=[0, 0, 0, 0], policy=policy)
    with api.Client(daemon_rank=0, gpu=0, ns=m.ns) as c:
        n = 8 << 20
        a = c.alloc(api.OCM_REMOTE_GPU, local_bytes=n, remote_bytes=n, stripe_unit=64 << 10)
        before = api.counters()
        for i, (size, loff, roff) in enumerate([(4, 0, 0), (4096, 0, 4096), (4096 + 12, 64, 65536 - 100),
                                                (65536, 4096, 3 << 16), (200000, 8, 1 << 20), (256 << 10, 0, 0)]):
            seed = 100 + i
            a.fill(seed=seed)                     # launch path writes the local half
            a.put(loff, roff, size)               # service reads it
            a.fill(seed=0)
            a.get(loff, roff, size)               # service writes the local half
            nb = (size // 4) * 4
            assert a.check(seed=seed, offset=loff - loff % 4 + (4 if loff % 4 else 0),
                           nbytes=max(0, nb - 8), first_word=(loff + 3) // 4) == 0, (size, loff, roff)
            # big put (launch path) then small get (service) of what it just wrote
            a.fill(seed=seed + 50)
            a.put(0, 0, n)
            a.fill(seed=0)
            a.get(0, 0, 4096)
            assert a.check(seed=seed + 50, nbytes=4096) == 0
        for k in range(5):
            time.sleep(0.02)                      # service idles out; the next op relaunches it
            a.fill(seed=7 + k)
            t0 = time.perf_counter()
            a.put(0, 0, 4096)
            assert time.perf_counter() - t0 < 1.0, "relaunch after idle exit stalled"
            a.fill(seed=0)
            a.get(0, 0, 4096)
            assert a.check(seed=7 + k, nbytes=4096) == 0
        assert api.counters()["n_put"] > before["n_put"]
        a.free()


@pytest.mark.parametrize("blocks", ["1", "64"])
def test_copy_service_gang(mesh_factory, monkeypatch, blocks):
    """Mid-size blocking ops on the service gang (every workgroup takes a share
    of the tiles, the last one publishes completion): odd sizes and offsets,
    striped over three owners, interleaved with launch-path writes."""
    monkeypatch.setenv("OCM_SERVICE_MAX", str(16 << 20))
    monkeypatch.setenv("OCM_SERVICE_BLOCKS", blocks)
    m = mesh_factory(4, gpus=[0, 0, 0, 0], policy="stripe")
    with api.Client(daemon_rank=0, gpu=0, ns=m.ns) as c:
        n = 24 << 20
        a = c.alloc(api.OCM_REMOTE_GPU, local_bytes=n, remote_bytes=n, stripe_unit=64 << 10)
        assert len(a.remote_info()["extents"]) == 3
        for i, (size, off) in enumerate([(96 << 10, 0), ((1 << 20) + 4, 4096), (3 << 20, 1 << 16),
                                         ((16 << 20) - 4, 8), (5 << 20, (7 << 20) + 64)]):
            seed = 300 + i
            a.fill(seed=seed)
            a.put(off, off, size)
            a.fill(seed=0)
            a.get(off, off, size)
            assert a.check(seed=seed, offset=off, nbytes=size - size % 4, first_word=off // 4) == 0, (size, off)
            a.fill(seed=seed + 50)
            a.put(0, 0, n)                        # launch path (above the service limit)
            a.fill(seed=0)
            a.get(0, 0, 2 << 20)                  # service gang reads what the launch wrote
            assert a.check(seed=seed + 50, nbytes=2 << 20) == 0
        a.free()


def test_copy_service_host_tier_large(mesh_factory):
    """Host-tier pairs keep blocking ops up to 16 MiB on the service gang (the
    default OCM_SERVICE_MAX_HOST), striped over two owners' pinned slabs; sizes
    around both service bounds, odd offsets, and the DMA path above them."""
    m = mesh_factory(3, gpus=[0, 0, 0], policy="stripe")
    with api.Client(daemon_rank=0, gpu=0, ns=m.ns) as c:
        n = 20 << 20
        a = c.alloc(api.OCM_REMOTE_GPU, local_bytes=n, remote_bytes=n, flags=api.OCM_ALLOC_HOST_TIER,
                    stripe_unit=1 << 20)
        assert all(e["tier"] == api.OCM_TIER_HOST for e in a.remote_info()["extents"])
        for i, (size, off) in enumerate([((4 << 20) + 4, 12), (8 << 20, 1 << 20), ((16 << 20) - 4, 4096),
                                         (16 << 20, 0), ((16 << 20) + 64, 64), (n, 0)]):
            seed = 700 + i
            a.fill(seed=seed)
            a.put(off, off, size)
            a.fill(seed=0)
            a.get(off, off, size)
            assert a.check(seed=seed, offset=off, nbytes=size - size % 4, first_word=off // 4) == 0, (size, off)
        a.free()


def test_launch_flag_completion(mesh_factory, monkeypatch):
    """Blocking launch-path ops complete on the kernel-published lane flag
    (service off): odd sizes/offsets up to the flag limit and above it (event
    path), six allocations over four lanes driven from three threads at once,
    so later launches on a lane overtake the flag value a waiter looks for."""
    import threading

    monkeypatch.setenv("OCM_SERVICE_MAX", "0")
    m = mesh_factory(2, gpus=[0, 0])
    with api.Client(daemon_rank=0, gpu=0, ns=m.ns) as c:
        n = 12 << 20
        allocs = [c.alloc(api.OCM_REMOTE_GPU, local_bytes=n, remote_bytes=n) for _ in range(6)]
        errors = []

        def worker(k):
            try:
                for j, (size, off) in enumerate([(4096, 0), (100000, 12), ((1 << 20) + 4, 4096), (4 << 20, 0),
                                                  ((8 << 20) + 64, 1 << 20)]):
                    for a in allocs[k::3]:
                        seed = 1000 + 10 * k + j
                        a.fill(seed=seed)
                        a.put(off, off, size)
                        a.fill(seed=0)
                        a.get(off, off, size)
                        bad = a.check(seed=seed, offset=off, nbytes=size - size % 4, first_word=off // 4)
                        if bad:
                            errors.append((k, size, off, bad))
            except Exception as e:  # noqa: BLE001 - reported below
                errors.append(repr(e))

        threads = [threading.Thread(target=worker, args=(k,)) for k in range(3)]
        for t in threads:
            t.start()
        for t in threads:
            t.join(timeout=100)
        assert not any(t.is_alive() for t in threads), "a blocking op never completed"
        assert not errors, errors
        for a in allocs:
            a.free()


def test_tensor_views_on_peer_memory(mesh_factory):
    """Zero-copy torch views: compute directly on the remote half (another
    daemon's HBM via IPC) and move it with one-sided ops."""
    m = mesh_factory(2, gpus=[0, 0])
    with api.Client(daemon_rank=0, gpu=0, ns=m.ns) as c:
        n = 1 << 20
        a = c.alloc(api.OCM_REMOTE_GPU, local_bytes=4 * n, remote_bytes=4 * n)
        loc = a.local_tensor(torch.float32)
        rem = a.remote_tensor(torch.float32)
        assert loc.device.type == "cuda" and rem.numel() == n
        loc.copy_(torch.arange(n, dtype=torch.float32, device="cuda:0"))
        a.put(0, 0, 4 * n)
        torch.cuda.synchronize()
        rem.mul_(2.0)                              # a torch kernel on peer memory
        torch.cuda.synchronize()
        a.get(0, 0, 4 * n)
        assert torch.equal(loc, 2.0 * torch.arange(n, dtype=torch.float32, device="cuda:0"))
        a.free()


def test_network_tier_hbm_owner(mesh_factory):
    # two "nodes" (host aliases) sharing the MI355X: rank1's HBM is reached through its
    # data server, the app's local half is device memory staged through pinned buffers
    m = mesh_factory(2, gpus=[0, 0], rank_env={0: {"OCM_HOST_ALIAS": "nodeA"}, 1: {"OCM_HOST_ALIAS": "nodeB"}})
    with api.Client(daemon_rank=0, gpu=0, ns=m.ns) as c:
        n = (24 << 20) + 4096
        a = c.alloc(api.OCM_REMOTE_GPU, local_bytes=n, remote_bytes=n)
        e = a.remote_info()["extents"][0]
        assert e["owner_rank"] == 1 and e["tier"] == api.OCM_TIER_GPU and e["net"]
        a.fill(seed=17)
        a.put(0, 0, n)
        a.fill(seed=0)
        a.get(0, 0, n)
        assert a.check(seed=17) == 0
        t = torch.arange(n // 4, dtype=torch.int32, device="cuda:0")
        a.local_tensor(torch.int32)[: n // 4].copy_(t)
        torch.cuda.synchronize()
        a.put(0, 4096, n - 4096)
        a.local_tensor(torch.int32).zero_()
        torch.cuda.synchronize()
        a.get(0, 4096, n - 4096)
        torch.cuda.synchronize()
        assert torch.equal(a.local_tensor(torch.int32)[: (n - 4096) // 4], t[: (n - 4096) // 4])
        assert c.stats(1)["gpu_used"] >= n
        a.free()


def test_async_lanes_per_allocation(mesh_factory):
    # async ops queue per allocation (lane streams): ops on different allocations
    # overlap, ocm_wait(a) waits for a only, blocking ops keep program order.
    m = mesh_factory(3, gpus=[0, 0, 0])
    with api.Client(daemon_rank=0, gpu=0, ns=m.ns) as c:
        n = 32 << 20
        allocs = [c.alloc(api.OCM_REMOTE_GPU, local_bytes=n, remote_bytes=n) for _ in range(6)]
        for i, a in enumerate(allocs):
            a.fill(seed=30 + i)
        for a in allocs:
            a.put(0, 0, n, async_=True)
        for a in reversed(allocs):
            a.wait()
        for a in allocs:
            a.fill(seed=0)
        for a in allocs:
            a.get(0, 0, n, async_=True)
        for i, a in enumerate(allocs):
            a.wait()
            assert a.check(seed=30 + i) == 0, i
        # async put, then a blocking get of the other half: the get waits for the put
        a = allocs[0]
        a.fill(seed=77)
        a.put(0, 0, n, async_=True)
        a.get(0, n // 2, n // 2)
        assert a.check(seed=77, offset=0, nbytes=n // 2, first_word=n // 8) == 0
        # NULL wait: everything
        for a in allocs:
            a.put(0, 0, n, async_=True)
        assert c.lib.ocm_wait(None) == 0
        for a in allocs:
            a.free()


def test_pinned_local_halves_are_pooled(mesh_factory):
    # RDMA/RMA kinds keep their local half in pinned host memory; it comes from a
    # per-process arena (shared 64 MiB chunks + cached dedicated chunks), so
    # allocations must never overlap and freed ranges must be reused.
    import random

    m = mesh_factory(2, gpus=[0, 0])
    rng = random.Random(5)
    with api.Client(daemon_rank=0, gpu=0, ns=m.ns) as c:
        live = {}
        seed = 100
        for rnd in range(4):
            for _ in range(12):
                n = rng.choice([4096, 100_000, 1 << 20, 5 << 20, 40 << 20])
                a = c.alloc(api.OCM_REMOTE_RDMA, local_bytes=n, remote_bytes=n)
                seed += 1
                a.fill(seed=seed)
                live[seed] = (a, n)
            for s, (a, n) in live.items():  # nothing overwrote anything
                assert a.check(seed=s) == 0, (rnd, s, n)
            for s in rng.sample(sorted(live), len(live) // 2):
                live.pop(s)[0].free()
        for s, (a, n) in list(live.items()):
            a.put(0, 0, n)
            a.fill(seed=0)
            a.get(0, 0, n)
            assert a.check(seed=s) == 0
            a.free()
        t0 = time.perf_counter()
        for _ in range(20):  # a cached dedicated chunk: no re-pinning
            c.alloc(api.OCM_REMOTE_RDMA, local_bytes=64 << 20, remote_bytes=1 << 20).free()
        assert (time.perf_counter() - t0) / 20 < 2e-3


def test_remote_to_remote_copy_one_launch(mesh_factory):
    # ocm_copy between two striped pairs with different stripe units and offsets:
    # every source segment becomes one descriptor of a single batched launch.
    m = mesh_factory(4, gpus=[0, 0, 0, 0], policy="stripe")
    with api.Client(daemon_rank=0, gpu=0, ns=m.ns) as c:
        n = 24 << 20
        a = c.alloc(api.OCM_REMOTE_GPU, local_bytes=n, remote_bytes=n, stripe_unit=64 << 10)
        b = c.alloc(api.OCM_REMOTE_GPU, local_bytes=n, remote_bytes=n, stripe_unit=256 << 10)
        a.fill(seed=31)
        a.put(0, 0, n)
        before = api.counters()["n_batch_launches"]
        k = (16 << 20) + 4096
        api.copy(b, a, k, src_offset=12288, dest_offset=4096)  # b.remote[4096:] <- a.remote[12288:]
        assert api.counters()["n_batch_launches"] == before + 1  # one launch, not one per 64 KiB segment
        b.fill(seed=0)
        b.get(4096, 4096, k)
        # a.local held pattern words from offset 0; a.remote[12288 + i] == pattern word (12288 + i) / 4
        assert b.check(seed=31, offset=4096, nbytes=k, first_word=12288 // 4) == 0
        a.free()
        b.free()


def test_threads_share_the_library(mesh_factory):
    # Blocking transfers wait outside the library lock: threads on different
    # allocations overlap, and every round trip stays exact.
    import threading

    m = mesh_factory(3, gpus=[0, 0, 0], policy="stripe")
    errors = []
    with api.Client(daemon_rank=0, gpu=0, ns=m.ns) as c:
        n = 64 << 20
        allocs = [c.alloc(api.OCM_REMOTE_GPU, local_bytes=n, remote_bytes=n) for _ in range(4)]

        def worker(i, a):
            try:
                for r in range(5):
                    s = 1000 + 10 * i + r
                    a.fill(seed=s)
                    a.put(0, 0, n)
                    a.fill(seed=0)
                    a.get(0, 0, n)
                    if a.check(seed=s) != 0:
                        errors.append((i, r))
                    a.batch([(0, 0, 4096, 8192), (1, 8192, 0, 4096)])  # batches interleave too
            except Exception as e:  # noqa: BLE001
                errors.append((i, repr(e)))

        ts = [threading.Thread(target=worker, args=(i, a)) for i, a in enumerate(allocs)]
        for t in ts:
            t.start()
        for t in ts:
            t.join(timeout=120)
        assert not errors, errors
        for a in allocs:
            a.free()


def test_host_tier_prefers_the_gpus_numa_node(mesh_factory):
    m = mesh_factory(1, gpus=[0])
    with api.Client(daemon_rank=0, gpu=0, ns=m.ns) as c:
        a = c.alloc(api.OCM_REMOTE_GPU, local_bytes=1 << 20, remote_bytes=1 << 20)  # N=1: host tier
        assert a.remote_info()["extents"][0]["tier"] == api.OCM_TIER_HOST
        import re

        node = int(re.search(r"host tier on NUMA node (-?\d+)", m.logs()).group(1))
        if node < 0:
            pytest.skip("no NUMA information for this GPU")
        maps = open(f"/proc/{m.daemons[0].proc.pid}/numa_maps").read()
        slab = [l for l in maps.splitlines() if "ocm_host_slab" in l]
        assert slab and all(f"prefer:{node}" in l for l in slab), slab
        a.free()


@pytest.mark.parametrize("proto", ["1", "0"])
def test_copy_service_protocols(mesh_factory, monkeypatch, proto):
    """Small blocking ops through the service with the write-through hand-off
    (default, OCM_SERVICE_PROTO=1) and the fenced one (0), unaligned sizes and
    offsets included: data verified, and the library's service diagnostics
    count every op."""
    monkeypatch.setenv("OCM_SERVICE_PROTO", proto)
    m = mesh_factory(2, gpus=[0, 0])
    with api.Client(daemon_rank=0, gpu=0, ns=m.ns) as c:
        n = 1 << 20
        a = c.alloc(api.OCM_REMOTE_GPU, local_bytes=n, remote_bytes=n)
        before = api.service_stats()["ops"]
        for i, (size, off) in enumerate([(4096, 0), (100, 4), (65536 + 12, 4096), (256 << 10, 1 << 16)]):
            a.fill(seed=40 + i)
            a.put(off, off, size)
            a.fill(seed=0)
            a.get(off, off, size)
            assert a.check(seed=40 + i, offset=off, nbytes=size - size % 4, first_word=off // 4) == 0, (size, off)
        st = api.service_stats()
        assert st["ops"] - before == 8, st
        assert st["relaunches"] >= 0, st
        assert st["gpu_us"] is not None and 0 < st["gpu_us"] < 1000, st
        a.free()


def test_autotune_installs_a_per_direction_choice(mesh_factory):
    """workloads.autotune on one process (no gather): every candidate runs on
    the GPU, the winner per direction is installed, and put/get under it keep
    the data intact (odd sizes and offsets, register and LDS variants)."""
    from oncilla_amd.models import workloads as wl

    m = mesh_factory(2, gpus=[0, 0], policy="stripe")
    with api.Client(daemon_rank=0, gpu=0, ns=m.ns) as c:
        n = 48 << 20
        a = c.alloc(api.OCM_REMOTE_GPU, local_bytes=n, remote_bytes=n)
        try:
            r = wl.autotune(a, 32 << 20, reps=1)
            assert r["get"] in wl.TUNING_CANDIDATES and r["put"] in wl.TUNING_CANDIDATES, r
            assert all(isinstance(v, float) for row in r["GiBps"].values() for v in row.values()), r
            for i, (size, off) in enumerate([(40 << 20, 0), ((8 << 20) + 4, 4096), ((33 << 20) - 4, 1 << 20)]):
                a.fill(seed=70 + i)
                a.put(off, off, size)
                a.fill(seed=0)
                a.get(off, off, size)
                assert a.check(seed=70 + i, offset=off, nbytes=size - size % 4, first_word=off // 4) == 0, (r, size)
            # explicit per-direction split: LDS-DMA puts, register gets
            api.set_tuning_dir(1, 2, 0, True)
            api.set_tuning_dir(0, 1, 256, False)
            a.fill(seed=99)
            a.put(0, 0, 40 << 20)
            a.fill(seed=0)
            a.get(0, 0, 40 << 20)
            assert a.check(seed=99, nbytes=40 << 20) == 0
        finally:
            api.set_tuning()
            a.free()


def test_stream_wait_orders_host_tier_memcpy(mesh_factory):
    """ocm_stream_wait must hold back a put whose pieces the CPU copies (pinned
    local half <-> host tier): the GPU write into the local half queued on
    another stream lands first (the memcpy ignored the dependency)."""
    m = mesh_factory(1, gpus=[0])
    with api.Client(daemon_rank=0, gpu=0, ns=m.ns) as c:
        n = 8 << 20
        a = c.alloc(api.OCM_REMOTE_RDMA, local_bytes=n, remote_bytes=n, flags=api.OCM_ALLOC_HOST_TIER)
        assert a.remote_info()["extents"][0]["tier"] == api.OCM_TIER_HOST
        loc = a.local_tensor()
        assert loc.device.type == "cpu" and loc.is_pinned()
        loc.zero_()
        src = torch.full((n,), 7, dtype=torch.uint8, device="cuda:0")
        st = torch.cuda.Stream(device=0)
        torch.cuda.synchronize()
        with torch.cuda.stream(st):
            torch.cuda._sleep(200_000_000)  # keep the stream busy for a while
            loc.copy_(src, non_blocking=True)  # D2H into the pinned local half, after the spin
        a.stream_wait(st)
        a.put(0, 0, n)
        st.synchronize()
        loc.zero_()
        a.get(0, 0, n)
        assert int((loc != 7).sum()) == 0
        a.free()


@pytest.mark.parametrize("host_tier", [False, True])
def test_torch_tensors_in_peer_hbm(mesh_factory, host_tier):
    """RemoteMemPool: tensors allocated under it are blocks of another daemon's HBM
    (same-GPU stand-in here) or its pinned host tier, used in place by torch
    kernels, and returned to the owner when torch releases them."""
    import gc

    from oncilla_amd.torch_pool import RemoteMemPool

    used = "host_used" if host_tier else "gpu_used"
    m = mesh_factory(2, gpus=[0, 0])
    with api.Client(daemon_rank=0, gpu=0, ns=m.ns) as c:
        before = c.stats(1)[used]
        pool = RemoteMemPool(c, remote_rank=1, host_tier=host_tier)
        with pool:
            x = torch.arange(1 << 22, device="cuda:0", dtype=torch.float32)
            w = torch.ones((1024, 1024), device="cuda:0")
        st = RemoteMemPool.stats()
        assert st["blocks"] >= 1 and st["bytes"] >= 16 << 20, st
        assert c.stats(1)[used] >= before + (16 << 20)
        y = torch.ones(4, device="cuda:0")  # outside the pool: ordinary device memory
        assert RemoteMemPool.stats() == st
        assert float((x * 2).sum()) == float(2 * torch.arange(1 << 22, dtype=torch.float64).sum())
        assert torch.equal(w @ w, torch.full((1024, 1024), 1024.0, device="cuda:0"))
        del x, w, y
        gc.collect()
        torch.cuda.synchronize()
        del pool
        gc.collect()
        torch.cuda.empty_cache()
        torch.cuda.synchronize()
        assert RemoteMemPool.stats()["blocks"] == 0
        deadline = time.time() + 10  # a capacity lease taken on rank 1 goes back after 2 s idle
        while c.stats(1)[used] != before and time.time() < deadline:
            time.sleep(0.1)
        assert c.stats(1)[used] == before


def test_torch_pool_random_churn(mesh_factory):
    """Random tensor sizes created and dropped under RemoteMemPool, each filled
    with its own value: torch splits and reuses the remote blocks, and no live
    tensor may ever see another's bytes (overlapping blocks would show)."""
    import gc
    import random

    from oncilla_amd.torch_pool import RemoteMemPool

    m = mesh_factory(2, gpus=[0, 0])
    rng = random.Random(5)
    with api.Client(daemon_rank=0, gpu=0, ns=m.ns) as c:
        pool = RemoteMemPool(c, remote_rank=1)
        live = {}
        for step in range(400):
            if live and rng.random() < 0.45:
                k = rng.choice(list(live))
                t, v = live.pop(k)
                assert bool((t == v).all()), (step, k)
                del t
            else:
                n = rng.choice([1, 7, 513, 4096, 100_000, 1 << 20, 3 << 20, 9 << 20])
                with pool:
                    t = torch.full((n,), float(step), device="cuda:0")
                live[step] = (t, float(step))
            if step % 50 == 49:
                for k, (t, v) in live.items():
                    assert bool((t == v).all()), (step, k)
                torch.cuda.empty_cache()  # hands free blocks back to the owner mid-run
        for k, (t, v) in live.items():
            assert bool((t == v).all()), k
        assert RemoteMemPool.stats()["blocks"] >= 1
        live.clear()
        del t  # the loop variable still holds the last tensor
        gc.collect()
        del pool
        gc.collect()
        torch.cuda.empty_cache()
        torch.cuda.synchronize()
        assert RemoteMemPool.stats()["blocks"] == 0



@pytest.mark.gpu
def test_selftest_on_this_node():
    """The node self-test on the GPU box: every owner daemon's round trip verified
    (one GPU: the daemon's pinned host tier), rates reported."""
    from oncilla_amd.utils.selftest import run

    rep = run(nbytes=16 << 20, samples=50)
    assert rep["ok"], rep
    assert all(p["get_GiBps"] > 1 and p["put_GiBps"] > 1 for p in rep["peers"].values()), rep

"""Tick control transport (daemon records over a collective).
On CPU the collective is the socket ring; on a GPU box `--ctrl rccl` uses
ncclAllGather over xGMI (N=1 on a single-GPU box)."""
import os
import subprocess
import sys
import textwrap

import pytest

from oncilla_amd import api


@pytest.fixture(autouse=True)
def _cpu_app(monkeypatch):
    monkeypatch.setenv("OCM_NO_GPU", "1")


def _seal_env(sealed):
    """"0": host-filled slots, "1": the socket stand-in for the RCCL seal kernel,
    "batch4": that, with ticks queued 4 at a time as the RCCL collective queues
    replays of a captured graph (OCM_TICK_GRAPH)."""
    if sealed == "batch4":
        return {"OCM_TICK_SOCKET_SEAL": "1", "OCM_TICK_SOCKET_BATCH": "4"}
    return {"OCM_TICK_SOCKET_SEAL": sealed}


def _wait_ticking(c, n):
    """Wait until every rank has completed a tick, without posting anything: idle ticks
    keep an idle mesh ticking, and the join is the first traffic. The fault-injection
    tests use this, so the first DO_ALLOC / DO_FREE is the test's own."""
    import time

    deadline = time.time() + 20
    while time.time() < deadline:
        if all(c.stats(r)["ctrl_ticks"] > 0 for r in range(n)):
            return
        time.sleep(0.02)
    raise AssertionError("the tick transport never ticked on every rank")


def _wait_tick_up(c, n):
    import time

    # The transport starts right after the mesh is complete; wait until every rank ticked.
    deadline = time.time() + 20
    while time.time() < deadline:
        a = c.alloc(api.OCM_REMOTE_RDMA, local_bytes=4096, remote_bytes=4096)
        a.free()
        if all(c.stats(r)["ctrl_ticks"] > 0 for r in range(n)):
            return
        time.sleep(0.05)
    raise AssertionError("tick transport never came up")


@pytest.mark.parametrize("sealed", ["0", "1", "batch4"])
def test_socket_tick_mesh_suite(mesh_factory, native, tool, sealed):
    # sealed=1: the socket collective emulates the RCCL seal kernel (outbox ring
    # sealed when the tick runs), so the device-sealed protocol runs multi-rank here
    m = mesh_factory(4, extra_args=["--ctrl", "socket"], env=_seal_env(sealed))
    with api.Client(daemon_rank=0, ns=m.ns) as c:
        _wait_tick_up(c, 4)
        t0 = [c.stats(r)["ctrl_ticks"] for r in range(4)]
        a = c.alloc(api.OCM_REMOTE_RDMA, local_bytes=8 << 20, remote_bytes=8 << 20, flags=api.OCM_ALLOC_STRIPE)
        assert len(a.remote_info()["extents"]) == 3
        a.fill(seed=5)
        a.put(0, 0, 8 << 20)
        a.fill(seed=0)
        a.get(0, 0, 8 << 20)
        assert a.check(seed=5) == 0
        a.free()
        t1 = [c.stats(r)["ctrl_ticks"] for r in range(4)]
        assert all(b > a_ for a_, b in zip(t0, t1)), (t0, t1)
    for orig in (1, 3):
        for args in (["1", "1", "2", "3"], ["3", "2", "4"], ["5", "8", "1"]):
            rc, out = tool([f"{native}/ocm_test", *args], env=dict(m.client_env(orig), OCM_NO_GPU="1"))
            assert rc == 0, out + m.logs()


@pytest.mark.parametrize("sealed", ["0", "1", "batch4"])
def test_socket_tick_concurrent_churn(mesh_factory, sealed):
    m = mesh_factory(4, extra_args=["--ctrl", "socket"], env=_seal_env(sealed))
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = textwrap.dedent(f"""
        import sys; sys.path.insert(0, {repo!r})
        from oncilla_amd import api
        from oncilla_amd.models import workloads as wl
        r = int(sys.argv[1])
        with api.Client(daemon_rank=r % 4, ns={m.ns!r}) as c:
            wl.churn(c, 40, api.OCM_REMOTE_RDMA, 64 << 10, 64 << 10, seed=r)
    """)
    procs = [subprocess.Popen([sys.executable, "-c", code, str(i)], stderr=subprocess.PIPE, text=True,
                              env=dict(os.environ, OCM_NO_GPU="1")) for i in range(8)]
    for p in procs:
        _, err = p.communicate(timeout=180)
        assert p.returncode == 0, err + m.logs()
    with api.Client(daemon_rank=0, ns=m.ns) as c:
        assert all(c.stats(r)["host_used"] == 0 for r in range(4))
        assert all(c.stats(r)["ctrl_ticks"] > 0 for r in range(4))


@pytest.mark.parametrize("sealed", ["0", "1", "batch4"])
def test_tick_peer_death_falls_back_to_tcp(mesh_factory, sealed):
    m = mesh_factory(3, extra_args=["--ctrl", "socket"], env=_seal_env(sealed))
    with api.Client(daemon_rank=0, ns=m.ns) as c:
        _wait_tick_up(c, 3)
        m.kill(2)
        import time

        time.sleep(0.3)
        a = c.alloc(api.OCM_REMOTE_RDMA, local_bytes=4096, remote_bytes=1 << 20)  # rank1 over TCP now
        assert a.remote_info()["extents"][0]["owner_rank"] == 1
        a.free()


@pytest.mark.parametrize("sealed", ["0", "1"])
def test_tick_failure_after_do_alloc_does_not_duplicate_it(mesh_factory, sealed):
    """when the tick transport fails, the sender re-sends over TCP
    every record it cannot prove delivered. Here rank0's tick fails right after
    the tick that carried its DO_ALLOC reached the owner (OCM_TICK_FAULT), so the
    owner receives that DO_ALLOC twice; it must allocate once (a second extent
    would leak, and a second response would free a live one)."""
    import time

    m = mesh_factory(3, extra_args=["--ctrl", "socket"],
                     env={"OCM_TICK_SOCKET_SEAL": sealed, "OCM_TICK_FAULT": "fail_after_do_alloc",
                          "OCM_LEASE_BYTES": "0"})
    with api.Client(daemon_rank=0, ns=m.ns) as c:
        deadline = time.time() + 20  # STATS records ride the ticks too: wait until every rank ticked
        while not all([c.stats(r)["ctrl_ticks"] > 0 for r in range(3)]):  # every rank asked: remote STATS tick
            assert time.time() < deadline, "tick transport never came up"
            time.sleep(0.05)
        held = []
        for i in range(6):  # the first DO_ALLOC trips the fault; the rest ride TCP
            a = c.alloc(api.OCM_REMOTE_RDMA, local_bytes=1 << 20, remote_bytes=1 << 20)
            a.fill(seed=60 + i)
            a.put(0, 0, 1 << 20)
            a.fill(seed=0)
            a.get(0, 0, 1 << 20)
            assert a.check(seed=60 + i) == 0
            held.append(a)
        used = sum(c.stats(r)["host_used"] for r in range(3))
        assert used == 6 << 20, f"{used} bytes placed for 6 x 1 MiB (a re-sent DO_ALLOC was served twice)"
        for a in held:
            a.free()
        deadline = time.time() + 5
        while sum(c.stats(r)["host_used"] for r in range(3)) and time.time() < deadline:
            time.sleep(0.05)
        assert all(c.stats(r)["host_used"] == 0 for r in range(3))
    logs = m.logs()
    assert "injected failure after a DO_ALLOC tick" in logs, logs
    assert "dropping a second copy of MSG_DO_ALLOC" in logs, logs
    assert logs.count("leaving the socket tick transport") == 3, logs  # the whole mesh left it together


@pytest.mark.parametrize("sealed", ["0", "1"])
def test_tick_failure_after_do_free_frees_once(mesh_factory, sealed):
    """the fallback marks re-sent records (kMsgResent) and the receiver
    compares only those with what the ticks delivered. Here the tick that carried
    a DO_FREE reaches the owner, then fails, so the owner gets that DO_FREE twice;
    it must free once, and allocations made afterwards (whose records may repeat
    earlier ones byte for byte) must all be served."""
    import time

    m = mesh_factory(3, extra_args=["--ctrl", "socket"],
                     env={"OCM_TICK_SOCKET_SEAL": sealed, "OCM_TICK_FAULT": "fail_after_do_free",
                          "OCM_LEASE_BYTES": "0"})
    with api.Client(daemon_rank=0, ns=m.ns) as c:
        _wait_ticking(c, 3)
        held = [c.alloc(api.OCM_REMOTE_RDMA, local_bytes=1 << 20, remote_bytes=1 << 20) for _ in range(4)]
        for a in held:  # the first DO_FREE trips the fault; the rest ride TCP
            a.free()
        deadline = time.time() + 5
        while sum(c.stats(r)["host_used"] for r in range(3)) and time.time() < deadline:
            time.sleep(0.05)
        assert all(c.stats(r)["host_used"] == 0 for r in range(3))
        again = []
        for i in range(6):
            a = c.alloc(api.OCM_REMOTE_RDMA, local_bytes=1 << 20, remote_bytes=1 << 20)
            a.fill(seed=80 + i)
            a.put(0, 0, 1 << 20)
            a.fill(seed=0)
            a.get(0, 0, 1 << 20)
            assert a.check(seed=80 + i) == 0
            again.append(a)
        used = sum(c.stats(r)["host_used"] for r in range(3))
        assert used == 6 << 20, f"{used} bytes placed for 6 x 1 MiB"
        for a in again:
            a.free()
    logs = m.logs()
    assert "injected failure after a DO_FREE tick" in logs, logs
    assert "dropping a second copy of MSG_DO_FREE" in logs, logs
    assert "dropping a second copy of MSG_DO_ALLOC" not in logs, logs


def test_socket_tick_self_loop(mesh_factory):
    # OCM_TICK_SELF routes a daemon's self-addressed records through the collective too.
    m = mesh_factory(1, extra_args=["--ctrl", "socket"], env={"OCM_TICK_SELF": "1"})
    with api.Client(daemon_rank=0, ns=m.ns) as c:
        _wait_tick_up(c, 1)
        a = c.alloc(api.OCM_REMOTE_RDMA, local_bytes=1 << 20, remote_bytes=1 << 20)
        a.free()
        assert c.stats(0)["ctrl_ticks"] > 0


RCCL_TICK_MODES = {
    "default": {},  # tagged slots, 6 us seal wait
    "done_kernel": {"OCM_TICK_DONE_KERNEL": "1", "OCM_TICK_SEAL_WAIT_US": "0"},
    "done_kernel_wait": {"OCM_TICK_DONE_KERNEL": "1"},
    "tagged_wait_seal2": {"OCM_TICK_DONE_KERNEL": "0", "OCM_TICK_SEAL_WAIT_US": "6", "OCM_TICK_SEAL_SPEC": "0"},
    "depth3_tagged_wait": {"OCM_TICK_DEPTH": "3", "OCM_TICK_DONE_KERNEL": "0", "OCM_TICK_SEAL_WAIT_US": "4"},
    "two_streams": {"OCM_TICK_STREAMS": "2"},
    "two_streams_depth3_done_kernel": {"OCM_TICK_STREAMS": "2", "OCM_TICK_DEPTH": "3", "OCM_TICK_DONE_KERNEL": "1"},
    "graph8": {"OCM_TICK_GRAPH": "8"},  # ticks queued as replays of a captured graph of 8
    "graph2_nowait": {"OCM_TICK_GRAPH": "2", "OCM_TICK_SEAL_WAIT_US": "0"},
    "no_graph": {"OCM_TICK_GRAPH": "0"},
}


@pytest.mark.gpu
@pytest.mark.parametrize("mode", sorted(RCCL_TICK_MODES))
def test_rccl_tick_single_gpu(mesh_factory, monkeypatch, mode):
    """ncclCommInitRank + ncclAllGather on the MI355X carry the daemon's own
    REQ_ALLOC/DO_ALLOC/FREED records (1-rank communicator, OCM_TICK_SELF), with a
    done kernel per tick or with completion read from the gathered slots' tags,
    and with the seal waiting for late records."""
    monkeypatch.delenv("OCM_NO_GPU", raising=False)
    m = mesh_factory(1, gpus=[0], extra_args=["--ctrl", "rccl"], env={"OCM_TICK_SELF": "1", **RCCL_TICK_MODES[mode]})
    with api.Client(daemon_rank=0, gpu=0, ns=m.ns) as c:
        _wait_tick_up(c, 1)
        before = c.stats(0)["ctrl_ticks"]
        for _ in range(20):  # many ticks through every ring slot
            c.alloc(api.OCM_REMOTE_GPU, local_bytes=4096, remote_bytes=4096).free()
        for flags in (api.OCM_ALLOC_LOOPBACK, 0):
            a = c.alloc(api.OCM_REMOTE_GPU, local_bytes=1 << 20, remote_bytes=1 << 20, flags=flags)
            a.fill(seed=1)
            a.put(0, 0, 1 << 20)
            a.fill(seed=0)
            a.get(0, 0, 1 << 20)
            assert a.check(seed=1) == 0
            a.free()
        assert c.stats(0)["ctrl_ticks"] > before
        assert c.stats(0)["ctrl"] == "rccl"  # never fell back
        st = api.tick_stats()  # the daemon's own records, post -> delivery through the allgather
        assert st["transport"] == 2 and st["own_records"] > 0 and st["hop_mean_us"] > 0, st
    logs = m.logs()
    assert "rccl tick transport" in logs
    if RCCL_TICK_MODES[mode].get("OCM_TICK_GRAPH", "0") != "0":
        assert "ticks per captured graph" in logs and "rccl tick graphs unavailable" not in logs, logs


@pytest.mark.gpu
@pytest.mark.parametrize("window_us", ["2000", "-1", "0"])
def test_rccl_idle_seals_wait_on_the_gpu_only_after_traffic(mesh_factory, monkeypatch, window_us):
    """An idle RCCL mesh keeps ticking (OCM_TICK_IDLE_US, 1 ms). An idle seal that waits
    for the doorbell on the GPU keeps a workgroup resident, which delays full-GPU GEMMs,
    so it waits there only within OCM_TICK_IDLE_DEVICE_US (2 ms) of the last tick that
    carried records, and later idle ticks wait on the host (-1: always on the GPU, the
    first cut; 0: always on the host). The daemon logs the split when it stops; records
    posted after the idle stretch still go through."""
    import re
    import time

    monkeypatch.delenv("OCM_NO_GPU", raising=False)
    m = mesh_factory(1, gpus=[0], extra_args=["--ctrl", "rccl"],
                     env={"OCM_TICK_SELF": "1", "OCM_TICK_STATS": "1", "OCM_LEASE_BYTES": "0",
                          "OCM_TICK_IDLE_DEVICE_US": window_us})
    with api.Client(daemon_rank=0, gpu=0, ns=m.ns) as c:
        _wait_tick_up(c, 1)
        for _ in range(10):
            c.alloc(api.OCM_REMOTE_GPU, local_bytes=4096, remote_bytes=4096).free()
        time.sleep(0.1)  # ~100 idle ticks
        c.alloc(api.OCM_REMOTE_GPU, local_bytes=4096, remote_bytes=4096).free()
        assert c.stats(0)["ctrl"] == "rccl"
    m.stop()
    logs = m.logs()
    found = re.search(r"idle ticks: (\d+) waited on the GPU, (\d+) on the host", logs)
    assert found, logs[-3000:]
    dev, host = int(found.group(1)), int(found.group(2))
    print(f"window {window_us} us: {dev} idle ticks waited on the GPU, {host} on the host")
    if window_us == "-1":
        assert host == 0 and dev >= 20, (dev, host)
    elif window_us == "0":
        assert dev == 0 and host >= 20, (dev, host)
    else:
        assert dev >= 1 and host >= 20, (dev, host)


def _ctrl(c, n):
    return [c.stats(r)["ctrl"] for r in range(n)]


def test_ctrl_auto_without_gpus_stays_on_tcp(mesh_factory):
    """--ctrl auto (the default): RCCL needs a GPU per rank; CPU daemons keep TCP
    and never start a tick transport."""
    m = mesh_factory(3)
    with api.Client(daemon_rank=0, ns=m.ns) as c:
        a = c.alloc(api.OCM_REMOTE_RDMA, local_bytes=1 << 20, remote_bytes=1 << 20, flags=api.OCM_ALLOC_STRIPE)
        a.free()
        assert _ctrl(c, 3) == ["tcp"] * 3
        assert all(c.stats(r)["ctrl_ticks"] == 0 for r in range(3))
    assert "daemon<->daemon records: tcp (--ctrl auto)" in m.logs()


@pytest.mark.parametrize("sealed", ["0", "1", "batch4"])
def test_ctrl_auto_eight_ranks_join_over_the_ticks(mesh_factory, sealed):
    """--ctrl auto with the CPU stand-in for RCCL (OCM_CTRL_AUTO_SOCKET): rank0
    starts the transport as each link comes up, every peer's join (ADD_NODE,
    NODE_LINKS) is the transport's first traffic, and the 8-rank mesh then
    carries striped allocations on it."""
    m = mesh_factory(8, env={"OCM_CTRL_AUTO_SOCKET": "1", **_seal_env(sealed)})
    with api.Client(daemon_rank=3, ns=m.ns) as c:
        assert _ctrl(c, 8) == ["socket"] * 8
        t0 = [c.stats(r)["ctrl_ticks"] for r in range(8)]
        assert all(t > 0 for t in t0), t0  # the joins ticked before any app traffic
        for i in range(4):
            a = c.alloc(api.OCM_REMOTE_RDMA, local_bytes=(7 << 20) + 5, remote_bytes=(7 << 20) + 5,
                        flags=api.OCM_ALLOC_STRIPE)
            assert len(a.remote_info()["extents"]) == 7
            a.fill(seed=80 + i)
            a.put(0, 0, 7 << 20)
            a.fill(seed=0)
            a.get(0, 0, 7 << 20)
            assert a.check(seed=80 + i, nbytes=7 << 20) == 0
            a.free()
    logs = m.logs()
    assert logs.count("joining rank0 (tick transport up") == 7, logs
    assert "falling back to TCP" not in logs and "leaving the" not in logs


def test_ctrl_auto_falls_back_to_tcp_when_the_transport_never_comes_up(mesh_factory):
    """A communicator that never forms (OCM_TICK_FAULT=init_hang): after
    OCM_TICK_UP_MS every rank leaves the transport, the deferred joins ride TCP,
    and the mesh serves allocations."""
    import time

    t0 = time.time()
    m = mesh_factory(4, env={"OCM_CTRL_AUTO_SOCKET": "1", "OCM_TICK_FAULT": "init_hang", "OCM_TICK_UP_MS": "400"})
    assert time.time() - t0 < 30
    with api.Client(daemon_rank=2, ns=m.ns) as c:
        a = c.alloc(api.OCM_REMOTE_RDMA, local_bytes=1 << 20, remote_bytes=1 << 20, flags=api.OCM_ALLOC_STRIPE)
        a.fill(seed=9)
        a.put(0, 0, 1 << 20)
        a.fill(seed=0)
        a.get(0, 0, 1 << 20)
        assert a.check(seed=9) == 0
        a.free()
        assert _ctrl(c, 4) == ["tcp (left ticks)"] * 4
        assert all(c.stats(r)["ctrl_ticks"] == 0 for r in range(4))
    logs = m.logs()
    assert "not up within OCM_TICK_UP_MS=400 ms" in logs, logs


@pytest.mark.parametrize("sealed", ["0", "1", "batch4"])
def test_a_wedged_collective_times_out_and_the_mesh_falls_back(mesh_factory, sealed):
    """A rank stops taking part in the ticks without any error (a wedged
    collective: OCM_TICK_FAULT=stall_after=N on rank 2). The other ranks' tick
    watchdog (OCM_TICK_TIMEOUT_MS) ends the transport, everybody leaves it, what
    the ticks had not delivered goes over TCP, and allocations keep working."""
    m = mesh_factory(3, extra_args=["--ctrl", "socket"],
                     env={**_seal_env(sealed), "OCM_TICK_TIMEOUT_MS": "400", "OCM_LEASE_BYTES": "0"},
                     rank_env={2: {"OCM_TICK_FAULT": "stall_after=30"}})
    with api.Client(daemon_rank=1, ns=m.ns) as c:
        for i in range(30):  # stalls part-way through: later ones need the TCP fallback
            a = c.alloc(api.OCM_REMOTE_RDMA, local_bytes=1 << 20, remote_bytes=1 << 20, flags=api.OCM_ALLOC_STRIPE)
            a.fill(seed=40 + i)
            a.put(0, 0, 1 << 20)
            a.fill(seed=0)
            a.get(0, 0, 1 << 20)
            assert a.check(seed=40 + i) == 0
            a.free()
        assert all(c.stats(r)["ctrl"] == "tcp (left ticks)" for r in range(3))
    logs = m.logs()
    assert "OCM_TICK_TIMEOUT_MS" in logs, logs
    assert logs.count("leaving the socket tick transport") == 3, logs


def test_a_rank_without_tick_batches_stays_in_step(mesh_factory):
    """Ticks queued 4 at a time (the socket stand-in for replays of a captured
    graph, OCM_TICK_GRAPH) on every rank but one, which queues them one at a time
    as an RCCL rank whose capture failed does (OCM_TICK_FAULT=no_batch). All
    ranks round their tick targets to the same quantum, so they keep joining the
    same collectives: striped allocations work and nobody leaves the transport."""
    m = mesh_factory(3, extra_args=["--ctrl", "socket"],
                     env={**_seal_env("batch4"), "OCM_TICK_TIMEOUT_MS": "2000", "OCM_LEASE_BYTES": "0"},
                     rank_env={1: {"OCM_TICK_FAULT": "no_batch"}})
    with api.Client(daemon_rank=2, ns=m.ns) as c:
        _wait_tick_up(c, 3)
        for i in range(20):
            a = c.alloc(api.OCM_REMOTE_RDMA, local_bytes=1 << 20, remote_bytes=1 << 20, flags=api.OCM_ALLOC_STRIPE)
            a.fill(seed=20 + i)
            a.put(0, 0, 1 << 20)
            a.fill(seed=0)
            a.get(0, 0, 1 << 20)
            assert a.check(seed=20 + i) == 0
            a.free()
        assert _ctrl(c, 3) == ["socket"] * 3
    logs = m.logs()
    assert "falling back to TCP" not in logs and "leaving the" not in logs, logs


@pytest.mark.parametrize("sealed", ["1", "batch4"])
def test_tick_stats_query(mesh_factory, sealed):
    """api.tick_stats(): the local daemon's tick transport statistics over the
    mailbox (MSG_TICK_STATS): ticks, own records from post to delivery, the host
    time per Collective::start, and how many ticks one start queues."""
    m = mesh_factory(3, extra_args=["--ctrl", "socket"], env={**_seal_env(sealed), "OCM_LEASE_BYTES": "0"})
    with api.Client(daemon_rank=1, ns=m.ns) as c:
        _wait_tick_up(c, 3)
        for _ in range(10):
            c.alloc(api.OCM_REMOTE_RDMA, local_bytes=4096, remote_bytes=1 << 20, remote_rank=2).free()
        st = api.tick_stats()
        assert st is not None and st["ticks"] > 0 and st["own_records"] > 0, st
        assert st["hop_mean_us"] > 0 and st["start_mean_us"] > 0, st
        assert st["transport"] == 1, st  # socket ticks
        assert st["ticks_per_start"] == (4 if sealed == "batch4" else 1), st


def test_tick_stats_on_tcp(mesh_factory):
    m = mesh_factory(2)
    with api.Client(daemon_rank=0, ns=m.ns) as c:
        st = api.tick_stats()
        assert st is not None and st["ticks"] == 0 and st["transport"] == 0, st


@pytest.mark.parametrize("idle_us", ["1000", "0"])
def test_idle_mesh_ticks_instead_of_tcp_wakes(mesh_factory, idle_us):
    """the tick control plane must not depend on TCP. With idle
    ticks (OCM_TICK_IDLE_US, default 1000) an idle 8-rank mesh keeps ticking, and a
    rank that posts into it rings the host-wide doorbell instead of sending
    MSG_TICK_WAKE over TCP: after bursts separated by idle gaps, no rank has sent a
    single TCP wake-up. With 0 (the round-3 protocol) every burst after idle starts
    with TCP wake-ups, which the counter shows."""
    import time

    m = mesh_factory(8, env={"OCM_CTRL_AUTO_SOCKET": "1", "OCM_TICK_SOCKET_SEAL": "1", "OCM_LEASE_BYTES": "0",
                             "OCM_TICK_IDLE_US": idle_us})
    with api.Client(daemon_rank=0, ns=m.ns) as c:
        assert _ctrl(c, 8) == ["socket"] * 8
        for i in range(5):
            time.sleep(0.03)  # past the 64 busy ticks: the mesh is idle again
            t0 = time.perf_counter()
            a = c.alloc(api.OCM_REMOTE_RDMA, local_bytes=4096, remote_bytes=1 << 20, remote_rank=1 + i)
            took = time.perf_counter() - t0
            a.free()
            assert took < 1.0, f"alloc after an idle gap took {took * 1e3:.1f} ms"
    wakes, idle = [], []
    for r in range(8):
        with api.Client(daemon_rank=r, ns=m.ns):
            st = api.tick_stats()
            wakes.append(st["tcp_wakes"])
            idle.append(st["idle_ticks"])
    if idle_us == "0":
        assert sum(wakes) > 0 and sum(idle) == 0, (wakes, idle)
    else:
        assert wakes == [0] * 8 and all(x > 0 for x in idle), (wakes, idle)
        assert "idle ticks, no TCP wake-ups" in m.logs()
    logs = m.logs()
    assert "falling back to TCP" not in logs and "leaving the" not in logs

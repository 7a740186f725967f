"""Failure detection and fault injection (the reference had none).
Daemons read OCM_FAULT=do_alloc_fail=N | drop_do_alloc=N | crash_after_allocs=N."""
import time

import pytest

from oncilla_amd import api


@pytest.fixture(autouse=True)
def _cpu_app(monkeypatch):
    monkeypatch.setenv("OCM_NO_GPU", "1")


def _roundtrip(a, n, seed):
    a.fill(seed=seed)
    a.put(0, 0, n)
    a.fill(seed=0)
    a.get(0, 0, n)
    assert a.check(seed=seed) == 0


def test_owner_refusal_is_replaced(mesh_factory):
    m = mesh_factory(3, rank_env={1: {"OCM_FAULT": "do_alloc_fail=1"}})
    with api.Client(daemon_rank=0, ns=m.ns) as c:
        a = c.alloc(api.OCM_REMOTE_RDMA, local_bytes=1 << 20, remote_bytes=1 << 20)
        # ring would pick rank 1; it refused once, so rank0 re-placed the extent elsewhere
        assert a.remote_info()["extents"][0]["owner_rank"] == 2
        _roundtrip(a, 1 << 20, 3)
        a.free()
        b = c.alloc(api.OCM_REMOTE_RDMA, local_bytes=4096, remote_bytes=1 << 20)  # fault used up
        assert b.remote_info()["extents"][0]["owner_rank"] == 1
        b.free()
        assert c.stats(2)["host_used"] == 0 and c.stats(1)["host_used"] == 0


def test_lost_request_times_out(mesh_factory):
    m = mesh_factory(2, rank_env={0: {"OCM_REQUEST_TIMEOUT_MS": "400"}, 1: {"OCM_FAULT": "drop_do_alloc=1"}})
    with api.Client(daemon_rank=0, ns=m.ns) as c:
        t0 = time.time()
        with pytest.raises(api.OcmError, match="timed out|Connection timed out"):
            c.alloc(api.OCM_REMOTE_RDMA, local_bytes=4096, remote_bytes=1 << 20)
        assert time.time() - t0 < 5
        a = c.alloc(api.OCM_REMOTE_RDMA, local_bytes=4096, remote_bytes=1 << 20)
        _roundtrip(a, 4096, 5)
        a.free()


def test_owner_crash_fails_pending_and_mesh_survives(mesh_factory):
    m = mesh_factory(3, rank_env={2: {"OCM_FAULT": "crash_after_allocs=0"}})
    with api.Client(daemon_rank=1, ns=m.ns) as c:
        t0 = time.time()
        with pytest.raises(api.OcmError):
            c.alloc(api.OCM_REMOTE_RDMA, local_bytes=4096, remote_bytes=1 << 20)  # ring -> rank 2 dies
        assert time.time() - t0 < 10
        time.sleep(0.2)
        a = c.alloc(api.OCM_REMOTE_RDMA, local_bytes=4096, remote_bytes=1 << 20)  # dead rank skipped
        assert a.remote_info()["extents"][0]["owner_rank"] == 0
        _roundtrip(a, 4096, 7)
        a.free()

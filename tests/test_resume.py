"""Checkpoint / resume of the rank0 directory (SURVEY §5 lists it as absent in
the reference; a rank0 loss there ended the mesh, src/mem.c:466-474).

rank0 checkpoints its directory to OCM_STATE_FILE. When it dies, the other
daemons keep serving (the data plane never involved rank0) and reconnect.
A restarted rank0 reloads the checkpoint, and every survivor reports the
extents it holds. Confirmed extents get their capacity re-reserved, frees made
while rank0 was away are dropped, and alloc ids continue past the old ones.
"""
import os
import signal
import time

import pytest

from oncilla_amd import api

MiB = 1 << 20


@pytest.fixture(autouse=True)
def _cpu_app(monkeypatch):
    monkeypatch.setenv("OCM_NO_GPU", "1")


def _wait(pred, timeout=10.0):
    deadline = time.time() + timeout
    while time.time() < deadline:
        if pred():
            return True
        time.sleep(0.02)
    return False


def test_rank0_restart_resumes_directory(mesh_factory, tmp_path):
    state = str(tmp_path / "directory.ckpt")
    m = mesh_factory(3, rank_env={0: {"OCM_STATE_FILE": state}}, extra_args=["--host-capacity", str(8 * MiB)])
    with api.Client(daemon_rank=1, ns=m.ns) as c:
        a = c.alloc(api.OCM_REMOTE_RDMA, local_bytes=4 * MiB, remote_bytes=4 * MiB)
        b = c.alloc(api.OCM_REMOTE_RDMA, local_bytes=MiB, remote_bytes=2 * MiB)
        assert a.remote_info()["extents"][0]["owner_rank"] == 2
        assert b.remote_info()["extents"][0]["owner_rank"] == 2
        a.fill(seed=1)
        a.put(0, 0, 4 * MiB)
        assert _wait(lambda: os.path.exists(state) and f"entry {b.remote_info()['alloc_id']} " in open(state).read())

        m.kill(0, signal.SIGKILL)
        # rank0 is gone: the data plane and frees to owners keep working ...
        a.fill(seed=0)
        a.get(0, 0, 4 * MiB)
        assert a.check(seed=1) == 0
        b.free()  # the owner frees it; rank0 never hears about it
        # ... placements need rank0 and fail fast instead of hanging
        t0 = time.time()
        with pytest.raises(api.OcmError):
            c.alloc(api.OCM_REMOTE_RDMA, local_bytes=4096, remote_bytes=MiB)
        assert time.time() - t0 < 5

        m.restart(0)  # returns once every survivor rejoined
        assert "resuming directory" in m.daemons[0].log()
        # b's 2 MiB were returned while rank0 was away, a's 4 MiB are still held:
        # exactly 4 MiB fit on owner 2 now.
        d = c.alloc(api.OCM_REMOTE_RDMA, local_bytes=4 * MiB, remote_bytes=4 * MiB)
        assert d.remote_info()["extents"][0]["owner_rank"] == 2
        e = c.alloc(api.OCM_REMOTE_RDMA, local_bytes=MiB, remote_bytes=MiB)
        assert e.remote_info()["extents"][0]["owner_rank"] != 2  # owner 2 is full (a + d)
        # ids continue after the checkpointed ones: no collision in the owners' tables
        assert d.remote_info()["alloc_id"] > a.remote_info()["alloc_id"]
        d.fill(seed=5)
        d.put(0, 0, 4 * MiB)
        a.free()
        d.fill(seed=0)
        d.get(0, 0, 4 * MiB)
        assert d.check(seed=5) == 0
        d.free()
        e.free()
        assert c.stats(2)["host_used"] == 0


def test_owner_restart_after_rank0_restart_drops_its_entries(mesh_factory, tmp_path):
    # An owner that comes back as a NEW process lost its memory: the resumed
    # directory must forget those extents instead of counting them as used.
    state = str(tmp_path / "directory.ckpt")
    m = mesh_factory(3, rank_env={0: {"OCM_STATE_FILE": state}}, extra_args=["--host-capacity", str(8 * MiB)])
    with api.Client(daemon_rank=1, ns=m.ns) as c:
        a = c.alloc(api.OCM_REMOTE_RDMA, local_bytes=4096, remote_bytes=6 * MiB)
        assert a.remote_info()["extents"][0]["owner_rank"] == 2
        assert _wait(lambda: os.path.exists(state) and f"entry {a.remote_info()['alloc_id']} " in open(state).read())
        m.kill(0, signal.SIGKILL)
        m.kill(2, signal.SIGKILL)
        m.daemons[2] = m._spawn(2)  # a new process; it waits for rank0 to come back
        m.restart(0)
        m._wait_ready([m.daemons[2]], 30)
        assert "dropped 1 allocations" in m.daemons[0].log()
        big = c.alloc(api.OCM_REMOTE_RDMA, local_bytes=4096, remote_bytes=6 * MiB)
        assert big.remote_info()["extents"][0]["owner_rank"] == 2  # the stale 6 MiB are not counted
        big.free()

"""BASELINE.json configs #4 and #5 on a real MI355X (CPU versions live in
test_mesh_cpu.py): HBM exhaustion spilling to the pinned host tier, and
8 concurrent GPU clients churning on a daemon mesh while one crashes."""
import os
import signal
import subprocess
import sys
import textwrap
import time

import pytest

from oncilla_amd import api

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MiB = 1 << 20


def test_hbm_exhaustion_spills_to_pinned_host(mesh_factory):
    # config #4: the owner may hand out 256 MiB of HBM; later chunks land in the host tier.
    m = mesh_factory(2, gpus=[0, 0], extra_args=["--gpu-capacity", str(256 * MiB)])
    with api.Client(daemon_rank=0, gpu=0, ns=m.ns) as c:
        chunk = 64 * MiB
        allocs = []
        for i in range(8):
            a = c.alloc(api.OCM_REMOTE_GPU, local_bytes=chunk, remote_bytes=chunk)
            allocs.append(a)
        tiers = [a.remote_info()["extents"][0]["tier"] for a in allocs]
        owners = [a.remote_info()["extents"][0]["owner_rank"] for a in allocs]
        # ring owner = rank 1: its 256 MiB of HBM take 4 chunks, the rest spill to its pinned host tier
        assert tiers == [api.OCM_TIER_GPU] * 4 + [api.OCM_TIER_HOST] * 4, (tiers, owners)
        assert owners == [1] * 8 and c.stats(1)["gpu_used"] == 256 * MiB
        for i, a in enumerate(allocs):
            a.fill(seed=60 + i)
            a.put(0, 0, chunk)
        for i, a in enumerate(allocs):
            a.fill(seed=0)
            a.get(0, 0, chunk)
            assert a.check(seed=60 + i) == 0, (i, tiers[i])
        assert c.stats(0)["n_spilled"] == 4  # rank0 reports the directory's count
        # NO_SPILL: HBM or nothing
        with pytest.raises(api.OcmError):
            c.alloc(api.OCM_REMOTE_GPU, local_bytes=4096, remote_bytes=chunk, flags=api.OCM_ALLOC_NO_SPILL)
        for a in allocs:
            a.free()
        assert c.stats(1)["gpu_used"] == 0 and c.stats(1)["host_used"] == 0


CLIENT = textwrap.dedent("""
    import os, signal, sys
    sys.path.insert(0, {repo!r})
    from oncilla_amd import api
    from oncilla_amd.models import workloads as wl
    r = int(sys.argv[1])
    with api.Client(daemon_rank=r % 4, gpu=0, ns={ns!r}) as c:
        if r == 7:  # the crasher: hold HBM on peers, then die without ocm_tini
            keep = [c.alloc(api.OCM_REMOTE_GPU, local_bytes=4096, remote_bytes=8 << 20) for _ in range(4)]
            print("crashing", flush=True)
            os.kill(os.getpid(), signal.SIGKILL)
        print(wl.churn(c, 40, api.OCM_REMOTE_GPU, 1 << 20, 1 << 20, seed=r), flush=True)
""")


def test_concurrent_gpu_clients_churn_and_crash(mesh_factory):
    # config #5: 8 app processes (GPU 0) on a 4-daemon mesh; client 7 crashes mid-run.
    m = mesh_factory(4, gpus=[0, 0, 0, 0], env={"OCM_LEASE_IDLE_MS": "100"})  # leases go back once idle
    code = CLIENT.format(repo=REPO, ns=m.ns)
    procs = [subprocess.Popen([sys.executable, "-c", code, str(i)], stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                              text=True) for i in range(8)]
    for i, p in enumerate(procs):
        out, err = p.communicate(timeout=300)
        if i == 7:
            assert p.returncode == -signal.SIGKILL and "crashing" in out, err
        else:
            assert p.returncode == 0 and "allocs" in out, err[-3000:] + m.logs()[-3000:]
    with api.Client(daemon_rank=0, gpu=0, ns=m.ns) as c:
        deadline = time.time() + 10
        while time.time() < deadline and any(c.stats(r)["gpu_used"] for r in range(4)):
            time.sleep(0.05)
        assert [c.stats(r)["gpu_used"] for r in range(4)] == [0, 0, 0, 0]
        assert c.stats(3)["n_reclaimed"] >= 4  # client 7 was attached to daemon 3

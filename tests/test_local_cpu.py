"""Config #1: one CPU-only daemon, loopback mailbox, malloc-backed local kinds.
Runs the reference-equivalent ocm_test 1-4 (reference test/ocm_test.c) and the
Python API against it."""
import os

import pytest

from oncilla_amd import api
from oncilla_amd.models import workloads as wl


@pytest.fixture
def one(mesh_factory):
    return mesh_factory(1)


@pytest.mark.parametrize("sub", [1, 3, 4, 5])
def test_ocm_test_alloc(one, tool, native, sub):
    rc, out = tool([f"{native}/ocm_test", "1", "1", "2", str(sub)], env=one.client_env(0))
    assert rc == 0, out + one.logs()
    assert "pass: test 1" in out


def test_ocm_test_alloc_gpu_kind_fails_without_gpu(one, tool, native):
    rc, out = tool([f"{native}/ocm_test", "1", "1", "2", "2"], env=dict(one.client_env(0), OCM_NO_GPU="1"))
    assert rc != 0 and "no GPU" in out


def test_ocm_test_onesided(one, tool, native):
    rc, out = tool([f"{native}/ocm_test", "2", "4", "4"], env=one.client_env(0))
    assert rc == 0, out + one.logs()


def test_ocm_test_twosided(one, tool, native):
    rc, out = tool([f"{native}/ocm_test", "3", "2", "4"], env=one.client_env(0))
    assert rc == 0, out + one.logs()


def test_ocm_test_bw_sweep(one, tool, native):
    rc, out = tool([f"{native}/ocm_test", "4", "0", "2", "8"], env=one.client_env(0))
    assert rc == 0, out + one.logs()
    assert out.count("GiB/s") == 2 * 18  # 64 B .. 8 MiB, read and write


def test_python_api_local(one, monkeypatch):
    monkeypatch.setenv("OCM_NO_GPU", "1")
    with api.Client(daemon_rank=0, ns=one.ns) as c:
        assert c.num_nodes == 1 and c.rank == 0 and c.device == -1
        h = c.alloc(api.OCM_LOCAL_HOST, local_bytes=1 << 20)
        assert not h.is_remote() and h.local_bytes == 1 << 20
        with pytest.raises(api.OcmError):
            h.remote_size()
        h.free()
        # remote pair on a single node lands in the host tier of the only daemon
        r = c.alloc(api.OCM_REMOTE_RDMA, local_bytes=1 << 20, remote_bytes=3 << 20)
        info = r.remote_info()
        assert info["extents"][0]["tier"] == api.OCM_TIER_HOST and info["remote_bytes"] == 3 << 20
        r.fill(seed=3)
        r.put(0, 1 << 20, 1 << 20)
        r.fill(seed=0)
        r.get(0, 1 << 20, 1 << 20)
        assert r.check(seed=3) == 0
        with pytest.raises(api.OcmError):
            r.put(0, 3 << 20, 16)  # past the remote end
        st = c.stats()
        assert st["host_used"] >= 3 << 20 and st["num_apps"] == 1
        r.free()
        assert c.stats()["host_used"] == 0


def test_alloc_latency_local(one, monkeypatch):
    monkeypatch.setenv("OCM_NO_GPU", "1")
    with api.Client(daemon_rank=0, ns=one.ns) as c:
        lat = wl.alloc_latency(c, api.OCM_LOCAL_HOST, 100, local_bytes=4096)
        # the reference's derived floor is ~0.5 ms (two 500 us mailbox polls)
        assert lat["alloc_p50_us"] < 500


def test_daemon_rejects_unknown_app_and_bad_requests(one, monkeypatch):
    monkeypatch.setenv("OCM_NO_GPU", "1")
    with api.Client(daemon_rank=0, ns=one.ns) as c:
        with pytest.raises(api.OcmError):
            c.alloc(api.OCM_REMOTE_RDMA, local_bytes=4096, remote_bytes=0)
        with pytest.raises(api.OcmError):
            c.alloc(99, local_bytes=4096)
        with pytest.raises(api.OcmError):
            c.alloc(api.OCM_REMOTE_RDMA, local_bytes=4096, remote_bytes=1 << 50)  # exceeds every tier


def test_tensor_views_cpu(one, monkeypatch):
    import torch

    monkeypatch.setenv("OCM_NO_GPU", "1")
    with api.Client(daemon_rank=0, ns=one.ns) as c:
        a = c.alloc(api.OCM_REMOTE_RDMA, local_bytes=4096, remote_bytes=4096)
        loc = a.local_tensor(torch.int32)
        loc.copy_(torch.arange(1024, dtype=torch.int32))
        a.put(0, 0, 4096)
        rem = a.remote_tensor(torch.int32)
        assert torch.equal(rem, torch.arange(1024, dtype=torch.int32))
        rem.add_(5)
        a.get(0, 0, 4096)
        assert int(loc[10]) == 15
        a.free()


def test_reference_style_daemon_launch(tmp_path, native, tool):
    """`oncillamem <nodefile>` exactly as the reference starts it (src/main.c:187-224):
    a 5-column nodefile with no GPU column and no --rank; the rank is the line
    whose dns column matches gethostname() (src/nodefile.c:92-103). Then the
    reference's ocm_test 1 (host kind) runs against it."""
    import socket
    import subprocess
    import time

    from oncilla_amd.parallel.mesh import free_ports

    port = free_ports(1)[0]
    nf = tmp_path / "nodefile"
    nf.write_text(f"#rank dns ethernet_ip ocm_port rdmacm_port\n0 {socket.gethostname()} 127.0.0.1 {port} 0\n")
    ns = f"refstyle{port}"
    env = dict(os.environ, OCM_NS=ns, OCM_NO_GPU="1")
    env.pop("OCM_RANK", None)
    env.pop("LOCAL_RANK", None)
    ready = tmp_path / "ready.json"
    d = subprocess.Popen([f"{native}/oncillamem", str(nf), "--gpu", "none", "--ready-file", str(ready),
                          "--watch-pid", str(os.getpid())], env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)
    try:
        deadline = time.time() + 20
        while not ready.exists() and time.time() < deadline and d.poll() is None:
            time.sleep(0.05)
        assert ready.exists(), d.stdout.read().decode() if d.poll() is not None else "daemon not ready"
        rc, out = tool([f"{native}/ocm_test", "1", "1", "2", "3"], env=dict(env, OCM_DAEMON_RANK="0"))
        assert rc == 0 and "completed successfully" in out, out
    finally:
        d.terminate()
        d.wait(timeout=10)


def test_mesh_on_open_address_needs_a_key(tmp_path, native):
    """A multi-daemon mesh whose port binds a non-loopback address refuses to start
    without OCM_MESH_KEY (its HELLO token would be a guessable constant), unless the
    operator opts out with OCM_MESH_INSECURE=1."""
    import subprocess

    from oncilla_amd.parallel.mesh import free_ports, write_nodefile

    ports = free_ports(2)
    nf = write_nodefile(str(tmp_path / "nodefile"), ports)
    env = dict(os.environ, OCM_NS=f"keyless{ports[0]}", OCM_NO_GPU="1")
    env.pop("OCM_MESH_KEY", None)
    env.pop("OCM_MESH_INSECURE", None)
    r = subprocess.run([f"{native}/ocmd", nf, "--rank", "1", "--gpu", "none", "--bind", "0.0.0.0"], env=env,
                       capture_output=True, text=True, timeout=30)
    assert r.returncode != 0 and "OCM_MESH_KEY" in (r.stdout + r.stderr)


def test_prometheus_metrics_exporter(mesh_factory, monkeypatch):
    """`python -m oncilla_amd metrics`: every daemon's counters as Prometheus gauges."""
    import threading
    import urllib.request

    from oncilla_amd import api
    from oncilla_amd.utils.metrics import serve

    monkeypatch.setenv("OCM_NO_GPU", "1")
    m = mesh_factory(3)
    ready, stop = threading.Event(), threading.Event()
    th = threading.Thread(target=serve, args=(m.ns, 0, 1, ready, stop), daemon=True)
    th.start()
    assert ready.wait(30)
    try:
        text = urllib.request.urlopen(f"http://127.0.0.1:{ready.port}/metrics", timeout=10).read().decode()
    finally:
        stop.set()
        th.join(10)
    for r in range(3):
        assert f'oncilla_up{{rank="{r}"}} 1' in text
        assert f'oncilla_host_capacity{{rank="{r}",gpu="-1"}}' in text
    assert "# TYPE oncilla_n_alloc gauge" in text
    assert 'oncilla_tick_own_records{rank="1"} 0' in text  # TCP mesh: no tick transport


def test_shared_memory_link_carries_the_rpcs_and_survives_idle_daemons(mesh_factory, monkeypatch):
    """The app's shared-memory link (ocm/shmlink.h) carries the RPCs; when the
    daemon has gone to sleep between requests the app wakes it over the socket,
    and when the app sleeps the daemon wakes it. Every round trip completes, with
    and without the link (OCM_SHM_LINK=0: the mailbox alone)."""
    import time

    monkeypatch.setenv("OCM_NO_GPU", "1")
    for link in ("1", "0"):
        monkeypatch.setenv("OCM_SHM_LINK", link)
        m = mesh_factory(2)
        with api.Client(daemon_rank=0, ns=m.ns) as c:
            before = api.counters()
            for i in range(40):
                a = c.alloc(api.OCM_REMOTE_RDMA, local_bytes=4096, remote_bytes=1 << 20)
                a.free()
                if i % 4 == 3:
                    time.sleep(0.002)  # past the daemon's 50 us spin: the next request must wake it
            after = api.counters()
            if link == "1":
                assert after["n_link_rpc"] - before["n_link_rpc"] >= 80
                assert after["n_link_wake"] - before["n_link_wake"] >= 10
            else:
                assert after["n_link_rpc"] == before["n_link_rpc"]


def test_threads_of_one_app_share_its_link(mesh_factory, monkeypatch):
    """Many threads of one app allocate and free at once: the library serializes
    its RPCs, so the link's single-producer rings stay single-producer, and every
    reply reaches the thread that asked (ctypes drops the GIL in the calls)."""
    from concurrent.futures import ThreadPoolExecutor

    monkeypatch.setenv("OCM_NO_GPU", "1")
    m = mesh_factory(2)
    with api.Client(daemon_rank=0, ns=m.ns) as c:
        before = api.counters()

        def work(t):
            for i in range(60):
                kind = api.OCM_REMOTE_RDMA if (t + i) % 2 else api.OCM_LOCAL_HOST
                a = c.alloc(kind, local_bytes=4096 * (1 + t), remote_bytes=(1 << 16) * (1 + i % 3))
                assert a.localbuf()[1] == 4096 * (1 + t)
                a.free()
            return t

        with ThreadPoolExecutor(8) as ex:
            assert sorted(ex.map(work, range(8))) == list(range(8))
        after = api.counters()
        assert after["n_link_rpc"] - before["n_link_rpc"] >= 8 * 60 * 2
        assert c.stats(0)["ctrl"] == "tcp"


def test_daemons_shut_down_in_order_on_sigterm(mesh_factory, monkeypatch):
    """SIGTERM reaches the event loop's signalfd (blocked before the HIP runtime
    starts any thread), so a daemon leaves through its shutdown path and exits 0
    instead of being killed by the signal's default action in some runtime thread."""
    monkeypatch.setenv("OCM_NO_GPU", "1")
    m = mesh_factory(2)
    with api.Client(daemon_rank=1, ns=m.ns) as c:
        c.alloc(api.OCM_REMOTE_RDMA, local_bytes=4096, remote_bytes=1 << 20).free()
    m.stop()
    assert [d.proc.returncode for d in m.daemons] == [0, 0]
    logs = m.logs()
    assert logs.count("shutting down") == 2 and logs.count("exiting (allocs") == 2


def test_app_falls_back_to_the_socket_when_the_daemon_declines_its_link(mesh_factory, monkeypatch):
    """A daemon that takes no links (OCM_SHM_LINK_ACCEPT=0, or one that found the
    offered memfd unusable) answers CONNECT on the socket; the app sees that and
    keeps every later request on the socket instead of waiting on a dead ring."""
    monkeypatch.setenv("OCM_NO_GPU", "1")
    m = mesh_factory(2, env={"OCM_SHM_LINK_ACCEPT": "0"})
    with api.Client(daemon_rank=0, ns=m.ns) as c:
        before = api.counters()["n_link_rpc"]
        for _ in range(20):
            c.alloc(api.OCM_REMOTE_RDMA, local_bytes=4096, remote_bytes=1 << 20).free()
        assert api.counters()["n_link_rpc"] == before


def test_connect_retries_while_the_mesh_joins_keep_the_link_in_step(monkeypatch, tmp_path):
    """An app that connects before its daemon's mesh is complete is told EAGAIN and
    CONNECTs again; each attempt offers a fresh link (the daemon attaches every offer
    with its counts at zero), so the app's requests after the join still ride the link."""
    import threading
    import time

    import uuid

    from oncilla_amd.parallel.mesh import Mesh, free_ports

    monkeypatch.setenv("OCM_NO_GPU", "1")
    ns, ports, key = f"m{uuid.uuid4().hex[:10]}", free_ports(2), "k" * 32
    (tmp_path / "a").mkdir()
    (tmp_path / "b").mkdir()
    m0 = Mesh(2, ns=ns, ports=ports, ranks=[0], key=key, workdir=str(tmp_path / "a"))
    m1 = Mesh(2, ns=ns, ports=ports, ranks=[1], key=key, workdir=str(tmp_path / "b"))
    errs = []
    starter = threading.Thread(target=lambda: m0.start(timeout=60))
    starter.start()
    try:
        time.sleep(0.3)
        box = {}

        def connect():
            try:
                box["c"] = api.Client(daemon_rank=0, ns=ns).__enter__()
            except Exception as e:  # noqa: BLE001 - reported below
                errs.append(e)

        t = threading.Thread(target=connect)
        t.start()
        time.sleep(1.0)  # the app keeps getting EAGAIN: rank 1 is not up yet
        m1.start(timeout=60)
        t.join(30)
        starter.join(30)
        assert not errs and "c" in box, errs
        c = box["c"]
        before = api.counters()["n_link_rpc"]
        for _ in range(10):
            c.alloc(api.OCM_REMOTE_RDMA, local_bytes=4096, remote_bytes=1 << 20).free()
        assert api.counters()["n_link_rpc"] - before >= 20
        # every retried CONNECT replaced the app's entry without closing
        # its pidfd; the daemon must hold exactly one pidfd for this app
        pid0 = m0.daemons[0].proc.pid
        pidfds = 0
        for fd in os.listdir(f"/proc/{pid0}/fd"):
            try:
                if "pidfd" in os.readlink(f"/proc/{pid0}/fd/{fd}"):
                    with open(f"/proc/{pid0}/fdinfo/{fd}") as f:
                        pidfds += f"Pid:\t{os.getpid()}\n" in f.read()
            except OSError:
                pass
        # one for the app, one for --watch-pid (Mesh makes its daemons watch this process);
        # the old code held one more per retried CONNECT (52 here)
        assert pidfds == 2, f"ocmd rank 0 holds {pidfds} pidfds on this process"
        c.__exit__(None, None, None)
    finally:
        m1.stop()
        m0.stop()


def test_selftest_cli_cpu(monkeypatch):
    """`python -m oncilla_amd selftest`: a temporary mesh, one verified round trip per
    owner daemon, exit code 0, and the JSON report's fields."""
    import json
    import subprocess
    import sys

    env = dict(os.environ, OCM_NO_GPU="1")
    r = subprocess.run([sys.executable, "-m", "oncilla_amd", "selftest", "--daemons", "3", "--bytes", str(1 << 20),
                        "--json"], capture_output=True, text=True, timeout=120, env=env,
                       cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    assert r.returncode == 0, r.stdout + r.stderr
    rep = json.loads(r.stdout.strip().splitlines()[-1])
    assert rep["ok"] and rep["daemons"] == 3 and sorted(rep["peers"]) == ["1", "2"]
    assert all(p["ok"] and p["bad_words"] == 0 for p in rep["peers"].values())
    assert rep["xgmi"] is False and rep["ctrl"] == "tcp"

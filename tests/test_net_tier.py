"""Network tier: remote memory on another node.

Daemons started with different host aliases (OCM_HOST_ALIAS) behave as if on
different nodes: the governor keeps placements on the origin's host when it has
peers there, places on the next node otherwise (or when the app names a remote
rank explicitly), and such extents are reached through the owner's data
server (PUT/GET records over TCP) instead of an IPC/memfd mapping.

Parity: reference src/rdma.c / src/extoll.c one-sided verbs to another host;
the reference's test 3/4 (cross-node RDMA/RMA) — SURVEY §4.
"""
import pytest

from oncilla_amd import api


@pytest.fixture(autouse=True)
def _cpu_app(monkeypatch):
    monkeypatch.setenv("OCM_NO_GPU", "1")


def hosts(*names):
    return {r: {"OCM_HOST_ALIAS": h} for r, h in enumerate(names)}


def test_two_nodes_remote_is_network(mesh_factory):
    m = mesh_factory(2, rank_env=hosts("nodeA", "nodeB"))
    with api.Client(daemon_rank=0, ns=m.ns) as c:
        a = c.alloc(api.OCM_REMOTE_RDMA, local_bytes=8 << 20, remote_bytes=8 << 20)
        ext = a.remote_info()["extents"]
        assert len(ext) == 1 and ext[0]["owner_rank"] == 1 and ext[0]["net"]
        a.fill(seed=7)
        a.put(0, 0, 8 << 20)
        a.fill(seed=0)
        a.get(0, 0, 8 << 20)
        assert a.check(seed=7) == 0
        # unaligned pieces through the same connection
        a.fill(seed=9)
        a.put(124, 4567, 1 << 20)
        a.fill(seed=0)
        a.get(124, 4567, 1 << 20)
        assert a.check(seed=9, offset=124, nbytes=1 << 20) == 0
        assert c.stats(1)["host_used"] >= 8 << 20
        a.free()
        assert c.stats(1)["host_used"] == 0


def test_data_ports_from_the_nodefile(mesh_factory):
    """The nodefile's 5th column (the reference's rdmacm port) fixes each data
    server's port, as a firewalled cluster needs; handles carry it."""
    from oncilla_amd.parallel.mesh import free_ports

    dports = free_ports(2)
    m = mesh_factory(2, rank_env=hosts("nodeA", "nodeB"), data_ports=dports)
    assert [r["data_port"] for r in m.ready_info()] == dports
    with api.Client(daemon_rank=0, ns=m.ns) as c:
        a = c.alloc(api.OCM_REMOTE_RDMA, local_bytes=1 << 20, remote_bytes=1 << 20)
        assert a.remote_info()["extents"][0]["net"]
        assert f":{dports[1]}:" in a.extent_handle(0).decode()
        a.fill(seed=5)
        a.put(0, 0, 1 << 20)
        a.fill(seed=0)
        a.get(0, 0, 1 << 20)
        assert a.check(seed=5) == 0
        a.free()


def test_same_host_preferred_over_network(mesh_factory):
    m = mesh_factory(4, rank_env=hosts("nodeA", "nodeA", "nodeB", "nodeB"))
    with api.Client(daemon_rank=2, ns=m.ns) as c:
        a = c.alloc(api.OCM_REMOTE_RDMA, local_bytes=1 << 20, remote_bytes=1 << 20)
        ext = a.remote_info()["extents"][0]
        assert ext["owner_rank"] == 3 and not ext["net"]
        # an explicit cross-node owner is honoured and goes over the network
        b = c.alloc(api.OCM_REMOTE_RDMA, local_bytes=1 << 20, remote_bytes=1 << 20, remote_rank=0)
        ext = b.remote_info()["extents"][0]
        assert ext["owner_rank"] == 0 and ext["net"]
        b.fill(seed=3)
        b.put(0, 0, 1 << 20)
        # remote -> remote copy between a same-node and a cross-node allocation
        api.copy(a, b, 1 << 20)  # remote -> remote: network source, same-node destination
        a.fill(seed=0)
        a.get(0, 0, 1 << 20)
        assert a.check(seed=3) == 0
        a.free()
        b.free()


def test_ocm_test_suite_across_nodes(mesh_factory, tool, native):
    m = mesh_factory(2, rank_env=hosts("nodeA", "nodeB"))
    for args in (["1", "1", "2", "3"], ["1", "1", "2", "4"], ["2", "4", "8"], ["3", "4", "4"], ["4", "1", "2", "4"]):
        rc, out = tool([f"{native}/ocm_test", *args], env=dict(m.client_env(0), OCM_NO_GPU="1"))
        assert rc == 0, out


def test_owner_loss_fails_network_ops(mesh_factory):
    m = mesh_factory(2, rank_env=hosts("nodeA", "nodeB"))
    with api.Client(daemon_rank=0, ns=m.ns) as c:
        a = c.alloc(api.OCM_REMOTE_RDMA, local_bytes=1 << 20, remote_bytes=1 << 20)
        a.put(0, 0, 4096)
        m.kill(1)
        with pytest.raises(api.OcmError):
            for _ in range(50):  # the first op may still drain into the socket buffer
                a.put(0, 0, 1 << 20)
                a.get(0, 0, 1 << 20)


@pytest.mark.parametrize("streams", ["1", "3"])
def test_parallel_streams_odd_split(mesh_factory, monkeypatch, streams):
    """Large network-tier ops are cut into parts on parallel connections
    (OCM_NET_STREAMS); odd sizes and offsets must land byte-exact."""
    monkeypatch.setenv("OCM_NET_STREAMS", streams)
    monkeypatch.setenv("OCM_NET_SPLIT_MIN", str(1 << 20))
    m = mesh_factory(2, rank_env=hosts("nodeA", "nodeB"))
    with api.Client(daemon_rank=0, ns=m.ns) as c:
        n = 16 << 20
        a = c.alloc(api.OCM_REMOTE_RDMA, local_bytes=n, remote_bytes=n)
        assert a.remote_info()["extents"][0]["net"]
        for i, (size, loff, roff) in enumerate([((5 << 20) + 123, 4, 4096 + 7), (n - 8, 0, 8), (3 << 20, 12, 0)]):
            a.fill(seed=50 + i)
            a.put(loff, roff, size)
            a.fill(seed=0)
            a.get(loff, roff, size)
            assert a.check(seed=50 + i, offset=loff, nbytes=size - size % 4, first_word=loff // 4) == 0, size
        a.free()


# ---- data-server capabilities (per-extent grants) ----

def _net_endpoint(handle: bytes):
    """'net:<ip>:<port>:<conn token>:<grant>' -> (ip, port, token, grant)."""
    tag, ip, port, tok, grant = handle.rstrip(b"\0").decode().split(":")
    assert tag == "net"
    return ip, int(port), int(tok, 16), int(grant, 16)


def _raw_conn(ip, port, tok):
    import socket
    import struct

    s = socket.create_connection((ip, port), timeout=20)
    s.sendall(struct.pack("<Q", tok))
    return s


def _recv_exact(s, n):
    buf = bytearray()
    while len(buf) < n:
        chunk = s.recv(min(n - len(buf), 1 << 20))
        assert chunk, "data server closed the connection"
        buf += chunk
    return bytes(buf)


def _raw_get_header(s, grant, off, n):
    import struct

    s.sendall(struct.pack("<IIQQQ", 0x4F434E44, 2, grant, off, n))
    magic, err, ln = struct.unpack("<IiQ", _recv_exact(s, 16))
    assert magic == 0x4F434E44
    return err, ln


def test_net_grant_bounds_each_request_by_its_extent(mesh_factory):
    """A request names its extent's grant and stays inside that extent: the
    slab around it, other extents and forged grants are refused (ADVICE r1:
    one token used to open every allocation on the owner)."""
    import ctypes
    import errno

    m = mesh_factory(2, rank_env=hosts("nodeA", "nodeB"))
    with api.Client(daemon_rank=0, ns=m.ns) as c:
        n = 1 << 20
        a = c.alloc(api.OCM_REMOTE_RDMA, local_bytes=n, remote_bytes=n)
        b = c.alloc(api.OCM_REMOTE_RDMA, local_bytes=n, remote_bytes=n)
        a.fill(seed=11)
        a.put(0, 0, n)
        ip, port, tok, ga = _net_endpoint(a.extent_handle(0))
        gb = _net_endpoint(b.extent_handle(0))[3]
        assert ga != gb and ga and gb
        s = _raw_conn(ip, port, tok)
        try:
            err, ln = _raw_get_header(s, ga, 4096, 8192)
            assert err == 0 and ln == 8192
            assert _recv_exact(s, 8192) == ctypes.string_at(a.local_ptr + 4096, 8192)
            assert _raw_get_header(s, ga, n - 8, 16)[0] == errno.EFAULT  # runs past the extent
            assert _raw_get_header(s, ga, 0, n + 1)[0] == errno.EFAULT
            assert _raw_get_header(s, ga ^ (1 << 17), 0, 8)[0] == errno.EACCES  # forged grant
            b.free()
            assert _raw_get_header(s, gb, 0, 8)[0] == errno.EACCES  # revoked at free
        finally:
            s.close()
        a.free()


def test_net_free_during_inflight_get_defers_release(mesh_factory):
    """Freeing an extent while a data-server GET still streams it must not pull
    the memory from under the copy: the last request releases it."""
    import ctypes
    import errno
    import time

    m = mesh_factory(2, rank_env=hosts("nodeA", "nodeB"))
    with api.Client(daemon_rank=0, ns=m.ns) as c:
        n = 32 << 20
        a = c.alloc(api.OCM_REMOTE_RDMA, local_bytes=n, remote_bytes=n)
        a.fill(seed=21)
        a.put(0, 0, n)
        want = ctypes.string_at(a.local_ptr, n)
        ip, port, tok, g = _net_endpoint(a.extent_handle(0))
        s = _raw_conn(ip, port, tok)
        try:
            err, ln = _raw_get_header(s, g, 0, n)
            assert err == 0 and ln == n
            head = _recv_exact(s, 1 << 20)  # the server is now blocked sending the rest
            a.free()
            time.sleep(0.2)
            assert c.stats(1)["host_used"] >= n  # still held by the in-flight GET
            got = head + _recv_exact(s, n - len(head))
            assert got == want
            deadline = time.time() + 10
            while c.stats(1)["host_used"] and time.time() < deadline:
                time.sleep(0.02)
            assert c.stats(1)["host_used"] == 0  # released by the request that finished
            assert _raw_get_header(s, g, 0, 8)[0] == errno.EACCES
        finally:
            s.close()

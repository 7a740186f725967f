"""Daemon robustness against malformed / adversarial mailbox traffic.

Any local process can reach a daemon's mailbox, so records are untrusted:
random bytes, wrong sizes, requests before CONNECT, absurd sizes (2^63), bad
stripe units, out-of-range ranks, unknown kinds. After the storm the daemons
must still be alive and serving; whatever the fuzzer got allocated must be
reclaimed when its connection closes, and other users must be refused.
"""
import os
import random
import socket
import struct
import subprocess
import sys
import textwrap
import time

import pytest

from oncilla_amd import api

MSG = struct.Struct("<IIiiQii128s")  # type, status, pid, rank, seq, src_rank, err, union
REQ = struct.Struct("<iiQIIIIQQii")   # orig, remote_rank, bytes, kind, flags, width, tier, unit, alloc_id, pid, n_ext
SHUTDOWN = 17  # MSG_SHUTDOWN: a legitimate same-user operation, not fuzzed


@pytest.fixture(autouse=True)
def _cpu_app(monkeypatch):
    monkeypatch.setenv("OCM_NO_GPU", "1")


def _connect(ns, rank=0):
    s = socket.socket(socket.AF_UNIX, socket.SOCK_SEQPACKET)
    s.connect(b"\0" + f"ocm_{ns}_d{rank}".encode())
    s.setblocking(False)  # (a socket timeout would make every recv wait it out)
    return s


def _req(rng, kind=None):
    big = rng.choice([0, 1, 4096, 1 << 20, (1 << 63) + 5, (1 << 64) - 1, rng.getrandbits(64)])
    return REQ.pack(rng.randint(-5, 9), rng.choice([-1, -7, 0, 1, 2, 1 << 30]), big,
                    kind if kind is not None else rng.randint(0, 9), rng.getrandbits(32), rng.choice([0, 1, 3, 9, 1 << 31]),
                    rng.randint(0, 5), rng.choice([0, 3, 16, 4096, 1 << 20, rng.getrandbits(64)]), rng.getrandbits(64),
                    rng.randint(-3, 1 << 30), rng.randint(-2, 1 << 16)).ljust(128, b"\0")


def _storm(ns, seed, n=3000):
    rng = random.Random(seed)
    s = _connect(ns)
    for i in range(n):
        r = rng.random()
        if r < 0.1:
            payload = os.urandom(rng.choice([1, 10, 159, 161, 300]))  # wrong sizes
        elif r < 0.3:
            payload = os.urandom(160)
        else:
            t = rng.choice([1, 2, 3, 5, 7, 9, 15, 16, 18, 19, 20, 0, 99, 1 << 31])
            if t == SHUTDOWN:
                continue
            payload = MSG.pack(t, rng.randint(0, 3), rng.randint(-5, 1 << 30), rng.randint(-3, 9), rng.getrandbits(64),
                               rng.randint(-3, 9), rng.randint(-3, 200), _req(rng))
        for _ in range(200):
            try:
                s.send(payload)
                break
            except BlockingIOError:
                time.sleep(0.001)  # daemon busy: its receive queue is full
            except OSError:
                s.close()
                s = _connect(ns)  # the daemon dropped us: come back
                break
        try:
            while s.recv(4096):  # drain replies
                pass
        except OSError:
            pass
    s.close()


def test_mailbox_fuzz_daemons_survive(mesh_factory):
    m = mesh_factory(3, extra_args=["--host-capacity", str(64 << 20)])
    for seed in range(3):
        _storm(m.ns, seed)
    time.sleep(0.3)
    assert all(d.alive() for d in m.daemons), m.logs()[-4000:]
    with api.Client(daemon_rank=0, ns=m.ns) as c:
        # the fuzzer's connections are gone: anything it obtained was reclaimed
        deadline = time.time() + 10
        while time.time() < deadline and any(c.stats(r)["host_used"] for r in range(3)):
            time.sleep(0.05)
        assert [c.stats(r)["host_used"] for r in range(3)] == [0, 0, 0], m.logs()[-4000:]
        a = c.alloc(api.OCM_REMOTE_RDMA, local_bytes=1 << 20, remote_bytes=1 << 20)
        a.fill(seed=5)
        a.put(0, 0, 1 << 20)
        a.fill(seed=0)
        a.get(0, 0, 1 << 20)
        assert a.check(seed=5) == 0
        a.free()
        # absurd sizes are refused, not wrapped around
        with pytest.raises(api.OcmError):
            c.alloc(api.OCM_REMOTE_RDMA, local_bytes=4096, remote_bytes=(1 << 63) + 4096)
        with pytest.raises(api.OcmError):
            c.alloc(api.OCM_REMOTE_RDMA, local_bytes=4096, remote_bytes=1 << 20, stripe_unit=3000)


@pytest.mark.skipif(os.geteuid() != 0, reason="needs root to switch to another uid")
def test_other_users_are_refused(mesh_factory):
    m = mesh_factory(1)
    code = textwrap.dedent(f"""
        import os, socket, sys
        os.setgid(65534); os.setuid(65534)
        s = socket.socket(socket.AF_UNIX, socket.SOCK_SEQPACKET)
        s.connect(b"\\0ocm_{m.ns}_d0")
        s.settimeout(5)
        try:
            s.send(bytes(160))  # the daemon may already have closed it (EPIPE)
            data = s.recv(160)
        except OSError as e:
            data = b""
        print("closed" if data == b"" else "served")
    """)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=30)
    assert r.stdout.strip() == "closed", r.stdout + r.stderr
    assert "refusing mailbox connection" in m.logs()
    assert m.daemons[0].alive()


def test_mesh_port_rejects_strangers(mesh_factory):
    # The daemon<->daemon TCP port: without a HELLO carrying the mesh token
    # nothing is processed - not even SHUTDOWN.
    m = mesh_factory(2)
    port = m.ports[0]
    rng = random.Random(7)
    for attempt in range(3):
        s = socket.create_connection(("127.0.0.1", port), timeout=5)
        if attempt == 0:
            recs = [MSG.pack(SHUTDOWN, 1, 0, 0, 0, 1, 0, bytes(128))]
        elif attempt == 1:
            recs = [MSG.pack(12, 1, 0, 1, 0xBAD, 1, 0, bytes(128)), MSG.pack(SHUTDOWN, 1, 0, 0, 0, 1, 0, bytes(128))]
        else:
            recs = [os.urandom(160) for _ in range(50)]
        for r in recs:
            try:
                s.sendall(r)
            except OSError:
                break
        s.settimeout(5)
        try:
            assert s.recv(160) == b""  # dropped
        except ConnectionResetError:
            pass
        s.close()
    time.sleep(0.2)
    assert all(d.alive() for d in m.daemons), m.logs()[-3000:]
    assert "dropping unauthenticated mesh link" in m.logs()
    with api.Client(daemon_rank=1, ns=m.ns) as c:  # the real mesh still works
        a = c.alloc(api.OCM_REMOTE_RDMA, local_bytes=4096, remote_bytes=1 << 20)
        assert a.remote_info()["extents"][0]["owner_rank"] == 0
        a.free()


def _siphash24(k0, k1, data):
    """SipHash-2-4 (the daemon's HELLO MAC), for crafting HELLOs here."""
    M = (1 << 64) - 1
    rotl = lambda x, b: ((x << b) | (x >> (64 - b))) & M  # noqa: E731
    v = [k0 ^ 0x736F6D6570736575, k1 ^ 0x646F72616E646F6D, k0 ^ 0x6C7967656E657261, k1 ^ 0x7465646279746573]

    def rnd():
        v[0] = (v[0] + v[1]) & M; v[1] = rotl(v[1], 13) ^ v[0]; v[0] = rotl(v[0], 32)  # noqa: E702
        v[2] = (v[2] + v[3]) & M; v[3] = rotl(v[3], 16) ^ v[2]  # noqa: E702
        v[0] = (v[0] + v[3]) & M; v[3] = rotl(v[3], 21) ^ v[0]  # noqa: E702
        v[2] = (v[2] + v[1]) & M; v[1] = rotl(v[1], 17) ^ v[2]; v[2] = rotl(v[2], 32)  # noqa: E702

    def absorb(m):
        v[3] ^= m
        rnd()
        rnd()
        v[0] ^= m

    full = len(data) & ~7
    for i in range(0, full, 8):
        absorb(int.from_bytes(data[i:i + 8], "little"))
    absorb(((len(data) & 0xFF) << 56) | int.from_bytes(data[full:], "little"))
    v[2] ^= 0xFF
    for _ in range(4):
        rnd()
    return v[0] ^ v[1] ^ v[2] ^ v[3]


def test_siphash_reference_vectors():
    key = bytes(range(16))
    k0, k1 = int.from_bytes(key[:8], "little"), int.from_bytes(key[8:], "little")
    assert _siphash24(k0, k1, b"") == 0x726FDB47DD0E0E31
    assert _siphash24(k0, k1, bytes(range(15))) == 0xA129CA6149BE45E5


def _hello(ns, key, src, dst, ts_ms, nonce):
    mat = (ns + "\x1f" + key).encode()
    k0 = _siphash24(0x6F6E63696C6C6131, 0x6D6573682D6B6579, mat)
    k1 = _siphash24(0x6F6E63696C6C6132, 0x6D6573682D6B6579, mat)
    words = struct.pack("<QQQQ", (src & 0xFFFFFFFF) | ((dst & 0xFFFFFFFF) << 32), ts_ms, nonce, 11)
    mac = _siphash24(k0, k1, words)
    body = struct.pack("<iiQQQ", src, dst, ts_ms, nonce, mac).ljust(128, b"\0")
    return MSG.pack(11, 0, 0, src, 0, src, 0, body)  # MSG_HELLO


def test_mesh_hello_is_signed_fresh_and_single_use(mesh_factory):
    """A HELLO needs a MAC under the mesh key, our rank as its destination, a
    timestamp within the window and a nonce never seen before: a recorded HELLO
    replayed on a new connection is refused."""
    m = mesh_factory(2, env={"OCM_MESH_KEY": "k3y-for-the-test"})
    port = m.ports[0]
    now = int(time.time() * 1000)

    def attempt(rec):
        before = m.logs().count("dropping unauthenticated mesh link")
        s = socket.create_connection(("127.0.0.1", port), timeout=5)
        s.sendall(rec)
        time.sleep(0.3)
        s.close()
        time.sleep(0.1)
        return m.logs().count("dropping unauthenticated mesh link") > before  # True: refused

    assert attempt(_hello(m.ns, "wrong key", 1, 0, now, 1))
    assert attempt(_hello(m.ns, m.key, 1, 1, now, 2))                    # addressed to another rank
    assert attempt(_hello(m.ns, m.key, 1, 0, now - 3600 * 1000, 3))       # an hour old
    good = _hello(m.ns, m.key, 1, 0, now, 0x5EED)
    assert not attempt(good)                                               # accepted
    assert attempt(good)                                                   # the same bytes again: replay
    assert all(d.alive() for d in m.daemons), m.logs()[-3000:]


def test_data_server_requires_token(mesh_factory):
    m = mesh_factory(2, rank_env={0: {"OCM_HOST_ALIAS": "A"}, 1: {"OCM_HOST_ALIAS": "B"}})
    port = m.ready_info()[1]["data_port"]
    assert port > 0
    s = socket.create_connection(("127.0.0.1", port), timeout=5)
    get = struct.pack("<IIIIQQ", 0x4F434E44, 2, 1, 1, 0, 4096)  # a well-formed GET, but no token first
    s.sendall(get)
    try:
        assert s.recv(64) == b""
    except ConnectionResetError:
        pass
    s.close()
    # apps get the token with the handle from their own daemon: the network tier works
    with api.Client(daemon_rank=0, ns=m.ns) as c:
        a = c.alloc(api.OCM_REMOTE_RDMA, local_bytes=1 << 20, remote_bytes=1 << 20)
        assert a.remote_info()["extents"][0]["net"]
        a.fill(seed=3)
        a.put(0, 0, 1 << 20)
        a.fill(seed=0)
        a.get(0, 0, 1 << 20)
        assert a.check(seed=3) == 0
        a.free()


def test_data_server_reaps_connections(mesh_factory):
    # Short-lived connections (scanners, reconnecting apps) must not pile up threads.
    m = mesh_factory(2, rank_env={0: {"OCM_HOST_ALIAS": "A"}, 1: {"OCM_HOST_ALIAS": "B"}})
    port = m.ready_info()[1]["data_port"]
    pid = m.daemons[1].proc.pid

    def threads():
        for line in open(f"/proc/{pid}/status"):
            if line.startswith("Threads:"):
                return int(line.split()[1])

    base = threads()
    for _ in range(300):
        s = socket.create_connection(("127.0.0.1", port), timeout=5)
        s.sendall(b"\0" * 8)  # wrong token: the server drops it
        s.close()
    s = socket.create_connection(("127.0.0.1", port), timeout=5)  # one more accept triggers the reaping
    s.close()
    time.sleep(0.3)
    assert threads() <= base + 3, (base, threads())
    assert m.daemons[1].alive()


@pytest.mark.skipif(os.geteuid() != 0, reason="needs root to switch to another uid")
def test_other_users_get_no_slab_fds(mesh_factory, monkeypatch):
    """With OCM_ALLOW_ANY_UID=1 another user may attach, but MSG_SLAB_FD hands it a
    host-tier slab only if one of its own allocations lives there: a memfd opens
    the whole slab, i.e. other apps' data."""
    monkeypatch.setenv("OCM_NO_GPU", "1")
    m = mesh_factory(1, env={"OCM_ALLOW_ANY_UID": "1"})
    with api.Client(daemon_rank=0, ns=m.ns) as c:
        a = c.alloc(api.OCM_REMOTE_RDMA, local_bytes=1 << 20, remote_bytes=1 << 20)  # host tier: slab 1
        code = textwrap.dedent(f"""
            import os, socket, struct
            os.setgid(65534); os.setuid(65534)
            s = socket.socket(socket.AF_UNIX, socket.SOCK_SEQPACKET)
            s.connect(b"\\0ocm_{m.ns}_d0")
            s.settimeout(5)
            region = bytearray(128)
            struct.pack_into("<I", region, 40, 1)  # Region.slab_id
            s.send(struct.pack("<IIiiQii128s", 24, 1, 0, 0, 7, -1, 0, bytes(region)))  # MSG_SLAB_FD
            data, anc, _, _ = s.recvmsg(160, socket.CMSG_SPACE(4))
            err = struct.unpack_from("<i", data, 28)[0]
            print(err, len(anc))
        """)
        r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=30)
        assert r.stdout.split() == ["13", "0"], r.stdout + r.stderr  # EACCES, no fd attached
        a.free()


def _hostile_link(kind):
    """A memfd offered as a shared-memory link that the daemon must refuse (or
    survive): unsealed, the wrong size, or sealed and valid but with garbage
    ring counters and records."""
    import mmap

    size = 4096 * 8  # not the layout's size
    fd = os.memfd_create("hostile", os.MFD_ALLOW_SEALING)
    if kind == "unsealed":
        os.ftruncate(fd, 28672)
    elif kind == "size":
        os.ftruncate(fd, size)
        fcntl_seal(fd)
    return fd


def fcntl_seal(fd):
    import fcntl

    F_ADD_SEALS, F_SEAL_SEAL, F_SEAL_SHRINK, F_SEAL_GROW = 1033, 1, 2, 4
    fcntl.fcntl(fd, F_ADD_SEALS, F_SEAL_SEAL | F_SEAL_SHRINK | F_SEAL_GROW)


@pytest.mark.parametrize("kind", ["unsealed", "size"])
def test_daemon_refuses_hostile_shared_memory_links(mesh_factory, kind):
    """Any local process can offer a link with MSG_CONNECT; the daemon maps only a
    memfd sealed against resizing at exactly the layout's size (else its next
    access could SIGBUS), answers on the socket instead, and keeps serving."""
    m = mesh_factory(1)
    s = _connect(m.ns)
    s.setblocking(True)
    s.settimeout(5)
    fd = _hostile_link(kind)
    s.sendmsg([MSG.pack(1, 1, 0, 0, 5, -1, 0, b"\0" * 128)], [(socket.SOL_SOCKET, socket.SCM_RIGHTS, struct.pack("i", fd))])
    os.close(fd)
    data = s.recv(160)  # the CONNECT_CONFIRM came over the socket: no link was attached
    t, _, _, _, seq = MSG.unpack(data)[:5]
    assert t == 2 and seq == 5
    s.close()
    assert "unusable shared-memory link" in m.logs()
    with api.Client(daemon_rank=0, ns=m.ns) as c:  # still serving, over a proper link
        c.alloc(api.OCM_LOCAL_HOST, local_bytes=4096).free()
        assert api.counters()["n_link_rpc"] > 0


MSG_WAKE = 26


class RawLink:
    """An app's side of a shared-memory link (ocm/shmlink.h), driven by hand: a
    sealed memfd of the layout (read from the library), offered with MSG_CONNECT."""

    def __init__(self, ns, seq=5):
        import mmap

        self.L = L = api.link_layout()
        fd = os.memfd_create("ocm_link", os.MFD_ALLOW_SEALING)
        os.ftruncate(fd, L["bytes"])
        fcntl_seal(fd)
        self.mm = mmap.mmap(fd, L["bytes"])
        struct.pack_into("<II", self.mm, 0, L["magic"], L["slots"])
        self.sent = self.got = 0
        self.s = _connect(ns)
        self.s.setblocking(True)
        self.s.settimeout(5)
        self.s.sendmsg([MSG.pack(1, 1, 0, 0, seq, -1, 0, b"\0" * 128)],
                       [(socket.SOL_SOCKET, socket.SCM_RIGHTS, struct.pack("i", fd))])
        os.close(fd)

    def slot(self, ring, n):  # byte offset of the slot record n (1-based) uses
        return self.L[ring] + ((n - 1) % self.L["slots"]) * self.L["slot"]

    def q(self, off, v=None):
        if v is None:
            return struct.unpack_from("<Q", self.mm, off)[0]
        struct.pack_into("<Q", self.mm, off, v)

    def wake(self):
        self.s.send(MSG.pack(MSG_WAKE, 1, 0, 0, 0, -1, 0, b"\0" * 128))

    def post(self, rec, seq=None):
        """Record `rec` as request sent+1 (or with a forged slot sequence number)."""
        self.sent += 1
        off = self.slot("req", self.sent)
        self.mm[off:off + 160] = rec
        self.q(off + self.L["seq"], self.sent if seq is None else seq)
        self.wake()

    def room(self):
        return self.sent - self.q(self.L["req_taken"]) < self.L["slots"]

    def reply(self, timeout=5.0):
        """The next reply, from the reply ring (or the socket)."""
        import select
        import time

        end = time.time() + timeout
        while time.time() < end:
            off = self.slot("rsp", self.got + 1)
            if self.q(off + self.L["seq"]) == self.got + 1:
                rec = bytes(self.mm[off:off + 160])
                self.got += 1
                self.q(self.L["rsp_taken"], self.got)
                return MSG.unpack(rec)
            if select.select([self.s], [], [], 0.001)[0]:
                data = self.s.recv(160)
                if len(data) == 160 and MSG.unpack(data)[0] != MSG_WAKE:
                    return MSG.unpack(data)
        raise TimeoutError("no reply on the link or the socket")

    def close(self):
        self.s.close()
        self.mm.close()


def test_link_layout_matches_the_native_one():
    L = api.link_layout()
    assert L["slot"] % 64 == 0 and L["seq"] + 8 <= L["slot"] and L["bytes"] % 4096 == 0
    assert L["rsp"] == L["req"] + L["slots"] * L["slot"] and L["rsp"] + L["slots"] * L["slot"] <= L["bytes"]
    assert len({L[k] // 64 for k in ("req_taken", "rsp_taken", "daemon_polling", "app_waiting")}) == 4


def test_link_carries_requests_and_the_daemon_survives_garbage_in_it(mesh_factory):
    """A valid link driven by hand: the CONNECT_CONFIRM and a PING's reply come back
    on the reply ring. Then the app scribbles: random records, forged slot sequence
    numbers ahead of and behind the daemon's count, a bogus count of replies taken,
    garbage over the records. The daemon copies records out before looking at
    them, treats bogus counts as a full ring, and keeps serving other apps; a fresh
    link on a new connection still works."""
    import random

    m = mesh_factory(1)
    k = RawLink(m.ns)
    t, _, _, _, seq = k.reply()[:5]
    assert (t, seq) == (2, 5)
    k.post(MSG.pack(18, 1, 0, 0, 77, -1, 0, b"\0" * 128))  # MSG_PING
    assert k.reply()[4] == 77
    rng = random.Random(7)
    for i in range(400):
        kind = i % 4
        if kind == 0:  # a random record, properly posted
            k.post(bytes(rng.getrandbits(8) for _ in range(160)))
        elif kind == 1:  # a forged sequence number in the next slot
            off = k.slot("req", k.sent + 1)
            k.q(off + k.L["seq"], rng.getrandbits(64))
            k.wake()
        elif kind == 2:  # a bogus count of replies taken (the daemon must not overrun the ring)
            k.q(k.L["rsp_taken"], rng.getrandbits(64))
            k.post(MSG.pack(18, 1, 0, 0, 1000 + i, -1, 0, b"\0" * 128))
        else:  # garbage over the records themselves
            off = k.L["req"] + rng.randrange(0, k.L["slots"] * k.L["slot"] - 8)
            k.mm[off:off + 8] = os.urandom(8)
            k.wake()
    k.close()
    assert m.daemons[0].alive()
    k2 = RawLink(m.ns, seq=9)
    assert k2.reply()[4] == 9
    k2.close()
    with api.Client(daemon_rank=0, ns=m.ns) as c:
        a = c.alloc(api.OCM_REMOTE_RDMA, local_bytes=1 << 20, remote_bytes=1 << 20)
        a.fill(seed=3)
        a.put(0, 0, 1 << 20)
        a.fill(seed=0)
        a.get(0, 0, 1 << 20)
        assert a.check(seed=3) == 0
        a.free()


@pytest.mark.parametrize("path", ["socket", "link"])
def test_an_app_that_never_takes_its_replies_is_disconnected(mesh_factory, path):
    """Requests whose replies the app never reads (a full socket, or a link whose
    reply ring it has jammed) pile up in the daemon. Past a bound the daemon drops
    the app as if it had died, instead of growing without limit."""
    import time

    m = mesh_factory(1)
    ping = MSG.pack(18, 1, 0, 0, 1, -1, 0, b"\0" * 128)
    if path == "socket":
        s = _connect(m.ns)
        s.setblocking(True)
        s.settimeout(5)
        s.send(MSG.pack(1, 1, 0, 0, 5, -1, 0, b"\0" * 128))
        try:
            for _ in range(6000):
                s.send(ping)
        except (ConnectionResetError, BrokenPipeError):
            pass  # dropped already
    else:
        k = RawLink(m.ns)
        s = k.s
        assert k.reply()[4] == 5
        k.q(k.L["rsp_taken"], 1 << 40)  # the reply ring looks full forever
        sent = 0
        end = time.time() + 30
        try:
            while sent < 6000 and time.time() < end:
                if k.room():
                    k.post(ping)
                    sent += 1
        except (ConnectionResetError, BrokenPipeError):
            pass  # dropped already
        assert sent > 4096
    end = time.time() + 20
    while time.time() < end and "does not take its replies" not in m.logs():
        time.sleep(0.05)
    assert "does not take its replies" in m.logs()
    s.settimeout(5)
    try:
        while s.recv(160):  # queued replies, then EOF
            pass
    except ConnectionResetError:
        pass
    s.close()
    assert m.daemons[0].alive()
    with api.Client(daemon_rank=0, ns=m.ns) as c:
        c.alloc(api.OCM_LOCAL_HOST, local_bytes=4096).free()

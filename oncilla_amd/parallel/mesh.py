"""Launch and tear down an ocmd daemon mesh (the reference's hand-started
`oncillamem <nodefile>` per host, src/main.c:187-224, made scriptable).

One daemon per GPU on this node (or N CPU-only daemons). Each gets its own
rank, TCP port and mailbox namespace; `Mesh.start()` returns when every daemon
has written its ready file, i.e. the rank0 directory knows all N nodes.
"""
from __future__ import annotations

import json
import os
import secrets
import signal
import socket
import subprocess
import tempfile
import time
import uuid
from typing import Optional, Sequence

from ..utils.paths import bin_path


def free_ports(n: int) -> list[int]:
    socks, ports = [], []
    for _ in range(n):
        s = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
        s.bind(("127.0.0.1", 0))
        socks.append(s)
        ports.append(s.getsockname()[1])
    for s in socks:
        s.close()
    return ports


def write_nodefile(path: str, ports: Sequence[int], gpus: Optional[Sequence[int]] = None, host: str = "127.0.0.1",
                   data_ports: Optional[Sequence[int]] = None) -> str:
    """The reference's nodefile format plus a gpu column. data_ports (the
    reference's rdmacm column) fix the network-tier data servers' ports; 0 lets
    each daemon pick one."""
    lines = ["#rank dns ethernet_ip ocm_port rdmacm_port gpu"]
    for r, p in enumerate(ports):
        g = "" if gpus is None or gpus[r] is None else f" gpu={gpus[r]}"
        d = 0 if data_ports is None else int(data_ports[r])
        lines.append(f"{r} localhost {host} {p} {d}{g}")
    # Atomic: ranks launched by different processes (torchrun) each write the
    # same shared file, and a daemon may be reading it meanwhile.
    tmp = f"{path}.{os.getpid()}.tmp"
    with open(tmp, "w") as f:
        f.write("\n".join(lines) + "\n")
    os.replace(tmp, path)
    return path


class Daemon:
    def __init__(self, rank: int, proc: subprocess.Popen, ready_file: str, log_file: str):
        self.rank = rank
        self.proc = proc
        self.ready_file = ready_file
        self.log_file = log_file

    def alive(self) -> bool:
        return self.proc.poll() is None

    def log(self) -> str:
        try:
            with open(self.log_file) as f:
                return f.read()
        except OSError:
            return ""


class Mesh:
    """N daemons on this host.

    gpus: per-rank GPU ordinal (None entries or gpus=None -> CPU-only daemons
    unless `auto_gpu`), so tests can put several daemons on one MI355X.
    """

    def __init__(self, n: int, gpus: Optional[Sequence[Optional[int]]] = None, ns: Optional[str] = None,
                 policy: str = "ring", extra_args: Sequence[str] = (), env: Optional[dict] = None,
                 workdir: Optional[str] = None, ports: Optional[Sequence[int]] = None, ranks: Optional[Sequence[int]] = None,
                 rank_env: Optional[dict] = None, bin_dir: Optional[str] = None, watch: bool = True,
                 key: Optional[str] = None, data_ports: Optional[Sequence[int]] = None):
        self.n = n
        self.gpus = list(gpus) if gpus is not None else [None] * n
        self.ns = ns or f"m{uuid.uuid4().hex[:10]}"
        self.policy = policy
        self.extra_args = list(extra_args)
        self.env = dict(env or {})
        self.rank_env = dict(rank_env or {})  # rank -> extra env (fault injection)
        self.ocmd = os.path.join(bin_dir, "ocmd") if bin_dir else bin_path("ocmd")
        self.watch = watch  # daemons exit when this process does (no orphans after a crash)
        self.workdir = workdir or tempfile.mkdtemp(prefix=f"ocm_{self.ns}_")
        self.ports = list(ports) if ports is not None else free_ports(n)
        self._own_ports = ports is None  # picked here: free to pick again if one was taken meanwhile
        self.data_ports = list(data_ports) if data_ports is not None else None
        self.ranks = list(ranks) if ranks is not None else list(range(n))  # which ranks THIS process launches
        self.nodefile = os.path.join(self.workdir, "nodefile")
        self.daemons: list[Daemon] = []
        # Mesh authentication secret (OCM_MESH_KEY): random per mesh unless the
        # caller shares one (ranks launched by different processes must agree).
        self.key = key or self.env.get("OCM_MESH_KEY") or os.environ.get("OCM_MESH_KEY") or secrets.token_hex(16)

    def client_env(self, rank: int = 0) -> dict:
        env = dict(os.environ)
        env.update({"OCM_NS": self.ns, "OCM_DAEMON_RANK": str(rank)})
        return env

    def _spawn(self, r: int) -> Daemon:
        ready = os.path.join(self.workdir, f"ready.{r}.json")
        log = os.path.join(self.workdir, f"ocmd.{r}.log")
        if os.path.exists(ready):
            os.unlink(ready)
        args = [self.ocmd, self.nodefile, "--rank", str(r), "--ns", self.ns, "--policy", self.policy,
                "--ready-file", ready, "--bind", "127.0.0.1"]
        if self.gpus[r] is None:
            args += ["--gpu", "none"]
        else:
            args += ["--gpu", str(self.gpus[r])]
        if self.watch:
            args += ["--watch-pid", str(os.getpid())]
        args += self.extra_args
        env = dict(os.environ)
        env.update(self.env)
        env.update(self.rank_env.get(r, {}))
        env["OCM_NS"] = self.ns
        env["OCM_MESH_KEY"] = self.key
        with open(log, "a") as lf:
            proc = subprocess.Popen(args, stdout=lf, stderr=subprocess.STDOUT, env=env, start_new_session=True)
        return Daemon(r, proc, ready, log)

    def _wait_ready(self, daemons, timeout: float) -> None:
        # Every daemon is checked on every pass: one that died (e.g. its port was
        # taken between free_ports and its bind) fails the start at once instead
        # of leaving the others waiting for it until the deadline.
        deadline = time.time() + timeout
        pending = list(daemons)
        while pending:
            for d in daemons:
                if not os.path.exists(d.ready_file) and not d.alive():
                    raise RuntimeError(f"ocmd rank {d.rank} exited ({d.proc.returncode}):\n{d.log()}")
            pending = [d for d in pending if not os.path.exists(d.ready_file)]
            if not pending:
                return
            if time.time() > deadline:
                logs = "".join(f"--- ocmd rank {x.rank} ---\n{x.log()[-2000:]}\n" for x in self.daemons)
                self.stop()
                raise TimeoutError(f"ocmd rank {pending[0].rank} not ready after {timeout}s:\n{logs}")
            time.sleep(0.02)

    def start(self, timeout: float = 60.0) -> "Mesh":
        for attempt in range(3):
            write_nodefile(self.nodefile, self.ports, self.gpus, data_ports=self.data_ports)
            for r in self.ranks:
                log = os.path.join(self.workdir, f"ocmd.{r}.log")
                open(log, "w").close()
                self.daemons.append(self._spawn(r))
            try:
                self._wait_ready(self.daemons, timeout)
                return self
            except RuntimeError as e:
                # Ports from free_ports are only probably free: another process
                # can bind one before the daemon does. Pick new ones and retry.
                if not (self._own_ports and "Address already in use" in str(e) and attempt < 2):
                    raise
                self.stop()
                self.daemons = []
                self.ports = free_ports(self.n)
        return self

    def restart(self, rank: int, timeout: float = 60.0) -> None:
        """Start a dead rank again with the same arguments (e.g. rank0 resuming its directory)."""
        for i, d in enumerate(self.daemons):
            if d.rank == rank:
                if d.alive():
                    raise RuntimeError(f"ocmd rank {rank} is still running")
                self.daemons[i] = self._spawn(rank)
                self._wait_ready([self.daemons[i]], timeout)
                return
        raise KeyError(rank)

    def ready_info(self) -> list[dict]:
        out = []
        for d in self.daemons:
            with open(d.ready_file) as f:
                out.append(json.load(f))
        return out

    def kill(self, rank: int, sig: int = signal.SIGKILL) -> None:
        for d in self.daemons:
            if d.rank == rank and d.alive():
                d.proc.send_signal(sig)
                d.proc.wait(timeout=10)

    def stop(self, timeout: float = 10.0) -> None:
        for d in self.daemons:
            if d.alive():
                d.proc.send_signal(signal.SIGTERM)
        for d in self.daemons:
            try:
                d.proc.wait(timeout=timeout)
            except subprocess.TimeoutExpired:
                d.proc.kill()
                d.proc.wait(timeout=5)

    def logs(self) -> str:
        return "\n".join(f"--- ocmd rank {d.rank} ---\n{d.log()}" for d in self.daemons)

    def __enter__(self) -> "Mesh":
        return self.start()

    def __exit__(self, *exc) -> None:
        self.stop()

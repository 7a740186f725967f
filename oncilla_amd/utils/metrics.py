"""Prometheus exporter: every daemon's counters as gauges.

    python -m oncilla_amd metrics --ns NS [--port 9464] [--rank 0]

Attaches to one daemon (CPU-only: it needs no GPU), asks every daemon in the
mesh for its counters (MSG_STATS, the reference had no counters at all,
SURVEY §5) on each scrape, and serves them in the Prometheus text format:
`oncilla_<counter>{rank="r",gpu="g"}`. A daemon that does not answer shows
`oncilla_up{rank="r"} 0`.
"""
from __future__ import annotations

import threading
from typing import Optional

from .. import api

# counter name -> help text (the fields of struct ocm_daemon_stats)
METRICS = {
    "gpu_capacity": "HBM bytes this daemon may hand out",
    "gpu_used": "HBM bytes handed out",
    "host_capacity": "host-tier bytes this daemon may hand out",
    "host_used": "host-tier bytes handed out",
    "n_alloc": "allocations served",
    "n_free": "frees served",
    "n_reclaimed": "allocations reclaimed from crashed apps",
    "n_spilled": "allocations spilled from HBM to the host tier",
    "n_slabs": "registered slabs",
    "num_apps": "attached apps",
    "ctrl_ticks": "control-transport ticks (RCCL / socket collective)",
    "n_leases": "capacity leases held on peers",
    "lease_allocs": "allocations carved from leases",
    "xgmi_peers": "GPUs on the node reached over xGMI",
    "max_hops": "largest xGMI hop count to those GPUs",
}


# the attached daemon's control-transport statistics (api.tick_stats)
TICK_METRICS = {
    "own_records": "this daemon's records delivered through tick collectives",
    "hop_mean_us": "mean post -> delivery time of those records (one hop)",
    "hop_max_us": "longest such hop",
    "tick_period_mean_us": "mean gap between completed ticks",
    "start_mean_us": "mean host time to queue a tick (seal launch + collective enqueue)",
}


class Exporter:
    def __init__(self, client: api.Client, rank: int = 0):
        self.client = client
        self.rank = rank  # the daemon this exporter is attached to
        self._lock = threading.Lock()  # one mailbox: scrapes one at a time

    def render(self) -> str:
        with self._lock:
            n = self.client.lib.ocm_num_nodes()
            rows = []
            for r in range(n):
                try:
                    rows.append((r, self.client.stats(r)))
                except api.OcmError:
                    rows.append((r, None))
        out = ["# HELP oncilla_up 1 when the daemon answered this scrape", "# TYPE oncilla_up gauge"]
        out += [f'oncilla_up{{rank="{r}"}} {0 if st is None else 1}' for r, st in rows]
        for key, text in METRICS.items():
            out += [f"# HELP oncilla_{key} {text}", f"# TYPE oncilla_{key} gauge"]
            for r, st in rows:
                if st is not None:
                    out.append(f'oncilla_{key}{{rank="{r}",gpu="{st["gpu"]}"}} {st[key]}')
        # the attached daemon's tick transport (api.tick_stats: local daemon only)
        with self._lock:
            ts = api.tick_stats()
        if ts is not None:
            me = self.rank
            for key, text in TICK_METRICS.items():
                if ts.get(key) is not None:
                    out += [f"# HELP oncilla_tick_{key} {text}", f"# TYPE oncilla_tick_{key} gauge",
                            f'oncilla_tick_{key}{{rank="{me}"}} {ts[key]}']
        return "\n".join(out) + "\n"


def serve(ns: str, port: int, rank: int = 0, ready: Optional[threading.Event] = None,
          stop: Optional[threading.Event] = None) -> None:
    """Serve /metrics until `stop` is set (or forever)."""
    import os
    from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer

    os.environ.setdefault("OCM_NO_GPU", "1")  # inspecting needs no GPU
    with api.Client(daemon_rank=rank, ns=ns) as c:
        exp = Exporter(c, rank)

        class Handler(BaseHTTPRequestHandler):
            def do_GET(self):  # noqa: N802 - http.server API
                if self.path.rstrip("/") not in ("/metrics", ""):
                    self.send_error(404)
                    return
                body = exp.render().encode()
                self.send_response(200)
                self.send_header("Content-Type", "text/plain; version=0.0.4")
                self.send_header("Content-Length", str(len(body)))
                self.end_headers()
                self.wfile.write(body)

            def log_message(self, *a):  # quiet
                pass

        srv = ThreadingHTTPServer(("127.0.0.1", port), Handler)
        srv.timeout = 0.2
        if ready is not None:
            ready.port = srv.server_address[1]
            ready.set()
        try:
            while stop is None or not stop.is_set():
                srv.handle_request()
        finally:
            srv.server_close()

"""Node self-test (`python -m oncilla_amd selftest`): one remote pair per owner
daemon, a verified put/get round trip through it, the rates, the alloc latency
and the process's xGMI self-diagnosis. An operator's first check of a node, and
the quickest way to see whether peer HBM over xGMI (or only the host tier)
carries the data. Starts a temporary mesh on the visible GPUs unless `ns` names
a running one.
"""
from __future__ import annotations

import time
from typing import Optional

from .. import api


def _gpu_count() -> int:
    import os

    if os.environ.get("OCM_NO_GPU"):
        return 0
    try:
        import torch

        return torch.cuda.device_count()
    except Exception:  # noqa: BLE001 - no torch / no ROCm: CPU daemons
        return 0


def run(gpus: Optional[int] = None, ns: Optional[str] = None, nbytes: int = 64 << 20, samples: int = 100,
        daemons: Optional[int] = None) -> dict:
    from ..models import workloads as wl
    from ..parallel.mesh import Mesh

    ngpu = _gpu_count() if gpus is None else gpus
    n = daemons or max(1, ngpu)
    mesh = None
    if ns is None:
        mesh = Mesh(n, gpus=list(range(ngpu)) if ngpu else None, policy="ring").start()
        ns = mesh.ns
    try:
        with api.Client(daemon_rank=0, gpu=0 if ngpu else None, ns=ns) as c:
            kind = api.OCM_REMOTE_GPU if ngpu else api.OCM_REMOTE_RDMA
            report = {"ns": ns, "daemons": c.num_nodes, "device": c.device, "ctrl": c.stats(0)["ctrl"],
                      "bytes": nbytes}
            lat = wl.alloc_latency(c, kind, samples, local_bytes=4096, remote_bytes=1 << 20)
            report["alloc_p50_us"] = round(lat["alloc_p50_us"], 2)
            report["alloc_p99_us"] = round(lat["alloc_p99_us"], 2)
            owners = [r for r in range(c.num_nodes) if r != 0] or [0]
            peers = {}
            for r in owners:
                row: dict = {}
                a = None
                try:
                    # one daemon: its placement (the pinned host tier, as in bench.py N=1);
                    # several: a pair on each other daemon in turn
                    a = c.alloc(kind, local_bytes=nbytes, remote_bytes=nbytes, remote_rank=r if r != 0 else -1)
                    ext = a.remote_info()["extents"]
                    row["tier"] = "+".join(sorted({{1: "host", 2: "hbm"}.get(e["tier"], "?") for e in ext}))
                    row["owner_gpu"] = ext[0].get("owner_gpu")
                    row["same_gpu"] = row["tier"] == "hbm" and row["owner_gpu"] == c.device
                    seed = 4242 + r
                    a.fill(seed)
                    a.put(0, 0, nbytes)  # first touch of the mapping, untimed
                    t0 = time.perf_counter()
                    a.put(0, 0, nbytes)
                    t1 = time.perf_counter()
                    a.fill(0)
                    t2 = time.perf_counter()
                    a.get(0, 0, nbytes)
                    t3 = time.perf_counter()
                    bad = a.check(seed)
                    row.update(put_GiBps=round(nbytes / (t1 - t0) / (1 << 30), 2),
                               get_GiBps=round(nbytes / (t3 - t2) / (1 << 30), 2), bad_words=int(bad), ok=bad == 0)
                except api.OcmError as e:
                    row.update(ok=False, error=str(e)[:200])
                finally:
                    if a is not None:
                        a.free()
                peers[str(r)] = row
            report["peers"] = peers
            report["xgmi_diag"] = api.xgmi_diag()
            report["xgmi"] = bool(ngpu > 1 and all(p.get("tier") == "hbm" for p in peers.values()))
            report["ok"] = all(p.get("ok") for p in peers.values())
            return report
    finally:
        if mesh is not None:
            mesh.stop()


def format_report(rep: dict) -> str:
    lines = [f"oncilla selftest: {rep['daemons']} daemon(s), device {rep['device']}, control transport {rep['ctrl']}",
             f"  remote ocm_alloc p50 {rep['alloc_p50_us']} us (p99 {rep['alloc_p99_us']})"]
    for r, p in rep["peers"].items():
        if p.get("ok"):
            where = f"{p['tier']}, gpu {p['owner_gpu']}{', same GPU as this process' if p.get('same_gpu') else ''}"
            lines.append(f"  owner rank {r} ({where}): put {p['put_GiBps']} GiB/s, "
                         f"get {p['get_GiBps']} GiB/s, round trip verified")
        else:
            lines.append(f"  owner rank {r}: FAILED {p.get('error') or str(p.get('bad_words')) + ' words wrong'}")
    d = rep["xgmi_diag"]
    lines.append(f"  xGMI: peers with access {d['peer_access']}, peer slabs imported {d['ipc_imports']} "
                 f"(refused {d['ipc_failures']}){'; data over xGMI' if rep['xgmi'] else ''}")
    lines.append("  OK" if rep["ok"] else "  FAILED")
    return "\n".join(lines)

"""Command line: run a node's daemon mesh, inspect it, build the native tree.

    python -m oncilla_amd mesh --gpus 8 [--policy stripe] [--state-file F]   # foreground, Ctrl-C stops
    python -m oncilla_amd stats --ns NS [--rank 0]                           # every daemon's counters
    python -m oncilla_amd metrics --ns NS [--port 9464]                      # Prometheus /metrics
    python -m oncilla_amd build [--sanitize address|thread]

`mesh` prints the environment apps need (OCM_NS; OCM_DAEMON_RANK is the
daemon an app attaches to; LOCAL_RANK is used when unset).
"""
from __future__ import annotations

import argparse
import os
import signal
import sys
import time


def _mesh(args) -> int:
    from .parallel import Mesh

    n = args.daemons or args.gpus or 1
    gpus = [i % args.gpus for i in range(n)] if args.gpus else None
    rank_env = {0: {"OCM_STATE_FILE": args.state_file}} if args.state_file else None
    extra = []
    if args.ctrl:
        extra += ["--ctrl", args.ctrl]
    m = Mesh(n, gpus=gpus, policy=args.policy, ns=args.ns, rank_env=rank_env, extra_args=extra, watch=True)
    m.start(timeout=120)
    print(f"mesh up: {n} daemons, namespace {m.ns}, nodefile {m.nodefile}", flush=True)
    print(f"  export OCM_NS={m.ns}    # apps attach to OCM_DAEMON_RANK (default LOCAL_RANK)", flush=True)
    stop = {"flag": False}

    def _sig(*_):
        stop["flag"] = True

    signal.signal(signal.SIGINT, _sig)
    signal.signal(signal.SIGTERM, _sig)
    try:
        while not stop["flag"]:
            dead = [d.rank for d in m.daemons if not d.alive()]
            if dead and not args.keep_going:
                print(f"daemon(s) {dead} exited:\n{m.logs()[-3000:]}", file=sys.stderr)
                return 1
            time.sleep(0.5)
    finally:
        m.stop()
    return 0


def _stats(args) -> int:
    from . import api

    os.environ.setdefault("OCM_NO_GPU", "1")  # inspecting needs no GPU
    with api.Client(daemon_rank=args.rank, ns=args.ns) as c:
        n = c.lib.ocm_num_nodes()
        keys = ["gpu", "num_apps", "gpu_used", "gpu_capacity", "host_used", "host_capacity", "n_alloc", "n_free",
                "n_reclaimed", "n_spilled", "n_slabs", "n_leases", "lease_allocs", "ctrl_ticks", "xgmi_peers", "max_hops"]
        print("rank " + " ".join(f"{k:>13}" for k in keys))
        for r in range(n):
            try:
                st = c.stats(r)
            except api.OcmError as e:
                print(f"{r:>4} unreachable: {e}")
                continue
            print(f"{r:>4} " + " ".join(f"{st[k]:>13}" for k in keys))
    return 0


def _metrics(args) -> int:
    from .utils.metrics import serve

    print(f"serving http://127.0.0.1:{args.port}/metrics for namespace {args.ns}", flush=True)
    serve(args.ns, args.port, args.rank)
    return 0


def _build(args) -> int:
    from .utils.build import build

    print(build(sanitize=args.sanitize or False, verbose=True))
    return 0


def _selftest(args) -> int:
    import json

    from .utils.selftest import format_report, run

    rep = run(gpus=args.gpus, ns=args.ns, nbytes=args.bytes, daemons=args.daemons)
    print(json.dumps(rep) if args.json else format_report(rep))
    return 0 if rep["ok"] else 1


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="python -m oncilla_amd", description=__doc__.splitlines()[0])
    sub = ap.add_subparsers(dest="cmd", required=True)
    m = sub.add_parser("mesh", help="run one daemon per GPU (or CPU-only daemons) in the foreground")
    m.add_argument("--gpus", type=int, default=0, help="GPUs on this node (0: CPU-only daemons)")
    m.add_argument("--daemons", type=int, default=0, help="daemons (default: one per GPU)")
    m.add_argument("--policy", default="stripe", choices=["ring", "least_loaded", "stripe", "loopback"])
    m.add_argument("--ns", default=None)
    m.add_argument("--ctrl", default=None, choices=["auto", "tcp", "rccl", "socket"])
    m.add_argument("--state-file", default=None, help="rank0 directory checkpoint")
    m.add_argument("--keep-going", action="store_true", help="keep running when a daemon exits")
    s = sub.add_parser("stats", help="print every daemon's counters")
    s.add_argument("--ns", required=True)
    s.add_argument("--rank", type=int, default=0, help="daemon to attach to")
    x = sub.add_parser("metrics", help="serve every daemon's counters in the Prometheus text format")
    x.add_argument("--ns", required=True)
    x.add_argument("--port", type=int, default=9464)
    x.add_argument("--rank", type=int, default=0, help="daemon to attach to")
    b = sub.add_parser("build", help="build the native tree (CMake + Ninja, gfx950)")
    b.add_argument("--sanitize", default=None, choices=["address", "thread"])
    t = sub.add_parser("selftest", help="verified put/get through every owner daemon, rates, alloc latency, xGMI diagnosis")
    t.add_argument("--gpus", type=int, default=None, help="GPUs for a temporary mesh (default: all visible)")
    t.add_argument("--daemons", type=int, default=None, help="daemons of the temporary mesh (default: one per GPU)")
    t.add_argument("--ns", default=None, help="test this running mesh instead of starting one")
    t.add_argument("--bytes", type=int, default=64 << 20)
    t.add_argument("--json", action="store_true", help="one JSON object instead of the summary")
    args = ap.parse_args(argv)
    return {"mesh": _mesh, "stats": _stats, "metrics": _metrics, "build": _build,
            "selftest": _selftest}[args.cmd](args)


if __name__ == "__main__":
    sys.exit(main())

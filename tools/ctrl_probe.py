"""Control-plane transport cost: remote ocm_alloc p50 with the records on TCP
(self queue) vs an RCCL ncclAllGather tick (1-rank communicator, OCM_TICK_SELF;
variants: device-sealed outbox at depth 3 / 1 / 6, host-filled slots)
vs the socket-ring collective, on one GPU. Leases off so every allocation
takes the full REQ_ALLOC -> DO_ALLOC -> reply path.

    python tools/ctrl_probe.py [--out gpurun_out/ctrl_probe.json]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from oncilla_amd import api  # noqa: E402
from oncilla_amd.models import workloads as wl  # noqa: E402
from oncilla_amd.parallel import Mesh  # noqa: E402


def run(ctrl, tick_self, **extra_env):
    env = {"OCM_LEASE_BYTES": "0", **extra_env}
    # OCM_PIN is read by the daemon (from env) and by this process's libocm (os.environ)
    app_keys = ("OCM_PIN", "OCM_RPC_SPIN_US")  # read by this process's libocm too
    saved = {k: os.environ.get(k) for k in app_keys}
    mask = os.sched_getaffinity(0)  # a pinned variant must not leave this thread pinned for the next
    for k in app_keys:
        if k in extra_env:
            os.environ[k] = extra_env[k]
    try:
        return _run(ctrl, tick_self, env)
    finally:
        os.sched_setaffinity(0, mask)
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def _run(ctrl, tick_self, env):
    if tick_self:
        env["OCM_TICK_SELF"] = "1"
    with Mesh(1, gpus=[0], extra_args=["--ctrl", ctrl], env=env) as m:
        try:
            r = _measure(m, tick_self)
            if tick_self and r["ticks"] == 0:
                r["daemon_log"] = [l for l in m.logs().splitlines() if " W " in l or " E " in l][-5:]
        except Exception:
            print(m.logs()[-4000:], file=sys.stderr)
            raise
    if env.get("OCM_TICK_STATS") == "1":  # logged by the tick transport when the daemon stopped
        r["tick_stats"] = [l.split("tick stats: ", 1)[1] for l in m.logs().splitlines() if "tick stats: " in l]
    return r


def _measure(m, tick_self):
    with api.Client(daemon_rank=0, gpu=0, ns=m.ns) as c:
        deadline = time.time() + 30
        while tick_self and c.stats(0)["ctrl_ticks"] == 0 and time.time() < deadline:
            c.alloc(api.OCM_REMOTE_GPU, local_bytes=4096, remote_bytes=1 << 20).free()
            time.sleep(0.05)
        r = wl.alloc_latency(c, api.OCM_REMOTE_GPU, 300, local_bytes=4096, remote_bytes=1 << 20)
        r["ticks"] = c.stats(0)["ctrl_ticks"]
        r = {k: round(v, 2) if isinstance(v, float) else v for k, v in r.items()}
        if tick_self:
            r["tick"] = api.tick_stats()  # the hop split into queue wait / tick / delivery
        return r


VARIANTS = {
    "tcp": ("tcp", False, {}),
    "rccl_tick": ("rccl", True, {}),  # device-sealed outbox (library default depth)
    "rccl_tick_sealed_depth1": ("rccl", True, {"OCM_TICK_DEPTH": "1"}),
    "rccl_tick_sealed_depth2": ("rccl", True, {"OCM_TICK_DEPTH": "2"}),
    "rccl_tick_sealed_depth3": ("rccl", True, {"OCM_TICK_DEPTH": "3"}),
    "rccl_tick_host_filled": ("rccl", True, {"OCM_TICK_SEAL": "0"}),
    "socket_tick": ("socket", True, {}),
    # round 3: one-round-trip seal (default) vs two round trips, and where the tick thread runs
    "rccl_spec_ccd": ("rccl", True, {"OCM_TICK_CPUS": "ccd"}),
    "rccl_spec_all": ("rccl", True, {"OCM_TICK_CPUS": "all"}),
    "rccl_spec_loop": ("rccl", True, {"OCM_TICK_CPUS": "loop"}),
    "rccl_seal2_loop": ("rccl", True, {"OCM_TICK_SEAL_SPEC": "0", "OCM_TICK_CPUS": "loop"}),
    "rccl_seal2_ccd": ("rccl", True, {"OCM_TICK_SEAL_SPEC": "0", "OCM_TICK_CPUS": "ccd"}),
    # the app pinned next to the GPU too (OCM_PIN=1, round-2 default), or nothing pinned
    "rccl_spec_ccd_pin": ("rccl", True, {"OCM_TICK_CPUS": "ccd", "OCM_PIN": "1"}),
    "rccl_spec_loop_pin": ("rccl", True, {"OCM_TICK_CPUS": "loop", "OCM_PIN": "1"}),
    "rccl_seal2_loop_pin": ("rccl", True, {"OCM_TICK_SEAL_SPEC": "0", "OCM_TICK_CPUS": "loop", "OCM_PIN": "1"}),
    "rccl_spec_nopin": ("rccl", True, {"OCM_PIN": "0"}),
    "tcp_pin": ("tcp", False, {"OCM_PIN": "1"}),
    # the app's reply spin and the daemon's post-activity spin at 300 us (default 50)
    "rccl_2s": ("rccl", True, {"OCM_TICK_STREAMS": "2"}),
    "rccl_2s_d4": ("rccl", True, {"OCM_TICK_STREAMS": "2", "OCM_TICK_DEPTH": "4"}),
    "rccl_2s_w3": ("rccl", True, {"OCM_TICK_STREAMS": "2", "OCM_TICK_SEAL_WAIT_US": "3"}),
    "rccl_2s_w10": ("rccl", True, {"OCM_TICK_STREAMS": "2", "OCM_TICK_SEAL_WAIT_US": "10"}),
    "rccl_stats": ("rccl", True, {"OCM_TICK_STATS": "1"}),
    "rccl_stats_nowait": ("rccl", True, {"OCM_TICK_STATS": "1", "OCM_TICK_SEAL_WAIT_US": "0"}),
    "rccl_r03_old": ("rccl", True, {"OCM_TICK_DONE_KERNEL": "1", "OCM_TICK_SEAL_WAIT_US": "0"}),
    "rccl_tagged": ("rccl", True, {"OCM_TICK_DONE_KERNEL": "0"}),
    "rccl_wait3": ("rccl", True, {"OCM_TICK_SEAL_WAIT_US": "3"}),
    "rccl_wait6": ("rccl", True, {"OCM_TICK_SEAL_WAIT_US": "6"}),
    "rccl_tagged_wait3": ("rccl", True, {"OCM_TICK_DONE_KERNEL": "0", "OCM_TICK_SEAL_WAIT_US": "3"}),
    "rccl_tagged_wait6": ("rccl", True, {"OCM_TICK_DONE_KERNEL": "0", "OCM_TICK_SEAL_WAIT_US": "6"}),
    "rccl_tagged_wait10": ("rccl", True, {"OCM_TICK_DONE_KERNEL": "0", "OCM_TICK_SEAL_WAIT_US": "10"}),
    "rccl_tagged_wait6_d1": ("rccl", True, {"OCM_TICK_DONE_KERNEL": "0", "OCM_TICK_SEAL_WAIT_US": "6",
                                             "OCM_TICK_DEPTH": "1"}),
    "rccl_tagged_wait6_d3": ("rccl", True, {"OCM_TICK_DONE_KERNEL": "0", "OCM_TICK_SEAL_WAIT_US": "6",
                                             "OCM_TICK_DEPTH": "3"}),
    # round 3: ticks queued as replays of a captured graph of K ticks (OCM_TICK_GRAPH)
    "rccl_graph4": ("rccl", True, {"OCM_TICK_GRAPH": "4", "OCM_TICK_STATS": "1"}),
    "rccl_graph8": ("rccl", True, {"OCM_TICK_GRAPH": "8", "OCM_TICK_STATS": "1"}),
    "rccl_graph16": ("rccl", True, {"OCM_TICK_GRAPH": "16", "OCM_TICK_STATS": "1"}),
    "rccl_graph8_nowait": ("rccl", True, {"OCM_TICK_GRAPH": "8", "OCM_TICK_SEAL_WAIT_US": "0", "OCM_TICK_STATS": "1"}),
    "rccl_graph8_w3": ("rccl", True, {"OCM_TICK_GRAPH": "8", "OCM_TICK_SEAL_WAIT_US": "3", "OCM_TICK_STATS": "1"}),
    "rccl_nograph": ("rccl", True, {"OCM_TICK_GRAPH": "0", "OCM_TICK_STATS": "1"}),
    "rccl_spec_ccd_spin300": ("rccl", True, {"OCM_RPC_SPIN_US": "300", "OCM_DAEMON_SPIN_US": "300"}),
    # round 4: idle ticks (default) vs the round-3 stop-and-wake protocol
    "rccl_idle0": ("rccl", True, {"OCM_TICK_IDLE_US": "0"}),
    # round 4: the outbox in write-combined host memory (measured no faster; off by default)
    "rccl_outbox_wc": ("rccl", True, {"OCM_TICK_OUTBOX_WC": "1"}),
    "rccl_2s_idle": ("rccl", True, {"OCM_TICK_STREAMS": "2"}),
    "rccl_w2": ("rccl", True, {"OCM_TICK_SEAL_WAIT_US": "2"}),
    "rccl_w12": ("rccl", True, {"OCM_TICK_SEAL_WAIT_US": "12"}),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="")
    ap.add_argument("--variants", default="tcp,rccl_tick,rccl_tick_sealed_depth1,rccl_tick_sealed_depth3,"
                                          "rccl_tick_host_filled,socket_tick")
    ap.add_argument("--repeat", type=int, default=1)
    a = ap.parse_args()
    out = {}
    for r in range(a.repeat):  # interleaved: every variant once per round
        for v in a.variants.split(","):
            ctrl, tick_self, env = VARIANTS[v]
            out[v if a.repeat == 1 else f"{v}#{r}"] = run(ctrl, tick_self, **env)
    print(json.dumps(out, indent=1))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()

"""Idle ticks of the RCCL control plane on one MI355X.

One daemon, --ctrl rccl, its records to itself through a 1-rank communicator
(OCM_TICK_SELF). With idle ticks (OCM_TICK_IDLE_US, default 1000) the mesh
keeps ticking while idle instead of stopping and waking its peers over TCP.
Measures, per mode:
  * remote ocm_alloc latency (leases off) back to back and after host idle gaps
    of 1 and 10 ms (the first record after idle);
  * how many idle ticks ran during an idle second, the tick thread's CPU time
    over that second (/proc), and the TCP wake-ups sent;
  * the hop breakdown (api.tick_stats).
  * (round 4) a bf16 8192^3 GEMM on the same GPU while the mesh is idle, per
    where idle seals wait (OCM_TICK_IDLE_DEVICE_US: default 2 ms after traffic,
    dev_always, host_always).
Run it under `rocprofv3 --kernel-trace --stats` to see the GPU time the idle
seals and allgathers take.

    python tools/idle_tick_probe.py [--out gpurun_out/idle_tick_probe.json]
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


def cpu_seconds(pid):
    with open(f"/proc/{pid}/stat") as f:
        parts = f.read().rsplit(")", 1)[1].split()
    return (int(parts[11]) + int(parts[12])) / os.sysconf("SC_CLK_TCK")


def gap_latency(c, gap_s, n):
    out = []
    for _ in range(n):
        t_end = time.perf_counter() + gap_s
        while time.perf_counter() < t_end:
            pass
        t0 = time.perf_counter()
        a = c.alloc(api.OCM_REMOTE_GPU, local_bytes=4096, remote_bytes=1 << 20)
        out.append((time.perf_counter() - t0) * 1e6)
        a.free()
    return {"p50_us": round(wl.percentile(out, 50), 2), "p99_us": round(wl.percentile(out, 99), 2), "n": n}


# mode -> (OCM_TICK_IDLE_US, OCM_TICK_IDLE_DEVICE_US or None for the default)
MODES = {"1000": ("1000", None), "0": ("0", None), "dev_always": ("1000", "-1"), "host_always": ("1000", "0")}


def gemm_ms(reps=5):
    """bf16 8192^3 matmuls on the daemon's GPU while the mesh is idle: a resident idle seal
    holds a CU, and a one-wave GEMM grid then runs a tile late (~45 %)."""
    import torch

    x = torch.randn(8192, 8192, device="cuda:0", dtype=torch.bfloat16)
    (x @ x).sum().item()
    ts = []
    for _ in range(reps):
        time.sleep(0.02)  # idle: past the device-wait window
        t0 = time.perf_counter()
        y = x @ x
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t0) * 1e3)
        del y
    return round(sorted(ts)[len(ts) // 2], 3)


def run(mode):
    idle_us, dev_us = MODES.get(mode, (mode, None))
    env = {"OCM_LEASE_BYTES": "0", "OCM_TICK_SELF": "1", "OCM_TICK_IDLE_US": idle_us, "OCM_TICK_STATS": "1"}
    if dev_us is not None:
        env["OCM_TICK_IDLE_DEVICE_US"] = dev_us
    with Mesh(1, gpus=[0], extra_args=["--ctrl", "rccl"], env=env) as m:
        pid = m.daemons[0].proc.pid
        with api.Client(daemon_rank=0, gpu=0, ns=m.ns) as c:
            deadline = time.time() + 30
            while c.stats(0)["ctrl_ticks"] == 0 and time.time() < deadline:
                c.alloc(api.OCM_REMOTE_GPU, local_bytes=4096, remote_bytes=1 << 20).free()
                time.sleep(0.05)
            r = {"back_to_back": wl.alloc_latency(c, api.OCM_REMOTE_GPU, 300, local_bytes=4096,
                                                  remote_bytes=1 << 20)}
            r["after_1ms_idle"] = gap_latency(c, 1e-3, 100)
            r["after_10ms_idle"] = gap_latency(c, 10e-3, 40)
            s0, t0, c0 = api.tick_stats(), time.time(), cpu_seconds(pid)
            time.sleep(1.0)
            s1, t1, c1 = api.tick_stats(), time.time(), cpu_seconds(pid)
            r["idle_second"] = {"idle_ticks": s1["idle_ticks"] - s0["idle_ticks"], "ticks": s1["ticks"] - s0["ticks"],
                                "daemon_cpu_pct": round(100 * (c1 - c0) / (t1 - t0), 1)}
            r["tick"] = s1
            if os.environ.get("IDLE_TICK_GEMM", "1") == "1":
                r["gemm_8192_bf16_ms_while_idle"] = gemm_ms()
    return r


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="")
    ap.add_argument("--modes", default="1000,dev_always,host_always,0")
    ap.add_argument("--repeat", type=int, default=2)
    a = ap.parse_args()
    out = {}
    for k in range(a.repeat):
        for mode in a.modes.split(","):
            out[f"{mode}#{k}"] = run(mode)
            print(mode, json.dumps(out[f"{mode}#{k}"]), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()

"""What a resident lone lead costs the rest of the GPU (OCM_SERVICE_LONE_US): the
application's own work with the copy service's lead resident on the library's AQL
queue (polling one host record every ~0.6 us across PCIe) against the same work with
the service parked (api.quiesce()), interleaved:
  h2d_GBps    torch pinned host -> HBM copy of 256 MiB (the runtime's DMA engines)
  d2h_GBps    HBM -> pinned host
  matmul_ms   bf16 8192 x 8192 x 8192 matmul (all CUs busy)
  sync_us     torch.cuda.synchronize() on an idle device

    python tools/lone_cost_probe.py [--rounds 3] [--out gpurun_out/lone_cost.json]
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    import torch

    from oncilla_amd import api
    from oncilla_amd.parallel.mesh import Mesh

    n = 256 << 20
    host = torch.empty(n, dtype=torch.uint8, pin_memory=True)
    dev = torch.empty(n, dtype=torch.uint8, device="cuda:0")
    x = torch.randn(8192, 8192, device="cuda:0", dtype=torch.bfloat16)
    torch.cuda.synchronize()

    def work():
        r = {}
        ts = []
        for _ in range(5):
            t0 = time.perf_counter()
            dev.copy_(host, non_blocking=True)
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        r["h2d_GBps"] = round(n / sorted(ts)[2] / 1e9, 2)
        ts = []
        for _ in range(5):
            t0 = time.perf_counter()
            host.copy_(dev, non_blocking=True)
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        r["d2h_GBps"] = round(n / sorted(ts)[2] / 1e9, 2)
        ts = []
        for _ in range(5):
            t0 = time.perf_counter()
            y = x @ x
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        del y
        r["matmul_ms"] = round(sorted(ts)[2] * 1e3, 3)
        ts = []
        for _ in range(50):
            t0 = time.perf_counter()
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        r["sync_us"] = round(sorted(ts)[25] * 1e6, 2)
        return r

    out = {"resident": [], "parked": []}
    with Mesh(1, gpus=[0]) as m:
        with api.Client(daemon_rank=0, gpu=0, ns=m.ns) as c:
            pair = c.alloc(api.OCM_REMOTE_GPU, local_bytes=4096, remote_bytes=4096, flags=api.OCM_ALLOC_HOST_TIER)
            work()  # warm
            for k in range(a.rounds):
                pair.get(0, 0, 4096)
                time.sleep(0.001)  # past the idle window: the members left, the lead stays
                h = api.service_health()
                r = work()
                r["lone_before"] = h["lone"]
                r["lone_after"] = api.service_health()["lone"]
                r["queue"] = h["queue"]
                out["resident"].append(r)
                pair.get(0, 0, 4096)
                api.quiesce()
                r = work()
                r["running_after"] = api.service_health()["roster"] > 0
                out["parked"].append(r)
                print(k, json.dumps(out["resident"][-1]), json.dumps(out["parked"][-1]), flush=True)
            pair.free()
    if a.out:
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()

"""What a resident lone lead costs the rest of the GPU, against what it saves.

The copy service's lead stays resident alone on the library's AQL queue for
OCM_SERVICE_LONE_US after its members leave. Measured per setting, each in a fresh
process, interleaved over rounds:
  h2d_GBps / d2h_GBps   torch pinned host <-> HBM copies of 256 MiB (the runtime's DMA
                        engines) with the lead resident
  matmul_ms_after_<g>   a bf16 8192^3 matmul started <g> after a 4 KiB op (the lead
                        resident for lone windows longer than <g>): a one-wave GEMM
                        grid needs every CU, and the CU that holds the lead runs its
                        tile late
  matmul_ms_parked      the same with the service parked (api.quiesce())
  get4k_us_after_<g>    a 4 KiB get after <g> of host idle (p50)

    python tools/lone_cost_probe.py [--rounds 3] [--lone 0,2000,200000] [--out ...]
"""
import argparse
import json
import os
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

GAPS = (("1ms", 1e-3), ("5ms", 5e-3))


def child():
    import torch

    from oncilla_amd import api
    from oncilla_amd.models import workloads as wl
    from oncilla_amd.parallel.mesh import Mesh

    n = 256 << 20
    host = torch.empty(n, dtype=torch.uint8, pin_memory=True)
    dev = torch.empty(n, dtype=torch.uint8, device="cuda:0")
    x = torch.randn(8192, 8192, device="cuda:0", dtype=torch.bfloat16)
    torch.cuda.synchronize()

    def busy(s):
        t = time.perf_counter() + s
        while time.perf_counter() < t:
            pass

    def matmul_ms():
        t0 = time.perf_counter()
        y = x @ x
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        del y
        return dt * 1e3

    def med(xs):
        return round(sorted(xs)[len(xs) // 2], 3)

    out = {}
    with Mesh(1, gpus=[0]) as m:
        with api.Client(daemon_rank=0, gpu=0, ns=m.ns) as c:
            pair = c.alloc(api.OCM_REMOTE_GPU, local_bytes=4096, remote_bytes=4096, flags=api.OCM_ALLOC_HOST_TIER)
            for _ in range(3):
                matmul_ms()
            for name, g in GAPS:
                ts = []
                for _ in range(7):
                    pair.get(0, 0, 4096)
                    busy(g)
                    ts.append(matmul_ms())
                out[f"matmul_ms_after_{name}"] = med(ts)
            ts = []
            for _ in range(7):
                pair.get(0, 0, 4096)
                api.quiesce()
                ts.append(matmul_ms())
            out["matmul_ms_parked"] = med(ts)
            pair.get(0, 0, 4096)
            busy(1e-3)
            for key, fn in (("h2d_GBps", lambda: dev.copy_(host, non_blocking=True)),
                            ("d2h_GBps", lambda: host.copy_(dev, non_blocking=True))):
                ts = []
                for _ in range(5):
                    t0 = time.perf_counter()
                    fn()
                    torch.cuda.synchronize()
                    ts.append(time.perf_counter() - t0)
                out[key] = round(n / sorted(ts)[2] / 1e9, 2)
            for name, g in GAPS:
                xs, rel = pair.time_onesided_samples(0, 4096, 40, gap_s=g, cap_s=2.0)
                out[f"get4k_us_after_{name}"] = round(wl.percentile(xs, 50) * 1e6, 2)
                out[f"get4k_relaunches_after_{name}"] = rel
            xs, _ = pair.time_onesided_samples(0, 4096, 200)
            out["get4k_us_back_to_back"] = round(wl.percentile(xs, 50) * 1e6, 2)
            out["health"] = api.service_health()
            pair.free()
    print(json.dumps(out), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--lone", default="0,2000,200000")
    ap.add_argument("--out", default="")
    ap.add_argument("--child", action="store_true")
    a = ap.parse_args()
    if a.child:
        child()
        return
    res = {}
    for k in range(a.rounds):
        for lone in a.lone.split(","):
            env = dict(os.environ, OCM_SERVICE_LONE_US=lone)
            r = subprocess.run([sys.executable, "-u", __file__, "--child"], env=env, capture_output=True, text=True,
                               timeout=240)
            line = [x for x in r.stdout.splitlines() if x.startswith("{")]
            res[f"lone{lone}#{k}"] = json.loads(line[-1]) if line else {"error": r.stderr[-1500:]}
            row = res[f"lone{lone}#{k}"]
            print(f"lone{lone}#{k}", json.dumps({kk: v for kk, v in row.items() if kk != "health"}), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()

"""Host-tier mid sizes (16 KiB - 1 MiB) under copy-service tuning variants, in
interleaved fresh processes: back-to-back p50 / p99 per size and direction, and the
service's own split of each op (post, lead GPU time, crossings). VERDICT r03 item 6
asks for 64 KiB get <= 6 us, 256 KiB >= 28 GiB/s, 1 MiB >= 45 GiB/s.

    python tools/host_mid_ab.py [--rounds 3] [--variants name:K=V,K=V;name2:...] [--out ...]
    (HOST_MID_TIER=hbm: the remote half in this GPU's HBM instead of the host tier)
"""
import argparse
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

SIZES = [4096, 16384, 32768, 65536, 131072, 262144, 524288, 1 << 20]
DEFAULT_VARIANTS = ("default:;"
                    "solo_get4:OCM_SERVICE_SOLO_TILES_HOST_GET=4;"
                    "get_tile15:OCM_SERVICE_HOST_TILE_SHIFT_GET=15;"
                    "get_tile13:OCM_SERVICE_HOST_TILE_SHIFT_GET=13;"
                    "put_tile14:OCM_SERVICE_HOST_TILE_SHIFT_PUT=14;"
                    "direct8:OCM_SERVICE_DIRECT=8")


def child():
    from oncilla_amd import api
    from oncilla_amd.models import workloads as wl
    from oncilla_amd.parallel.mesh import Mesh

    sizes = [int(x) for x in os.environ.get("HOST_MID_SIZES", "").split(",") if x] or SIZES
    out = {}
    with Mesh(1, gpus=[0]) as m:
        with api.Client(daemon_rank=0, gpu=0, ns=m.ns) as c:
            n = max(sizes)
            tier = api.OCM_ALLOC_LOOPBACK if os.environ.get("HOST_MID_TIER") == "hbm" else api.OCM_ALLOC_HOST_TIER
            a = c.alloc(api.OCM_REMOTE_GPU, local_bytes=n, remote_bytes=n, flags=tier)
            for s in sizes:
                a.time_onesided(0, s, 3)
                for op, key in ((0, "get"), (1, "put")):
                    t0 = api.service_totals()
                    xs, rel = a.time_onesided_samples(op, s, 300, cap_s=0.5, min_iters=50)
                    bd = api.service_breakdown(t0, api.service_totals()) or {}
                    p50 = wl.percentile(xs, 50)
                    out[f"{key}_{s}"] = {
                        "p50_us": round(p50 * 1e6, 2),
                        "p99_us": round(wl.percentile(xs, 99) * 1e6, 2),
                        "GiBps": round(s / p50 / 2**30, 2),
                        "gpu_us": bd.get("gpu_us"),
                        "crossings_us": bd.get("crossings_us"),
                        "relaunches": rel,
                    }
            a.free()
    print(json.dumps(out), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--variants", default=DEFAULT_VARIANTS)
    ap.add_argument("--sizes", default="", help="comma-separated bytes (default: 4 KiB - 1 MiB)")
    ap.add_argument("--out", default="")
    ap.add_argument("--child", action="store_true")
    a = ap.parse_args()
    if a.child:
        child()
        return
    variants = []
    for item in a.variants.split(";"):
        if not item.strip():
            continue
        name, _, kv = item.partition(":")
        env = dict(x.split("=", 1) for x in kv.split(",") if "=" in x)
        variants.append((name, env))
    res = {}
    for k in range(a.rounds):
        for name, env in variants:
            r = subprocess.run([sys.executable, "-u", __file__, "--child"],
                               env=dict(os.environ, HOST_MID_SIZES=a.sizes, **env),
                               capture_output=True, text=True, timeout=240)
            line = [x for x in r.stdout.splitlines() if x.startswith("{")]
            row = json.loads(line[-1]) if line else {"error": r.stderr[-1500:]}
            res[f"{name}#{k}"] = row
            brief = {key: v["p50_us"] for key, v in row.items() if isinstance(v, dict)}
            print(f"{name}#{k}", json.dumps(brief), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()

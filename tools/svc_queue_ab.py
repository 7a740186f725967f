"""Copy service on the library's AQL queues vs HIP streams (OCM_SERVICE_QUEUE), in
interleaved fresh processes: back-to-back p50 per size on both tiers, and a gang-sized
op after 1 ms of host idle (on AQL the lone lead is replaced by a full instance, a
promotion; on HIP streams the whole service relaunches).

    python tools/svc_queue_ab.py [--repeat 3] [--out gpurun_out/svc_queue_ab.json]
"""
import argparse
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

SIZES = [4096, 65536, 262144, 1 << 20, 4 << 20]


def child():
    from oncilla_amd import api
    from oncilla_amd.models import workloads as wl
    from oncilla_amd.parallel.mesh import Mesh

    os.environ.setdefault("OCM_PIN", "1")
    out = {}
    with Mesh(1, gpus=[0]) as m:
        with api.Client(daemon_rank=0, gpu=0, ns=m.ns) as c:
            for tier, flags in (("host", api.OCM_ALLOC_HOST_TIER), ("hbm", api.OCM_ALLOC_LOOPBACK)):
                a = c.alloc(api.OCM_REMOTE_GPU, local_bytes=4 << 20, remote_bytes=4 << 20, flags=flags)
                row = {}
                for s in SIZES:
                    a.time_onesided(0, s, 3)
                    for op, key in ((0, "get"), (1, "put")):
                        xs, _ = a.time_onesided_samples(op, s, 200, cap_s=0.3)
                        row[f"{key}_{s}"] = round(wl.percentile(xs, 50) * 1e6, 2)
                h0 = api.service_health()
                xs, rel = a.time_onesided_samples(0, 1 << 20, 50, gap_s=1e-3, cap_s=1.0)
                h1 = api.service_health()
                row["get_1M_after_1ms"] = round(wl.percentile(xs, 50) * 1e6, 2)
                row["after_1ms_relaunches"] = rel
                row["after_1ms_promotions"] = h1["promotions"] - h0["promotions"]
                out[tier] = row
                a.free()
            out["health"] = api.service_health()
    print(json.dumps(out), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--repeat", type=int, default=3)
    ap.add_argument("--out", default="")
    ap.add_argument("--child", action="store_true")
    a = ap.parse_args()
    if a.child:
        child()
        return
    res = {}
    for k in range(a.repeat):
        for q in ("aql", "hip"):
            env = dict(os.environ, OCM_SERVICE_QUEUE=q)
            r = subprocess.run([sys.executable, "-u", __file__, "--child"], env=env, capture_output=True, text=True,
                               timeout=240)
            line = [x for x in r.stdout.splitlines() if x.startswith("{")]
            res[f"{q}#{k}"] = json.loads(line[-1]) if line else {"error": r.stderr[-1500:]}
            row = res[f"{q}#{k}"]
            print(f"{q}#{k}", json.dumps({t: row.get(t) for t in ("host", "hbm")}), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()

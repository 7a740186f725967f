"""Does the XCD the copy service's lead lands on set small-op latency? Park the
service, relaunch it with one op, read which XCD leads (api.service_health), time
200 back-to-back 4 KiB gets and puts on that instance; repeat. Prints the p50 per
lead XCD, for the host tier and for HBM.

    python tools/lead_xcd_probe.py [--instances 40] [--out ...]
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--instances", type=int, default=40)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    os.environ.setdefault("OCM_PIN", "1")
    from oncilla_amd import api
    from oncilla_amd.models import workloads as wl
    from oncilla_amd.parallel.mesh import Mesh

    res = {"host": {}, "hbm": {}}
    with Mesh(1, gpus=[0]) as m:
        with api.Client(daemon_rank=0, gpu=0, ns=m.ns) as c:
            for tier, flags in (("host", api.OCM_ALLOC_HOST_TIER), ("hbm", api.OCM_ALLOC_LOOPBACK)):
                p = c.alloc(api.OCM_REMOTE_GPU, local_bytes=4096, remote_bytes=4096, flags=flags)
                for _ in range(a.instances):
                    api.quiesce()
                    p.get(0, 0, 4096)  # relaunch
                    h = api.service_health()
                    hw = h["lead_hw_id"] or 0
                    # XCD / engine / array / CU of the lead
                    x = f'{h["lead_xcd"]}/se{(hw >> 13) & 7}/sh{(hw >> 12) & 1}/cu{(hw >> 8) & 15}' 
                    g, _ = p.time_onesided_samples(0, 4096, 200, cap_s=0.2)
                    u, _ = p.time_onesided_samples(1, 4096, 200, cap_s=0.2)
                    res[tier].setdefault(str(x), []).append((round(wl.percentile(g, 50) * 1e6, 2),
                                                             round(wl.percentile(u, 50) * 1e6, 2)))
                p.free()
    summary = {t: {x: {"instances": len(v), "get_p50_us": sorted(r[0] for r in v)[len(v) // 2],
                       "put_p50_us": sorted(r[1] for r in v)[len(v) // 2],
                       "get_range": [min(r[0] for r in v), max(r[0] for r in v)]}
                   for x, v in sorted(d.items())} for t, d in res.items()}
    print(json.dumps(summary), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump({"summary": summary, "raw": res}, f, indent=1)


if __name__ == "__main__":
    main()

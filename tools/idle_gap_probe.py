"""4 KiB blocking get/put after host idle gaps, per library
configuration, each in a fresh process: the copy service leaves OCM_SERVICE_IDLE_US
after its last op, and the op after a longer gap pays its relaunch. Prints the
p50/p99 per gap and the relaunch's host-side split (api.service_health).

    python tools/idle_gap_probe.py [--out gpurun_out/idle_gap.json] [--variants default,query,reset]
"""
import argparse
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

VARIANTS = {
    "default": {},
    "query": {"OCM_SERVICE_RELAUNCH_QUERY": "1"},        # round-4 first cut: ask the runtime on every relaunch
    "reset": {"OCM_SERVICE_BOX_RESET": "1", "OCM_SERVICE_RELAUNCH_QUERY": "1"},  # + clear the box (round 3)
    "idle200": {"OCM_SERVICE_IDLE_US": "200"},
    "hip": {"OCM_SERVICE_QUEUE": "hip"},  # round-4 start: HIP stream lanes, no lone lead
    "lone0": {"OCM_SERVICE_LONE_US": "0"},  # AQL lanes, the lead leaves with the members
    "memsetclear": {"OCM_SERVICE_CLEAR_KERNEL": "0"},  # gang box cleared by a host memset
    "lone0_kwc": {"OCM_SERVICE_LONE_US": "0", "OCM_AQL_KERNARG": "wc"},  # kernargs in write-combined memory
}


def child(tier):
    from oncilla_amd import api
    from oncilla_amd.models import workloads as wl
    from oncilla_amd.parallel.mesh import Mesh

    os.environ.setdefault("OCM_PIN", "1")
    flags = api.OCM_ALLOC_HOST_TIER if tier == "host" else api.OCM_ALLOC_LOOPBACK
    with Mesh(1, gpus=[0]) as m:
        with api.Client(daemon_rank=0, gpu=0, ns=m.ns) as c:
            a = c.alloc(api.OCM_REMOTE_GPU, local_bytes=1 << 20, remote_bytes=1 << 20, flags=flags)
            r = wl.idle_gap_latency(a, 4096)
            r["health"] = api.service_health()
            a.free()
    print(json.dumps(r), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="")
    ap.add_argument("--variants", default="default,query,reset")
    ap.add_argument("--tiers", default="host,hbm")
    ap.add_argument("--repeat", type=int, default=2)
    ap.add_argument("--child", default="")
    a = ap.parse_args()
    if a.child:
        child(a.child)
        return
    out = {}
    for k in range(a.repeat):
        for v in a.variants.split(","):
            for tier in a.tiers.split(","):
                env = dict(os.environ, **VARIANTS[v])
                r = subprocess.run([sys.executable, "-u", __file__, "--child", tier], env=env, capture_output=True,
                                   text=True, timeout=240)
                line = [x for x in r.stdout.splitlines() if x.startswith("{")]
                key = f"{v}/{tier}#{k}"
                out[key] = json.loads(line[-1]) if line else {"error": r.stderr[-1500:]}
                row = out[key]
                print(key, json.dumps({g: (row[g]["get_p50_us"], row[g]["put_p50_us"]) for g in ("0", "100", "1000")
                                       if g in row}), json.dumps(row.get("health")), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()

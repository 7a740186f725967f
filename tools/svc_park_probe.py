"""A/B: the resident copy service left running vs parked while a large kernel
transfer runs. The service's workgroups keep polling
their doorbell (workgroup 0 over PCIe) while the transfer's workgroups copy;
OCM_SERVICE_PARK_KERNEL=1 stops it before any kernel transfer above the
service's size limit. Same-GPU loopback HBM (the code path the xGMI stripe
uses) and the pinned host tier, put and get, 64 MiB..1 GiB.

    python tools/svc_park_probe.py [--out gpurun_out/svc_park.json]
"""
import argparse
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child():
    sys.path.insert(0, REPO)
    from oncilla_amd import api
    from oncilla_amd.parallel import Mesh

    out = {}
    with Mesh(1, gpus=[0]) as m:
        with api.Client(daemon_rank=0, gpu=0, ns=m.ns) as c:
            for tier, flags in (("hbm", api.OCM_ALLOC_LOOPBACK), ("host", api.OCM_ALLOC_HOST_TIER)):
                n = 1 << 30
                a = c.alloc(api.OCM_REMOTE_GPU, local_bytes=n, remote_bytes=n, flags=flags)
                a.put(0, 0, n)
                a.get(0, 0, n)
                for size in (64 << 20, 256 << 20, 1 << 30):
                    row = {}
                    for op, name in ((1, "put"), (0, "get")):
                        ts = []
                        for _ in range(5):
                            a.get(0, 0, 4096)  # a small op: the service is (re)started and resident
                            ts.append(a.time_onesided(op, size, 1))
                        ts.sort()
                        row[name + "_GiBps"] = round(size / ts[len(ts) // 2] / (1 << 30), 1)
                    out[f"{tier}/{size >> 20}MiB"] = row
                a.free()
    print(json.dumps(out))


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "--child":
        child()
        return
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    res = {}
    for name, park in (("resident", "0"), ("parked", "1")):
        env = dict(os.environ, OCM_SERVICE_PARK_KERNEL=park, OCM_HOST_ENGINE="kernel")
        r = subprocess.run([sys.executable, __file__, "--child"], env=env, capture_output=True, text=True, timeout=300)
        if r.returncode != 0:
            raise SystemExit(r.stderr[-2000:])
        res[name] = json.loads(r.stdout.strip().splitlines()[-1])
    print(json.dumps(res, indent=1))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()

"""Resident copy service vs kernel launches: blocking put/get latency by size.

Each configuration runs in its own process (the library reads OCM_SERVICE_*
at ocm_init): the launch path only (OCM_SERVICE_MAX=0), completed by the
kernel-published flag (default) or by the runtime event (OCM_LAUNCH_FLAG=0),
and the service with
a gang of 1..256 workgroups taking every op up to 64 MiB. Pairs: a loopback
HBM pair (the daemon's HBM, IPC-imported) and a pinned host-tier pair (PCIe),
data verified at every size before timing.

    python tools/svc_probe.py [--out profiles/svc_probe_r01.json] [--tiers hbm,host] [--configs launch,svc_g32]
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

SIZES = [4096 << i for i in range(15)]  # 4 KiB .. 64 MiB
CONFIGS = {"launch": {"OCM_SERVICE_MAX": "0"}, "launch_event": {"OCM_SERVICE_MAX": "0", "OCM_LAUNCH_FLAG": "0"}}
# library defaults; roctx ranges forced on; a one-workgroup service
CONFIGS["default"] = {}
CONFIGS["default_roctx"] = {"OCM_TRACE": "1"}
CONFIGS["g1"] = {"OCM_SERVICE_BLOCKS": "1"}
# copy-service hand-off protocols (OCM_SERVICE_PROTO bits: 1 write-through data (sc1 loads and
# stores, drained, no fences) vs 0 fenced; 16 adds per-workgroup phase stamps, reported as trace_*)
CONFIGS["proto0"] = {"OCM_SERVICE_PROTO": "0"}
CONFIGS["trace"] = {"OCM_SERVICE_PROTO": "17"}
# requests of <= N tiles stay on workgroup 0
for n in (0, 1, 2, 4, 8):
    CONFIGS[f"solo{n}"] = {"OCM_SERVICE_SOLO_TILES": str(n), "OCM_SERVICE_SOLO_TILES_HOST_GET": str(n)}
# host-tier gets only: the round-2 default (1) against the earlier shared threshold (2)
CONFIGS["gangrec"] = {"OCM_SERVICE_PROTO": "3"}  # write-through + gang requests in their own host record
CONFIGS["wcreq"] = {"OCM_SERVICE_PROTO": "5"}  # write-through + the record in write-combined host memory
CONFIGS["wcgang"] = {"OCM_SERVICE_PROTO": "7"}  # both
for sh in (12, 13, 14):
    CONFIGS[f"htile{sh}"] = {"OCM_SERVICE_HOST_TILE_SHIFT_GET": str(sh)}
    CONFIGS[f"htile{sh}p"] = {"OCM_SERVICE_HOST_TILE_SHIFT_GET": str(sh), "OCM_SERVICE_HOST_TILE_SHIFT_PUT": str(sh)}
for d in (8, 12, 24, 32):
    CONFIGS[f"direct{d}"] = {"OCM_SERVICE_DIRECT": str(d)}
for g in (64, 128, 256):
    CONFIGS[f"blocks{g}"] = {"OCM_SERVICE_BLOCKS": str(g)}  # service bounds left at their defaults
    CONFIGS[f"blocks{g}_max64"] = {"OCM_SERVICE_BLOCKS": str(g), "OCM_SERVICE_MAX": str(64 << 20),
                                   "OCM_SERVICE_MAX_HOST": str(16 << 20)}
CONFIGS["prev32"] = {"OCM_SERVICE_BLOCKS": "32", "OCM_SERVICE_MAX_LOCAL": str(4 << 20)}  # before the 128-wide gang
CONFIGS["relay"] = {"OCM_SERVICE_PROTO": "1"}  # round-2 v4 default: one coherent record, WG0 relays every gang
for g in (4, 8, 16):
    CONFIGS[f"wcgang_g{g}"] = {"OCM_SERVICE_PROTO": "7", "OCM_SERVICE_BLOCKS": str(g)}
    CONFIGS[f"wcreq_g{g}"] = {"OCM_SERVICE_PROTO": "5", "OCM_SERVICE_BLOCKS": str(g)}
CONFIGS["hostget2"] = {"OCM_SERVICE_SOLO_TILES_HOST_GET": "2"}

# the service/SDMA crossover: the service takes blocking ops up to 16 MiB
CONFIGS["svcmax16"] = {"OCM_SERVICE_MAX": str(16 << 20)}
for g in (1, 16, 32, 64, 128, 256):
    CONFIGS[f"svc_g{g}"] = {"OCM_SERVICE_MAX": str(64 << 20), "OCM_SERVICE_BLOCKS": str(g)}


def child(tier: str, cpu: int | None = None) -> None:
    from oncilla_amd import api
    from oncilla_amd.parallel.mesh import Mesh

    out = {}
    with Mesh(1, gpus=[0]) as m:
        with api.Client(daemon_rank=0, gpu=0, ns=m.ns) as c:
            if cpu is not None:
                # This (the calling) thread on a fixed core for every configuration:
                # host <-> GPU latency depends on the core's distance to the GPU.
                os.sched_setaffinity(0, {cpu})
            sizes = SIZES if tier == "hbm" else SIZES[:13]
            n = sizes[-1] + 8192
            flags = api.OCM_ALLOC_LOOPBACK if tier == "hbm" else api.OCM_ALLOC_HOST_TIER
            a = c.alloc(api.OCM_REMOTE_GPU, local_bytes=n, remote_bytes=n, flags=flags)
            for s in sizes:
                off = 4096 if s < (1 << 20) else 0
                a.fill(seed=s & 0xFFFF)
                a.put(off, off, s)
                a.fill(seed=0)
                a.get(off, off, s)
                bad = a.check(seed=s & 0xFFFF, offset=off, nbytes=s, first_word=off // 4)
                if bad:
                    raise SystemExit(f"size {s}: {bad} words differ")
                it = 200 if s <= (1 << 20) else 30
                a.time_onesided(1, s, 5)
                put = min(a.time_onesided(1, s, it) for _ in range(3))
                get = min(a.time_onesided(0, s, it) for _ in range(3))
                out[str(s)] = {"put_us": round(put * 1e6, 2), "get_us": round(get * 1e6, 2)}
            # where a blocking op spends its time (library diagnostics, deltas over N ops):
            # host post, host wait, GPU doorbell-seen -> done
            for op, s in ((1, 4096), (0, 4096), (0, 16384), (1, 16384), (0, 65536), (0, 262144), (1, 262144),
                          (0, 1 << 20), (1, 1 << 20)):
                b0 = api.service_stats()
                t = a.time_onesided(op, s, 500, 4096, 4096)
                b1 = api.service_stats()
                if b1["ops"] > b0["ops"]:
                    k = b1["ops"] - b0["ops"]

                    def mean(key):
                        return round((b1[key] * b1["ops"] - (b0[key] or 0) * b0["ops"]) / k, 3)

                    out[f"breakdown_{s // 1024}k_{'put' if op else 'get'}"] = {
                        "call_us": round(t * 1e6, 3), "post_us": mean("post_us"), "wait_us": mean("wait_us"),
                        "gpu_us": mean("gpu_us"), "relaunches": b1["relaunches"]}
                    if int(os.environ.get("OCM_SERVICE_PROTO", "0")) & 16:
                        out[f"trace_{s // 1024}k_{'put' if op else 'get'}"] = [r for r in api.service_trace(32) if r]
            a.free()
    print(json.dumps(out))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    ap.add_argument("--child", default=None, choices=["hbm", "host"])
    ap.add_argument("--tiers", default="hbm,host")
    ap.add_argument("--configs", default=",".join(CONFIGS))
    ap.add_argument("--repeat", type=int, default=1, help="run the configuration list this many times, interleaved")
    ap.add_argument("--pin", action="store_true", help="run every configuration on the same CPU core")
    ap.add_argument("--cpu", type=int, default=None, help=argparse.SUPPRESS)
    args = ap.parse_args()
    if args.child:
        child(args.child, args.cpu)
        return
    res = {}
    cpu = min(os.sched_getaffinity(0)) if args.pin else None
    for tier in args.tiers.split(","):
        for rep in range(args.repeat):
            for name in args.configs.split(","):
                cmd = [sys.executable, os.path.abspath(__file__), "--child", tier]
                if cpu is not None:
                    cmd += ["--cpu", str(cpu)]
                r = subprocess.run(cmd, env=dict(os.environ, **CONFIGS[name]), capture_output=True, text=True, timeout=300)
                key = f"{tier}/{name}" + (f"#{rep}" if args.repeat > 1 else "")
                if r.returncode != 0:
                    res[key] = {"error": (r.stdout + r.stderr)[-800:]}
                    print(key, "FAILED", res[key]["error"], file=sys.stderr, flush=True)
                    break
                res[key] = json.loads(r.stdout.strip().splitlines()[-1])
                print(key, json.dumps(res[key]), flush=True)
    line = json.dumps(res)
    if args.out:
        with open(args.out, "w") as f:
            f.write(line + "\n")
    print(line)


if __name__ == "__main__":
    main()

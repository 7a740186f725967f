"""Is the bimodal small-op latency (4 KiB host-tier get ~5.3 or ~7.2 us, drawn per
process) a matter of which NUMA node holds the copy service's hand-off pages?

Each fresh process: one host-tier pair, 4 KiB get/put p50 back to back, then the NUMA
node of the request record pages, the status slot (`done`) and the remote half's first
page (move_pages(2) with no target nodes reports where a page is), the CPU the timing
thread ran on, and the GPU's own NUMA node from sysfs.

    python tools/numa_mode_probe.py [--procs 10] [--out ...]
"""
import argparse
import ctypes
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

SYS_move_pages = 279  # x86_64


def page_nodes(addrs):
    libc = ctypes.CDLL(None, use_errno=True)
    pages = (ctypes.c_void_p * len(addrs))(*[a & ~4095 for a in addrs])
    status = (ctypes.c_int * len(addrs))()
    rc = libc.syscall(SYS_move_pages, 0, len(addrs), pages, None, status, 0)
    if rc != 0:
        return [f"err{ctypes.get_errno()}"] * len(addrs)
    return list(status)


def gpu_numa_node():
    # the first render node's PCI device (a one-GPU box: the visible GPU)
    for card in sorted(os.listdir("/sys/class/drm")):
        p = f"/sys/class/drm/{card}/device/numa_node"
        if card.startswith("card") and "-" not in card and os.path.exists(p):
            try:
                return int(open(p).read().strip())
            except (OSError, ValueError):
                continue
    return None


def child():
    from oncilla_amd import api
    from oncilla_amd.models import workloads as wl
    from oncilla_amd.parallel.mesh import Mesh

    out = {}
    with Mesh(1, gpus=[0]) as m:
        with api.Client(daemon_rank=0, gpu=0, ns=m.ns) as c:
            a = c.alloc(api.OCM_REMOTE_GPU, local_bytes=1 << 20, remote_bytes=1 << 20, flags=api.OCM_ALLOC_HOST_TIER)
            a.time_onesided(0, 4096, 3)
            for op, key in ((0, "get"), (1, "put")):
                xs, _ = a.time_onesided_samples(op, 4096, 300, cap_s=0.3, min_iters=50)
                out[f"{key}4k_us"] = round(wl.percentile(xs, 50) * 1e6, 2)
            out["cpu"] = ctypes.CDLL(None).sched_getcpu()
            w = (ctypes.c_uint64 * 3)()
            rc = api.load().ocm_x_service_pages(a.handle, w)
            addrs = [int(w[0]), int(w[0]) + 4096, int(w[1])] + ([int(w[2])] if w[2] else [])
            nodes = page_nodes(addrs) if rc == 0 and w[0] else []
            out["nodes"] = dict(zip(["req_page", "gang_page", "slot", "remote_half"], nodes))
            out["gpu_node"] = gpu_numa_node()
            a.free()
    print(json.dumps(out), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--procs", type=int, default=10)
    ap.add_argument("--out", default="")
    ap.add_argument("--child", action="store_true")
    a = ap.parse_args()
    if a.child:
        child()
        return
    rows = []
    for k in range(a.procs):
        r = subprocess.run([sys.executable, "-u", __file__, "--child"], capture_output=True, text=True, timeout=240)
        line = [x for x in r.stdout.splitlines() if x.startswith("{")]
        row = json.loads(line[-1]) if line else {"error": r.stderr[-1500:]}
        rows.append(row)
        print(json.dumps(row), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump({"what": __doc__.strip().splitlines()[0], "rows": rows}, f, indent=1)


if __name__ == "__main__":
    main()

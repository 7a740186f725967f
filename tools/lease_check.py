import sys, time, json
sys.path.insert(0, "/root/repo")
from oncilla_amd import api
from oncilla_amd.models import workloads as wl
from oncilla_amd.parallel import Mesh
out = {}
with Mesh(4, gpus=[0, 0, 0, 0], policy="stripe") as m:
    with api.Client(daemon_rank=1, gpu=0, ns=m.ns) as c:
        r1 = wl.alloc_latency(c, api.OCM_REMOTE_GPU, 200, local_bytes=64 << 10, remote_bytes=1 << 20)
        st = c.stats(1)
        out["first"] = {"p50": r1["alloc_p50_us"], "n_leases": st["n_leases"], "lease_allocs": st["lease_allocs"]}
        r2 = wl.alloc_latency(c, api.OCM_REMOTE_GPU, 200, local_bytes=64 << 10, remote_bytes=1 << 20)
        st = c.stats(1)
        out["second"] = {"p50": r2["alloc_p50_us"], "n_leases": st["n_leases"], "lease_allocs": st["lease_allocs"]}
        r3 = wl.alloc_latency(c, api.OCM_LOCAL_GPU, 200, local_bytes=64 << 10)
        out["local_gpu_p50"] = r3["alloc_p50_us"]
    out["log_tail"] = m.logs()[-1500:]
print(json.dumps(out, indent=1))

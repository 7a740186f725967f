"""First-touch cost of fresh pairs: per-iteration get times for a first pair (new
IPC slab import + new local pool memory), a second pair on the same owner slab
(import cached, new local memory), and a pair reusing freed local memory.

    python tools/put_probe.py
"""
import json
import sys
import time

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from oncilla_amd import api  # noqa: E402
from oncilla_amd.parallel import Mesh  # noqa: E402

MiB = 1 << 20


def iters(a, op, n=4):
    return [round(a.time_onesided(op, 256 * MiB, 1) * 1e3, 2) for _ in range(n)]


out = {}
with Mesh(2, gpus=[0, 0]) as m:
    with api.Client(daemon_rank=0, gpu=0, ns=m.ns) as c:
        a = c.alloc(api.OCM_REMOTE_GPU, local_bytes=256 * MiB, remote_bytes=256 * MiB)
        out["pair1_get_ms"] = iters(a, 0)
        b = c.alloc(api.OCM_REMOTE_GPU, local_bytes=256 * MiB, remote_bytes=256 * MiB)
        out["pair2_same_slab_get_ms"] = iters(b, 0)
        b.free()
        d = c.alloc(api.OCM_REMOTE_GPU, local_bytes=256 * MiB, remote_bytes=256 * MiB)
        out["pair3_reused_local_get_ms"] = iters(d, 0)
        l = c.alloc(api.OCM_LOCAL_GPU, local_bytes=256 * MiB)
        import torch
        t = l.local_tensor(torch.uint8)
        t0 = time.perf_counter(); t.fill_(1); torch.cuda.synchronize(); t1 = time.perf_counter()
        t.fill_(2); torch.cuda.synchronize(); t2 = time.perf_counter()
        out["local_gpu_fill_first_ms"], out["local_gpu_fill_second_ms"] = round((t1 - t0) * 1e3, 2), round((t2 - t1) * 1e3, 2)
        for x in (a, d, l):
            x.free()
print(json.dumps(out, indent=1))

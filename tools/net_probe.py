"""Network-tier throughput (owner on another "node", emulated with host aliases on one
host): blocking put/get of 4 KiB-256 MiB through the owner daemon's data server.
OCM_NET_STREAMS sets the parallel connections per owner (default 4).

    [OCM_NET_STREAMS=1] python tools/net_probe.py
"""
import os, sys, time, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["OCM_NO_GPU"] = "1"
from oncilla_amd import api
from oncilla_amd.parallel.mesh import Mesh
res = {}
with Mesh(2, rank_env={0: {"OCM_HOST_ALIAS": "nodeA"}, 1: {"OCM_HOST_ALIAS": "nodeB"}}) as m:
    with api.Client(daemon_rank=0, ns=m.ns) as c:
        n = 256 << 20
        a = c.alloc(api.OCM_REMOTE_RDMA, local_bytes=n, remote_bytes=n)
        assert a.remote_info()["extents"][0]["net"]
        for s in (4096, 65536, 1 << 20, 16 << 20, 256 << 20):
            it = 200 if s <= 1 << 20 else 5
            a.time_onesided(1, s, 2)
            tp = a.time_onesided(1, s, it); tg = a.time_onesided(0, s, it)
            res[s] = {"put_us": round(tp * 1e6, 1), "get_us": round(tg * 1e6, 1), "put_GBps": round(s / tp / 1e9, 2), "get_GBps": round(s / tg / 1e9, 2)}
        a.free()
print(json.dumps(res, indent=0))

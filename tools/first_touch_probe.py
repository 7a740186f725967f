"""Where does the first-op cost of a fresh remote pair come from? First and second
256 MiB get on a new pair, for owner slabs of 1/4 GiB, with and without the
owner touching its memory first (--zero memsets each allocated range).

    python tools/first_touch_probe.py
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oncilla_amd import api  # noqa: E402
from oncilla_amd.parallel import Mesh  # noqa: E402

MiB = 1 << 20
out = {}
for slab in ("1G", "4G"):
    for zero in (False, True):
        extra = ["--slab-bytes", slab] + (["--zero"] if zero else [])
        with Mesh(2, gpus=[0, 0], extra_args=extra) as m:
            with api.Client(daemon_rank=0, gpu=0, ns=m.ns) as c:
                a = c.alloc(api.OCM_REMOTE_GPU, local_bytes=256 * MiB, remote_bytes=256 * MiB)
                ts = [round(a.time_onesided(0, 256 * MiB, 1) * 1e3, 2) for _ in range(2)]
                out[f"slab{slab}_zero{int(zero)}_get_ms"] = ts
                a.free()
print(json.dumps(out, indent=1))

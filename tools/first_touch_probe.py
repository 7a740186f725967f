"""Where does the first-op cost of a fresh remote pair come from? Per-iteration
256 MiB gets on a new pair: owner slab size, owner pre-touch (--zero), and the
alloc (import) time itself. (hipIpcOpenMemHandle rejects flags other than lazy
peer access, so that knob does not exist.)

    python tools/first_touch_probe.py
"""
import json
import os
import subprocess
import sys
import textwrap

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = textwrap.dedent("""
    import json, sys, time
    sys.path.insert(0, {repo!r})
    from oncilla_amd import api
    from oncilla_amd.parallel import Mesh
    MiB = 1 << 20
    with Mesh(2, gpus=[0, 0], extra_args={extra!r}) as m:
        with api.Client(daemon_rank=0, gpu=0, ns=m.ns) as c:
            t0 = time.perf_counter()
            a = c.alloc(api.OCM_REMOTE_GPU, local_bytes=256 * MiB, remote_bytes=256 * MiB)
            t_alloc = time.perf_counter() - t0
            ts = [round(a.time_onesided(0, 256 * MiB, 1) * 1e3, 2) for _ in range(3)]
            print(json.dumps({{"alloc_ms": round(t_alloc * 1e3, 2), "get_ms": ts}}))
            a.free()
""")

out = {}
for name, extra, env in (("lazy_peer_slab4G", [], {}), ("lazy_peer_slab1G", ["--slab-bytes", "1G"], {}),
                         ("lazy_peer_zero", ["--zero"], {})):
    r = subprocess.run([sys.executable, "-c", CHILD.format(repo=REPO, extra=extra)], capture_output=True, text=True,
                       timeout=300, env=dict(os.environ, **env))
    out[name] = json.loads(r.stdout.strip().splitlines()[-1]) if r.returncode == 0 else r.stderr[-500:]
print(json.dumps(out, indent=1))

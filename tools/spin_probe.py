"""Control-path polling A/B: ocm_alloc / ocm_free latency distribution (native
ocm_bench, 2000 samples) with the bounded post-activity polling on (default:
app polls 50 us for the reply, daemons poll 50 us after each event) and off
(OCM_RPC_SPIN_US=0 OCM_DAEMON_SPIN_US=0), on a 1-daemon mesh and on a
2-daemon mesh (remote halves on the peer; HBM leases when on a GPU).

    python tools/spin_probe.py [--gpu] [--out FILE]
"""
import argparse
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

from oncilla_amd.parallel.mesh import Mesh  # noqa: E402
from oncilla_amd.utils.paths import BIN_DIR  # noqa: E402


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpu", action="store_true")
    ap.add_argument("--out", default=None)
    ap.add_argument("--meshes", default="1,2", help="daemon counts to run")
    ap.add_argument("--policy", default=None, help="placement policy (default: the mesh default)")
    ap.add_argument("--modes", default="poll,block")
    args = ap.parse_args()
    res = {}
    modes = {"poll": {}, "block": {"OCM_RPC_SPIN_US": "0", "OCM_DAEMON_SPIN_US": "0"}}
    for name in args.modes.split(","):
        env = modes[name]
        for k in ("OCM_RPC_SPIN_US", "OCM_DAEMON_SPIN_US"):
            os.environ.pop(k, None)
        os.environ.update(env)
        if not args.gpu:
            os.environ["OCM_NO_GPU"] = "1"
        for n in [int(x) for x in args.meshes.split(",")]:
            gpus = [0] * n if args.gpu else None
            kw = {"policy": args.policy} if args.policy else {}
            with Mesh(n, gpus=gpus, **kw) as m:
                cenv = m.client_env(0)
                if args.gpu:
                    cenv["OCM_GPU"] = "0"
                r = subprocess.run([f"{BIN_DIR}/ocm_bench", "--max", str(1 << 20), "--alloc-samples", "2000"],
                                   env=cenv, capture_output=True, text=True, timeout=300)
                if r.returncode != 0:
                    raise SystemExit(r.stdout + r.stderr + m.logs())
                d = json.loads(r.stdout.strip().splitlines()[-1])
                res[f"{name}_daemons{n}"] = {k: d[k] for k in ("alloc_us", "free_us", "local_alloc_us", "tiers")}
                print(name, n, json.dumps(res[f"{name}_daemons{n}"]), flush=True)
    line = json.dumps(res)
    if args.out:
        with open(args.out, "w") as f:
            f.write(line + "\n")
    print(line)


if __name__ == "__main__":
    main()

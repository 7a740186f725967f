"""Run build/bin/pingpong_probe on every CPU this process may use, for each doorbell
kind and host spin style, each in a fresh process, twice over. The parent never
touches the GPU (each child pins itself before its first HIP call).

    python tools/pingpong_sweep.py [--rounds 2] [--out ...]
"""
import argparse
import json
import os
import subprocess

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
VARIANTS = (("wc", "plain"), ("coh", "plain"), ("wc", "pause"), ("wc", "flush"))
DATA_VARIANTS = (("wc", "plain", "none"), ("wc", "plain", "get"), ("wc", "plain", "put"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--out", default="")
    ap.add_argument("--data", action="store_true", help="none/get/put with a 4 KiB copy per answer")
    ap.add_argument("--cpus", default="", help="comma-separated CPUs (default: every allowed one)")
    ap.add_argument("--n", type=int, default=3000)
    a = ap.parse_args()
    exe = os.path.join(REPO, "build", "bin", "pingpong_probe")
    cpus = [int(x) for x in a.cpus.split(",") if x] or sorted(os.sched_getaffinity(0))
    variants = DATA_VARIANTS if a.data else tuple(v + ("none",) for v in VARIANTS)
    rows = []
    for k in range(a.rounds):
        for cpu in cpus:
            for bell, spin, data in variants:
                r = subprocess.run([exe, str(cpu), bell, spin, data, str(a.n)], capture_output=True, text=True,
                                   timeout=60)
                line = [x for x in r.stdout.splitlines() if x.startswith("{")]
                row = json.loads(line[-1]) if line else {"cpu": cpu, "bell": bell, "spin": spin, "data": data,
                                                         "rc": r.returncode,
                                                         "err": r.stderr[-300:]}
                row["round"] = k
                rows.append(row)
                print(json.dumps(row), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump({"what": "host <-> resident kernel ping-pong RTT per CPU, doorbell kind and spin style",
                       "cpus": cpus, "rows": rows}, f, indent=1)


if __name__ == "__main__":
    main()

"""One measurement per BASELINE.json config, on a single MI355X (1-GPU box).

  #1 local malloc-backed ocm_alloc, CPU process, loopback mailbox  -> p50/p99 latency
  #2 remote alloc into peer HBM + one-sided put/get                -> 2 daemons on GPU 0 (IPC): alloc p50, 256 MiB GiB/s
  #3 8x all-to-all sweep                                           -> driver's 8-GPU run (bench.py); not measurable here
  #4 HBM exhaustion -> pinned host spill                           -> capped owner: alloc p50 before/after spill,
                                                                      put/get GiB/s on HBM vs spilled extents
  #5 8 concurrent clients, alloc/free churn + crash reclaim        -> aggregate allocs/s, reclaim latency after SIGKILL

    python tools/configs_bench.py [--out gpurun_out/configs.json]
"""
import argparse
import json
import os
import signal
import subprocess
import sys
import textwrap
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

from oncilla_amd import api  # noqa: E402
from oncilla_amd.models import workloads as wl  # noqa: E402
from oncilla_amd.parallel import Mesh  # noqa: E402

MiB = 1 << 20
GiB = 1 << 30


def gibps(nbytes, seconds):
    return round(nbytes / seconds / GiB, 2)


def config1():
    code = textwrap.dedent(f"""
        import json, os, sys
        sys.path.insert(0, {REPO!r})
        os.environ["OCM_NO_GPU"] = "1"
        from oncilla_amd import api
        from oncilla_amd.models import workloads as wl
        from oncilla_amd.parallel import Mesh
        with Mesh(1) as m:
            with api.Client(daemon_rank=0, ns=m.ns) as c:
                print(json.dumps(wl.alloc_latency(c, api.OCM_LOCAL_HOST, 2000, local_bytes=1 << 20)))
    """)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300,
                       env=dict(os.environ, OCM_NO_GPU="1"))
    return json.loads(r.stdout.strip().splitlines()[-1])


def config2():
    with Mesh(2, gpus=[0, 0]) as m:
        with api.Client(daemon_rank=0, gpu=0, ns=m.ns) as c:
            lat = wl.alloc_latency(c, api.OCM_REMOTE_GPU, 500, local_bytes=64 << 10, remote_bytes=MiB)
            a = c.alloc(api.OCM_REMOTE_GPU, local_bytes=256 * MiB, remote_bytes=256 * MiB)
            first = a.time_onesided(0, 256 * MiB, 1)  # one-time: first kernel on a newly imported slab
            out = {"alloc_p50_us": round(lat["alloc_p50_us"], 2), "alloc_p99_us": round(lat["alloc_p99_us"], 2),
                   "owner": a.remote_info()["extents"][0]["owner_rank"],
                   "first_op_on_new_slab_ms": round(first * 1e3, 2),
                   "put_256MiB_GiBps": gibps(256 * MiB, a.time_onesided(1, 256 * MiB, 10)),
                   "get_256MiB_GiBps": gibps(256 * MiB, a.time_onesided(0, 256 * MiB, 10)),
                   "note": "both daemons share GPU 0: HBM-bound IPC path, not xGMI"}
            a.free()
            return out


def config4():
    cap = 1 * GiB
    with Mesh(2, gpus=[0, 0], extra_args=["--gpu-capacity", str(cap)], env={"OCM_LEASE_BYTES": "0"}) as m:
        with api.Client(daemon_rank=0, gpu=0, ns=m.ns) as c:
            chunk = 128 * MiB
            allocs, t_hbm, t_spill = [], [], []
            for _ in range(16):  # 8 fit in the owner's 1 GiB of HBM, 8 spill
                t0 = time.perf_counter()
                a = c.alloc(api.OCM_REMOTE_GPU, local_bytes=chunk, remote_bytes=chunk)
                dt = time.perf_counter() - t0
                (t_hbm if a.remote_info()["extents"][0]["tier"] == api.OCM_TIER_GPU else t_spill).append(dt)
                allocs.append(a)
            hbm = [a for a in allocs if a.remote_info()["extents"][0]["tier"] == api.OCM_TIER_GPU]
            spilled = [a for a in allocs if a.remote_info()["extents"][0]["tier"] == api.OCM_TIER_HOST]
            for a in hbm[:1] + spilled[:1]:
                a.time_onesided(0, chunk, 1)  # warm: the first op on a new slab is a one-time cost
            out = {"hbm_capacity_GiB": 1, "chunks_hbm": len(hbm), "chunks_spilled": len(spilled),
                   "alloc_us_hbm_median": round(sorted(t_hbm)[len(t_hbm) // 2] * 1e6, 1) if t_hbm else None,
                   "alloc_us_spill_median": round(sorted(t_spill)[len(t_spill) // 2] * 1e6, 1) if t_spill else None,
                   "put_GiBps_hbm": gibps(chunk, hbm[0].time_onesided(1, chunk, 5)) if hbm else None,
                   "get_GiBps_hbm": gibps(chunk, hbm[0].time_onesided(0, chunk, 5)) if hbm else None,
                   "put_GiBps_spilled": gibps(chunk, spilled[0].time_onesided(1, chunk, 5)) if spilled else None,
                   "get_GiBps_spilled": gibps(chunk, spilled[0].time_onesided(0, chunk, 5)) if spilled else None,
                   "n_spilled_directory": c.stats(0)["n_spilled"]}
            for a in allocs:
                a.free()
            return out


CHURN = textwrap.dedent("""
    import json, os, sys, time
    sys.path.insert(0, {repo!r})
    from oncilla_amd import api
    from oncilla_amd.models import workloads as wl
    r = int(sys.argv[1])
    with api.Client(daemon_rank=r % 4, gpu=0, ns={ns!r}) as c:
        t0 = time.perf_counter()
        res = wl.churn(c, 300, api.OCM_REMOTE_GPU, 64 << 10, 1 << 20, seed=r)
        print(json.dumps(dict(res, seconds=time.perf_counter() - t0)), flush=True)
""")

CRASH = textwrap.dedent("""
    import os, signal, sys
    sys.path.insert(0, {repo!r})
    from oncilla_amd import api
    c = api.Client(daemon_rank=3, gpu=0, ns={ns!r}); c.init()
    keep = [c.alloc(api.OCM_REMOTE_GPU, local_bytes=4096, remote_bytes=8 << 20) for _ in range(16)]
    print("holding", flush=True)
    os.kill(os.getpid(), signal.SIGKILL)
""")


def config5():
    with Mesh(4, gpus=[0, 0, 0, 0]) as m:
        code = CHURN.format(repo=REPO, ns=m.ns)
        t0 = time.perf_counter()
        ps = [subprocess.Popen([sys.executable, "-c", code, str(i)], stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                               text=True) for i in range(8)]
        res = []
        for p in ps:
            out, err = p.communicate(timeout=600)
            if p.returncode != 0:
                raise RuntimeError(err[-2000:])
            res.append(json.loads(out.strip().splitlines()[-1]))
        wall = time.perf_counter() - t0
        allocs = sum(r["allocs"] for r in res)
        slowest = max(r["seconds"] for r in res)
        # crash reclaim: a client holding 16 allocations is SIGKILLed
        with api.Client(daemon_rank=0, gpu=0, ns=m.ns) as c:
            # (leases from the churn may serve the crasher's allocations, so watch the
            # daemon's reclaim counter rather than HBM usage)
            before = c.stats(3)["n_reclaimed"]
            p = subprocess.Popen([sys.executable, "-c", CRASH.format(repo=REPO, ns=m.ns)], stdout=subprocess.PIPE,
                                 text=True)
            assert "holding" in p.stdout.readline()
            p.wait(timeout=60)
            t_kill = time.perf_counter()
            while c.stats(3)["n_reclaimed"] < before + 16 and time.perf_counter() - t_kill < 10:
                time.sleep(0.0002)
            reclaim_ms = (time.perf_counter() - t_kill) * 1e3
            reclaimed = c.stats(3)["n_reclaimed"] - before
        return {"clients": 8, "daemons": 4, "allocs_total": allocs, "verified_roundtrips": allocs,
                "allocs_per_s_aggregate": round(allocs / slowest, 1), "wall_s": round(wall, 2),
                "crash_reclaim_ms": round(reclaim_ms, 2), "reclaimed_allocations": reclaimed,
                "note": "each churn allocation is also written, read back and checked (64 KiB)"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    out = {"config1_local_alloc_cpu": config1(), "config2_remote_pair_same_gpu": config2(),
           "config3": "8-GPU all-to-all: driver scaling run of bench.py",
           "config4_spill": config4(), "config5_churn_crash": config5()}
    print(json.dumps(out, indent=1))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()

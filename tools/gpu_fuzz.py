"""Randomised put/get against a host-side shadow of both halves.

Every step picks an operation at random:
- write random bytes into the local half
- blocking or async put/get of a random (size, local offset, remote offset)
- a batch of disjoint ops in one launch
- a plan of 1-3 such batches built into a HIP graph and replayed twice (GPU only)
- torch writes on one stream -> async op after ocm_stream_wait -> snapshot on another stream after
  ocm_stream_signal, with no host sync in between (GPU only)
- a full read-back check
Sizes run from 1 B to 24 MiB, so every path is drawn: copy-service solo and gang, launch path, DMA engines,
unaligned heads and tails, and stripe-unit crossings. After each step the local half must equal its shadow.
The remote half is checked through full gets. The pair is placed on a loopback HBM owner, a striped HBM pair,
or the pinned host tier, or (config `net`) on a daemon of another "node", through the network tier's data server.
Config `copy` fuzzes two-sided ocm_copy between allocations of every kind.

    python tools/gpu_fuzz.py [--seconds 60] [--seed 1] [--configs hbm,stripe,host] [--out f.json]

Exit 0 and one JSON line when every check passed. On the first mismatch it exits 1 and names the step.
"""
from __future__ import annotations

import argparse
import contextlib
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402

CONFIGS = {
    # name: (daemons, policy, alloc flags name, stripe unit)
    "hbm": (2, "ring", "OCM_ALLOC_LOOPBACK", 0),
    "stripe": (4, "stripe", "OCM_ALLOC_STRIPE", 64 << 10),
    "host": (2, "ring", "OCM_ALLOC_HOST_TIER", 0),
    # the owner on another "node" (OCM_HOST_ALIAS): the network tier's data server
    "net": (2, "ring", "OCM_ALLOC_NO_SPILL", 0),
}
RANK_ENV = {"net": {0: {"OCM_HOST_ALIAS": "nodeA"}, 1: {"OCM_HOST_ALIAS": "nodeB"}}}
NO_PLANS = {"net"}  # plans need device-addressable extents


def _size(rng, cap):
    r = rng.random()
    if r < 0.35:
        n = int(rng.integers(1, 4097))            # small: service solo, odd sizes
    elif r < 0.7:
        n = int(rng.integers(4096, 1 << 20))      # mid: service gang
    elif r < 0.92:
        n = int(rng.integers(1 << 20, 8 << 20))   # launch path / host-tier gang
    else:
        n = int(rng.integers(8 << 20, 24 << 20))  # above the service limits
    return max(1, min(n, cap))


def fuzz(client, api, name, seconds, seed, nbytes):
    import torch

    daemons, policy, flag, unit = CONFIGS[name]
    flags = getattr(api, flag)
    a = client.alloc(api.OCM_REMOTE_GPU if client.device >= 0 else api.OCM_REMOTE_RDMA, local_bytes=nbytes,
                     remote_bytes=nbytes, flags=flags, stripe_unit=unit)
    if name == "net" and not all(e["net"] for e in a.remote_info()["extents"]):
        raise AssertionError(f"net: the remote half is not on another node: {a.remote_info()}")
    rng = np.random.default_rng(seed)
    local = a.local_tensor()
    on_dev = local.is_cuda
    shadow_l = np.zeros(nbytes, dtype=np.uint8)
    shadow_r = np.zeros(nbytes, dtype=np.uint8)
    local.zero_()
    a.put(0, 0, nbytes)  # both halves zero
    if on_dev:
        torch.cuda.synchronize()

    def sync_local():
        if on_dev:
            torch.cuda.synchronize()

    def check_local(step, what):
        got = local.cpu().numpy() if on_dev else local.numpy()
        bad = np.flatnonzero(got != shadow_l)
        if bad.size:
            raise AssertionError(f"{name} step {step} ({what}): {bad.size} local bytes differ, first at {bad[0]}")

    def rand_batch():
        # disjoint local and remote ranges: the ops of one batch run concurrently
        k = int(rng.integers(2, 17))
        span = nbytes // k
        lslots, rslots = rng.permutation(k), rng.permutation(k)
        ops = []
        for i in range(k):
            n = int(rng.integers(1, max(2, min(span, 1 << 20))))
            lo = int(lslots[i]) * span + int(rng.integers(0, span - n + 1))
            ro = int(rslots[i]) * span + int(rng.integers(0, span - n + 1))
            ops.append((int(rng.random() < 0.5), lo, ro, n))
        return ops

    def apply_batch(ops):
        for put, lo, ro, n in ops:  # disjoint: order does not matter
            if put:
                shadow_r[ro:ro + n] = shadow_l[lo:lo + n]
        for put, lo, ro, n in ops:
            if not put:
                shadow_l[lo:lo + n] = shadow_r[ro:ro + n]

    streams = (torch.cuda.Stream(device=local.device), torch.cuda.Stream(device=local.device)) if on_dev else None
    counts = {}
    t_end = time.time() + seconds
    step = 0
    while time.time() < t_end:
        step += 1
        r = rng.random()
        if r < 0.15:
            n = _size(rng, nbytes)
            off = int(rng.integers(0, nbytes - n + 1))
            data = rng.integers(0, 256, n, dtype=np.uint8)
            local[off:off + n].copy_(torch.from_numpy(data))
            sync_local()
            shadow_l[off:off + n] = data
            what = "write_local"
        elif r < 0.75:
            n = _size(rng, nbytes)
            loff = int(rng.integers(0, nbytes - n + 1))
            roff = int(rng.integers(0, nbytes - n + 1))
            put = rng.random() < 0.5
            asy = rng.random() < 0.25
            (a.put if put else a.get)(loff, roff, n, async_=asy)
            if asy:
                a.wait()
            if put:
                shadow_r[roff:roff + n] = shadow_l[loff:loff + n]
            else:
                shadow_l[loff:loff + n] = shadow_r[roff:roff + n]
            what = f"{'put' if put else 'get'}{'_async' if asy else ''}"
        elif r < 0.85:
            ops = rand_batch()
            asy = rng.random() < 0.3
            a.batch(ops, async_=asy)
            if asy:
                a.wait()
            apply_batch(ops)
            what = "batch"
        elif r < 0.9 and on_dev and name not in NO_PLANS:
            # a plan: 1-3 batch stages run in order, captured once, replayed twice
            stages = [rand_batch() for _ in range(int(rng.integers(1, 4)))]
            with client.plan() as plan:
                for ops in stages:
                    plan.add(a, ops)
                for _ in range(2):
                    plan.launch()
                    for ops in stages:
                        apply_batch(ops)
            what = "plan"
        elif r < 0.93 and on_dev:
            # Stream interop, no host sync between the steps: torch writes the local
            # half on s1 (behind a GPU sleep, so a missing wait reads stale bytes),
            # the async op waits for s1 (ocm_stream_wait), and s2 snapshots the local
            # half after the op (ocm_stream_signal).
            n = _size(rng, nbytes)
            off = int(rng.integers(0, nbytes - n + 1))
            data = rng.integers(0, 256, n, dtype=np.uint8)
            dev = torch.from_numpy(data).to(local.device)
            torch.cuda.synchronize()
            s1, s2 = streams
            with torch.cuda.stream(s1):
                if hasattr(torch.cuda, "_sleep"):
                    torch.cuda._sleep(200000)
                local[off:off + n].copy_(dev)
            shadow_l[off:off + n] = data
            a.stream_wait(s1)
            m = _size(rng, nbytes)
            loff = int(rng.integers(0, nbytes - m + 1))
            roff = int(rng.integers(0, nbytes - m + 1))
            put = rng.random() < 0.5
            (a.put if put else a.get)(loff, roff, m, async_=True)
            if put:
                shadow_r[roff:roff + m] = shadow_l[loff:loff + m]
            else:
                shadow_l[loff:loff + m] = shadow_r[roff:roff + m]
            a.stream_signal(s2)
            with torch.cuda.stream(s2):
                snap = local.clone()
            s2.synchronize()
            a.wait()
            bad = np.flatnonzero(snap.cpu().numpy() != shadow_l)
            if bad.size:
                raise AssertionError(f"{name} step {step} (streams): snapshot differs at {bad.size} bytes")
            what = "streams_put" if put else "streams_get"
        else:
            # the remote half, through a full get
            a.get(0, 0, nbytes)
            shadow_l[:] = shadow_r
            what = "full_get"
        counts[what] = counts.get(what, 0) + 1
        check_local(step, what)
    a.get(0, 0, nbytes)
    shadow_l[:] = shadow_r
    check_local(step, "final")
    a.free()
    return {"steps": step, "ops": counts}


def fuzz_threads(client, api, name, seconds, seed, nbytes, threads):
    """`threads` threads at once, each on its own pair: the library's shared
    machinery (copy service, lanes, library stream, locks) under concurrency."""
    import threading

    out, errs = [None] * threads, []

    def work(k):
        try:
            out[k] = fuzz(client, api, name, seconds, seed * 100 + k, nbytes // threads)
        except Exception as e:  # noqa: BLE001 - reported below
            errs.append(f"thread {k}: {e}")

    ts = [threading.Thread(target=work, args=(k,)) for k in range(threads)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    if errs:
        raise AssertionError("; ".join(errs))
    return {"threads": threads, "steps": sum(o["steps"] for o in out)}


class _Obj:
    """One allocation and the shadows of its halves."""

    def __init__(self, api, client, kind, nbytes, flags=0):
        import torch

        remote = kind in (api.OCM_REMOTE_GPU, api.OCM_REMOTE_RDMA)
        self.a = client.alloc(kind, local_bytes=nbytes, remote_bytes=nbytes if remote else 0, flags=flags)
        self.remote = remote
        self.t = self.a.local_tensor()
        self.t.zero_()
        if self.t.is_cuda:
            torch.cuda.synchronize()
        self.l = np.zeros(nbytes, dtype=np.uint8)
        self.r = np.zeros(nbytes, dtype=np.uint8) if remote else None
        if remote:
            self.a.put(0, 0, nbytes)

    def local_now(self):
        return self.t.cpu().numpy() if self.t.is_cuda else self.t.numpy().copy()


def fuzz_copy(client, api, seconds, seed, nbytes):
    """ocm_copy (two-sided) between random kinds, modelled step by step:
    op_flag 0 swaps dst and src; local->remote stages through dst's local half
    (local[src_offset_2] -> remote[dest_offset_2]); remote->local reads into
    src's local half first; remote->remote copies directly."""
    import torch

    rng = np.random.default_rng(seed)
    on_gpu = client.device >= 0
    kinds = [api.OCM_LOCAL_HOST, api.OCM_REMOTE_RDMA, api.OCM_REMOTE_RDMA]
    if on_gpu:
        kinds += [api.OCM_LOCAL_GPU, api.OCM_REMOTE_GPU, api.OCM_REMOTE_GPU]
    objs = [_Obj(api, client, k, nbytes, api.OCM_ALLOC_HOST_TIER if i % 2 else 0) for i, k in enumerate(kinds)]
    counts = {}
    t_end = time.time() + seconds
    step = 0
    while time.time() < t_end:
        step += 1
        if rng.random() < 0.2:
            o = objs[int(rng.integers(len(objs)))]
            n = _size(rng, nbytes)
            off = int(rng.integers(0, nbytes - n + 1))
            data = rng.integers(0, 256, n, dtype=np.uint8)
            o.t[off:off + n].copy_(torch.from_numpy(data))
            if o.t.is_cuda:
                torch.cuda.synchronize()
            o.l[off:off + n] = data
            what = "write_local"
        else:
            i, j = rng.choice(len(objs), 2, replace=False)
            dst, src = objs[int(i)], objs[int(j)]
            n = _size(rng, nbytes)
            so, do, so2, do2 = (int(rng.integers(0, nbytes - n + 1)) for _ in range(4))
            flag = int(rng.random() < 0.6)
            api.copy(dst.a, src.a, n, src_offset=so, dest_offset=do, src_offset_2=so2, dest_offset_2=do2,
                     op_flag=flag)
            d, sr = (dst, src) if flag else (src, dst)
            if not sr.remote and not d.remote:
                d.l[do:do + n] = sr.l[so:so + n]
            elif not sr.remote and d.remote:
                d.l[do:do + n] = sr.l[so:so + n]
                d.r[do2:do2 + n] = d.l[so2:so2 + n]
            elif sr.remote and not d.remote:
                sr.l[so2:so2 + n] = sr.r[do2:do2 + n]
                d.l[do:do + n] = sr.l[so:so + n]
            else:
                d.r[do:do + n] = sr.r[so:so + n]
            what = ("local" if not sr.remote else "remote") + "_to_" + ("local" if not d.remote else "remote")
        counts[what] = counts.get(what, 0) + 1
        for k, o in enumerate(objs):
            bad = np.flatnonzero(o.local_now() != o.l)
            if bad.size:
                raise AssertionError(f"copy step {step} ({what}): object {k} local differs at {bad.size} bytes")
    for k, o in enumerate(objs):  # remote halves, through full gets
        if o.remote:
            o.a.get(0, 0, nbytes)
            if not np.array_equal(o.local_now(), o.r):
                raise AssertionError(f"copy final: object {k} remote half differs")
        o.a.free()
    return {"steps": step, "ops": counts}


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=60)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--configs", default="hbm,stripe,host,copy")
    ap.add_argument("--bytes", type=int, default=32 << 20)
    ap.add_argument("--threads", type=int, default=1, help="threads, each fuzzing its own pair at once")
    ap.add_argument("--ns", default=None, help="attach to this running mesh instead of starting one per config")
    ap.add_argument("--daemon-rank", type=int, default=0)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()

    from oncilla_amd import api
    from oncilla_amd.parallel.mesh import Mesh

    import torch

    gpu = 0 if torch.cuda.device_count() > 0 and not os.environ.get("OCM_NO_GPU") else None
    res = {}
    for i, name in enumerate(args.configs.split(",")):
        daemons, policy, _, _ = CONFIGS.get(name, (2, "ring", None, 0))
        with contextlib.ExitStack() as stack:
            # --ns: attach to a running mesh (several fuzzing apps at once); else a mesh per config
            ns = args.ns or stack.enter_context(Mesh(daemons, gpus=[gpu] * daemons, policy=policy,
                                                     rank_env=RANK_ENV.get(name))).ns
            with api.Client(daemon_rank=args.daemon_rank, gpu=gpu, ns=ns) as c:
                try:
                    secs = args.seconds / len(args.configs.split(","))
                    if name == "copy":
                        res[name] = fuzz_copy(c, api, secs, args.seed + i, min(args.bytes, 8 << 20))
                    elif args.threads > 1:
                        res[name] = fuzz_threads(c, api, name, secs, args.seed + i, args.bytes, args.threads)
                    else:
                        res[name] = fuzz(c, api, name, secs, args.seed + i, args.bytes)
                except AssertionError as e:
                    print(json.dumps({"ok": False, "config": name, "error": str(e)}), flush=True)
                    return 1
        print(name, json.dumps(res[name]), flush=True)
    # a run is clean only if no copy-service op timed out
    # (no 10 s stall, no fallback to launches) and no instance left an op unfinished.
    health = api.service_health()
    ok = health["aborts"] == 0 and health["incomplete_exits"] == 0 and not health["wedged"]
    line = json.dumps({"ok": ok, "seed": args.seed, "bytes": args.bytes, "configs": res, "service_health": health})
    if args.out:
        with open(args.out, "w") as f:
            f.write(line + "\n")
    print(line)
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())

#!/usr/bin/env python3
"""Headline benchmark: remote one-sided put/get GiB/s + p50 ocm_alloc latency.

BASELINE.json metric: "remote put/get GiB/s + p50 ocm_alloc latency, 4 KiB-1 GiB,
1/2/4/8 MI355X". The workload is the reference's R/W sweep (`ocm_test 4`,
reference test/ocm_test.c:323-425): a 2 GiB+1 remote pair, one-sided reads and
writes of every power-of-two size — here 4 KiB .. 1 GiB — each op blocking, as
in the reference. The reference never timed it; we do.

One step = for every size s: get(s) then put(s), on every rank concurrently.
Each rank is one app process on its own MI355X with its own ocmd daemon; the
daemons form one mesh (rank0 = master/placement). Remote halves are placed by
the governor:
  pattern "stripe" (default): striped over every peer GPU (all xGMI links),
  pattern "ring": reference placement (orig_rank + 1) % N, one peer per rank.
With a single GPU there is no peer HBM: the remote half lives in the daemon's
pinned host tier (PCIe), like the reference's single-node coercion to host
memory (src/alloc.c:82-83).

  python bench.py [--gpus N --steps K --warmup W]
  torchrun --nproc-per-node N bench.py --gpus N ...
Rank 0 prints ONE JSON line. value = total bytes moved by all ranks per
second (GiB/s) over the K timed steps, timed max-over-ranks.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

METRIC = "remote put/get GiB/s + p50 ocm_alloc latency, 4 KiB-1 GiB, 1/2/4/8 MI355X"
GiB = float(1 << 30)


def parse():
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=None)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--device", choices=["auto", "gpu", "cpu"], default="auto")
    ap.add_argument("--min-bytes", type=int, default=4096)
    ap.add_argument("--max-bytes", type=int, default=None, help="largest transfer (default 1 GiB; 16 MiB on CPU)")
    ap.add_argument("--pattern", choices=["stripe", "ring"], default="stripe")
    ap.add_argument("--remote", choices=["auto", "loopback", "host"], default="auto",
                    help="auto: governor placement; loopback: the rank's own daemon HBM (IPC); host: pinned host tier")
    ap.add_argument("--alloc-samples", type=int, default=200)
    ap.add_argument("--no-characterize", action="store_true")
    ap.add_argument("--no-autotune", action="store_true",
                    help="N>1: skip the setup-time kernel autotune over the xGMI links (library defaults)")
    ap.add_argument("--no-hw-baseline", action="store_true", help="skip the N>1 runtime peer-copy extras")
    ap.add_argument("--no-optim-extra", action="store_true", help="skip the fused remote-Adam extra")
    ap.add_argument("--no-ctrl-extra", action="store_true",
                    help="N>1: skip the control-plane extra (alloc p50 with the records on TCP vs RCCL ticks)")
    ap.add_argument("--json-out", default=None)
    return ap.parse_args()


def coord_init(world: int):
    """gloo group for coordination only: touches no GPU, so every rank can
    start its daemon before HIP is initialised in this process. Every
    collective is bounded (OCM_BENCH_TIMEOUT_S, default 300 s): a rank that
    hangs makes the others fail with a diagnostic instead of burning the
    job's time limit."""
    if world <= 1:
        return None
    from datetime import timedelta

    import torch.distributed as dist

    dist.init_process_group("gloo", timeout=timedelta(seconds=float(os.environ.get("OCM_BENCH_TIMEOUT_S", "300"))))
    return dist


def gather_obj(dist, obj, world):
    if dist is None:
        return [obj]
    out = [None] * world
    dist.all_gather_object(out, obj)
    return out


class BenchAbort(RuntimeError):
    """A phase failed on at least one rank; every rank raises it together."""

    def __init__(self, phase: str, errors: dict):
        super().__init__(f"phase {phase!r} failed on rank(s) {sorted(errors, key=int)}")
        self.phase = phase
        self.errors = errors


class Phases:
    """Run each setup/measurement step on every rank, then agree on the outcome.

    A step that raises on one rank is published through the same all-gather the
    other ranks wait on, so all of them stop together (BenchAbort) instead of
    waiting in a barrier the failed rank never reaches. Test hook:
    OCM_BENCH_RAISE="<rank>:<phase>" raises inside that phase on that rank
    (OCM_BENCH_RAISE_ONCE: only the first time that phase runs)."""

    def __init__(self, dist, world: int, rank: int):
        self.dist, self.world, self.rank = dist, world, rank
        self.current = "init"
        inj = os.environ.get("OCM_BENCH_RAISE", "")
        self.inject = tuple(inj.split(":", 1)) if ":" in inj else None
        once = os.environ.get("OCM_BENCH_RAISE_ONCE", "")  # the same, first run of the phase only
        self.inject_once = tuple(once.split(":", 1)) if ":" in once else None

    def run(self, name: str, fn):
        self.current = name
        if self.rank == 0:
            # progress on stderr (stdout carries only the final JSON line): a long N=8 setup
            # (RCCL bootstrap, autotune) is never mistaken for a hang by a silence watchdog
            print(f"[bench] {time.strftime('%H:%M:%S')} phase {name}", file=sys.stderr, flush=True)
        val, err = None, None
        try:
            if self.inject and int(self.inject[0]) == self.rank and self.inject[1] == name:
                raise RuntimeError(f"injected failure (OCM_BENCH_RAISE) in phase {name}")
            if self.inject_once and int(self.inject_once[0]) == self.rank and self.inject_once[1] == name:
                self.inject_once = None
                raise RuntimeError(f"injected failure (OCM_BENCH_RAISE_ONCE) in phase {name}")
            val = fn()
        except Exception as e:  # noqa: BLE001 - published to every rank below
            err = f"{type(e).__name__}: {e}"[:600]
            print(f"rank {self.rank}: phase {name} failed: {err}", file=sys.stderr, flush=True)
        res = gather_obj(self.dist, {"err": err}, self.world)
        errs = {str(i): r["err"] for i, r in enumerate(res) if r["err"]}
        if errs:
            raise BenchAbort(name, errs)
        return val


def _local(fn):
    """Run a rank-local measurement; (value, None) or (None, error string)."""
    try:
        return fn(), None
    except Exception as e:  # noqa: BLE001 - recorded, never fatal
        return None, repr(e)[:200]


def hw_baseline_extras(dist, world: int, rank: int, local_rank: int) -> dict:
    """The runtime's own peer copy (ring r -> r+1, all ranks at once) and rank 0's link table."""
    import torch

    from oncilla_amd import api

    out = {}
    peer = (local_rank + 1) % world
    n_b = 256 << 20
    visible = bool(_local(lambda: torch.cuda.device_count() >= world)[0])
    bufs, err = _local(lambda: (torch.empty(n_b, dtype=torch.uint8, device=f"cuda:{local_rank}"),
                                torch.empty(n_b, dtype=torch.uint8, device=f"cuda:{peer}")) if visible else None)

    def run(reps):
        src, dst = bufs
        t0 = time.perf_counter()
        for _ in range(reps):
            dst.copy_(src)
        torch.cuda.synchronize(local_rank)
        torch.cuda.synchronize(peer)
        return (time.perf_counter() - t0) / reps

    if bufs:
        _, err = _local(lambda: run(1))
    if dist is not None:
        dist.barrier()
    tb = None
    if bufs and not err:
        tb, err = _local(lambda: run(3))
    res = gather_obj(dist, {"t": tb, "err": err, "visible": visible}, world)
    if all(r["visible"] for r in res):
        errs = [r["err"] for r in res if r["err"]]
        out["torch_peer_copy_ring_256MiB_GiBps"] = (
            {"error": errs[0]} if errs else round(world * n_b / max(r["t"] for r in res) / GiB, 2))
    if rank == 0:
        links, _ = _local(lambda: {str(p): api.link_info(local_rank, p) for p in range(world) if p != local_rank})
        if links:
            out["links_from_rank0"] = links
    del bufs
    return out

def optim_extra(client, dist, world: int, local_rank: int, elems: int = 64 << 20) -> dict:
    """Fused remote-Adam step (models.OffloadedAdam) with the optimizer state placed by
    the governor (striped over the peers' HBM for N>1: every rank at once, all-to-all
    over xGMI; the host tier for N=1). After the timed region; never affects the metric."""
    import torch

    from oncilla_amd.models import OffloadedAdam

    synced = [False]

    def run():
        p = torch.zeros(elems, device=f"cuda:{local_rank}").requires_grad_()
        p.grad = torch.randn(elems, device=f"cuda:{local_rank}")
        opt = OffloadedAdam([p], client, lr=1e-3)
        try:
            ext = opt.allocs[0].remote_info()["extents"]
            for _ in range(2):
                opt.step()
            torch.cuda.synchronize(local_rank)
            if dist is not None:
                synced[0] = True
                dist.barrier()
            t0 = time.perf_counter()
            for _ in range(5):
                opt.step()
            torch.cuda.synchronize(local_rank)
            return {"s": (time.perf_counter() - t0) / 5, "extents": len(ext),
                    "tier": "+".join(sorted({{1: "host", 2: "hbm"}[e["tier"]] for e in ext}))}
        finally:
            opt.close()

    r, err = _local(run) if dist is None else (None, None)
    if dist is not None:
        # every rank reaches the barrier inside run() or this one, then the gather
        try:
            r = run()
        except Exception as e:  # noqa: BLE001 - recorded
            err = repr(e)[:200]
            if not synced[0]:
                dist.barrier()
    res = gather_obj(dist, {"r": r, "err": err}, world)
    errs = [x["err"] for x in res if x["err"]]
    if errs:
        return {"error": errs[0]}
    t = max(x["r"]["s"] for x in res)
    return {"params_per_rank": elems, "ms_per_step": round(t * 1e3, 3), "state_tier": res[0]["r"]["tier"],
            "state_extents": res[0]["r"]["extents"],
            "state_GiBps_per_rank": round(16 * elems / t / (1 << 30), 2)}


def peer_table(client, use_gpu: bool, world: int, rank: int, local_rank: int, nbytes: int) -> dict:
    """Rank 0 alone, after the timed region: one remote pair on each peer in
    turn (remote_rank = p, unloaded links), blocking put/get of `nbytes`, and
    the link type/hops between the two GPUs. The per-link view of the striped
    all-to-all number (reference: one pair per remote node, test/ocm_test.c:323-425)."""
    from oncilla_amd import api

    out = {}
    if rank != 0:
        return out
    kind = api.OCM_REMOTE_GPU if use_gpu else api.OCM_REMOTE_RDMA
    for p in range(world):
        if p == rank:
            continue

        def one():
            a = client.alloc(kind, local_bytes=nbytes, remote_bytes=nbytes, remote_rank=p)
            try:
                ext = a.remote_info()["extents"]
                a.fill(seed=77 + p)
                a.put(0, 0, nbytes)
                a.fill(seed=0)
                a.get(0, 0, nbytes)
                bad = a.check(seed=77 + p)
                if bad:
                    raise RuntimeError(f"{bad} words differ after the round trip to rank {p}")
                t_put = a.time_onesided(1, nbytes, 3)
                t_get = a.time_onesided(0, nbytes, 3)
                row = {"put_GiBps": round(nbytes / t_put / GiB, 2), "get_GiBps": round(nbytes / t_get / GiB, 2),
                       "owner_rank": ext[0]["owner_rank"], "owner_gpu": ext[0]["owner_gpu"],
                       "tier": {1: "host", 2: "hbm"}[ext[0]["tier"]]}
                if use_gpu and ext[0]["owner_gpu"] >= 0:
                    row["link"] = api.link_info(local_rank, ext[0]["owner_gpu"])
                return row
            finally:
                a.free()

        row, err = _local(one)
        out[str(p)] = row if row is not None else {"error": err}
    return out


def ctrl_extra(dist, world: int, rank: int, local_rank: int, use_gpu: bool, samples: int = 100) -> dict:
    """N>1, after the timed region, with the sweep's mesh gone: a fresh mesh per
    control transport (records between daemons on persistent TCP links, then
    on tick collectives: RCCL over xGMI on GPUs, the socket ring on CPU),
    leases off so every allocation takes REQ_ALLOC -> DO_ALLOC -> reply
    through the transport; every rank measures remote ocm_alloc p50 at once."""
    import secrets

    from oncilla_amd import api
    from oncilla_amd.models import workloads as wl
    from oncilla_amd.parallel.mesh import Mesh, free_ports

    out = {}
    kind = api.OCM_REMOTE_GPU if use_gpu else api.OCM_REMOTE_RDMA
    all_gpus = gather_obj(dist, local_rank, world) if use_gpu else []
    for ctrl in ("tcp", "rccl" if use_gpu else "socket"):
        if ctrl == "rccl" and len(set(all_gpus)) < world:
            # RCCL needs one rank per GPU: a one-GPU rehearsal (OCM_BENCH_SHARE_GPU) cannot build the communicator
            out[ctrl] = {"skipped": "ranks share a GPU (RCCL needs one rank per GPU)"}
            continue
        ports, key = gather_obj(dist, (free_ports(world), secrets.token_hex(16)) if rank == 0 else None, world)[0]
        ns = f"ctrl{ctrl}_{ports[0]}"
        gpus = list(all_gpus) if use_gpu else [None] * world
        mesh = Mesh(world, gpus=gpus, ns=ns, policy="ring", ports=ports, ranks=[rank], key=key,
                    workdir=os.path.join("/tmp", f"ocm_{ns}"), extra_args=["--ctrl", ctrl],
                    env={"OCM_LEASE_BYTES": "0"})
        os.makedirs(mesh.workdir, exist_ok=True)
        up, err = _local(lambda: mesh.start(timeout=60))
        res = gather_obj(dist, {"err": err}, world)
        r, err = None, next((x["err"] for x in res if x["err"]), None)
        if err is None:
            def run():
                with api.Client(daemon_rank=rank, gpu=(local_rank if use_gpu else None), ns=ns) as c:
                    up = True
                    if ctrl != "tcp":
                        # The transport comes up after the mesh is complete (an RCCL
                        # communicator over 8 GPUs can take seconds to initialise);
                        # until then records ride TCP.
                        deadline = time.time() + 30
                        while c.stats(rank)["ctrl_ticks"] == 0 and time.time() < deadline:
                            c.alloc(kind, local_bytes=4096, remote_bytes=1 << 20).free()
                        up = c.stats(rank)["ctrl_ticks"] > 0
                    lat = wl.alloc_latency(c, kind, samples, local_bytes=4096, remote_bytes=1 << 20)
                    lat["ticks"] = c.stats(rank)["ctrl_ticks"]
                    lat["up"] = up
                    # this rank's records from post to delivery in a gathered tick (one hop)
                    lat["tick"] = api.tick_stats() if ctrl != "tcp" else None
                    return lat

            r, err = _local(run)
        res = gather_obj(dist, {"r": r, "err": err}, world)
        _local(mesh.stop)
        errs = [x["err"] for x in res if x["err"]]
        if errs:
            out[ctrl] = {"error": errs[0]}
            continue
        out[ctrl] = {"alloc_p50_us": round(max(x["r"]["alloc_p50_us"] for x in res), 2),
                     "alloc_p99_us": round(max(x["r"]["alloc_p99_us"] for x in res), 2),
                     "free_p50_us": round(max(x["r"]["free_p50_us"] for x in res), 2),
                     "ticks_rank0": res[0]["r"]["ticks"], "samples_per_rank": samples,
                     "transport_up_all_ranks": all(x["r"]["up"] for x in res)}
        ticks = [x["r"].get("tick") for x in res]
        if any(ticks):
            out[ctrl]["hop_mean_us_per_rank"] = [t["hop_mean_us"] if t else None for t in ticks]
            # the hop split: waiting for a tick / the tick itself / the event loop's pickup
            out[ctrl]["hop_split_us_rank0"] = ({k: ticks[0][k] for k in ("hop_wait_mean_us", "hop_exec_mean_us",
                                                                          "deliver_mean_us")} if ticks[0] else None)
            out[ctrl]["tick_period_mean_us_rank0"] = ticks[0]["tick_period_mean_us"] if ticks[0] else None
            out[ctrl]["start_mean_us_rank0"] = ticks[0]["start_mean_us"] if ticks[0] else None
            # idle ticks instead of TCP wake-ups (OCM_TICK_IDLE_US): no rank woke a peer over TCP
            out[ctrl]["tcp_wakes_all_ranks"] = sum(t["tcp_wakes"] for t in ticks if t)
            out[ctrl]["idle_ticks_rank0"] = ticks[0]["idle_ticks"] if ticks[0] else None
    return out


def error_result(world: int, args, phase: str, errors: dict) -> dict:
    return {"metric": METRIC, "value": None, "unit": "GiB/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "uint8", "error": f"phase {phase!r} failed", "phase": phase, "rank_errors": errors}


def main() -> int:
    args = parse()
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    n_gpus = args.gpus if args.gpus is not None else world
    if n_gpus != world:
        print(f"--gpus {n_gpus} but WORLD_SIZE={world}; launch with torch.distributed.run for N>1", file=sys.stderr)
        return 2

    import torch  # noqa: F401  (device count without HIP init)

    ndev = torch.cuda.device_count()
    use_gpu = args.device == "gpu" or (args.device == "auto" and ndev > 0)
    if use_gpu and os.environ.get("OCM_BENCH_SHARE_GPU"):
        # Rehearsal mode for a 1-GPU box: every rank (and daemon) on GPU 0, so the
        # N-rank mesh, placement and IPC paths run without N devices.
        local_rank = 0
    max_bytes = args.max_bytes or ((1 << 30) if use_gpu else (16 << 20))
    if use_gpu:
        # This benchmark opts in to the library's app pinning (OCM_PIN=1: the thread
        # that calls ocm_init, and what it starts later, on the GPU's L3 complex,
        # off the daemon's core). Measured on one box: 4 KiB get/put 5.04 / 4.17 us
        # pinned, 5.11-5.15 / 4.19-4.26 unpinned, 6.07-6.45 / 5.21-5.89 with the
        # process confined to the GPU's NUMA node (profiles/numa_small_r03.json).
        # The library itself leaves applications unpinned unless they ask.
        os.environ.setdefault("OCM_PIN", "1")

    from oncilla_amd import api
    from oncilla_amd.models import workloads as wl
    from oncilla_amd.parallel.mesh import Mesh, free_ports
    from oncilla_amd.utils.paths import is_built

    dist = coord_init(world)
    ph = Phases(dist, world, rank)
    mesh = client = None
    result, rc = {}, 0
    try:
        def setup():
            if use_gpu and local_rank >= ndev:
                raise RuntimeError(f"LOCAL_RANK {local_rank} but only {ndev} GPUs visible")
            if rank == 0 and not is_built():
                from oncilla_amd.utils.build import build

                build()

        ph.run("setup", setup)
        # ---- daemon mesh: one ocmd per rank / GPU ----
        # rank 0 picks every daemon port while holding them all bound, so no two
        # ranks of this node can be handed the same ephemeral port
        import secrets

        ports, mesh_key = gather_obj(dist, (free_ports(world), secrets.token_hex(16)) if rank == 0 else None, world)[0]
        ns = f"bench{os.environ.get('MASTER_PORT', '0')}_{ports[0]}"
        workdir = os.path.join("/tmp", f"ocm_{ns}")
        os.makedirs(workdir, exist_ok=True)
        gpus = [(local_rank if use_gpu else None) for _ in range(world)]
        if use_gpu:
            # every rank's GPU ordinal (single node: LOCAL_RANK == RANK)
            gpus = gather_obj(dist, local_rank, world)
        policy = "stripe" if args.pattern == "stripe" else "ring"
        # Fault-injection hook for rehearsals: OCM_BENCH_FAULT="<rank>:<OCM_FAULT spec>"
        # gives that rank's daemon the spec (csrc/src/daemon/mesh.cpp fault injection).
        rank_env = {}
        bf = os.environ.get("OCM_BENCH_FAULT", "")
        if ":" in bf:
            fr, spec = bf.split(":", 1)
            rank_env[int(fr)] = {"OCM_FAULT": spec}
        mesh = Mesh(world, gpus=gpus, ns=ns, policy=policy, workdir=workdir, ports=ports, ranks=[rank],
                    rank_env=rank_env, key=mesh_key)
        ph.run("mesh_start", lambda: mesh.start(timeout=120))

        def attach():
            c = api.Client(daemon_rank=rank, gpu=(local_rank if use_gpu else None), ns=ns)
            if not use_gpu:
                os.environ["OCM_NO_GPU"] = "1"
            c.init()
            return c

        client = ph.run("client_init", attach)
        remote_kind = api.OCM_REMOTE_GPU if use_gpu else api.OCM_REMOTE_RDMA

        rflags = {"auto": 0, "loopback": api.OCM_ALLOC_LOOPBACK, "host": api.OCM_ALLOC_HOST_TIER}[args.remote]
        # Peer HBM unusable on this node (e.g. cross-device IPC refused on the first real
        # multi-GPU node): measure with the remote halves in the peers' pinned host tiers
        # instead of reporting nothing, and say so in the JSON (fallback, config.remote_tier).
        can_fall_back = world > 1 and args.remote == "auto"
        fallback = None

        # ---- p50 ocm_alloc latency (remote pair, and the local malloc path) ----
        def latency(flags):
            def run():
                st0, _ = _local(lambda: client.stats(rank))
                link0 = api.counters()["n_link_rpc"]
                lat_remote = wl.alloc_latency(client, remote_kind, args.alloc_samples, local_bytes=64 << 10,
                                              remote_bytes=1 << 20, flags=flags)
                link1 = api.counters()["n_link_rpc"]
                st1, _ = _local(lambda: client.stats(rank))
                lat_local = wl.alloc_latency(client, api.OCM_LOCAL_HOST, args.alloc_samples, local_bytes=1 << 20)
                leases = st1["lease_allocs"] if st1 else None
                if st0 and st1:
                    # How the remote allocations were served: carved from a capacity lease
                    # (no daemon<->daemon record) or through the mesh on the control transport.
                    # app_link_rpcs: the app's requests that rode the shared-memory link to its daemon
                    lat_remote["via"] = {"lease": st1["lease_allocs"] - st0["lease_allocs"],
                                         "ctrl": st1["ctrl"], "ctrl_ticks": st1["ctrl_ticks"] - st0["ctrl_ticks"],
                                         "app_link_rpcs": link1 - link0}
                return lat_remote, lat_local, leases

            return run

        try:
            lat_remote, lat_local, leases = ph.run("alloc_latency", latency(rflags))
        except BenchAbort as e:
            if not can_fall_back:
                raise
            fallback = {"from": "peer hbm", "to": "peer host tier", "phase": e.phase, "rank_errors": e.errors}
            rflags = api.OCM_ALLOC_HOST_TIER
            lat_remote, lat_local, leases = ph.run("alloc_latency", latency(rflags))

        # ---- the sweep pair: 2 x max + 1 bytes each side (reference: 2 GiB + 1) ----
        pair_bytes = 2 * max_bytes + 1

        # verify: pattern -> put -> clobber -> get -> check
        def verify(pair):
            pair.fill(seed=1234 + rank, nbytes=max_bytes)
            pair.put(0, 0, max_bytes)
            pair.fill(seed=0, nbytes=max_bytes)
            pair.get(0, 0, max_bytes)
            bad = pair.check(seed=1234 + rank, nbytes=max_bytes)
            if bad:
                raise RuntimeError(f"{bad} words differ after put/get round trip")

        def prepare(flags):
            """Allocate the pair, pick the kernel configuration over the links (setup,
            untimed: every rank at once, the slowest rank decides; CPU runs do it too,
            so the multi-rank protocol is tested) and verify a round trip."""
            held = {}

            def alloc():
                held["pair"] = client.alloc(remote_kind, local_bytes=pair_bytes, remote_bytes=pair_bytes, flags=flags)
                return held["pair"]

            try:
                pair = ph.run("pair_alloc", alloc)
                tuned = None
                if world > 1 and not args.no_autotune:
                    tuned = ph.run("autotune", lambda: wl.autotune(pair, min(256 << 20, max_bytes), reps=5,
                                                                   gather=lambda obj: gather_obj(dist, obj, world)))
                ph.run("verify", lambda: verify(pair))
                return pair, tuned
            except BenchAbort:
                if "pair" in held:
                    _local(held["pair"].free)
                raise

        try:
            pair, tuned = prepare(rflags)
        except BenchAbort as e:
            if not can_fall_back or fallback is not None:
                raise
            fallback = {"from": "peer hbm", "to": "peer host tier", "phase": e.phase, "rank_errors": e.errors}
            pair, tuned = prepare(api.OCM_ALLOC_HOST_TIER)
        info = pair.remote_info()
        sizes = wl.sweep_sizes(args.min_bytes, max_bytes)

        def warmup():
            for _ in range(args.warmup):
                wl.rw_sweep_step(pair, sizes)

        ph.run("warmup", warmup)

        def sync():
            if use_gpu:
                # the copy service is a persistent kernel: park it, or a device-wide
                # synchronize waits for its idle exit (OCM_SERVICE_IDLE_US, 50 us)
                api.quiesce()
                torch.cuda.synchronize(local_rank)

        # ---- timed region: barrier + sync on both sides; the phase's all-gather is the closing barrier ----
        if dist is not None:
            dist.barrier()
        sync()

        def timed():
            t0 = time.perf_counter()
            moved = 0
            for _ in range(args.steps):
                moved += wl.rw_sweep_step(pair, sizes)
            sync()
            return time.perf_counter() - t0, moved

        elapsed, moved = ph.run("timed", timed)

        # Self-diagnosis of the data path, per rank: peer access, IPC imports of
        # other GPUs' HBM, and the transport that carried this rank's control records.
        def rank_diag():
            d = api.xgmi_diag() if use_gpu else {"device": -1, "peer_access": 0, "ipc_imports": 0, "ipc_failures": 0}
            st, _ = _local(lambda: client.stats(rank))
            d["ctrl"] = st["ctrl"] if st else None
            d["remote_gpus"] = sorted({e["owner_gpu"] for e in info["extents"] if e["tier"] == api.OCM_TIER_GPU})
            if use_gpu:
                # copy-service health: ops that timed out (and fell back to launches),
                # gang ops sized below their width because fewer workgroups were resident
                d["service"] = api.service_health()
            return d

        diag, _ = _local(rank_diag)
        # max over ranks of elapsed, sum of bytes
        stats = gather_obj(dist, {"elapsed": elapsed, "moved": moved, "lat": lat_remote, "lat_local": lat_local,
                                  "extents": info["extents"], "leases": leases, "diag": diag}, world)
        t_max = max(s["elapsed"] for s in stats)
        total = sum(s["moved"] for s in stats)

        sweep = {}
        if not args.no_characterize:
            ch = ph.run("characterize", lambda: wl.characterize(pair, sizes, breakdown_max=(4 << 20) if use_gpu else 0))
            chs = gather_obj(dist, ch, world)
            for s in sizes:
                # headline per size: the p50 of ops timed one by one (slowest rank); p99
                # and mean alongside, so an outlier moves p99 rather than the row
                g = max(c[s]["get_s"] for c in chs)
                p = max(c[s]["put_s"] for c in chs)
                sweep[str(s)] = {"get_GiBps": round(world * s / g / GiB, 3), "put_GiBps": round(world * s / p / GiB, 3),
                                 "get_us": round(g * 1e6, 2), "put_us": round(p * 1e6, 2),
                                 "get_p99_us": round(max(c[s]["get_p99_s"] for c in chs) * 1e6, 2),
                                 "put_p99_us": round(max(c[s]["put_p99_s"] for c in chs) * 1e6, 2),
                                 "get_mean_us": round(max(c[s]["get_mean_s"] for c in chs) * 1e6, 2),
                                 "put_mean_us": round(max(c[s]["put_mean_s"] for c in chs) * 1e6, 2),
                                 "ops": min(min(c[s]["get_n"], c[s]["put_n"]) for c in chs),
                                 "relaunches": sum(c[s]["get_relaunches"] + c[s]["put_relaunches"] for c in chs)}
                if chs[0][s].get("service"):
                    # rank 0's copy-service breakdown per op (us): host post, GPU doorbell-seen
                    # -> done, and the crossings (doorbell read + completion write over PCIe)
                    sweep[str(s)]["service_rank0"] = chs[0][s]["service"]
        # ---- small ops after host idle gaps: every rank at once ----
        idle_gap = {}
        if not args.no_characterize:
            ig = ph.run("idle_gap", lambda: wl.idle_gap_latency(pair, 4096))
            igs = gather_obj(dist, ig, world)
            idle_gap.update(wl.merge_idle_gap_rows(igs))
            # the headline small-op rows run pinned (OCM_PIN=1, set above for GPU runs);
            # the library default leaves apps unpinned, so time 4 KiB ops unpinned too
            def unpinned():
                mask = os.sched_getaffinity(0)
                try:
                    os.sched_setaffinity(0, range(os.cpu_count() or 1))
                    out = {}
                    for op, key in ((0, "get"), (1, "put")):
                        xs, _ = pair.time_onesided_samples(op, 4096, 300, cap_s=0.5)
                        out[f"{key}_p50_us"] = round(wl.percentile(xs, 50) * 1e6, 2)
                    return out
                finally:
                    os.sched_setaffinity(0, mask)

            if use_gpu and os.environ.get("OCM_PIN") == "1":
                up, _ = _local(unpinned)
                ups = gather_obj(dist, up, world)
                if all(ups):
                    idle_gap["unpinned_back_to_back"] = {k: max(u[k] for u in ups) for k in ups[0]}
            base = idle_gap.get("0")
            if base and "1000" in idle_gap:
                idle_gap["ratio_1ms_vs_back_to_back"] = {
                    k: round(idle_gap["1000"][f"{k}_p50_us"] / base[f"{k}_p50_us"], 2) for k in ("get", "put")}
        # ---- extras, after the timed region (never affect the metric) ----
        # Every rank reaches every collective below even when its local part
        # fails, so a failure is recorded instead of deadlocking the job.
        optim = {}
        if use_gpu and not args.no_optim_extra:
            optim = optim_extra(client, dist, world, local_rank)
        baseline = {}
        if use_gpu and world > 1 and not args.no_hw_baseline:
            baseline = hw_baseline_extras(dist, world, rank, local_rank)
        peers = {}
        if world > 1:
            # every rank is done with the sweep pair's owners before rank 0 loads one link at a time
            gather_obj(dist, None, world)
            peers = peer_table(client, use_gpu, world, rank, local_rank, min(256 << 20, max_bytes))
            gather_obj(dist, None, world)
        ph.run("free", pair.free)

        value = total / t_max / GiB
        tiers = sorted({e["tier"] for s in stats for e in s["extents"]})
        diags = [s["diag"] or {} for s in stats]
        # xGMI carried the sweep only if every rank's remote half sat in OTHER GPUs'
        # HBM, imported over IPC with peer access: a fallback or a host tier is PCIe.
        xgmi = bool(world > 1 and not fallback and tiers == [api.OCM_TIER_GPU] and all(
            d.get("peer_access", 0) >= 1 and d.get("ipc_imports", 0) >= 1 and d.get("remote_gpus")
            and d.get("device", -1) not in d["remote_gpus"] for d in diags))
        result = {
            "metric": METRIC,
            "value": round(value, 3),
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(t_max / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "uint8",
            "data": "synthetic (hash-pattern fill, put/get round trip verified on device)",
            "config": {
                "model": "ocm_test-4 R/W sweep, 2x1GiB+1 remote pair per rank" if max_bytes == 1 << 30
                else f"ocm_test-4 R/W sweep, max {max_bytes} B",
                "global_batch": world,
                "seq_len": max_bytes,
                "parallelism": f"{args.pattern}{world}",
                "pattern": args.pattern,
                "remote": args.remote,
                "remote_tier": "+".join({1: "host", 2: "hbm"}[t] for t in tiers),
                "extents_per_pair": len(stats[0]["extents"]),
                "sizes": f"{args.min_bytes}..{max_bytes} x2",
                "device": "gpu" if use_gpu else "cpu",
                "app_pin": os.environ.get("OCM_PIN", "") if use_gpu else "",
            },
            "alloc_p50_us": round(max(s["lat"]["alloc_p50_us"] for s in stats), 2),
            "alloc_p99_us": round(max(s["lat"]["alloc_p99_us"] for s in stats), 2),
            "free_p50_us": round(max(s["lat"]["free_p50_us"] for s in stats), 2),
            "local_alloc_p50_us": round(max(s["lat_local"]["alloc_p50_us"] for s in stats), 2),
            "alloc_p50_us_per_rank": [round(s["lat"]["alloc_p50_us"], 2) for s in stats],
            "lease_allocs_per_rank": [s["leases"] for s in stats],
            "alloc_via_per_rank": [s["lat"].get("via") for s in stats],
            "xgmi": xgmi,
            "ranks": diags,
            # no copy-service op timed out on any rank (no 10 s stall, no fallback to launches)
            "service_clean": all(not d.get("service") or (d["service"]["aborts"] == 0 and
                                                          d["service"]["incomplete_exits"] == 0) for d in diags),
            "sweep": sweep,
        }
        if idle_gap:
            # 4 KiB blocking get/put after 0 / 100 / 1000 / 10000 us of host idle: p50 / p99
            # (us, slowest rank) and copy-service relaunches (all ranks)
            result["idle_gap_4k"] = idle_gap
        if tuned:
            result["autotune"] = tuned
        if fallback:
            result["fallback"] = fallback
        if optim:
            result["fused_remote_adam"] = optim
        if baseline:
            result["hw_baseline"] = baseline
        if peers:
            result["peers_from_rank0"] = peers
        if world > 1 and not args.no_ctrl_extra:
            # needs this process's library detached from the sweep's mesh first
            _local(client.close)
            client = None
            _local(mesh.stop)
            mesh = None
            result["control_plane"] = ctrl_extra(dist, world, rank, local_rank, use_gpu)
    except BenchAbort as e:
        result, rc = error_result(world, args, e.phase, e.errors), 1
    except Exception as e:  # noqa: BLE001 - a collective timed out or failed: report, never hang
        result, rc = error_result(world, args, ph.current, {str(rank): f"{type(e).__name__}: {e}"[:600]}), 1
    finally:
        if client is not None:
            _local(client.close)
        if mesh is not None:
            _local(mesh.stop)
    if rank == 0:
        line = json.dumps(result)
        print(line, flush=True)
        if args.json_out:
            with open(args.json_out, "w") as f:
                f.write(line + "\n")
    if dist is not None:
        # Rank 0 has printed: only now may a failed rank exit (torchrun tears every
        # worker down as soon as one exits non-zero). Bounded by the group timeout.
        _local(dist.barrier)
        _local(dist.destroy_process_group)
    return rc


if __name__ == "__main__":
    sys.exit(main())

"""bench.py contract on CPU (1 rank, and 2 ranks under torch.distributed.run/gloo)."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
        "vs_baseline", "dtype", "data", "config"}


def _last_json(out):
    lines = [l for l in out.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out
    return json.loads(lines[0])


def test_bench_single(native):
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--device", "cpu", "--steps", "2", "--warmup",
                        "1", "--max-bytes", str(1 << 20), "--alloc-samples", "20"], capture_output=True, text=True,
                       timeout=300, cwd="/tmp")
    assert r.returncode == 0, r.stderr
    res = _last_json(r.stdout)
    assert KEYS <= set(res) and res["n_gpus"] == 1 and res["value"] > 0
    assert res["alloc_p50_us"] > 0 and res["config"]["remote_tier"] == "host"


# "ticks": the main mesh's records ride tick collectives as they would over RCCL on a
# GPU node (--ctrl auto with the socket stand-in), device-sealed and queued 4 at a time
TICK_ENV = {"OCM_CTRL_AUTO_SOCKET": "1", "OCM_TICK_SOCKET_SEAL": "1", "OCM_TICK_SOCKET_BATCH": "4"}


@pytest.mark.parametrize("n,mode", [(2, "tcp"), (8, "tcp"), (8, "ticks")])
def test_bench_multi_rank(native, n, mode):
    # the driver's multi-GPU launch shape (torch.distributed.run, one daemon per rank), on gloo + CPU daemons
    env = dict(os.environ, **(TICK_ENV if mode == "ticks" else {}))
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n),
                        "--master-addr", "127.0.0.1", "--master-port", str(29533 + n + (mode == "ticks")),
                        os.path.join(REPO, "bench.py"),
                        "--gpus", str(n), "--device", "cpu", "--steps", "2", "--warmup", "1", "--max-bytes",
                        str(4 << 20), "--alloc-samples", "20"], capture_output=True, text=True, timeout=300, cwd="/tmp",
                       env=env)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-1500:]
    res = _last_json(r.stdout)
    assert res["n_gpus"] == n and res["value"] > 0 and res["config"]["parallelism"] == f"stripe{n}"
    assert res["config"]["extents_per_pair"] == n - 1  # 8 MiB+1 pair = 9 stripe units: every peer gets one
    # the setup-time autotune ran its all-rank protocol and agreed on one pick per direction
    assert res["autotune"]["ranks"] == n and res["autotune"]["get"] in res["autotune"]["GiBps"], res["autotune"]
    assert len(res["alloc_p50_us_per_rank"]) == n
    # self-diagnosis: every rank reports its data-path state and control transport;
    # CPU ranks move no byte over xGMI, so the flag must say so
    assert res["xgmi"] is False and len(res["ranks"]) == n, res.get("ranks")
    assert all(d["ctrl"] in ("tcp", "socket", "rccl") and d["peer_access"] == 0 for d in res["ranks"]), res["ranks"]
    if mode == "ticks":
        assert all(d["ctrl"] == "socket" for d in res["ranks"]), res["ranks"]
    # control-plane extra: the same allocation path on TCP links and on socket-collective ticks
    cp = res["control_plane"]
    assert "alloc_p50_us" in cp["tcp"] and "alloc_p50_us" in cp["socket"], cp
    assert cp["tcp"]["alloc_p50_us"] > 0 and cp["tcp"]["ticks_rank0"] == 0, cp
    assert cp["socket"]["alloc_p50_us"] > 0 and cp["socket"]["ticks_rank0"] > 0, cp
    # per-rank hop latency of the tick transport (api.tick_stats on every rank; a rank
    # that posted nothing through the ticks has none)
    hops = cp["socket"]["hop_mean_us_per_rank"]
    assert len(hops) == n and all(h is None or h > 0 for h in hops) and any(hops), cp
    assert cp["socket"]["start_mean_us_rank0"] > 0, cp
    # idle ticks: the socket control plane woke nobody over TCP
    assert cp["socket"]["tcp_wakes_all_ranks"] == 0 and cp["socket"]["idle_ticks_rank0"] > 0, cp


def test_bench_extras_helpers_run(native):
    # The N>1 extras only run on multi-GPU nodes (the driver's scaling run):
    # exercise their code here so a Python error cannot hide until then.
    sys.path.insert(0, REPO)
    import bench

    b = bench.hw_baseline_extras(None, 2, 0, 0)
    assert isinstance(b, dict)
    assert bench._local(lambda: 1 / 0)[1].startswith("ZeroDivisionError")


class RoundTrip:
    """The data path of a fake pair for autotune's per-candidate verification: a
    pattern seed travels local -> remote -> local; `corrupt(cfg)` spoils a put."""
    corrupt = staticmethod(lambda cfg: False)

    def fill(self, seed, offset=0, nbytes=None):
        self.local = seed

    def put(self, lo, ro, n):
        self.remote = -1 if self.corrupt(self.cur[1]) else self.local

    def get(self, lo, ro, n):
        self.local = self.remote

    def check(self, seed, offset=0, nbytes=None):
        return 0 if self.local == seed else 17


def test_autotune_picks_fastest_by_slowest_rank(native, monkeypatch):
    """workloads.autotune: per-direction pick by the slowest rank, failing candidates
    excluded, and the same number of collectives on every path (no deadlock)."""
    from oncilla_amd import api
    from oncilla_amd.models import workloads as wl

    cur = {}
    monkeypatch.setattr(api, "set_tuning_dir", lambda op, v, b, nt: cur.__setitem__(op, (v, b, nt)))
    # seconds per (variant, blocks, nt, op) on this rank; the "other rank" is 2x slower on reg_b256 puts
    cands = {"auto": (0, 0, 1), "reg_b256": (1, 256, 1), "lds_default": (2, 0, 1), "broken": (1, 64, 0)}
    mine = {(0, 0, 1): (3.0, 3.0), (1, 256, 1): (2.0, 1.0), (2, 0, 1): (1.5, 2.5)}

    class FakePair(RoundTrip):
        last = None

        def time_onesided(self, op, n, iters):
            cfg = self.last = cur[op]
            if cfg == (1, 64, 0):
                raise RuntimeError("launch failed")
            return mine[cfg][op]

    pair = FakePair()
    pair.cur = cur
    calls = []

    def gather(obj):  # two ranks; the other one is 4x slower with reg_b256
        calls.append(obj)
        if isinstance(obj, tuple) and obj[0] is not None and pair.last == (1, 256, 1):
            return [obj, (obj[0] * 4.0, None)]
        return [obj, obj]

    r = wl.autotune(pair, 1 << 20, gather=gather, candidates=cands)
    assert r["get"] == "lds_default", r
    assert r["put"] == "lds_default", r  # reg_b256 is fastest here but not on the other rank
    assert "error" in r["GiBps"]["broken"]["get"] and "error" in r["GiBps"]["broken"]["put"]
    # 2 gathers per (candidate, direction), 1 for its verification, 1 for the rank count
    assert len(calls) == (2 * 2 + 1) * len(cands) + 1
    assert cur[0] == cands[r["get"]] and cur[1] == cands[r["put"]]


@pytest.mark.parametrize("inject", [("OCM_BENCH_RAISE", "5:verify"), ("OCM_BENCH_FAULT", "3:crash_after_allocs=0")])
def test_bench_eight_ranks_fail_fast(native, inject):
    """A failure on one of 8 ranks (a raised phase, or its daemon dying at the
    first DO_ALLOC) ends every rank within the bound: non-zero exit, and rank 0
    prints one JSON line naming the phase and the failing ranks' messages."""
    import time

    env = dict(os.environ, OCM_BENCH_TIMEOUT_S="90", **{inject[0]: inject[1]})
    t0 = time.time()
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "8",
                        "--master-addr", "127.0.0.1", "--master-port", str(29561 + len(inject[1])),
                        os.path.join(REPO, "bench.py"), "--gpus", "8", "--device", "cpu", "--steps", "1", "--warmup",
                        "1", "--max-bytes", str(1 << 20), "--alloc-samples", "10"], capture_output=True, text=True,
                       timeout=280, cwd="/tmp", env=env)
    assert time.time() - t0 < 270
    assert r.returncode != 0
    res = _last_json(r.stdout)
    assert res["value"] is None and res["error"] and res["rank_errors"], res
    if inject[0] == "OCM_BENCH_RAISE":
        assert res["phase"] == "verify" and list(res["rank_errors"]) == ["5"]


@pytest.mark.parametrize("phase", ["verify", "alloc_latency"])
def test_bench_falls_back_to_host_tier_when_peer_hbm_fails(native, phase):
    """--device gpu paths cannot run here, so drive the fallback on CPU ranks by
    injecting a failure into the first run of a phase: the bench redoes it with the
    remote halves in the host tier and still reports a measured value, with the
    fallback recorded."""
    env = dict(os.environ, OCM_BENCH_RAISE_ONCE=f"1:{phase}")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(29591 + len(phase)), os.path.join(REPO, "bench.py"),
                        "--gpus", "2", "--device", "cpu", "--steps", "1", "--warmup", "1", "--max-bytes",
                        str(1 << 20), "--alloc-samples", "10"], capture_output=True, text=True, timeout=300,
                       cwd="/tmp", env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    res = _last_json(r.stdout)
    assert res["value"] > 0 and res["fallback"]["phase"] == phase and list(res["fallback"]["rank_errors"]) == ["1"]
    assert res["xgmi"] is False  # a fallback is never an xGMI number


def test_autotune_never_installs_the_dma_baseline(native, monkeypatch):
    """the runtime's copy engines stay a reported baseline. Even when
    "dma" is the fastest candidate, a kernel configuration is installed."""
    from oncilla_amd import api
    from oncilla_amd.models import workloads as wl

    cur = {}
    monkeypatch.setattr(api, "set_tuning_dir", lambda op, v, b, nt: cur.__setitem__(op, (v, b, nt)))
    cands = {"auto": (0, 0, 1), "reg_b256": (1, 256, 1), "dma": (3, 0, 1)}
    secs = {(0, 0, 1): 2e-4, (1, 256, 1): 1.5e-4, (3, 0, 1): 1e-4}

    class FakePair(RoundTrip):
        cur = None

        def time_onesided(self, op, n, iters):
            return secs[cur[op]]

    pair = FakePair()
    pair.cur = cur
    r = wl.autotune(pair, 1 << 20, candidates=cands)
    assert r["get"] == "reg_b256" and r["put"] == "reg_b256", r
    assert r["baselines"] == ["dma"] and r["GiBps"]["dma"]["get"] > r["GiBps"]["reg_b256"]["get"], r
    assert cur[0] == (1, 256, 1) and cur[1] == (1, 256, 1)


def test_autotune_drops_a_fast_candidate_that_corrupts_data(native, monkeypatch):
    """The fastest candidate whose round trip comes back wrong (on one rank only)
    is reported as an error and never installed."""
    from oncilla_amd import api
    from oncilla_amd.models import workloads as wl

    cur = {}
    monkeypatch.setattr(api, "set_tuning_dir", lambda op, v, b, nt: cur.__setitem__(op, (v, b, nt)))
    cands = {"auto": (0, 0, 1), "fast_but_wrong": (5, 0, 1), "reg_b256": (1, 256, 1)}
    secs = {(0, 0, 1): 2e-4, (1, 256, 1): 1.5e-4, (5, 0, 1): 0.5e-4}

    class FakePair(RoundTrip):
        def time_onesided(self, op, n, iters):
            return secs[cur[op]]

    pair = FakePair()
    pair.cur = cur
    pair.corrupt = staticmethod(lambda cfg: cfg == (5, 0, 1))

    def gather(obj):  # rank 1 agrees on timings; its verification is the same as ours
        return [obj, obj]

    r = wl.autotune(pair, 1 << 20, gather=gather, candidates=cands)
    assert r["get"] == "reg_b256" and r["put"] == "reg_b256", r
    assert "verification" in r["GiBps"]["fast_but_wrong"]["get"]["error"], r


def _fake_autotune(monkeypatch, secs, cands, gather=None):
    """autotune over a fake pair whose per-config seconds come from secs[(cfg, op)] or secs[cfg]."""
    from oncilla_amd import api
    from oncilla_amd.models import workloads as wl

    cur = {}
    monkeypatch.setattr(api, "set_tuning_dir", lambda op, v, b, nt: cur.__setitem__(op, (v, b, nt)))

    class FakePair(RoundTrip):
        def time_onesided(self, op, n, iters):
            v = secs[cur[op]]
            return v[op] if isinstance(v, tuple) else v

    pair = FakePair()
    pair.cur = cur
    return wl.autotune(pair, 1 << 20, gather=gather, candidates=cands), cur


def test_autotune_keeps_auto_within_the_margin(native, monkeypatch):
    """candidates within 3 % of auto (noise at 5 reps) never
    replace it; one that is 10 % faster on every rank does; the margins are recorded."""
    cands = {"auto": (0, 0, 1), "reg_b256": (1, 256, 1), "lds_default": (2, 0, 1)}
    # get: both candidates 2 % faster (a tie); put: lds_default 10 % faster
    secs = {(0, 0, 1): (1.0, 1.0), (1, 256, 1): (0.98, 0.985), (2, 0, 1): (0.98, 0.90)}
    r, cur = _fake_autotune(monkeypatch, secs, cands)
    assert r["get"] == "auto" and r["put"] == "lds_default", r
    assert r["margin_required"] == 0.03 and r["reps"] == 5
    assert abs(r["margins"]["get"]["reg_b256"] - 0.02) < 1e-6 and abs(r["margins"]["put"]["lds_default"] - 0.1) < 1e-6
    assert cur[0] == (0, 0, 1) and cur[1] == (2, 0, 1)


def test_autotune_needs_the_margin_on_every_rank(native, monkeypatch):
    """A candidate 20 % faster on rank 0 but only 1 % faster on rank 1 keeps auto."""
    cands = {"auto": (0, 0, 1), "reg_b256": (1, 256, 1)}
    secs = {(0, 0, 1): 1.0, (1, 256, 1): 0.8}

    def gather(obj):  # rank 1: reg_b256 is 0.99 of auto there
        if isinstance(obj, tuple) and obj[0] == 0.8:
            return [obj, (0.99, None)]
        return [obj, obj]

    r, _ = _fake_autotune(monkeypatch, secs, cands, gather=gather)
    assert r["get"] == "auto" and r["put"] == "auto", r
    assert abs(r["margins"]["get"]["reg_b256"] - 0.01) < 1e-6, r["margins"]


def test_autotune_never_installs_a_get_only_variant_for_puts(native, monkeypatch):
    """Push-based gets (variant 5) compete for gets only; their 'put' is auto's path."""
    cands = {"auto": (0, 0, 1), "push": (5, 0, 1), "reg_b256": (1, 256, 1)}
    secs = {(0, 0, 1): 1.0, (5, 0, 1): 0.5, (1, 256, 1): 0.9}
    r, _ = _fake_autotune(monkeypatch, secs, cands)
    assert r["get"] == "push" and r["put"] == "reg_b256", r
    assert "push" not in r["margins"]["put"], r["margins"]


def test_push_candidates_are_opt_in(monkeypatch):
    """push-based gets stay out of the default candidates until a
    multi-GPU box has run them (OCM_AUTOTUNE_PUSH=1 opts in)."""
    from oncilla_amd.models import workloads as wl

    monkeypatch.delenv("OCM_AUTOTUNE_PUSH", raising=False)
    assert not any(v[0] == 5 for v in wl.default_candidates().values())
    monkeypatch.setenv("OCM_AUTOTUNE_PUSH", "1")
    assert {"push", "push_b1024"} <= set(wl.default_candidates())


def test_idle_gap_rows_merge_ragged_ranks():
    # Relaunch timings exist only on ranks that relaunched: a merge keyed on one rank's
    # row raised on some ranks and not others, which then waited in different
    # collectives (found in the 8-rank one-GPU rehearsal with HIP lanes).
    from oncilla_amd.models import workloads as wl

    a = {"0": {"get_p50_us": 5.0, "get_relaunches": 0}, "1000": {"get_p50_us": 6.0, "get_relaunches": 2,
                                                              "get_relaunch_host_us": 3.0}}
    b = {"0": {"get_p50_us": 5.5, "get_relaunches": 0}, "1000": {"get_p50_us": 6.5, "get_relaunches": 0}}
    for order in ([a, b], [b, a]):
        m = wl.merge_idle_gap_rows(order)
        assert m["0"] == {"get_p50_us": 5.5, "get_relaunches": 0}
        assert m["1000"] == {"get_p50_us": 6.5, "get_relaunches": 2, "get_relaunch_host_us": 3.0}
        assert list(m) == ["0", "1000"]


def test_bench_ranks_started_without_torchrun(native, tmp_path):
    # tools/launch_ranks.sh: the one-GPU 8-rank rehearsal starts its ranks from a
    # shell loop (no Python parent with the GPU open); the env:// rendezvous and the
    # JSON line on rank 0's stdout must be the same as under torchrun.
    r = subprocess.run(["bash", os.path.join(REPO, "tools", "launch_ranks.sh"), "2", "29597",
                        os.path.join(REPO, "bench.py"), "--gpus", "2", "--device", "cpu", "--steps", "1", "--warmup",
                        "1", "--max-bytes", str(1 << 20), "--alloc-samples", "10", "--no-ctrl-extra"],
                       capture_output=True, text=True, timeout=300, cwd="/tmp",
                       env=dict(os.environ, RANKLOG_DIR=str(tmp_path)))
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-1500:] + (tmp_path / "rank1.log").read_text()[-1500:]
    res = _last_json(r.stdout)
    assert res["n_gpus"] == 2 and res["value"] > 0 and len(res["ranks"]) == 2, res
    assert (tmp_path / "rank1.log").exists()

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


@pytest.mark.parametrize("n", [2, 8])
def test_bench_multi_rank(native, n):
    # the driver's multi-GPU launch shape (torch.distributed.run, one daemon per rank), on gloo + CPU daemons
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n),
                        "--master-addr", "127.0.0.1", "--master-port", str(29533 + n), os.path.join(REPO, "bench.py"),
                        "--gpus", str(n), "--device", "cpu", "--steps", "2", "--warmup", "1", "--max-bytes",
                        str(4 << 20), "--alloc-samples", "20"], capture_output=True, text=True, timeout=300, cwd="/tmp")
    assert r.returncode == 0, r.stderr[-3000:]
    res = _last_json(r.stdout)
    assert res["n_gpus"] == n and res["value"] > 0 and res["config"]["parallelism"] == f"stripe{n}"
    assert res["config"]["extents_per_pair"] == n - 1  # 8 MiB+1 pair = 9 stripe units: every peer gets one


def test_bench_extras_helpers_run(native):
    # The N>1 extras only run on multi-GPU nodes (the driver's scaling run):
    # exercise their code here so a Python error cannot hide until then.
    sys.path.insert(0, REPO)
    import bench

    class FakePair:
        def time_onesided(self, op, n, iters):
            return 1e-3

    t = bench.xgmi_tuning_extras(FakePair(), None, 2, 1 << 20)
    assert set(t) == set(bench.TUNING_GRID)
    assert all("put_GiBps" in v and "error" not in v for v in t.values()), t
    b = bench.hw_baseline_extras(None, 2, 0, 0)
    assert isinstance(b, dict)
    assert bench._local(lambda: 1 / 0)[1].startswith("ZeroDivisionError")

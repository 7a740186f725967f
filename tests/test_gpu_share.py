"""The driver's multi-rank launch rehearsed on ONE MI355X (every rank and daemon on
GPU 0, OCM_BENCH_SHARE_GPU=1): several processes' copy services, launches and
daemons share the GPU, the condition under which round 3's gang completion
stalled for 10 s. The run must be clean: every
rank's copy service without a timeout, and no library warning on any rank."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_shared_gpu_rehearsal_is_clean():
    env = dict(os.environ, OCM_BENCH_SHARE_GPU="1")
    r = subprocess.run([sys.executable, "-u", "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "4",
                        "--master-addr", "127.0.0.1", "--master-port", "29681", os.path.join(REPO, "bench.py"),
                        "--gpus", "4", "--steps", "2", "--warmup", "1", "--max-bytes", str(64 << 20),
                        "--alloc-samples", "50", "--no-ctrl-extra", "--no-hw-baseline", "--no-optim-extra"],
                       capture_output=True, text=True, timeout=110, cwd="/tmp", env=env)
    assert r.returncode == 0, r.stderr[-4000:]
    res = json.loads([line for line in r.stdout.splitlines() if line.startswith("{")][-1])
    print(json.dumps({k: res.get(k) for k in ("value", "service_clean", "xgmi")}),
          [d.get("service") for d in res["ranks"]])
    assert res["n_gpus"] == 4 and res["value"] > 0 and res["xgmi"] is False, res
    assert res["service_clean"] is True, res["ranks"]
    warns = [line for line in (r.stdout + r.stderr).splitlines() if "[ocm W" in line or "[ocm E" in line]
    assert not warns, warns[:20]
    # every size was measured op by op (p50 headline, p99 beside it)
    row = res["sweep"][str(1 << 20)]
    assert row["ops"] >= 5 and row["get_p99_us"] >= row["get_us"] > 0, row

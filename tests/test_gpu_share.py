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
    env = dict(os.environ, OCM_BENCH_SHARE_GPU="1", OCM_BENCH_TIMEOUT_S="90")
    log = os.path.join(REPO, "gpurun_out", "test_gpu_share.log")
    os.makedirs(os.path.dirname(log), exist_ok=True)
    with open(log, "w") as lf:
        # the output goes to a file (kept under gpurun_out/): a hang leaves the phase it stopped in
        p = subprocess.Popen([sys.executable, "-u", "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node",
                              "4", "--master-addr", "127.0.0.1", "--master-port", "29681",
                              os.path.join(REPO, "bench.py"), "--gpus", "4", "--steps", "2", "--warmup", "1",
                              "--max-bytes", str(64 << 20), "--alloc-samples", "50", "--no-ctrl-extra",
                              "--no-hw-baseline", "--no-optim-extra"],
                             stdout=lf, stderr=subprocess.STDOUT, text=True, cwd="/tmp", env=env,
                             start_new_session=True)
        try:
            rc = p.wait(timeout=120)
        except subprocess.TimeoutExpired:
            os.killpg(p.pid, 9)
            p.wait(timeout=30)
            raise AssertionError("the rehearsal did not finish in 120 s: " + open(log).read()[-3000:])
    out = open(log).read()
    assert rc == 0, out[-4000:]
    res = json.loads([line for line in out.splitlines() if line.startswith("{")][-1])
    print(json.dumps({k: res.get(k) for k in ("value", "service_clean", "xgmi")}),
          [d.get("service") for d in res["ranks"]])
    assert res["n_gpus"] == 4 and res["value"] > 0 and res["xgmi"] is False, res
    assert res["service_clean"] is True, res["ranks"]
    warns = [line for line in out.splitlines() if "[ocm W" in line or "[ocm E" in line]
    assert not warns, warns[:20]
    # every size was measured op by op (p50 headline, p99 beside it)
    row = res["sweep"][str(1 << 20)]
    assert row["ops"] >= 5 and row["get_p99_us"] >= row["get_us"] > 0, row

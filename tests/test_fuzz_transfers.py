"""Randomised put/get/batch sequences against a host-side shadow of both halves
(tools/gpu_fuzz.py): every transfer path, unaligned offsets, odd sizes, async
and batched ops, on a loopback HBM owner, a striped pair and the host tier."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(seconds, env, nbytes, extra=()):
    r = subprocess.run([sys.executable, os.path.join(REPO, "tools", "gpu_fuzz.py"), "--seconds", str(seconds),
                        "--seed", "7", "--bytes", str(nbytes), *extra], capture_output=True, text=True, timeout=300,
                       env=env)
    line = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert r.returncode == 0 and line, (r.stdout + r.stderr)[-3000:]
    res = json.loads(line[-1])
    assert res["ok"] and all(v["steps"] > 20 for v in res["configs"].values()), res
    return res


def test_fuzz_transfers_cpu(native):
    _run(6, dict(os.environ, OCM_NO_GPU="1"), 4 << 20)


@pytest.mark.gpu
def test_fuzz_transfers_gpu(native):
    res = _run(24, dict(os.environ), 32 << 20)
    if os.path.isdir(os.path.join(REPO, "gpurun_out")):
        with open(os.path.join(REPO, "gpurun_out", "fuzz_gpu.json"), "w") as f:
            json.dump(res, f)


@pytest.mark.gpu
def test_fuzz_transfers_threads_gpu(native):
    """Four threads, each on its own pair, at once. This caught plans built by
    stream capture failing when another thread synchronized the device during
    the capture; plans are now built from explicit graph nodes."""
    _run(15, dict(os.environ), 32 << 20, ("--threads", "4", "--configs", "hbm,stripe,host"))

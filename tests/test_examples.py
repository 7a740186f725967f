"""The examples/ programs run as documented (C example against a CPU mesh,
Python quickstart on CPU and GPU, KV offload on GPU)."""
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env=None, timeout=300):
    r = subprocess.run(args, capture_output=True, text=True, timeout=timeout, cwd="/tmp", env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    return r.stdout


def test_c_example_against_cpu_mesh(mesh_factory, native):
    m = mesh_factory(2)
    out = _run([f"{native}/ocm_example_hello", "4"], env=dict(m.client_env(0), OCM_NO_GPU="1"))
    assert "round trip through rank 1" in out and "0 bad words" in out


def test_quickstart_cpu(native):
    out = _run([sys.executable, os.path.join(REPO, "examples", "quickstart.py")], env=dict(os.environ, OCM_NO_GPU="1"))
    assert "round trip, striped over ranks [1, 2]" in out


@pytest.mark.gpu
def test_quickstart_gpu(native):
    env = {k: v for k, v in os.environ.items() if k != "OCM_NO_GPU"}
    out = _run([sys.executable, os.path.join(REPO, "examples", "quickstart.py"), "--gpu", "0"], env=env)
    assert "round trip" in out


@pytest.mark.gpu
def test_kv_offload_example(native):
    out = _run([sys.executable, os.path.join(REPO, "examples", "kv_offload.py")])
    assert "64 KV blocks swapped out and back" in out


def test_cli_mesh_and_stats(native):
    import signal
    import time

    p = subprocess.Popen([sys.executable, "-m", "oncilla_amd", "mesh", "--daemons", "3", "--ns", "clitest42"],
                         cwd=REPO, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                         env=dict(os.environ, OCM_NO_GPU="1"))
    try:
        line = p.stdout.readline()
        assert "mesh up: 3 daemons" in line, line + p.stderr.read()
        out = _run([sys.executable, "-m", "oncilla_amd", "stats", "--ns", "clitest42"],
                   env=dict(os.environ, OCM_NO_GPU="1", PYTHONPATH=REPO))
        assert len([l for l in out.splitlines() if l.strip()[:1].isdigit()]) == 3, out
    finally:
        p.send_signal(signal.SIGINT)
        p.wait(timeout=30)
    assert p.returncode == 0


def test_train_offload_cpu(native):
    out = _run([sys.executable, os.path.join(REPO, "examples", "train_offload.py"), "--steps", "150"],
               env=dict(os.environ, OCM_NO_GPU="1"))
    assert "mode=staged" in out and "loss" in out


@pytest.mark.gpu
@pytest.mark.parametrize("bf16", [False, True])
def test_train_offload_gpu(native, bf16):
    env = {k: v for k, v in os.environ.items() if k != "OCM_NO_GPU"}
    out = _run([sys.executable, os.path.join(REPO, "examples", "train_offload.py"), "--gpu", "0", "--steps", "150"]
               + (["--bf16"] if bf16 else []), env=env)
    assert "mode=fused" in out and "peer HBM" in out


def _torchrun(n, port, extra, env=None):
    return _run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n),
                 "--master-addr", "127.0.0.1", "--master-port", str(port),
                 os.path.join(REPO, "examples", "train_zero.py")] + extra, env=env)


def test_train_zero_cpu(native):
    out = _torchrun(2, 29661, ["--cpu"], env=dict(os.environ, OCM_NO_GPU="1"))
    assert "2 ranks" in out and "host tier" in out and "mode=staged" in out


@pytest.mark.gpu
def test_train_zero_gpu_shared(native):
    env = {k: v for k, v in os.environ.items() if k != "OCM_NO_GPU"}
    out = _torchrun(2, 29662, ["--share-gpu"], env=env)
    assert "2 ranks" in out and "peer HBM" in out and "mode=fused" in out


@pytest.mark.gpu
def test_remote_weights_gpu(native):
    out = _run([sys.executable, os.path.join(REPO, "examples", "remote_weights.py")])
    assert "forward matches the local copy: True" in out

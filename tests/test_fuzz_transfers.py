"""Randomised put/get/batch sequences against a host-side shadow of both halves
(tools/gpu_fuzz.py): every transfer path, unaligned offsets, odd sizes, async
and batched ops, on a loopback HBM owner, a striped pair and the host tier."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(seconds, env, nbytes, extra=(), min_steps=20):
    r = subprocess.run([sys.executable, os.path.join(REPO, "tools", "gpu_fuzz.py"), "--seconds", str(seconds),
                        "--seed", "7", "--bytes", str(nbytes), *extra], capture_output=True, text=True, timeout=300,
                       env=env)
    line = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert r.returncode == 0 and line, (r.stdout + r.stderr)[-3000:]
    res = json.loads(line[-1])
    assert res["ok"] and all(v["steps"] > min_steps for v in res["configs"].values()), res
    return res


def test_fuzz_transfers_cpu(native):
    # each config gets a slice of the 8 s; on a loaded CPU runner the two-sided
    # copy config can fall under 20 steps, so only ask that every config ran
    _run(8, dict(os.environ, OCM_NO_GPU="1"), 4 << 20, ("--configs", "hbm,stripe,host,net,copy"), min_steps=5)


@pytest.mark.gpu
def test_fuzz_transfers_gpu(native):
    res = _run(25, dict(os.environ), 32 << 20, ("--configs", "hbm,stripe,host,net,copy"))
    if os.path.isdir(os.path.join(REPO, "gpurun_out")):
        with open(os.path.join(REPO, "gpurun_out", "fuzz_gpu.json"), "w") as f:
            json.dump(res, f)


@pytest.mark.gpu
def test_fuzz_transfers_threads_gpu(native):
    """Four threads, each on its own pair, at once. This caught plans built by
    stream capture failing when another thread synchronized the device during
    the capture; plans are now built from explicit graph nodes."""
    _run(15, dict(os.environ), 32 << 20, ("--threads", "4", "--configs", "hbm,stripe,host"))


def _procs(mesh_factory, env, seconds, nbytes):
    """Three fuzzing apps at once on one 4-daemon mesh, attached to different
    daemons: the daemons serve concurrent allocations, frees and imports while
    the apps move data."""
    m = mesh_factory(4, gpus=[None if env.get("OCM_NO_GPU") else 0] * 4, policy="stripe")
    ps = [subprocess.Popen([sys.executable, os.path.join(REPO, "tools", "gpu_fuzz.py"), "--ns", m.ns,
                            "--daemon-rank", str(k), "--seconds", str(seconds), "--seed", str(90 + k),
                            "--bytes", str(nbytes), "--configs", "hbm,stripe,host"],
                           stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, env=env) for k in range(3)]
    outs = [p.communicate(timeout=300)[0] for p in ps]
    for p, out in zip(ps, outs):
        assert p.returncode == 0, out[-3000:] + m.logs()[-2000:]
        assert json.loads([l for l in out.splitlines() if l.startswith("{")][-1])["ok"]
    assert all(d.alive() for d in m.daemons)


def test_fuzz_apps_share_a_mesh_cpu(native, mesh_factory, monkeypatch):
    monkeypatch.setenv("OCM_NO_GPU", "1")
    _procs(mesh_factory, dict(os.environ, OCM_NO_GPU="1"), 6, 4 << 20)


@pytest.mark.gpu
def test_fuzz_apps_share_a_mesh_gpu(native, mesh_factory):
    _procs(mesh_factory, dict(os.environ), 15, 16 << 20)


@pytest.mark.gpu
@pytest.mark.parametrize("proto", ["7", "1", "9", "15+strict", "47+strict"])
def test_fuzz_service_protocols_gpu(native, proto):
    """The copy service's other hand-off protocols stay correct now that the default
    (15) completes gangs through per-workgroup done words: 7 = the device-scope
    counter, 1 = write-through without the gang record (relayed gangs), 9 = that
    with per-workgroup done words. "+strict": every request takes the peer-HBM
    (STRICT) hand-off (OCM_SERVICE_STRICT=1), fenced (15) or write-through behind
    its acquire (47 = 15 | STRICTWT)."""
    p, _, strict = proto.partition("+")
    env = dict(os.environ, OCM_SERVICE_PROTO=p, **({"OCM_SERVICE_STRICT": "1"} if strict else {}))
    _run(8, env, 16 << 20, ("--configs", "hbm,host"))

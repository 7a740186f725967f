"""Raw one-sided backend (ocm/xgmi.h), the xGMI counterpart of the reference's
IB and EXTOLL backends, driven by the paired client/daemon tools exactly like
reference test/ib_client.c + test/ib_daemon.c (tests 0-3)."""
import os
import subprocess
import uuid

import pytest


def _run_pair(native, test, mb, server_gpu, client_gpu, env):
    ep = f"t{uuid.uuid4().hex[:10]}"
    srv = subprocess.Popen([f"{native}/ocm_xgmi_daemon", ep, str(mb), str(server_gpu)], stdout=subprocess.PIPE,
                           stderr=subprocess.STDOUT, text=True, env=env)
    try:
        assert "listening" in srv.stdout.readline()
        cli = subprocess.run([f"{native}/ocm_xgmi_client", ep, str(test), str(mb), str(client_gpu)],
                             capture_output=True, text=True, timeout=120, env=env)
        out = srv.communicate(timeout=60)[0]
        assert cli.returncode == 0, cli.stdout + cli.stderr + out
        assert srv.returncode == 0, out
        return cli.stdout
    finally:
        if srv.poll() is None:
            srv.kill()


@pytest.mark.parametrize("test", [0, 1, 2, 3])
def test_backend_cpu(native, test):
    out = _run_pair(native, test, 2, -1, -1, dict(os.environ, OCM_NO_GPU="1"))
    if test == 3:
        assert out.count("GiB/s") == 2 * 16  # 64 B .. 2 MiB, read and write


@pytest.mark.gpu
@pytest.mark.parametrize("server_gpu,client_gpu", [(0, 0), (-1, 0), (0, -1)])
@pytest.mark.parametrize("test", [0, 1, 3])
def test_backend_gpu(native, test, server_gpu, client_gpu):
    _run_pair(native, test, 64, server_gpu, client_gpu, dict(os.environ))

"""Shared fixtures: the native build, daemon meshes, the GPU marker.

Every test that needs an MI355X is marked `@pytest.mark.gpu`; everything else
runs on CPU-only daemons (the reference's single-node loopback config plus
multi-daemon meshes on one host).
"""
from __future__ import annotations

import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run with -m gpu on the GPU box)")
    config.addinivalue_line("markers", "slow: long-running")
    config.addinivalue_line("markers", "expects_abort: the test provokes a copy-service timeout on purpose")


@pytest.fixture(scope="session")
def native():
    """Build the native tree once per session (no-op when up to date)."""
    from oncilla_amd.utils.build import build
    from oncilla_amd.utils.paths import BIN_DIR

    build()
    return BIN_DIR


@pytest.fixture
def mesh_factory(native):
    from oncilla_amd.parallel.mesh import Mesh

    made = []

    def make(n, **kw):
        m = Mesh(n, **kw).start()
        made.append(m)
        return m

    yield make
    for m in made:
        m.stop()


def run_tool(args, env=None, timeout=120):
    import subprocess

    r = subprocess.run(args, env=env, capture_output=True, text=True, timeout=timeout)
    return r.returncode, r.stdout + r.stderr


@pytest.fixture
def tool():
    return run_tool


def gpu_count() -> int:
    try:
        import torch

        return torch.cuda.device_count()
    except Exception:
        return 0

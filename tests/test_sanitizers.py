"""Host-code sanitizers (the reference had only -Wall -Werror).
Builds the tree with -fsanitize=address,undefined (build-asan/) and runs the
daemon mesh + reference-equivalent tests on the instrumented binaries; any
ASan/UBSan report fails the test."""
import os
import subprocess

import pytest

from oncilla_amd.parallel.mesh import Mesh
from oncilla_amd.utils.build import build

SAN_ENV = {"ASAN_OPTIONS": "detect_leaks=0:abort_on_error=0:halt_on_error=1", "UBSAN_OPTIONS": "print_stacktrace=1",
           "OCM_NO_GPU": "1"}
BAD = ("ERROR: AddressSanitizer", "runtime error:", "ERROR: LeakSanitizer")


@pytest.fixture(scope="module")
def asan_bin():
    return os.path.join(build(sanitize=True), "bin")


def test_unit_tests_under_asan(asan_bin):
    r = subprocess.run([f"{asan_bin}/ocm_unit_tests"], capture_output=True, text=True, timeout=300,
                       env=dict(os.environ, **SAN_ENV))
    assert r.returncode == 0 and not any(b in r.stderr for b in BAD), r.stdout + r.stderr


def test_mesh_under_asan(asan_bin):
    m = Mesh(3, bin_dir=asan_bin, env=SAN_ENV).start(timeout=120)
    try:
        env = dict(m.client_env(1), **SAN_ENV)
        for args in (["1", "1", "2", "1"], ["1", "1", "2", "3"], ["2", "4", "4"], ["3", "2", "4"], ["5", "4", "1"],
                     ["4", "1", "2", "2"]):
            r = subprocess.run([f"{asan_bin}/ocm_test", *args], capture_output=True, text=True, timeout=300, env=env)
            assert r.returncode == 0 and not any(b in r.stderr for b in BAD), f"{args}\n{r.stdout}\n{r.stderr}"
    finally:
        m.stop()
    logs = m.logs()
    assert not any(b in logs for b in BAD), logs


@pytest.fixture(scope="module")
def tsan_bin():
    return os.path.join(build(sanitize="thread"), "bin")


def test_unit_tests_under_tsan(tsan_bin):
    # the native unit tests run the tick transport's thread against a 1-rank
    # socket collective, plain and batched
    r = subprocess.run([f"{tsan_bin}/ocm_unit_tests"], capture_output=True, text=True, timeout=300,
                       env=dict(os.environ, OCM_NO_GPU="1", TSAN_OPTIONS="halt_on_error=0"))
    assert r.returncode == 0 and "ThreadSanitizer" not in r.stderr, r.stdout + r.stderr


@pytest.mark.parametrize("sealed", ["0", "1", "batch4"])
def test_threads_under_tsan(tsan_bin, sealed):
    # Threads in the daemon: the tick transport thread (socket collective; sealed=1
    # adds the outbox ring the RCCL seal kernel reads, emulated on the CPU) and
    # the network-tier data server (rank 2 is alone on "node B", so its app's
    # remote halves live on node A and are streamed through rank 0/1 servers).
    # batch4: ticks queued 4 at a time, the stand-in for replays of captured tick graphs
    seal = {"OCM_TICK_SOCKET_SEAL": "1", "OCM_TICK_SOCKET_BATCH": "4"} if sealed == "batch4" else {"OCM_TICK_SOCKET_SEAL": sealed}
    env = {"OCM_NO_GPU": "1", "TSAN_OPTIONS": "halt_on_error=0", **seal}
    hosts = {0: {"OCM_HOST_ALIAS": "A"}, 1: {"OCM_HOST_ALIAS": "A"}, 2: {"OCM_HOST_ALIAS": "B"}}
    m = Mesh(3, bin_dir=tsan_bin, env=env, extra_args=["--ctrl", "socket"], rank_env=hosts).start(timeout=120)
    try:
        for args in (["1", "1", "2", "3"], ["2", "4", "8"], ["3", "2", "4"], ["4", "1", "2", "2"]):
            r = subprocess.run([f"{tsan_bin}/ocm_test", *args], capture_output=True, text=True, timeout=300,
                               env=dict(m.client_env(2), **env))
            assert r.returncode == 0 and "ThreadSanitizer" not in r.stderr, f"{args}\n{r.stdout}\n{r.stderr}"
    finally:
        m.stop()
    logs = m.logs()
    assert "WARNING: ThreadSanitizer" not in logs, logs


def test_resume_net_tier_and_fuzz_under_asan(asan_bin, tmp_path):
    # The newer daemon paths under ASan/UBSan: network tier (node split by host
    # alias), rank0 checkpoint -> kill -> restart -> reconcile, and a mailbox storm.
    import signal
    import sys as _sys

    _sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from test_fuzz_mailbox import _storm

    state = str(tmp_path / "dir.ckpt")
    hosts = {0: {"OCM_HOST_ALIAS": "A", "OCM_STATE_FILE": state}, 1: {"OCM_HOST_ALIAS": "A"},
             2: {"OCM_HOST_ALIAS": "B"}}
    m = Mesh(3, bin_dir=asan_bin, env=SAN_ENV, rank_env=hosts).start(timeout=120)
    try:
        env = dict(m.client_env(2), **SAN_ENV)  # rank 2 is alone on node B: network tier
        for args in (["2", "4", "8"], ["3", "2", "4"]):
            r = subprocess.run([f"{asan_bin}/ocm_test", *args], capture_output=True, text=True, timeout=300, env=env)
            assert r.returncode == 0 and not any(b in r.stderr for b in BAD), f"{args}\n{r.stdout}\n{r.stderr}"
        _storm(m.ns, seed=11, n=1500)
        m.kill(0, signal.SIGKILL)
        m.restart(0, timeout=120)
        r = subprocess.run([f"{asan_bin}/ocm_test", "2", "4", "8"], capture_output=True, text=True, timeout=300,
                           env=dict(m.client_env(1), **SAN_ENV))
        assert r.returncode == 0 and not any(b in r.stderr for b in BAD), r.stdout + r.stderr
    finally:
        m.stop()
    logs = m.logs()
    assert not any(b in logs for b in BAD), logs[-6000:]

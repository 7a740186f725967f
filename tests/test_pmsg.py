"""Mailbox ping-pong (reference test/pmsg_daemon.c + test/pmsg_client.c)."""
import json
import os
import subprocess
import uuid


def test_pmsg_pingpong(native):
    env = dict(os.environ, OCM_NS=f"pp{uuid.uuid4().hex[:8]}")
    srv = subprocess.Popen([f"{native}/ocm_pmsg_pingpong", "server", "3"], env=env, stdout=subprocess.PIPE, text=True)
    try:
        assert srv.stdout.readline().strip() == "ready"
        r = subprocess.run([f"{native}/ocm_pmsg_pingpong", "client", "3", "2000"], env=env, capture_output=True,
                           text=True, timeout=60)
        assert r.returncode == 0, r.stderr
        res = json.loads(r.stdout.strip().splitlines()[-1])
        assert res["count"] == 2000
        # blocking mq receive, no 500 us poll (reference src/main.c:125): well under 0.5 ms
        assert res["p50_us"] < 500
        assert srv.wait(timeout=10) == 0
    finally:
        if srv.poll() is None:
            srv.kill()

"""Tracing: per-process counters and the OCM_TRACE_FILE op log."""
import json

from oncilla_amd import api


def test_counters_and_trace_file(mesh_factory, native, tool, tmp_path, monkeypatch):
    monkeypatch.setenv("OCM_NO_GPU", "1")
    m = mesh_factory(2)
    log = tmp_path / "ops.jsonl"
    rc, out = tool([f"{native}/ocm_test", "2", "1", "1"], env=dict(m.client_env(0), OCM_TRACE_FILE=str(log),
                                                                      OCM_NO_GPU="1"))
    assert rc == 0, out
    recs = [json.loads(l) for l in log.read_text().splitlines()]
    ops = [r["op"] for r in recs]
    assert ops.count("alloc") == 1 and ops.count("free") == 1
    assert ops.count("put") >= 1 and ops.count("get") >= 1
    assert all(r["us"] >= 0 for r in recs)

    with api.Client(daemon_rank=1, ns=m.ns) as c:
        before = api.counters()
        a = c.alloc(api.OCM_REMOTE_RDMA, local_bytes=1 << 16, remote_bytes=1 << 16)
        a.put(0, 0, 1 << 16)
        a.get(0, 0, 1 << 15)
        a.free()
        after = api.counters()
    assert after["n_put"] - before["n_put"] == 1 and after["bytes_get"] - before["bytes_get"] == 1 << 15
    assert after["n_alloc"] - before["n_alloc"] == 1 and after["n_free"] - before["n_free"] == 1

"""Native unit tests (wire layout, nodefile, range allocator, governor, stripe
geometry, host-tier arena) and the ABI layout seen from Python."""
import ctypes

from oncilla_amd import api


def test_native_unit_binary(native, tool):
    rc, out = tool([f"{native}/ocm_unit_tests"])
    assert rc == 0, out
    for name in ("layout", "nodefile", "range_alloc", "governor", "governor_hosts", "stripe_geometry", "arena_host"):
        assert f"PASS {name}" in out


def test_abi_layout(native):
    lay = api.layout()
    # reference inc/oncillamem.h:39-58 and the 160-byte wire record
    assert lay["msg"] == 160 and lay["msg_union_offset"] == 32
    assert lay["ocm_params"] == 48 == ctypes.sizeof(api.OcmParams)
    assert lay["ocm_alloc_params"] == 24 == ctypes.sizeof(api.OcmAllocParams)
    assert lay["ipc_handle"] == 64
    assert (api.OCM_LOCAL_HOST, api.OCM_LOCAL_RMA, api.OCM_REMOTE_RMA, api.OCM_LOCAL_RDMA, api.OCM_REMOTE_RDMA,
            api.OCM_LOCAL_GPU, api.OCM_REMOTE_GPU) == tuple(range(1, 8))

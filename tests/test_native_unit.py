"""Native unit tests (wire layout, nodefile, range allocator, governor, stripe
geometry, host-tier arena) and the ABI layout seen from Python."""
import ctypes

import pytest

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


@pytest.mark.parametrize("src,min_kernels", [("xfer.hip", 9), ("optim.hip", 1)])
def test_kernels_use_no_scratch(src, min_kernels):
    # Resource check of every gfx950 kernel: a dynamically indexed local array
    # (e.g. a copied extent table) lands in scratch and costs a memory round
    # trip per access on the hot path. The compiler reports it per kernel.
    import os
    import re
    import subprocess

    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17",
                        f"-I{repo}/csrc/include", "-c", f"{repo}/csrc/src/kernels/{src}", "-o", os.devnull,
                        "-Rpass-analysis=kernel-resource-usage"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    names = re.findall(r"Function Name: (\S+)", r.stderr)
    scratch = [int(v) for v in re.findall(r"ScratchSize \[bytes/lane\]: (\d+)", r.stderr)]
    spills = [int(v) for v in re.findall(r"VGPRs Spill: (\d+)", r.stderr)]
    assert len(names) >= min_kernels and len(scratch) == len(names)
    assert all(s == 0 for s in scratch), dict(zip(names, scratch))
    assert all(s == 0 for s in spills), dict(zip(names, spills))


def test_example_nodefiles_parse(native, tool):
    """examples/nodefiles/* parse with the daemon's own parser (the reference
    format, the one-node 8-GPU layout, two nodes with fixed data ports)."""
    import glob
    import os

    files = sorted(glob.glob(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                          "examples", "nodefiles", "*")))
    assert len(files) >= 3
    rc, out = tool([f"{native}/ocm_unit_tests", "--nodefile", *files])
    assert rc == 0, out
    assert "OK" in out and "16 daemons" in out and "8 daemons" in out


def test_embedded_service_code_object_layout(native):
    # libocm dispatches the copy service on its own AQL queue from a device code
    # object embedded at build time (ocm/aql.h), writing the explicit arguments
    # (ServiceKernelArgs, 88 bytes) and then the COv5 hidden arguments at fixed
    # offsets after them. Check the layout in the code object's metadata, and that
    # the object is inside libocm.so.
    import os
    import re
    import subprocess

    from oncilla_amd.utils.paths import lib_path

    co = os.path.join(os.path.dirname(os.path.dirname(lib_path())), "ocm_devcode.co")
    notes = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-readelf", "--notes", co], capture_output=True, text=True,
                           check=True).stdout
    assert "amdgcn-amd-amdhsa--gfx950" in notes
    kern = [k for k in re.split(r"\n  - ", notes) if re.search(r"\.name:\s+ocm_service_kernel\s", k)]
    assert len(kern) == 1, "ocm_service_kernel missing from the embedded code object"
    args = {kind: (int(off), int(size)) for off, size, kind in
            re.findall(r"\.offset:\s+(\d+)\s+\.size:\s+(\d+)\s+\.value_kind:\s+(\S+)", kern[0])}
    assert args["by_value"] == (0, 88), args
    # The kernel reads its grid size from its own arguments, so it needs no hidden
    # argument; if the compiler still declares them, they sit where the dispatch writes them.
    if "hidden_block_count_x" in args:
        assert args["hidden_block_count_x"][0] == 88 and args["hidden_group_size_x"][0] == 100, args
        assert args["hidden_grid_dims"][0] == 88 + 64, args
    assert int(re.search(r"\.kernarg_segment_size:\s+(\d+)", kern[0]).group(1)) <= 4096
    blob = open(co, "rb").read()
    assert blob[:4] == b"\x7fELF" and blob in open(lib_path(), "rb").read()

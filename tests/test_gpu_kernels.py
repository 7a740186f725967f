"""Numerics of the gfx950 transfer kernels against a plain PyTorch reference
of the same copy (exact byte equality; random data, odd sizes/offsets)."""
import pytest
import torch

from oncilla_amd import ops

pytestmark = pytest.mark.gpu

DEV = "cuda:0"


def _rand(n, seed):
    g = torch.Generator(device="cpu").manual_seed(seed)
    return torch.randint(0, 256, (n,), dtype=torch.uint8, generator=g).to(DEV)


@pytest.mark.parametrize("variant", [ops.XFER_REG, ops.XFER_LDS])
@pytest.mark.parametrize("n,soff,doff", [(1, 0, 0), (15, 1, 0), (16, 0, 0), (17, 3, 3), (4095, 0, 7),
                                         (32768, 0, 0), (32769, 16, 32), (1 << 20, 5, 9), ((8 << 20) + 48, 0, 0),
                                         ((64 << 20) + 4, 4, 4)])
def test_device_copy_matches_torch(variant, n, soff, doff):
    src = _rand(n + soff, n)
    dst = torch.zeros(n + doff + 64, dtype=torch.uint8, device=DEV)
    ref = dst.clone()
    ref[doff:doff + n] = src[soff:soff + n]
    ops.xfer(src[soff:], [dst[doff:]], 0, 0, n, put=True, variant=variant)
    torch.cuda.synchronize()
    assert torch.equal(dst, ref)


@pytest.mark.parametrize("variant", [ops.XFER_REG, ops.XFER_LDS])
@pytest.mark.parametrize("n_ext,unit", [(2, 4096), (3, 65536), (7, 1 << 20), (8, 32768)])
@pytest.mark.parametrize("put", [True, False])
def test_striped_matches_reference(variant, n_ext, unit, put):
    total = n_ext * unit * 5 + 12345
    rem_off, nbytes = unit // 2 + 3, total - unit - 100
    ext_len = ((rem_off + nbytes) // unit // n_ext + 2) * unit
    exts = [_rand(ext_len, 100 + i) for i in range(n_ext)]
    lin = _rand(nbytes + 64, 7)
    exts_ref = [e.clone() for e in exts]
    lin_ref = lin.clone()
    ops.striped_reference(lin_ref, exts_ref, unit, rem_off, nbytes, put)
    ops.xfer(lin, exts, unit, rem_off, nbytes, put=put, variant=variant)
    torch.cuda.synchronize()
    assert torch.equal(lin, lin_ref)
    for a, b in zip(exts, exts_ref):
        assert torch.equal(a, b)


def test_grid_sizes_and_small_grids():
    n = (3 << 20) + 7
    src = _rand(n, 1)
    for blocks in (1, 7, 256, 4096):
        dst = torch.zeros(n, dtype=torch.uint8, device=DEV)
        ops.xfer(src, [dst], 0, 0, n, put=True, blocks=blocks)
        torch.cuda.synchronize()
        assert torch.equal(dst, src)


def test_copy_bandwidth_sane():
    n = 1 << 30
    a = torch.empty(n, dtype=torch.uint8, device=DEV)
    b = torch.empty(n, dtype=torch.uint8, device=DEV)
    t = ops.device_copy_seconds(b, a, n, iters=5)
    gbps = 2 * n / t / 1e9  # read + write
    assert gbps > 1000, f"HBM copy only {gbps:.0f} GB/s"

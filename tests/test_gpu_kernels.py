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


@pytest.mark.parametrize("variant", [ops.XFER_REG, ops.XFER_LDS, ops.XFER_PCIE])
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


@pytest.mark.parametrize("variant", [ops.XFER_REG, ops.XFER_LDS, ops.XFER_PCIE])
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


@pytest.mark.parametrize("n_ext,unit", [(1, 0), (2, 4096), (3, 65536), (7, 1 << 20), (8, 32768)])
def test_push_get_kernel_matches_reference(n_ext, unit):
    # The push-get kernel (XFER_PUSH) with every extent in its mask: byte-exact
    # against the torch oracle, striped or not, unaligned offsets included.
    total = max(n_ext, 1) * max(unit, 65536) * 5 + 12345
    rem_off, nbytes = (unit // 2 + 3) if n_ext > 1 else 5, total - max(unit, 4096) - 100
    ext_len = ((rem_off + nbytes) // max(unit, 1) // n_ext + 2) * unit if n_ext > 1 else rem_off + nbytes + 64
    exts = [_rand(ext_len, 500 + i) for i in range(n_ext)]
    lin = _rand(nbytes + 64, 9)
    exts_ref = [e.clone() for e in exts]
    lin_ref = lin.clone()
    ops.striped_reference(lin_ref, exts_ref, unit if n_ext > 1 else 1, rem_off, nbytes, False)
    ops.xfer(lin, exts, unit, rem_off, nbytes, put=False, variant=ops.XFER_PUSH)
    torch.cuda.synchronize()
    assert torch.equal(lin, lin_ref)


@pytest.mark.parametrize("put", [True, False])
@pytest.mark.parametrize("n_ext,unit", [(1, 0), (3, 4096), (2, 1 << 20)])
def test_pcie_kernel_on_pinned_host_memory(put, n_ext, unit):
    # The host-tier path: extents in pinned host memory, the linear side in HBM,
    # write-through stores into the host on puts. Byte-exact against torch.
    total = (n_ext * max(unit, 1 << 20) * 3) + 4099
    rem_off, nbytes = 4096 + 5, total - 8192
    ext_len = (rem_off + nbytes) // n_ext + 2 * max(unit, 4096) if n_ext > 1 else rem_off + nbytes + 64
    exts = [_rand(ext_len, 300 + i).cpu().pin_memory() for i in range(n_ext)]
    lin = _rand(nbytes + 64, 8)
    exts_ref = [e.clone() for e in exts]
    lin_ref = lin.clone()
    ops.striped_reference(lin_ref, exts_ref, unit if n_ext > 1 else 1, rem_off, nbytes, put)
    ops.xfer(lin, exts, unit, rem_off, nbytes, put=put, variant=ops.XFER_PCIE)
    torch.cuda.synchronize()
    assert torch.equal(lin, lin_ref)
    for a, b in zip(exts, exts_ref):
        assert torch.equal(a, b)


@pytest.mark.parametrize("put", [True, False])
def test_register_kernel_write_through_matches_reference(monkeypatch, put):
    # OCM_XFER_NT=2: the register kernel with sc1 (write-through) loads and stores,
    # an autotune candidate over xGMI; byte-exact, striped, unaligned.
    monkeypatch.setenv("OCM_XFER_NT", "2")
    n_ext, unit = 3, 65536
    total = n_ext * unit * 5 + 12345
    rem_off, nbytes = unit // 2 + 3, total - unit - 100
    ext_len = ((rem_off + nbytes) // unit // n_ext + 2) * unit
    exts = [_rand(ext_len, 700 + i) for i in range(n_ext)]
    lin = _rand(nbytes + 64, 11)
    exts_ref = [e.clone() for e in exts]
    lin_ref = lin.clone()
    ops.striped_reference(lin_ref, exts_ref, unit, rem_off, nbytes, put)
    ops.xfer(lin, exts, unit, rem_off, nbytes, put=put, variant=ops.XFER_REG)
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


def _disjoint_ranges(rng, space, lens):
    """Random disjoint placement of ranges with the given lengths inside [0, space)."""
    n = len(lens)
    slack = space - sum(lens)
    assert slack >= 0
    cuts = sorted(rng.randint(0, slack) for _ in range(n))
    order = list(range(n))
    rng.shuffle(order)
    offs, pos, prev = [0] * n, 0, 0
    for k, i in enumerate(order):
        pos += cuts[k] - prev
        prev = cuts[k]
        offs[i] = pos
        pos += lens[i]
    return offs


@pytest.mark.parametrize("n_ext,unit,n_ops,max_len", [(1, 0, 1, 100000), (1, 0, 48, 9000), (3, 4096, 49, 9000),
                                                      (3, 65536, 700, 3000), (7, 1 << 20, 2000, 1500),
                                                      (8, 32768, 64, 70000), (2, 16, 300, 100)])
def test_batch_kernel_matches_reference(n_ext, unit, n_ops, max_len):
    # Mixed puts/gets with unaligned sizes and offsets; local ranges disjoint and
    # remote ranges disjoint, so every op reads initial data and order is irrelevant.
    import random

    rng = random.Random(n_ops * 31 + n_ext)
    total = 8 << 20
    ext_len = total if n_ext == 1 else ((total // unit) // n_ext + 2) * unit
    exts = [_rand(ext_len, 500 + i) for i in range(n_ext)]
    lin = _rand(total, 9)
    lens = [rng.randint(1, max_len) for _ in range(n_ops)]
    loffs, roffs = _disjoint_ranges(rng, total, lens), _disjoint_ranges(rng, total, lens)
    ops_list = [(rng.random() < 0.5, loffs[i], roffs[i], lens[i]) for i in range(n_ops)]
    lin0, exts0 = lin.clone(), [e.clone() for e in exts]
    ref_lin, ref_exts = lin.clone(), [e.clone() for e in exts]
    for put, lo, ro, nb in ops_list:
        if put:
            ops.striped_reference(lin0[lo:], ref_exts, unit, ro, nb, put=True)
        else:
            ops.striped_reference(ref_lin[lo:], exts0, unit, ro, nb, put=False)
    ops.batch(lin, exts, unit, ops_list)
    torch.cuda.synchronize()
    assert torch.equal(lin, ref_lin)
    for e, r in zip(exts, ref_exts):
        assert torch.equal(e, r)

"""Direct access to the gfx950 transfer kernels on torch tensors.

Used by the numerics tests (kernel vs a plain PyTorch reference of the same
copy) and by the kernel micro-benchmarks. The kernels live in libocm.so
(csrc/src/kernels/xfer.hip); this module fails loudly when it is missing.
"""
from __future__ import annotations

import ctypes

from .. import api

XFER_AUTO, XFER_REG, XFER_LDS, XFER_PCIE, XFER_PUSH = 0, 1, 2, 4, 5


def _ptr(t) -> int:
    return t.data_ptr()


def xfer(lin, exts: list, unit: int, rem_off: int, nbytes: int, put: bool, variant: int = XFER_AUTO,
         blocks: int = 0, sync: bool = True) -> None:
    """Striped one-sided transfer between uint8 tensors on one device.

    put=True : lin[0:nbytes] -> striped[rem_off : rem_off+nbytes]
    put=False: striped[rem_off : rem_off+nbytes] -> lin[0:nbytes]
    Unit u of the striped space is exts[u % n][(u // n) * unit + within].
    sync=False enqueues on the null stream (ordered with torch's default stream).
    """
    lib = api.load()
    n = len(exts)
    arr = (ctypes.c_void_p * n)(*[_ptr(e) for e in exts])
    rc = lib.ocm_x_xfer(lin.device.index or 0, ctypes.c_void_p(_ptr(lin)), arr, n, unit, rem_off, nbytes,
                        1 if put else 0, variant, blocks, 1 if sync else 0)
    if rc != 0:
        raise api.OcmError("ocm_x_xfer failed")


def striped_reference(lin, exts: list, unit: int, rem_off: int, nbytes: int, put: bool) -> None:
    """Plain PyTorch implementation of the same transfer (the numerics oracle)."""
    n = len(exts)
    pos, done = rem_off, 0
    while done < nbytes:
        u, within = divmod(pos, unit) if n > 1 else (0, pos)
        take = min((unit - within) if n > 1 else nbytes - done, nbytes - done)
        e = exts[u % n] if n > 1 else exts[0]
        eoff = (u // n) * unit + within if n > 1 else pos
        if put:
            e[eoff:eoff + take].copy_(lin[done:done + take])
        else:
            lin[done:done + take].copy_(e[eoff:eoff + take])
        pos += take
        done += take


def device_copy_seconds(dst, src, nbytes: int, variant: int = XFER_REG, blocks: int = 0, nontemporal: bool = True,
                        iters: int = 20) -> float:
    """Event-timed seconds per copy of `nbytes` between two device tensors."""
    lib = api.load()
    return lib.ocm_x_time_device_copy(dst.device.index or 0, ctypes.c_void_p(_ptr(dst)), ctypes.c_void_p(_ptr(src)),
                                      nbytes, variant, blocks, 1 if nontemporal else 0, iters)


def batch(lin, exts: list, unit: int, ops, iters: int = 1) -> None:
    """Batched one-sided ops between device tensors with the gfx950 batch kernel
    (no daemons): ops = [(put, lin_off, rem_off, nbytes)], remote side striped
    over `exts` in `unit`-byte units (the libocm layout)."""
    lib = api.load()
    n = len(exts)
    arr = (ctypes.c_void_p * n)(*[_ptr(e) for e in exts])
    flat = (ctypes.c_uint64 * (4 * max(1, len(ops))))()
    for i, (put, lo, ro, nb) in enumerate(ops):
        flat[4 * i:4 * i + 4] = [lo, ro, nb, 1 if put else 0]
    rc = lib.ocm_x_batch(lin.device.index or 0, ctypes.c_void_p(_ptr(lin)), arr, n, unit, flat, len(ops), iters)
    if rc != 0:
        raise api.OcmError("ocm_x_batch failed")

"""An owner-side view of a remote extent: a process on the OWNER's GPU.

The one-sided data path runs on the initiator's GPU; the owner's GPU never
takes part (like RDMA: the reference's remote CPU is idle after setup,
src/rdma.c:46-85). What the owner's GPU *sees* is still what matters to an
application that computes on disaggregated memory from both sides: bytes an
app put over xGMI must be visible to a kernel on the owner's GPU, and bytes a
kernel there wrote must come back through the app's next get, across the copy
service, launches and the service's idle exits.

`OwnerView` starts a helper process pinned to the owner's device. It maps the
extent's slab from its export handle (hipIpcOpenMemHandle on the device that
holds the memory, the canonical IPC import) and fills / checks the word
pattern there with libocm's gfx950 pattern kernels, on that device. Commands
travel over the helper's stdin/stdout, so the mapping stays open across ops.

    v = OwnerView(alloc, extent=0)
    alloc.fill(seed=1); alloc.put(0, 0, n)
    assert v.check(seed=1, nbytes=n) == 0     # a kernel on the owner's GPU verifies
    v.fill(seed=2, nbytes=n)                  # ... and writes
    alloc.get(0, 0, n); assert alloc.check(seed=2, nbytes=n) == 0
    v.close()
"""
from __future__ import annotations

import ctypes
import os
import subprocess
import sys


class OwnerView:
    def __init__(self, alloc, extent: int = 0, timeout: float = 120.0):
        reg = alloc.extent_region(extent)
        if reg["owner_gpu"] < 0:
            raise ValueError("owner-side views need an extent in a GPU's HBM")
        self.device = reg["owner_gpu"]
        self.offset = reg["offset"]
        self.bytes = reg["bytes"]
        self.timeout = timeout
        handle = alloc.extent_handle(extent).hex()
        repo = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        env = dict(os.environ, PYTHONPATH=repo + os.pathsep + os.environ.get("PYTHONPATH", ""))
        self.proc = subprocess.Popen([sys.executable, "-u", "-m", "oncilla_amd.utils.owner_side", str(self.device),
                                      handle, str(self.offset), str(self.bytes)],
                                     stdin=subprocess.PIPE, stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                                     text=True, env=env)
        ready = self._read()
        if ready != "ready":
            raise RuntimeError(f"owner-side helper failed: {ready} {self._stderr()}")

    def _stderr(self) -> str:
        try:
            return self.proc.stderr.read()[-2000:] if self.proc.poll() is not None else ""
        except Exception:  # noqa: BLE001 - diagnostics only
            return ""

    def _read(self) -> str:
        line = self.proc.stdout.readline()
        return line.strip() if line else f"helper exited ({self.proc.poll()})"

    def _cmd(self, *words) -> int:
        self.proc.stdin.write(" ".join(str(w) for w in words) + "\n")
        self.proc.stdin.flush()
        out = self._read()
        try:
            v = int(out)
        except ValueError:
            raise RuntimeError(f"owner-side helper: {out} {self._stderr()}") from None
        if v < 0:
            raise RuntimeError(f"owner-side helper: {' '.join(map(str, words))} failed")
        return v

    def fill(self, seed: int, offset: int = 0, nbytes: int | None = None) -> None:
        """Write the word pattern into the extent with a kernel on the owner's GPU."""
        n = self.bytes - offset if nbytes is None else nbytes
        self._cmd("fill", seed, offset, n)

    def check(self, seed: int, offset: int = 0, nbytes: int | None = None) -> int:
        """Mismatching words of the extent, counted by a kernel on the owner's GPU."""
        n = self.bytes - offset if nbytes is None else nbytes
        return self._cmd("check", seed, offset, n)

    def close(self) -> None:
        if self.proc.poll() is None:
            try:
                self.proc.stdin.write("quit\n")
                self.proc.stdin.flush()
                self.proc.wait(timeout=30)
            except Exception:  # noqa: BLE001
                self.proc.kill()
                self.proc.wait()

    def __enter__(self) -> "OwnerView":
        return self

    def __exit__(self, *exc) -> None:
        self.close()


def _serve(argv) -> int:
    from .paths import lib_path

    dev, handle, offset, nbytes = int(argv[0]), bytes.fromhex(argv[1]), int(argv[2]), int(argv[3])
    lib = ctypes.CDLL(lib_path())
    lib.ocm_x_ipc_open.argtypes = [ctypes.c_int, ctypes.c_char_p, ctypes.POINTER(ctypes.c_void_p)]
    lib.ocm_x_ipc_close.argtypes = [ctypes.c_int, ctypes.c_void_p]
    lib.ocm_x_pattern_dev.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64,
                                      ctypes.c_uint32, ctypes.c_int]
    lib.ocm_x_pattern_dev.restype = ctypes.c_longlong
    base = ctypes.c_void_p()
    if lib.ocm_x_ipc_open(dev, handle, ctypes.byref(base)) != 0 or not base.value:
        print("ipc-open-failed", flush=True)
        return 1
    print("ready", flush=True)
    for line in sys.stdin:
        w = line.split()
        if not w or w[0] == "quit":
            break
        op, seed, off, n = w[0], int(w[1]), int(w[2]), int(w[3])
        if off < 0 or n < 0 or off + n > nbytes or off % 4:
            print(-1, flush=True)
            continue
        p = ctypes.c_void_p(base.value + offset + off)
        # pattern word index = byte offset in the extent / 4 (what Allocation.fill/check use)
        r = lib.ocm_x_pattern_dev(dev, p, n // 4, off // 4, seed, 1 if op == "check" else 0)
        print(int(r), flush=True)
    lib.ocm_x_ipc_close(dev, base)
    return 0


if __name__ == "__main__":
    sys.exit(_serve(sys.argv[1:]))

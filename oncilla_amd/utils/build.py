"""Build driver for the native tree: CMake + Ninja, hipcc for gfx950.

`__graft_entry__.build()` calls :func:`build`. Everything lands in ``build/``
inside the repository (``build/lib/libocm.so``, ``build/bin/ocmd`` ...).
"""
from __future__ import annotations

import os
import shutil
import subprocess

from .paths import BUILD_DIR, REPO

ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")


def _env() -> dict:
    env = dict(os.environ)
    env["PATH"] = f"{ROCM}/bin:{ROCM}/llvm/bin:" + env.get("PATH", "")
    env.setdefault("PYTORCH_ROCM_ARCH", "gfx950")
    return env


def build(jobs: int | None = None, sanitize: bool | str = False, verbose: bool = False) -> str:
    """Configure (once) and build every native target. Returns the build dir.

    sanitize: False, True / "address" (ASan+UBSan, ``build-asan``) or
    "thread" (TSan, ``build-tsan``); host code only.
    """
    jobs = jobs or min(16, os.cpu_count() or 8)
    env = _env()
    gen = ["-G", "Ninja"] if shutil.which("ninja", path=env["PATH"]) else []
    if sanitize is True:
        sanitize = "address"
    bdir = BUILD_DIR if not sanitize else BUILD_DIR + ("-tsan" if sanitize == "thread" else "-asan")
    if not os.path.exists(os.path.join(bdir, "CMakeCache.txt")):
        cmd = [
            "cmake", "-S", REPO, "-B", bdir, *gen,
            f"-DCMAKE_HIP_COMPILER={ROCM}/llvm/bin/clang++",
            f"-DCMAKE_CXX_COMPILER={ROCM}/llvm/bin/clang++",
            f"-DCMAKE_PREFIX_PATH={ROCM}",
            "-DCMAKE_BUILD_TYPE=Release",
            "-DCMAKE_HIP_ARCHITECTURES=gfx950",
        ]
        if sanitize:
            cmd.append("-DOCM_SANITIZE=" + ("thread" if sanitize == "thread" else "ON"))
        subprocess.run(cmd, check=True, env=env, capture_output=not verbose)
    subprocess.run(["cmake", "--build", bdir, "-j", str(jobs)], check=True, env=env,
                   capture_output=not verbose)
    return bdir

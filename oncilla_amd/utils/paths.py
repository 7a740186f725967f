"""Locations of the native build products (in-tree, so they travel to the GPU box)."""
from __future__ import annotations

import os

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
BUILD_DIR = os.environ.get("OCM_BUILD_DIR", os.path.join(REPO, "build"))
BIN_DIR = os.path.join(BUILD_DIR, "bin")
LIB_DIR = os.path.join(BUILD_DIR, "lib")


def lib_path() -> str:
    return os.path.join(LIB_DIR, "libocm.so")


def bin_path(name: str) -> str:
    return os.path.join(BIN_DIR, name)


def is_built() -> bool:
    return all(
        os.path.exists(p)
        for p in (lib_path(), bin_path("ocmd"), bin_path("ocm_test"), bin_path("ocm_unit_tests"))
    )

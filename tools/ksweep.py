#!/usr/bin/env python3
"""Grid/variant sweep of the transfer kernel on HBM->HBM copies (event-timed in C)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from oncilla_amd import ops  # noqa: E402

n = 1 << 30
src = torch.randint(0, 255, (n,), dtype=torch.uint8, device="cuda:0")
dst = torch.empty_like(src)
res = {}
for s in (1 << 20, 4 << 20, 16 << 20, 64 << 20, 256 << 20, 1 << 30):
    it = max(5, min(400, (8 << 30) // s))
    row = {}
    for var, name in ((ops.XFER_REG, "reg"), (ops.XFER_LDS, "lds")):
        for b in (128, 256, 512, 1024, 2048):
            for nt in (True, False):
                t = ops.device_copy_seconds(dst, src, s, var, b, nt, it)
                row[f"{name}_b{b}_{'nt' if nt else 'c'}"] = round(s / t / 1e9, 1)
    best = max(row, key=row.get)
    res[s] = {"best": best, "best_GBps": row[best], "all": row}
    print(s, best, row[best], file=sys.stderr, flush=True)
print(json.dumps(res))

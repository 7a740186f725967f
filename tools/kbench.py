#!/usr/bin/env python3
"""Transfer-kernel micro-benchmark on one MI355X.

Measures the gfx950 put/get kernel (csrc/src/kernels/xfer.hip) against the
vendor paths on the same buffers:
  hbm      HBM -> HBM copy: xfer REG/LDS (grid sweep, nt on/off) vs torch copy_ (blit)
  d2h/h2d  device <-> pinned host: xfer kernel through the mapped pointer vs
           hipMemcpyAsync (SDMA) via torch non_blocking copies
  latency  4 KiB .. 256 KiB launch+complete wall time
Prints one JSON document (GB/s = 1e9 bytes moved per second, one direction).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from oncilla_amd import ops  # noqa: E402


def ev_time(fn, iters):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / 1e3 / iters


def wall_time(fn, iters):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
        torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--max-bytes", type=int, default=1 << 30)
    ap.add_argument("--quick", action="store_true")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    n = args.max_bytes
    src = torch.randint(0, 255, (n,), dtype=torch.uint8, device=dev)
    dst = torch.empty(n, dtype=torch.uint8, device=dev)
    out = {"device": torch.cuda.get_device_name(0), "hbm": {}, "d2h": {}, "h2d": {}, "latency_us": {}}

    sizes = [1 << 20, 16 << 20, 256 << 20, n] if not args.quick else [16 << 20, n]
    for s in sizes:
        it = max(3, min(200, (4 << 30) // s))
        row = {"torch_copy": s / ev_time(lambda: dst[:s].copy_(src[:s]), it) / 1e9}
        for blocks in (256, 512, 1024, 2048):
            row[f"reg_b{blocks}"] = s / ev_time(lambda: ops.xfer(src, [dst], 0, 0, s, True, ops.XFER_REG, blocks, sync=False), it) / 1e9
        row["reg_b1024_nt_evt"] = s / ops.device_copy_seconds(dst, src, s, ops.XFER_REG, 1024, True, it) / 1e9
        row["reg_b1024_cached_evt"] = s / ops.device_copy_seconds(dst, src, s, ops.XFER_REG, 1024, False, it) / 1e9
        row["lds_b512_evt"] = s / ops.device_copy_seconds(dst, src, s, ops.XFER_LDS, 512, True, it) / 1e9
        row["lds_b1024_evt"] = s / ops.device_copy_seconds(dst, src, s, ops.XFER_LDS, 1024, True, it) / 1e9
        out["hbm"][s] = {k: round(v, 1) for k, v in row.items()}
        print(f"hbm {s}: {out['hbm'][s]}", file=sys.stderr, flush=True)

    hn = min(n, 256 << 20)
    host = torch.empty(hn, dtype=torch.uint8).pin_memory()
    for s in ([1 << 20, 16 << 20, hn] if not args.quick else [hn]):
        it = max(3, min(100, (1 << 30) // s))
        d2h = {
            "sdma": s / ev_time(lambda: host[:s].copy_(src[:s], non_blocking=True), it) / 1e9,
            "xfer_b256": s / ev_time(lambda: ops.xfer(src, [host], 0, 0, s, True, ops.XFER_REG, 256, sync=False), it) / 1e9,
            "xfer_b1024": s / ev_time(lambda: ops.xfer(src, [host], 0, 0, s, True, ops.XFER_REG, 1024, sync=False), it) / 1e9,
        }
        h2d = {
            "sdma": s / ev_time(lambda: dst[:s].copy_(host[:s], non_blocking=True), it) / 1e9,
            "xfer_b256": s / ev_time(lambda: ops.xfer(dst, [host], 0, 0, s, False, ops.XFER_REG, 256, sync=False), it) / 1e9,
            "xfer_b1024": s / ev_time(lambda: ops.xfer(dst, [host], 0, 0, s, False, ops.XFER_REG, 1024, sync=False), it) / 1e9,
        }
        out["d2h"][s] = {k: round(v, 1) for k, v in d2h.items()}
        out["h2d"][s] = {k: round(v, 1) for k, v in h2d.items()}
        print(f"d2h {s}: {out['d2h'][s]}  h2d {s}: {out['h2d'][s]}", file=sys.stderr, flush=True)

    for s in (4096, 65536, 262144):
        out["latency_us"][s] = {
            "xfer_hbm": round(wall_time(lambda: ops.xfer(src, [dst], 0, 0, s, True, sync=False), 200) * 1e6, 2),
            "torch_copy_hbm": round(wall_time(lambda: dst[:s].copy_(src[:s]), 200) * 1e6, 2),
            "sdma_d2h": round(wall_time(lambda: host[:s].copy_(src[:s], non_blocking=True), 200) * 1e6, 2),
            "xfer_d2h": round(wall_time(lambda: ops.xfer(src, [host], 0, 0, s, True, ops.XFER_REG, 64, sync=False), 200) * 1e6, 2),
        }
    print(json.dumps(out))


if __name__ == "__main__":
    main()

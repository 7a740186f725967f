#!/usr/bin/env python3
"""Host<->device bandwidth on one MI355X with several engines in parallel:
1 vs 2 vs 4 SDMA streams, and SDMA + transfer kernel splitting one buffer."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from oncilla_amd import ops  # noqa: E402

n = 512 << 20
dev = torch.device("cuda:0")
d = torch.empty(n, dtype=torch.uint8, device=dev)
h = torch.empty(n, dtype=torch.uint8).pin_memory()
streams = [torch.cuda.Stream() for _ in range(4)]


def timeit(fn, it=10):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    for st in streams:
        e.wait(st) if False else None
    torch.cuda.synchronize()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / 1e3 / it


def split_sdma(k, d2h):
    def go():
        cur = torch.cuda.current_stream()
        chunk = n // k
        for i in range(k):
            st = streams[i]
            st.wait_stream(cur)
            with torch.cuda.stream(st):
                if d2h:
                    h[i * chunk:(i + 1) * chunk].copy_(d[i * chunk:(i + 1) * chunk], non_blocking=True)
                else:
                    d[i * chunk:(i + 1) * chunk].copy_(h[i * chunk:(i + 1) * chunk], non_blocking=True)
        for i in range(k):
            cur.wait_stream(streams[i])
    return go


def hybrid(frac_kernel, d2h):
    def go():
        cur = torch.cuda.current_stream()
        kb = int(n * frac_kernel) // 4096 * 4096
        st = streams[0]
        st.wait_stream(cur)
        with torch.cuda.stream(st):
            if d2h:
                h[kb:].copy_(d[kb:], non_blocking=True)
            else:
                d[kb:].copy_(h[kb:], non_blocking=True)
        if kb:
            ops.xfer(d, [h], 0, 0, kb, put=d2h, sync=False)  # null stream
        cur.wait_stream(st)
    return go


out = {}
for d2h in (True, False):
    key = "d2h" if d2h else "h2d"
    r = {}
    for k in (1, 2, 4):
        r[f"sdma_x{k}"] = round(n / timeit(split_sdma(k, d2h)) / 1e9, 2)
    for f in (0.25, 0.5):
        r[f"hybrid_kernel{int(f*100)}"] = round(n / timeit(hybrid(f, d2h)) / 1e9, 2)
    r["kernel_only"] = round(n / timeit(lambda: ops.xfer(d, [h], 0, 0, n, put=d2h, sync=False)) / 1e9, 2)
    out[key] = r
    print(key, r, file=sys.stderr, flush=True)
print(json.dumps(out))

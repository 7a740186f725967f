"""Which footprint of a resident poller delays a full-GPU GEMM (the cost of the
copy service's lone lead). A bf16 8192^3 torch matmul, timed on its own stream,
with nothing resident and with one persistent workgroup of 64 or 256 threads, light
or ~100 VGPRs (build/lib/libresident_probe.so), interleaved.

    python tools/resident_cost_probe.py [--rounds 3] [--out ...]
"""
import argparse
import ctypes
import json
import os
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    import torch

    lib = ctypes.CDLL(os.path.join(REPO, "build", "lib", "libresident_probe.so"))
    x = torch.randn(8192, 8192, device="cuda:0", dtype=torch.bfloat16)
    st = torch.cuda.current_stream()

    def mm():
        ts = []
        for _ in range(7):
            t0 = time.perf_counter()
            y = x @ x
            st.synchronize()
            ts.append(time.perf_counter() - t0)
            del y
        return round(sorted(ts)[3] * 1e3, 3)

    mm()
    res = {}
    for k in range(a.rounds):
        for name, thr, heavy in (("none", 0, 0), ("wave64_light", 64, 0), ("wg256_light", 256, 0),
                                 ("wave64_heavy", 64, 1), ("wg256_heavy", 256, 1)):
            if thr:
                assert lib.ocmp_start(thr, heavy) == 0
                time.sleep(0.001)
            t = mm()
            if thr:
                assert lib.ocmp_stop() == 0
            res.setdefault(name, []).append(t)
        print(k, json.dumps({n: v[-1] for n, v in res.items()}), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()

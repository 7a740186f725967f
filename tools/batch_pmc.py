"""Daemon-free driver of the batch kernel for rocprofv3 counter runs:
32768 random 4 KiB gets from a 3-extent striped buffer (64 KiB units), 20 launches.

    cd /tmp && rocprofv3 --kernel-trace --pmc FETCH_SIZE -d out -- python3 $REPO/tools/batch_pmc.py
Expected per launch: 128 MiB read and 128 MiB written (each byte once).
"""
import os
import random
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from oncilla_amd import ops  # noqa: E402


def main():
    unit, n_ext, piece, count = 64 << 10, 3, 4096, 32768
    ext_bytes = 256 << 20
    exts = [torch.empty(ext_bytes, dtype=torch.uint8, device="cuda:0").random_(0, 255) for _ in range(n_ext)]
    lin = torch.zeros(count * piece, dtype=torch.uint8, device="cuda:0")
    rng = random.Random(1)
    slots = rng.sample(range(n_ext * ext_bytes // piece - 16), count)
    batch = [(False, i * piece, s * piece, piece) for i, s in enumerate(slots)]
    ops.batch(lin, exts, unit, batch, iters=20)
    torch.cuda.synchronize()
    print(f"{count} x {piece} B gets x 20 launches done")


if __name__ == "__main__":
    main()

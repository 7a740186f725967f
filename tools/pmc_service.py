"""Workload for rocprofv3 --pmc passes over the data-plane kernels.

On a loopback HBM pair (the owner daemon's HBM, IPC-mapped) and a pinned host-tier pair it runs:
- 200 blocking 1 MiB puts and 200 gets: one resident service_kernel dispatch serves all of them;
- 8 puts and 8 gets of 256 MiB: xfer kernel launches (on the host tier: the PCIe streaming kernel);
- 4 fused remote-Adam steps over 64 Mi fp32 parameters with the moments in the host tier (round 3's
  PCIe variant of the kernel).
Per-dispatch FETCH_SIZE / WRITE_SIZE then show how many bytes each kernel moved for the bytes requested,
including the service's polling overhead.

    rocprofv3 --pmc FETCH_SIZE --kernel-trace -d out -o fetch -- python3 tools/pmc_service.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from oncilla_amd import api  # noqa: E402
from oncilla_amd.parallel.mesh import Mesh  # noqa: E402


def main() -> None:
    with Mesh(2, gpus=[0, 0]) as m:
        with api.Client(daemon_rank=0, gpu=0, ns=m.ns) as c:
            for flags, tier in ((api.OCM_ALLOC_LOOPBACK, "hbm"), (api.OCM_ALLOC_HOST_TIER, "host")):
                n = 256 << 20
                a = c.alloc(api.OCM_REMOTE_GPU, local_bytes=n, remote_bytes=n, flags=flags)
                for i in range(200):
                    a.put(0, (i % 64) << 20, 1 << 20)
                for i in range(200):
                    a.get(0, (i % 64) << 20, 1 << 20)
                for _ in range(8):
                    a.put(0, 0, n)
                for _ in range(8):
                    a.get(0, 0, n)
                a.free()
                print(f"{tier}: 200 x 1 MiB put + get (service), 8 x 256 MiB put + get (launches)", flush=True)
            import torch

            from oncilla_amd.models import OffloadedAdam

            p = torch.zeros(64 << 20, device="cuda:0").requires_grad_()
            p.grad = torch.randn(64 << 20, device="cuda:0")
            opt = OffloadedAdam([p], c, lr=1e-3, flags=api.OCM_ALLOC_HOST_TIER)
            for _ in range(4):
                opt.step()
            opt.synchronize()
            opt.close()
            print("adam: 4 fused steps, 64 Mi params, moments in the host tier", flush=True)


if __name__ == "__main__":
    main()

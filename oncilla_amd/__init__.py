"""oncilla_amd — MI355X-native disaggregated memory (OncillaMem capabilities).

Native core (C++/HIP, built in-tree under ``build/``):
  * ``ocmd``       per-GPU daemon: mailbox control plane, rank0 governor,
                   HBM / pinned-host-tier arenas, mesh protocol, crash reclaim
  * ``libocm.so``  the ``oncillamem.h`` C ABI: ocm_alloc/free/copy/copy_onesided
                   with gfx950 put/get kernels over xGMI peer mappings
Python: ``api`` (ctypes binding), ``parallel`` (mesh launcher, torch.distributed
glue), ``models`` (benchmark workloads), ``ops`` (raw transfer kernels).
"""
__version__ = "0.1.0"

from . import api  # noqa: F401
from .api import (  # noqa: F401
    OCM_LOCAL_GPU,
    OCM_LOCAL_HOST,
    OCM_REMOTE_GPU,
    OCM_REMOTE_RDMA,
    OCM_REMOTE_RMA,
    Allocation,
    Client,
    OcmError,
)

"""Multi-daemon / multi-GPU orchestration: the ocmd mesh launcher and the
torch.distributed (RCCL) glue for one-process-per-GPU runs."""
from .mesh import Mesh, free_ports, write_nodefile

__all__ = ["Mesh", "free_ports", "write_nodefile"]

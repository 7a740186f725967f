"""Raw access to the gfx950 transfer kernels (tests, micro-benchmarks)."""
from .xfer import XFER_AUTO, XFER_LDS, XFER_PCIE, XFER_PUSH, XFER_REG, batch, device_copy_seconds, striped_reference, xfer

__all__ = ["XFER_AUTO", "XFER_LDS", "XFER_PCIE", "XFER_PUSH", "XFER_REG", "batch", "device_copy_seconds", "striped_reference", "xfer"]

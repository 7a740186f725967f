"""Workloads on the runtime: the BASELINE.json configs (#1-#5) and a serving
use of disaggregated memory (paged KV-cache offload)."""
from .kv_offload import PagedKVOffload, coalesce
from .optim_offload import OffloadedAdam, OffloadedAdamW
from .workloads import alloc_latency, characterize, churn, percentile, rw_sweep_step, spill_probe, sweep_sizes

__all__ = ["OffloadedAdam", "OffloadedAdamW", "PagedKVOffload", "alloc_latency", "characterize", "churn", "coalesce", "percentile", "rw_sweep_step",
           "spill_probe", "sweep_sizes"]

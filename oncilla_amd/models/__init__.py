"""Benchmark workloads (BASELINE.json configs #1-#5)."""
from .workloads import alloc_latency, characterize, churn, percentile, rw_sweep_step, spill_probe, sweep_sizes

__all__ = ["alloc_latency", "characterize", "churn", "percentile", "rw_sweep_step", "spill_probe", "sweep_sizes"]

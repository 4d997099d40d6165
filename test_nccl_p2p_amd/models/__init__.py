"""Traffic models: which point-to-point message sizes real parallel LLM
workloads put on the xGMI fabric, so sweeps measure the sizes that matter."""

from .traffic import PRESETS, ModelShape, ParallelConfig, traffic_for  # noqa: F401

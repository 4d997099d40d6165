"""Statistics, report formatting/parsing, scaling curves, RCCL environment.

`report` is imported lazily so `python -m test_nccl_p2p_amd.utils.report`
runs it as a fresh module."""

from .stats import percentile, summarize  # noqa: F401


def __getattr__(name):
    if name in ("compat_matrix_text", "parse_compat"):
        from . import report

        return getattr(report, name)
    raise AttributeError(name)

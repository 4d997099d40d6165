"""Statistics, report formatting/parsing, scaling curves, RCCL environment."""

from .report import compat_matrix_text, parse_compat  # noqa: F401
from .stats import percentile, summarize  # noqa: F401

"""Sample statistics, identical conventions to csrc/stats.cpp (linear
interpolation between closest ranks, numpy's default percentile)."""

from __future__ import annotations

import math
from typing import Dict, Iterable, List, Sequence


def percentile(samples: Iterable[float], q: float) -> float:
    s = sorted(samples)
    if not s:
        return 0.0
    if q <= 0:
        return s[0]
    if q >= 100:
        return s[-1]
    pos = q / 100.0 * (len(s) - 1)
    lo = int(math.floor(pos))
    hi = min(lo + 1, len(s) - 1)
    return s[lo] + (s[hi] - s[lo]) * (pos - lo)


def summarize(samples: Sequence[float]) -> Dict[str, float]:
    s = list(samples)
    if not s:
        return {"n": 0, "min": 0.0, "max": 0.0, "mean": 0.0, "stdev": 0.0, "p50": 0.0, "p90": 0.0, "p99": 0.0}
    mean = sum(s) / len(s)
    var = sum((x - mean) ** 2 for x in s) / (len(s) - 1) if len(s) > 1 else 0.0
    return {"n": len(s), "min": min(s), "max": max(s), "mean": mean, "stdev": math.sqrt(var),
            "p50": percentile(s, 50), "p90": percentile(s, 90), "p99": percentile(s, 99)}


def offdiag_summary(m: List[List[float]], skip_zero: bool = True) -> Dict[str, float]:
    n = len(m)
    vals = [m[i][j] for i in range(n) for j in range(n) if (n == 1 or i != j) and not (skip_zero and m[i][j] == 0)]
    if not vals:
        return {"min": 0.0, "mean": 0.0, "max": 0.0, "cells": 0}
    return {"min": min(vals), "mean": sum(vals) / len(vals), "max": max(vals), "cells": len(vals)}

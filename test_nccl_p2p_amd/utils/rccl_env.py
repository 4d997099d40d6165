"""RCCL / NCCL environment knobs relevant to point-to-point performance.

The reference sets none and inherits whatever NCCL_* the shell has
(SURVEY.md §2.6).  These are captured into every result so a number is never
reported without the tuning that produced it, and ``scripts/rccl_sweep.sh``
sweeps them.  Presence of each knob was checked against the strings of
ROCm 7.2's librccl.so during the survey.
"""

from __future__ import annotations

import os
from typing import Dict

P2P_KNOBS = (
    "NCCL_NCHANNELS_PER_PEER",
    "NCCL_MIN_P2P_NCHANNELS",
    "NCCL_MAX_P2P_NCHANNELS",
    "NCCL_P2P_NVL_CHUNKSIZE",
    "NCCL_P2P_PCI_CHUNKSIZE",
    "NCCL_BUFFSIZE",
    "NCCL_PROTO",
    "NCCL_P2P_LL_THRESHOLD",
    "NCCL_P2P_READ_ENABLE",
    "NCCL_P2P_USE_CUDA_MEMCPY",
    "NCCL_RUNTIME_CONNECT",
    "RCCL_P2P_BATCH_ENABLE",
    "RCCL_P2P_BATCH_THRESHOLD",
    "NCCL_DEBUG",
    "HSA_ENABLE_IPC_MODE_LEGACY",
)


def capture() -> Dict[str, str]:
    """Every NCCL_/RCCL_/HSA_ variable currently set, plus the known knobs."""
    out = {k: v for k, v in os.environ.items() if k.startswith(("NCCL_", "RCCL_", "HSA_"))}
    for k in P2P_KNOBS:
        out.setdefault(k, "")
    return dict(sorted(out.items()))

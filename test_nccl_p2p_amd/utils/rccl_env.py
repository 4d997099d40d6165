"""RCCL / NCCL environment knobs relevant to point-to-point performance.

The reference sets none and inherits whatever NCCL_* the shell has
(SURVEY.md §2.6).  Every result records the environment it ran under: the
native engine writes it (csrc/provenance.cpp: env_knobs_json, the
``provenance`` object of the bench JSON and of ``p2p_matrix --json``).  This
module is the Python-side list of the knobs the sweeps vary and the snapshot
the sweep scripts store next to their rows (scripts/xgmi_pair_sweep.py,
scripts/rccl_env_sweep.py).  Presence of each knob was checked against the
strings of ROCm 7.2's librccl.so during the survey.
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
    "NCCL_P2P_NET_CHUNKSIZE",
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
    "GPU_MAX_HW_QUEUES",
)


def capture() -> Dict[str, str]:
    """Every NCCL_/RCCL_/HSA_ variable currently set, plus the known knobs."""
    out = {k: v for k, v in os.environ.items() if k.startswith(("NCCL_", "RCCL_", "HSA_", "GPU_MAX_HW_QUEUES"))}
    for k in P2P_KNOBS:
        out.setdefault(k, "")
    return dict(sorted(out.items()))

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
from typing import Dict, List, Tuple

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


def linked_librccl() -> str:
    """The librccl.so that csrc/ links against: the one torch bundles (Makefile RTDIR)."""
    import torch

    return os.path.join(os.path.dirname(torch.__file__), "lib", "librccl.so")


# Each pattern starts with a literal (a linear scan of the 300+ MB library).
_FORMAT_RES = (
    rb"(?:Channel|CollNet) %02d[^\x00\n]*? via [^\x00\n]*",  # connections
    rb"%d coll channels, [^\x00\n]*p2p channels per peer",  # channel counts
    rb"comm %p rank %d nRanks %d nNodes %d[^\x00\n]*",  # ranks / nodes
    rb"RCCL Unroll Factor \([a-z-]+\): %d",
)


def log_formats(path: str) -> Tuple[str, List[str]]:
    """(RCCL version, sorted printf formats of the INFO lines csrc/rccl_log.cpp parses).

    Read from a librccl's bytes: the connection lines (``Channel cc/i :
    a[bus] -> b[bus] via P2P/IPC … comm 0x… nRanks NN``) and the init lines
    parse_rccl_init reads.  The file is memory-mapped and searched; nothing in
    it is loaded or run.
    """
    import mmap
    import re

    with open(path, "rb") as f, mmap.mmap(f.fileno(), 0, access=mmap.ACCESS_READ) as m:
        found = re.search(rb"RCCL version : ([0-9][0-9.]*[0-9])", m)
        ver = found.group(1).decode() if found else ""
        fmts = sorted({x.decode() for r in _FORMAT_RES for x in re.findall(r, m)})
    return ver, fmts


def read_pinned_formats(path: str) -> List[str]:
    """The formats of a tests/data/rccl_<version>_log_formats.txt file."""
    with open(path) as f:
        return [line.rstrip("\n") for line in f if line.strip() and not line.startswith("#")]

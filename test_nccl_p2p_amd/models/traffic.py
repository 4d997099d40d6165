"""Point-to-point traffic of parallel LLM training/serving on one MI355X node.

The reference measures a single 32 MiB message size (p2p_matrix.cc:124).
Which sizes matter depends on the workload that will run over the fabric;
this module derives them from a model shape and a parallel layout:

* pipeline parallel (PP): each stage boundary sends one activation (forward)
  and one activation-gradient (backward) per micro-batch to the neighbour
  stage -> the ``ring`` mode, message = micro_batch * seq * hidden * bytes.
* expert parallel (EP): every MoE layer dispatches tokens to the experts'
  ranks and combines them back -> the ``allpairs`` mode, per-peer message =
  tokens * top_k * hidden * bytes / ep (uniform routing).
* context parallel (CP, ring attention): each step passes one K/V chunk to the
  next rank -> the ``ring`` mode, message = 2 * (seq / cp) * kv_heads *
  head_dim * bytes per layer.

``traffic_for`` returns the sizes and the matching p2p_matrix invocation.
These are analytic models (no checkpoint or dataset involved).
"""

from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, List


@dataclass(frozen=True)
class ModelShape:
    name: str
    hidden: int
    layers: int
    heads: int
    kv_heads: int
    head_dim: int
    experts: int = 0
    top_k: int = 0


@dataclass(frozen=True)
class ParallelConfig:
    tp: int = 1
    pp: int = 1
    ep: int = 1
    cp: int = 1
    micro_batch: int = 1
    seq_len: int = 4096
    dtype_bytes: int = 2  # bf16 activations


PRESETS: Dict[str, ModelShape] = {
    "llama3-8b": ModelShape("llama3-8b", 4096, 32, 32, 8, 128),
    "llama3-70b": ModelShape("llama3-70b", 8192, 80, 64, 8, 128),
    "llama3-405b": ModelShape("llama3-405b", 16384, 126, 128, 8, 128),
    "mixtral-8x7b": ModelShape("mixtral-8x7b", 4096, 32, 32, 8, 128, experts=8, top_k=2),
    "deepseek-v3": ModelShape("deepseek-v3", 7168, 61, 128, 128, 128, experts=256, top_k=8),
}


def _pow2_floor(x: int) -> int:
    p = 1
    while p * 2 <= x:
        p *= 2
    return p


def traffic_for(model: ModelShape, par: ParallelConfig) -> Dict[str, object]:
    out: Dict[str, object] = {"model": model.name, "flows": []}
    flows: List[Dict[str, object]] = []
    tokens = par.micro_batch * par.seq_len // max(par.cp, 1)
    if par.pp > 1:
        # Sequence-parallel TP shards the boundary activation over tp ranks.
        act = tokens * model.hidden * par.dtype_bytes // max(par.tp, 1)
        flows.append({"pattern": "pp-activation", "mode": "ring", "dir": "uni", "bytes": act,
                      "per_step": 2 * (par.pp - 1), "note": "fwd activation + bwd grad per micro-batch"})
    if par.ep > 1 and model.experts:
        per_peer = tokens * model.top_k * model.hidden * par.dtype_bytes // par.ep
        flows.append({"pattern": "ep-dispatch", "mode": "allpairs", "dir": "bi", "bytes": per_peer,
                      "per_step": 2 * model.layers, "note": "dispatch + combine per MoE layer"})
    if par.cp > 1:
        kv = 2 * (par.seq_len // par.cp) * model.kv_heads * model.head_dim * par.dtype_bytes * par.micro_batch
        flows.append({"pattern": "cp-kv-ring", "mode": "ring", "dir": "uni", "bytes": kv,
                      "per_step": (par.cp - 1) * model.layers, "note": "K/V chunk per ring-attention step"})
    out["flows"] = flows
    sizes = sorted({_pow2_floor(int(f["bytes"])) for f in flows if int(f["bytes"]) > 0})
    out["sweep"] = sizes
    cmds = []
    for f in flows:
        cmds.append("mpirun -n %d ./build/p2p_matrix --mode %s --dir %s --size %d --verify"
                    % (max(par.pp, par.ep, par.cp), f["mode"], f["dir"], f["bytes"]))
    out["commands"] = cmds
    return out

"""torch.distributed harness: the same schedules over gloo (CPU) or nccl (RCCL).

BASELINE.json config 1 — "2-rank CPU/gloo send/recv of a 4 KiB buffer
(plumbing, runs without a GPU)" — is this module with backend gloo.  It runs
the Python mirror of the native schedules (``parallel/schedule.py``) with
``dist.batch_isend_irecv`` groups, verifies payloads against the PyTorch PRNG
reference, times each cell with barriers + perf_counter (the reference's
wall-clock bracket, /root/reference/p2p_matrix.cc:146-176) and prints the
reference-compatible matrices through ``utils.report``.

It is a plumbing / cross-check path: the measured data plane of the framework
is the native engine (``build/p2p_matrix``, ``bench.py``).

    torchrun --nproc-per-node 2 -m test_nccl_p2p_amd.parallel.gloo_harness --size 4K
"""

from __future__ import annotations

import argparse
import sys
import time
from typing import Dict, List, Optional

import torch
import torch.distributed as dist

from ..ops.buffers import payload_seed, reference_bytes
from ..utils.report import compat_matrix_text
from ..utils.stats import summarize
from .schedule import Phase, make_schedule
from .session import init_control_plane


def _post(phase: Phase, rank: int, send: torch.Tensor, recvs: List[torch.Tensor]):
    ops = []
    for peer in phase.send_to[rank]:
        ops.append(dist.P2POp(dist.isend, send, peer))
    for i, peer in enumerate(phase.recv_from[rank]):
        ops.append(dist.P2POp(dist.irecv, recvs[i], peer))
    return ops


def _run_iteration(phase: Phase, rank: int, send: torch.Tensor, recvs: List[torch.Tensor]) -> None:
    # Self flows are local copies (gloo has no send-to-self).
    self_slots = [i for i, p in enumerate(phase.recv_from[rank]) if p == rank]
    for i in self_slots:
        recvs[i].copy_(send)
    ops = [op for op in _post(phase, rank, send, recvs) if op.peer != rank]
    if ops:
        for w in dist.batch_isend_irecv(ops):
            w.wait()


def run_phase(phase: Phase, nbytes: int, iters: int, warmup: int, verify: bool, device: str, salt: int = 0) -> Dict:
    rank = dist.get_rank() if dist.is_initialized() else 0
    active = phase.participates(rank)
    send = reference_bytes(nbytes, payload_seed(rank, nbytes, salt), device)
    recvs = [torch.zeros(nbytes, dtype=torch.uint8, device=device) for _ in phase.recv_from[rank]]

    def sync():
        if device != "cpu":
            torch.cuda.synchronize()

    def barrier():
        if dist.is_initialized():
            dist.barrier()

    barrier()
    if phase.idle:
        return {"idle": True, "seconds": 0.0, "gbps": 0.0, "samples_us": [], "mismatches": 0}
    if active:
        for _ in range(warmup):
            _run_iteration(phase, rank, send, recvs)
        sync()
    barrier()
    t0 = time.perf_counter()
    samples = []
    if active:
        for _ in range(iters):
            a = time.perf_counter()
            _run_iteration(phase, rank, send, recvs)
            sync()
            samples.append((time.perf_counter() - a) * 1e6)
    barrier()
    secs = time.perf_counter() - t0
    mism = 0
    if verify and active:
        for i, peer in enumerate(phase.recv_from[rank]):
            want = reference_bytes(nbytes, payload_seed(peer, nbytes, salt), device)
            mism += int((recvs[i] != want).sum().item())
    t = torch.tensor([secs, float(mism)], dtype=torch.float64)
    if dist.is_initialized():
        allv = [torch.zeros_like(t) for _ in range(dist.get_world_size())]
        dist.all_gather(allv, t)
        secs = max(float(v[0]) for v in allv)
        mism = int(sum(float(v[1]) for v in allv))
    per_iter = secs / iters
    gbps = nbytes * len(phase.flows) * 8.0 / per_iter / 1e9
    return {"idle": False, "seconds": per_iter, "gbps": gbps, "samples_us": samples, "mismatches": mism}


def run(mode: str = "pair", directions=("uni", "bi"), nbytes: int = 4096, iters: int = 100, warmup: int = 5,
        verify: bool = True, device: str = "cpu", out=sys.stdout) -> Dict:
    rank = dist.get_rank() if dist.is_initialized() else 0
    n = dist.get_world_size() if dist.is_initialized() else 1
    results = {}
    for d in directions:
        phases = make_schedule(mode, d, n)
        cells = [run_phase(p, nbytes, iters, warmup, verify, device, salt=i) for i, p in enumerate(phases)]
        results[d] = {"phases": [p.label for p in phases], "cells": cells}
        if mode == "pair" and rank == 0 and out is not None:
            m = [[0.0] * n for _ in range(n)]
            for p, c in zip(phases, cells):
                m[p.row][p.col] = c["gbps"]
            out.write(compat_matrix_text(m, d, leading_newline=(d == "bi")))
            out.flush()
    results["latency_us"] = summarize([s for d in directions for c in results[d]["cells"] for s in c["samples_us"]])
    results["mismatches"] = sum(c["mismatches"] for d in directions for c in results[d]["cells"])
    return results


def main(argv: Optional[List[str]] = None) -> int:
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--mode", default="pair")
    ap.add_argument("--dir", default="both", choices=["uni", "bi", "both"])
    ap.add_argument("--size", default="4K")
    ap.add_argument("--iters", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--backend", default="gloo", choices=["gloo", "nccl"])
    args = ap.parse_args(argv)
    from .. import require_native

    env = init_control_plane(args.backend)
    device = "cpu"
    if args.backend == "nccl":
        torch.cuda.set_device(env.local_rank)
        device = "cuda:%d" % env.local_rank
    nbytes = require_native().parse_size(args.size)
    dirs = ("uni", "bi") if args.dir == "both" else (args.dir,)
    res = run(args.mode, dirs, nbytes, args.iters, args.warmup, True, device)
    if env.rank == 0:
        lat = res["latency_us"]
        print("\n# %s over %s: %d rank(s), %s, per-iteration p50 %.1f us, mismatches %d"
              % (args.mode, args.backend, env.world, args.size, lat["p50"], res["mismatches"]))
    if dist.is_initialized():
        dist.destroy_process_group()
    return 0 if res["mismatches"] == 0 else 2


if __name__ == "__main__":
    sys.exit(main())

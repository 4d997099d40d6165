#!/usr/bin/env python3
"""A/B of the StepDriver posting variants on this node's GPUs (1 rank: the
RCCL self path): one group per message vs one group per step (--batch) vs
hipGraph-captured steps (--graph), at several message sizes.

    python scripts/step_variants.py [--sizes 64K,1M,32M] [--msgs 8] [--steps 50]
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import test_nccl_p2p_amd  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="64K,1M,32M")
    ap.add_argument("--msgs", type=int, default=8)
    ap.add_argument("--steps", type=int, default=50)
    a = ap.parse_args()
    nat = test_nccl_p2p_amd.require_native()
    torch.cuda.set_device(0)
    sess = nat.Session(0, 1, device=0, transport="rccl")
    for sz in [nat.parse_size(s) for s in a.sizes.split(",")]:
        for batch, graph in [(False, False), (True, False), (False, True), (True, True)]:
            d = nat.StepDriver(sess, "self", "bi", sz, a.msgs, True, batch, graph)
            d.connect()
            d.run_steps(0, 5)
            d.sync()
            d.reset()
            t0 = time.perf_counter()
            d.run_steps(5, a.steps)
            d.sync()
            dt = time.perf_counter() - t0
            ms = sorted(d.step_ms())
            bad = d.verify_last()
            gbs = d.job_bytes_per_step(0) * a.steps / dt / 1e9
            print("%6s batch=%d graph=%d: wall %.1f GB/s, step p50 %.1f us (GPU), mismatches %d"
                  % (nat.format_size(sz), batch, graph, gbs, ms[len(ms) // 2] * 1e3, bad), flush=True)
            del d


if __name__ == "__main__":
    main()

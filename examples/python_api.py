#!/usr/bin/env python3
"""Tour of the Python API on one GPU (or CPU with --transport host).

    python examples/python_api.py [--transport rccl|ipc|host]
    torchrun --nproc-per-node 2 examples/python_api.py --transport host
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import test_nccl_p2p_amd  # noqa: E402
from test_nccl_p2p_amd.models import PRESETS, ParallelConfig, traffic_for  # noqa: E402
from test_nccl_p2p_amd.parallel.session import create_session  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--transport", default="rccl")
    a = ap.parse_args()
    nat = test_nccl_p2p_amd.require_native()

    # 1) Device kernels on torch tensors (GPU only).
    if a.transport != "host" and torch.cuda.is_available():
        from test_nccl_p2p_amd.ops import fill_, reference_bytes, verify

        t = torch.empty(1 << 20, dtype=torch.uint8, device="cuda")
        fill_(t, seed=42)
        assert torch.equal(t.cpu(), reference_bytes(1 << 20, 42))
        print("verify:", verify(t, 42))

    # 2) A session: bootstrap + transport (collective under torchrun).
    sess = create_session(a.transport)
    print("rank %d/%d on %s" % (sess.rank, sess.world, sess.device_desc))

    # 3) One schedule run -> JSON (same schema as p2p_matrix --json).
    r = json.loads(sess.run(mode="tournament", dir="bi", bytes=8 << 20, iters=16, warmup=4, verify=True))
    if sess.rank == 0:
        print("tournament GB/s min/mean/max: %.1f / %.1f / %.1f" % (r["gbs_min"], r["gbs_mean"], r["gbs_max"]))

    # 4) Latency matrix.
    lat = json.loads(sess.latency(8, 200, 20))
    if sess.rank == 0:
        print("p50 one-way latency per pair (us):", [round(p["one_way_us"]["p50"], 2) for p in lat["pairs"]])

    # 5) Step driver: what bench.py times.
    d = nat.StepDriver(sess, "tournament" if sess.world > 1 else "self", "bi", 4 << 20, 4, True, True, False)
    d.connect()
    d.run_steps(0, 8)
    d.sync()
    print("rank %d step ms:" % sess.rank, [round(x, 3) for x in d.step_ms()], "mismatches", d.verify_last())
    del d

    # 6) Which sizes matter for a real workload?
    t = traffic_for(PRESETS["llama3-70b"], ParallelConfig(pp=8, micro_batch=1, seq_len=8192))
    if sess.rank == 0:
        print("llama3-70b PP=8 hop message:", nat.format_size(t["flows"][0]["bytes"]), "->", t["commands"][0])
    del sess


if __name__ == "__main__":
    main()

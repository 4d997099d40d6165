#!/usr/bin/env python3
"""Multi-op copy kernel: one launch over several (dst, src) ops vs one op of
the same total size.  The IPC transport launches a group's receives as one
multi-copy grid (kernels.hip multi_copy_kernel); a bench step at the default
shape is 32 receives of 32 MiB = two launches of 16 ops.

    python scripts/probes/copy_ops_probe.py            # current lookup
    (round 2's A/B; its P2P_COPY_LOOKUP=linear / P2P_COPY_MAX_OPS knobs were
    removed from the kernel in round 5, profiles/r2_copy_lookup/ keeps the numbers)
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--total", default="512M")
    ap.add_argument("--ops", default="1,2,4,8,16")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--uneven", type=int, default=1, help="1: also 16 ops of alternating sizes (binary search path)")
    a = ap.parse_args()
    import torch
    from test_nccl_p2p_amd import require_native
    nat = require_native()
    total = nat.parse_size(a.total)
    src = torch.empty(total, dtype=torch.uint8, device="cuda")
    dst = torch.empty(total, dtype=torch.uint8, device="cuda")
    nat.fill(src.data_ptr(), total, 7)
    stream = torch.cuda.current_stream().cuda_stream
    s0, d0 = src.data_ptr(), dst.data_ptr()

    def run(label, ops):
        for _ in range(3):
            nat.copy_many(ops, stream)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.reps):
            nat.copy_many(ops, stream)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / a.reps
        ok = torch.equal(src, dst)
        row = {"case": label, "ops": len(ops), "us": round(us, 1), "tbs": round(total / us / 1e6, 3), "ok": ok,
               "lookup": os.environ.get("P2P_COPY_LOOKUP", "auto")}
        print(json.dumps(row), flush=True)
        dst.zero_()

    for k in [int(x) for x in a.ops.split(",")]:
        per = total // k
        run("even", [(d0 + i * per, s0 + i * per, per) for i in range(k)])
    if a.uneven:
        sizes, off, ops = [], 0, []
        unit = total // 24
        unit -= unit % 4096
        for i in range(16):
            sizes.append(unit * (1 if i % 2 == 0 else 2))
        sizes[-1] = total - sum(sizes[:-1])
        for sz in sizes:
            ops.append((d0 + off, s0 + off, sz))
            off += sz
        run("uneven", ops)


if __name__ == "__main__":
    main()

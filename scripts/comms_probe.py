#!/usr/bin/env python3
"""RCCL communicators per rank vs step throughput on the 1-GPU self path.

One StepDriver step = --msgs self send/recv messages of --size in one group
(bench.py's N=1 step).  With K communicators the messages are spread over K
RCCL send/recv kernels on K streams (csrc/transport_rccl.cpp).  Run once per
GPU_MAX_HW_QUEUES setting (it is read when HIP initialises):

    GPU_MAX_HW_QUEUES=4 python scripts/comms_probe.py --comms 1,2,3,4,6,8
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--comms", default="1,2,3,4,6,8")
    ap.add_argument("--size", default="32M")
    ap.add_argument("--msgs", type=int, default=8)
    ap.add_argument("--steps", type=int, default=60)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--graph", type=int, default=0, help="1: replay each step as a captured hipGraph")
    a = ap.parse_args()
    from test_nccl_p2p_amd import require_native
    nat = require_native()
    size = nat.parse_size(a.size)
    rows = []
    for k in [int(x) for x in a.comms.split(",")]:
        s = nat.Session(0, 1, device=0, transport="rccl:%d" % k if k > 1 else "rccl", timeout_s=120)
        d = nat.StepDriver(s, "self", "bi", size, a.msgs, False, True, bool(a.graph))
        d.connect()
        d.run_steps(0, 5)
        d.sync()
        best, post = 0.0, 0.0
        for r in range(a.reps):
            t0 = time.perf_counter()
            d.run_steps(5 + r * a.steps, a.steps)
            t1 = time.perf_counter()
            d.sync()
            dt = time.perf_counter() - t0
            if size * a.msgs * a.steps / dt / 1e9 > best:
                best, post = size * a.msgs * a.steps / dt / 1e9, (t1 - t0) / a.steps * 1e6
        del d
        lat = json.loads(s.latency(8, 300, 30))["pairs"][0]["one_way_us"]["p50"]
        rows.append({"comms": k, "graph": a.graph, "gbs": round(best, 1), "host_post_us_per_step": round(post, 1),
                     "lat8_p50_us": round(lat, 2),
                     "gpu_us_per_step": round(size * a.msgs / best / 1e3, 1),
                     "hw_queues": os.environ.get("GPU_MAX_HW_QUEUES", "default")})
        print(json.dumps(rows[-1]), flush=True)
        del s


if __name__ == "__main__":
    main()

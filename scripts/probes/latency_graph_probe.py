#!/usr/bin/env python3
"""Small-message self send/recv on one GPU: eager groups vs hipGraph replay.

One step = one grouped 8-byte self send/recv (the latency ping-pong's shape on
one GPU).  Reports the median per-step GPU time from the StepDriver marks for
eager posting and for a captured graph replayed per step.

    python scripts/probes/latency_graph_probe.py [--bytes 8] [--steps 2000]
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--bytes", type=int, default=8)
    ap.add_argument("--steps", type=int, default=2000)
    a = ap.parse_args()
    from test_nccl_p2p_amd import require_native
    nat = require_native()
    s = nat.Session(0, 1, device=0, transport="rccl", timeout_s=120)
    for graph in (False, True):
        d = nat.StepDriver(s, "self", "bi", max(a.bytes, 16), 1, False, True, graph)
        d.connect()
        d.run_steps(0, 100)
        d.sync()
        d.reset()
        d.run_steps(100, a.steps)
        d.sync()
        ms = d.step_ms()
        print(json.dumps({"graph": graph, "bytes": max(a.bytes, 16), "step_us_p50": round(statistics.median(ms) * 1e3, 2),
                          "step_us_min": round(min(ms) * 1e3, 2)}), flush=True)
        del d
    del s


if __name__ == "__main__":
    main()

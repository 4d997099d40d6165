#!/usr/bin/env python3
"""Probes RCCL send/recv correctness at large message sizes (self path, one
GPU) with device-side verification, varying iterations and the comm mode.

    python scripts/probes/rccl_size_probe.py [iters] [sizes...]
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import test_nccl_p2p_amd  # noqa: E402


def main():
    nat = test_nccl_p2p_amd.require_native()
    torch.cuda.set_device(0)
    sess = nat.Session(0, 1, device=0, transport="rccl")
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 1
    sizes = [int(x) for x in sys.argv[2:]] or [(1 << 30) + 16, (3 << 29), (1 << 31) - 16, (1 << 31) + 16,
                                               (5 << 30) + 16]
    for b in sizes:
        for it, wu in ((iters, 0), (iters, 1)):
            r = json.loads(sess.run(mode="self", dir="uni", bytes=b, iters=it, warmup=wu, verify=True, warm=False))
            ph = r["phases"][0]
            print("%12d B (%.3f GiB) iters=%d warmup=%d: mismatching words %d, %.1f GB/s"
                  % (b, b / 2**30, it, wu, ph["mismatches"], ph["flows"][0]["gbs"]), flush=True)


if __name__ == "__main__":
    main()

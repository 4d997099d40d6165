#!/usr/bin/env python3
"""Does the device-memory footprint change streaming bandwidth?  Measures the
gfx950 copy and fill kernels on fresh 32 MiB / 1 GiB buffers after allocating
(and touching) 0, 16, 64 and 128 GiB of other device memory, with plain
hipMalloc (torch caching allocator) buffers.

    python scripts/probes/footprint_probe.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import test_nccl_p2p_amd  # noqa: E402


def timed(fn, reps=20):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / reps * 1e-3


def main():
    nat = test_nccl_p2p_amd.require_native()
    torch.cuda.set_device(0)
    stream = torch.cuda.current_stream().cuda_stream
    ballast = []
    held = 0
    for target in (0, 16, 64, 128):
        while held < target:
            t = torch.empty(4 << 30, dtype=torch.uint8, device="cuda")
            t.fill_(1)
            ballast.append(t)
            held += 4
        torch.cuda.synchronize()
        for sz in (32 << 20, 1 << 30):
            src = torch.empty(sz, dtype=torch.uint8, device="cuda")
            dst = torch.empty(sz, dtype=torch.uint8, device="cuda")
            nat.fill(src.data_ptr(), sz, 3, stream, 1)
            tc = timed(lambda: nat.copy(dst.data_ptr(), src.data_ptr(), sz, stream))
            tf = timed(lambda: nat.fill(dst.data_ptr(), sz, 3, stream, 1))
            print("ballast %4d GiB  %6d MiB: copy %.2f TB/s payload, fill %.2f TB/s"
                  % (held, sz >> 20, sz / tc / 1e12, sz / tf / 1e12), flush=True)
            del src, dst
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()

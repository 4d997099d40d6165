#!/usr/bin/env python3
"""Grid-cap sweep for the verify kernels (the reduction epilogue makes the
best grid differ from fill/copy's full grid).  Kernel time only (events)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import test_nccl_p2p_amd  # noqa: E402


def timed(fn, reps=10):
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
    st = torch.cuda.current_stream().cuda_stream
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    for gib in (1, 4):
        sz = gib << 30
        buf = torch.empty(sz, dtype=torch.uint8, device="cuda")
        p = buf.data_ptr()
        nat.fill(p, sz, 3, st)
        for name, impl in (("lds8-nt", 1), ("stride", 2)):
            out = []
            for per_cu in (4, 8, 16, 32, 64, 256, 4096):
                cap = cus * per_cu
                t = timed(lambda: nat.verify_launch(p, sz, 3, impl, True, st, cap))
                out.append("%d/CU %.2f" % (per_cu, sz / t / 1e12))
            print("%dG %-6s " % (gib, name) + "  ".join(out), flush=True)
        del buf
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()

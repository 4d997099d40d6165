#!/usr/bin/env python3
"""Bandwidth of the gfx950 buffer kernels (fill, verify-register, verify-LDS,
checksum) vs the HBM3E roofline.  Used for the A/B that decides the default
verify staging and as the workload for the rocprofv3
runs in scripts/profile.sh.

    python scripts/kernel_bench.py [--sizes 64M,1G,4G] [--reps 10] [--json out.json]
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import test_nccl_p2p_amd  # noqa: E402
from test_nccl_p2p_amd.ops import buffers  # noqa: E402

HBM_MEASURED_TBS = 6.29  # float4 copy, MI355X_MICROARCH.md


def timed(fn, reps):
    """Median seconds per launch: `reps` launches after 3 warm ones, each
    between its own event pair (as tests/test_zz_perf_floors_gpu.py times
    them; one window over a few launches reads a single stall as a slow
    kernel)."""
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for s, e in ev:
        s.record()
        fn()
        e.record()
    torch.cuda.synchronize()
    return statistics.median(s.elapsed_time(e) for s, e in ev) * 1e-3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="64M,256M,1G,4G")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    nat = test_nccl_p2p_amd.require_native()
    torch.cuda.set_device(0)
    stream = torch.cuda.current_stream().cuda_stream
    rows = []
    for sz in [nat.parse_size(s) for s in a.sizes.split(",")]:
        buf = torch.empty(sz, dtype=torch.uint8, device="cuda")
        ptr = buf.data_ptr()
        t_fill = timed(lambda: nat.fill(ptr, sz, 7, stream, 1), a.reps)
        res = {}
        for name, impl, check in [("verify_lds8", 1, True), ("verify_stride", 2, True),
                                  ("checksum_lds8", 1, False), ("checksum_stride", 2, False)]:
            # Kernel time only: reset + verify + finalize launches, no readback.
            t = timed(lambda: nat.verify_launch(ptr, sz, 7, impl, check, stream), a.reps)
            res[name] = t
            assert nat.verify(ptr, sz, 7, impl, True, stream)[0] == 0
        # The batched post-timing check (dev::launch_multi_verify): the buffer
        # as 32 MiB slots with a PRNG stream each, like a bench step's
        # receive slots; reset + verify + finalize per 32 slots, no readback.
        chunk = 32 << 20
        if sz % chunk == 0:
            jobs = [(ptr + i * chunk, chunk, 1000 + i) for i in range(sz // chunk)]
            for p_, n_, seed_ in jobs:
                nat.fill(p_, n_, seed_, stream)
            res["verify_multi32m"] = timed(lambda: nat.verify_many_launch(jobs, stream), a.reps)
            assert all(m == 0 for m, _, _ in nat.verify_many(jobs, stream))
            nat.fill(ptr, sz, 7, stream)
        row = {"bytes": sz, "fill_tbs": sz / t_fill / 1e12}
        # Roofs measured the same way: torch zero_() (write-only) and copy_()
        # (read + write, counted once like ours), and our IPC copy kernel.
        dst = torch.empty_like(buf)
        row["torch_zero_tbs"] = sz / timed(lambda: buf.zero_(), a.reps) / 1e12
        row["torch_copy_tbs"] = sz / timed(lambda: dst.copy_(buf), a.reps) / 1e12
        row["copy_kernel_tbs"] = sz / timed(lambda: nat.copy(dst.data_ptr(), ptr, sz, stream), a.reps) / 1e12
        # The cross-GPU form (system-scope sc0 sc1 buffer accesses) on local
        # memory: what the coherence bits cost when nothing is remote.
        row["copy_coherent_tbs"] = sz / timed(lambda: nat.copy(dst.data_ptr(), ptr, sz, stream, coherent=True),
                                              a.reps) / 1e12
        nat.fill(ptr, sz, 7, stream)
        nat.copy(dst.data_ptr(), ptr, sz, stream)
        assert nat.verify(dst.data_ptr(), sz, 7, 1, True, stream)[0] == 0
        dst.zero_()
        nat.copy(dst.data_ptr(), ptr, sz, stream, coherent=True)
        assert nat.verify(dst.data_ptr(), sz, 7, 1, True, stream)[0] == 0
        del dst
        for k, t in res.items():
            row[k + "_tbs"] = sz / t / 1e12
        row["fill_geom"] = nat.fill_geometry(sz)
        row["verify_lds8_geom"] = nat.verify_geometry(sz, 1)
        row["verify_stride_geom"] = nat.verify_geometry(sz, 2)
        rows.append(row)
        print("%6s  fill %.2f  verify lds8 %.2f / stride %.2f  checksum lds8 %.2f / stride %.2f TB/s"
              "  (HBM measured roof %.2f)"
              % (nat.format_size(sz), row["fill_tbs"], row["verify_lds8_tbs"], row["verify_stride_tbs"],
                 row["checksum_lds8_tbs"], row["checksum_stride_tbs"], HBM_MEASURED_TBS), flush=True)
        print("        roofs: torch zero_ %.2f  torch copy_ %.2f  ours copy %.2f TB/s (copy counts bytes once)"
              % (row["torch_zero_tbs"], row["torch_copy_tbs"], row["copy_kernel_tbs"]), flush=True)
        if "verify_multi32m_tbs" in row:
            print("        batched verify, 32 MiB slots: %.2f TB/s" % row["verify_multi32m_tbs"], flush=True)
        del buf
        torch.cuda.empty_cache()
    if a.json:
        with open(a.json, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Interleaved A/B of the verify staging: the LDS-DMA
verify (lds8; 4 KiB per wave below 2 GiB, 8 KiB from 2 GiB) against register
staging (stride) on one buffer, plus the variants that could explain a gap
between them -- the grid cap (max_grid) and the batched kernel over the same
bytes as one job or as 32 MiB slots.  (Round 6's experiments ran here as a
temporary impl 3: profiles/r6_verify_ab/.)  Every round times every variant (`reps` launches, each on its own
event pair, median), the order reversed on alternate rounds, so drift of the
clock or the HBM temperature hits all variants alike; the result per variant
is the median over rounds.

    python scripts/verify_ab.py [--sizes 1G,4G] [--rounds 12] [--reps 5] [--json out.json]
"""
import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import test_nccl_p2p_amd  # noqa: E402


def per_launch_ms(fn, reps):
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for s, e in ev:
        s.record()
        fn()
        e.record()
    torch.cuda.synchronize()
    return [s.elapsed_time(e) for s, e in ev]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="1G,4G")
    ap.add_argument("--rounds", type=int, default=12)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--grids", default="2048,4096", help="max_grid variants of both kernels")
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    nat = test_nccl_p2p_amd.require_native()
    torch.cuda.set_device(0)
    stream = torch.cuda.current_stream().cuda_stream
    out = {}
    for sz in [nat.parse_size(s) for s in a.sizes.split(",")]:
        buf = torch.empty(sz, dtype=torch.uint8, device="cuda")
        ptr = buf.data_ptr()
        chunk = 32 << 20
        # The batched kernel's buffer: its own allocation, 32 MiB slots with a
        # PRNG stream each (a bench step's receive slots).
        sbuf = torch.empty(sz, dtype=torch.uint8, device="cuda")
        slots = [(sbuf.data_ptr() + i * chunk, chunk, 1000 + i) for i in range(sz // chunk)]
        for p_, n_, s_ in slots:
            nat.fill(p_, n_, s_, stream)
        variants = {
            "lds8": lambda: nat.verify_launch(ptr, sz, 7, 1, True, stream),
            "stride": lambda: nat.verify_launch(ptr, sz, 7, 2, True, stream),
            "multi_1job": lambda: nat.verify_many_launch([(ptr, sz, 7)], stream),
            "multi_32m_slots_interleaved": lambda: nat.verify_many_launch(slots, stream),
        }
        for g in [int(x) for x in a.grids.split(",") if x]:
            variants["lds8_g%d" % g] = (lambda g=g: nat.verify_launch(ptr, sz, 7, 1, True, stream, g))
            variants["stride_g%d" % g] = (lambda g=g: nat.verify_launch(ptr, sz, 7, 2, True, stream, g))
        nat.fill(ptr, sz, 7, stream)
        assert nat.verify(ptr, sz, 7, 1, True, stream)[0] == 0
        assert nat.verify(ptr + 16, sz - 4096 - 37, 7, 1, True, stream)[0] > 0  # wrong offset: must fail
        # warm: 0.3 s of launches
        for _ in range(max(4, int(0.3 / (sz / 6e12)))):
            variants["lds8"]()
        torch.cuda.synchronize()
        names = list(variants)
        ms = {k: [] for k in names}
        for r in range(a.rounds):
            for k in (names if r % 2 == 0 else names[::-1]):
                ms[k].append(statistics.median(per_launch_ms(variants[k], a.reps)))
        # The same kernels back to back (not interleaved): each variant's
        # rounds one after the other.
        b2b = {}
        for k, fn in (("multi_32m_slots", lambda: nat.verify_many_launch(slots, stream)),
                      ("lds8_back_to_back", variants["lds8"]), ("stride_back_to_back", variants["stride"])):
            b2b[k] = [statistics.median(per_launch_ms(fn, a.reps)) for _ in range(a.rounds)]
        assert all(m == 0 for m, _, _ in nat.verify_many(slots, stream))
        row = {k: round(sz / (statistics.median(v) * 1e-3) / 1e12, 3) for k, v in list(ms.items()) + list(b2b.items())}
        # Per-round ratio lds8 / stride (same round, adjacent launches).
        ratios = [s / l for l, s in zip(ms["lds8"], ms["stride"])]
        row["lds_over_stride_median_of_rounds"] = round(statistics.median(ratios), 4)
        row["lds_over_stride_rounds"] = [round(x, 4) for x in ratios]
        row["verify_geometry_lds8"] = nat.verify_geometry(sz, 1)
        row["verify_geometry_stride"] = nat.verify_geometry(sz, 2)
        out[nat.format_size(sz)] = row
        print(nat.format_size(sz), json.dumps(row), flush=True)
        del buf, sbuf
        torch.cuda.empty_cache()
    if a.json:
        with open(a.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Step-level view of a rocprofv3 kernel trace (run_kernel_trace.csv): the
duration of the large copy / send-recv kernels of the timed steps and the
idle gaps between consecutive ones, i.e. what each step boundary costs.

    python scripts/trace_gaps.py gpurun_out/x/run_kernel_trace.csv [--match multi_copy] [--min-grid 100000]
"""
import argparse
import csv
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("traces", nargs="+")
    ap.add_argument("--match", default="multi_copy", help="substring of the kernel name")
    ap.add_argument("--min-grid", type=int, default=100000, help="smallest grid (workgroups) counted")
    ap.add_argument("--last", type=int, default=40, help="kernels from the end of the trace (the timed steps)")
    a = ap.parse_args()
    for f in a.traces:
        rows = list(csv.DictReader(open(f)))
        ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"],
                     int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"]))) for r in rows)
        big = [k for k in ks if a.match in k[2] and k[3] >= a.min_grid][-a.last:]
        if len(big) < 2:
            print(f, "fewer than 2 matching kernels")
            continue
        durs = [(k[1] - k[0]) / 1e3 for k in big]
        gaps = [(b[0] - x[1]) / 1e3 for x, b in zip(big, big[1:])]
        steps = [g for g in gaps if g > 1.0]
        print("%s: %d kernels, duration p50 %.1f us; gaps > 1 us: %d, p50 %.1f us; all gaps p50 %.1f us" % (
            f, len(big), statistics.median(durs), len(steps), statistics.median(steps) if steps else 0.0,
            statistics.median(gaps)))


if __name__ == "__main__":
    main()

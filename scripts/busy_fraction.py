#!/usr/bin/env python3
"""How busy the GPU was with the transfer kernels over a run: from a
rocprofv3 kernel trace (<name>_kernel_trace.csv), the union of the matching
kernels' intervals against the span from the first one's start to the last
one's end, plus each kernel's duration and the idle gaps between busy
stretches.  It shows where a method's time goes: the reference's method
(p2p_matrix.cc:153-176, a host sync after every message) leaves the GPU idle
between messages, ours posts them back to back.

    python scripts/busy_fraction.py gpurun_out/x/ref_kernel_trace.csv [--match rcclGenericKernel] [--last 128] [--json out.json]
"""
import argparse
import csv
import json
import statistics


def busy_stats(intervals):
    """intervals: [(start_ns, end_ns)].  Returns span, busy time (union),
    busy fraction, kernel p50 duration and the idle gaps between busy
    stretches (all in microseconds)."""
    iv = sorted(intervals)
    if not iv:
        return None
    merged = [list(iv[0])]
    for s, e in iv[1:]:
        if s <= merged[-1][1]:
            merged[-1][1] = max(merged[-1][1], e)
        else:
            merged.append([s, e])
    span = merged[-1][1] - merged[0][0]
    busy = sum(e - s for s, e in merged)
    gaps = [(b[0] - a[1]) / 1e3 for a, b in zip(merged, merged[1:])]
    return {
        "kernels": len(iv),
        "span_us": round(span / 1e3, 1),
        "busy_us": round(busy / 1e3, 1),
        "busy_fraction": round(busy / span, 4) if span else 1.0,
        "kernel_p50_us": round(statistics.median((e - s) / 1e3 for s, e in iv), 2),
        "idle_gaps": len(gaps),
        "idle_gap_p50_us": round(statistics.median(gaps), 2) if gaps else 0.0,
    }


def read_trace(path, match, last=0):
    """The matching kernels' (start, end), in start order; the last `last`
    of them (the timed iterations) when last > 0."""
    with open(path) as f:
        iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in csv.DictReader(f)
                    if match in r["Kernel_Name"])
    return iv[-last:] if last > 0 else iv


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("traces", nargs="+")
    ap.add_argument("--match", default="rcclGenericKernel", help="substring of the kernel name")
    ap.add_argument("--last", type=int, default=0,
                    help="only the last N matching kernels (the timed iterations; 0: all)")
    ap.add_argument("--json", default=None, help="also write the results here")
    a = ap.parse_args(argv)
    out = {}
    for path in a.traces:
        st = busy_stats(read_trace(path, a.match, a.last))
        out[path] = st
        if st is None:
            print("%s: no kernel matches %r" % (path, a.match))
            continue
        print("%s: %d kernels over %.1f us, busy %.1f%%; kernel p50 %.1f us; %d idle gaps, p50 %.1f us" % (
            path, st["kernels"], st["span_us"], 100 * st["busy_fraction"], st["kernel_p50_us"], st["idle_gaps"],
            st["idle_gap_p50_us"]))
    if a.json:
        with open(a.json, "w") as f:
            json.dump(out, f, indent=1)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())

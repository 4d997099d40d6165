#!/usr/bin/env python3
"""How busy the GPU kept the matching kernels of a rocprofv3 kernel trace
(`*_kernel_trace.csv`): the kernels are split into bursts at idle gaps longer
than --gap-ms, and each burst of at least --min-kernels kernels gets its span,
the time at least one kernel ran (union), the mean and peak number of kernels
running at once, and the hardware queues they ran on.  With several RCCL
communicators each on its own stream, this shows whether their kernels
overlapped or ran one after another.

    python scripts/kernel_overlap.py gpurun_out/prof/bench/bench_kernel_trace.csv [--match rcclGenericKernel]
"""
import argparse
import csv
import json


def bursts(kernels, gap_ns):
    """Splits (start, end, queue) tuples sorted by start into runs separated
    by more than gap_ns of no matching kernel running."""
    out, cur, end = [], [], None
    for k in kernels:
        if cur and k[0] - end > gap_ns:
            out.append(cur)
            cur = []
        cur.append(k)
        end = k[1] if len(cur) == 1 else max(end, k[1])
    if cur:
        out.append(cur)
    return out


def overlap_stats(ks):
    """Span, union busy time, mean and peak concurrency of one burst (ns)."""
    events = sorted([(s, 1) for s, _, _ in ks] + [(e, -1) for _, e, _ in ks])
    busy = peak = running = 0
    last = events[0][0]
    for t, d in events:
        if running > 0:
            busy += t - last
        running += d
        peak = max(peak, running)
        last = t
    span = max(e for _, e, _ in ks) - min(s for s, _, _ in ks)
    total = sum(e - s for s, e, _ in ks)
    return {"kernels": len(ks), "span_ms": round(span / 1e6, 4), "busy_ms": round(busy / 1e6, 4),
            "busy_fraction": round(busy / span, 4) if span else None,
            "mean_concurrency": round(total / busy, 3) if busy else None, "peak_concurrency": peak,
            "kernel_us_p50": round(sorted(e - s for s, e, _ in ks)[len(ks) // 2] / 1e3, 2),
            "queues": len({q for _, _, q in ks})}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--match", default="rcclGenericKernel", help="substring of the kernel name")
    ap.add_argument("--gap-ms", type=float, default=1.0, help="idle time that ends a burst")
    ap.add_argument("--min-kernels", type=int, default=64, help="smallest burst reported")
    ap.add_argument("--json", action="store_true", help="one JSON line per burst")
    a = ap.parse_args()
    with open(a.trace) as f:
        ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Queue_Id", ""))
                    for r in csv.DictReader(f) if a.match in r["Kernel_Name"])
    for i, b in enumerate(bursts(ks, int(a.gap_ms * 1e6))):
        if len(b) < a.min_kernels:
            continue
        st = dict(overlap_stats(b), burst=i)
        if a.json:
            print(json.dumps(st))
        else:
            print("burst %(burst)d: %(kernels)d kernels on %(queues)d queue(s), span %(span_ms).3f ms, busy "
                  "%(busy_ms).3f ms (%(busy_fraction).1f%%), mean %(mean_concurrency).2f / peak "
                  "%(peak_concurrency)d kernels at once, kernel p50 %(kernel_us_p50).1f us"
                  % dict(st, busy_fraction=100 * st["busy_fraction"]))


if __name__ == "__main__":
    main()

"""Reference-compatible matrix text, its parser, and scaling tables.

``compat_matrix_text`` reproduces /root/reference/p2p_matrix.cc's printf
sequence byte for byte (title :134/:189, corner "   D\\D" :135/:190, column
ids "%6d " :137/:192, row ids "%6d " :143/:198, cells "%6.02f " with 0.00 on
the diagonal :149/:179/:204/:260, newline per row :184/:265).
``parse_compat`` reads such output back (also the native binary's), which is
how the test-suite and scaling scripts consume ``mpirun ... > result.txt``
files (the reference's .gitignore lists result.txt).
"""

from __future__ import annotations

import json
import re
import statistics
from typing import Dict, Iterable, List, Optional

UNI_TITLE = "Evaluating the Uni-Directional NCCL P2P Bandwidth (Gbps)"
BI_TITLE = "Evaluating the Bi-Directional NCCL P2P Bandwidth (Gbps)"


def compat_matrix_text(m: List[List[float]], direction: str, leading_newline: Optional[bool] = None) -> str:
    n = len(m)
    lead = (direction == "bi") if leading_newline is None else leading_newline
    title = UNI_TITLE if direction == "uni" else BI_TITLE
    out = ["\n" if lead else "", title, "\n", "   D\\D"]
    out += ["%6d " % i for i in range(n)]
    out.append("\n")
    for r in range(n):
        out.append("%6d " % r)
        for c in range(n):
            out.append("%6.02f " % (0.0 if r == c else m[r][c]))
        out.append("\n")
    return "".join(out)


_CELL = re.compile(r"-?\d+\.\d\d")


def parse_compat(text: str) -> Dict[str, List[List[float]]]:
    """Returns {"uni": matrix, "bi": matrix} (Gbps) found in reference-format text.

    Cells are split by the fixed "%6.02f " layout when it holds and by
    whitespace otherwise (values >= 1000 overflow the 6-char field, exactly as
    the reference's printf does)."""
    res: Dict[str, List[List[float]]] = {}
    lines = text.splitlines()
    i = 0
    while i < len(lines):
        line = lines[i]
        key = "uni" if line.strip() == UNI_TITLE else "bi" if line.strip() == BI_TITLE else None
        if key is None:
            i += 1
            continue
        header = lines[i + 1]
        n = len(header.replace("   D\\D", "").split())
        rows = []
        for r in range(n):
            toks = lines[i + 2 + r].split()
            assert int(toks[0]) == r, "row label mismatch"
            rows.append([float(t) for t in toks[1:1 + n]])
        res[key] = rows
        i += 2 + n
    return res


def gbps_to_gbs(m: List[List[float]]) -> List[List[float]]:
    return [[v / 8.0 for v in row] for row in m]


def offdiag(m: List[List[float]]) -> List[float]:
    return [m[i][j] for i in range(len(m)) for j in range(len(m[i])) if i != j]


def fabric_findings(tournament: Optional[List[List[float]]] = None, uni: Optional[List[List[float]]] = None,
                    bi: Optional[List[List[float]]] = None, link_check: Optional[dict] = None,
                    unparsed: Optional[List[str]] = None, min_ratio: float = 0.5,
                    bi_at_least_uni: bool = True) -> List[str]:
    """What is wrong with a node's fabric by checks that need no hardware
    number; [] when all pass.  On a fully connected xGMI
    node every link is alike, so
      * no off-diagonal cell of the bench's tournament matrix (GB/s) or of
        the reference's uni matrix (p2p_matrix.cc:177, Gbps) is below
        min_ratio x the median cell: a degraded link or a mis-posted
        communicator shows up as one slow cell;
      * every bi cell (both directions summed, :258) is at least its uni cell;
      * RCCL carried every direct xGMI pair over its P2P transport
        (link_check) and parsed every connected peer's lines (unparsed).
    Missing inputs are not judged.  (A rehearsal on one GPU, over loopback
    sockets that share one CPU, asks less: a lower min_ratio and no bi >= uni,
    tests/test_multi_gpu.py.)"""
    out = []
    for name, m in (("tournament matrix_gbs", tournament), ("compat uni", uni)):
        cells = offdiag(m) if m else []
        if len(cells) < 2:
            continue
        med = statistics.median(cells)
        for i in range(len(m)):
            for j in range(len(m)):
                if i != j and m[i][j] < min_ratio * med:
                    out.append("%s: cell %d->%d %.2f < %.2f x median %.2f" % (name, i, j, m[i][j], min_ratio, med))
    if uni and bi and bi_at_least_uni:
        for i in range(min(len(uni), len(bi))):
            for j in range(min(len(uni[i]), len(bi[i]))):
                if i != j and bi[i][j] < uni[i][j]:
                    out.append("compat bi cell %d<->%d %.2f below its uni cell %.2f" % (i, j, bi[i][j], uni[i][j]))
    if link_check is not None and not link_check.get("ok", True):
        out.append("link_check: %d direct xGMI pair(s) not on RCCL's P2P transport: %s"
                   % (len(link_check.get("not_p2p") or []), ", ".join((link_check.get("not_p2p") or [])[:16])))
    if unparsed:
        out.append("RCCL connection lines not parsed for %s" % ", ".join(unparsed[:16]))
    return out


def read_json_lines(path: str) -> List[dict]:
    out = []
    with open(path) as f:
        for line in f:
            line = line.strip()
            if line.startswith("{"):
                out.append(json.loads(line))
    return out


def _get(r: dict, *path, fmt: str = "%.1f") -> str:
    v = r
    for k in path:
        if not isinstance(v, dict) or v.get(k) is None:
            return "-"
        v = v[k]
    return fmt % v if isinstance(v, (int, float)) else str(v)


def _aggregate(r: dict) -> float:
    """All flows together, GB/s: `aggregate_gbs` (round 2 on), or `value` in
    lines written while `value` was the aggregate (round 1)."""
    return r["aggregate_gbs"] if r.get("aggregate_gbs") is not None else r["value"]


def _ring_hop(r: dict) -> str:
    ex = r.get("extras") or {}
    if (ex.get("ring_hop") or {}).get("hop_us_p50") is not None:
        return "%.2f" % ex["ring_hop"]["hop_us_p50"]
    return _get(r, "extras", "ring_hop_8b", "iter_us_p50", fmt="%.2f")


def _reference_cells(r: dict) -> str:
    """The reference methodology's mean cell: uni / bi (round 3 on), or the
    single uni number of round-2 lines."""
    ref = r.get("reference_semantics") or {}
    if "uni" in ref:
        def cell(d):
            return _get(ref, d, "median") if _get(ref, d, "median") != "-" else _get(ref, d, "gbs_mean")
        return "%s / %s" % (cell("uni"), cell("bi"))
    return _get(r, "reference_semantics", "cell_gbs_mean")


def _ratios(r: dict) -> str:
    m = r.get("method_ratio") or {}
    if not m and r.get("concurrency_ratio") is None:
        return "-"
    return "%s / %s / %s" % (m.get("uni", "-") or "-", m.get("bi", "-") or "-", _get(r, "concurrency_ratio"))


SELF_COPY = "self-copy (on-GPU HBM)"
XGMI_LINK = "xgmi-link per direction"
FALLBACK = "fallback"


def value_kind(r: dict) -> str:
    """What a line's `value` measures (its `value_kind`):
    the on-GPU self copy at N = 1 (the diagonal the reference prints as 0.00,
    p2p_matrix.cc:147-151), the per-link, per-direction xGMI cell from N = 2,
    or the fallback data plane's number.  Lines from before the field are
    classed the same way from n_gpus and headline_fallback."""
    if r.get("value_kind"):
        return r["value_kind"]
    if r.get("headline_fallback"):
        return FALLBACK
    return SELF_COPY if r.get("n_gpus") == 1 else XGMI_LINK


def _kind_order(kind: str) -> int:
    return {XGMI_LINK: 0, SELF_COPY: 2, FALLBACK: 3}.get(kind, 1)


def scaling_table(results: Iterable[dict]) -> str:
    """Markdown tables of bench.py lines (one per GPU count), one table per
    value_kind: `value` (the mean cell of the matrix, GB/s per direction),
    aggregate and per-GPU GB/s, the cell rate relative to N = 2 of the SAME
    kind (weak scaling: per-GPU work is fixed, so an ideal fabric keeps every
    cell's rate), matrix min / mean, p50 latency, and the untimed comparisons
    the line carries: the reference's methodology on the same communicator,
    all-pairs aggregate, the ring token hop, the IPC engines and the device
    ping-pong.  The N = 1 self copy (HBM-bound, no link) and fallback lines
    get tables of their own and never enter a ratio with the link rows: read
    from `value` alone a 1 -> 8 curve would show a ~40x "drop" at N = 2."""
    rows = sorted((r for r in results if r.get("value") is not None), key=lambda r: r["n_gpus"])
    kinds = sorted({value_kind(r) for r in rows}, key=lambda k: (_kind_order(k), k))
    out = []
    for kind in kinds:
        krows = [r for r in rows if value_kind(r) == kind]
        base = next((r for r in krows if r["n_gpus"] == 2), None) if kind != SELF_COPY else None
        if out:
            out.append("")
        out.append("value_kind: %s%s" % (kind, " (no link: not comparable with the link rows)" if kind == SELF_COPY
                                          else " (not RCCL: the metric's value is null)" if kind == FALLBACK else ""))
        out += _kind_table(krows, base)
    for r in rows:
        out += transport_lines(r) + pair_sweep_lines(r)
    return "\n".join(out)


def _kind_table(rows, base) -> List[str]:
    out = ["| GPUs | value: mean cell GB/s | aggregate GB/s | per-GPU GB/s | cell rate vs 2 GPUs | RCCL comms "
           "| matrix min / mean GB/s | p50 latency us | reference-method cell GB/s (uni / bi) "
           "| method ratio (uni / bi) / concurrency ratio | all-pairs 1 GiB aggregate GB/s "
           "| ring hop 8 B us | IPC pull / push / SDMA / relay GB/s | relay pair 0->1 GB/s | device ping-pong us "
           "| headline fallback |",
           "|---|---|---|---|---|---|---|---|---|---|---|---|---|---|---|---|"]
    for r in rows:
        eff = ""
        if base and r["n_gpus"] >= 2 and base["value"]:
            eff = "%.1f%%" % (100.0 * r["value"] / base["value"])
        relay = (r.get("ipc_transport") or {}).get("relay") or {}
        relay_pair = (relay.get("pair_0_1") or [{}])[0]
        agg = _aggregate(r)
        fb = r.get("headline_fallback")
        out.append("| %d | %.1f | %.1f | %.1f | %s | %s | %s / %s | %s | %s | %s | %s | %s | %s / %s / %s / %s | %s | %s "
                   "| %s |" % (
            r["n_gpus"], r["value"], agg, agg / r["n_gpus"], eff, _get(r, "posting", "rccl_comms", fmt="%d"),
            _get(r, "matrix_gbs_min", fmt="%.2f"), _get(r, "matrix_gbs_mean", fmt="%.2f"),
            _get(r, "p50_latency_us", fmt="%.2f"), _reference_cells(r), _ratios(r),
            _get(r, "extras", "allpairs_1g", "aggregate_gbs"), _ring_hop(r),
            _get(r, "ipc_transport", "value_gbs"),
            _get(r, "ipc_transport", "push", "value_gbs"), _get(r, "ipc_transport", "sdma", "value_gbs"),
            _get(r, "ipc_transport", "relay", "value_gbs"), relay_pair.get("gbs", "-"),
            _get(r, "ipc_transport", "device_pingpong_p50_us", fmt="%.2f"),
            "%s -> %s" % (fb["from"], fb["to"]) if fb else "-"))
    return out


def transport_lines(r: dict) -> List[str]:
    """How RCCL carried the pairs of a line (matrix_transport: the transport
    class per pair from RCCL's INFO log) and the op limits it set up
    (provenance.rccl_peers): e.g. "P2P 56/56", a fallback to SHM or NET shows
    up here before it shows up as a slow link."""
    m = r.get("matrix_transport")
    if not isinstance(m, list) or r.get("n_gpus", 0) < 2:
        return []
    n = len(m)
    counts = {}
    for a in range(n):
        for b in range(n):
            if a != b:
                k = m[a][b] or "unknown"
                counts[k] = counts.get(k, 0) + 1
    line = "RCCL transports, %d GPUs: %s" % (r["n_gpus"], ", ".join(
        "%s %d/%d" % (k, v, n * (n - 1)) for k, v in sorted(counts.items())))
    peers = [p for rk in ((r.get("provenance") or {}).get("rccl_peers") or []) if rk
             for p in rk.get("peers", []) if p.get("transport") != "self"]
    if peers:
        ch = sorted({p.get("op_channels") for p in peers})
        lim = sorted({p.get("op_limit") for p in peers})
        line += "; p2p channels per op %s, op limit %s MiB" % ("/".join(map(str, ch)),
                                                              "/".join(str((x or 0) >> 20) for x in lim))
    out = ["", line]
    lc = r.get("link_check")
    if isinstance(lc, dict) and not lc.get("ok", True):
        out.append("WRONG TRANSPORT on %d of %d direct xGMI pairs: %s" % (
            len(lc["not_p2p"]), lc["direct_xgmi_pairs"], ", ".join(lc["not_p2p"][:16])))
    return out


def pair_sweep_lines(r: dict) -> List[str]:
    """The winner per cell of a line's xGMI pair sweep (bench.py
    --xgmi-sweep, on at N = 2): row, GB/s (bi: both directions) and the gain
    over RCCL with one communicator and no knobs; corrupt and skipped rows."""
    sw = r.get("xgmi_pair_sweep")
    if not isinstance(sw, dict):
        return []
    head = "xGMI pair sweep, %d GPUs%s:" % (r["n_gpus"], " (emulated: %s)" % sw["emulated"] if sw.get("emulated") else "")
    if not sw.get("best"):
        return ["", head + " %s" % (sw.get("error") or "no verified row")[:200]]
    out = ["", head]
    for cell, b in sorted(sw["best"].items()):
        gain = " (%.2fx RCCL, 1 communicator)" % b["gain"] if b.get("gain") else ""
        out.append("- %s: %s %.2f GB/s%s" % (cell, b["row"], b["cell_gbs"], gain))
    for cell, b in sorted((sw.get("best_rccl") or {}).items()):
        if b["row"] != (sw["best"].get(cell) or {}).get("row"):
            gain = " (%.2fx)" % b["gain"] if b.get("gain") else ""
            out.append("- %s, best RCCL: %s %.2f GB/s%s" % (cell, b["row"], b["cell_gbs"], gain))
    for key in ("corrupt", "skipped"):
        if sw.get(key):
            out.append("- %s rows: %s" % (key, ", ".join(sw[key])))
    return out


def repeat_line(r: dict) -> str:
    """One p2p_matrix --repeat summary record: the median of the runs' mean
    cells, their range and the spread ((max - min) / median)."""
    spread = (r["max"] - r["min"]) / r["median"] if r["median"] else 0.0
    return "%-10s %-3s %10d B, %d runs: GB/s median %.2f (min %.2f, max %.2f, spread %.1f%%)" % (
        r["mode"], r["dir"], r["bytes"], len(r["runs"]), r["median"], r["min"], r["max"], 100.0 * spread)


def bench_compat_text(r: dict, key: str = "reference_semantics") -> str:
    """The reference's two printed matrices for a bench.py line, from its
    config-3 matrices (`reference_semantics`: the reference's own method, or
    `pair_serial_events`: ours on its schedule): GB/s x 8 = Gbps, bi = both
    directions summed, in the exact format p2p_matrix.cc prints -- what
    `mpirun -n N ./p2p_matrix > result.txt` would have shown on that node."""
    sec = r.get(key) or {}
    out = []
    for d in ("uni", "bi"):
        m = (sec.get(d) or {}).get("matrix_gbs")
        if m:
            out.append(compat_matrix_text([[v * 8.0 for v in row] for row in m], d))
    return "".join(out)


def summarize_compat(text: str) -> str:
    """GB/s min/mean/max (off-diagonal) of each reference-format matrix."""
    from .stats import offdiag_summary

    lines = []
    for key, m in parse_compat(text).items():
        s = offdiag_summary(gbps_to_gbs(m))
        lines.append("%s: %d ranks, GB/s min %.2f mean %.2f max %.2f over %d cells"
                     % (key, len(m), s["min"], s["mean"], s["max"], s["cells"]))
    return "\n".join(lines)


def _lines_in_text(text: str) -> list:
    out = []
    for line in text.splitlines():
        if line.startswith('{"metric"'):
            try:
                out.append(json.loads(line))
            except ValueError:
                pass
    return out


def bench_lines_in(obj) -> list:
    """Every bench line (a dict with `metric` and `n_gpus`) nested anywhere in
    a JSON document, in document order; a line's own fields are not searched.
    A record that keeps the run's stdout as text (the driver's `tail`) gives
    the whole line from it, in preference to an abridged parsed copy."""
    if isinstance(obj, dict):
        if "metric" in obj and "n_gpus" in obj:
            return [obj]
        whole = [x for v in obj.values() if isinstance(v, str) for x in _lines_in_text(v)]
        if whole:
            return whole
        return [x for v in obj.values() for x in bench_lines_in(v)]
    if isinstance(obj, list):
        return [x for v in obj for x in bench_lines_in(v)]
    return []


def main(argv=None) -> int:
    """python -m test_nccl_p2p_amd.utils.report FILE...

    Reference-format text (e.g. `mpirun ... > result.txt`) -> GB/s summary;
    bench.py JSON lines -> scaling table; p2p_matrix --json lines -> per-run
    min/mean GB/s."""
    import argparse

    ap = argparse.ArgumentParser(description=main.__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("files", nargs="+")
    a = ap.parse_args(argv)
    all_bench = []
    for path in a.files:
        text = open(path).read()
        print("== %s" % path)
        recs = []
        for line in text.splitlines():
            line = line.strip()
            if line.startswith("{"):
                try:
                    recs.append(json.loads(line))
                except ValueError:
                    pass
        if not recs:
            # A pretty-printed record that holds bench lines, such as the
            # driver's BENCH_rNN.json ("parsed") or SCALE_rNN.json.
            try:
                recs = bench_lines_in(json.loads(text))
            except ValueError:
                pass
        bench = [r for r in recs if "metric" in r and "n_gpus" in r]
        runs = [r for r in recs if r.get("type") == "run"]
        if bench:
            print(scaling_table(bench))
            all_bench.extend(bench)
            for r in bench:
                for key in ("reference_semantics", "pair_serial_events"):
                    txt = bench_compat_text(r, key)
                    if txt and r.get("n_gpus", 1) > 1:
                        print("-- %s, %d GPUs, in the reference's format:" % (key, r["n_gpus"]))
                        print(txt, end="")
        for r in runs:
            print("%-10s %-3s %10d B x %4d: GB/s min %.2f mean %.2f max %.2f%s"
                  % (r["mode"], r["dir"], r["bytes"], r["iters"], r["gbs_min"], r["gbs_mean"], r["gbs_max"],
                     "  (run %d)" % r["repeat"] if r.get("repeat") else ""))
        for r in recs:
            if r.get("type") == "repeats":  # p2p_matrix --repeat R
                print(repeat_line(r))
        if UNI_TITLE in text or BI_TITLE in text:
            print(summarize_compat(text))
    if len({r["n_gpus"] for r in all_bench}) > 1:  # one line per GPU count across files: the scaling curve
        print("== scaling")
        print(scaling_table(all_bench))
    return 0


if __name__ == "__main__":
    import sys

    sys.exit(main())

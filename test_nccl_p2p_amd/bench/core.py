"""Shared pieces of bench.py: logging, the deadline and its watchdog, the
result reporter, and the pure functions behind the headline numbers (unit
tested in tests/test_bench_unit.py through bench.py's re-exports)."""

from __future__ import annotations

import json
import math
import os
import socket
import statistics
import sys
import threading
import time

import torch

from test_nccl_p2p_amd.bench.faults import candidate_hang, hang_requested  # noqa: F401 (re-exported)
from test_nccl_p2p_amd.utils.proc import kill_children

METRIC = "pairwise P2P GB/s matrix (min/mean) + p50 latency at 1/2/4/8 MI355X"
BASELINE_VALUE = None  # the reference publishes no numbers
RESERVE_S = 15.0  # kept free at the end of the deadline for the JSON line and teardown
T0 = [time.monotonic()]  # the deadline counts from here; bench.py sets it at process start


def set_start(t0: float):
    T0[0] = t0


def log(*a):
    print("[%7.1fs]" % (time.monotonic() - T0[0]), *a, file=sys.stderr, flush=True)


def claim_stdout() -> int:
    """Points fd 1 at stderr for the whole run and returns a private duplicate
    of the real stdout.  RCCL (version banner) and gloo ("Rank i is connected
    to ...") print on stdout from every rank; the driver contract wants exactly
    one JSON line there, written by rank 0 through the returned fd."""
    sys.stdout.flush()
    real = os.dup(1)
    os.dup2(2, 1)
    return real


def free_port() -> int:
    """A free port below Linux's ephemeral range (32768-60999), so that no
    outgoing connection takes it before the child process binds it."""
    import random

    rng = random.Random()
    for _ in range(256):
        port = rng.randrange(20000, 32000)
        s = socket.socket()
        try:
            s.bind(("127.0.0.1", port))
            return port
        except OSError:
            continue
        finally:
            s.close()
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def first_comms(transport: str, comms: int) -> int:
    """Communicators of the session bench.py opens first (the headline one)."""
    return comms if transport == "rccl" and comms > 0 else 1


def posting_candidates(transport: str, comms: int, batch: int, n: int = 1, hw_queues: int = 4):
    """(communicators, batch) pairs the tuning laps time against each other.

    comms: > 0 fixed, -1 = RCCL picks: on one GPU between 1 and 4, and 8 when
    the process has >= 8 hardware queues (measured: 2, 3 and 6 are slower
    there, and 8 communicators beat 4 only with 8 queues, profiles/r2_step_shape/,
    profiles/r3_hwq/); between 1, 2, 4 and 8 across GPUs, where no measurement
    has fixed the count for an xGMI link yet (other transports: 1).  batch: 1
    one group per step, 0 one group per message, -1 = both (K = 1 only: with
    several communicators per-message groups cannot overlap)."""
    auto = ([1, 4] + ([8] if hw_queues >= 8 else [])) if n == 1 else [1, 2, 4, 8]
    comms_choices = ([comms] if comms > 0 else auto) if transport == "rccl" else [1]
    batch_choices = [batch] if batch >= 0 else [0, 1]
    return [(c, b) for c in comms_choices for b in batch_choices if c == 1 or b == 1 or len(batch_choices) == 1]


def tuning_steps(phases: int, min_steps: int = 8, lap_enough: int = 4) -> int:
    """Steps per tuning pass: whole laps of the schedule (every cell once per
    lap).  A schedule of fewer than lap_enough rounds (one GPU, N = 2, 3) runs
    laps up to min_steps steps, so a one-round schedule is not timed on a few
    ~1.5 ms steps; one lap of a longer schedule (N = 8: 7 rounds of 4 GiB per
    flow over xGMI) is long enough as it is."""
    if phases >= lap_enough:
        return phases
    return phases * max(1, math.ceil(min_steps / phases))


def headline_stats(job_bytes: float, flows_total: int, steps: int, elapsed: float):
    """(value, aggregate): the mean per-flow, per-direction rate and the sum
    over all flows, both from the barrier-bracketed wall clock, in GB/s."""
    aggregate = job_bytes / elapsed / 1e9
    mean_flows = flows_total / steps
    return aggregate / mean_flows, aggregate


def cell_matrix(n: int, steps, flows_of, all_ms, bytes_per_flow: float):
    """Per-cell GB/s medians and sample counts.  A flow's time in a step is
    the LONGER of its two endpoints' step durations (the conservative choice,
    the same as p2p_matrix's per-flow time, csrc/runner.cpp run_phase): the
    endpoint that started first also waited for its partner."""
    cells = {}
    for i, k in enumerate(steps):
        for (src, dst) in flows_of(k):
            ms = max(all_ms[src][i], all_ms[dst][i])
            if ms > 0:
                cells.setdefault((src, dst), []).append(bytes_per_flow / (ms * 1e-3) / 1e9)
    matrix = [[0.0] * n for _ in range(n)]
    samples = [[0] * n for _ in range(n)]
    for (s, d), v in cells.items():
        matrix[s][d] = statistics.median(v)
        samples[s][d] = len(v)
    return matrix, samples, cells


def pick_depth(steps: int, phases: int) -> int:
    """Receive generations so that no timed step overwrites another's slots."""
    return max(1, math.ceil(steps / phases))


class Deadline:
    """One deadline for the whole run, counted from process start."""

    def __init__(self, seconds: float):
        self.end = T0[0] + seconds

    def left(self) -> float:
        return self.end - time.monotonic()


# Posting candidates' waits.  Every wait of a session is
# bounded by its timeout (the transports' bounded polls abort and fail), so a
# candidate that hangs costs what its session's timeout says, not --timeout:
#   * the first candidate (the headline session's; it must work, or the
#     headline fails over to the fallback data plane) gets FIRST_SHARE of the
#     time the deadline leaves, at least CANDIDATE_MIN_S, at most --timeout;
#   * every later (droppable) candidate gets CANDIDATE_COST_FACTOR x what the
#     first one took to connect and run one tuning pass, at least
#     CANDIDATE_MIN_S, and never more than CANDIDATE_SHARE of the time left;
#   * all tuning together stays within TUNING_SHARE of the time left when it
#     starts: a droppable candidate whose budget would not fit is skipped.
CANDIDATE_MIN_S = 10.0
CANDIDATE_COST_FACTOR = 10.0
CANDIDATE_SHARE = 0.15
FIRST_SHARE = 0.25
TUNING_SHARE = 0.4


def first_candidate_budget(timeout: float, left: float) -> float:
    """Seconds any one wait of the first posting candidate may take, `left`
    being what the deadline leaves (less RESERVE_S)."""
    return min(timeout, max(CANDIDATE_MIN_S, FIRST_SHARE * left))


def candidate_budget(first_cost: float, left: float, timeout: float) -> float:
    """Seconds any one wait of a droppable candidate may take: scaled from
    the first candidate's measured connect + one pass (slowest rank), capped
    by a share of the time left and by --timeout."""
    return min(timeout, CANDIDATE_SHARE * max(0.0, left),
               max(CANDIDATE_MIN_S, CANDIDATE_COST_FACTOR * first_cost))


def process_age() -> float:
    """Seconds since this process started, by the kernel's record of its start
    (/proc/self/stat starttime against /proc/uptime, 10 ms ticks); 0 if
    unknown."""
    try:
        with open("/proc/self/stat") as f:
            start_ticks = int(f.read().rsplit(")", 1)[1].split()[19])
        with open("/proc/uptime") as f:
            up = float(f.read().split()[0])
        return max(0.0, up - start_ticks / os.sysconf("SC_CLK_TCK"))
    except (OSError, ValueError, IndexError):
        return 0.0


class Timeline:
    """Where the run's wall time went, for the JSON line (timeline_s; VERDICT
    r4 item 2): contiguous phases from process start, each begin() closing the
    open one, so the entries add up to the time from process start to the
    snapshot.  The first entry is the interpreter's start up to bench.py's
    first line (T0); the open entry at a watchdog emit names the phase the
    deadline caught."""

    def __init__(self, t0: float):
        self.start = time.monotonic() - process_age()
        self.start = min(self.start, t0)
        self.lock = threading.Lock()
        self.entries = [["startup", t0 - self.start]]
        self.name, self.t = "imports", t0

    def begin(self, name: str):
        with self.lock:
            now = time.monotonic()
            self.entries.append([self.name, now - self.t])
            self.name, self.t = name, now

    def snapshot(self, deadline=None) -> dict:
        with self.lock:
            now = time.monotonic()
            entries = [[n, round(s, 4)] for n, s in self.entries] + [[self.name, round(now - self.t, 4)]]
            return {"entries": entries, "open": self.name, "total_s": round(now - self.start, 4),
                    "deadline_left_s": round(deadline.left(), 3) if deadline is not None else None}


class Reporter:
    """Holds the result and prints it exactly once (rank 0): at the normal end
    of the run, or from the watchdog when the deadline passes first."""

    def __init__(self, rank: int, real_stdout: int, json_out, timeline=None, deadline=None):
        self.rank = rank
        self.fd = real_stdout
        self.json_out = json_out
        self.timeline = timeline  # its snapshot goes into every line (timeline_s)
        self.deadline = deadline
        self.lock = threading.Lock()
        self.result = None  # set once the timed region is measured
        self.done = False

    def update(self, **kv):
        with self.lock:
            if self.result is not None:
                self.result.update(kv)

    def emit(self, **extra) -> bool:
        with self.lock:
            if self.done:
                return False
            self.done = True
            if self.rank != 0:
                return True
            res = dict(self.result) if self.result is not None else {
                "metric": METRIC, "value": None, "unit": "GB/s", "error": "the timed steps did not finish"}
            res.update(extra)
            if self.timeline is not None:
                res["timeline_s"] = self.timeline.snapshot(self.deadline)
            line = json.dumps(res)
            os.write(self.fd, (line + "\n").encode())
            if self.json_out:
                with open(self.json_out, "w") as f:
                    f.write(line + "\n")
            return True


ABORT_GRACE_S = 3.0
ABORT_LINGER_S = 1.0
# Set once the watchdog has fired: from then on it owns the process's exit
# status (bench.py main waits for it instead of returning or raising).
WATCHDOG_FIRED = threading.Event()


def start_watchdog(deadline: Deadline, reporter: Reporter, nat, state) -> threading.Event:
    """At the deadline: print the JSON line with what is finished (the section
    still running is named), have the communicators aborted so their kernels
    exit, and end the process.  Exit 0 when the headline was measured.

    The abort is requested, not performed, here: the main thread may be inside
    RCCL, and aborting a communicator from this thread meanwhile crashed it
    (SIGSEGV on 3 of 8 ranks, profiles/r4_rehearsal/).  Every bounded wait of
    the transports polls the request and aborts on its own thread; should the
    main thread be outside the engine (no native call open: a gloo barrier, a
    torch sync), the communicators are aborted from here (nat.abort_if_idle).
    That runs on a helper thread with the GIL released: an abort
    that never returns (a kernel that never exits, a stuck proxy thread) holds
    the helper, not this thread, which ends the process ABORT_GRACE_S after
    the deadline whatever the abort is doing (process exit tears the GPU
    queues down); the line says which happened."""
    stop = threading.Event()

    def run():
        while not stop.wait(max(0.05, min(1.0, deadline.left()))):
            if deadline.left() <= 0:
                break
        if stop.is_set():
            return
        WATCHDOG_FIRED.set()
        try:
            log("bench: deadline reached during %s; printing what is done" % state.get("section"))
            errors = dict(state.get("errors") or {})
            if state.get("section"):
                errors[state["section"]] = "deadline reached while running"
            reporter.emit(deadline_hit=True, untimed_skipped=state.get("skipped") or None,
                          section_errors=errors or None)
            kill_children(state)
            outcome = {"how": None, "aborting": False}
            done = threading.Event()

            def aborter():
                try:
                    nat.request_abort()
                    t_end = time.monotonic() + ABORT_GRACE_S
                    while time.monotonic() < t_end:
                        if nat.abort_done():
                            outcome["how"] = "aborted by the main thread's wait"
                            break
                        # The main thread outside the engine (a gloo barrier, a
                        # torch sync, Python): no RCCL call can be running, abort
                        # from here.
                        outcome["aborting"] = True
                        idle = nat.abort_if_idle()
                        outcome["aborting"] = False
                        if idle:
                            outcome["how"] = "aborted by the watchdog (engine idle)"
                            break
                        time.sleep(0.02)
                except Exception as e:  # noqa: BLE001 -- the process ends either way
                    outcome["how"] = "abort failed: %s" % e
                finally:
                    done.set()

            threading.Thread(target=aborter, name="bench-aborter", daemon=True).start()
            done.wait(ABORT_GRACE_S)
            how = outcome["how"] or ("abort from the watchdog (engine idle) still running after %.1f s"
                                     if outcome["aborting"] else "not aborted within %.1f s") % ABORT_GRACE_S
            log("bench: communicators %s" % how)
            # Every rank's watchdog fires at about the same time; a launcher
            # (torchrun) SIGTERMs the other ranks as soon as one exits, which
            # would cut a peer's own abort short.  Linger until a common point
            # (ABORT_LINGER_S past the deadline, at least that long after the
            # abort), so the ranks end together.
            time.sleep(max(ABORT_LINGER_S, deadline.end + ABORT_GRACE_S - time.monotonic()))
        finally:
            # Whatever happened above, the process ends here (bench.py's main
            # thread waits for it once WATCHDOG_FIRED is set).
            try:
                sys.stderr.flush()
            finally:
                os._exit(0 if reporter.result is not None else 4)

    threading.Thread(target=run, name="bench-watchdog", daemon=True).start()
    return stop


# Untimed sections in the order bench.py runs them, with the seconds each one
# keeps reserved: the BASELINE configs come first -- 3 the
# N x N matrices by the reference's method and by ours, 4 all-pairs, 5 ring
# and the ring hop, 2 the single-pair sweep -- and while one runs, the slices
# of those after it stay free, so a slow section cannot crowd a later config
# out.  The IPC comparisons and the xGMI pair sweep come after them and get
# whatever is left.  (self_sweep, config 2's sizes on the self cell, runs at
# N = 1 only, pair_sweep_0_1 at N > 1 only.)
SECTION_SLICES = (("latency", 5.0), ("latency_preposted", 5.0), ("reference_semantics", 12.0),
                  ("reference_semantics_stock", 12.0),
                  ("pair_serial_events", 12.0), ("allpairs_1g", 8.0), ("ring_256m", 5.0), ("ring_hop", 3.0),
                  ("self_sweep", 4.0), ("pair_sweep_0_1", 10.0))


# Share of the slack beyond a section's own slice that its optional work (the
# reference-method matrices' repeats, sections.py section()) may use.  At N = 8
# at xGMI-like speed (tests/test_torchrun_cpu.py's rehearsal: one run of a
# direction mode ~6-8 s) 0.2 gives each mode of the reference matrices ~4 runs
# and ours ~2, and leaves the IPC comparisons across the links their time;
# 0.3 gave 5-6 and 3-4 but left the comparisons ~40 s less.
REPEAT_SLACK_SHARE = 0.2


def reserved_after(name: str, active) -> float:
    """Seconds the sections after `name` (those of SECTION_SLICES in
    `active`) keep reserved while `name` runs; 0 for sections not planned."""
    names = [s for s, _ in SECTION_SLICES]
    if name not in names:
        return 0.0
    return sum(sec for (s, sec) in SECTION_SLICES[names.index(name) + 1:] if s in active)


def pair_matrix_summary(run: dict, n: int) -> dict:
    """A pair-mode run (report.cpp run JSON) valued like the reference's
    printed cells: each phase (one ordered pair, or the self cell) moves the
    bytes of all its flows per iteration (compat_gbps: a bi cell is both
    directions summed, p2p_matrix.cc:258), here in GB/s (= Gbps / 8).  Row =
    sender."""
    m = [[0.0] * n for _ in range(n)]
    cells = []
    for ph in run["phases"]:
        v = ph["compat_gbps"] / 8.0
        r, c = (ph["row"], ph["col"]) if ph["row"] >= 0 else (0, 0)
        m[r][c] = round(v, 3)
        cells.append(v)
    return {"gbs_min": round(min(cells), 3) if cells else None,
            "gbs_mean": round(statistics.mean(cells), 3) if cells else None, "cells": len(cells),
            "mismatches": sum(ph["mismatches"] for ph in run["phases"]), "matrix_gbs": m}


def combine_runs(runs, n: int) -> dict:
    """R repeats of one reference-method matrix (pair_matrix_summary each,
    VERDICT r5 item 1): the matrix is the per-cell median over the runs
    (gbs_min / gbs_mean over its cells), `runs` each run's mean cell, and
    median / min / max / spread of those; the ratios are taken from `median`.
    One reference run (p2p_matrix.cc:153-177) is a single wall-clock shot per
    cell; its spread across records was +-9% (686.7-819.0 GB/s on the self
    cell in round 5)."""
    per_run = [r["gbs_mean"] for r in runs if r.get("gbs_mean") is not None]
    m = [[round(statistics.median([r["matrix_gbs"][a][b] for r in runs]), 3) for b in range(n)] for a in range(n)]
    cells = [m[a][b] for a in range(n) for b in range(n) if (a != b or n == 1)]
    med = statistics.median(per_run) if per_run else None
    return {"gbs_min": round(min(cells), 3) if cells else None,
            "gbs_mean": round(statistics.mean(cells), 3) if cells else None,
            "cells": runs[0]["cells"] if runs else 0,
            "mismatches": sum(r["mismatches"] for r in runs),
            "matrix_gbs": m,
            "runs": [round(x, 3) for x in per_run],
            "median": round(med, 3) if med is not None else None,
            "min": round(min(per_run), 3) if per_run else None,
            "max": round(max(per_run), 3) if per_run else None,
            "spread": round((max(per_run) - min(per_run)) / med, 4) if per_run and med else None}


def child_runs(ref: dict, iters: dict, slice_left: float, start_s: float) -> dict:
    """Runs per direction mode for the stock-settings child: as many as the
    in-process matrices had (ref[d]["runs"]), or as many as the slice left
    holds after the child's start at their measured time per run
    (ref[d]["run_s"], with 20% margin) -- at least one."""
    per_dir = max(0.0, slice_left - start_s) / max(1, len(iters))
    out = {}
    for d in iters:
        have = len(ref[d].get("runs") or [1])
        fit = int(per_dir / (1.2 * max(ref[d].get("run_s") or 0.0, 1e-3)))
        out[d] = max(1, min(have, fit))
    return out


def method_ratios(ours: dict, ref: dict, value: float, n: int) -> dict:
    """method_ratio[dir]: our methodology over the reference's on the same
    serial pair schedule (the median over repeats of each run's mean cell,
    combine_runs; a record without repeats: its mean cell; warmup + hipEvents
    + pipelined iterations vs host clock + a sync per message), per direction
    mode.  concurrency_ratio: the headline's tournament cell (per link and
    direction, every disjoint pair at once) over our serial bi cell per
    direction (both directions summed / 2) -- the schedule's gain alone; None
    at n == 1, where there are no pairs."""
    def mean(d, k):
        x = (d or {}).get(k) or {}
        return x.get("median") if x.get("median") is not None else x.get("gbs_mean")

    out = {"method_ratio": {}, "concurrency_ratio": None}
    for k in ("uni", "bi"):
        a, b = mean(ours, k), mean(ref, k)
        out["method_ratio"][k] = round(a / b, 3) if a and b else None
    bi = mean(ours, "bi")
    if n > 1 and bi and value:
        out["concurrency_ratio"] = round(value / (bi / 2.0), 3)
    return out


def link_check(rank_links, matrix_transport):
    """Pairs whose GPUs share a direct xGMI link (provenance.rank_links
    "XGMI/1", hipExtGetLinkTypeAndHopCount) but which RCCL carried over
    anything but its P2P transport (matrix_transport, from its INFO log): the
    same rule as p2p_matrix --min-gbs (rccl_log.cpp link_transport_mismatch).
    A node where RCCL fell back to SHM or NET would otherwise only look like
    slow links.  None when either matrix is missing (one GPU, no RCCL log)."""
    if not rank_links or not matrix_transport:
        return None
    n = min(len(rank_links), len(matrix_transport))
    direct, wrong = 0, []
    for a in range(n):
        for b in range(n):
            if a == b or rank_links[a][b] != "XGMI/1":
                continue
            direct += 1
            t = matrix_transport[a][b]
            if t and t not in ("?", "P2P", "self"):
                wrong.append("%d->%d %s" % (a, b, t))
    return {"direct_xgmi_pairs": direct, "not_p2p": wrong, "ok": not wrong}


def unparsed_peers(reports):
    """"rank->peer" for every remote peer on the same host whose RCCL
    connection lines were not parsed although the rank exchanged messages
    with it (link_report unparsed_peers, csrc/rccl_log.hpp
    rccl_unparsed_peers): RCCL's log format changed and those peers' ops stay
    at the 2-channel default.  None without RCCL link reports."""
    if not isinstance(reports, list) or not any(reports):
        return None
    return ["%d->%d" % (r["rank"], u["peer"]) for r in reports if r for u in r.get("unparsed_peers") or []]


def bench_fabric_findings(result: dict, n: int):
    """The multi-GPU tier's fabric checks (utils/report.py fabric_findings)
    on what one bench line holds: the tournament matrix, the serial-pair uni
    and bi matrices of pair_serial_events (our method: warmup, events; else
    the reference's method), link_check and unparsed_peers.  [] when all
    pass; None at N = 1.  Informational: the line never fails on it."""
    from test_nccl_p2p_amd.utils.report import fabric_findings

    if n < 2:
        return None
    ser = next((result.get(k) for k in ("pair_serial_events", "reference_semantics")
                if isinstance(result.get(k), dict) and "error" not in result[k]), None) or {}
    uni = (ser.get("uni") or {}).get("matrix_gbs")
    bi = (ser.get("bi") or {}).get("matrix_gbs")
    return fabric_findings(result.get("matrix_gbs"), uni, bi, result.get("link_check"), result.get("unparsed_peers"))


def default_device(local_rank: int) -> int:
    """LOCAL_RANK, modulo the visible GPUs: a launcher that gives each rank
    one visible GPU (HIP_VISIBLE_DEVICES per process) leaves every rank on
    its device 0.  torch.cuda.device_count() does not initialise the GPU."""
    count = torch.cuda.device_count()
    return local_rank % count if count > 0 else local_rank

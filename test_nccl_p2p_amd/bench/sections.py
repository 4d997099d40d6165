"""The untimed sections of bench.py, after the timed steps and under one
deadline: latency, the reference's methodology, the other BASELINE configs
(all-pairs, ring, ring hop, single-pair sweep), the IPC comparisons and the
xGMI pair sweep."""

from __future__ import annotations

import gc
import json
import os
import shutil
import statistics
import subprocess
import sys
import tempfile
import time

import torch.distributed as dist

from test_nccl_p2p_amd.bench.compare import REF_STOCK, steps_through, stock_env
from test_nccl_p2p_amd.bench.core import (REPEAT_SLACK_SHARE, RESERVE_S, SECTION_SLICES, child_runs, combine_runs,
                                          free_port, log, method_ratios, pair_matrix_summary, reserved_after)
from test_nccl_p2p_amd.utils.proc import run_child

HERE = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))  # the repository root
CHILD_START_S = 6.0  # a bench.py child's start to its first RCCL run (~4.6 s on the box, profiles/r5_final/)


class SectionsMixin:
    """BenchRun's untimed sections (collective)."""

    # ---- untimed sections: one deadline, waits shortened to the time left --
    def budget_left(self) -> float:
        return min(self.args.untimed_budget - (time.monotonic() - self.untimed_t0), self.deadline.left() - RESERVE_S)

    def section(self, name, fn, min_s=2.0, budgeted=True, sessions=True):
        """Runs one untimed section if every rank has time for it; an error is
        logged and returned in its place ({"error": ...}).  budgeted=False:
        only the deadline counts, not --untimed-budget (the headline's own
        latency).  The slices of the BASELINE sections after this one
        (SECTION_SLICES) stay reserved: self.slice_left is what this one may
        plan with.  Every wait of the live sessions is bounded by all the time
        left (not the slice: a wait that expires aborts the session); the
        watchdog prints the line at the deadline whatever runs.  A section
        that failed may leave the live sessions in disagreement across ranks,
        so later sections that use them (sessions=True) are skipped."""
        left = self.budget_left() if budgeted else self.deadline.left() - RESERVE_S
        wait_left = left
        # When the time left cannot hold every remaining slice, each keeps its
        # proportional share (the first ones are not starved).
        later = reserved_after(name, self.active_sections)
        mine = dict(SECTION_SLICES).get(name, 0.0)
        if 0 < left < later + mine:
            later *= left / (later + mine)
        left -= later
        # One collective per section: a failure may be local to some ranks
        # (a hung rank leaves the others here until the watchdog fires).
        broken = sessions and self.broken
        # (Its own timeline entry: a rank whose peer stopped responding waits
        # here, and the watchdog's line then shows that wait as the open one.)
        self.timeline.begin("agree:" + name)
        if not self.agree(left > min_s and not broken):
            self.timeline.begin("untimed")
            self.state["skipped"].append(name)
            self.log0("bench: skipping %s: %s" % (name, "the sessions failed in %s" % self.broken if broken
                                                  else "no time left (or another rank's sessions failed)"))
            return None
        self.slice_left = left
        # Its own share, for work that is optional (the reference matrices'
        # repeats): its SECTION_SLICES slice plus REPEAT_SLACK_SHARE of the
        # slack beyond it, so repeats cannot take all the time the sections
        # after the BASELINE ones (the IPC comparisons, the xGMI pair sweep)
        # would get, yet a node's 300 s deadline still leaves the N = 8
        # reference matrices room for a few runs each (one run of both
        # direction modes there is ~12 s over xGMI).
        self.slice_own = min(left, mine + REPEAT_SLACK_SHARE * max(0.0, left - mine)) if mine else left
        self.slice_t0 = time.monotonic()
        for s in self.live:
            s.set_timeout(max(1.0, min(self.args.timeout, wait_left)))
        self.state["section"] = name
        self.timeline.begin("section:" + name)
        self.faults.section(name)
        try:
            return fn()
        except Exception as e:  # noqa: BLE001 -- reported in the JSON
            log("bench: %s failed: %s" % (name, e))
            self.state["errors"][name] = str(e)[:300]
            if sessions:
                self.broken = name
            return {"error": str(e)[:300]}
        finally:
            self.state["section"] = None
            self.timeline.begin("untimed")

    def agreed_min(self, v: float) -> float:
        """The smallest of every rank's `v` (collective)."""
        return -self.h.sess.allreduce_max(-float(v)) if self.n > 1 else float(v)

    def slice_remaining(self) -> float:
        """Seconds the running section has left of its slice."""
        return self.slice_left - (time.monotonic() - self.slice_t0)

    def own_slice_remaining(self) -> float:
        """Seconds the running section has left of its own SECTION_SLICES
        share (slice_own)."""
        return self.slice_own - (time.monotonic() - self.slice_t0)

    def plan_sections(self):
        """The SECTION_SLICES sections this run will attempt (their slices are
        reserved while the ones before them run)."""
        args, n = self.args, self.n
        active = {"latency"}
        if args.latency_preposted > 0:
            active.add("latency_preposted")
        if args.ref_iters > 0:
            active |= {"reference_semantics", "pair_serial_events"}
            if self.stock_reference_planned():
                active.add("reference_semantics_stock")
        if n > 1 and args.extras:
            active |= {"allpairs_1g", "ring_256m", "ring_hop"}
        if n > 1 and args.sweep:
            active.add("pair_sweep_0_1")
        if n == 1 and args.sweep:
            active.add("self_sweep")
        self.active_sections = active
        self.slice_left, self.slice_own, self.slice_t0 = 0.0, 0.0, time.monotonic()
        self.broken = None

    # At most this many processes may hold one GPU (the test boxes' limit is
    # 16, pytest included): a child per rank doubles the ranks on a GPU.
    MAX_PROCS_PER_GPU = 15

    def stock_reference_planned(self) -> bool:
        """reference_semantics_stock runs for an RCCL headline (the stock
        settings are RCCL's and HIP's), when a child per rank still leaves
        the GPU within MAX_PROCS_PER_GPU processes (same answer on every
        rank: the provenance is shared)."""
        if not (self.args.ref_stock and self.args.ref_iters > 0 and self.transport_used == "rccl" and self.use_gpu):
            return False
        devs = (self.h.provenance or {}).get("rank_devices") or []
        keys = [d.get("pci") or "dev%s" % d.get("device") for d in devs]
        per_gpu = max([keys.count(k) for k in keys] or [self.n])
        return 2 * per_gpu <= self.MAX_PROCS_PER_GPU

    def latency_sections(self):
        """Host-posted ping-pong through the headline session, then the same
        pre-posted: batches of exchanges wait behind a stream gate on every
        rank and run back to back once all are posted, so those samples are
        the operation's GPU-timeline latency without the host's posting rate."""
        args, n, sess = self.args, self.n, self.h.sess
        nbytes = self.nat.parse_size(args.latency_size)

        def ping(preposted):
            # Exchanges that fit the section's slice: a short calibration pass
            # first (on xGMI a few ms; 8 ranks over loopback sockets took 18 s
            # for the full 300, profiles/r5_reh8/), agreed on every rank.
            iters = args.latency_iters
            if iters > 20:
                t0 = time.monotonic()
                sess.latency(nbytes, 10, 2, preposted)
                per = max(1e-6, (time.monotonic() - t0) / 12)
                fit = int(self.slice_remaining() / per) - min(50, iters)
                iters = int(self.agreed_min(max(20, min(iters, fit))))
            m = [[0.0] * n for _ in range(n)]
            lat = json.loads(sess.latency(nbytes, iters, min(50, iters), preposted))
            for p in lat["pairs"]:  # a < b; the ping-pong's one-way time holds for both directions
                m[p["a"]][p["b"]] = m[p["b"]][p["a"]] = round(p["one_way_us"]["p50"], 3)
            p50s = [p["one_way_us"]["p50"] for p in lat["pairs"]]
            return {"p50": float(statistics.median(p50s)) if p50s else None, "matrix": m, "method": lat["method"],
                    "iters": iters}

        r = self.section("latency", lambda: ping(0), budgeted=False)
        if isinstance(r, dict) and r.get("p50") is not None:
            self.reporter.update(p50_latency_us=round(r["p50"], 3), latency_p50_us_matrix=r["matrix"],
                                 latency_iters=r["iters"])
        if args.latency_preposted > 0:
            r = self.section("latency_preposted", lambda: ping(args.latency_preposted), budgeted=False)
            if isinstance(r, dict) and r.get("p50") is not None and r.get("method") == "preposted":
                self.reporter.update(p50_latency_preposted_us=round(r["p50"], 3),
                                     latency_preposted_p50_us_matrix=r["matrix"])

    def reference_section(self):
        """BASELINE config 3 by two methods on the reference's own schedule
        (serial ordered pairs, one at a time, p2p_matrix.cc:141-267), both
        directions modes (uni, and bi with both directions summed, :258):
          * reference_semantics: the reference's methodology on one
            communicator -- host clock, a stream sync per message, no warmup;
          * pair_serial_events: ours on the same schedule -- warmup, hipEvent
            timing, pipelined iterations, the headline's posting, every
            delivery verified.
        method_ratio (ours / the reference's, same schedule) and
        concurrency_ratio (tournament headline / serial pairs, same method)
        separate the two changes the headline makes.  With one GPU the
        reference prints only the diagonal; both methods then run on the self
        cell (uni only) so the method ratio still compares them.  The
        iterations shrink, and say so, when a time model (the headline's
        measured rate, then each direction mode's own) says the full count
        would not fit the section's slice."""
        args, n, h = self.args, self.n, self.h
        if args.ref_iters <= 0:
            return
        dirs = ("uni", "bi") if n > 1 else ("uni",)
        cells = n * (n - 1) if n > 1 else 1
        # GB/s per cell; the reference's method ran ~3.5x below our cell rate
        # on the self path, so its estimate assumes a quarter.
        rate = max(h.value or 1.0, 1e-3) * 1e9

        def matrices(session, timing, warmup, verify, slowdown):
            # Iterations per direction mode from the time the slice leaves it:
            # the first at the headline's rate (slowed by `slowdown`) plus a
            # fixed 10 ms per cell (barriers, fill, verify), later ones at the
            # previous mode's measured time per cell and iteration.  Agreed on
            # every rank.  Then the same matrix again, up to --ref-runs runs
            # in all, while this mode's share of the section's own slice
            # holds one more (at N = 1 a run is ~6 ms, so
            # all of them; at N = 8 over xGMI about one); combine_runs keeps
            # each run's mean cell and the median the ratios use.
            out, per_iter = {}, self.size * slowdown / rate + 50e-6
            for d in dirs:
                left = self.slice_remaining() / (len(dirs) - len(out))
                fit = int((left / cells - 0.01) / per_iter) - warmup
                # The fewest iterations a matrix is worth (8) must fit too: at
                # a slow link rate the minimum alone can take many times the
                # slice (8 ranks over loopback sockets: 88 s in a 6 s slice,
                # the deadline hit, profiles/r5_reh8c/).  Agreed on every rank.
                least = min(8, args.ref_iters)
                need = cells * ((warmup + least) * per_iter + 0.01)
                if not self.agree(need <= 1.5 * left):
                    out[d] = {"skipped": "the fewest iterations (%d + %d warmup) would take ~%.1f s, %.1f s left"
                                         % (least, warmup, need, left)}
                    break
                iters = int(self.agreed_min(min(args.ref_iters, max(least, fit))))
                # This mode's share of the section's own slice, fixed when it
                # starts (what an earlier mode left unused carries over).
                d_t0, d_share = time.monotonic(), self.own_slice_remaining() / (len(dirs) - len(out))
                runs, run_secs = [], []
                while True:
                    t0 = time.monotonic()
                    r = json.loads(session.run(mode="pair" if n > 1 else "self", dir=d, bytes=self.size, iters=iters,
                                               warmup=warmup, timing=timing, verify=verify, warm=warmup > 0))
                    run_s = self.allmax(time.monotonic() - t0)
                    runs.append(pair_matrix_summary(r, n))
                    run_secs.append(run_s)
                    # Everything the run took, charged to its iterations (conservative).
                    per_iter = max(1e-6, run_s / cells / (warmup + iters))
                    left_d = d_share - (time.monotonic() - d_t0)
                    if len(runs) >= max(1, args.ref_runs) or not self.agree(1.2 * run_s + 0.05 <= left_d):
                        break
                out[d] = dict(combine_runs(runs, n), iters=iters, run_s=round(statistics.median(run_secs), 4))
                if iters != args.ref_iters:
                    out[d]["iters_scaled_from"] = args.ref_iters
            return out

        def reference_semantics():
            out = matrices(h.ref_sess or h.sess, "wallclock", 0, False, 4.0)
            uni = (out.get("uni") or {}).get("median")
            return dict(out, size=self.size, comms=1,
                        # One stream for both directions: the reference's bi loop
                        # receives on a second stream (p2p_matrix.cc:214-225),
                        # which cost ~35% on the self cell (profiles/r6_cli_ab2/),
                        # so its bi cells read high here if anything.
                        method="reference semantics: serial ordered pairs, wall clock, stream sync per message, no "
                               "warmup, one stream" + ("" if n > 1 else " (applied to the self cell)"),
                        # Kept from round 2: the headline cell over the
                        # reference's uni cell (schedule and method together).
                        value_ratio=round(h.value / uni, 3) if uni else None)

        def pair_serial_events():
            out = matrices(h.sess, "events", 8, not args.no_verify, 1.5)
            return dict(out, size=self.size, comms=h.comms,
                        method="ours on the reference's schedule: serial ordered pairs, 8 warmup iterations, hipEvent "
                               "timing, iterations posted back to back, the headline's posting, every delivery verified")

        def reference_semantics_stock():
            # The same matrices and iterations in a child per rank with the
            # stock RCCL / HIP settings: the headline's process runs RCCL's
            # kernels at unroll 4, 8 HW queues and RCCL's INFO log, which the
            # reference's stock setup would not.
            iters = {d: v["iters"] for d, v in ref.items() if d in dirs and isinstance(v, dict) and "iters" in v}
            if not iters:
                return {"skipped": "the reference-method matrices it repeats were skipped"}
            # As many runs as the in-process matrices had, repeated inside the
            # child (its start, ~4.6 s, is paid once), or as many as this
            # section's slice holds at their measured time per run, at least
            # one; agreed (the same numbers on every rank: ref is collective).
            runs = child_runs(ref, iters, -self.allmax(-self.own_slice_remaining()), CHILD_START_S)
            r = self.child_job(REF_STOCK, ["--child-ref-iters", json.dumps(iters), "--child-ref-runs",
                                           json.dumps(runs), "--hw-queues", "0"], env=stock_env())
            if r is None or "error" in r:
                return r
            uni = (r.get("uni") or {}).get("median")
            return dict(r, size=self.size, comms=1, method=ref["method"] + "; stock RCCL / HIP settings",
                        value_ratio=round(h.value / uni, 3) if uni else None)

        self.log0("bench: reference-method matrices")
        ref = self.section("reference_semantics", reference_semantics, 5.0)
        self.reporter.update(reference_semantics=ref)
        if self.stock_reference_planned() and isinstance(ref, dict) and "error" not in ref:
            self.log0("bench: reference-method matrices, stock settings (child)")
            stock = self.section("reference_semantics_stock", reference_semantics_stock, 5.0, sessions=False)
            self.reporter.update(reference_semantics_stock=stock)
        else:
            stock = None
        ours = self.section("pair_serial_events", pair_serial_events, 5.0)
        ratios = method_ratios(ours if isinstance(ours, dict) else None, ref if isinstance(ref, dict) else None,
                               h.value, n)
        stock_ratios = method_ratios(ours if isinstance(ours, dict) else None,
                                     stock if isinstance(stock, dict) else None, h.value, n)
        self.reporter.update(pair_serial_events=ours, method_ratio_stock=stock_ratios["method_ratio"], **ratios)

    def extras_sections(self):
        """The other BASELINE.json configs, measured after the timed region so
        one driver run records them too: all-pairs concurrent exchange at 1 GiB
        (bisection: every GPU drives all N-1 xGMI links at once), the ring
        neighbour exchange at 256 MiB, the pipeline-parallel hop latency as a
        dependent token chain 0 -> 1 -> ... -> N-1 -> 0, and the single-pair
        (0 -> 1) bandwidth sweep 4 KiB -> 4 GiB (config 2; only cell (0, 1) is
        scheduled, the other ranks just join the barriers)."""
        args, n, nat, h = self.args, self.n, self.nat, self.h

        def concurrent_config(mode_x, dir_x, nbytes, iters):
            # Iterations the slice holds, at the headline's per-flow rate with
            # every rank's flows sharing it (a rank sends to up to N - 1 peers
            # at once): on xGMI a few ms each; over 8 loopback ranks an
            # all-pairs iteration at 1 GiB took ~4 s (profiles/r5_reh8d/).
            # At least one; agreed on every rank.
            flows = (n - 1) if mode_x == "allpairs" else 1
            per_iter = flows * nbytes / (max(h.value or 1.0, 1e-3) * 1e9) + 0.01
            fit = int(self.slice_remaining() / per_iter) - 1
            iters = int(self.agreed_min(max(1, min(iters, fit))))
            r = json.loads(h.sess.run(mode=mode_x, dir=dir_x, bytes=nbytes, iters=iters, warmup=1, timing="events",
                                      verify=not args.no_verify, warm=True))
            ph = r["phases"][0]
            flows = [f["gbs"] for f in ph["flows"]]
            p50s = [f["iter_us"]["p50"] for f in ph["flows"]]
            return {"aggregate_gbs": round(ph["agg_gbs"], 2), "per_gpu_egress_gbs": round(ph["agg_gbs"] / n, 2),
                    "flow_gbs_min": round(min(flows), 2), "flow_gbs_mean": round(statistics.mean(flows), 2),
                    "iter_us_p50": round(statistics.median(p50s), 1), "bytes": nbytes, "iters": iters,
                    "mismatches": ph["mismatches"]}

        def ring_hop():
            r = json.loads(h.sess.ring_latency(nat.parse_size(args.latency_size), 100, 10, False))
            return {"hop_us_p50": round(r["hop_us"]["p50"], 3), "hop_us_p99": round(r["hop_us"]["p99"], 3),
                    "lap_us_p50": round(r["lap_us"]["p50"], 3), "laps": r["laps"], "bytes": r["bytes"],
                    "method": "dependent token chain 0 -> 1 -> ... -> N-1 -> 0, each hop forwards after its "
                              "receive completed (grouped send/recv on the stream); hop = lap / N, rank 0's hipEvents"}

        def pair_cell(session, nbytes, iters):
            # Cell 0 -> 1 alone (N > 1), or the self cell (N = 1).
            cells = [(0, 1)] if n > 1 else []
            r = json.loads(session.run(mode="pair" if n > 1 else "self", dir="uni", bytes=nbytes, iters=iters,
                                       warmup=2, timing="events", verify=not args.no_verify, warm=False, cells=cells))
            fl = [f for ph in r["phases"] for f in ph["flows"]]
            return fl[0] if fl else None

        def size_sweep():
            # 4 KiB -> --sweep-max in powers of 4, every delivery verified,
            # while the slice lasts (the same decision on every rank); a size's
            # cost is estimated at the rate the previous one ran.
            sweep, rate = [], max(h.value or 1.0, 1e-3)
            for nbytes in [b for b in (4096 << (2 * k) for k in range(11)) if b <= nat.parse_size(args.sweep_max)]:
                iters = max(8, min(200, (2 << 30) // nbytes))  # >= 8 samples for the p50
                est = (iters + 2) * (nbytes / (rate * 1e9) + 50e-6)
                if not self.agree(self.slice_remaining() > est + 1.0):
                    sweep.append({"bytes": nbytes, "skipped": "no time left in the section's slice"})
                    break
                self.log0("bench: %s sweep %d B" % ("pair" if n > 1 else "self", nbytes))
                f = pair_cell(h.sess, nbytes, iters)
                if f:
                    rate = max(f["gbs"], 1e-3)
                    sweep.append({"bytes": nbytes, "iters": iters, "gbs": round(f["gbs"], 2),
                                  "iter_us_p50": round(f["iter_us"]["p50"], 2), "mismatches": f.get("mismatches", -1)})
            return sweep

        def one_comm():
            # The same cell on one communicator (what the sweep ran with K of
            # them), at the bench's message size and 256 MiB.
            return [{"bytes": nb, "gbs": round(f["gbs"], 2)}
                    for nb in (self.size, 256 << 20) for f in [pair_cell(h.ref_sess, nb, 16)] if f]

        if n == 1:
            # the sweep's code path on the self cell, so
            # every driver record (N = 1) runs it; BASELINE config 2's sizes.
            if args.sweep:
                sw = self.section("self_sweep", size_sweep, 2.0)
                if sw is not None:
                    extras = {"self_sweep": sw, "self_sweep_rccl_comms": h.comms}
                    if h.ref_sess is not None and h.ref_sess is not h.sess:
                        oc = self.section("self_one_comm", one_comm)
                        if oc is not None:
                            extras["self_one_comm"] = oc
                    self.reporter.update(extras=extras)
            return

        extras = None
        if args.extras:
            self.log0("bench: all-pairs / ring extras")
            extras = {}
            # Keyed by the BASELINE config names; the sizes can be lowered for
            # CPU rehearsals (all-pairs holds N - 1 receive slots per rank).
            for name, mode_x, dir_x, nbytes, iters in (
                    ("allpairs_1g", "allpairs", "bi", nat.parse_size(args.allpairs_size), 4),
                    ("ring_256m", "ring", "uni", nat.parse_size(args.ring_size), 8)):
                # A fixed handful of iterations (well under a second at 256 MiB -
                # 1 GiB on xGMI), so half the ring's 5 s slice is enough: under
                # a tight deadline the proportional shares leave it just under 5.
                v = self.section(name, lambda: concurrent_config(mode_x, dir_x, nbytes, iters), 2.5)
                if v is not None:
                    extras[name] = v
            v = self.section("ring_hop", ring_hop)
            if v is not None:
                extras["ring_hop"] = v
            self.reporter.update(extras=extras)
        if args.sweep:
            sw = self.section("pair_sweep_0_1", size_sweep, 10.0)
            if sw is not None:
                extras = dict(extras or {}, pair_sweep_0_1=sw, pair_sweep_rccl_comms=h.comms)
                if h.ref_sess is not None and h.ref_sess is not h.sess:
                    oc = self.section("pair_0_1_one_comm", one_comm)
                    if oc is not None:
                        extras["pair_0_1_one_comm"] = oc
            self.reporter.update(extras=extras)

    def isolated(self, transport, recv_budget=0):
        """steps_through() for `transport` in a child process per rank (with
        `recv_budget` bytes of receive slots each; 0: the child's default).  The
        comparisons drive the hand-written data plane (hipIpc mappings, signal
        kernels, relays) across GPUs; if one of them faults or hangs on some
        node, only the child dies, and the headline line still gets printed
        with the error in its place."""
        args = self.args
        extra = ["--mode", self.mode, "--steps", str(args.steps), "--warmup", str(args.warmup),
                 "--msgs", str(args.msgs), "--latency-iters", str(args.latency_iters),
                 "--latency-size", args.latency_size, "--child-batch", str(int(self.h.batch)),
                 "--recv-budget", str(int(recv_budget))]
        if args.no_verify:
            extra.append("--no-verify")
        return self.child_job(transport, extra)

    def child_job(self, child, extra, env=None):
        """bench.py --child `child` on every rank (its own TCP bootstrap on a
        port rank 0 picks), bounded by the time left; rank 0 returns the
        child's JSON (an error record if it wrote none), the others None."""
        args, n, rank = self.args, self.n, self.env.rank
        box = [free_port() if rank == 0 else None]
        if n > 1:
            dist.broadcast_object_list(box, src=0)
        out_path = os.path.join(tempfile.gettempdir(), "p2p_bench_child_%d_%d.json" % (box[0], rank))
        limit = min(args.child_timeout, max(5.0, self.budget_left()))
        cmd = [sys.executable, os.path.join(HERE, "bench.py"), "--gpus", str(n), "--size", args.size,
               "--child", child, "--child-port", str(box[0]), "--child-out", out_path,
               "--timeout", str(max(5.0, min(args.timeout, limit)))] + list(extra)
        if args.device is not None:
            cmd += ["--device", str(args.device)]
        rc = run_child(self.state, cmd, limit, env=env)
        self.barrier()
        res = None
        if rank == 0:
            try:
                with open(out_path) as f:
                    res = json.load(f)
            except (OSError, ValueError):
                res = {"error": "child process failed (exit status %s)" % rc, "transport": child}
        try:
            os.unlink(out_path)
        except OSError:
            pass
        return res

    def comparisons(self):
        """The same tournament steps through the hand-written data plane on
        the same links, untimed by the contract: the gfx950 multi-copy kernel
        pulling from hipIpc-mapped peer buffers ("pull", one-sided), the
        rendezvous engine that writes into the receiver's slot ("push"), the
        SDMA copy engines pulling instead of CUs ("sdma"), and multi-path push
        with two-hop relays through GPUs whose links are idle ("relay").  With
        one GPU the same engines run the self step (the GPU copies to itself
        through its own mapping), next to RCCL's self copy.  (With --transport
        host the same code path runs on the CPU transport, for tests.)"""
        args, n = self.args, self.n
        extra_transport = {"rccl": "ipc", "ipc": "ipc", "ipc:push": "ipc", "ipc:relay": "ipc", "host": "host",
                           "shm": "host"}.get(self.transport_used)
        if not (args.ipc_extra and extra_transport):
            return
        runs = [(extra_transport, None)]
        if extra_transport == "ipc":
            runs += [("ipc:push", "push"), ("ipc:sdma", "sdma")] + ([("ipc:relay", "relay")] if n > 2 else [])
            wanted = [e.strip() for e in args.ipc_engines.split(",") if e.strip()]
            runs = [(t, k) for (t, k) in runs if (k or "pull") in wanted]
        engines = {"ipc": "gfx950 multi-copy kernel, one-sided pull over hipIpc mappings",
                   "ipc:push": "ready/done flags + gfx950 multi-copy kernel writing into the peer's slot",
                   "ipc:sdma": "one-sided pull by the SDMA copy engines (hipMemcpyAsync per receive)",
                   "ipc:relay": "push over the direct link + two-hop stripes relayed through GPUs whose links are "
                                "idle (routing.hpp)"}
        value, batch = self.h.value, self.h.batch

        def compare(transport):
            # Ranks sharing a GPU split its free memory.  Every rank first
            # releases what the sections before it held (sessions, drivers and
            # their buffers), and only then does any rank read the free memory:
            # read while a peer on the same GPU was still freeing, it came out
            # short and halved the comparison's receive generations (8 ranks
            # on one GPU: verify_coverage 0.5).
            gc.collect()
            self.gpu_sync()
            self.barrier()
            budget = self.recv_budget(self.h.provenance)
            if args.isolate:
                return self.isolated(transport, budget)
            isess = self.create_session(transport, device=self.device,
                                        timeout_s=min(90.0, max(5.0, self.budget_left())))
            try:
                return steps_through(self.nat, isess, args, self.mode, self.size, batch, transport, budget)
            finally:
                del isess

        ipc = None
        for transport, key in runs:
            self.log0("bench: %s comparison" % transport)
            r = self.section(transport, lambda: compare(transport), 20.0, sessions=False)
            if r is None or self.env.rank != 0:
                continue
            if transport in engines:
                r["engine"] = engines[transport]
            if isinstance(r.get("value_gbs"), (int, float)) and value > 0:
                r["ratio_to_headline"] = round(r["value_gbs"] / value, 3)
            if key is None:
                ipc = dict(r, **(ipc or {}))
            else:
                ipc = dict(ipc or {}, **{key: r})
            self.reporter.update(ipc_transport=ipc)

    def xgmi_sweep_section(self):
        """The xGMI pair-cell tuning sweep in whatever time
        the deadline leaves: RCCL at 1, 2, 4 and 8 communicators, the IPC
        engines, then RCCL's channel / chunk / protocol / batch / read knobs,
        on cell 0 -> 1 (uni) and 0 <-> 1 (bi), every row verified; rows that do
        not fit are listed as skipped.  Rank 0 runs it as a child job while the
        other ranks wait at a barrier (their sessions are closed by then)."""
        args, n = self.args, self.n
        pcis = [d.get("pci") for d in (self.h.provenance or {}).get("rank_devices", [])]
        distinct = len(pcis) == n and all(pcis) and len(set(pcis)) == n
        on = args.xgmi_sweep if args.xgmi_sweep >= 0 else int(n == 2 and distinct and self.use_gpu)
        if n < 2 or not on:
            return
        if not self.use_gpu:
            emulate = "host"
        elif distinct:
            emulate = ""
        else:
            emulate = "rccl" if os.environ.get("P2P_RCCL_DISTINCT_HOSTS") == "1" else "ipc"

        def sweep():
            res = None
            if self.env.rank == 0:
                try:
                    res = self.run_pair_sweep(emulate)
                except Exception as e:  # noqa: BLE001 -- the other ranks wait at the barrier below
                    res = {"error": str(e)[:300]}
            self.barrier()
            return res

        r = self.section("xgmi_pair_sweep", sweep, 30.0, sessions=False)
        if r is not None and self.env.rank == 0:
            self.reporter.update(xgmi_pair_sweep=r)

    def run_pair_sweep(self, emulate):
        """scripts/xgmi_pair_sweep.py within the time left; returns its rows
        (cell GB/s and p50 per direction and size; bi = both directions
        summed, like the reference's bi matrix) and the winner per cell."""
        args, n = self.args, self.n
        budget = self.budget_left() - 15.0
        out = tempfile.mkdtemp(prefix="p2p_xgmi_sweep_")
        cmd = [sys.executable, os.path.join(HERE, "scripts", "xgmi_pair_sweep.py"), "--np", str(n), "--out", out,
               "--sizes", args.xgmi_sweep_sizes, "--rows", "rccl,ipc,knobs", "--budget", "%.0f" % budget,
               "--row-timeout", "%.0f" % min(float(os.environ.get("P2P_XGMI_SWEEP_ROW_TIMEOUT", 90)), budget)]
        if emulate:
            cmd += ["--emulate", emulate]
        log("bench: xGMI pair sweep (%.0f s%s)" % (budget, ", emulated: " + emulate if emulate else ""))
        t0 = time.monotonic()
        try:
            with open(os.path.join(out, "sweep.log"), "w") as lf:
                rc = run_child(self.state, cmd, budget + 15.0, stdout=lf, stderr=subprocess.STDOUT)
            res = {"rc": rc, "seconds": round(time.monotonic() - t0, 1), "budget_s": round(budget, 1),
                   "emulated": emulate or None, "sizes": args.xgmi_sweep_sizes, "cell": "0 -> 1 (uni), 0 <-> 1 (bi)",
                   "rows": {}}
            rows_path = os.path.join(out, "rows.jsonl")
            if os.path.exists(rows_path):
                with open(rows_path) as f:
                    for line in f:
                        r = json.loads(line)
                        res["rows"][r["name"]] = dict(
                            {"rc": r["rc"], "seconds": r.get("seconds")},
                            **{k: {"cell_gbs": round(c["cell_gbs"], 2), "p50_us": round(c["p50_us"], 2)}
                               for k, c in (r.get("cells") or {}).items()})
            # The best RCCL row per cell too: the setting the headline itself
            # could use on this link (the IPC engines are a different data plane).
            base = res["rows"].get("rccl-comms1", {})
            best_rccl = {}
            for name, row in res["rows"].items():
                for cell, c in row.items():
                    if name.startswith("rccl-") and row["rc"] == 0 and isinstance(c, dict) and (
                            cell not in best_rccl or c["cell_gbs"] > best_rccl[cell]["cell_gbs"]):
                        b0 = (base.get(cell) or {}).get("cell_gbs")
                        best_rccl[cell] = {"row": name, "cell_gbs": c["cell_gbs"],
                                           "gain": round(c["cell_gbs"] / b0, 4) if b0 else None}
            res["best_rccl"] = best_rccl or None
            try:
                with open(os.path.join(out, "summary.json")) as f:
                    summary = json.load(f)
                res["best"] = {k: {"row": b["row"], "cell_gbs": round(b["cell_gbs"], 2), "gain": b.get("gain")}
                               for k, b in summary["best"].items()}
                res.update(skipped=summary["rows_skipped"] or None, corrupt=summary["corrupt_rows"] or None,
                           failed_row=summary["failed_row"])
            except (OSError, ValueError, KeyError):
                with open(os.path.join(out, "sweep.log")) as f:
                    res["error"] = f.read()[-600:] or "the sweep wrote no summary"
            return res
        finally:
            shutil.rmtree(out, ignore_errors=True)

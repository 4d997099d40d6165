"""The headline of bench.py: posting selection, the W warmup and K timed
steps through RCCL (the verified warmup and its rechunking fallback, the link
report), the JSON line's timed part, and the IPC fallback should RCCL fail."""

from __future__ import annotations

import json
import os
import statistics
import time
import types

import torch
import torch.distributed as dist

from test_nccl_p2p_amd.bench.core import (BASELINE_VALUE, METRIC, RESERVE_S, TUNING_SHARE, candidate_budget,
                                          cell_matrix, first_candidate_budget, first_comms, headline_stats,
                                          link_check, log, pick_depth, posting_candidates, tuning_steps,
                                          unparsed_peers)
from test_nccl_p2p_amd.bench.faults import emulate_hang
from test_nccl_p2p_amd.utils.report import FALLBACK, SELF_COPY, XGMI_LINK


def hw_queues() -> int:
    """GPU_MAX_HW_QUEUES in effect for this process (HIP's default: 4)."""
    try:
        return int(os.environ.get("GPU_MAX_HW_QUEUES") or 4)
    except ValueError:
        return 4


def ranks_on_my_gpu(provenance, rank: int, device: int) -> int:
    """Ranks sharing this rank's GPU (provenance.rank_devices), matched by PCI
    bus id where known -- under a launcher that shows each rank only its own
    GPU every rank is on device 0 -- else by device index; at least 1."""
    devs = (provenance or {}).get("rank_devices") or []
    mine = next((d for d in devs if d.get("rank") == rank), None)
    if mine and mine.get("pci"):
        return sum(1 for d in devs if d.get("pci") == mine["pci"]) or 1
    return sum(1 for d in devs if d.get("device") == device) or 1


class HeadlineMixin:
    """BenchRun's headline methods (collective, like every BenchRun method)."""

    def recv_budget(self, provenance) -> int:
        """Bytes of receive slots a driver of this rank may allocate: --recv-budget,
        else 0.4 of the GPU's free memory now, split between the ranks on the
        same GPU (they allocate at the same time)."""
        args = self.args
        if args.recv_budget.strip() not in ("", "0"):
            return self.nat.parse_size(args.recv_budget)
        if not self.use_gpu:
            return 256 << 20
        free_b, _ = torch.cuda.mem_get_info(self.device)
        return int(0.4 * free_b / ranks_on_my_gpu(provenance, self.env.rank, self.device))

    # ---- the headline -------------------------------------------------------
    def measure(self, transport):
        """Posting selection, then the W warmup and K timed steps of the headline
        through `transport`; returns what the report needs."""
        args, nat, n, mode, size = self.args, self.nat, self.n, self.mode, self.size
        headline = transport + (":%d" % args.comms if transport == "rccl" and args.comms > 1 else "")
        tl, pre = self.timeline, ("fallback/" if self.fallback else "")
        # The first candidate's budget: a share of the time the deadline
        # leaves, so that should it hang the fallback still fits (core.py).
        first_budget = first_candidate_budget(args.timeout, self.deadline.left() - RESERVE_S)
        tl.begin(pre + "session_init")
        sess = self.create_session(headline, device=self.device, timeout_s=first_budget)
        self.log0("bench: %d rank(s), %s, %s" % (n, sess.transport, sess.device_desc))
        self.faults.fail_headline(transport)
        tl.begin(pre + "provenance")
        provenance = json.loads(sess.provenance(self.device if self.use_gpu else -1))
        provenance.pop("type", None)

        # Receive-slot budget: every message of every timed step gets its own
        # slot, up to this much memory per rank (ranks sharing a GPU split it).
        budget = self.recv_budget(provenance)

        # ---- posting selection (select_posting), before the W warmup steps
        # of the chosen candidate.
        self.state["section"] = "tuning"
        choices = posting_candidates(transport, args.comms, args.batch, n, hw_queues=hw_queues())
        c0 = first_comms(transport, args.comms)
        sessions = {c0: sess}

        def session_for(c, timeout_s):
            if c not in sessions:
                name = transport + (":%d" % c if transport == "rccl" and c > 1 else "")
                sessions[c] = self.create_session(name, device=self.device, timeout_s=timeout_s)
            else:
                sessions[c].set_timeout(timeout_s)
            return sessions[c]

        phases = len(nat.schedule(mode, "bi", n))
        sel = self.select_posting(transport, choices, c0, sessions, session_for, first_budget, phases, pre)
        comms, batch = sel.comms, sel.batch
        tl.begin(pre + "headline/session")
        sess = session_for(comms, args.timeout)
        # A single-communicator session stays for the reference-method comparison
        # (the reference uses one communicator); other candidates are closed.
        ref_sess = sessions.get(1)
        if ref_sess is not None:
            ref_sess.set_timeout(args.timeout)
        closing = [c for c in sessions if c not in (comms, 1)]
        if closing:
            # Its own entry: closing a session is ncclCommDestroy per
            # communicator (p2p_matrix.cc:270), not headline work.
            tl.begin(pre + "headline/close_candidates")
            for c in closing:
                del sessions[c]

        # ---- the headline driver: W warmup steps, poison, K timed steps -------
        self.state["section"] = "headline"
        tl.begin(pre + "headline/connect")
        drv = nat.StepDriver(sess, mode, "bi", size, args.msgs, not args.no_verify, bool(batch), bool(args.graph),
                             depth=pick_depth(args.steps, phases), recv_budget=budget, salt=1)
        drv.connect()
        rccl_peers, matrix_transport = (self.link_report(sess) if transport == "rccl" else (None, None))
        tl.begin(pre + "headline/warmup")
        drv.run_steps(0, args.warmup)
        drv.sync()
        chunking = None
        if transport == "rccl" and not args.no_verify and args.warmup > 0:
            chunking = self.verify_warmup(drv, [x for x in (sess, ref_sess) if x is not None])
        tl.begin(pre + "headline/poison")
        drv.poison()  # untimed: every receive slot zeroed; a slot passes verification only if a timed step wrote it
        self.gpu_sync()
        drv.reset()

        tl.begin(pre + "headline/timed")
        self.barrier()
        self.gpu_sync()
        self.barrier()
        t0 = time.perf_counter()
        drv.run_steps(args.warmup, args.steps)
        t_posted = time.perf_counter()  # host done posting (diagnostic: a host-bound run posts for ~all of it)
        drv.sync()
        self.gpu_sync()
        self.barrier()
        t1 = time.perf_counter()
        elapsed = sess.allreduce_max(t1 - t0)

        steps = list(range(args.warmup, args.warmup + args.steps))
        job_bytes = sum(drv.job_bytes_per_step(k) for k in steps)
        flows_total = sum(drv.flows_per_step(k) for k in steps)
        value, aggregate = headline_stats(job_bytes, flows_total, args.steps, elapsed)

        # Per-step GPU durations of every rank -> per-cell bandwidth.
        tl.begin(pre + "headline/matrix")
        my_ms = drv.step_ms()
        post_ms = list(drv.post_ms())
        all_ms = [None] * n
        if n > 1:
            dist.all_gather_object(all_ms, my_ms)
        else:
            all_ms = [my_ms]
        matrix, samples, cells = cell_matrix(n, steps, drv.phase_flows, all_ms, size * args.msgs)
        offdiag = [matrix[s][d] for (s, d) in cells if s != d or n == 1]

        # The post-timing check of every slot a timed step wrote (batched:
        # Transport::verify_many), timed for the record (verify_detail.seconds).
        tl.begin(pre + "headline/verify")
        v0 = time.perf_counter()
        vr = drv.verify_steps(args.warmup, args.steps) if not args.no_verify else None
        if vr is not None:
            vr["seconds"] = round(time.perf_counter() - v0, 4)
        depth, recv_bytes = drv.depth, drv.recv_bytes
        # Everything after this is untimed; release the timed driver's buffers
        # first so the comparisons run on the same memory footprint as the
        # timed steps did.
        del drv
        return types.SimpleNamespace(
            sess=sess, ref_sess=ref_sess, sessions=sessions, provenance=provenance, comms=comms, batch=batch,
            failed=sel.failed, skipped=sel.skipped, budgets=sel.budgets, first_cost=sel.first_cost, reason=sel.reason,
            tuning=sel.tuning, tuning_passes=sel.tuning_passes, elapsed=elapsed, flows_total=flows_total, value=value,
            aggregate=aggregate, my_ms=my_ms, matrix=matrix, samples=samples, cells=cells, offdiag=offdiag,
            expected=n * (n - 1) if n > 1 else 1, vr=vr, mismatches=vr["mismatches"] if vr else -1, depth=depth,
            recv_bytes=recv_bytes, chunking=chunking, rccl_peers=rccl_peers, matrix_transport=matrix_transport,
            host_post_ms=(t_posted - t0) * 1e3, post_ms=post_ms)

    def select_posting(self, transport, choices, c0, sessions, session_for, first_budget, phases, pre):
        """Posting selection: whole untimed laps of the schedule per candidate
        (one group per step vs one per message; RCCL: one communicator vs
        several whose send/recv kernels run side by side, posting_candidates),
        timed by the slowest rank.  Every wait of a candidate is bounded by its
        budget (first_candidate_budget / candidate_budget), so one that hangs
        on some rank is dropped on every rank in seconds, not at --timeout; the
        first candidate (the headline session's) must work, or this raises.
        `sessions` (communicator count -> session) is pruned as it goes."""
        args = self.args
        out = types.SimpleNamespace(tuning={}, tuning_passes={}, failed={}, skipped={}, budgets={}, first_cost=None)
        tune_k = tuning_steps(phases) * args.tune_laps
        if args.tune_laps <= 0 or len(choices) == 1:
            out.comms, out.batch = choices[0]
            out.reason = "single candidate" if len(choices) == 1 else "no tuning laps (--tune-laps 0): first candidate"
            return out
        tuning_t0 = time.monotonic()
        tuning_cap = TUNING_SHARE * max(0.0, self.deadline.left() - RESERVE_S)
        for i, (c, b) in enumerate(choices):
            key = "comms%d_%s" % (c, "batch" if b else "per_message")
            droppable = i > 0 or c != c0
            if droppable and out.first_cost is not None:
                wait_s = candidate_budget(out.first_cost, self.deadline.left() - RESERVE_S, args.timeout)
                used = time.monotonic() - tuning_t0
                if not self.agree(wait_s >= 1.0 and used + wait_s <= tuning_cap):
                    out.skipped[key] = "no time left: budget %.1f s, tuning used %.1f of %.1f s" % (
                        wait_s, used, tuning_cap)
                    self.log0("bench: posting candidate %s skipped: %s" % ((c, b), out.skipped[key]))
                    continue
            else:
                wait_s = first_budget
            out.budgets[key] = round(wait_s, 2)
            passes, connect_s, err, t_phase = self.try_candidate(transport, c, b, key, wait_s, session_for, tune_k, pre)
            if err is None:
                out.tuning[(c, b)] = min(passes)
                out.tuning_passes[(c, b)] = passes
                if out.first_cost is None:
                    out.first_cost = self.allmax(connect_s) + min(passes) * tune_k
                # Only the best communicator count so far, the headline session
                # and the single communicator (kept for the reference-method
                # comparison) stay open.
                best_c = min(out.tuning, key=out.tuning.get)[0]
                closing = [cc for cc in sessions if cc not in (c0, 1, best_c)
                           and not any(cc == c2 for (c2, _) in choices[i + 1:])]
                if closing:
                    # The losers' teardown (ncclCommDestroy per communicator)
                    # gets its own entry: charged to the pass it read as a slow
                    # tuning pass.
                    self.timeline.begin("%stuning/%s/close" % (pre, key))
                    for cc in closing:
                        del sessions[cc]
                continue
            # Failed (on every rank alike).  A wait that ran out its budget on
            # the slowest rank is reported as a timeout.
            self.timeline.begin("%stuning/%s/dropped" % (pre, key))
            if self.allmax(time.monotonic() - t_phase) >= 0.9 * wait_s:
                err = "timed out (waits bounded at %.1f s): %s" % (wait_s, err)
            if not droppable:
                raise RuntimeError("first posting candidate %s: %s" % (key, err))
            out.failed[key] = err
            self.log0("bench: posting candidate %s dropped: %s" % ((c, b), err))
            # Its session may be out of step across ranks (an aborted
            # communicator, a transfer cut off mid-message): closed on every
            # rank, and opened afresh should the headline need it.
            sessions.pop(c, None)
        out.comms, out.batch = min(out.tuning, key=out.tuning.get)
        out.reason = ("fastest of %d candidate(s): best of %d pass(es) of %d untimed step(s) each (%s lap(s) of %d "
                      "round(s)), slowest rank's clock" % (len(out.tuning), max(1, args.tune_passes), tune_k,
                                                          args.tune_laps, phases))
        return out

    def try_candidate(self, transport, c, b, key, wait_s, session_for, tune_k, pre):
        """One posting candidate (c communicators, batch b) on every rank: its
        session (waits bounded at wait_s), connect, then --tune-passes timed
        passes back to back, the fastest counting: the first pass carries the
        candidate's first-use costs, and one short pass is noisy (with a
        single 4-step pass, 2 of 16 one-GPU runs picked 4 communicators over 8
        and lost 15%, profiles/r3b_nt_ab/).  Every outcome is agreed on every
        rank.  Returns (seconds per step of each pass, connect seconds, error
        or None, when the failing phase began)."""
        args, nat, n, tl = self.args, self.nat, self.n, self.timeline
        d, err, connect_s, passes = None, None, 0.0, []
        hang = self.faults.candidate(transport, c, b)
        t_phase = time.monotonic()
        tl.begin("%stuning/%s/init" % (pre, key))
        try:
            s_c = session_for(c, wait_s)
            tl.begin("%stuning/%s/connect" % (pre, key))
            if hang == "connect":
                emulate_hang(wait_s)
            d = nat.StepDriver(s_c, self.mode, "bi", self.size, args.msgs, False, bool(b), bool(args.graph))
            d.connect()
            connect_s = time.monotonic() - t_phase
            self.faults.candidate_fail(c, b, "connect")
        except Exception as e:  # noqa: BLE001 -- reported, and the candidate is skipped everywhere
            err = str(e)[:200]
        if not self.agree(err is None):
            return passes, connect_s, err or "failed on another rank", t_phase
        for p in range(max(1, args.tune_passes)):
            self.barrier()
            tl.begin("%stuning/%s/pass%d" % (pre, key, p))
            t_phase = time.monotonic()
            w0 = time.perf_counter()
            try:
                if p == 0 and hang == "unbounded":
                    s_c.set_timeout(3600.0)
                elif p == 0 and hang in ("tuning", "stall"):
                    emulate_hang(wait_s, hang)
                d.run_steps(0, tune_k)
                d.sync()
                self.faults.candidate_fail(c, b, "tuning")
            except Exception as e:  # noqa: BLE001 -- same agreement as above
                err = str(e)[:200]
            w = time.perf_counter() - w0
            # The pass entry ends once every rank has finished it (the
            # agreement on its outcome returns then), so it is the slowest
            # rank's pass as tuning_passes_ms_per_step records it; the
            # bookkeeping after it gets an entry of its own.
            ok = self.agree(err is None)
            tl.begin("%stuning/%s/agree" % (pre, key))
            if not ok:
                return passes, connect_s, err or "failed on another rank", t_phase
            passes.append(self.allmax(w) / tune_k)
        return passes, connect_s, None, t_phase

    def verify_warmup(self, drv, sessions):
        """RCCL 2.26 / 2.27 deliver only the first half of an op whose share
        of one p2p channel exceeds 16 MiB, silently (scripts/rccl_half_repro.cpp);
        the transport posts messages in ops of 16 MiB x the channels RCCL's
        INFO log reports for each peer (transport_rccl.cpp derive_op_limits).
        As a second line of defence the warmup's deliveries are verified
        (collectively); should any word be wrong, every session caps its ops
        at 16, 4, then 1 MiB, graphs are recorded again, every slot is zeroed
        once every rank has drained, and the warmup runs again, until it
        verifies.  P2P_RECHUNK=0 turns the fallback off (the timed check then
        reports the loss).  Returns what was seen and done (posting.chunking)."""
        args, sess = self.args, sessions[0]
        peer = (self.env.rank + 1) % self.n
        bad = drv.verify_steps(0, args.warmup)["mismatches"]
        out = {"op_limit_bytes": sess.max_chunk(peer), "warmup_mismatches": bad, "fallback": None, "cap_bytes": None,
               "recaptured_graphs": 0}
        if bad and os.environ.get("P2P_RECHUNK") == "0":
            out["fallback"] = "off (P2P_RECHUNK=0)"
            return out
        tried = []
        for c in (16 << 20, 4 << 20, 1 << 20):
            if bad == 0:
                break
            # Agreed on every rank: all post the same steps, so all take the same branch.
            current = int(sess.allreduce_max(float(sess.max_chunk(peer) or self.size)))
            if c >= current:
                continue
            self.log0("bench: %d wrong words in the warmup: messages now posted as ops of <= %d MiB" % (bad, c >> 20))
            for s in sessions:
                s.set_chunk_cap(c)
            drv.recapture()
            drv.clear()
            drv.run_steps(0, args.warmup)
            drv.sync()
            bad = drv.verify_steps(0, args.warmup)["mismatches"]
            tried.append({"cap_bytes": c, "warmup_mismatches": bad})
            out["cap_bytes"] = c
        if tried:
            out.update(fallback=tried, op_limit_bytes=sess.max_chunk(peer), recaptured_graphs=drv.recaptures)
        return out

    def link_report(self, sess):
        """What RCCL set up (transport_rccl.cpp link_report): per rank, the p2p
        channels of each communicator and, per peer, the transport its INFO log
        shows (P2P = xGMI through IPC, SHM, NET), the channels connected and the
        op limit in use; plus matrix_transport, the N x N transport classes
        (row = rank, col = peer).  Collective."""
        try:
            reports = json.loads(sess.link_reports())
        except Exception as e:  # noqa: BLE001 -- recorded, never fatal
            return {"error": str(e)[:200]}, None
        if not any(reports):
            return None, None
        matrix = [[(r["peers"][p]["transport"] or "?") if r else "?" for p in range(self.n)] for r in reports]
        return reports, matrix

    def headline(self):
        """Measures the headline; should RCCL itself fail on this node
        (communicator setup, a peer connection, a stalled transfer: every wait
        is bounded by --timeout and aborts the communicators), the same steps
        run through the hand-written IPC data plane instead and the line says
        so (headline_fallback).  With --fallback 0, or if that fails too, the
        line carries the error and value null; returns that exit status."""
        args = self.args
        err = None
        try:
            self.h = self.measure(args.transport)
        except Exception as e:  # noqa: BLE001 -- reported in the JSON line
            err = str(e)[:300]
        # Outside the except block the failed attempt's frames are released, and
        # with them its sessions (aborted communicators, their streams, buffers).
        if err is None:
            return None
        log("bench: headline through %s failed: %s" % (args.transport, err))
        # The failure is collective (a communicator that cannot be set up or a
        # stalled transfer times out on every rank): all ranks meet here first.
        self.agree(False)
        to = args.fallback_to
        if not (args.fallback and args.transport in ("rccl", "host") and to != args.transport
                and (self.use_gpu or to in ("host", "shm"))):
            self.reporter.emit(error="headline failed: " + err, transport=args.transport)
            return 5
        self.fallback = {"from": args.transport, "to": to, "error": err}
        self.transport_used = to
        self.state["section"] = "fallback"
        err2 = None
        try:
            self.h = self.measure(to)
        except Exception as e2:  # noqa: BLE001
            err2 = str(e2)[:300]
        if err2 is None:
            return None
        log("bench: fallback headline failed: %s" % err2)
        self.reporter.emit(error="headline failed: %s; fallback through %s failed: %s" % (err, to, err2),
                           transport=args.transport, headline_fallback=self.fallback)
        return 5

    def value_kind(self) -> str:
        """SELF_COPY at N = 1 (no link: the diagonal the reference prints as
        0.00, p2p_matrix.cc:147-151), XGMI_LINK from N = 2 on GPUs, FALLBACK
        when the headline ran on the fallback data plane; a CPU transport's
        link otherwise (tests)."""
        if self.fallback:
            return FALLBACK
        if self.n == 1:
            return SELF_COPY if self.use_gpu else "self-copy (host memory, not a GPU)"
        if not self.use_gpu:
            return "%s-link per direction (not xGMI)" % self.h.sess.transport
        # Ranks sharing a GPU (the emulated node of the tests: PCI bus ids
        # repeat) move bytes within one GPU's memory, not over a link.
        devs = (self.h.provenance or {}).get("rank_devices") or []
        pcis = [d.get("pci") for d in devs]
        if len(pcis) == self.n and all(pcis) and len(set(pcis)) < self.n:
            return "emulated: %d ranks on %d GPU(s), per direction (not xGMI)" % (self.n, len(set(pcis)))
        return XGMI_LINK

    def base_result(self) -> dict:
        """The JSON line as far as the timed steps go; the untimed sections
        fill in the rest (Reporter.update)."""
        args, h, n, nat = self.args, self.h, self.n, self.nat
        headline_transport = h.sess.transport
        vr = h.vr
        # A headline that ran on the fallback data plane is not the metric's
        # (RCCL send/recv): value is null, the fallback's number stays beside it.
        value = None if self.fallback else round(h.value, 3)
        fallback = dict(self.fallback, value_gbs=round(h.value, 3)) if self.fallback else None
        return {
            "metric": METRIC,
            "value": value,
            # What `value` measures: utils/report.py
            # scaling_table never puts two kinds in one ratio.
            "value_kind": self.value_kind(),
            "unit": "GB/s",
            "n_gpus": n,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(h.elapsed / args.steps * 1e3, 4),
            "host_post_ms_per_step": round(h.host_post_ms / args.steps, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": (round(value / BASELINE_VALUE, 4) if BASELINE_VALUE and value else None),
            "dtype": "uint8",
            "data": "synthetic (device PRNG-filled payloads, one stream per message; every timed delivery verified "
                    "on the device after timing)",
            "config": {
                "model": "p2p_matrix: %s %s, %s x %d msgs/step"
                         % ("RCCL ncclSend/ncclRecv" if headline_transport == "rccl"
                            else headline_transport + " transport",
                            "self send/recv (uni)" if self.mode == "self" else self.mode + " bidirectional",
                            nat.format_size(self.size), args.msgs),
                "global_batch": args.msgs * n,
                "seq_len": self.size,
                "parallelism": "p2p%d" % n,
            },
            "value_definition": "mean cell of the GB/s matrix: all flows' bytes / slowest rank's barrier-bracketed "
                                "wall time / mean flows per step (per direction, 1 GB = 1e9 B)",
            "aggregate_gbs": round(h.aggregate, 3),
            "flows_per_step": round(h.flows_total / args.steps, 3),
            "matrix_gbs_min": round(min(h.offdiag), 3) if h.offdiag else None,
            "matrix_gbs_mean": round(statistics.mean(h.offdiag), 3) if h.offdiag else None,
            "matrix_cells": "%d/%d" % (len(h.cells), h.expected),
            # BASELINE config 3: the full N x N pairwise matrices (row = sender;
            # GB/s per direction, median over steps, a cell's time = the longer
            # of its endpoints'; p50 one-way latency, us).
            "matrix_gbs": [[round(v, 2) for v in row] for row in h.matrix],
            "matrix_samples": h.samples,
            "latency_p50_us_matrix": [[0.0] * n for _ in range(n)],
            "p50_latency_us": None,
            "p50_latency_preposted_us": None,
            "latency_preposted_p50_us_matrix": None,
            "latency_bytes": nat.parse_size(args.latency_size),
            "latency_iters": None,
            "per_gpu_gbs": round(h.aggregate / n, 3),
            "rank0_step_ms_p50": round(statistics.median(h.my_ms) if h.my_ms else 0.0, 4),
            # Every timed step's GPU time on rank 0, and what the wall-clock
            # bracket adds to their sum (launch of the first step, the final
            # sync and barrier): why `value` sits below `matrix_gbs_mean`.
            "rank0_step_ms": [round(x, 4) for x in h.my_ms],
            "bracket_overhead_ms": round(h.elapsed * 1e3 - sum(h.my_ms), 4) if h.my_ms else None,
            # Host time rank 0 took to post each timed step (the GPU runs ahead of
            # nothing but the first: later steps are posted while earlier ones run).
            "rank0_post_ms": [round(x, 4) for x in h.post_ms],
            "verify_mismatches": h.mismatches,
            "verify_coverage": (round(vr["verified_msgs"] / vr["timed_msgs"], 4) if vr and vr["timed_msgs"] else None),
            "verify_detail": vr,
            "recv_slot_generations": h.depth,
            "recv_slot_bytes_per_rank": h.recv_bytes,
            "transport": headline_transport,
            "posting": {"batch": bool(h.batch), "graph": bool(args.graph), "rccl_comms": h.comms, "chunking": h.chunking,
                        "hw_queues": {"GPU_MAX_HW_QUEUES": hw_queues(),
                                      "environment_had": os.environ.get("P2P_HW_QUEUES_ENV") or None},
                        "dropped": h.failed or None, "skipped": h.skipped or None, "selection": h.reason,
                        "candidate_budget_s": h.budgets or None,
                        "first_candidate_cost_s": round(h.first_cost, 4) if h.first_cost is not None else None,
                        "tuning_ms_per_step": {"comms%d_%s" % (c, "batch" if b else "per_message"): round(v * 1e3, 4)
                                               for (c, b), v in h.tuning.items()} or None,
                        "tuning_passes_ms_per_step": {"comms%d_%s" % (c, "batch" if b else "per_message"):
                                                      [round(v * 1e3, 4) for v in vs]
                                                      for (c, b), vs in h.tuning_passes.items()} or None},
            "provenance": dict(h.provenance, rccl_peers=h.rccl_peers),
            "matrix_transport": h.matrix_transport,
            "link_check": link_check(h.provenance.get("rank_links"), h.matrix_transport),
            # Peers whose RCCL connection lines did not parse:
            # [] when every connected peer's lines were read.
            "unparsed_peers": unparsed_peers(h.rccl_peers),
            "fabric_findings": None,
            "reference_semantics": None,
            "reference_semantics_stock": None,
            "pair_serial_events": None,
            "method_ratio": None,
            "method_ratio_stock": None,
            "concurrency_ratio": None,
            "extras": None,
            "ipc_transport": None,
            "xgmi_pair_sweep": None,
            "untimed_skipped": None,
            "headline_fallback": fallback,
            "note": ("n_gpus=1 has no inter-GPU link: value is RCCL's on-GPU self send/recv copy (HBM-bound), the "
                     "diagonal the reference prints as 0.00. From n_gpus=2 every step is one tournament round of "
                     "disjoint pairs, each pair on its own xGMI link; value is the mean per-link, per-direction cell "
                     "rate and aggregate_gbs the whole fabric")
                    if n == 1 else
                    ("each step is one tournament round: %d disjoint pairs exchange in both directions, one xGMI link "
                     "per pair; value = mean cell (per link and direction), aggregate_gbs = all pairs together"
                     % (n // 2)),
        }

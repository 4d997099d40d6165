#!/usr/bin/env python3
"""Headline benchmark: pairwise P2P GB/s matrix (min/mean) + p50 latency.

Metric and configs come from BASELINE.json ("pairwise P2P GB/s matrix
(min/mean) + p50 latency at 1/2/4/8 MI355X").  The reference
(/root/reference/p2p_matrix.cc) measures an N x N matrix of NCCL send/recv
bandwidth at 32 MiB per message (:124), one cell at a time, 128 messages per
cell (:132); this bench measures the same matrix on MI355X through the native
engine (RCCL ncclSend/ncclRecv over xGMI, hipEvent timing, gfx950 fill /
verify kernels).

One step = one round of the round-robin "tournament" schedule: the N ranks
form N/2 disjoint pairs (xGMI is fully connected point-to-point, so pairs never
share a link) and every pair exchanges --msgs messages of --size bytes in both
directions (default 128 x 32 MiB = 4 GiB per flow: one step is one of the
reference's cells, 128 x 32 MiB, p2p_matrix.cc:124,132, for every pair at
once), posted back to back inside ncclGroupStart/End.  Consecutive steps
walk through the N-1 rounds, so after N-1 steps every cell of the matrix has
been measured; per-GPU work per step is constant as N grows (weak scaling).
With one GPU the step is a self send/recv (uni: the GPU copies to itself; the
reference prints only the diagonal 0.00 there).

value = the mean cell of the matrix: bytes delivered by all flows during the K
timed steps / the slowest rank's wall time between two barrier +
torch.cuda.synchronize() brackets / the mean number of flows per step, in GB/s
(1e9 B/s) per direction.  aggregate_gbs is the same numerator without the
division (all flows together).

Verification covers the timed work: every message of a step is sent from its
own region of the send buffer (its own PRNG stream) into its own receive slot,
every step into its own generation of slots; all slots are zeroed after the
warmup and every slot a timed step wrote is checked on the device afterwards
(verify_mismatches / verify_coverage).

Every untimed section after the timed steps is bounded by one deadline counted
from process start (--deadline): each section's waits are shortened to the
time left, sections that would not fit are skipped (untimed_skipped), and a
watchdog prints the JSON line with what is done when the deadline passes.

At N = 2 on two distinct GPUs the time the deadline leaves after every other
section goes to the xGMI pair-cell tuning sweep (scripts/xgmi_pair_sweep.py:
RCCL communicator counts, the IPC engines, RCCL knobs; every row verified),
recorded in xgmi_pair_sweep.

Should RCCL itself fail on every rank (a communicator that cannot be set up, a
connection or transfer that stalls past --timeout), the same steps are timed
through the hand-written IPC data plane, but the metric names RCCL: value is
null and the IPC number is kept beside it (headline_fallback.value_gbs);
--fallback 0 reports the error alone.

Usage (driver contract):
  python bench.py --gpus 1 --steps K --warmup W
  python -m torch.distributed.run --nnodes=1 --nproc-per-node N \\
      --master-addr 127.0.0.1 --master-port P bench.py --gpus N --steps K --warmup W
"""

from __future__ import annotations

import argparse
import os
import sys
import time

T0 = time.monotonic()  # the deadline counts from here (process start, give or take the interpreter)


def set_hw_queues(argv) -> None:
    """--hw-queues Q (default 8, 0 = leave the environment alone): HIP's
    hardware queues per process, GPU_MAX_HW_QUEUES, which HIP reads when it
    initialises -- before argparse runs, hence this early look at argv.  The
    box's environment says 4 (HIP's default).  With RCCL's kernels at unroll
    4, 8 queues and 8 communicators move the 1-GPU step 7% faster than 4 and
    4 (profiles/r3_hwq/); the tuning laps still pick the communicator count.
    The value in effect and the environment's are recorded (posting.hw_queues)."""
    q = os.environ.get("P2P_BENCH_HW_QUEUES") or "8"  # (experiments: the default without --hw-queues)
    for i, a in enumerate(argv):
        if a == "--hw-queues" and i + 1 < len(argv):
            q = argv[i + 1]
        elif a.startswith("--hw-queues="):
            q = a.split("=", 1)[1]
    os.environ["P2P_HW_QUEUES_ENV"] = os.environ.get("GPU_MAX_HW_QUEUES", "")
    stash_stock_env()
    try:
        qn = int(q)
    except ValueError:  # argparse reports a bad --hw-queues; a bad P2P_BENCH_HW_QUEUES falls back
        qn = 8
    if 0 < qn <= 32:  # more is refused by parse_args
        os.environ["GPU_MAX_HW_QUEUES"] = str(qn)


# What this process changes about RCCL / HIP before they start (the queue
# count here, RCCL's unroll factor and INFO log in the native transport).  The
# environment as it was is kept, so reference_semantics_stock can run the
# reference's methodology in a child with the stock settings.
STOCK_ENV_KEYS = ("GPU_MAX_HW_QUEUES", "RCCL_UNROLL_FACTOR", "NCCL_DEBUG", "NCCL_DEBUG_FILE", "NCCL_DEBUG_SUBSYS")


def user_value(k, environ=None):
    """`k` as the user set it.  A parent process whose native engine set
    RCCL's variables (P2P_RCCL_ENV_OWNER: its pid) recorded what each one
    replaced in P2P_RCCL_PREV_<k> ("=<value>", or "" for unset); this process
    inherited its settings, not the user's (csrc/rccl_log.cpp
    undo_inherited_rccl_env, which the native side applies the same way)."""
    env = os.environ if environ is None else environ
    owner = env.get("P2P_RCCL_ENV_OWNER")
    prev = env.get("P2P_RCCL_PREV_" + k)
    if owner and owner != str(os.getpid()) and prev is not None:
        return prev[1:] if prev.startswith("=") else None
    return env.get(k)


def stash_stock_env() -> None:
    import json

    if "P2P_STOCK_ENV" not in os.environ:  # a child keeps its parent's record
        os.environ["P2P_STOCK_ENV"] = json.dumps({k: user_value(k) for k in STOCK_ENV_KEYS})


if __name__ == "__main__":  # (not when tests import this module)
    set_hw_queues(sys.argv[1:])

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from test_nccl_p2p_amd.bench import core  # noqa: E402

core.set_start(T0)
# Re-exported: the pure functions the unit tests pin (tests/test_bench_unit.py).
from test_nccl_p2p_amd.bench.compare import child_main, steps_through  # noqa: E402,F401
from test_nccl_p2p_amd.bench.core import (METRIC, Deadline, Reporter, Timeline, bench_fabric_findings,  # noqa: E402,F401
                                          candidate_budget, cell_matrix, claim_stdout, default_device,
                                          first_candidate_budget, first_comms, free_port,
                                          headline_stats, link_check, log, pick_depth, posting_candidates,
                                          process_age, start_watchdog, tuning_steps)
from test_nccl_p2p_amd.bench.faults import Faults  # noqa: E402
from test_nccl_p2p_amd.bench.headline import HeadlineMixin  # noqa: E402
from test_nccl_p2p_amd.bench.sections import SectionsMixin  # noqa: E402


def parse_args(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=28)
    ap.add_argument("--warmup", type=int, default=7)
    ap.add_argument("--size", default="32M", help="message size (reference: 32 MiB, p2p_matrix.cc:124)")
    ap.add_argument("--msgs", type=int, default=128,
                    help="messages per direction per step (128 x 32 MiB = 4 GiB per flow, the reference's cell "
                         "(p2p_matrix.cc:132); at N = 1 the step takes ~1.5 ms and the barrier + sync bracket costs "
                         "~1%% of the timed region, against ~4%% at 32 messages, profiles/r3_hwq/)")
    ap.add_argument("--mode", default="tournament", choices=["tournament", "ring", "allpairs", "pair", "self"])
    ap.add_argument("--transport", default="rccl", choices=["rccl", "ipc", "ipc:sdma", "ipc:push", "ipc:relay", "host", "shm"],
                    help="rccl (headline) | ipc = one-sided gfx950 copy kernel over hipIpc mappings | host = CPU (tests)")
    ap.add_argument("--comms", type=int, default=-1,
                    help="rccl: communicators per rank; the messages of a step are spread over them and their "
                         "send/recv kernels run side by side (-1: the tuning laps pick: 1, 4 or 8 on one GPU, 8 "
                         "only with >= 8 HW queues; 1, 2, 4 or 8 across GPUs; posting_candidates)")
    ap.add_argument("--device", type=int, default=None, help="GPU index (default LOCAL_RANK)")
    ap.add_argument("--hw-queues", type=int, default=8,
                    help="GPU_MAX_HW_QUEUES for this process, set before HIP starts (0: the environment's); more "
                         "queues let more communicators' kernels run side by side (set_hw_queues)")
    ap.add_argument("--latency-iters", type=int, default=300)
    ap.add_argument("--latency-size", default="8")
    ap.add_argument("--latency-preposted", type=int, default=16,
                    help="also time the ping-pong posted this many exchanges at a time behind a stream gate "
                         "(GPU-timeline latency, p50_latency_preposted_us; 0 = off)")
    ap.add_argument("--no-verify", action="store_true")
    ap.add_argument("--batch", type=int, default=-1,
                    help="1: all msgs of a step in one group (one launch); 0: one group per message; "
                         "-1: the tuning laps time both and the faster posting is used")
    ap.add_argument("--tune-laps", type=int, default=1,
                    help="untimed laps of the schedule per posting candidate, before the W warmup steps "
                         "(0: no tuning, the first candidate is used)")
    ap.add_argument("--tune-passes", type=int, default=2,
                    help="timed passes per posting candidate, back to back; the fastest counts (the first carries "
                         "first-use costs; tuning_passes_ms_per_step records them all)")
    ap.add_argument("--graph", type=int, default=0, help="1: replay each step as a captured hipGraph")
    ap.add_argument("--recv-budget", default="0",
                    help="receive-slot memory per rank (0: 40%% of free HBM / ranks per GPU); caps the slot "
                         "generations, and so verify_coverage")
    ap.add_argument("--json-out", default=None, help="also write the result line to this file")
    ap.add_argument("--ipc-extra", type=int, default=1,
                    help="1: also run the timed steps through the IPC engines (pull, push, sdma; relay from N = 3) "
                         "after the timed region, untimed by the contract, each in a child process per rank")
    ap.add_argument("--ipc-engines", default="pull,push,sdma,relay",
                    help="engines of the IPC comparison, in this order (relay only from N = 3)")
    ap.add_argument("--extras", type=int, default=1,
                    help="1: also measure all-pairs 1 GiB, ring 256 MiB and the ring token hop after the timed "
                         "region (N > 1)")
    ap.add_argument("--allpairs-size", default="1G", help="message size of the all-pairs extra (BASELINE config 4: 1 GiB)")
    ap.add_argument("--ring-size", default="256M", help="message size of the ring extra (BASELINE config 5: 256 MiB)")
    ap.add_argument("--sweep", type=int, default=1,
                    help="1: also sweep the single pair 0 -> 1 (N > 1; the self cell at N = 1) over 4 KiB .. "
                         "--sweep-max in powers of 4, verified, after the timed region")
    ap.add_argument("--sweep-max", default="4G", help="largest message of the pair sweep")
    ap.add_argument("--ref-iters", type=int, default=128,
                    help="iterations per cell of the reference-methodology comparison (0 = skip)")
    ap.add_argument("--ref-runs", type=int, default=7,
                    help="runs of each reference-method matrix (reference_semantics, its stock-settings child, "
                         "pair_serial_events): all of them at N = 1 (a run is a few ms), at N >= 2 as many as the "
                         "section's slice holds, at least one; the ratios use the median run")
    ap.add_argument("--fallback", type=int, default=1,
                    help="1: should the RCCL headline fail (setup, connection, stalled transfer), time the same steps "
                         "through the IPC data plane and keep that number in headline_fallback.value_gbs (value stays "
                         "null: the metric is RCCL's); 0: report the error only")
    ap.add_argument("--fallback-to", default="ipc", help=argparse.SUPPRESS)  # tests: host -> shm
    ap.add_argument("--isolate", type=int, default=1,
                    help="1: run each untimed transport comparison in a child process per rank (a fault there "
                         "cannot take the headline down); 0: in this process (halves the processes per GPU)")
    ap.add_argument("--timeout", type=float, default=120.0,
                    help="seconds any one wait of the headline session may take before it aborts and fails")
    ap.add_argument("--deadline", type=float, default=300.0,
                    help="seconds from process start by which the JSON line is printed; untimed sections are "
                         "shortened or skipped to fit, and a watchdog prints what is done when it passes")
    ap.add_argument("--untimed-budget", type=float, default=480.0,
                    help="seconds for all untimed sections after the timed steps (within --deadline)")
    ap.add_argument("--child-timeout", type=float, default=300.0,
                    help="seconds allowed to each untimed comparison process")
    ap.add_argument("--xgmi-sweep", type=int, default=-1,
                    help="the xGMI pair-cell tuning sweep (scripts/xgmi_pair_sweep.py: RCCL communicator counts, the "
                         "IPC engines, RCCL knobs on cell 0 -> 1, every row verified) in the time left after the other "
                         "sections: -1 at N = 2 on distinct GPUs, 1 at any N >= 2 (emulated where ranks share a GPU, "
                         "on the CPU host transport for --transport host), 0 never")
    ap.add_argument("--xgmi-sweep-sizes", default="32M,1G", help="message sizes of the pair sweep")
    ap.add_argument("--child", default=None, help=argparse.SUPPRESS)
    ap.add_argument("--child-port", type=int, default=0, help=argparse.SUPPRESS)
    ap.add_argument("--child-out", default=None, help=argparse.SUPPRESS)
    ap.add_argument("--child-batch", type=int, default=1, help=argparse.SUPPRESS)
    ap.add_argument("--child-ref-iters", default="{}", help=argparse.SUPPRESS)  # ref-stock: {"uni": I, "bi": I}
    ap.add_argument("--child-ref-runs", default="{}", help=argparse.SUPPRESS)  # ref-stock: {"uni": R, "bi": R}
    ap.add_argument("--ref-stock", type=int, default=1,
                    help="1: also run the reference's methodology in a child with the stock RCCL / HIP settings "
                         "(RCCL's own unroll, the environment's HW queues, no INFO log): reference_semantics_stock")
    args = ap.parse_args(argv)
    # Counts out of range fail here, before any rank starts, naming the option.
    at_least = {"gpus": 1, "steps": 1, "warmup": 0, "msgs": 1, "latency_iters": 1, "latency_preposted": 0,
                "tune_laps": 0, "tune_passes": 1, "ref_iters": 0, "ref_runs": 1, "hw_queues": 0}
    for name, lo in at_least.items():
        if getattr(args, name) < lo:
            ap.error("--%s must be >= %d, got %d" % (name.replace("_", "-"), lo, getattr(args, name)))
    if args.hw_queues > 32:
        ap.error("--hw-queues must be <= 32, got %d" % args.hw_queues)
    if args.comms == 0 or args.comms < -1:
        ap.error("--comms must be -1 (tuned) or >= 1, got %d" % args.comms)
    if args.batch not in (-1, 0, 1):
        ap.error("--batch must be -1, 0 or 1, got %d" % args.batch)
    for name in ("timeout", "deadline", "child_timeout"):
        if not getattr(args, name) > 0:
            ap.error("--%s must be > 0, got %g" % (name.replace("_", "-"), getattr(args, name)))
    if args.untimed_budget < 0:
        ap.error("--untimed-budget must be >= 0, got %g" % args.untimed_budget)
    return args


class BenchRun(HeadlineMixin, SectionsMixin):
    """One rank of a bench.py run.  Every method is collective (all ranks
    call it in the same order): the headline (posting selection, W warmup
    and K timed steps, with the IPC fallback; test_nccl_p2p_amd/bench/headline.py),
    then the untimed sections (bench/sections.py), all under one deadline
    counted from process start."""

    def __init__(self, args, real_stdout: int):
        from test_nccl_p2p_amd import require_native
        from test_nccl_p2p_amd.parallel.session import create_session, init_control_plane

        self.args = args
        self.timeline = Timeline(T0)
        self.timeline.begin("init")
        self.nat = require_native()
        self.create_session = create_session
        self.deadline = Deadline(args.deadline)
        self.env = init_control_plane("gloo", timeout_s=max(60.0, args.deadline))
        if args.gpus != self.env.world:
            log("bench: --gpus %d but WORLD_SIZE=%d; using WORLD_SIZE" % (args.gpus, self.env.world))
        self.n = self.env.world
        self.use_gpu = args.transport not in ("host", "shm")
        self.device = default_device(self.env.local_rank) if args.device is None else args.device
        if self.use_gpu:
            torch.cuda.set_device(self.device)
        self.faults = Faults(self.env.rank, self.env.world)  # the test hooks, read once (bench/faults.py)
        self.reporter = Reporter(self.env.rank, real_stdout, args.json_out, self.timeline, self.deadline)
        self.state = {"section": "setup", "skipped": [], "errors": {}}
        start_watchdog(self.deadline, self.reporter, self.nat, self.state)
        self.size = self.nat.parse_size(args.size)
        self.mode = "self" if self.n == 1 else args.mode
        self.h = None              # the headline's measurement (measure())
        self.fallback = None       # headline_fallback of the JSON line
        self.transport_used = args.transport
        self.live = []             # sessions whose waits the untimed sections bound
        self.untimed_t0 = None

    # ---- collectives over the gloo control plane ---------------------------
    def barrier(self):
        if self.n > 1:
            dist.barrier()

    def gpu_sync(self):
        if self.use_gpu:
            torch.cuda.synchronize()

    def agree(self, ok: bool) -> bool:
        """True when every rank reports ok (the candidates are collective)."""
        if self.n == 1:
            return ok
        t = torch.tensor([1 if ok else 0], dtype=torch.int32)
        dist.all_reduce(t, op=dist.ReduceOp.MIN)
        return bool(t.item())

    def allmax(self, v: float) -> float:
        """The largest of every rank's `v`, over the gloo control plane (not a
        native session's bootstrap, which a failed candidate may leave out of
        step)."""
        if self.n == 1:
            return float(v)
        t = torch.tensor([float(v)], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    def log0(self, msg: str):
        if self.env.rank == 0:
            log(msg)

    # ---- the headline -------------------------------------------------------
    def run(self) -> int:
        rc = self.headline()
        if rc is not None:
            return rc
        h = self.h
        self.reporter.result = self.base_result()
        lc = self.reporter.result.get("link_check")
        if lc and not lc["ok"]:
            self.log0("bench: WRONG TRANSPORT: RCCL carried %d of %d direct xGMI pairs over something else than "
                      "P2P: %s" % (len(lc["not_p2p"]), lc["direct_xgmi_pairs"], ", ".join(lc["not_p2p"][:16])))
        up = self.reporter.result.get("unparsed_peers")
        if up:
            self.log0("bench: WARN RCCL connection lines not parsed for %s: their ops stay at the 2-channel limit "
                      "(raw lines: provenance.rccl_peers[].unparsed_peers)" % ", ".join(up[:16]))
        self.log0("bench: value %.2f GB/s per cell (aggregate %.2f GB/s), %.4f ms/step, verify %s" % (
            h.value, h.aggregate, h.elapsed / self.args.steps * 1e3, h.vr))

        self.untimed_t0 = time.monotonic()
        self.timeline.begin("untimed")
        self.plan_sections()
        self.live = list({id(x): x for x in (h.sess, h.ref_sess) if x is not None}.values())
        self.latency_sections()
        self.reference_section()
        self.extras_sections()
        # The comparisons open sessions of their own; close the headline's
        # first so they run alone, as the timed steps did.
        self.live.clear()
        h.sess = h.ref_sess = h.sessions = None
        self.comparisons()
        self.xgmi_sweep_section()

        self.timeline.begin("report")
        self.reporter.update(untimed_skipped=self.state["skipped"] or None,
                             section_errors=self.state["errors"] or None)
        if self.env.rank == 0:
            ff = bench_fabric_findings(self.reporter.result, self.n)
            self.reporter.update(fabric_findings=ff)
            for f in ff or []:
                log("bench: fabric: " + f)
            log("bench: GB/s matrix (row=src, col=dst), median over steps:")
            for r in range(self.n):
                log("  " + " ".join("%8.2f" % h.matrix[r][c] for c in range(self.n)))
        self.reporter.emit()
        # The watchdog stays armed: should the teardown below hang, it ends the
        # process at the deadline (the line is out already, so it exits 0).  A
        # peer whose watchdog ended it first breaks this barrier; that is no
        # error of the measurement either.
        self.timeline.begin("teardown")
        self.faults.teardown()
        try:
            self.barrier()
            if self.n > 1 and dist.is_initialized():
                dist.destroy_process_group()
        except Exception as e:  # noqa: BLE001 -- the line is out
            log("bench: teardown: %s (the result line is out)" % str(e)[:200])
        # The timeline ends at the JSON line; this is the whole process (a
        # test holds the timeline's total against it).
        self.log0("bench: process wall %.3f s" % process_age())
        return 0 if h.mismatches in (0, -1) else 3


def main(argv=None) -> int:
    args = parse_args(argv)
    if args.child:
        return child_main(args)
    try:
        rc = BenchRun(args, claim_stdout()).run()
    except BaseException:
        if not core.WATCHDOG_FIRED.is_set():
            raise
        rc = None
    if core.WATCHDOG_FIRED.is_set():
        # The deadline's watchdog printed the line and ends the process with
        # its own status (0 with a result, 4 without) once the communicators
        # are aborted; a main thread that got here meanwhile -- e.g. through a
        # peer whose exit broke a gloo collective -- must not end it first.
        while True:
            time.sleep(1.0)
    return rc


if __name__ == "__main__":
    sys.exit(main())

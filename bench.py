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
directions (default 32 x 32 MiB = 1 GiB per flow; the reference's cell is
128 x 32 MiB, p2p_matrix.cc:132), posted back to back inside
ncclGroupStart/End.  Consecutive steps
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
through the hand-written IPC data plane and the line says so
(headline_fallback); --fallback 0 reports the error with value null instead.

Usage (driver contract):
  python bench.py --gpus 1 --steps K --warmup W
  python -m torch.distributed.run --nnodes=1 --nproc-per-node N \\
      --master-addr 127.0.0.1 --master-port P bench.py --gpus N --steps K --warmup W
"""

from __future__ import annotations

import argparse
import json
import math
import os
import shutil
import socket
import statistics
import subprocess
import sys
import tempfile
import threading
import time
import types

T0 = time.monotonic()  # the deadline counts from here (process start, give or take the interpreter)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from test_nccl_p2p_amd.utils.proc import kill_children, run_child  # noqa: E402

METRIC = "pairwise P2P GB/s matrix (min/mean) + p50 latency at 1/2/4/8 MI355X"
BASELINE_VALUE = None  # the reference publishes no numbers
RESERVE_S = 15.0  # kept free at the end of the deadline for the JSON line and teardown
HERE = os.path.dirname(os.path.abspath(__file__))


def log(*a):
    print("[%7.1fs]" % (time.monotonic() - T0), *a, file=sys.stderr, flush=True)


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


def posting_candidates(transport: str, comms: int, batch: int, n: int = 1):
    """(communicators, batch) pairs the tuning laps time against each other.

    comms: > 0 fixed, -1 = RCCL picks: between 1 and 4 on one GPU (measured:
    2, 3, 6 and 8 are slower there, profiles/r2_step_shape/), between 1, 2, 4
    and 8 across GPUs, where no measurement has fixed the count for an xGMI
    link yet (other transports: 1).  batch: 1 one group per step, 0 one group
    per message, -1 = both (K = 1 only: with several communicators
    per-message groups cannot overlap)."""
    auto = [1, 4] if n == 1 else [1, 2, 4, 8]
    comms_choices = ([comms] if comms > 0 else auto) if transport == "rccl" else [1]
    batch_choices = [batch] if batch >= 0 else [0, 1]
    return [(c, b) for c in comms_choices for b in batch_choices if c == 1 or b == 1 or len(batch_choices) == 1]


def tuning_steps(phases: int, min_steps: int = 4) -> int:
    """Steps per candidate: whole laps of the schedule (every cell once per
    lap), at least min_steps so a one-round schedule is not timed on one step."""
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
        self.end = T0 + seconds

    def left(self) -> float:
        return self.end - time.monotonic()


class Reporter:
    """Holds the result and prints it exactly once (rank 0): at the normal end
    of the run, or from the watchdog when the deadline passes first."""

    def __init__(self, rank: int, real_stdout: int, json_out):
        self.rank = rank
        self.fd = real_stdout
        self.json_out = json_out
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
            line = json.dumps(res)
            os.write(self.fd, (line + "\n").encode())
            if self.json_out:
                with open(self.json_out, "w") as f:
                    f.write(line + "\n")
            return True


def start_watchdog(deadline: Deadline, reporter: Reporter, nat, state) -> threading.Event:
    """At the deadline: print the JSON line with what is finished (the section
    still running is named), abort every RCCL communicator so its kernels exit,
    and end the process.  Exit 0 when the headline was measured."""
    stop = threading.Event()

    def run():
        while not stop.wait(max(0.05, min(1.0, deadline.left()))):
            if deadline.left() <= 0:
                break
        if stop.is_set():
            return
        log("bench: deadline reached during %s; printing what is done" % state.get("section"))
        errors = dict(state.get("errors") or {})
        if state.get("section"):
            errors[state["section"]] = "deadline reached while running"
        reporter.emit(deadline_hit=True, untimed_skipped=state.get("skipped") or None, section_errors=errors or None)
        kill_children(state)
        try:
            nat.run_abort_hooks()
        except Exception:  # noqa: BLE001 -- the process ends either way
            pass
        sys.stderr.flush()
        os._exit(0 if reporter.result is not None else 4)

    threading.Thread(target=run, name="bench-watchdog", daemon=True).start()
    return stop


def steps_through(nat, isess, args, mode, size, batch, transport, deadline=None):
    """The timed steps again through another transport session (untimed by
    the contract); any error is reported instead of failing the run."""
    try:
        n = isess.world
        phases = len(nat.schedule(mode, "bi", n))
        idrv = nat.StepDriver(isess, mode, "bi", size, args.msgs, not args.no_verify, bool(batch), False,
                              depth=pick_depth(args.steps, phases), salt=2)
        say = (lambda m: log("bench: %s: %s" % (transport, m))) if isess.rank == 0 else (lambda m: None)
        idrv.connect()
        say("connected (%d receive generations)" % idrv.depth)
        idrv.run_steps(0, args.warmup)
        idrv.sync()
        idrv.poison()
        isess.barrier()
        say("warm")
        i0 = time.perf_counter()
        idrv.run_steps(args.warmup, args.steps)
        idrv.sync()
        isess.barrier()
        say("timed steps done")
        ielapsed = isess.allreduce_max(time.perf_counter() - i0)
        steps = range(args.warmup, args.warmup + args.steps)
        value, aggregate = headline_stats(sum(idrv.job_bytes_per_step(k) for k in steps),
                                          sum(idrv.flows_per_step(k) for k in steps), args.steps, ielapsed)
        vr = idrv.verify_steps(args.warmup, args.steps) if not args.no_verify else None
        out = {"value_gbs": round(value, 3), "aggregate_gbs": round(aggregate, 3),
               "ms_per_step": round(ielapsed / args.steps * 1e3, 4),
               "verify_mismatches": vr["mismatches"] if vr else -1,
               "verify_coverage": round(vr["verified_msgs"] / vr["timed_msgs"], 4) if vr and vr["timed_msgs"] else None,
               "transport": transport}
        del idrv
        # Device-initiated ping-pong and ring token chain: one wave per GPU
        # writes into the peer's memory and spins on its own inbox (no host,
        # no runtime in the loop) -- the fabric's latency, next to RCCL's.
        if transport == "ipc":
            dl = json.loads(isess.device_latency(nat.parse_size(args.latency_size), args.latency_iters,
                                                 min(100, args.latency_iters)))
            out["device_pingpong_p50_us"] = round(statistics.median(p["one_way_us"]["p50"] for p in dl["pairs"]), 3)
            # BASELINE config 3's latency matrix at the fabric floor: one-way
            # p50 per pair (symmetric; self on the diagonal at N = 1).
            dm = [[0.0] * n for _ in range(n)]
            for p in dl["pairs"]:
                dm[p["a"]][p["b"]] = dm[p["b"]][p["a"]] = round(p["one_way_us"]["p50"], 3)
            out["device_latency_p50_us_matrix"] = dm
            if n > 1:
                rl = json.loads(isess.ring_latency(nat.parse_size(args.latency_size), 100, 10, True))
                out["device_ring_hop_p50_us"] = round(rl["hop_us"]["p50"], 3)
                out["device_ring_lap_p50_us"] = round(rl["lap_us"]["p50"], 3)
        # Multi-path: the reference's single-pair cell (0 -> 1, every other
        # GPU idle) with the message striped over the direct link and two-hop
        # relays through the idle GPUs.
        if transport == "ipc:relay":
            pair = []
            for nbytes in (size, 256 << 20):
                r = json.loads(isess.run(mode="pair", dir="uni", bytes=nbytes, iters=16, warmup=2,
                                         timing="events", verify=not args.no_verify, warm=False, cells=[(0, 1)]))
                fl = [f for ph in r["phases"] for f in ph["flows"]]
                if fl:
                    pair.append({"bytes": nbytes, "gbs": round(fl[0]["gbs"], 2),
                                 "iter_us_p50": round(fl[0]["iter_us"]["p50"], 2),
                                 "mismatches": fl[0].get("mismatches", -1)})
            out["pair_0_1"] = pair
        return out
    except Exception as e:  # report, never fail the headline
        return {"error": str(e)[:300], "transport": transport}


def child_main(args) -> int:
    """--child: one rank of an untimed comparison run (see isolated() in
    main).  Bootstraps its own native TCP star on --child-port (no
    torch.distributed: the parent's store is busy) and writes rank 0's result
    to --child-out."""
    from test_nccl_p2p_amd.utils.proc import die_with_parent

    die_with_parent()
    claim_stdout()
    from test_nccl_p2p_amd import require_native
    from test_nccl_p2p_amd.parallel.session import dist_env

    nat = require_native()
    env = dist_env()
    device = default_device(env.local_rank) if args.device is None else args.device
    size = nat.parse_size(args.size)
    if env.rank == 0:
        log("bench: child %s started" % args.child)
    try:
        sess = nat.Session(env.rank, env.world, host=env.master_addr, port=args.child_port, device=device,
                           transport=args.child, timeout_s=min(90.0, args.timeout))
        out = steps_through(nat, sess, args, args.mode, size, args.child_batch, args.child)
        del sess
    except Exception as e:
        out = {"error": str(e)[:300], "transport": args.child}
    if env.rank == 0:
        log("bench: child %s done" % args.child)
        with open(args.child_out, "w") as f:
            json.dump(out, f)
    return 0


def parse_args(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=28)
    ap.add_argument("--warmup", type=int, default=7)
    ap.add_argument("--size", default="32M", help="message size (reference: 32 MiB, p2p_matrix.cc:124)")
    ap.add_argument("--msgs", type=int, default=32,
                    help="messages per direction per step (32 x 32 MiB = 1 GiB per flow: at N = 1 the step takes "
                         "~0.45 ms, so the barrier + sync bracket costs ~3%% of the timed region instead of ~10%% "
                         "at 8 messages, profiles/r2_step_shape/)")
    ap.add_argument("--mode", default="tournament", choices=["tournament", "ring", "allpairs", "pair", "self"])
    ap.add_argument("--transport", default="rccl", choices=["rccl", "ipc", "ipc:sdma", "ipc:push", "ipc:relay", "host", "shm"],
                    help="rccl (headline) | ipc = one-sided gfx950 copy kernel over hipIpc mappings | host = CPU (tests)")
    ap.add_argument("--comms", type=int, default=-1,
                    help="rccl: communicators per rank; the messages of a step are spread over them and their "
                         "send/recv kernels run side by side (-1: the tuning laps pick 1 or 4)")
    ap.add_argument("--device", type=int, default=None, help="GPU index (default LOCAL_RANK)")
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
                    help="1: also sweep the single pair 0 -> 1 over 4 KiB .. --sweep-max (N > 1, after the timed region)")
    ap.add_argument("--sweep-max", default="4G", help="largest message of the pair sweep")
    ap.add_argument("--ref-iters", type=int, default=128,
                    help="iterations per cell of the reference-methodology comparison (0 = skip)")
    ap.add_argument("--fallback", type=int, default=1,
                    help="1: should the RCCL headline fail (setup, connection, stalled transfer), time the same steps "
                         "through the IPC data plane and say so in headline_fallback; 0: report the error only")
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
    return ap.parse_args(argv)


def default_device(local_rank: int) -> int:
    """LOCAL_RANK, modulo the visible GPUs: a launcher that gives each rank
    one visible GPU (HIP_VISIBLE_DEVICES per process) leaves every rank on
    its device 0.  torch.cuda.device_count() does not initialise the GPU."""
    count = torch.cuda.device_count()
    return local_rank % count if count > 0 else local_rank


def hang_requested(section: str, rank: int) -> bool:
    """Test hook: P2P_BENCH_HANG="<section>@<rank>" makes that rank stop
    responding inside that untimed section."""
    spec = os.environ.get("P2P_BENCH_HANG", "")
    return bool(spec) and spec == "%s@%d" % (section, rank)


class BenchRun:
    """One rank of a bench.py run.  Every method is collective (all ranks
    call it in the same order): the headline (posting selection, W warmup
    and K timed steps, with the IPC fallback), then the untimed sections, all
    under one deadline counted from process start."""

    def __init__(self, args, real_stdout: int):
        from test_nccl_p2p_amd import require_native
        from test_nccl_p2p_amd.parallel.session import create_session, init_control_plane

        self.args = args
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
        self.reporter = Reporter(self.env.rank, real_stdout, args.json_out)
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

    def log0(self, msg: str):
        if self.env.rank == 0:
            log(msg)

    # ---- the headline -------------------------------------------------------
    def measure(self, transport):
        """Posting selection, then the W warmup and K timed steps of the headline
        through `transport`; returns what the report needs."""
        args, nat, n, mode, size = self.args, self.nat, self.n, self.mode, self.size
        headline = transport + (":%d" % args.comms if transport == "rccl" and args.comms > 1 else "")
        sess = self.create_session(headline, device=self.device, timeout_s=args.timeout)
        self.log0("bench: %d rank(s), %s, %s" % (n, sess.transport, sess.device_desc))
        # Test hook: P2P_BENCH_FAIL_HEADLINE=<transport> fails the headline
        # through that transport on every rank, as a communicator that cannot
        # be set up does.
        if os.environ.get("P2P_BENCH_FAIL_HEADLINE") == transport:
            raise RuntimeError("injected headline failure")
        provenance = json.loads(sess.provenance(self.device if self.use_gpu else -1))
        provenance.pop("type", None)

        # Receive-slot budget: every message of every timed step gets its own
        # slot, up to this much memory per rank (ranks sharing a GPU split it).
        budget = 0 if args.recv_budget.strip() in ("", "0") else nat.parse_size(args.recv_budget)
        if budget == 0 and self.use_gpu:
            free_b, _ = torch.cuda.mem_get_info(self.device)
            same_gpu = sum(1 for d in provenance.get("rank_devices", []) if d["device"] == self.device) or 1
            budget = int(0.4 * free_b / same_gpu)
        elif budget == 0:
            budget = 256 << 20

        # ---- posting selection: whole untimed laps of the schedule per
        # candidate (one group per step vs one per message; RCCL: one
        # communicator vs several whose send/recv kernels run side by side,
        # posting_candidates), timed by the slowest rank, before the W warmup
        # steps of the chosen one.
        self.state["section"] = "tuning"
        choices = posting_candidates(transport, args.comms, args.batch, n)
        c0 = first_comms(transport, args.comms)
        sessions = {c0: sess}

        def session_for(c):
            if c not in sessions:
                # A candidate that stalls is aborted and dropped after --timeout.
                sessions[c] = self.create_session("rccl:%d" % c if c > 1 else "rccl", device=self.device,
                                                  timeout_s=args.timeout)
            return sessions[c]

        tuning, failed = {}, {}
        phases = len(nat.schedule(mode, "bi", n))
        tune_k = tuning_steps(phases) * args.tune_laps
        if args.tune_laps > 0 and len(choices) > 1:
            for i, (c, b) in enumerate(choices):
                key = "comms%d_%s" % (c, "batch" if b else "per_message")
                # The headline session's first candidate must work; anything else
                # (another communicator count, another posting) may be dropped.
                droppable = i > 0 or c != c0
                d, err = None, None
                try:
                    d = nat.StepDriver(session_for(c), mode, "bi", size, args.msgs, False, bool(b), bool(args.graph))
                    d.connect()
                    # Test hook: P2P_BENCH_FAIL_CANDIDATE="<comms>,<batch>" fails
                    # that candidate on the last rank only.
                    if os.environ.get("P2P_BENCH_FAIL_CANDIDATE") == "%d,%d" % (c, b) and self.env.rank == n - 1:
                        raise RuntimeError("injected candidate failure")
                except Exception as e:  # noqa: BLE001 -- reported, and the candidate is skipped everywhere
                    err = str(e)[:200]
                if self.agree(err is None):
                    self.barrier()
                    w0 = time.perf_counter()
                    try:
                        d.run_steps(0, tune_k)
                        d.sync()
                        if (os.environ.get("P2P_BENCH_FAIL_CANDIDATE") == "%d,%d,tuning" % (c, b)
                                and self.env.rank == n - 1):
                            raise RuntimeError("injected tuning failure")
                    except Exception as e:  # noqa: BLE001 -- same agreement as above
                        err = str(e)[:200]
                    w = time.perf_counter() - w0
                    if self.agree(err is None):
                        tuning[(c, b)] = sess.allreduce_max(w) / tune_k
                        del d
                        # Only the best communicator count so far, the headline
                        # session and the single communicator (kept for the
                        # reference-method comparison) stay open.
                        best_c = min(tuning, key=tuning.get)[0]
                        for cc in [cc for cc in sessions if cc not in (c0, 1, best_c)]:
                            if not any(cc == c2 for (c2, _) in choices[i + 1:]):
                                del sessions[cc]
                        continue
                if not droppable:
                    raise RuntimeError(err or "the first posting candidate failed on another rank")
                failed[key] = err or "failed on another rank"
                log("bench: posting candidate %s dropped: %s" % ((c, b), failed[key]))
                del d
                if c != c0 and not any(cc == c for (cc, _) in tuning):
                    sessions.pop(c, None)
            comms, batch = min(tuning, key=tuning.get)
            reason = "fastest of %d candidate(s) over %d untimed step(s) each (%s lap(s) of %d round(s)), slowest " \
                     "rank's clock" % (len(tuning), tune_k, args.tune_laps, phases)
        else:
            comms, batch = choices[0]
            reason = "single candidate" if len(choices) == 1 else "no tuning laps (--tune-laps 0): first candidate"
        sess = session_for(comms)
        # A single-communicator session stays for the reference-method comparison
        # (the reference uses one communicator); other candidates are closed.
        ref_sess = sessions.get(1)
        for c in list(sessions):
            if c not in (comms, 1):
                del sessions[c]

        # ---- the headline driver: W warmup steps, poison, K timed steps -------
        self.state["section"] = "headline"
        drv = nat.StepDriver(sess, mode, "bi", size, args.msgs, not args.no_verify, bool(batch), bool(args.graph),
                             depth=pick_depth(args.steps, phases), recv_budget=budget, salt=1)
        drv.connect()
        drv.run_steps(0, args.warmup)
        drv.sync()
        chunking = None
        if transport == "rccl" and not args.no_verify and args.warmup > 0:
            chunking = self.verify_warmup(drv, [x for x in (sess, ref_sess) if x is not None])
        drv.poison()  # untimed: every receive slot zeroed; a slot passes verification only if a timed step wrote it
        self.gpu_sync()
        drv.reset()

        self.barrier()
        self.gpu_sync()
        self.barrier()
        t0 = time.perf_counter()
        drv.run_steps(args.warmup, args.steps)
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
        my_ms = drv.step_ms()
        all_ms = [None] * n
        if n > 1:
            dist.all_gather_object(all_ms, my_ms)
        else:
            all_ms = [my_ms]
        matrix, samples, cells = cell_matrix(n, steps, drv.phase_flows, all_ms, size * args.msgs)
        offdiag = [matrix[s][d] for (s, d) in cells if s != d or n == 1]

        vr = drv.verify_steps(args.warmup, args.steps) if not args.no_verify else None
        depth, recv_bytes = drv.depth, drv.recv_bytes
        # Everything after this is untimed; release the timed driver's buffers
        # first so the comparisons run on the same memory footprint as the
        # timed steps did.
        del drv
        return types.SimpleNamespace(
            sess=sess, ref_sess=ref_sess, sessions=sessions, provenance=provenance, comms=comms, batch=batch,
            failed=failed, reason=reason, tuning=tuning, elapsed=elapsed, flows_total=flows_total, value=value,
            aggregate=aggregate, my_ms=my_ms, matrix=matrix, samples=samples, cells=cells, offdiag=offdiag,
            expected=n * (n - 1) if n > 1 else 1, vr=vr, mismatches=vr["mismatches"] if vr else -1, depth=depth,
            recv_bytes=recv_bytes, chunking=chunking)

    def verify_warmup(self, drv, sessions):
        """RCCL 2.26 delivers exactly half of a message whose share of one p2p
        channel exceeds 16 MiB, silently; the transport posts messages in ops
        under that for the channel counts it can know (transport_rccl.cpp),
        but RCCL does not report how many channels it gives a remote peer.
        So the warmup's deliveries are verified (collectively), and should
        any word be wrong every session posts its messages as smaller ops
        (16, 4, 1 MiB) and the warmup runs again, until it verifies.  Returns
        what was seen and done (posting.chunking)."""
        args = self.args
        peer = (self.env.rank + 1) % self.n
        bad = drv.verify_steps(0, args.warmup)["mismatches"]
        out = {"max_chunk_bytes": sessions[0].max_chunk(peer), "warmup_mismatches": bad, "fallback": None}
        tried = []
        for c in (16 << 20, 4 << 20, 1 << 20):
            if bad == 0:
                break
            current = sessions[0].max_chunk(peer)
            if current and c >= current:
                continue
            self.log0("bench: %d wrong words in the warmup: messages now posted as ops of <= %d MiB" % (bad, c >> 20))
            for s in sessions:
                s.set_max_chunk(c)
            drv.run_steps(0, args.warmup)
            drv.sync()
            bad = drv.verify_steps(0, args.warmup)["mismatches"]
            tried.append({"max_chunk_bytes": c, "warmup_mismatches": bad})
        if tried:
            out.update(fallback=tried, max_chunk_bytes=sessions[0].max_chunk(peer))
        return out

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

    def base_result(self) -> dict:
        """The JSON line as far as the timed steps go; the untimed sections
        fill in the rest (Reporter.update)."""
        args, h, n, nat = self.args, self.h, self.n, self.nat
        headline_transport = h.sess.transport
        vr = h.vr
        return {
            "metric": METRIC,
            "value": round(h.value, 3),
            "unit": "GB/s",
            "n_gpus": n,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(h.elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": (round(h.value / BASELINE_VALUE, 4) if BASELINE_VALUE else None),
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
            "per_gpu_gbs": round(h.aggregate / n, 3),
            "rank0_step_ms_p50": round(statistics.median(h.my_ms) if h.my_ms else 0.0, 4),
            "verify_mismatches": h.mismatches,
            "verify_coverage": (round(vr["verified_msgs"] / vr["timed_msgs"], 4) if vr and vr["timed_msgs"] else None),
            "verify_detail": vr,
            "recv_slot_generations": h.depth,
            "recv_slot_bytes_per_rank": h.recv_bytes,
            "transport": headline_transport,
            "posting": {"batch": bool(h.batch), "graph": bool(args.graph), "rccl_comms": h.comms, "chunking": h.chunking,
                        "dropped": h.failed or None, "selection": h.reason,
                        "tuning_ms_per_step": {"comms%d_%s" % (c, "batch" if b else "per_message"): round(v * 1e3, 4)
                                               for (c, b), v in h.tuning.items()} or None},
            "provenance": h.provenance,
            "reference_semantics": None,
            "extras": None,
            "ipc_transport": None,
            "xgmi_pair_sweep": None,
            "untimed_skipped": None,
            "headline_fallback": self.fallback,
            "note": ("n_gpus=1 has no inter-GPU link: value is RCCL's on-GPU self send/recv copy (HBM-bound), the "
                     "diagonal the reference prints as 0.00. From n_gpus=2 every step is one tournament round of "
                     "disjoint pairs, each pair on its own xGMI link; value is the mean per-link, per-direction cell "
                     "rate and aggregate_gbs the whole fabric")
                    if n == 1 else
                    ("each step is one tournament round: %d disjoint pairs exchange in both directions, one xGMI link "
                     "per pair; value = mean cell (per link and direction), aggregate_gbs = all pairs together"
                     % (n // 2)),
        }

    # ---- untimed sections: one deadline, waits shortened to the time left --
    def budget_left(self) -> float:
        return min(self.args.untimed_budget - (time.monotonic() - self.untimed_t0), self.deadline.left() - RESERVE_S)

    def section(self, name, fn, min_s=2.0, budgeted=True):
        """Runs one untimed section if every rank has time for it, with every
        wait of the live sessions bounded by the time left; an error is logged
        and returned in its place ({"error": ...}).  budgeted=False: only the
        deadline counts, not --untimed-budget (the headline's own latency)."""
        left = self.budget_left() if budgeted else self.deadline.left() - RESERVE_S
        if not self.agree(left > min_s):
            self.state["skipped"].append(name)
            self.log0("bench: no time left; skipping %s" % name)
            return None
        for s in self.live:
            s.set_timeout(max(1.0, min(self.args.timeout, left)))
        self.state["section"] = name
        if hang_requested(name, self.env.rank):
            log("bench: injected hang in %s on rank %d" % (name, self.env.rank))
            while True:
                time.sleep(1)
        try:
            return fn()
        except Exception as e:  # noqa: BLE001 -- reported in the JSON
            log("bench: %s failed: %s" % (name, e))
            self.state["errors"][name] = str(e)[:300]
            return {"error": str(e)[:300]}
        finally:
            self.state["section"] = None

    def latency_sections(self):
        """Host-posted ping-pong through the headline session, then the same
        pre-posted: batches of exchanges wait behind a stream gate on every
        rank and run back to back once all are posted, so those samples are
        the operation's GPU-timeline latency without the host's posting rate."""
        args, n, sess = self.args, self.n, self.h.sess
        nbytes = self.nat.parse_size(args.latency_size)

        def ping(preposted):
            m = [[0.0] * n for _ in range(n)]
            lat = json.loads(sess.latency(nbytes, args.latency_iters, min(50, args.latency_iters), preposted))
            for p in lat["pairs"]:  # a < b; the ping-pong's one-way time holds for both directions
                m[p["a"]][p["b"]] = m[p["b"]][p["a"]] = round(p["one_way_us"]["p50"], 3)
            p50s = [p["one_way_us"]["p50"] for p in lat["pairs"]]
            return {"p50": float(statistics.median(p50s)) if p50s else None, "matrix": m, "method": lat["method"]}

        r = self.section("latency", lambda: ping(0), budgeted=False)
        if isinstance(r, dict) and r.get("p50") is not None:
            self.reporter.update(p50_latency_us=round(r["p50"], 3), latency_p50_us_matrix=r["matrix"])
        if args.latency_preposted > 0:
            r = self.section("latency_preposted", lambda: ping(args.latency_preposted), budgeted=False)
            if isinstance(r, dict) and r.get("p50") is not None and r.get("method") == "preposted":
                self.reporter.update(p50_latency_preposted_us=round(r["p50"], 3),
                                     latency_preposted_p50_us_matrix=r["matrix"])

    def reference_section(self):
        """The reference's own methodology on one communicator (serial ordered
        pairs, host clock, one stream sync per message, no warmup,
        p2p_matrix.cc:141-186), at the same message size.  With one GPU the
        reference prints only the diagonal; its methodology is then applied to
        the self cell, so the ratio still compares the two methods."""
        args, n, h = self.args, self.n, self.h

        def reference_semantics():
            r = json.loads((h.ref_sess or h.sess).run(mode="pair" if n > 1 else "self", dir="uni", bytes=self.size,
                                                      iters=args.ref_iters, warmup=0, timing="wallclock",
                                                      verify=False, warm=False))
            fl = [f["gbs"] for ph in r["phases"] for f in ph["flows"] if f["src"] != f["dst"] or n == 1]
            mean = statistics.mean(fl) if fl else 0.0
            return {"cell_gbs_min": round(min(fl), 3) if fl else None, "cell_gbs_mean": round(mean, 3),
                    "iters": args.ref_iters, "size": self.size,
                    "method": "reference semantics: serial ordered pairs, wall clock, stream sync per message, no "
                              "warmup" + ("" if n > 1 else " (applied to the self cell)"),
                    # Both are per-cell rates: ours from the pipelined timed
                    # steps, the reference's from its serial cells.
                    "value_ratio": round(h.value / mean, 3) if mean > 0 else None}

        if args.ref_iters > 0:
            self.log0("bench: reference-semantics matrix")
            self.reporter.update(reference_semantics=self.section("reference_semantics", reference_semantics, 5.0))

    def extras_sections(self):
        """The other BASELINE.json configs, measured after the timed region so
        one driver run records them too: all-pairs concurrent exchange at 1 GiB
        (bisection: every GPU drives all N-1 xGMI links at once), the ring
        neighbour exchange at 256 MiB, the pipeline-parallel hop latency as a
        dependent token chain 0 -> 1 -> ... -> N-1 -> 0, and the single-pair
        (0 -> 1) bandwidth sweep 4 KiB -> 4 GiB (config 2; only cell (0, 1) is
        scheduled, the other ranks just join the barriers)."""
        args, n, nat, h = self.args, self.n, self.nat, self.h
        if n == 1:
            return

        def concurrent_config(mode_x, dir_x, nbytes, iters):
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
            r = json.loads(session.run(mode="pair", dir="uni", bytes=nbytes, iters=iters, warmup=2, timing="events",
                                       verify=not args.no_verify, warm=False, cells=[(0, 1)]))
            fl = [f for ph in r["phases"] for f in ph["flows"]]
            return fl[0] if fl else None

        def pair_sweep():
            sweep = []
            for nbytes in [b for b in (4096 << (2 * k) for k in range(11)) if b <= nat.parse_size(args.sweep_max)]:
                self.log0("bench: pair sweep %d B" % nbytes)
                iters = max(4, min(200, (2 << 30) // nbytes))
                f = pair_cell(h.sess, nbytes, iters)
                if f:
                    sweep.append({"bytes": nbytes, "iters": iters, "gbs": round(f["gbs"], 2),
                                  "iter_us_p50": round(f["iter_us"]["p50"], 2), "mismatches": f.get("mismatches", -1)})
            return sweep

        def pair_one_comm():
            # The same single pair on one communicator (what the sweep ran with
            # K of them), at the bench's message size and 256 MiB.
            return [{"bytes": nb, "gbs": round(f["gbs"], 2)}
                    for nb in (self.size, 256 << 20) for f in [pair_cell(h.ref_sess, nb, 16)] if f]

        extras = None
        if args.extras:
            self.log0("bench: all-pairs / ring extras")
            extras = {}
            # Keyed by the BASELINE config names; the sizes can be lowered for
            # CPU rehearsals (all-pairs holds N - 1 receive slots per rank).
            for name, mode_x, dir_x, nbytes, iters in (
                    ("allpairs_1g", "allpairs", "bi", nat.parse_size(args.allpairs_size), 4),
                    ("ring_256m", "ring", "uni", nat.parse_size(args.ring_size), 8)):
                v = self.section(name, lambda: concurrent_config(mode_x, dir_x, nbytes, iters), 5.0)
                if v is not None:
                    extras[name] = v
            v = self.section("ring_hop", ring_hop)
            if v is not None:
                extras["ring_hop"] = v
            self.reporter.update(extras=extras)
        if args.sweep:
            sw = self.section("pair_sweep_0_1", pair_sweep, 10.0)
            if sw is not None:
                extras = dict(extras or {}, pair_sweep_0_1=sw, pair_sweep_rccl_comms=h.comms)
                if h.ref_sess is not None and h.ref_sess is not h.sess:
                    oc = self.section("pair_0_1_one_comm", pair_one_comm)
                    if oc is not None:
                        extras["pair_0_1_one_comm"] = oc
            self.reporter.update(extras=extras)

    def isolated(self, transport):
        """steps_through() for `transport` in a child process per rank.  The
        comparisons drive the hand-written data plane (hipIpc mappings, signal
        kernels, relays) across GPUs; if one of them faults or hangs on some
        node, only the child dies, and the headline line still gets printed
        with the error in its place."""
        args, n, rank = self.args, self.n, self.env.rank
        box = [free_port() if rank == 0 else None]
        if n > 1:
            dist.broadcast_object_list(box, src=0)
        out_path = os.path.join(tempfile.gettempdir(), "p2p_bench_child_%d_%d.json" % (box[0], rank))
        limit = min(args.child_timeout, max(5.0, self.budget_left()))
        cmd = [sys.executable, os.path.abspath(__file__), "--gpus", str(n), "--steps", str(args.steps),
               "--warmup", str(args.warmup), "--size", args.size, "--msgs", str(args.msgs), "--mode", self.mode,
               "--latency-iters", str(args.latency_iters), "--latency-size", args.latency_size,
               "--child", transport, "--child-port", str(box[0]), "--child-out", out_path,
               "--child-batch", str(int(self.h.batch)), "--timeout", str(max(5.0, min(args.timeout, limit)))]
        if args.no_verify:
            cmd.append("--no-verify")
        if args.device is not None:
            cmd += ["--device", str(args.device)]
        rc = run_child(self.state, cmd, limit)
        self.barrier()
        res = None
        if rank == 0:
            try:
                with open(out_path) as f:
                    res = json.load(f)
            except (OSError, ValueError):
                res = {"error": "comparison process failed (exit status %s)" % rc, "transport": transport}
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
            if args.isolate:
                return self.isolated(transport)
            isess = self.create_session(transport, device=self.device,
                                        timeout_s=min(90.0, max(5.0, self.budget_left())))
            try:
                return steps_through(self.nat, isess, args, self.mode, self.size, batch, transport)
            finally:
                del isess

        ipc = None
        for transport, key in runs:
            self.log0("bench: %s comparison" % transport)
            r = self.section(transport, lambda: compare(transport), 20.0)
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

        r = self.section("xgmi_pair_sweep", sweep, 30.0)
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

    def run(self) -> int:
        rc = self.headline()
        if rc is not None:
            return rc
        h = self.h
        self.reporter.result = self.base_result()
        self.log0("bench: value %.2f GB/s per cell (aggregate %.2f GB/s), %.4f ms/step, verify %s" % (
            h.value, h.aggregate, h.elapsed / self.args.steps * 1e3, h.vr))

        self.untimed_t0 = time.monotonic()
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

        self.reporter.update(untimed_skipped=self.state["skipped"] or None,
                             section_errors=self.state["errors"] or None)
        if self.env.rank == 0:
            log("bench: GB/s matrix (row=src, col=dst), median over steps:")
            for r in range(self.n):
                log("  " + " ".join("%8.2f" % h.matrix[r][c] for c in range(self.n)))
        self.reporter.emit()
        # The watchdog stays armed: should the teardown below hang, it ends the
        # process at the deadline (the line is out already, so it exits 0).
        self.barrier()
        if self.n > 1 and dist.is_initialized():
            dist.destroy_process_group()
        return 0 if h.mismatches in (0, -1) else 3


def main(argv=None) -> int:
    args = parse_args(argv)
    if args.child:
        return child_main(args)
    return BenchRun(args, claim_stdout()).run()


if __name__ == "__main__":
    sys.exit(main())

#!/usr/bin/env python3
"""Headline benchmark: pairwise P2P GB/s matrix (min/mean) + p50 latency.

Metric and configs come from BASELINE.json ("pairwise P2P GB/s matrix
(min/mean) + p50 latency at 1/2/4/8 MI355X").  The reference
(/root/reference/p2p_matrix.cc) measures an N x N matrix of NCCL send/recv
bandwidth at 32 MiB per message; this bench measures the same matrix on
MI355X through the native engine (RCCL ncclSend/ncclRecv over xGMI, hipEvent
timing, gfx950 fill/verify kernels).

One step = one round of the round-robin "tournament" schedule: the N ranks
form N/2 disjoint pairs (xGMI is fully connected point-to-point, so pairs never
share a link) and every pair exchanges --msgs messages of --size bytes in both
directions, posted back to back inside ncclGroupStart/End.  Consecutive steps
walk through the N-1 rounds, so after N-1 steps every cell of the matrix has
been measured; per-GPU work per step is constant as N grows (weak scaling).
With one GPU the step is a self send/recv (the reference prints only the
diagonal 0.00 there).

value = bytes sent by all ranks during the K timed steps / the slowest rank's
wall time between two barrier + torch.cuda.synchronize() brackets, in GB/s
(1e9 B/s).  Payloads are PRNG-filled on the device and the last step's receive
buffers are verified on the device after the timed region.

Usage (driver contract):
  python bench.py --gpus 1 --steps K --warmup W
  python -m torch.distributed.run --nnodes=1 --nproc-per-node N \
      --master-addr 127.0.0.1 --master-port P bench.py --gpus N --steps K --warmup W
"""

from __future__ import annotations

import argparse
import json
import os
import socket
import statistics
import subprocess
import sys
import tempfile
import time

import torch
import torch.distributed as dist

METRIC = "pairwise P2P GB/s matrix (min/mean) + p50 latency at 1/2/4/8 MI355X"
BASELINE_VALUE = None  # the reference publishes no numbers


def log(*a):
    print(*a, file=sys.stderr, flush=True)


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
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def first_comms(transport: str, comms: int) -> int:
    """Communicators of the session bench.py opens first (the headline one)."""
    return comms if transport == "rccl" and comms > 0 else 1


def posting_candidates(transport: str, comms: int, batch: int, warmup: int):
    """(communicators, batch) pairs the warmup steps time against each other.

    comms: > 0 fixed, -1 = RCCL picks between 1 and 4 (other transports: 1).
    batch: 1 one group per step, 0 one group per message, -1 = both (K = 1
    only: with several communicators per-message groups cannot overlap).
    With fewer warmup steps than candidates only the last one is kept."""
    comms_choices = ([comms] if comms > 0 else [1, 4]) if transport == "rccl" else [1]
    batch_choices = [batch] if batch >= 0 or warmup < 2 else [0, 1]
    if batch_choices == [-1]:
        batch_choices = [1]
    choices = [(c, b) for c in comms_choices for b in batch_choices if c == 1 or b == 1 or len(batch_choices) == 1]
    if warmup < len(choices):
        choices = choices[-1:]
    return choices


def steps_through(nat, isess, args, mode, size, batch, transport):
    """The timed steps again through another transport session (untimed by
    the contract); any error is reported instead of failing the run."""
    try:
        idrv = nat.StepDriver(isess, mode, "bi", size, args.msgs, not args.no_verify, bool(batch), False)
        idrv.connect()
        idrv.run_steps(0, args.warmup)
        idrv.sync()
        isess.barrier()
        i0 = time.perf_counter()
        idrv.run_steps(args.warmup, args.steps)
        idrv.sync()
        isess.barrier()
        ielapsed = isess.allreduce_max(time.perf_counter() - i0)
        ijob = sum(idrv.job_bytes_per_step(args.warmup + k) for k in range(args.steps))
        out = {"value_gbs": round(ijob / ielapsed / 1e9, 3), "ms_per_step": round(ielapsed / args.steps * 1e3, 4),
               "verify_mismatches": idrv.verify_last() if not args.no_verify else -1,
               "transport": transport}
        del idrv
        # Device-initiated ping-pong: one wave per GPU writes the message
        # into the peer's memory and spins on its own inbox (no host, no
        # runtime in the loop) -- the fabric's latency, next to RCCL's.
        if transport == "ipc":
            dl = json.loads(isess.device_latency(nat.parse_size(args.latency_size), args.latency_iters,
                                                 min(100, args.latency_iters)))
            out["device_pingpong_p50_us"] = round(statistics.median(p["one_way_us"]["p50"] for p in dl["pairs"]), 3)
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
    claim_stdout()
    from test_nccl_p2p_amd import require_native
    from test_nccl_p2p_amd.parallel.session import dist_env

    nat = require_native()
    env = dist_env()
    device = env.local_rank if args.device is None else args.device
    size = nat.parse_size(args.size)
    try:
        sess = nat.Session(env.rank, env.world, host=env.master_addr, port=args.child_port, device=device,
                           transport=args.child, timeout_s=90.0)
        out = steps_through(nat, sess, args, args.mode, size, args.child_batch, args.child)
        del sess
    except Exception as e:
        out = {"error": str(e)[:300], "transport": args.child}
    if env.rank == 0:
        with open(args.child_out, "w") as f:
            json.dump(out, f)
    return 0


def parse_args(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=28)
    ap.add_argument("--warmup", type=int, default=7)
    ap.add_argument("--size", default="32M", help="message size (reference: 32 MiB, p2p_matrix.cc:124)")
    ap.add_argument("--msgs", type=int, default=8, help="messages per direction per step")
    ap.add_argument("--mode", default="tournament", choices=["tournament", "ring", "allpairs", "pair", "self"])
    ap.add_argument("--transport", default="rccl", choices=["rccl", "ipc", "ipc:sdma", "ipc:push", "ipc:relay", "host", "shm"],
                    help="rccl (headline) | ipc = one-sided gfx950 copy kernel over hipIpc mappings | host = CPU (tests)")
    ap.add_argument("--comms", type=int, default=-1,
                    help="rccl: communicators per rank; the messages of a step are spread over them and their "
                         "send/recv kernels run side by side (-1: the warmup picks 1 or 4)")
    ap.add_argument("--device", type=int, default=None, help="GPU index (default LOCAL_RANK)")
    ap.add_argument("--latency-iters", type=int, default=300)
    ap.add_argument("--latency-size", default="8")
    ap.add_argument("--no-verify", action="store_true")
    ap.add_argument("--batch", type=int, default=-1,
                    help="1: all msgs of a step in one group (one launch); 0: one group per message; "
                         "-1: the W warmup steps are split between both and the faster posting is timed")
    ap.add_argument("--graph", type=int, default=0, help="1: replay each step as a captured hipGraph")
    ap.add_argument("--json-out", default=None, help="also write the result line to this file")
    ap.add_argument("--ipc-extra", type=int, default=1,
                    help="1: also run the tournament steps through the IPC transport (N > 1, after the timed region)")
    ap.add_argument("--extras", type=int, default=1,
                    help="1: also measure all-pairs 1 GiB and ring 256 MiB after the timed region (N > 1)")
    ap.add_argument("--sweep", type=int, default=1,
                    help="1: also sweep the single pair 0 -> 1 over 4 KiB .. --sweep-max (N > 1, after the timed region)")
    ap.add_argument("--sweep-max", default="4G", help="largest message of the pair sweep")
    ap.add_argument("--ref-iters", type=int, default=128,
                    help="iterations per cell of the reference-methodology comparison (0 = skip)")
    ap.add_argument("--isolate", type=int, default=1,
                    help="1: run each untimed transport comparison in a child process per rank (a fault there "
                         "cannot take the headline down); 0: in this process (halves the processes per GPU)")
    ap.add_argument("--timeout", type=float, default=120.0,
                    help="seconds any one wait of the headline session may take before it aborts and fails")
    ap.add_argument("--untimed-budget", type=float, default=480.0,
                    help="seconds for all untimed sections after the timed steps; later ones are skipped")
    ap.add_argument("--child-timeout", type=float, default=300.0,
                    help="seconds allowed to each untimed comparison process")
    ap.add_argument("--child", default=None, help=argparse.SUPPRESS)
    ap.add_argument("--child-port", type=int, default=0, help=argparse.SUPPRESS)
    ap.add_argument("--child-out", default=None, help=argparse.SUPPRESS)
    ap.add_argument("--child-batch", type=int, default=1, help=argparse.SUPPRESS)
    return ap.parse_args(argv)


def main(argv=None) -> int:
    args = parse_args(argv)
    if args.child:
        return child_main(args)
    real_stdout = claim_stdout()
    from test_nccl_p2p_amd import require_native
    from test_nccl_p2p_amd.parallel.session import create_session, init_control_plane

    nat = require_native()
    env = init_control_plane("gloo")
    if args.gpus != env.world:
        log("bench: --gpus %d but WORLD_SIZE=%d; using WORLD_SIZE" % (args.gpus, env.world))
    n = env.world
    use_gpu = args.transport not in ("host", "shm")
    device = env.local_rank if args.device is None else args.device
    if use_gpu:
        torch.cuda.set_device(device)

    def barrier():
        if n > 1:
            dist.barrier()

    def gpu_sync():
        if use_gpu:
            torch.cuda.synchronize()

    size = nat.parse_size(args.size)
    headline = args.transport + (":%d" % args.comms if args.transport == "rccl" and args.comms > 1 else "")
    sess = create_session(headline, device=device, timeout_s=args.timeout)
    if env.rank == 0:
        log("bench: %d rank(s), %s, %s" % (n, sess.transport, sess.device_desc))
    mode = "self" if n == 1 else args.mode

    # Warmup (untimed, W steps in total) also picks the posting: one group
    # per step vs one group per message, and (RCCL) one communicator vs
    # several whose send/recv kernels run side by side.  The W steps are
    # split between the candidates and the fastest, by the slowest rank's
    # clock, is timed.  connect() has already established every connection
    # of every round.
    choices = posting_candidates(args.transport, args.comms, args.batch, args.warmup)
    sessions = {first_comms(args.transport, args.comms): sess}

    def session_for(c):
        if c not in sessions:
            # A candidate that stalls is aborted and dropped after --timeout.
            sessions[c] = create_session("rccl:%d" % c if c > 1 else "rccl", device=device, timeout_s=args.timeout)
        return sessions[c]

    def agree(ok: bool) -> bool:
        """True when every rank reports ok (the candidates are collective)."""
        if n == 1:
            return ok
        t = torch.tensor([1 if ok else 0], dtype=torch.int32)
        dist.all_reduce(t, op=dist.ReduceOp.MIN)
        return bool(t.item())

    tuning = {}
    drivers = {}
    failed = {}
    done = 0
    for i, (c, b) in enumerate(choices):
        # A candidate other than the first that fails anywhere (e.g. a second
        # RCCL communicator on a node where it was never tried) is dropped on
        # every rank instead of ending the run.
        d, err = None, None
        try:
            d = nat.StepDriver(session_for(c), mode, "bi", size, args.msgs, not args.no_verify, bool(b),
                               bool(args.graph))
            d.connect()
            # Test hook: P2P_BENCH_FAIL_CANDIDATE="<comms>,<batch>" fails that
            # candidate on the last rank only.
            if os.environ.get("P2P_BENCH_FAIL_CANDIDATE") == "%d,%d" % (c, b) and env.rank == n - 1:
                raise RuntimeError("injected candidate failure")
        except Exception as e:  # noqa: BLE001 -- reported, and the candidate is skipped everywhere
            err = str(e)[:200]
        # The headline session's first candidate must work; anything else
        # (another communicator count, another posting) may be dropped.
        droppable = (c, b) != choices[0] or c != first_comms(args.transport, args.comms)
        if droppable and not agree(err is None):
            failed["comms%d_%s" % (c, "batch" if b else "per_message")] = err or "failed on another rank"
            log("bench: posting candidate %s dropped: %s" % ((c, b), err or "failed on another rank"))
            d = None
            if c != first_comms(args.transport, args.comms):
                sessions.pop(c, None)
            continue
        if err is not None:
            raise RuntimeError(err)
        k = (args.warmup - done) // (len(choices) - i)
        if k > 0:
            barrier()
            w0 = time.perf_counter()
            try:
                d.run_steps(done, k)
                d.sync()
                # Test hook: "<comms>,<batch>,warmup" fails it here instead.
                if os.environ.get("P2P_BENCH_FAIL_CANDIDATE") == "%d,%d,warmup" % (c, b) and env.rank == n - 1:
                    raise RuntimeError("injected warmup failure")
            except Exception as e:  # noqa: BLE001 -- same agreement as above
                err = str(e)[:200]
            if not agree(err is None):
                if not droppable:
                    raise RuntimeError(err or "warmup failed on another rank")
                failed["comms%d_%s" % (c, "batch" if b else "per_message")] = err or "failed on another rank"
                log("bench: posting candidate %s dropped in warmup: %s" % ((c, b), err or "failed on another rank"))
                d = None
                if c != first_comms(args.transport, args.comms):
                    sessions.pop(c, None)
                continue
            barrier()
            tuning[(c, b)] = sessions[c].allreduce_max(time.perf_counter() - w0) / k
            done += k
        drivers[(c, b)] = d
    if not drivers:  # every candidate was dropped: the headline session, one group per step
        c0 = first_comms(args.transport, args.comms)
        d = nat.StepDriver(sessions[c0], mode, "bi", size, args.msgs, not args.no_verify, True, bool(args.graph))
        d.connect()
        drivers[(c0, 1)] = d
    comms, batch = (min(tuning, key=tuning.get) if len(tuning) == len(drivers) and tuning
                    else list(drivers)[-1])
    drv = drivers.pop((comms, batch))
    del drivers, d  # the other postings' buffers go before the timed region
    sess = sessions[comms]
    # A single-communicator session stays for the reference-method comparison
    # (the reference uses one communicator); other candidates are closed.
    ref_sess = sessions.get(1)
    for c in list(sessions):
        if c not in (comms, 1):
            del sessions[c]
    gpu_sync()
    drv.reset()

    barrier()
    gpu_sync()
    barrier()
    t0 = time.perf_counter()
    drv.run_steps(args.warmup, args.steps)
    drv.sync()
    gpu_sync()
    barrier()
    t1 = time.perf_counter()
    elapsed = sess.allreduce_max(t1 - t0)

    job_bytes = sum(drv.job_bytes_per_step(args.warmup + k) for k in range(args.steps))
    value = job_bytes / elapsed / 1e9

    # Per-step GPU durations of every rank -> per-flow bandwidth.  The later
    # arriving endpoint of a pair sees only the transfer (the earlier one also
    # waits), so a flow's time is the min of its two endpoints' step times.
    my_ms = drv.step_ms()
    all_ms = [None] * n
    if n > 1:
        dist.all_gather_object(all_ms, my_ms)
    else:
        all_ms = [my_ms]
    cells = {}
    for k in range(args.steps):
        step = args.warmup + k
        for (src, dst) in drv.phase_flows(step):
            ms = min(all_ms[src][k], all_ms[dst][k]) if src != dst else all_ms[src][k]
            if ms > 0:
                cells.setdefault((src, dst), []).append(size * args.msgs / (ms * 1e-3) / 1e9)
    matrix = [[0.0] * n for _ in range(n)]
    for (s, d), v in cells.items():
        matrix[s][d] = statistics.median(v)
    offdiag = [v for (s, d), vs in cells.items() for v in [statistics.median(vs)] if s != d or n == 1]
    covered = len(cells)
    expected = n * (n - 1) if n > 1 else 1

    mismatches = drv.verify_last() if not args.no_verify else -1
    # Everything below is untimed; release the timed driver's buffers first so
    # the comparisons run on the same memory footprint as the timed steps did.
    del drv

    # The untimed sections share one time budget (--untimed-budget): each
    # starts only if every rank still has time left, so a section that stalls
    # until its session's --timeout cannot push the JSON line past a driver's
    # limit.  Skipped sections are listed in the JSON.
    untimed_t0 = time.perf_counter()
    skipped = []

    def budget_left():
        return args.untimed_budget - (time.perf_counter() - untimed_t0)

    def in_budget(name):
        if agree(budget_left() > 0):
            return True
        skipped.append(name)
        if env.rank == 0:
            log("bench: untimed budget spent; skipping %s" % name)
        return False

    def guarded(name, fn):
        """Runs one untimed measurement; an error is logged and returned in
        its place ({"error": ...}), so the headline line is still printed.
        (The RCCL transport bounds every wait, so a failure on one rank
        surfaces on the others as an error too, not as a hang.)"""
        try:
            return fn()
        except Exception as e:  # noqa: BLE001 -- reported in the JSON
            log("bench: %s failed: %s" % (name, e))
            return {"error": str(e)[:300]}

    lat_matrix = [[0.0] * n for _ in range(n)]

    def latency():
        lat = json.loads(sess.latency(nat.parse_size(args.latency_size), args.latency_iters,
                                      min(50, args.latency_iters)))
        for p in lat["pairs"]:  # a < b; the ping-pong's one-way time holds for both directions
            lat_matrix[p["a"]][p["b"]] = lat_matrix[p["b"]][p["a"]] = round(p["one_way_us"]["p50"], 3)
        p50s = [p["one_way_us"]["p50"] for p in lat["pairs"]]
        return statistics.median(p50s) if p50s else None

    p50 = guarded("latency", latency)
    if isinstance(p50, dict):  # the error is in the log; the field stays null
        p50 = None

    # The reference's own methodology on one communicator, for comparison
    # (serial ordered pairs, host clock, one stream sync per message,
    # p2p_matrix.cc:141-186), at the same message size.  Untimed by the
    # driver's bracket; skipped on one GPU where the reference measures nothing.
    def reference_semantics():
        r = json.loads((ref_sess or sess).run(mode="pair", dir="uni", bytes=size, iters=args.ref_iters, warmup=0,
                                              timing="wallclock", verify=False, warm=False))
        return {"cell_gbs_min": round(r["gbs_min"], 3), "cell_gbs_mean": round(r["gbs_mean"], 3),
                "iters": args.ref_iters, "size": size,
                "method": "reference semantics: serial ordered pairs, wall clock, stream sync per message",
                # The reference moves one cell at a time, so its matrix-wide
                # throughput is its cell rate; ours is `value`.
                "value_ratio": round(value / r["gbs_mean"], 3) if r["gbs_mean"] > 0 else None}

    ref = None
    if n > 1 and args.ref_iters > 0 and in_budget("reference_semantics"):
        if env.rank == 0:
            log("bench: reference-semantics matrix")
        ref = guarded("reference semantics", reference_semantics)

    # The other BASELINE.json configs, measured after the timed region so one
    # driver run records them too: all-pairs concurrent exchange at 1 GiB
    # (bisection: every GPU drives all N-1 xGMI links at once) and the ring
    # neighbour exchange at 256 MiB (pipeline-parallel hop).
    def concurrent_config(mode_x, dir_x, nbytes, iters):
        r = json.loads(sess.run(mode=mode_x, dir=dir_x, bytes=nbytes, iters=iters, warmup=1, timing="events",
                                verify=False, warm=True))
        ph = r["phases"][0]
        flows = [f["gbs"] for f in ph["flows"]]
        p50s = [f["iter_us"]["p50"] for f in ph["flows"]]
        return {"aggregate_gbs": round(ph["agg_gbs"], 2), "per_gpu_egress_gbs": round(ph["agg_gbs"] / n, 2),
                "flow_gbs_min": round(min(flows), 2), "flow_gbs_mean": round(statistics.mean(flows), 2),
                "iter_us_p50": round(statistics.median(p50s), 1), "bytes": nbytes, "iters": iters}

    extras = None
    if n > 1 and args.extras:
        if env.rank == 0:
            log("bench: all-pairs / ring extras")
        extras = {}
        # ring_hop_8b: the pipeline-parallel hop latency -- every rank sends
        # 8 bytes to its successor each iteration; iter_us_p50 is the hop time.
        for name, mode_x, dir_x, nbytes, iters in (("allpairs_1g", "allpairs", "bi", 1 << 30, 4),
                                                   ("ring_256m", "ring", "uni", 256 << 20, 8),
                                                   ("ring_hop_8b", "ring", "uni", 8, 200)):
            if in_budget(name):
                extras[name] = guarded(name, lambda: concurrent_config(mode_x, dir_x, nbytes, iters))

    # BASELINE.json config 2: single-pair (0 -> 1) send/recv bandwidth sweep,
    # 4 KiB -> 4 GiB in x4 steps, events-timed, uni-directional; only cell
    # (0, 1) is scheduled, so the other ranks just join the barriers.
    def pair_cell(session, nbytes, iters):
        r = json.loads(session.run(mode="pair", dir="uni", bytes=nbytes, iters=iters, warmup=2, timing="events",
                                   verify=False, warm=False, cells=[(0, 1)]))
        fl = [f for ph in r["phases"] for f in ph["flows"]]
        return fl[0] if fl else None

    def pair_sweep():
        sweep = []
        for nbytes in [b for b in (4096 << (2 * k) for k in range(11)) if b <= nat.parse_size(args.sweep_max)]:
            if env.rank == 0:
                log("bench: pair sweep %d B" % nbytes)
            iters = max(4, min(200, (2 << 30) // nbytes))
            f = pair_cell(sess, nbytes, iters)
            if f:
                sweep.append({"bytes": nbytes, "iters": iters, "gbs": round(f["gbs"], 2),
                              "iter_us_p50": round(f["iter_us"]["p50"], 2)})
        return sweep

    def pair_one_comm():
        # The same single pair on one communicator (what the sweep ran with K
        # of them), at the bench's message size and 256 MiB.
        return [{"bytes": nb, "gbs": round(f["gbs"], 2)}
                for nb in (size, 256 << 20) for f in [pair_cell(ref_sess, nb, 16)] if f]

    if n > 1 and args.sweep and in_budget("pair_sweep_0_1"):
        extras = dict(extras or {}, pair_sweep_0_1=guarded("pair sweep", pair_sweep), pair_sweep_rccl_comms=comms)
        if ref_sess is not None and ref_sess is not sess and in_budget("pair_0_1_one_comm"):
            extras["pair_0_1_one_comm"] = guarded("one-communicator pair", pair_one_comm)

    # The same tournament steps through the hand-written data plane (IPC
    # transport: one-sided pulls of hipIpc-mapped peer buffers by the gfx950
    # copy kernel) on the same links, for comparison with RCCL.  Untimed by the
    # contract; any error is reported in the JSON instead of failing the run.
    # The comparisons below open sessions of their own; close the headline one
    # first so they run alone, as the timed steps did.
    headline_transport = sess.transport
    del sess, ref_sess, sessions

    # (with --transport host the same code path runs on the CPU transport, for tests)
    extra_transport = {"rccl": "ipc", "ipc": "ipc", "ipc:push": "ipc", "ipc:relay": "ipc", "host": "host",
                       "shm": "host"}.get(args.transport)

    def isolated(transport):
        """steps_through() for `transport` in a child process per rank.  The
        comparisons drive the hand-written data plane (hipIpc mappings,
        signal kernels, relays) across GPUs; if one of them faults or hangs
        on some node, only the child dies, and the headline line still gets
        printed with the error in its place."""
        box = [free_port() if env.rank == 0 else None]
        if n > 1:
            dist.broadcast_object_list(box, src=0)
        out_path = os.path.join(tempfile.gettempdir(), "p2p_bench_child_%d_%d.json" % (box[0], env.rank))
        cmd = [sys.executable, os.path.abspath(__file__), "--gpus", str(n), "--steps", str(args.steps),
               "--warmup", str(args.warmup), "--size", args.size, "--msgs", str(args.msgs), "--mode", mode,
               "--latency-iters", str(args.latency_iters), "--latency-size", args.latency_size,
               "--child", transport, "--child-port", str(box[0]), "--child-out", out_path,
               "--child-batch", str(int(batch))]
        if args.no_verify:
            cmd.append("--no-verify")
        if args.device is not None:
            cmd += ["--device", str(args.device)]
        try:
            rc = subprocess.run(cmd, timeout=min(args.child_timeout, max(30.0, budget_left()))).returncode
        except subprocess.TimeoutExpired:
            rc = "timeout"
        barrier()
        res = None
        if env.rank == 0:
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

    # The hand-written data plane on the same links: the gfx950 multi-copy
    # kernel pulling from hipIpc-mapped peer buffers ("pull", one-sided), the
    # rendezvous engine that writes into the receiver's slot ("push"), the
    # SDMA copy engines pulling instead of CUs ("sdma"), and multi-path push
    # with two-hop relays through GPUs whose links are idle ("relay").
    ipc = None
    if n > 1 and args.ipc_extra and extra_transport:
        runs = [(extra_transport, None)]
        if extra_transport == "ipc":
            runs += [("ipc:push", "push"), ("ipc:sdma", "sdma")] + ([("ipc:relay", "relay")] if n > 2 else [])
        engines = {"ipc": "gfx950 multi-copy kernel, one-sided pull over hipIpc mappings",
                   "ipc:push": "ready/done flags + gfx950 multi-copy kernel writing into the peer's slot",
                   "ipc:sdma": "one-sided pull by the SDMA copy engines (hipMemcpyAsync per receive)",
                   "ipc:relay": "push over the direct link + two-hop stripes relayed through GPUs whose links are "
                                "idle (routing.hpp)"}
        for transport, key in runs:
            if not in_budget(transport):
                continue
            if env.rank == 0:
                log("bench: %s comparison" % transport)
            if args.isolate:
                r = isolated(transport)
            else:
                try:
                    isess = create_session(transport, device=device, timeout_s=90.0)
                    r = steps_through(nat, isess, args, mode, size, batch, transport)
                    del isess
                except Exception as e:  # report, never fail the headline
                    r = {"error": str(e)[:300], "transport": transport}
            if env.rank != 0:
                continue
            if transport in engines:
                r["engine"] = engines[transport]
            if key is None:
                ipc = r
            else:
                ipc[key] = r

    step_ms_med = statistics.median(my_ms) if my_ms else 0.0
    result = {
        "metric": METRIC,
        "value": round(value, 3),
        "unit": "GB/s",
        "n_gpus": n,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": (round(value / BASELINE_VALUE, 4) if BASELINE_VALUE else None),
        "dtype": "uint8",
        "data": "synthetic (device PRNG-filled payloads, verified after timing)",
        "config": {
            "model": "p2p_matrix: %s %s-bidirectional, %s x %d msgs/step"
                     % ("RCCL ncclSend/ncclRecv" if headline_transport == "rccl" else headline_transport + " transport",
                        mode, nat.format_size(size), args.msgs),
            "global_batch": args.msgs * n,
            "seq_len": size,
            "parallelism": "p2p%d" % n,
        },
        "matrix_gbs_min": round(min(offdiag), 3) if offdiag else None,
        "matrix_gbs_mean": round(statistics.mean(offdiag), 3) if offdiag else None,
        "matrix_cells": "%d/%d" % (covered, expected),
        # BASELINE config 3: the full N x N pairwise matrices (row = sender;
        # GB/s per direction, median over steps; p50 one-way latency, us).
        "matrix_gbs": [[round(v, 2) for v in row] for row in matrix],
        "latency_p50_us_matrix": lat_matrix,
        "p50_latency_us": round(p50, 3) if p50 is not None else None,
        "latency_bytes": nat.parse_size(args.latency_size),
        "per_gpu_gbs": round(value / n, 3),
        "rank0_step_ms_p50": round(step_ms_med, 4),
        "verify_mismatches": mismatches,
        "transport": headline_transport,
        "posting": {"batch": bool(batch), "graph": bool(args.graph), "rccl_comms": comms, "dropped": failed or None,
                    "warmup_ms_per_step": {"comms%d_%s" % (c, "batch" if b else "per_message"): round(v * 1e3, 4)
                                           for (c, b), v in tuning.items()}},
        "reference_semantics": ref,
        "extras": extras,
        "ipc_transport": ipc,
        "untimed_skipped": skipped or None,
        "note": ("n_gpus=1 has no inter-GPU link: value is RCCL's on-GPU self send/recv copy (HBM-bound). "
                 "From n_gpus=2 every step is one tournament round of disjoint pairs, each pair on its own xGMI "
                 "link, so value grows with the number of pairs (per-GPU rate = one link's bandwidth)")
                if n == 1 else
                ("each step is one tournament round: %d disjoint pairs exchange in both directions, one xGMI link "
                 "per pair; value = all pairs together" % (n // 2)),
    }
    if env.rank == 0:
        log("bench: GB/s matrix (row=src, col=dst), median over steps:")
        for r in range(n):
            log("  " + " ".join("%8.2f" % matrix[r][c] for c in range(n)))
        line = json.dumps(result)
        os.write(real_stdout, (line + "\n").encode())
        if args.json_out:
            with open(args.json_out, "w") as f:
                f.write(line + "\n")
    barrier()
    if n > 1 and dist.is_initialized():
        dist.destroy_process_group()
    return 0 if mismatches in (0, -1) else 3


if __name__ == "__main__":
    sys.exit(main())

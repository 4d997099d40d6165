"""The timed steps again through another transport (the untimed IPC
comparisons of bench.py), in this process or as a child job per rank."""

from __future__ import annotations

import json
import os
import statistics
import time

from test_nccl_p2p_amd.bench.core import (claim_stdout, combine_runs, default_device, headline_stats, log,
                                          pair_matrix_summary, pick_depth)

REF_STOCK = "ref-stock"  # --child: the reference's methodology with RCCL's and HIP's stock settings


def stock_env(environ=None) -> dict:
    """The environment for reference_semantics_stock: what bench.py found at
    start for the queue count, RCCL's unroll factor and its log (P2P_STOCK_ENV),
    RCCL's own unroll (P2P_RCCL_UNROLL=0) and no private INFO log
    (P2P_RCCL_LOG=0), so the child runs the kernels, queues and logging the
    reference's stock NCCL setup would."""
    env = dict(os.environ if environ is None else environ)
    orig = json.loads(env.get("P2P_STOCK_ENV") or "{}")
    for k, v in orig.items():
        if v is None:
            env.pop(k, None)
        else:
            env[k] = v
    env.update(P2P_RCCL_UNROLL="0", P2P_RCCL_LOG="0")
    return env


def reference_stock(nat, sess, args, dirs, iters, runs=None) -> dict:
    """--child ref-stock: the pair (self at N = 1) matrices by the reference's
    methodology -- one communicator, host clock, a stream sync per message, no
    warmup, no connection warm-up (p2p_matrix.cc:141-267) -- per direction
    mode, `iters[d]` iterations per cell and `runs[d]` runs (those of
    reference_semantics), combined as there (combine_runs)."""
    n = sess.world
    out = {}
    for d in dirs:
        rs = []
        for _ in range(max(1, int((runs or {}).get(d, 1)))):
            r = json.loads(sess.run(mode="pair" if n > 1 else "self", dir=d, bytes=nat.parse_size(args.size),
                                    iters=int(iters[d]), warmup=0, timing="wallclock", verify=False, warm=False))
            rs.append(pair_matrix_summary(r, n))
        out[d] = dict(combine_runs(rs, n), iters=int(iters[d]))
    out["env"] = {k: os.environ.get(k) for k in ("GPU_MAX_HW_QUEUES", "RCCL_UNROLL_FACTOR", "NCCL_DEBUG",
                                                 "P2P_RCCL_UNROLL", "P2P_RCCL_LOG")}
    return out


def steps_through(nat, isess, args, mode, size, batch, transport, recv_budget=0):
    """The timed steps again through another transport session (untimed by
    the contract); any error is reported (and logged by rank 0) instead of
    failing the run.  recv_budget: receive-slot bytes this rank may allocate
    (0: a quarter of the free memory, which ranks sharing a GPU must not use)."""
    say = (lambda m: log("bench: %s: %s" % (transport, m))) if isess.rank == 0 else (lambda m: None)
    try:
        n = isess.world
        phases = len(nat.schedule(mode, "bi", n))
        idrv = nat.StepDriver(isess, mode, "bi", size, args.msgs, not args.no_verify, bool(batch), False,
                              depth=pick_depth(args.steps, phases), recv_budget=int(recv_budget), salt=2)
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
        say("failed: %s" % str(e)[:300])
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
        transport = "rccl" if args.child == REF_STOCK else args.child
        sess = nat.Session(env.rank, env.world, host=env.master_addr, port=args.child_port, device=device,
                           transport=transport, timeout_s=min(90.0, args.timeout))
        if args.child == REF_STOCK:
            iters = json.loads(args.child_ref_iters)
            out = reference_stock(nat, sess, args, [d for d in ("uni", "bi") if d in iters], iters,
                                  json.loads(args.child_ref_runs))
        else:
            budget = 0 if args.recv_budget.strip() in ("", "0") else nat.parse_size(args.recv_budget)
            out = steps_through(nat, sess, args, args.mode, size, args.child_batch, args.child, budget)
        del sess
    except Exception as e:
        out = {"error": str(e)[:300], "transport": args.child}
    if env.rank == 0:
        log("bench: child %s done" % args.child)
        with open(args.child_out, "w") as f:
            json.dump(out, f)
    return 0



#!/usr/bin/env python3
"""One-command tuning sweep of the xGMI pair cell.

Runs the pair cell 0 -> 1 (uni) and 0 <-> 1 (bi) at 32 MiB and 1 GiB through
build/p2p_matrix under every setting that can move a single xGMI link:

  rccl rows   --comms 1, 2, 4, 8 (messages spread over K communicators / streams)
              NCCL_NCHANNELS_PER_PEER, NCCL_P2P_NVL_CHUNKSIZE / NCCL_P2P_NET_CHUNKSIZE,
              NCCL_PROTO, RCCL_P2P_BATCH_ENABLE / RCCL_P2P_BATCH_THRESHOLD,
              NCCL_P2P_READ_ENABLE (peer reads vs writes over the link),
              P2P_RCCL_REGISTER=1|2 (user buffers registered with every
              communicator / allocated by ncclMemAlloc: RCCL may then move
              data straight between the user buffers instead of through its
              staging FIFO, csrc/transport_rccl.cpp),
              P2P_RCCL_MAX_CHUNK=1G (1 GiB ops instead of 16 MiB x the p2p
              channels RCCL's INFO log reports for the peer: RCCL loses the
              second half of an op above 16 MiB per p2p channel,
              scripts/rccl_half_repro.cpp, so this row is corrupt unless the
              link gets >= 64 channels)
  ipc rows    --ipc-engine kernel (one-sided pull by the gfx950 copy kernel),
              sdma, push, relay (stripes through idle third GPUs, N >= 3)

Every row runs with --verify and with the verified-warmup fallback off
(P2P_RECHUNK=0), so a setting under which RCCL delivers wrong bytes shows as
such instead of being re-posted in smaller ops under the same label.  A row
whose data does not verify (rc 2) is recorded as corrupt, never wins, and the
sweep goes on; every row also records the transport and p2p channels RCCL set
up for the pair (the p2p_matrix {"type":"links"} record); any other failure (crash, hang, timeout) ends the
sweep, so the GPU is never driven again after a fault.  Every row's cell GB/s,
p50 per message and the environment it ran under are written to
<out>/rows.jsonl.
<out>/summary.json names the winning setting per (direction, size) and the
gain over the default (RCCL, one communicator, no knobs).

It measures a link, so it needs N >= 2 GPUs and refuses N = 1.  ``--emulate``
validates the whole script without a second GPU: ranks share GPU 0 through
the IPC transport (``--emulate ipc``; the RCCL rows are skipped), through RCCL
itself (``--emulate rccl``: every rank claims a host of its own,
P2P_RCCL_DISTINCT_HOSTS=1, and RCCL links them over its socket transport on
loopback; every row runs, the GB/s are not xGMI's) or run on the CPU host
transport (``--emulate host``, build/p2p_matrix_host).  The reference has no tuning at
all: it inherits whatever NCCL_* the shell has (p2p_matrix.cc:126-131).

    python scripts/xgmi_pair_sweep.py --np 8 --out gpurun_out/xgmi_sweep
    python scripts/xgmi_pair_sweep.py --np 2 --emulate ipc --sizes 4M,32M
    python scripts/xgmi_pair_sweep.py --np 3 --emulate rccl --sizes 4M
    python scripts/xgmi_pair_sweep.py --np 2 --emulate host --sizes 64K
"""
from __future__ import annotations

import argparse
import json
import os
import shlex
import signal
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from test_nccl_p2p_amd.utils import rccl_env  # noqa: E402
from test_nccl_p2p_amd.utils.proc import die_with_parent, pdeathsig_prefix  # noqa: E402
MPIRUN = os.environ.get("P2P_MPIRUN", "/opt/conda/bin/mpirun")
# --emulate rccl: one host id per rank, so RCCL accepts ranks sharing GPU 0
# (csrc/transport_rccl.cpp) and connects them through loopback sockets.
EMULATE_RCCL_ENV = {"P2P_RCCL_DISTINCT_HOSTS": "1", "NCCL_SOCKET_IFNAME": "lo", "NCCL_IB_DISABLE": "1"}

# RCCL knobs that act on point-to-point traffic within a node.  Each entry is
# applied on top of the default environment at --comms 1, then the best knob
# set is re-run at the best communicator count.
RCCL_KNOBS = [
    {"NCCL_NCHANNELS_PER_PEER": "2"},
    {"NCCL_NCHANNELS_PER_PEER": "8"},
    {"NCCL_NCHANNELS_PER_PEER": "16", "NCCL_MIN_P2P_NCHANNELS": "16"},
    {"NCCL_NCHANNELS_PER_PEER": "32", "NCCL_MIN_P2P_NCHANNELS": "32", "NCCL_MAX_P2P_NCHANNELS": "64"},
    {"NCCL_P2P_NVL_CHUNKSIZE": "524288"},
    {"NCCL_P2P_NVL_CHUNKSIZE": "2097152"},
    {"NCCL_P2P_NET_CHUNKSIZE": "2097152"},
    {"NCCL_PROTO": "Simple"},
    {"NCCL_PROTO": "LL128"},
    {"RCCL_P2P_BATCH_ENABLE": "1"},
    {"RCCL_P2P_BATCH_ENABLE": "1", "RCCL_P2P_BATCH_THRESHOLD": "1048576"},
    {"NCCL_P2P_READ_ENABLE": "0"},
    {"NCCL_P2P_READ_ENABLE": "1"},
    {"P2P_RCCL_REGISTER": "1"},
    {"P2P_RCCL_REGISTER": "2"},
    # Ops of up to 1 GiB to the peer instead of 16 MiB x the channels RCCL's
    # INFO log reports for it: exact only if the link has >= 64 p2p channels
    # (16 MiB each), "corrupt" otherwise (the row runs with P2P_RECHUNK=0).
    {"P2P_RCCL_MAX_CHUNK": "1G"},
    # RCCL's kernel unroll factor: the transport asks for 4 (profiles/r3_unroll/,
    # +7% / +22% on the self path); RCCL's own pre-set 1 and 2 on the link.
    {"P2P_RCCL_UNROLL": "0"},
    {"RCCL_UNROLL_FACTOR": "2"},
]
COMMS = [1, 2, 4, 8]
IPC_ENGINES = ["kernel", "sdma", "push", "relay"]


def parse_args(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--np", type=int, default=0, help="ranks (default: visible GPUs)")
    ap.add_argument("--sizes", default="32M,1G")
    ap.add_argument("--dirs", default="uni,bi")
    ap.add_argument("--iters", default="auto")
    ap.add_argument("--out", default="gpurun_out/xgmi_sweep")
    ap.add_argument("--emulate", choices=["", "ipc", "rccl", "host"], default="",
                    help="validate without a second GPU: ranks share GPU 0 (ipc; rccl over RCCL's socket transport) "
                         "or use the CPU (host)")
    ap.add_argument("--rows", default="rccl,knobs,ipc", help="row groups to run, in this order: rccl, knobs, ipc")
    ap.add_argument("--budget", type=float, default=900.0, help="seconds for the whole sweep; rows that would "
                    "start after it is spent are listed as skipped")
    ap.add_argument("--row-timeout", type=float, default=180.0)
    ap.add_argument("--dry-run", action="store_true", help="print the rows and exit")
    ap.add_argument("--resume", action="store_true",
                    help="keep the rows already in <out>/rows.jsonl (a killed sweep continues where it stopped)")
    return ap.parse_args(argv)


def visible_gpus() -> int:
    # Device count without initialising the GPU (no HIP call in this process).
    vis = os.environ.get("HIP_VISIBLE_DEVICES") or os.environ.get("ROCR_VISIBLE_DEVICES")
    if vis:
        return len([v for v in vis.split(",") if v.strip()])
    try:
        return len([d for d in os.listdir("/dev/dri") if d.startswith("renderD")])
    except OSError:
        return 0


def plan_rows(args, np_):
    """Every (name, transport args, env) row of the sweep, in run order: the
    row groups in the order --rows names them (a budgeted sweep runs the
    groups it cares about most first)."""
    rows = []
    rccl_ok = args.emulate in ("", "rccl")
    for group in [g.strip() for g in args.rows.split(",") if g.strip()]:
        if group == "rccl" and rccl_ok:
            for k in COMMS:
                rows.append({"name": "rccl-comms%d" % k, "args": ["--transport", "rccl", "--comms", str(k)], "env": {}})
        elif group == "knobs" and rccl_ok:
            for env in RCCL_KNOBS:
                name = "rccl-" + "-".join("%s=%s" % (k.replace("P2P_", "").replace("NCCL_", "").replace("RCCL_", "").lower(),
                                                     v) for k, v in env.items())
                rows.append({"name": name, "args": ["--transport", "rccl", "--comms", "1"], "env": env, "knob": True})
        elif group == "ipc" and args.emulate != "host":
            for eng in IPC_ENGINES:
                if eng == "relay" and np_ < 3:
                    continue  # relay needs a third GPU to route through
                a = ["--transport", "ipc", "--ipc-engine", eng]
                rows.append({"name": "ipc-" + eng, "args": a, "env": {"P2P_IPC_POOL": "4G"} if eng == "relay" else {}})
    if args.emulate == "host":
        rows.append({"name": "host", "args": ["--transport", "host"], "env": {}})
    return rows


def cell_result(js_path, dirs):
    """{(dir, bytes): {...}} for the 0-1 cell of every pair run in the file."""
    out = {}
    with open(js_path) as fh:
        for line in fh:
            rec = json.loads(line)
            if rec.get("type") != "run" or rec.get("dir") not in dirs:
                continue
            for ph in rec["phases"]:
                if (ph["row"], ph["col"]) != (0, 1):
                    continue
                flows = ph["flows"]
                gbs = [f["gbs"] for f in flows]
                out[(rec["dir"], rec["bytes"])] = {
                    "cell_gbs": sum(gbs),  # bi: both directions, like the reference's bi matrix
                    "per_dir_gbs": sum(gbs) / len(gbs),
                    "p50_us": max(f["iter_us"]["p50"] for f in flows),
                    "mismatches": ph["mismatches"],
                    "iters": rec["iters"],
                }
    return out


def link_result(js_path):
    """Rank 0's view of peer 1 from the run's {"type":"links"} record: the
    transport class RCCL connected it through, the p2p channels, the op limit."""
    with open(js_path) as fh:
        for line in fh:
            rec = json.loads(line)
            if rec.get("type") == "links" and rec.get("ranks") and rec["ranks"][0]:
                r0 = rec["ranks"][0]
                peer = r0["peers"][1] if len(r0.get("peers", [])) > 1 else {}
                return {"transport": peer.get("transport"), "via": peer.get("via"),
                        "channels_connected": peer.get("channels_connected"), "op_channels": peer.get("op_channels"),
                        "op_limit": peer.get("op_limit"), "source": r0.get("op_limit_source")}
    return None


def run_row(args, row, np_, exe, tag, t_end=None):
    """One row as its own mpirun job, in a session of its own: on a timeout
    the whole job (launcher, proxies, ranks) is killed, so no rank is left
    driving a GPU.  t_end caps the row's time at the sweep's budget."""
    js = os.path.join(args.out, "%s.json" % tag)
    if os.path.exists(js):
        os.remove(js)
    limit = args.row_timeout if t_end is None else max(5.0, min(args.row_timeout, t_end - time.time()))
    # setpriv --pdeathsig: the launcher dies with this script (bench.py starts
    # the sweep as a child that dies with the bench, utils/proc.py).
    cmd = pdeathsig_prefix() + [
        MPIRUN, "-n", str(np_), exe, "--mode", "pair", "--cells", "0-1", "--dir", "both", "--sizes", args.sizes,
        "-n", args.iters, "--verify", "--no-compat", "--json", js, "--timeout", str(max(5, int(limit) - 5))]
    cmd += row["args"]
    if args.emulate in ("ipc", "rccl"):
        cmd += ["--device", "0"]
    env = dict(os.environ, P2P_RECHUNK="0", **row["env"])
    if args.emulate == "rccl":
        env.update(EMULATE_RCCL_ENV)
    t0 = time.time()
    proc = subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                            start_new_session=True)
    try:
        _, err = proc.communicate(timeout=limit + 10)
        rc = proc.returncode
    except subprocess.TimeoutExpired:
        try:
            os.killpg(proc.pid, signal.SIGKILL)
        except ProcessLookupError:
            pass
        proc.communicate()
        rc, err = 124, "row timed out after %.0f s" % limit
    rec = {"name": row["name"], "env": row["env"], "args": row["args"], "rc": rc, "seconds": round(time.time() - t0, 2),
           "cmd": " ".join(shlex.quote(c) for c in cmd)}
    if rc == 0:
        res = cell_result(js, set(args.dirs.split(",")))
        rec["cells"] = {"%s/%d" % k: v for k, v in sorted(res.items())}
        rec["link_0_1"] = link_result(js)
        bad = sum(v["mismatches"] for v in res.values())
        if bad or not res:
            rec["rc"] = 2
            rec["error"] = "verify mismatches %d" % bad if bad else "no 0-1 cell in the output"
    else:
        rec["error"] = err[-1500:]
    return rec


def summarize(rows, dirs, sizes_seen):
    base = next((r for r in rows if r["name"] == "rccl-comms1" and r["rc"] == 0), None)
    if base is None:
        base = next((r for r in rows if r["rc"] == 0), None)
    best = {}
    for r in rows:
        if r["rc"] != 0:
            continue
        for key, c in r["cells"].items():
            if key not in best or c["cell_gbs"] > best[key]["cell_gbs"]:
                best[key] = {"row": r["name"], "env": r["env"], "args": r["args"], "cell_gbs": c["cell_gbs"],
                             "p50_us": c["p50_us"]}
    for key, b in best.items():
        if base and key in base["cells"]:
            b["baseline_row"] = base["name"]
            b["baseline_gbs"] = base["cells"][key]["cell_gbs"]
            b["gain"] = round(b["cell_gbs"] / base["cells"][key]["cell_gbs"], 4)
    return best


def main(argv=None) -> int:
    die_with_parent()  # when started by bench.py (P2P_PARENT_PID)
    args = parse_args(argv)
    np_ = args.np or (2 if args.emulate else visible_gpus())
    if np_ < 2:
        print("xgmi_pair_sweep: needs N >= 2 ranks on distinct GPUs (found %d); a 1-GPU box has no xGMI link. "
              "Use --emulate ipc|host to validate the script." % np_, file=sys.stderr)
        return 1
    exe = os.path.join(ROOT, "build", "p2p_matrix_host" if args.emulate == "host" else "p2p_matrix")
    rows = plan_rows(args, np_)
    if args.dry_run:
        for r in rows:
            print(r["name"], " ".join(r["args"]), " ".join("%s=%s" % kv for kv in r["env"].items()))
        return 0
    if not args.emulate and visible_gpus() < np_:
        print("xgmi_pair_sweep: %d ranks but %d visible GPUs" % (np_, visible_gpus()), file=sys.stderr)
        return 1
    if not os.path.exists(exe):
        print("xgmi_pair_sweep: %s not built (make)" % exe, file=sys.stderr)
        return 1
    if not os.path.exists(MPIRUN):
        print("xgmi_pair_sweep: no mpirun at %s (P2P_MPIRUN)" % MPIRUN, file=sys.stderr)
        return 1
    os.makedirs(args.out, exist_ok=True)
    t_end = time.time() + args.budget
    done, skipped, failed, corrupt = [], [], None, []
    rows_path = os.path.join(args.out, "rows.jsonl")
    kept = {}
    if args.resume and os.path.exists(rows_path):
        # Rows that finished (clean or corrupt) are kept; a row that crashed
        # or timed out runs again.
        with open(rows_path) as fh:
            for line in fh:
                rec = json.loads(line)
                if rec.get("rc") in (0, 2):
                    kept[rec["name"]] = rec
    with open(rows_path, "w") as f:
        for rec in kept.values():
            f.write(json.dumps(rec) + "\n")
        for i, row in enumerate(rows):
            if row["name"] in kept:
                rec = kept[row["name"]]
                done.append(rec)
                if rec["rc"] == 2:
                    corrupt.append(rec["name"])
                print("%-40s kept from the previous run (rc=%d)" % (rec["name"], rec["rc"]), flush=True)
                continue
            # A row starts only if the longest row so far still fits.
            longest = max([r["seconds"] for r in done if "seconds" in r] + [5.0])
            if failed is not None or time.time() + longest > t_end:
                skipped.append(row["name"])
                continue
            rec = run_row(args, row, np_, exe, "row%02d" % i, t_end)
            f.write(json.dumps(rec) + "\n")
            f.flush()
            done.append(rec)
            cells = " ".join("%s %.1f" % (k, v["cell_gbs"]) for k, v in rec.get("cells", {}).items())
            print("%-40s rc=%d %6.1fs %s" % (rec["name"], rec["rc"], rec["seconds"], cells or rec.get("error", "")[-200:]),
                  flush=True)
            if rec["rc"] == 2:
                corrupt.append(rec["name"])  # wrong bytes under this setting: a finding, not a fault
            elif rec["rc"] != 0:
                failed = rec["name"]  # never keep driving the GPU after a failure
        # Best knob set at the best communicator count (knobs ran at --comms 1).
        knob_rows = [r for r in done if r["rc"] == 0 and any(r["name"] == x["name"] and x.get("knob") for x in rows)]
        comm_rows = [r for r in done if r["rc"] == 0 and r["name"].startswith("rccl-comms")]
        longest = max([r["seconds"] for r in done if "seconds" in r] + [5.0])
        if failed is None and knob_rows and comm_rows and time.time() + longest < t_end:
            key = sorted(comm_rows[0]["cells"])[-1]
            bk = max(knob_rows, key=lambda r: r["cells"].get(key, {}).get("cell_gbs", 0))
            bc = max(comm_rows, key=lambda r: r["cells"].get(key, {}).get("cell_gbs", 0))
            if bc["name"] != "rccl-comms1":
                combo = {"name": bk["name"] + "+" + bc["name"].split("-")[1], "env": bk["env"],
                         "args": ["--transport", "rccl"] + bc["args"][2:]}
                rec = run_row(args, combo, np_, exe, "combo", t_end)
                f.write(json.dumps(rec) + "\n")
                done.append(rec)
                print("%-40s rc=%d %6.1fs" % (rec["name"], rec["rc"], rec["seconds"]), flush=True)
    summary = {"np": np_, "emulate": args.emulate or None, "sizes": args.sizes, "dirs": args.dirs,
               "base_env": rccl_env.capture(), "rows_run": len(done), "rows_skipped": skipped, "failed_row": failed,
               "corrupt_rows": corrupt,
               "best": summarize(done, args.dirs, args.sizes)}
    with open(os.path.join(args.out, "summary.json"), "w") as f:
        json.dump(summary, f, indent=1)
    print(json.dumps({"best": summary["best"], "failed_row": failed, "corrupt_rows": corrupt, "rows_skipped": skipped}))
    return 2 if failed or corrupt else 0


if __name__ == "__main__":
    sys.exit(main())

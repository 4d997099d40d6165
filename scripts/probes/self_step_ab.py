#!/usr/bin/env python3
"""A/B of the GPU tier's RCCL self-step floor (tests/test_zz_perf_floors_gpu.py
_self_step_gbs: 32 MiB x 8 self messages in one group, median of 20 steps
after 5) across the settings that changed between rounds 3 and 4 (ADVICE r4:
the four-communicator rate fell from ~2300-2600 to ~1900 GB/s):

  * GPU_MAX_HW_QUEUES 4 (the box, and so the pytest process) vs 8 (bench.py);
  * RCCL's unroll: 4 (the transport's default) vs RCCL's own (P2P_RCCL_UNROLL=0);
  * the op limit: 16 MiB x channels (default) vs unsplit (P2P_RCCL_MAX_CHUNK=0);
  * messages per step: 8 (the floor's shape) vs 32.

Each setting runs in a child process of its own (HIP and RCCL read their
variables once), the list twice, interleaved.  One JSON line per run.

    python scripts/probes/self_step_ab.py [--rounds 2] [--out gpurun_out/self_step_ab.jsonl]
"""
import argparse
import json
import os
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

CONFIGS = [
    # name, env, comms, msgs
    ("q4_k1_m8", {"GPU_MAX_HW_QUEUES": "4"}, 1, 8),
    ("q4_k4_m8", {"GPU_MAX_HW_QUEUES": "4"}, 4, 8),
    ("q8_k4_m8", {"GPU_MAX_HW_QUEUES": "8"}, 4, 8),
    ("q4_k4_m8_unroll_rccl", {"GPU_MAX_HW_QUEUES": "4", "P2P_RCCL_UNROLL": "0"}, 4, 8),
    ("q4_k1_m8_unroll_rccl", {"GPU_MAX_HW_QUEUES": "4", "P2P_RCCL_UNROLL": "0"}, 1, 8),
    ("q4_k4_m8_unsplit", {"GPU_MAX_HW_QUEUES": "4", "P2P_RCCL_MAX_CHUNK": "0"}, 4, 8),
    ("q4_k1_m8_unsplit", {"GPU_MAX_HW_QUEUES": "4", "P2P_RCCL_MAX_CHUNK": "0"}, 1, 8),
    ("q4_k4_m32", {"GPU_MAX_HW_QUEUES": "4"}, 4, 32),
    ("q8_k8_m32", {"GPU_MAX_HW_QUEUES": "8"}, 8, 32),
    # In one process, in this order (the floor test runs one, then four
    # communicators; the pytest process has opened many sessions before).
    ("q4_seq_k1_k4", {"GPU_MAX_HW_QUEUES": "4"}, "1+4", 8),
    ("q4_seq_k4_k4", {"GPU_MAX_HW_QUEUES": "4"}, "4+4", 8),
    ("q4_seq_k1x6_k4", {"GPU_MAX_HW_QUEUES": "4"}, "1+1+1+1+1+1+4", 8),
    ("q4_seq_k8_k4", {"GPU_MAX_HW_QUEUES": "4"}, "8+4", 8),
    ("q8_seq_k1_k4", {"GPU_MAX_HW_QUEUES": "8"}, "1+4", 8),
    # Work on the null stream first ("t": a torch kernel on the current,
    # i.e. default, stream; "f": the fill kernel on stream 0), as the kernel
    # tests do before the GPU tier's floor (profiles/r5_floor_bisect/).
    ("q4_null_torch_k4", {"GPU_MAX_HW_QUEUES": "4"}, "t+4", 8),
    ("q4_null_fill_k4", {"GPU_MAX_HW_QUEUES": "4"}, "f+4", 8),
    ("q8_null_fill_k4", {"GPU_MAX_HW_QUEUES": "8"}, "f+4", 8),
    ("q4_null_fill_k1", {"GPU_MAX_HW_QUEUES": "4"}, "f+1", 8),
]


def child(seq: str, msgs: int) -> None:
    """Sessions of the communicator counts in `seq` ("1+4": one, then four)
    one after the other in this process; the last one's rate is printed."""
    sys.path.insert(0, ROOT)
    import test_nccl_p2p_amd

    nat = test_nccl_p2p_amd.require_native()
    steps = str(seq).split("+")
    rec = None
    for st in steps:
        if st == "t":
            import torch

            torch.ones(1 << 20, device="cuda").mul_(2)
            torch.cuda.synchronize()
        elif st == "f":
            import torch

            buf = torch.empty(64 << 20, dtype=torch.uint8, device="cuda")
            nat.fill(buf.data_ptr(), 64 << 20, 1, 0)
            torch.cuda.synchronize()
            del buf
        else:
            rec = one_session(nat, int(st), msgs)
    print(json.dumps(dict(rec, earlier=steps[:-1])))


def one_session(nat, comms: int, msgs: int) -> dict:
    s = nat.Session(0, 1, device=0, transport="rccl:%d" % comms if comms > 1 else "rccl", timeout_s=60)
    d = nat.StepDriver(s, "self", "bi", 32 << 20, msgs, False, True, False)
    d.connect()
    d.run_steps(0, 5)
    d.sync()
    d.reset()
    d.run_steps(5, 20)
    d.sync()
    ms = d.step_ms()
    rep = json.loads(s.link_reports())[0] or {}
    peer = (rep.get("peers") or [{}])[0]
    del d, s
    return {"gbs_median": msgs * (32 << 20) / (statistics.median(ms) * 1e-3) / 1e9,
            "step_ms_median": statistics.median(ms), "op_limit": peer.get("op_limit"),
            "unroll": [c.get("unroll") for c in rep.get("comms") or []]}


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "self_step_ab.jsonl"))
    ap.add_argument("--only", default="", help="comma-separated config names (default: all)")
    ap.add_argument("--child", default=None, help=argparse.SUPPRESS)
    a = ap.parse_args()
    if a.child:
        c, m = a.child.split(",")
        child(c, int(m))
        return 0
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    rows = {}
    with open(a.out, "w") as f:
        for r in range(a.rounds):
            for name, env, comms, msgs in CONFIGS:
                if a.only and name not in a.only.split(","):
                    continue
                e = dict(os.environ, **env)
                p = subprocess.run([sys.executable, os.path.abspath(__file__), "--child", "%s,%d" % (comms, msgs)],
                                   capture_output=True, text=True, timeout=120, env=e)
                line = [x for x in p.stdout.splitlines() if x.startswith("{")]
                rec = dict(json.loads(line[-1]) if line else {"error": p.stderr[-400:]}, name=name, round=r,
                           rc=p.returncode)
                f.write(json.dumps(rec) + "\n")
                f.flush()
                rows.setdefault(name, []).append(rec.get("gbs_median"))
                print("%-24s round %d  %s GB/s  %s" % (name, r, "%.1f" % rec["gbs_median"] if "gbs_median" in rec
                                                        else "ERR", rec.get("error", "")[-200:]), flush=True)
                if p.returncode != 0:
                    return p.returncode
    print("\nsummary (GB/s per round):")
    for name, v in rows.items():
        print("  %-24s %s" % (name, "  ".join("%.1f" % x for x in v if x is not None)))
    return 0


if __name__ == "__main__":
    sys.exit(main())

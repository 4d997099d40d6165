#!/usr/bin/env python3
"""Sweeps RCCL point-to-point knobs (never hard-code them
silently) over build/p2p_matrix runs and tabulates GB/s per message size.

    python scripts/rccl_env_sweep.py --mode self --sizes 1M:1G:4 --out gpurun_out/sweep
    mpirun-free: runs the binary directly (1 rank) unless --launcher is given,
    e.g. --launcher "/opt/conda/bin/mpirun -n 2".
"""
import argparse
import json
import os
import shlex
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CONFIGS = [
    {},
    {"NCCL_NCHANNELS_PER_PEER": "4"},
    {"NCCL_NCHANNELS_PER_PEER": "8"},
    {"NCCL_NCHANNELS_PER_PEER": "16"},
    {"NCCL_MIN_P2P_NCHANNELS": "16", "NCCL_NCHANNELS_PER_PEER": "16"},
    {"NCCL_MIN_P2P_NCHANNELS": "32", "NCCL_MAX_P2P_NCHANNELS": "64", "NCCL_NCHANNELS_PER_PEER": "32"},
    {"NCCL_P2P_NVL_CHUNKSIZE": "1048576"},
    {"NCCL_PROTO": "Simple"},
    {"RCCL_P2P_BATCH_ENABLE": "1"},
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", default="self")
    ap.add_argument("--dir", default="bi")
    ap.add_argument("--sizes", default="64K:1G:4")
    ap.add_argument("--iters", default="auto")
    ap.add_argument("--out", default="gpurun_out/sweep")
    ap.add_argument("--launcher", default="")
    ap.add_argument("--timeout", type=int, default=240)
    a = ap.parse_args()
    os.makedirs(a.out, exist_ok=True)
    exe = os.path.join(ROOT, "build", "p2p_matrix")
    table = []
    for i, cfg in enumerate(CONFIGS):
        js = os.path.join(a.out, "cfg%02d.json" % i)
        cmd = shlex.split(a.launcher) + [exe, "--mode", a.mode, "--dir", a.dir, "--sizes", a.sizes, "-n", a.iters,
                                         "--no-compat", "--json", js]
        env = dict(os.environ, **cfg)
        r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=a.timeout)
        if r.returncode != 0:
            print("config %s failed rc=%d: %s" % (cfg, r.returncode, r.stderr[-500:]), flush=True)
            break  # never keep driving the GPU after a failure
        row = {"env": cfg, "gbs": {}}
        with open(js) as fh:
            for line in fh:
                rec = json.loads(line)
                if rec["type"] == "run":
                    row["gbs"][rec["bytes"]] = rec["gbs_mean"]
        table.append(row)
        print(json.dumps(row), flush=True)
    with open(os.path.join(a.out, "summary.json"), "w") as f:
        json.dump(table, f, indent=1)


if __name__ == "__main__":
    sys.exit(main())

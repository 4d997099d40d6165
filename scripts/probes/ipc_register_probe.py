#!/usr/bin/env python3
"""Repeated buffer-set registration through the IPC transport (2+ ranks on
one GPU, torchrun): one Session.run per size, printing progress, so a failing
export/import is pinned to a size and engine.

    torchrun --nproc-per-node 2 scripts/probes/ipc_register_probe.py ipc:push
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from test_nccl_p2p_amd import require_native  # noqa: E402
from test_nccl_p2p_amd.parallel.session import create_session, init_control_plane  # noqa: E402


def main():
    transport = sys.argv[1] if len(sys.argv) > 1 else "ipc:push"
    env = init_control_plane("gloo")
    torch.cuda.set_device(0)
    sess = create_session(transport, device=0, timeout_s=60.0)
    for cells in ([(0, 1)], []):
        for nbytes in [4096 << (2 * k) for k in range(9)]:
            r = json.loads(sess.run(mode="pair", dir="uni", bytes=nbytes, iters=4, warmup=1, timing="events",
                                    verify=True, warm=False, cells=cells))
            bad = sum(ph["mismatches"] for ph in r["phases"])
            if env.rank == 0:
                print("%s cells=%s %10d B ok, mismatches %d" % (transport, cells, nbytes, bad), flush=True)
    del sess


if __name__ == "__main__":
    main()

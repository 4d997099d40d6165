"""torchrun helper: one StepDriver session with a progress line per stage on
every rank (debugging a stalled step path; tests/test_ipc_gpu.py).

    torchrun --nproc-per-node N tests/scripts/step_probe.py <transport> [mode] [size] [msgs] [depth] [steps]
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from test_nccl_p2p_amd import require_native  # noqa: E402
from test_nccl_p2p_amd.parallel.session import create_session  # noqa: E402

T0 = time.monotonic()


def main():
    a = sys.argv[1:] + [None] * 6
    transport, mode = a[0] or "ipc:push", a[1] or "tournament"
    nat = require_native()
    size = nat.parse_size(a[2] or "32M")
    msgs, depth, steps = int(a[3] or 8), int(a[4] or 5), int(a[5] or 14)
    rank = int(os.environ.get("RANK", 0))

    def say(m):
        print("[%6.2fs] rank %d: %s" % (time.monotonic() - T0, rank, m), file=sys.stderr, flush=True)

    device = None
    if not transport.startswith(("host", "shm")):
        import torch
        device = int(os.environ.get("P2P_FUZZ_DEVICE", os.environ.get("LOCAL_RANK", 0)))
        torch.cuda.set_device(device)
    sess = create_session(transport, device=device, timeout_s=float(os.environ.get("P2P_FUZZ_TIMEOUT", "60")))
    say("session")
    d = nat.StepDriver(sess, mode, "bi", size, msgs, True, True, False, depth=depth, salt=2)
    say("driver (depth %d, %d receive bytes)" % (d.depth, d.recv_bytes))
    d.connect()
    say("connected")
    d.run_steps(0, 3)
    d.sync()
    say("warm")
    d.poison()
    sess.barrier()
    d.run_steps(3, steps)
    d.sync()
    sess.barrier()
    v = d.verify_steps(3, steps)
    say("verified %s" % v)
    del d, sess
    say("closed")
    return 0 if v["mismatches"] == 0 else 2


if __name__ == "__main__":
    sys.exit(main())

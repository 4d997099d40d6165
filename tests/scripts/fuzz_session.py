"""torchrun helper: random verified message groups through a native session
(tests/test_multi_gpu.py, tests/test_torchrun_cpu.py).

    torchrun --nproc-per-node N tests/scripts/fuzz_session.py <transport> [rounds]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from test_nccl_p2p_amd.parallel.session import create_session  # noqa: E402


def main():
    transport = sys.argv[1] if len(sys.argv) > 1 else "host"
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    device = None
    if not transport.startswith(("host", "shm")):
        import torch
        # P2P_FUZZ_DEVICE pins every rank to one GPU (the IPC transport's
        # several-processes-per-GPU emulation); default: LOCAL_RANK.
        device = int(os.environ.get("P2P_FUZZ_DEVICE", os.environ.get("LOCAL_RANK", 0)))
        torch.cuda.set_device(device)
    sess = create_session(transport, device=device, timeout_s=float(os.environ.get("P2P_FUZZ_TIMEOUT", "120")))
    bad = sess.fuzz(rounds=rounds, seed=11, max_bytes=8 << 20)
    total = sess.allreduce_sum(float(bad))
    if sess.rank == 0:
        print("FUZZ %s mismatches %d" % (transport, int(total)))
    del sess
    return 0 if total == 0 else 2


if __name__ == "__main__":
    sys.exit(main())

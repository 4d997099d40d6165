"""bench.py helpers that need no GPU and no launcher."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import bench  # noqa: E402


def test_posting_candidates_default_rccl():
    # W = 7: one communicator per-message and batched, four communicators batched.
    assert bench.posting_candidates("rccl", -1, -1, 7) == [(1, 0), (1, 1), (4, 1)]


def test_posting_candidates_fixed_and_other_transports():
    assert bench.posting_candidates("rccl", 4, -1, 7) == [(4, 1)]
    assert bench.posting_candidates("rccl", 1, 1, 7) == [(1, 1)]
    assert bench.posting_candidates("ipc", -1, -1, 7) == [(1, 0), (1, 1)]
    assert bench.posting_candidates("host", 4, 0, 7) == [(1, 0)]


def test_posting_candidates_short_warmup_keeps_the_last():
    assert bench.posting_candidates("rccl", -1, -1, 2) == [(4, 1)]
    assert bench.posting_candidates("rccl", -1, -1, 1) == [(4, 1)]
    assert bench.posting_candidates("shm", -1, -1, 0) == [(1, 1)]


def test_first_comms():
    assert bench.first_comms("rccl", -1) == 1
    assert bench.first_comms("rccl", 4) == 4
    assert bench.first_comms("ipc", 4) == 1


def test_bench_help_lists_transports():
    args = bench.parse_args([])
    assert args.transport == "rccl" and args.comms == -1 and args.isolate == 1
    for t in ("ipc:relay", "shm"):
        assert bench.parse_args(["--transport", t]).transport == t

"""The RCCL log-line formats pinned in tests/data match the linked library.

RCCL's xGMI P2P transport never runs on a one-GPU box, so the INFO lines a
node run prints are pinned from the printf formats compiled into the
librccl.so that csrc/ links (scripts/rccl_formats.py); the host test
test_rccl_log_formats_of_the_library expands and parses each one.
This test keeps that file honest: a different library version, or a format
the file lacks, fails here with the command that re-pins it.
"""

import glob
import os

import pytest

from test_nccl_p2p_amd.utils import rccl_env

DATA = os.path.join(os.path.dirname(__file__), "data")


def _pinned():
    files = sorted(glob.glob(os.path.join(DATA, "rccl_*_log_formats.txt")))
    assert len(files) == 1, files
    ver = os.path.basename(files[0])[len("rccl_"):-len("_log_formats.txt")]
    return ver, rccl_env.read_pinned_formats(files[0])


def test_pinned_formats_cover_what_the_parser_needs():
    _, fmts = _pinned()
    vias = {f.split(" via ")[1].split("/")[0] for f in fmts if " via " in f}
    assert {"P2P", "SHM", "NET", "COLLNET"} <= vias
    # Every P2P format names both ends as rank[bus] before " via ".
    for f in fmts:
        if " via P2P/" in f:
            head = f.split(" via ")[0]
            assert head.startswith("Channel %02d/") and head.count("[%") == 2, f
    # The init lines parse_rccl_init reads.
    assert any(f.endswith("%d p2p channels, %d p2p channels per peer") for f in fmts)
    assert any(" nRanks %d nNodes %d " in f for f in fmts)
    assert sum(f.startswith("RCCL Unroll Factor (") for f in fmts) == 2


def test_pinned_formats_match_the_linked_library():
    lib = rccl_env.linked_librccl()
    if not os.path.exists(lib):
        pytest.skip("no librccl.so next to torch: %s" % lib)
    ver, fmts = rccl_env.log_formats(lib)
    pinned_ver, pinned = _pinned()
    hint = "re-pin with `python scripts/rccl_formats.py --write` and re-run the host tests"
    assert ver == pinned_ver, "linked RCCL %s, formats pinned for %s: %s" % (ver, pinned_ver, hint)
    assert fmts == pinned, hint


def test_log_formats_reads_a_synthetic_library(tmp_path):
    blob = (
        b"\x7fELF\x00junk\x00RCCL version : 9.1.2\x00"
        b"Channel %02d/%01d : %d[%lx] -> %d[%lx] via P2P/NEW%s comm %p nRanks %02d\x00"
        b"Channel %02d/%02d :\x00not a format\x00RCCL Unroll Factor (pre-set): %d\x00"
    )
    p = tmp_path / "librccl.so"
    p.write_bytes(blob)
    assert rccl_env.log_formats(str(p)) == (
        "9.1.2",
        ["Channel %02d/%01d : %d[%lx] -> %d[%lx] via P2P/NEW%s comm %p nRanks %02d", "RCCL Unroll Factor (pre-set): %d"],
    )

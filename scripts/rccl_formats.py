#!/usr/bin/env python3
"""Pin the formats of the RCCL log lines that csrc/rccl_log.cpp parses.

The per-peer op limit comes from RCCL's ``Channel cc/1 : a[bus] -> b[bus] via
P2P/…`` INFO lines (csrc/rccl_log.cpp parse_rccl_connections).  The xGMI P2P
transport cannot run on one GPU (RCCL refuses two ranks on one device), so the
lines a node run will print are pinned here from the library itself: the
printf formats of the connection and init lines compiled into the linked
librccl.so are read from its bytes and written to tests/data/rccl_<version>_log_formats.txt.
tests/host/test_main.cpp (test_rccl_log_formats_of_the_library) expands
every format and parses the result; tests/test_rccl_formats.py checks that the
file still matches the library.

    python scripts/rccl_formats.py            # print version and formats
    python scripts/rccl_formats.py --write    # (re)write the pinned file
"""

import argparse
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

from test_nccl_p2p_amd.utils.rccl_env import log_formats, linked_librccl  # noqa: E402

HEADER = (
    "# The printf formats of the RCCL INFO lines csrc/rccl_log.cpp parses, compiled\n"
    "# into the librccl.so that torch bundles (RCCL version : {ver}), the library\n"
    "# csrc/ links against.  Read from the binary's bytes (scripts/rccl_formats.py);\n"
    "# nothing was run.  One format a line.\n"
)


def pinned_path(ver: str) -> str:
    root = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
    return os.path.normpath(os.path.join(root, "tests", "data", "rccl_%s_log_formats.txt" % ver))


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    ap.add_argument("--lib", default=None, help="librccl.so to read (default: the one csrc/ links)")
    ap.add_argument("--write", action="store_true", help="write tests/data/rccl_<version>_log_formats.txt")
    a = ap.parse_args()
    lib = a.lib or linked_librccl()
    ver, fmts = log_formats(lib)
    if not ver or not fmts:
        print("no RCCL version / log formats found in %s" % lib, file=sys.stderr)
        return 1
    print("%s: RCCL %s, %d log formats" % (lib, ver, len(fmts)))
    for f in fmts:
        print("  " + f)
    if a.write:
        out = pinned_path(ver)
        with open(out, "w") as f:
            f.write(HEADER.format(ver=ver))
            f.writelines(x + "\n" for x in fmts)
        print("wrote " + out)
    return 0


if __name__ == "__main__":
    sys.exit(main())

#!/usr/bin/env python3
"""Does RCCL read RCCL_UNROLL_FACTOR at every communicator's init, or once per
process?  Opens sessions under different values in one process and prints
the factor RCCL's INFO log reports for each (link_reports comms[].unroll)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import test_nccl_p2p_amd as t  # noqa: E402

nat = t.require_native()
for u in ("4", "1", "2", "4"):
    os.environ["RCCL_UNROLL_FACTOR"] = u
    s = nat.Session(0, 1, device=0, transport="rccl", timeout_s=60)
    r = json.loads(s.link_reports())[0]
    print("set", u, "-> RCCL log says", [c["unroll"] for c in r["comms"]], flush=True)
    del s

"""Run under torchrun (2+ ranks, CPU): the Python Session API over the host
transport -- cell-restricted runs, latency, the device ping-pong refusal, and
a StepDriver -- as bench.py uses them."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

from test_nccl_p2p_amd import require_native  # noqa: E402
from test_nccl_p2p_amd.parallel.session import create_session, init_control_plane  # noqa: E402


def main():
    nat = require_native()
    env = init_control_plane("gloo")
    sess = create_session("host", timeout_s=60.0)
    r = json.loads(sess.run(mode="pair", dir="uni", bytes=64 << 10, iters=3, warmup=1, verify=True, warm=False,
                            cells=[(0, 1)]))
    flows = [(f["src"], f["dst"]) for ph in r["phases"] for f in ph["flows"]]
    assert flows == [(0, 1)], flows
    assert all(ph["mismatches"] == 0 for ph in r["phases"])
    lat = json.loads(sess.latency(8, 20, 5))
    assert lat["method"] == "host" and len(lat["pairs"]) == env.world * (env.world - 1) // 2
    try:
        sess.device_latency(8, 10, 2)
        raise AssertionError("device ping-pong must be refused on the host transport")
    except RuntimeError as e:
        assert "one-sided transport" in str(e), e
    drv = nat.StepDriver(sess, "tournament", "bi", 16 << 10, 2, True, True, False)
    drv.connect()
    drv.run_steps(0, 2 * drv.phases)
    drv.sync()
    assert drv.verify_last() == 0
    assert len(drv.step_ms()) == 2 * drv.phases
    sess.barrier()
    if env.rank == 0:
        print("SESSION API OK", flush=True)


if __name__ == "__main__":
    main()

"""Performance floors of the GPU tier.  They still fail the tier, but this
file sorts after every correctness test (and conftest.py orders the `perf`
marker last), so a missed floor under `pytest -x` can no longer hide the RCCL
correctness tests (VERDICT r3 "do this" #1: the driver's GPU tier stopped at
a 3.42 TB/s fill reading and never ran test_rccl_gpu.py).

Method (not a 5-launch window after an idle GPU):
  * a sustained warm-up of >= 100 ms of 1 GiB fills first;
  * every launch timed on its own event pair, 20 launches, median;
  * torch's zero_() and copy_() timed the same way in the same window as the
    in-process roofs, so the floor is relative as well as absolute;
  * a "cold" series after 2 s of idling records whether the first launches
    after idle are slow (clock ramp) -- recorded, never asserted;
  * every series is printed, and written to $P2P_TEST_LOG_DIR/perf_floors.json
    when that is set (the GPU sessions point it under gpurun_out/);
  * the medians go into conftest.PERF_RECORDS before any floor is asserted,
    so the session's PERF line carries the box's rates, pass or fail.
The fill replaces the reference's cudaMemset (p2p_matrix.cc:129-130)."""
import json
import os
import statistics
import time

import pytest
import torch

from conftest import PERF_RECORDS
from test_nccl_p2p_amd.ops import verify

pytestmark = [pytest.mark.gpu, pytest.mark.perf]

GIB = 1 << 30


@pytest.fixture(scope="module", autouse=True)
def _gpu(native):
    assert torch.cuda.is_available(), "GPU tier needs a GPU"
    torch.cuda.set_device(0)


def per_launch_ms(fn, reps=20):
    """Kernel time of each of `reps` back-to-back launches (one event pair
    around each, all recorded before the single synchronize)."""
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for s, e in ev:
        s.record()
        fn()
        e.record()
    torch.cuda.synchronize()
    return [s.elapsed_time(e) for s, e in ev]


def tbs(ms_list, nbytes):
    return nbytes / (statistics.median(ms_list) * 1e-3) / 1e12


def warm(fn, seconds=0.1):
    """Launch fn back to back until `seconds` of GPU work have completed."""
    t0 = time.perf_counter()
    n = 0
    while time.perf_counter() - t0 < seconds or n < 16:
        for _ in range(16):
            fn()
        torch.cuda.synchronize()
        n += 16
    return n


def _record(name, rec):
    d = os.environ.get("P2P_TEST_LOG_DIR")
    if d:
        os.makedirs(d, exist_ok=True)
        path = os.path.join(d, "perf_floors.json")
        old = {}
        if os.path.exists(path):
            with open(path) as f:
                old = json.load(f)
        old[name] = rec
        with open(path, "w") as f:
            json.dump(old, f, indent=1)


def test_kernel_bandwidth_floors(native):
    """1 GiB fill / LDS-DMA verify / copy against absolute floors at ~75-80%
    of the lowest per-launch medians this test measured in round 4 (fill
    6.93, verify with its reset + finalize launches 5.80, copy 3.14 TB/s:
    profiles/r4_gpu_tier/, r4_tier2/, r4_final/) and the fill against 0.8 x
    torch's zero_() measured in the same window."""
    buf = torch.empty(GIB, dtype=torch.uint8, device="cuda")
    dst = torch.empty_like(buf)
    stream = torch.cuda.current_stream().cuda_stream
    ptr, dptr = buf.data_ptr(), dst.data_ptr()

    def fill(impl):
        return lambda: native.fill(ptr, GIB, 1, stream, impl)

    # Cold series first: 2 s idle, then launches with no warm-up.
    torch.cuda.synchronize()
    time.sleep(2.0)
    cold = per_launch_ms(fill(0))
    warm_launches = warm(fill(0))
    series = {
        "fill": per_launch_ms(fill(0)),            # the default (FillImpl::Auto)
        "zero_": per_launch_ms(lambda: buf.zero_()),
    }
    native.fill(ptr, GIB, 1, stream, 0)
    assert verify(buf, 1, impl="stride").ok
    series["verify_lds8"] = per_launch_ms(lambda: native.verify_launch(ptr, GIB, 1, 1, True, stream))
    series["verify_stride"] = per_launch_ms(lambda: native.verify_launch(ptr, GIB, 1, 2, True, stream))
    series["copy"] = per_launch_ms(lambda: native.copy(dptr, ptr, GIB, stream))
    series["copy_"] = per_launch_ms(lambda: dst.copy_(buf))
    series["fill_again"] = per_launch_ms(fill(0))  # same window, after the others
    native.copy(dptr, ptr, GIB, stream)
    assert verify(dst, 1).ok
    rates = {k: round(tbs(v, GIB), 3) for k, v in series.items()}
    rates["fill_cold"] = round(tbs(cold, GIB), 3)
    rec = {"tbs_median": rates, "warm_launches": warm_launches,
           "per_launch_ms": dict(series, fill_cold=cold)}
    _record("kernel_bandwidth_floors", rec)
    for k in ("fill", "zero_", "verify_lds8", "verify_stride", "copy", "copy_", "fill_cold"):
        PERF_RECORDS[k] = rates[k]
    print(json.dumps(rates))
    for k, v in rec["per_launch_ms"].items():
        print("%-12s %s" % (k, " ".join("%.3f" % x for x in v)))
    msg = json.dumps(rec)
    assert rates["fill"] > 5.5, msg
    assert rates["fill"] >= 0.8 * rates["zero_"], msg
    assert rates["verify_lds8"] > 4.6, msg
    assert rates["copy"] > 2.5, msg  # payload bytes (read once + written once)


def test_verify_staging_ab(native):
    """VERDICT r5 item 3 (LDS staging must be shown not to cost
    bandwidth): the LDS-DMA verify (lds8, the default) and register staging
    (stride) timed alternately in one process on the same buffer -- 12
    rounds per size, each round 5 event-timed launches of each (the order
    reversed every other round), the median per kernel -- at 1 GiB and 4
    GiB.  lds_over_stride = the stride kernel's time over the LDS kernel's,
    summed over both sizes (>= 1: LDS staging costs nothing); per size too.
    Floor 0.97 on the sum, 0.95 per size.  (scripts/verify_ab.py runs the
    same A/B with the grid-cap and batched-kernel variants.)"""
    stream = torch.cuda.current_stream().cuda_stream
    ms = {}
    for gib in (1, 4):
        nbytes = gib * GIB
        buf = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
        ptr = buf.data_ptr()
        native.fill(ptr, nbytes, 3, stream, 0)
        assert verify(buf, 3).ok

        def lds():
            native.verify_launch(ptr, nbytes, 3, 1, True, stream)

        def stride():
            native.verify_launch(ptr, nbytes, 3, 2, True, stream)

        warm(lds, 0.2)
        runs = {"lds8": [], "stride": []}
        for r in range(12):
            for name, fn in ((("lds8", lds), ("stride", stride)) if r % 2 == 0 else
                             (("stride", stride), ("lds8", lds))):
                runs[name].append(statistics.median(per_launch_ms(fn, 5)))
        ms[gib] = {k: statistics.median(v) for k, v in runs.items()}
        ms[gib]["rounds"] = runs
        del buf
        torch.cuda.empty_cache()
    per_size = {"%dg" % g: round(m["stride"] / m["lds8"], 4) for g, m in ms.items()}
    total = round(sum(m["stride"] for m in ms.values()) / sum(m["lds8"] for m in ms.values()), 4)
    rates = {"%dg_%s" % (g, k): round(g * GIB / (m[k] * 1e-3) / 1e12, 3) for g, m in ms.items() for k in ("lds8", "stride")}
    rec = {"lds_over_stride": total, "per_size": per_size, "tbs": rates,
           "rounds_ms": {"%dg" % g: m["rounds"] for g, m in ms.items()}}
    _record("verify_staging_ab", rec)
    PERF_RECORDS["lds_over_stride"] = total
    PERF_RECORDS.update({"lds_over_stride_" + k: v for k, v in per_size.items()})
    print(json.dumps(rec))
    assert total >= 0.97, rec
    assert min(per_size.values()) >= 0.95, rec


SELF_STEP_CHILD = """
import json, statistics, sys
from test_nccl_p2p_amd import require_native
nat = require_native()
out = {}
for transport in ("rccl", "rccl:4"):
    s = nat.Session(0, 1, device=0, transport=transport, timeout_s=120)
    d = nat.StepDriver(s, "self", "bi", 32 << 20, 8, False, True, False)
    d.connect()
    d.run_steps(0, 5)
    d.sync()
    d.reset()
    d.run_steps(5, 20)
    d.sync()
    ms = d.step_ms()
    del d, s
    out[transport] = {"gbs_median": 8 * (32 << 20) / (statistics.median(ms) * 1e-3) / 1e9, "step_ms": ms}
print("RESULT " + json.dumps(out))
"""


def test_self_copy_rate_floors(native):
    """The RCCL self step (32 MiB x 8 self messages in one group, median of
    20 steps after 5) through one and four communicators, measured in a
    fresh process with the environment's hardware queues (4 on the box), as
    bench.py's ranks run.  Inside the tier's process the four-communicator
    rate fell to ~1800-1970 GB/s: the kernel tests before it launch work on
    HIP's null stream, which then holds one of the process's 4 hardware
    queues, so two of the transport's four streams share one (ADVICE r4;
    profiles/r5_floor_bisect/: 2177-2381 fresh, 1876-1976 after a fill on the
    null stream, 2410-2582 with 8 queues).  Floors at ~80% of the fresh
    rates measured (one: 1172-1238, four: 2177-2451 GB/s, profiles/r5_tier1/,
    r5_floor_bisect/), and four at least 1.5x one (1.84-2.03x): a lost
    multi-communicator speedup or a slower RCCL posting fails here."""
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = subprocess.run([sys.executable, "-c", SELF_STEP_CHILD], capture_output=True, text=True, timeout=240,
                         cwd=root)
    assert out.returncode == 0, out.stderr[-3000:]
    res = json.loads([l for l in out.stdout.splitlines() if l.startswith("RESULT ")][-1][len("RESULT "):])
    one, four = res["rccl"]["gbs_median"], res["rccl:4"]["gbs_median"]
    rec = {"rccl": res["rccl"], "rccl:4": res["rccl:4"], "ratio": four / one, "process": "fresh child"}
    _record("self_copy_rate_floors", rec)
    PERF_RECORDS.update(rccl=round(one, 1), rccl4=round(four, 1))
    print("rccl %.1f  rccl:4 %.1f GB/s  ratio %.2f" % (one, four, four / one))
    assert one > 950.0, rec
    assert four > 1750.0, rec
    assert four >= 1.5 * one, rec

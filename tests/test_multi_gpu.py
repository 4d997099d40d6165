"""Tier T4: the RCCL data plane across real GPUs.  Runs only
where >= 2 MI355X are visible (skipped on the 1-GPU test boxes; the 8-GPU
scaling runs happen through bench.py on a full node).

The driver gives the whole `pytest -m gpu` run one 900 s step.  The
single-GPU tests took 364-391 s of it on the round-3 tree
(profiles/r3b_close/pytest_gpu*.log), so this tier is sized to fit the
rest: each test's subprocess limits add up to its BUDGET_S entry, the
measured single-GPU time + the sum of the budgets stays under conftest's
SESSION_LIMIT_S (checked on the CPU by
tests/test_scripts_cpu.py::test_multi_gpu_tier_fits_the_driver_step), and
conftest.py starts a test only if the session's elapsed time + its budget
still fits.  conftest orders this tier after the single-GPU correctness
tests (the RCCL tiers included) and before the perf floors.  The tests run
in the order of what they prove: the reference's matrix over xGMI first,
then the concurrent modes, bench.py, the hand-written data plane and the
fuzzers."""
import json
import os
import sys

import pytest

from conftest import MPIRUN, PERF_RECORDS, ROOT, ensure_built, free_port, run_logged
from test_nccl_p2p_amd.utils.report import fabric_findings, offdiag, parse_compat


# P2P_REHEARSE_MULTI_GPU=N: run this tier with N ranks on the one GPU of a
# test box (conftest.py puts every rank on device 0 and gives each its own
# RCCL host, so RCCL connects them over its socket transport, not xGMI).  It
# checks the command lines, the assertions and the budgets before a node run.
REHEARSAL = int(os.environ.get("P2P_REHEARSE_MULTI_GPU") or 0)
# Loopback sockets move ~5-8 GB/s per pair, xGMI ~50: the rehearsal's benches
# send a quarter of the messages per step (8 ranks share the one box's
# sockets: a sixteenth) and its link check a lower floor; with 8 ranks the
# concurrent modes stop at 16 MiB instead of 64.
BENCH_MSGS = (["--msgs", "8"] if REHEARSAL >= 8 else ["--msgs", "32"]) if REHEARSAL else []
MIN_GBS = "0.05" if REHEARSAL else "1"
CONCURRENT_SIZES = "1M,16M" if REHEARSAL >= 8 else "1M,64M"
# 8 ranks over one box's loopback sockets took 77-98 s per communicator
# setting for the concurrent modes, and the reference's matrices 60 s of
# their 60 (profiles/r4_reh8/); a node's xGMI takes seconds.
CONCURRENT_TIMEOUT_S = 150 if REHEARSAL >= 8 else None
# test_fabric_is_uniform's cell bound in a rehearsal (a node: 0.5 x the median).
REHEARSAL_MIN_RATIO = 0.25
# 8 ranks on one GPU plus a comparison child per rank would pass the test
# box's 16 processes per GPU; on a node each rank has a GPU of its own.
ISOLATE = ["--isolate", "0"] if REHEARSAL >= 8 else []


def _gpus() -> int:
    if REHEARSAL:
        return REHEARSAL
    try:
        import torch

        return torch.cuda.device_count()
    except Exception:  # pragma: no cover
        return 0


pytestmark = [pytest.mark.gpu, pytest.mark.multigpu, pytest.mark.skipif(_gpus() < 2, reason="needs >= 2 GPUs")]

# Worst-case seconds of every test (the sum of its subprocess limits).
BUDGET_S = {
    "test_reference_matrix_all_gpus": 60,
    "test_concurrent_modes_all_gpus": 50,
    "test_bench_all_gpus": 95,
    "test_ipc_engines_all_gpus": 60,
    "test_fuzz_all_gpus": 35,
    "test_cli_fuzz_relay_all_gpus": 35,
    "test_bench_two_gpus_pair_sweep": 95,
    "test_fabric_is_uniform": 5,
}

# What the correctness tests measured, for test_fabric_is_uniform (the
# session's memory; also written under $P2P_TEST_LOG_DIR when set).
FABRIC = {}


def _keep(name, value):
    FABRIC[name] = value
    d = os.environ.get("P2P_TEST_LOG_DIR")
    if d:
        os.makedirs(d, exist_ok=True)
        with open(os.path.join(d, "fabric_%s.json" % name), "w") as f:
            json.dump(value, f)


@pytest.fixture(scope="module")
def exe():
    ensure_built("gpu")
    return os.path.join(ROOT, "build", "p2p_matrix")


def _n():
    return min(_gpus(), 8)


@pytest.mark.skipif(not os.path.exists(MPIRUN), reason="no mpirun")
def test_reference_matrix_all_gpus(exe, tmp_path):
    """The reference's two matrices (mpirun -n N ./p2p_matrix) over xGMI,
    every timed delivery verified in a receive generation of its own, and
    the transport RCCL used for every pair recorded: a pair with a direct
    xGMI link carried by anything but RCCL's P2P transport fails."""
    n = _n()
    js = tmp_path / "r.json"
    out = run_logged([MPIRUN, "-n", str(n), exe, "--verify", "-n", "16", "--json", str(js), "--timeout", "45",
                      "--min-gbs", MIN_GBS], BUDGET_S["test_reference_matrix_all_gpus"] * (2 if REHEARSAL >= 8 else 1),
                     "reference_matrix_all_gpus")
    assert out.returncode == 0, out.stderr[-3000:]
    m = parse_compat(out.stdout)
    for key in ("uni", "bi"):
        for i in range(n):
            for j in range(n):
                assert (m[key][i][j] == 0.0) == (i == j)
    assert "verification: OK" in out.stdout
    _keep("compat", m)
    recs = [json.loads(l) for l in js.read_text().splitlines()]
    assert all(r["verify_coverage"] == 1 for r in recs if r["type"] == "run")
    # Which RCCL transport carried each pair (RCCL's INFO log); --min-gbs
    # would have failed a direct xGMI pair carried by SHM or NET.
    links = [r for r in recs if r["type"] == "links"][0]
    assert [links["matrix_transport"][a][a] for a in range(n)] == ["self"] * n, links["matrix_transport"]
    assert "WRONG TRANSPORT" not in out.stderr


@pytest.mark.skipif(not os.path.exists(MPIRUN), reason="no mpirun")
def test_concurrent_modes_all_gpus(exe):
    """Tournament, ring and all-pairs, verified, with one RCCL communicator
    and with four (messages >= 1 MiB spread over them, side streams
    synchronised only around buffer work)."""
    n = _n()
    for comms in ("1", "4"):
        out = run_logged([MPIRUN, "-n", str(n), exe, "--comms", comms, "--mode", "tournament,ring,allpairs",
                          "--sizes", CONCURRENT_SIZES, "-n", "8", "--verify", "--latency", "--no-compat", "--timeout",
                          "60" if CONCURRENT_TIMEOUT_S else "20"],
                         CONCURRENT_TIMEOUT_S or BUDGET_S["test_concurrent_modes_all_gpus"] / 2,
                         "concurrent_modes_comms%s" % comms)
        assert out.returncode == 0, out.stderr[-3000:]
        assert "verification: OK" in out.stdout and "FAILED" not in out.stdout


def test_bench_all_gpus():
    n = _n()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n), "--master-addr",
           "127.0.0.1", "--master-port", str(free_port()), "bench.py", "--gpus", str(n), "--steps", "14",
           "--warmup", "7", "--deadline", "80", "--sweep-max", "256M", "--timeout", "45"] + BENCH_MSGS + ISOLATE
    out = run_logged(cmd, BUDGET_S["test_bench_all_gpus"], "bench_all_gpus", cwd=ROOT)
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    r = json.loads(lines[0]) if lines else {}
    progress = "\n".join(l for l in out.stderr.splitlines() if "bench:" in l or "fatal" in l or "Error" in l
                         or "Traceback" in l or "exitcode" in l)
    assert out.returncode == 0, (progress[-3000:], {k: r.get(k) for k in ("deadline_hit", "section_errors",
                                                                          "untimed_skipped", "verify_mismatches")})
    _keep("bench", {k: r.get(k) for k in ("matrix_gbs", "link_check", "unparsed_peers", "matrix_transport", "value",
                                          "aggregate_gbs", "timeline_s", "posting")})
    assert r["n_gpus"] == n and r["verify_mismatches"] == 0 and r["value"] > 0
    assert r["matrix_cells"] == "%d/%d" % (n * (n - 1), n * (n - 1))
    assert len(r["matrix_transport"]) == n


@pytest.mark.skipif(not os.path.exists(MPIRUN), reason="no mpirun")
def test_ipc_engines_all_gpus(exe):
    """The hand-written data plane across real xGMI links: pull (remote reads),
    push (rendezvous + remote writes) and relay (push + two-hop stripes through
    GPUs with idle links; the pair mode's single cells use every GPU),
    verified, plus the device ping-pong matrix."""
    n = _n()
    for engine in ("kernel", "push", "relay"):
        modes = "tournament,allpairs,pair" if engine == "relay" else "tournament,allpairs"
        out = run_logged([MPIRUN, "-n", str(n), exe, "--transport", "ipc", "--ipc-engine", engine,
                          "--mode", modes, "--sizes", "1M,64M", "-n", "4", "--verify",
                          "--device-latency", "--latency-iters", "200", "--no-compat", "--timeout", "15"],
                         BUDGET_S["test_ipc_engines_all_gpus"] / 3, "ipc_engines_%s" % engine)
        assert out.returncode == 0, (engine, out.stderr[-3000:])
        assert "verification: OK" in out.stdout and "FAILED" not in out.stdout
        assert "device-initiated ping-pong" in out.stdout


def test_fuzz_all_gpus():
    """Random verified message groups across every GPU through RCCL with four
    communicators per rank (both ends must route every message alike)."""
    n = _n()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n),
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), "tests/scripts/fuzz_session.py",
           "rccl:4", "20"]
    out = run_logged(cmd, BUDGET_S["test_fuzz_all_gpus"], "fuzz_all_gpus", cwd=ROOT)
    assert out.returncode == 0, out.stderr[-3000:]
    assert "FUZZ rccl:4 mismatches 0" in out.stdout


@pytest.mark.skipif(not os.path.exists(MPIRUN), reason="no mpirun")
def test_cli_fuzz_relay_all_gpus(exe):
    """p2p_matrix --fuzz across every GPU over the relay engine, whose stripes
    cross third GPUs: random groups (random pairs incl. self, 1 B .. 16 MiB)."""
    n = _n()
    out = run_logged([MPIRUN, "-n", str(n), exe, "--transport", "ipc", "--ipc-engine", "relay", "--mode", "pair",
                      "--size", "16M", "-n", "2", "--fuzz", "30", "--no-compat", "--timeout", "25"],
                     BUDGET_S["test_cli_fuzz_relay_all_gpus"], "cli_fuzz_relay_all_gpus")
    assert out.returncode == 0, out.stderr[-3000:]
    assert "all verified" in out.stdout


def test_bench_two_gpus_pair_sweep():
    """The driver's N = 2 bench on two distinct GPUs: the time left after the
    other sections goes to the xGMI pair sweep (on by default there), whose
    rows cross the real link, every one verified.  The other untimed sections
    are off here (test_bench_all_gpus runs them), so the sweep has the time:
    the one-GPU rehearsal with them on skipped it for lack of time."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(free_port()), "bench.py", "--gpus", "2", "--steps", "14", "--warmup", "7",
           "--deadline", "75", "--xgmi-sweep-sizes", "32M", "--ipc-extra", "0", "--extras", "0", "--sweep", "0",
           "--ref-iters", "0", "--latency-preposted", "0", "--latency-iters", "50",
           "--timeout", "45"] + BENCH_MSGS + (["--xgmi-sweep", "1"] if REHEARSAL else [])
    out = run_logged(cmd, BUDGET_S["test_bench_two_gpus_pair_sweep"], "bench_two_gpus_pair_sweep", cwd=ROOT)
    assert out.returncode == 0, out.stderr[-3000:]
    r = json.loads([l for l in out.stdout.splitlines() if l.startswith("{")][0])
    sw = r["xgmi_pair_sweep"]
    assert sw is not None, (r["untimed_skipped"], out.stderr[-2000:])
    assert sw["emulated"] == ("rccl" if REHEARSAL else None) and sw["rows"]["rccl-comms1"]["rc"] == 0, sw
    assert sw["best"] and sw["best_rccl"], sw


@pytest.mark.perf
def test_fabric_is_uniform():
    """the links the correctness tests above measured,
    checked for what a healthy fully connected xGMI node must show, with no
    hardware number: no off-diagonal cell of the bench's tournament matrix or
    of the reference's uni matrix below half the median cell (a degraded link,
    a mis-posted communicator), every bi cell (both directions summed,
    p2p_matrix.cc:258) at least its uni cell (:177), RCCL's P2P transport on
    every direct pair and every connected peer's RCCL lines parsed.  Reads
    what they kept and runs nothing; ordered with the perf floors."""
    if not FABRIC:
        pytest.skip("no multi-GPU measurement kept (those tests did not run or failed)")
    bench = FABRIC.get("bench") or {}
    compat = FABRIC.get("compat") or {}
    tour = bench.get("matrix_gbs")
    if tour:
        cells = offdiag(tour)
        PERF_RECORDS.update(xgmi_cell_min=round(min(cells), 2), xgmi_cell_mean=round(sum(cells) / len(cells), 2))
    # A rehearsal's "links" are RCCL sockets over loopback, 4-8 ranks sharing
    # one box's CPU: cells spread 2-4x and a bi cell can come in below its uni
    # cell (profiles/r5_reh8/), so it checks the flow with looser bounds.
    findings = fabric_findings(tour, compat.get("uni"), compat.get("bi"), bench.get("link_check"),
                               bench.get("unparsed_peers"), min_ratio=REHEARSAL_MIN_RATIO if REHEARSAL else 0.5,
                               bi_at_least_uni=not REHEARSAL)
    assert not findings, "\n".join(findings + ["tournament GB/s: %s" % tour, "compat uni Gbps: %s" % compat.get("uni"),
                                               "compat bi Gbps: %s" % compat.get("bi"),
                                               "transports: %s" % bench.get("matrix_transport")])

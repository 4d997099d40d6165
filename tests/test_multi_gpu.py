"""Tier T4: the RCCL data plane across real GPUs.  Runs only
where >= 2 MI355X are visible (skipped on the 1-GPU test boxes; the 8-GPU
scaling runs happen through bench.py on a full node)."""
import json
import os
import subprocess
import sys

import pytest

from conftest import MPIRUN, ROOT, ensure_built, free_port
from test_nccl_p2p_amd.utils.report import parse_compat


def _gpus() -> int:
    try:
        import torch

        return torch.cuda.device_count()
    except Exception:  # pragma: no cover
        return 0


pytestmark = [pytest.mark.gpu, pytest.mark.skipif(_gpus() < 2, reason="needs >= 2 GPUs")]


@pytest.fixture(scope="module")
def exe():
    ensure_built("gpu")
    return os.path.join(ROOT, "build", "p2p_matrix")


def _n():
    return min(_gpus(), 8)


@pytest.mark.skipif(not os.path.exists(MPIRUN), reason="no mpirun")
def test_reference_matrix_all_gpus(exe, tmp_path):
    n = _n()
    js = tmp_path / "r.json"
    out = subprocess.run([MPIRUN, "-n", str(n), exe, "--verify", "-n", "16", "--json", str(js)],
                         capture_output=True, text=True, timeout=900)
    assert out.returncode == 0, out.stderr[-3000:]
    m = parse_compat(out.stdout)
    for key in ("uni", "bi"):
        for i in range(n):
            for j in range(n):
                assert (m[key][i][j] == 0.0) == (i == j)
    assert "verification: OK" in out.stdout


@pytest.mark.skipif(not os.path.exists(MPIRUN), reason="no mpirun")
def test_concurrent_modes_all_gpus(exe):
    n = _n()
    out = subprocess.run([MPIRUN, "-n", str(n), exe, "--mode", "tournament,ring,allpairs", "--sizes", "1M,256M",
                          "-n", "8", "--verify", "--latency", "--no-compat"], capture_output=True, text=True, timeout=900)
    assert out.returncode == 0, out.stderr[-3000:]
    assert "verification: OK" in out.stdout and "FAILED" not in out.stdout


def test_bench_all_gpus():
    n = _n()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n), "--master-addr",
           "127.0.0.1", "--master-port", str(free_port()), "bench.py", "--gpus", str(n), "--steps", "14",
           "--warmup", "7"]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=900, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-3000:]
    r = json.loads([l for l in out.stdout.splitlines() if l.startswith("{")][0])
    assert r["n_gpus"] == n and r["verify_mismatches"] == 0
    assert r["matrix_cells"] == "%d/%d" % (n * (n - 1), n * (n - 1))


@pytest.mark.skipif(not os.path.exists(MPIRUN), reason="no mpirun")
@pytest.mark.parametrize("engine", ["kernel", "push", "relay"])
def test_ipc_engines_all_gpus(exe, engine):
    """The hand-written data plane across real xGMI links: pull (remote reads),
    push (rendezvous + remote writes) and relay (push + two-hop stripes through
    GPUs with idle links; the pair mode's single cells use every GPU),
    verified, plus the device ping-pong matrix."""
    n = _n()
    modes = "tournament,allpairs,pair" if engine == "relay" else "tournament,allpairs"
    out = subprocess.run([MPIRUN, "-n", str(n), exe, "--transport", "ipc", "--ipc-engine", engine,
                          "--mode", modes, "--sizes", "1M,256M", "-n", "8", "--verify",
                          "--device-latency", "--latency-iters", "200", "--no-compat", "--timeout", "120"],
                         capture_output=True, text=True, timeout=900)
    assert out.returncode == 0, out.stderr[-3000:]
    assert "verification: OK" in out.stdout and "FAILED" not in out.stdout
    assert "device-initiated ping-pong" in out.stdout


@pytest.mark.skipif(not os.path.exists(MPIRUN), reason="no mpirun")
def test_several_communicators_all_gpus(exe):
    """--comms 4 across real xGMI links: messages >= 1 MiB spread over four
    RCCL communicators per rank (side streams synchronised only around buffer
    work), every mode verified."""
    n = _n()
    out = subprocess.run([MPIRUN, "-n", str(n), exe, "--comms", "4", "--mode", "pair,tournament,ring,allpairs",
                          "--sizes", "64K,1M,256M", "-n", "8", "--verify", "--no-compat", "--timeout", "120"],
                         capture_output=True, text=True, timeout=900)
    assert out.returncode == 0, out.stderr[-3000:]
    assert "verification: OK" in out.stdout and "FAILED" not in out.stdout


def test_fuzz_all_gpus():
    """Random verified message groups across every GPU through RCCL with one
    and with four communicators per rank."""
    n = _n()
    for transport in ("rccl", "rccl:4"):
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n),
               "--master-addr", "127.0.0.1", "--master-port", str(free_port()), "tests/scripts/fuzz_session.py",
               transport, "20"]
        out = subprocess.run(cmd, capture_output=True, text=True, timeout=900, cwd=ROOT)
        assert out.returncode == 0, out.stderr[-3000:]
        assert "FUZZ %s mismatches 0" % transport in out.stdout


@pytest.mark.skipif(not os.path.exists(MPIRUN), reason="no mpirun")
@pytest.mark.parametrize("args", [["--comms", "4"], ["--transport", "ipc", "--ipc-engine", "relay"]])
def test_cli_fuzz_all_gpus(exe, args):
    """p2p_matrix --fuzz across every GPU: random groups (random pairs incl.
    self, 1 B .. 64 MiB) over four RCCL communicators, and over the relay
    engine, whose stripes cross third GPUs."""
    n = _n()
    out = subprocess.run([MPIRUN, "-n", str(n), exe] + args + ["--mode", "pair", "--size", "64M", "-n", "2",
                                                                "--fuzz", "40", "--no-compat", "--timeout", "120"],
                         capture_output=True, text=True, timeout=900)
    assert out.returncode == 0, out.stderr[-3000:]
    assert "all verified" in out.stdout


def test_bench_two_gpus_pair_sweep():
    """The driver's N = 2 bench on two distinct GPUs: after the other sections
    the time left goes to the xGMI pair sweep (on by default there), whose
    rows cross the real link, every one verified."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(free_port()), "bench.py", "--gpus", "2", "--steps", "14", "--warmup", "7"]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=900, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-3000:]
    r = json.loads([l for l in out.stdout.splitlines() if l.startswith("{")][0])
    sw = r["xgmi_pair_sweep"]
    assert sw["emulated"] is None and sw["rows"]["rccl-comms1"]["rc"] == 0, sw
    assert sw["best"] and sw["best_rccl"], sw

import functools
import os
import shutil
import subprocess
import sys
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

MPIRUN = os.environ.get("P2P_MPIRUN", "/opt/conda/bin/mpirun")


# The driver runs the whole `pytest -m gpu` session as one 900 s step.  A
# multi-GPU test (tests/test_multi_gpu.py, each with a worst-case BUDGET_S)
# starts only if the session's elapsed time plus that worst case still ends
# by SESSION_LIMIT_S; the remaining 60 s are for the perf floors, which run
# last.  tests/test_scripts_cpu.py checks the measured single-GPU duration +
# the sum of the budgets against the same limit.
SESSION_LIMIT_S = 840.0
_SESSION_T0 = [time.monotonic()]


@functools.lru_cache(maxsize=None)
def _gpu_count() -> int:
    try:
        import torch

        return torch.cuda.device_count()  # does not initialise HIP on this image
    except Exception:  # pragma: no cover
        return 0


def pytest_sessionstart(session):
    _SESSION_T0[0] = time.monotonic()
    if os.environ.get("P2P_REHEARSE_MULTI_GPU"):
        # tests/test_multi_gpu.py rehearsed on one GPU: every rank on device 0
        # (p2p_matrix: P2P_DEVICE; bench.py: LOCAL_RANK mod the visible GPUs;
        # the fuzz script: P2P_FUZZ_DEVICE), each rank an RCCL host of its own.
        os.environ.update(P2P_DEVICE="0", P2P_FUZZ_DEVICE="0", P2P_RCCL_DISTINCT_HOSTS="1",
                          NCCL_SOCKET_IFNAME="lo", NCCL_IB_DISABLE="1")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an AMD MI355X (gfx950) GPU")
    config.addinivalue_line("markers", "mpi: needs the MPICH mpirun launcher")
    config.addinivalue_line("markers", "multigpu: needs >= 2 GPUs; starts only within SESSION_LIMIT_S")
    config.addinivalue_line("markers", "perf: a performance floor; ordered after every correctness test")
    config.addinivalue_line("markers", "emulated: several ranks on one GPU; skipped where the multi-GPU tier "
                                       "runs the same flow across real GPUs")


def tier_rank(item) -> int:
    """Run order: single-GPU / CPU correctness, then the multi-GPU tier, then
    the perf floors (a floor miss under -x cannot hide a correctness test)."""
    if item.get_closest_marker("perf") is not None:
        return 2
    if item.get_closest_marker("multigpu") is not None:
        return 1
    return 0


def pytest_collection_modifyitems(session, config, items):
    items.sort(key=tier_rank)  # stable: file and definition order within a tier


# The perf floors' measurements (tests/test_zz_perf_floors_gpu.py record(),
# tests/test_multi_gpu.py), kept in memory so the session's last lines carry
# them whether the floors pass or not: the driver keeps only the tail of a
# GPU tier's output, and a passing test's prints are captured (VERDICT r4
# item 4).  name -> value; the PERF line prints them in insertion order.
PERF_RECORDS = {}


def perf_line(records) -> str:
    """One line: PERF k=v ... (kernels in TB/s, RCCL steps in GB/s)."""
    return "PERF " + " ".join("%s=%s" % (k, ("%.4g" % v) if isinstance(v, float) else v)
                              for k, v in records.items())


def pytest_terminal_summary(terminalreporter, exitstatus, config):
    if PERF_RECORDS:
        terminalreporter.write_line(perf_line(PERF_RECORDS))


def pytest_runtest_setup(item):
    if item.get_closest_marker("emulated") is not None and _gpu_count() >= 2:
        pytest.skip("one-GPU emulation: tests/test_multi_gpu.py runs this flow across the real GPUs here")
    if item.get_closest_marker("multigpu") is None:
        return
    budget = getattr(item.module, "BUDGET_S", {}).get(item.originalname)
    if budget is None:
        pytest.fail("multi-GPU test without a BUDGET_S entry")
    elapsed = time.monotonic() - _SESSION_T0[0]
    if elapsed + budget > SESSION_LIMIT_S:
        pytest.skip("%.0f s into the session, %s's worst case (%d s) would pass the %.0f s limit of the driver's "
                    "GPU-test step" % (elapsed, item.originalname, budget, SESSION_LIMIT_S))


def run_logged(cmd, timeout, name="child", **kw):
    """subprocess.run(cmd, capture_output=True, text=True, timeout=...) whose
    stderr and stdout also land, as they are written, in
    $P2P_TEST_LOG_DIR/<name>.log and <name>.out when that is set (the GPU
    sessions set it under gpurun_out/): a long run inside a test shows its
    progress there instead of looking silent."""
    log_dir = os.environ.get("P2P_TEST_LOG_DIR")
    if not log_dir:
        return subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, **kw)
    os.makedirs(log_dir, exist_ok=True)
    err_path = os.path.join(log_dir, "%s.log" % name)
    out_path = os.path.join(log_dir, "%s.out" % name)
    with open(err_path, "w") as err, open(out_path, "w") as out:
        proc = subprocess.Popen(cmd, stdout=out, stderr=err, text=True, **kw)
        try:
            proc.wait(timeout=timeout)
        except subprocess.TimeoutExpired:
            proc.kill()
            proc.wait()
            raise
    with open(err_path) as fe, open(out_path) as fo:
        return subprocess.CompletedProcess(cmd, proc.returncode, fo.read(), fe.read())


def ensure_built(target: str) -> None:
    """Builds a Makefile target in-tree if its artefact is missing."""
    subprocess.run(["make", "-C", ROOT, "-j8", target], check=True, capture_output=True)


@pytest.fixture(scope="session")
def host_build():
    ensure_built("host")
    return os.path.join(ROOT, "build")


@pytest.fixture(scope="session")
def native():
    ensure_built("ext")
    import test_nccl_p2p_amd

    return test_nccl_p2p_amd.require_native()


@pytest.fixture(scope="session")
def mpirun():
    if not (os.path.exists(MPIRUN) or shutil.which("mpirun")):
        pytest.skip("mpirun not available")
    return MPIRUN if os.path.exists(MPIRUN) else shutil.which("mpirun")


def free_port() -> int:
    """A port P with P and P + 1 both free: torchrun's store takes P and the
    native TCP bootstrap listens on MASTER_PORT + 1 (csrc/bootstrap.cpp).

    Drawn at random below Linux's ephemeral range (32768-60999): a port the
    kernel handed out for bind(0) is also what outgoing connections use, so
    between this check and the launcher's bind another process's client
    socket could take it (EADDRINUSE in the GPU tier)."""
    import random
    import socket

    rng = random.Random()
    for _ in range(256):
        p = rng.randrange(20000, 32000)
        socks = []
        try:
            for q in (p, p + 1):
                t = socket.socket()
                socks.append(t)
                t.bind(("127.0.0.1", q))
            return p
        except OSError:
            continue
        finally:
            for t in socks:
                t.close()
    raise RuntimeError("no free port pair in 20000-32000")

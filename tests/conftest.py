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


# The multi-GPU tier (tests/test_multi_gpu.py) shares the driver's 900 s
# `pytest -m gpu` step with the single-GPU tests (~260 s): once it has used
# this much, its remaining tests are skipped with a reason.
MULTI_GPU_TIER_S = 550.0
_MULTI_GPU_T0 = []


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an AMD MI355X (gfx950) GPU")
    config.addinivalue_line("markers", "mpi: needs the MPICH mpirun launcher")
    config.addinivalue_line("markers", "multigpu: needs >= 2 GPUs; shares the MULTI_GPU_TIER_S budget")


def pytest_runtest_setup(item):
    if item.get_closest_marker("multigpu") is None:
        return
    if not _MULTI_GPU_T0:
        _MULTI_GPU_T0.append(time.monotonic())
    elif time.monotonic() - _MULTI_GPU_T0[0] > MULTI_GPU_TIER_S:
        pytest.skip("the multi-GPU tier used its %.0f s of the driver's GPU-test step" % MULTI_GPU_TIER_S)


def run_logged(cmd, timeout, name="child", **kw):
    """subprocess.run(cmd, capture_output=True, text=True, timeout=...) whose
    stderr also lands, as it is written, in $P2P_TEST_LOG_DIR/<name>.log when
    that is set (the GPU sessions set it under gpurun_out/): a long bench run
    inside a test shows its progress there instead of looking silent."""
    log_dir = os.environ.get("P2P_TEST_LOG_DIR")
    if not log_dir:
        return subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, **kw)
    os.makedirs(log_dir, exist_ok=True)
    path = os.path.join(log_dir, "%s.log" % name)
    with open(path, "w") as err:
        proc = subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=err, text=True, **kw)
        try:
            out, _ = proc.communicate(timeout=timeout)
        except subprocess.TimeoutExpired:
            proc.kill()
            proc.communicate()
            raise
    with open(path) as f:
        return subprocess.CompletedProcess(cmd, proc.returncode, out, f.read())


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

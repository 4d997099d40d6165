"""Tier T0: the C++ host unit tests (csrc/ logic without a GPU)."""
import os
import subprocess


def test_native_host_unit_tests(host_build):
    exe = os.path.join(host_build, "p2p_host_tests")
    out = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stdout[-4000:] + out.stderr[-4000:]
    assert " 0 failures" in out.stdout


def test_host_code_under_asan_ubsan(mpirun):
    """Host code under AddressSanitizer + UBSan (SURVEY.md §5 race detection /
    sanitizers row): the unit tests, then 3-rank MPI jobs over the TCP and
    shared-memory transports through every mode with verification and
    latency."""
    from conftest import ROOT
    out = subprocess.run(["make", "-j2", "asan"], cwd=ROOT, capture_output=True, text=True, timeout=900)
    assert out.returncode == 0, out.stdout[-4000:] + out.stderr[-4000:]
    assert " 0 failures" in out.stdout
    exe = os.path.join(ROOT, "build", "asan", "p2p_matrix_host")
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0", UBSAN_OPTIONS="print_stacktrace=1")
    for transport, sizes in (("host", "4K:64K:4"), ("shm", "4K,2M")):
        # shm: 2 MiB messages wrap the 1 MiB rings, under the sanitizers too.
        run = subprocess.run([mpirun, "-n", "3", exe, "--transport", transport, "--mode", "all", "--sizes", sizes,
                              "-n", "3", "--verify", "--latency", "--latency-iters", "20"],
                             capture_output=True, text=True, timeout=300, env=env)
        assert run.returncode == 0, run.stderr[-4000:]
        assert "AddressSanitizer" not in run.stderr and "runtime error" not in run.stderr
        assert "verification: OK" in run.stdout


def test_host_code_under_tsan(mpirun):
    """Host code under ThreadSanitizer (SURVEY.md §5 race detection row): the
    unit tests run every rank of a multi-rank case as a thread of one process
    (bootstrap collectives, the TCP and shared-memory transports, abort_if_idle
    against in-flight native calls), so a race between ranks, the abort path
    and the logging fails the run (halt_on_error); then 3-rank MPI jobs of the
    host binary over both CPU transports."""
    from conftest import ROOT
    out = subprocess.run(["make", "-j2", "tsan"], cwd=ROOT, capture_output=True, text=True, timeout=900)
    assert out.returncode == 0, out.stdout[-4000:] + out.stderr[-4000:]
    assert " 0 failures" in out.stdout and "ThreadSanitizer" not in out.stdout + out.stderr
    exe = os.path.join(ROOT, "build", "tsan", "p2p_matrix_host")
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1")
    for transport in ("host", "shm"):
        run = subprocess.run([mpirun, "-n", "3", exe, "--transport", transport, "--mode", "all", "--sizes", "4K,2M",
                              "-n", "3", "--verify", "--latency", "--latency-iters", "20"],
                             capture_output=True, text=True, timeout=300, env=env)
        assert run.returncode == 0, run.stderr[-4000:]
        assert "ThreadSanitizer" not in run.stderr
        assert "verification: OK" in run.stdout

"""Tier T0: the C++ host unit tests (csrc/ logic without a GPU)."""
import os
import subprocess


def test_native_host_unit_tests(host_build):
    exe = os.path.join(host_build, "p2p_host_tests")
    out = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stdout[-4000:] + out.stderr[-4000:]
    assert " 0 failures" in out.stdout

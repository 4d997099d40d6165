"""The Python API tour (examples/python_api.py) runs as documented."""
import os
import subprocess
import sys

import pytest

from conftest import ROOT

EXAMPLE = os.path.join(ROOT, "examples", "python_api.py")


def test_python_api_example_host(native):
    out = subprocess.run([sys.executable, EXAMPLE, "--transport", "host"], capture_output=True, text=True,
                         timeout=300, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-3000:]
    assert "tournament GB/s" in out.stdout and "mismatches 0" in out.stdout


@pytest.mark.gpu
def test_python_api_example_rccl(native):
    out = subprocess.run([sys.executable, EXAMPLE, "--transport", "rccl"], capture_output=True, text=True,
                         timeout=300, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-3000:]
    assert "verify:" in out.stdout and "mismatches 0" in out.stdout

"""Loader for the in-tree native extension ``_p2pcore``.

The extension is built in-tree by ``make ext`` (or ``__graft_entry__.build()``).
There is deliberately no pure-Python fallback for the data plane: on a GPU box
a missing extension must fail loudly instead of silently measuring something
else.
"""

from __future__ import annotations

import importlib
import os
import subprocess
import sys

_mod = None
_err: Exception | None = None

REPO_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _load():
    global _mod, _err
    if _mod is not None or _err is not None:
        return
    try:
        _mod = importlib.import_module("test_nccl_p2p_amd._p2pcore")
    except ImportError as e:  # pragma: no cover - depends on the build
        _err = e


def native_available() -> bool:
    _load()
    return _mod is not None


def build_native(quiet: bool = True) -> None:
    """Builds the extension and the executables in-tree with make."""
    cmd = ["make", "-C", REPO_ROOT, "-j8", "all"]
    out = subprocess.run(cmd, capture_output=quiet, text=True)
    if out.returncode != 0:
        raise RuntimeError("native build failed:\n" + (out.stdout or "") + (out.stderr or ""))
    global _err
    _err = None
    _load()


def require_native():
    """Returns the extension module or raises with build instructions."""
    _load()
    if _mod is None:
        raise ImportError(
            "test_nccl_p2p_amd._p2pcore is not built (run `make ext` in %s): %s" % (REPO_ROOT, _err)
        )
    return _mod


def native():
    return require_native()


if __name__ == "__main__":  # pragma: no cover
    build_native(quiet=False)
    print(require_native().__file__, file=sys.stderr)

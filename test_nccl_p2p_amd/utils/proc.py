"""Child processes that cannot outlive the run that started them.

bench.py starts its untimed comparisons and the xGMI pair sweep as child jobs
in sessions of their own, so that a timeout can kill a job's whole tree
(launcher, proxies, ranks) with one killpg.  A session of its own also takes
the child out of the launcher's process group, though: should the driver kill
the bench (its process group) the child would keep driving a GPU.  The child
therefore asks the kernel to kill it when its parent goes (PR_SET_PDEATHSIG),
and checks that the parent it was started for is still the one it has, for
the case where the parent died before the request took effect.
"""
from __future__ import annotations

import os
import shutil
import signal
import subprocess

PARENT_ENV = "P2P_PARENT_PID"
_PR_SET_PDEATHSIG = 1


def child_env(env=None) -> dict:
    """The environment for a child that should die with this process."""
    return dict(os.environ if env is None else env, **{PARENT_ENV: str(os.getpid())})


def die_with_parent() -> bool:
    """In a child started with child_env(): SIGKILL when the parent exits
    (Linux; a no-op elsewhere or without the variable).  Exits at once if the
    parent is already gone.  True when the request is in place."""
    expected = os.environ.get(PARENT_ENV)
    if not expected:
        return False
    try:
        import ctypes

        libc = ctypes.CDLL(None, use_errno=True)
        if libc.prctl(_PR_SET_PDEATHSIG, int(signal.SIGKILL), 0, 0, 0) != 0:
            return False
    except (OSError, AttributeError):
        return False
    if os.getppid() != int(expected):
        os._exit(1)
    return True


def pdeathsig_prefix() -> list:
    """Command prefix giving a launched program the same guarantee
    (util-linux setpriv), or [] where setpriv is missing."""
    exe = shutil.which("setpriv")
    return [exe, "--pdeathsig", "KILL"] if exe else []


def run_child(state: dict, cmd, timeout: float, **kw):
    """Runs `cmd` in a session of its own (one killpg takes its whole tree
    down) with child_env(), registered in state["children"] while it runs so
    that a watchdog can kill_children(state) before ending the process; at
    `timeout` the same happens here.  Returns the exit status, or "timeout"."""
    proc = subprocess.Popen(cmd, start_new_session=True, env=child_env(kw.pop("env", None)), **kw)
    state.setdefault("children", []).append(proc)
    try:
        return proc.wait(timeout=timeout)
    except subprocess.TimeoutExpired:
        kill_children(state, [proc])
        return "timeout"
    finally:
        state["children"].remove(proc)


def kill_children(state: dict, procs=None) -> None:
    """SIGKILL to the sessions of `procs` (default: every registered child)."""
    for proc in list(procs if procs is not None else state.get("children", [])):
        try:
            os.killpg(proc.pid, signal.SIGKILL)
        except (ProcessLookupError, PermissionError):
            pass
        proc.wait()

"""bench.py's fault-injection hooks, read from the environment once.

The measured flow (bench/headline.py, bench/sections.py, bench.py) reads no
hook variable itself: it holds one Faults object and calls a named point --
fail_headline, candidate, candidate_fail, section, teardown -- which does
nothing unless its variable asked for it.  The reference's whole error
policy is three check macros (p2p_matrix.cc:15-42); these hooks exist so the
tests can drive every bounded wait and fallback of the bench (a candidate
that fails or hangs, a hung section, a rank that leaves during teardown)
without touching the measured code.

The variables (docs/ENVIRONMENT.md):
  P2P_BENCH_FAIL_HEADLINE=<transport>       the headline through <transport>
                                            fails on every rank
  P2P_BENCH_FAIL_CANDIDATE=<c>,<b>[,tuning] posting candidate (c comms, batch
                                            b) fails on the last rank, in its
                                            connect (or its tuning pass)
  P2P_BENCH_HANG=<spec>[;<spec>...]         <section>@<rank>: that rank stops
                                            inside the untimed section;
                                            teardown@<rank>: that rank exits in
                                            the teardown; candidate:...: see
                                            candidate_hang
"""

from __future__ import annotations

import os
import time

HANG_KINDS = ("tuning", "connect", "stall", "unbounded")


def _hang_specs(spec=None):
    raw = os.environ.get("P2P_BENCH_HANG", "") if spec is None else spec
    return [s for s in raw.split(";") if s]


def hang_requested(section: str, rank: int, spec=None) -> bool:
    """P2P_BENCH_HANG="<section>@<rank>": that rank stops responding inside
    that untimed section (`spec`: the variable's value, else the
    environment's)."""
    return "%s@%d" % (section, rank) in _hang_specs(spec)


def candidate_hang(transport: str, comms: int, batch: int, rank: int, spec=None):
    """P2P_BENCH_HANG="candidate:[<transport>:]<comms>,<batch>[:<how>]@<rank>"
    (several, separated by ';') makes that rank misbehave in that posting
    candidate.  Returns <how> for this rank and candidate, else None:
      tuning (default): in the first tuning pass it posts nothing, as a peer
                whose transfer never completes, and its own wait ends only at
                its session's timeout (the candidate's budget);
      connect:  the same in the candidate's connect;
      stall:    in the first tuning pass it stops in Python, outside the
                engine (the deadline watchdog aborts the communicators
                itself, abort_if_idle);
      unbounded: its session's timeout is lifted for the first tuning pass,
                which it runs as usual: next to a stalled peer it waits
                inside the transport until the watchdog's cooperative abort."""
    for s in _hang_specs(spec):
        if not s.startswith("candidate:") or "@" not in s:
            continue
        what, at = s[len("candidate:"):].rsplit("@", 1)
        parts = what.split(":")
        how = parts.pop() if parts and parts[-1] in HANG_KINDS else "tuning"
        if len(parts) == 2:
            if parts[0] != transport:
                continue
            parts = parts[1:]
        if len(parts) == 1 and parts[0] == "%d,%d" % (comms, batch) and at == str(rank):
            return how
    return None


def emulate_hang(seconds: float, how: str = "tuning"):
    """A candidate hang (candidate_hang): this rank posts nothing and waits as
    a transport wait that never completes does, until its session's timeout
    (the candidate's budget), then fails; or ("stall") stops outside the
    engine for good."""
    from test_nccl_p2p_amd.bench.core import log

    if how == "stall":
        log("bench: injected stall outside the engine")
        while True:
            time.sleep(1.0)
    log("bench: injected hang for the candidate's budget (%.1f s)" % seconds)
    time.sleep(seconds)
    raise RuntimeError("injected hang: no progress within %.1f s" % seconds)


class Faults:
    """Every bench hook of this process, read once (see the module doc)."""

    def __init__(self, rank: int = 0, world: int = 1, environ=None):
        env = os.environ if environ is None else environ
        self.rank, self.world = rank, world
        self.headline_transport = env.get("P2P_BENCH_FAIL_HEADLINE") or None
        self.fail_candidate = env.get("P2P_BENCH_FAIL_CANDIDATE") or None
        self.hang_spec = env.get("P2P_BENCH_HANG", "")

    def fail_headline(self, transport: str):
        """The headline through `transport` fails on every rank, as a
        communicator that cannot be set up does."""
        if self.headline_transport == transport:
            raise RuntimeError("injected headline failure")

    def candidate(self, transport: str, comms: int, batch: int):
        """How this rank misbehaves in that posting candidate (candidate_hang),
        or None."""
        return candidate_hang(transport, comms, batch, self.rank, self.hang_spec)

    def candidate_fail(self, comms: int, batch: int, phase: str):
        """Fails posting candidate (comms, batch) on the last rank in `phase`
        ("connect" or "tuning")."""
        want = "%d,%d" % (comms, batch) + ("" if phase == "connect" else "," + phase)
        if self.fail_candidate == want and self.rank == self.world - 1:
            raise RuntimeError("injected %s" % ("candidate failure" if phase == "connect" else phase + " failure"))

    def section(self, name: str):
        """This rank stops responding inside untimed section `name`."""
        if hang_requested(name, self.rank, self.hang_spec):
            from test_nccl_p2p_amd.bench.core import log

            log("bench: injected hang in %s on rank %d" % (name, self.rank))
            while True:
                time.sleep(1)

    def teardown(self):
        """This rank ends in the teardown, as one whose watchdog fired a little
        before the others' (its process started earlier)."""
        if hang_requested("teardown", self.rank, self.hang_spec):
            from test_nccl_p2p_amd.bench.core import log

            log("bench: injected exit in the teardown on rank %d" % self.rank)
            os._exit(0)

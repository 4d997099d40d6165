"""Pure-Python mirror of ``csrc/schedule.cpp``.

Used by the torch.distributed (gloo / nccl) harness, and cross-checked against
the native schedules in the test suite so both engines run identical
communication patterns.  Modes (see csrc/schedule.hpp for the rationale):

* ``pair``       — the reference's serial (src, dst) cells, row-major, diagonal
                   idle (/root/reference/p2p_matrix.cc:141-152, 196-207)
* ``ring``       — r -> r+1 (bi adds r -> r-1): pipeline-parallel hops
* ``allpairs``   — every rank to every peer in one group: EP all-to-all
* ``tournament`` — round-robin rounds of disjoint pairs
* ``self``       — each rank to itself
"""

from __future__ import annotations

from dataclasses import dataclass, field
from typing import List, Tuple

MODES = ("pair", "ring", "allpairs", "tournament", "self")


@dataclass
class Phase:
    label: str
    n: int
    row: int = -1
    col: int = -1
    idle: bool = False
    flows: List[Tuple[int, int]] = field(default_factory=list)
    send_to: List[List[int]] = field(default_factory=list)
    recv_from: List[List[int]] = field(default_factory=list)

    def __post_init__(self):
        if not self.send_to:
            self.send_to = [[] for _ in range(self.n)]
            self.recv_from = [[] for _ in range(self.n)]

    def add(self, src: int, dst: int) -> None:
        self.send_to[src].append(dst)
        self.recv_from[dst].append(src)
        self.flows.append((src, dst))

    def participates(self, r: int) -> bool:
        return bool(self.send_to[r] or self.recv_from[r])


def round_robin_rounds(n: int) -> List[List[Tuple[int, int]]]:
    """Circle-method 1-factorisation; identical to p2p::round_robin_rounds."""
    if n < 2:
        return []
    m = n if n % 2 == 0 else n + 1
    fixed = m - 1
    rounds = []
    for r in range(m - 1):
        pairs = []

        def push(a, b):
            if a < n and b < n:
                pairs.append((min(a, b), max(a, b)))

        push(fixed, r)
        for k in range(1, m // 2):
            push((r + k) % (m - 1), (r - k + (m - 1)) % (m - 1))
        rounds.append(sorted(pairs))
    return rounds


def _self(n: int) -> List[Phase]:
    p = Phase("self", n)
    for r in range(n):
        p.add(r, r)
    return [p]


def make_schedule(mode: str, direction: str, n: int) -> List[Phase]:
    if mode not in MODES:
        raise ValueError("unknown mode %r" % mode)
    if direction not in ("uni", "bi"):
        raise ValueError("direction must be uni or bi")
    if mode == "self" or (n == 1 and mode in ("ring", "allpairs", "tournament")):
        return _self(n)
    phases: List[Phase] = []
    if mode == "pair":
        for src in range(n):
            for dst in range(n):
                p = Phase("%d->%d" % (src, dst), n, row=src, col=dst)
                if src == dst:
                    p.idle = True
                else:
                    p.add(src, dst)
                    if direction == "bi":
                        p.add(dst, src)
                phases.append(p)
    elif mode == "ring":
        p = Phase("ring+1" if direction == "uni" else "ring+-1", n)
        for r in range(n):
            p.add(r, (r + 1) % n)
        if direction == "bi" and n > 2:
            for r in range(n):
                p.add(r, (r + n - 1) % n)
        phases.append(p)
    elif mode == "allpairs":
        p = Phase("all-pairs", n)
        for k in range(1, n):
            for r in range(n):
                p.add(r, (r + k) % n)
        phases.append(p)
    elif mode == "tournament":
        for i, rnd in enumerate(round_robin_rounds(n)):
            if direction == "bi":
                p = Phase("round %d" % i, n)
                for a, b in rnd:
                    p.add(a, b)
                    p.add(b, a)
                phases.append(p)
            else:
                up, down = Phase("round %d a" % i, n), Phase("round %d b" % i, n)
                for a, b in rnd:
                    up.add(a, b)
                    down.add(b, a)
                phases += [up, down]
    return phases

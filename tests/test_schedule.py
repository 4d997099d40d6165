"""Schedules: Python mirror == native, and the structural properties the
measurement relies on (reference order, disjoint tournament rounds)."""
import itertools

import pytest

from test_nccl_p2p_amd.parallel.schedule import MODES, make_schedule, round_robin_rounds


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("direction", ["uni", "bi"])
def test_python_matches_native(native, mode, direction):
    for n in range(1, 10):
        py = [(p.label, p.row, p.col, p.idle, p.flows, list(zip(p.send_to, p.recv_from)))
              for p in make_schedule(mode, direction, n)]
        nat = [(p["label"], p["row"], p["col"], p["idle"], [tuple(f) for f in p["flows"]],
                [tuple(r) for r in p["ranks"]]) for p in native.schedule(mode, direction, n)]
        assert py == nat, (mode, direction, n)


def test_pair_is_reference_row_major():
    ph = make_schedule("pair", "uni", 4)
    assert [(p.row, p.col) for p in ph] == list(itertools.product(range(4), range(4)))
    assert [p.idle for p in ph] == [r == c for r, c in itertools.product(range(4), range(4))]


@pytest.mark.parametrize("n", [2, 3, 4, 5, 8, 16])
def test_round_robin(n):
    rounds = round_robin_rounds(n)
    seen = set()
    for r in rounds:
        ranks = [x for p in r for x in p]
        assert len(ranks) == len(set(ranks))
        seen.update(r)
    assert seen == set(itertools.combinations(range(n), 2))
    assert len(rounds) == (n - 1 if n % 2 == 0 else n)


def test_tournament_bi_is_perfect_matching_for_8():
    for p in make_schedule("tournament", "bi", 8):
        assert len(p.flows) == 8
        assert all(len(p.send_to[r]) == 1 and len(p.recv_from[r]) == 1 for r in range(8))


def test_allpairs_slots():
    p = make_schedule("allpairs", "bi", 8)[0]
    assert len(p.flows) == 56
    assert all(sorted(p.recv_from[r]) == [x for x in range(8) if x != r] for r in range(8))


def test_plan_routes_binding(native):
    """The relay engine's route planner through the Python binding: a single
    pair on 8 ranks gets the direct link + 6 relays in equal 4 KiB-aligned
    shares; a bi-directional tournament round gets 6 half-share relays per
    flow; all-pairs is never relayed; small messages stay direct."""
    size = 32 << 20
    (single,) = native.plan_routes(8, [(0, 1)], size)
    assert [s[0] for s in single][0] == -1 and sorted(s[0] for s in single[1:]) == [2, 3, 4, 5, 6, 7]
    assert sum(s[2] for s in single) == size and all(s[2] % 4096 == 0 for s in single[1:])
    spans = sorted((s[1], s[2]) for s in single)
    assert spans[0][0] == 0 and all(a[0] + a[1] == b[0] for a, b in zip(spans, spans[1:]))
    assert all(s[1] % 4096 == 0 for s in single) and single[0][1] + single[0][2] == size
    (odd,) = native.plan_routes(4, [(3, 1)], 1822205)  # unaligned: stripes still start aligned
    assert all(s[1] % 4096 == 0 for s in odd) and sum(s[2] for s in odd) == 1822205
    rnd = [(0, 1), (1, 0), (2, 3), (3, 2), (4, 5), (5, 4), (6, 7), (7, 6)]
    for plan in native.plan_routes(8, rnd, size):
        assert len(plan) == 7 and plan[0][2] > 1.5 * plan[1][2]
    allp = [(a, b) for a in range(4) for b in range(4) if a != b]
    assert all(len(p) == 1 for p in native.plan_routes(4, allp, size))
    assert len(native.plan_routes(8, [(0, 1)], 64 << 10)[0]) == 1
    assert len(native.plan_routes(8, [(0, 1)], size, max_relays=2)[0]) == 3

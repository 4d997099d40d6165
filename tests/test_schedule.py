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

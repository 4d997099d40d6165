"""Property-based checks (hypothesis) of the native host helpers every
measurement rests on: the relay route planner, the schedules, the payload
PRNG fill/verify pair, block placement and size parsing.  Each property is
checked on the C++ code through the extension (csrc/routing.cpp,
csrc/schedule.cpp, csrc/transport_host.cpp, csrc/bootstrap.cpp,
csrc/units.cpp); the example-based tests pin specific cases."""
import collections

import pytest

hypothesis = pytest.importorskip("hypothesis")
from hypothesis import given, settings, strategies as st  # noqa: E402

SETTINGS = settings(max_examples=150, deadline=None)


@st.composite
def groups(draw):
    """(n, flows, bytes): a group of directed flows, duplicates and self
    flows allowed, with message sizes around the relay threshold."""
    n = draw(st.integers(1, 12))
    flow = st.tuples(st.integers(0, n - 1), st.integers(0, n - 1))
    flows = draw(st.lists(flow, min_size=1, max_size=3 * n))
    size = draw(st.one_of(st.integers(1, 1 << 16), st.integers((1 << 20) - 4096, 1 << 31)))
    return n, flows, size


@SETTINGS
@given(groups(), st.sampled_from([-1, 0, 1, 3]), st.sampled_from([1.0, 0.5, 2.0]))
def test_plan_routes_partitions_every_message(native, group, max_relays, weight):
    """Every flow's stripes tile [0, bytes) exactly, the direct stripe comes
    first and is never empty, relay stripes start 4 KiB-aligned, a relay is
    never an endpoint nor a rank whose legs the group already uses directly,
    and duplicate flows get identical plans."""
    n, flows, size = group
    plans = native.plan_routes(n, flows, size, relay_weight=weight, max_relays=max_relays)
    assert len(plans) == len(flows)
    busy = {(a, b) for a, b in flows if a != b}
    by_flow = {}
    for (a, b), plan in zip(flows, plans):
        assert plan[0][0] == -1 and plan[0][2] > 0
        spans = sorted((off, nb) for _, off, nb in plan)
        assert spans[0][0] == 0 and all(x[0] + x[1] == y[0] for x, y in zip(spans, spans[1:]))
        assert spans[-1][0] + spans[-1][1] == size
        vias = [v for v, _, _ in plan[1:]]
        assert len(vias) == len(set(vias))
        if max_relays >= 0:
            assert len(vias) <= max_relays
        if a == b or n <= 2 or size < (1 << 20):
            assert len(plan) == 1
        for v, off, nb in plan[1:]:
            assert 0 <= v < n and v not in (a, b)
            assert (a, v) not in busy and (v, b) not in busy
            assert off % 4096 == 0 and nb % 4096 == 0 and nb > 0
        by_flow.setdefault((a, b), plan)
        assert by_flow[(a, b)] == plan


MODES = ["pair", "ring", "allpairs", "tournament", "self"]


@SETTINGS
@given(st.sampled_from(MODES), st.sampled_from(["uni", "bi"]), st.integers(1, 24))
def test_schedules_cover_the_matrix(native, mode, direction, n):
    """Per-rank send/recv lists agree with each phase's flows; pair and
    tournament cover every ordered off-diagonal cell (pair bi twice, once per
    cell of the row-major order), a tournament phase is a matching, and
    all-pairs is every cell in one group."""
    phases = native.schedule(mode, direction, n)
    cells = collections.Counter()
    for p in phases:
        sends = [(r, d) for r, (to, _) in enumerate(p["ranks"]) for d in to]
        recvs = [(s, r) for r, (_, frm) in enumerate(p["ranks"]) for s in frm]
        assert sorted(sends) == sorted(recvs) == sorted(tuple(f) for f in p["flows"])
        assert p["idle"] == (not p["flows"])
        cells.update(tuple(f) for f in p["flows"])
        if mode == "tournament" and n > 1:
            assert all(len(to) <= 1 and len(frm) <= 1 for to, frm in p["ranks"])
    off_diag = {(a, b) for a in range(n) for b in range(n) if a != b}
    if mode == "self" or (n == 1 and mode != "pair"):
        assert cells == collections.Counter({(r, r): 1 for r in range(n)})
    elif mode == "pair":
        assert len(phases) == n * n
        assert set(cells) == off_diag and set(cells.values()) <= {1 if direction == "uni" else 2}
    elif mode in ("tournament", "allpairs"):
        assert set(cells) == off_diag and set(cells.values()) == ({1} if off_diag else set())
        if mode == "allpairs":
            assert len(phases) == 1
    else:  # ring
        want = {(r, (r + 1) % n) for r in range(n)}
        if direction == "bi" and n > 2:
            want |= {(r, (r - 1) % n) for r in range(n)}
        assert set(cells) == want


@SETTINGS
@given(st.integers(1, 1 << 14), st.integers(0, (1 << 64) - 1), st.data())
def test_fill_verify_detects_any_corrupt_byte(native, size, seed, data):
    """A filled buffer verifies clean; one flipped byte is exactly one
    mismatching word, reported at its word offset."""
    buf = bytearray(native.host_fill(size, seed))
    assert len(buf) == size
    assert native.host_verify(bytes(buf), seed)[0] == 0
    i = data.draw(st.integers(0, size - 1))
    buf[i] ^= data.draw(st.integers(1, 255))
    mismatches, _, first_bad = native.host_verify(bytes(buf), seed)
    assert mismatches == 1 and first_bad == 4 * (i // 4)


@SETTINGS
@given(st.integers(16, 4096), st.integers(0, (1 << 63) - 1))
def test_verify_rejects_another_seed(native, size, seed):
    buf = native.host_fill(size, seed)
    assert native.host_verify(buf, seed + 1)[0] > 0


@SETTINGS
@given(st.integers(1, 6), st.integers(1, 8), st.data())
def test_block_placement(native, hosts, per_host, data):
    """Contiguous blocks of equal size place every rank (local rank =
    position in its block); interleaving hosts or uneven blocks is refused."""
    ids = data.draw(st.lists(st.integers(1, (1 << 63) - 1), min_size=hosts, max_size=hosts, unique=True))
    blocks = [h for h in ids for _ in range(per_host)]
    rank = data.draw(st.integers(0, len(blocks) - 1))
    p = native.compute_placement(blocks, rank)
    assert p["ok"] and p["num_hosts"] == hosts and p["ranks_per_host"] == per_host
    assert p["local_rank"] == rank % per_host
    if hosts > 1 and per_host > 1:
        interleaved = [ids[r % hosts] for r in range(len(blocks))]
        assert not native.compute_placement(interleaved, rank)["ok"]
        uneven = blocks + [ids[0]]
        assert not native.compute_placement(uneven, 0)["ok"]


@SETTINGS
@given(st.one_of(st.integers(1, 1 << 48), st.integers(0, 40).map(lambda k: 1 << k)))
def test_size_format_round_trips(native, size):
    assert native.parse_size(native.format_size(size)) == size


@SETTINGS
@given(st.integers(1, 4), st.lists(st.lists(st.floats(0.5, 5000.0), min_size=16, max_size=16), min_size=1, max_size=9))
def test_combine_runs_summarises_every_run(n, cells):
    """bench/core.py combine_runs (the reference-method repeats, VERDICT r5
    item 1): one `runs` entry per run (its mean cell), median / min / max in
    order, a spread of (max - min) / median, every cell of the combined matrix
    the median of that cell over the runs, and mismatches summed."""
    import statistics

    from test_nccl_p2p_amd.bench.core import combine_runs, pair_matrix_summary

    pairs = [(a, b) for a in range(n) for b in range(n) if a != b] if n > 1 else [(-1, -1)]
    runs = [pair_matrix_summary({"phases": [{"row": a, "col": b, "compat_gbps": 8 * v[i], "mismatches": i % 2}
                                            for i, (a, b) in enumerate(pairs)]}, n) for v in cells]
    c = combine_runs(runs, n)
    assert c["runs"] == [round(r["gbs_mean"], 3) for r in runs]
    assert c["min"] <= c["median"] <= c["max"] and c["spread"] >= 0
    assert abs(c["median"] - statistics.median(r["gbs_mean"] for r in runs)) < 1e-3
    for i, (a, b) in enumerate(pairs):
        a, b = (0, 0) if a < 0 else (a, b)
        per_run = [r["matrix_gbs"][a][b] for r in runs]
        assert min(per_run) - 1e-3 <= c["matrix_gbs"][a][b] <= max(per_run) + 1e-3
    assert c["mismatches"] == sum(r["mismatches"] for r in runs) and c["cells"] == len(pairs)

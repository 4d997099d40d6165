"""bench.py helpers that need no GPU and no launcher."""
import os
import sys

import pytest

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import bench  # noqa: E402


def test_posting_candidates_default_rccl():
    # One communicator per-message and batched, four communicators batched.
    assert bench.posting_candidates("rccl", -1, -1) == [(1, 0), (1, 1), (4, 1)]
    # With 8 hardware queues (bench.py's default) one GPU also tries 8 communicators.
    assert bench.posting_candidates("rccl", -1, -1, 1, hw_queues=8) == [(1, 0), (1, 1), (4, 1), (8, 1)]
    # Across GPUs the communicator count for one xGMI link is open: 1, 2, 4, 8.
    assert bench.posting_candidates("rccl", -1, -1, 8) == [(1, 0), (1, 1), (2, 1), (4, 1), (8, 1)]
    assert bench.posting_candidates("rccl", 4, -1, 8) == [(4, 1)]


def test_posting_candidates_fixed_and_other_transports():
    assert bench.posting_candidates("rccl", 4, -1) == [(4, 1)]
    assert bench.posting_candidates("rccl", 1, 1) == [(1, 1)]
    assert bench.posting_candidates("rccl", -1, 1) == [(1, 1), (4, 1)]
    assert bench.posting_candidates("ipc", -1, -1) == [(1, 0), (1, 1)]
    assert bench.posting_candidates("host", 4, 0) == [(1, 0)]


def test_tuning_steps_are_whole_laps():
    # N = 8: 7 rounds, one lap covers every cell; N = 1 / 2: one round, 8 steps.
    assert bench.tuning_steps(7) == 7
    assert bench.tuning_steps(4) == 4
    assert bench.tuning_steps(3) == 9
    assert bench.tuning_steps(1) == 8
    assert bench.tuning_steps(1, min_steps=4) == 4


def test_first_comms():
    assert bench.first_comms("rccl", -1) == 1
    assert bench.first_comms("rccl", 4) == 4
    assert bench.first_comms("ipc", 4) == 1


def test_headline_value_is_the_mean_cell():
    # 8 ranks, 4 pairs x 2 directions = 8 flows per step, 20 steps of 8 x 32 MiB
    # per flow, 2 s: aggregate = all bytes / 2 s; value = aggregate / 8.
    per_flow = 8 * (32 << 20)
    job = 20 * 8 * per_flow
    value, aggregate = bench.headline_stats(job, 20 * 8, 20, 2.0)
    assert abs(aggregate - job / 2.0 / 1e9) < 1e-9
    assert abs(value - aggregate / 8) < 1e-9
    # One GPU: one self flow per step, value == aggregate.
    v1, a1 = bench.headline_stats(20 * per_flow, 20, 20, 0.5)
    assert v1 == a1


def test_cell_matrix_takes_the_longer_endpoint():
    flows = {0: [(0, 1), (1, 0)], 1: [(0, 1), (1, 0)]}
    all_ms = [[1.0, 2.0], [4.0, 1.0]]  # rank 0 / rank 1 per-step ms
    m, samples, cells = bench.cell_matrix(2, [0, 1], lambda k: flows[k], all_ms, 1e6)
    # step 0: max(1, 4) = 4 ms -> 0.25 GB/s; step 1: max(2, 1) = 2 ms -> 0.5 GB/s
    assert cells[(0, 1)] == [0.25, 0.5] and m[0][1] == 0.375 and samples[0][1] == 2
    assert samples[0][0] == 0 and m[1][1] == 0.0


def test_pick_depth_covers_the_timed_steps():
    assert bench.pick_depth(20, 7) == 3 and bench.pick_depth(20, 1) == 20 and bench.pick_depth(1, 7) == 1


def test_bench_help_lists_transports():
    args = bench.parse_args([])
    assert args.transport == "rccl" and args.comms == -1 and args.isolate == 1 and args.deadline == 300.0
    for t in ("ipc:relay", "shm"):
        assert bench.parse_args(["--transport", t]).transport == t


@pytest.mark.parametrize("argv,msg", [
    (["--steps", "0"], "--steps must be >= 1"), (["--warmup", "-1"], "--warmup must be >= 0"),
    (["--gpus", "0"], "--gpus must be >= 1"), (["--msgs", "0"], "--msgs must be >= 1"),
    (["--comms", "0"], "--comms must be -1 (tuned) or >= 1"), (["--batch", "2"], "--batch must be -1, 0 or 1"),
    (["--tune-passes", "0"], "--tune-passes must be >= 1"), (["--ref-runs", "0"], "--ref-runs must be >= 1"),
    (["--hw-queues", "64"], "--hw-queues must be <= 32"), (["--deadline", "0"], "--deadline must be > 0"),
    (["--timeout", "-3"], "--timeout must be > 0"), (["--untimed-budget", "-1"], "--untimed-budget must be >= 0"),
])
def test_bench_rejects_out_of_range_counts(argv, msg, capsys):
    """Counts out of range stop bench.py at argument parsing, naming the
    option (before any rank, GPU or rendezvous starts)."""
    with pytest.raises(SystemExit) as e:
        bench.parse_args(argv)
    assert e.value.code == 2 and msg in capsys.readouterr().err


def test_default_device_wraps_to_the_visible_gpus(monkeypatch):
    monkeypatch.setattr(bench.torch.cuda, "device_count", lambda: 8)
    assert [bench.default_device(r) for r in (0, 3, 7)] == [0, 3, 7]
    monkeypatch.setattr(bench.torch.cuda, "device_count", lambda: 1)  # one visible GPU per process
    assert [bench.default_device(r) for r in (0, 3, 7)] == [0, 0, 0]
    monkeypatch.setattr(bench.torch.cuda, "device_count", lambda: 0)  # CPU transports
    assert bench.default_device(5) == 5


def test_pair_matrix_summary_bi_is_both_directions():
    """A pair-mode run valued like the reference's printed cells: the bi
    phase's compat_gbps counts both directions' bytes (p2p_matrix.cc:258's
    x2), and GB/s = Gbps / 8; self runs land on the diagonal."""
    from test_nccl_p2p_amd.bench.core import pair_matrix_summary
    run = {"phases": [{"row": 0, "col": 1, "compat_gbps": 800.0, "mismatches": 0},
                      {"row": 1, "col": 0, "compat_gbps": 400.0, "mismatches": 2}]}
    s = pair_matrix_summary(run, 2)
    assert s["matrix_gbs"] == [[0.0, 100.0], [50.0, 0.0]]
    assert s["gbs_min"] == 50.0 and s["gbs_mean"] == 75.0 and s["cells"] == 2 and s["mismatches"] == 2
    # One bi exchange of 1 GB each way in 1 s: flows 2 x 1e9 B -> 16 Gbps -> 2 GB/s, twice one direction.
    bi = {"phases": [{"row": 0, "col": 1, "compat_gbps": 2 * 1e9 * 8 / 1e9, "mismatches": 0}]}
    assert pair_matrix_summary(bi, 2)["gbs_mean"] == 2.0
    self_run = {"phases": [{"row": -1, "col": -1, "compat_gbps": 80.0, "mismatches": 0}]}
    assert pair_matrix_summary(self_run, 1)["matrix_gbs"] == [[10.0]]


def test_method_and_concurrency_ratios():
    from test_nccl_p2p_amd.bench.core import method_ratios
    ours = {"uni": {"gbs_mean": 60.0}, "bi": {"gbs_mean": 100.0}}
    ref = {"uni": {"gbs_mean": 20.0}, "bi": {"gbs_mean": 50.0}}
    r = method_ratios(ours, ref, 65.0, 8)
    # same schedule, two methods; then the tournament cell vs the serial bi cell per direction (100 / 2)
    assert r == {"method_ratio": {"uni": 3.0, "bi": 2.0}, "concurrency_ratio": 1.3}
    assert method_ratios(ours, None, 65.0, 8)["method_ratio"] == {"uni": None, "bi": None}
    one = method_ratios({"uni": {"gbs_mean": 2400.0}}, {"uni": {"gbs_mean": 700.0}}, 2300.0, 1)
    assert one["method_ratio"]["uni"] == 3.429 and one["method_ratio"]["bi"] is None and one["concurrency_ratio"] is None


def test_section_slices():
    """While a BASELINE section runs, the slices of the planned ones after it
    stay reserved (the BASELINE configs run first)."""
    from test_nccl_p2p_amd.bench.core import SECTION_SLICES, reserved_after
    names = [n for n, _ in SECTION_SLICES]
    assert names.index("reference_semantics") < names.index("allpairs_1g") < names.index("pair_sweep_0_1")
    active = set(names)
    assert reserved_after("pair_sweep_0_1", active) == 0.0
    assert reserved_after("allpairs_1g", active) == sum(s for n, s in SECTION_SLICES[names.index("allpairs_1g") + 1:])
    assert reserved_after("latency", {"latency", "ring_hop"}) == dict(SECTION_SLICES)["ring_hop"]
    assert reserved_after("ipc", active) == 0.0


def test_hw_queues_set_before_hip(monkeypatch):
    """--hw-queues reaches GPU_MAX_HW_QUEUES before HIP starts; the
    environment's value is kept for the record; 0 leaves it alone."""
    monkeypatch.setenv("GPU_MAX_HW_QUEUES", "4")
    bench.set_hw_queues([])
    assert os.environ["GPU_MAX_HW_QUEUES"] == "8" and os.environ["P2P_HW_QUEUES_ENV"] == "4"
    monkeypatch.setenv("GPU_MAX_HW_QUEUES", "4")
    bench.set_hw_queues(["--steps", "3", "--hw-queues", "0"])
    assert os.environ["GPU_MAX_HW_QUEUES"] == "4"
    bench.set_hw_queues(["--hw-queues=12"])
    assert os.environ["GPU_MAX_HW_QUEUES"] == "12"
    assert bench.parse_args(["--hw-queues", "0"]).hw_queues == 0 and bench.parse_args([]).hw_queues == 8


def test_recv_budget_split_between_ranks_on_one_gpu(monkeypatch):
    import types

    from test_nccl_p2p_amd.bench import headline

    run = types.SimpleNamespace(args=types.SimpleNamespace(recv_budget="0"), use_gpu=True, device=0,
                                env=types.SimpleNamespace(rank=0),
                                nat=types.SimpleNamespace(parse_size=lambda s: {"2G": 2 << 30}[s]))
    monkeypatch.setattr(headline.torch.cuda, "mem_get_info", lambda d: (100 << 30, 288 << 30))
    prov = {"rank_devices": [{"device": 0}] * 4 + [{"device": 1}] * 4}
    budget = headline.HeadlineMixin.recv_budget
    # Four ranks on device 0 allocate at once: each plans with 0.4 of a quarter.
    assert budget(run, prov) == int(0.4 * (100 << 30) / 4)
    assert budget(run, {}) == int(0.4 * (100 << 30))
    run.args.recv_budget = "2G"
    assert budget(run, prov) == 2 << 30
    run.args.recv_budget, run.use_gpu = "0", False
    assert budget(run, prov) == 256 << 20


def test_ranks_on_my_gpu_match_by_pci():
    """A launcher that shows each rank only its own GPU puts every rank on
    device 0: the PCI bus id, not the index, tells whether ranks share a GPU."""
    from test_nccl_p2p_amd.bench.headline import ranks_on_my_gpu

    own = {"rank_devices": [{"rank": r, "device": 0, "pci": "0000:%02x:00.0" % (0x10 + r)} for r in range(8)]}
    assert ranks_on_my_gpu(own, 3, 0) == 1
    shared = {"rank_devices": [{"rank": r, "device": 0, "pci": "0000:8b:00.0"} for r in range(4)]}
    assert ranks_on_my_gpu(shared, 2, 0) == 4
    # No PCI ids (CPU transports): the device index decides, as before.
    assert ranks_on_my_gpu({"rank_devices": [{"rank": r, "device": r % 2, "pci": ""} for r in range(4)]}, 0, 0) == 2
    assert ranks_on_my_gpu({}, 0, 0) == 1


def test_link_check_flags_direct_xgmi_pairs_not_on_p2p():
    """bench.py's link_check: a pair whose GPUs share a direct xGMI link but
    which RCCL carried over SHM or NET is listed (the --min-gbs rule of
    p2p_matrix); unknown transports, two-hop links and one GPU are not."""
    links = [["same-gpu", "XGMI/1", "XGMI/1", "XGMI/2"],
             ["XGMI/1", "same-gpu", "XGMI/1", "XGMI/1"],
             ["XGMI/1", "XGMI/1", "same-gpu", "XGMI/1"],
             ["XGMI/2", "XGMI/1", "XGMI/1", "same-gpu"]]
    t = [["self", "P2P", "SHM", "NET"],
         ["P2P", "self", "?", "P2P"],
         ["NET", "P2P", "self", "P2P"],
         ["SHM", "P2P", "P2P", "self"]]
    lc = bench.link_check(links, t)
    assert lc == {"direct_xgmi_pairs": 10, "not_p2p": ["0->2 SHM", "2->0 NET"], "ok": False}
    ok = bench.link_check(links, [["self" if a == b else "P2P" for b in range(4)] for a in range(4)])
    assert ok["ok"] and ok["not_p2p"] == [] and ok["direct_xgmi_pairs"] == 10
    # Ranks sharing one GPU (emulated node, NET by design) have no direct link.
    emu = bench.link_check([["same-gpu"] * 2] * 2, [["self", "NET"], ["NET", "self"]])
    assert emu == {"direct_xgmi_pairs": 0, "not_p2p": [], "ok": True}
    assert bench.link_check(None, t) is None and bench.link_check(links, None) is None


def test_stock_env_restores_what_bench_changed():
    """reference_semantics_stock's child environment: the queue count, RCCL's
    unroll factor and log settings as bench.py found them at start, RCCL's own
    unroll and no private INFO log."""
    import json

    from test_nccl_p2p_amd.bench.compare import stock_env

    env = {"GPU_MAX_HW_QUEUES": "8", "RCCL_UNROLL_FACTOR": "4", "NCCL_DEBUG": "INFO",
           "NCCL_DEBUG_FILE": "/tmp/p2p_rccl_info_1.log", "NCCL_DEBUG_SUBSYS": "INIT,P2P", "OTHER": "x",
           "P2P_STOCK_ENV": json.dumps({"GPU_MAX_HW_QUEUES": "4", "RCCL_UNROLL_FACTOR": None, "NCCL_DEBUG": "VERSION",
                                        "NCCL_DEBUG_FILE": None, "NCCL_DEBUG_SUBSYS": None})}
    s = stock_env(env)
    assert s["GPU_MAX_HW_QUEUES"] == "4" and s["NCCL_DEBUG"] == "VERSION" and s["OTHER"] == "x"
    for k in ("RCCL_UNROLL_FACTOR", "NCCL_DEBUG_FILE", "NCCL_DEBUG_SUBSYS"):
        assert k not in s
    assert s["P2P_RCCL_UNROLL"] == "0" and s["P2P_RCCL_LOG"] == "0"
    assert env["RCCL_UNROLL_FACTOR"] == "4"  # the caller's mapping is left alone


def test_stock_reference_only_for_rccl_within_the_process_limit():
    """reference_semantics_stock starts a child per rank: planned for an RCCL
    headline only, and only while two processes per rank sharing a GPU stay
    within the box's limit (8 ranks on one GPU + 8 children + pytest = 17 was
    killed by the process guard)."""
    import types

    from test_nccl_p2p_amd.bench.sections import SectionsMixin

    def run(transport, pcis, ref_stock=1):
        o = SectionsMixin()
        o.args = types.SimpleNamespace(ref_stock=ref_stock, ref_iters=128)
        o.transport_used, o.use_gpu, o.n, o.device = transport, True, len(pcis), 0
        o.h = types.SimpleNamespace(provenance={"rank_devices": [{"rank": r, "device": 0, "pci": p}
                                                                 for r, p in enumerate(pcis)]})
        return o.stock_reference_planned()

    assert run("rccl", ["a"]) and run("rccl", ["a", "b", "c", "d", "e", "f", "g", "h"])
    assert run("rccl", ["a"] * 4) and not run("rccl", ["a"] * 8)
    assert not run("ipc", ["a"]) and not run("rccl", ["a"], ref_stock=0)


def test_candidate_budgets():
    from test_nccl_p2p_amd.bench import core

    # The first candidate: a quarter of the time left, at least 10 s, at most --timeout.
    assert core.first_candidate_budget(120.0, 280.0) == 70.0
    assert core.first_candidate_budget(120.0, 20.0) == 10.0
    assert core.first_candidate_budget(30.0, 280.0) == 30.0
    # Later candidates: 10 x the first one's connect + pass, at least 10 s,
    # never more than 15% of the time left (nor --timeout).
    assert core.candidate_budget(0.05, 280.0, 120.0) == 10.0
    assert abs(core.candidate_budget(3.0, 280.0, 120.0) - 30.0) < 1e-9
    assert abs(core.candidate_budget(6.0, 280.0, 120.0) - 42.0) < 1e-9
    assert abs(core.candidate_budget(0.05, 40.0, 120.0) - 6.0) < 1e-9
    assert core.candidate_budget(6.0, -5.0, 120.0) == 0.0


def test_candidate_hang_hook(monkeypatch):
    from test_nccl_p2p_amd.bench.core import candidate_hang as hang

    monkeypatch.setenv("P2P_BENCH_HANG", "candidate:4,1@3")
    assert hang("rccl", 4, 1, 3) == "tuning" and hang("host", 4, 1, 3) == "tuning"
    assert hang("rccl", 4, 1, 2) is None and hang("rccl", 4, 0, 3) is None
    monkeypatch.setenv("P2P_BENCH_HANG", "candidate:host:1,0:connect@0")
    assert hang("host", 1, 0, 0) == "connect" and hang("shm", 1, 0, 0) is None
    monkeypatch.setenv("P2P_BENCH_HANG", "candidate:rccl:1,0:stall@1;candidate:rccl:1,0:unbounded@0")
    assert hang("rccl", 1, 0, 1) == "stall" and hang("rccl", 1, 0, 0) == "unbounded" and hang("ipc", 1, 0, 0) is None
    monkeypatch.setenv("P2P_BENCH_HANG", "latency@3")
    assert hang("rccl", 1, 0, 3) is None


def test_timeline_entries_are_contiguous():
    import time

    from test_nccl_p2p_amd.bench.core import Deadline, Timeline, process_age

    assert process_age() > 0
    t0 = time.monotonic()
    tl = Timeline(t0)
    tl.begin("a")
    time.sleep(0.02)
    tl.begin("b")
    snap = tl.snapshot(Deadline(1000.0))
    names = [n for n, _ in snap["entries"]]
    assert names == ["startup", "imports", "a", "b"] and snap["open"] == "b"
    # Contiguous from process start: the entries add up to the total.
    assert abs(sum(s for _, s in snap["entries"]) - snap["total_s"]) < 1e-3
    assert dict(snap["entries"])["a"] >= 0.019
    assert snap["total_s"] >= process_age() - 0.05 and snap["deadline_left_s"] > 0


def test_unparsed_peers_summary():
    from test_nccl_p2p_amd.bench.core import unparsed_peers

    assert unparsed_peers(None) is None and unparsed_peers({"error": "x"}) is None and unparsed_peers([None]) is None
    reps = [{"rank": 0, "unparsed_peers": []}, {"rank": 1, "unparsed_peers": [{"peer": 3, "lines": ["x"]}]}, None]
    assert unparsed_peers(reps) == ["1->3"]
    assert unparsed_peers([{"rank": 0, "unparsed_peers": []}]) == []


def test_bench_fabric_findings():
    from test_nccl_p2p_amd.bench.core import bench_fabric_findings

    assert bench_fabric_findings({"matrix_gbs": [[0.0]]}, 1) is None
    even = [[0.0, 50.0, 51.0], [49.0, 0.0, 50.0], [50.0, 52.0, 0.0]]
    uni = {"matrix_gbs": [[0.0, 48.0, 48.0], [48.0, 0.0, 48.0], [48.0, 48.0, 0.0]]}
    bi = {"matrix_gbs": [[0.0, 96.0, 96.0], [96.0, 0.0, 96.0], [96.0, 96.0, 0.0]]}
    r = {"matrix_gbs": even, "pair_serial_events": {"uni": uni, "bi": bi}, "link_check": None, "unparsed_peers": []}
    assert bench_fabric_findings(r, 3) == []
    slow = dict(r, matrix_gbs=[[0.0, 50.0, 51.0], [49.0, 0.0, 50.0], [50.0, 12.0, 0.0]])
    assert bench_fabric_findings(slow, 3) == ["tournament matrix_gbs: cell 2->1 12.00 < 0.50 x median 50.00"]
    # The reference's method stands in when our serial run failed or is missing.
    low_bi = {"matrix_gbs": [[0.0, 40.0, 96.0], [96.0, 0.0, 96.0], [96.0, 96.0, 0.0]]}
    ref = dict(r, pair_serial_events={"error": "x"}, reference_semantics={"uni": uni, "bi": low_bi})
    assert bench_fabric_findings(ref, 3) == ["compat bi cell 0<->1 40.00 below its uni cell 48.00"]


def test_stock_env_ignores_an_engine_parents_settings():
    """A process started by one whose native engine set RCCL's variables (a
    pytest process that ran RCCL tests, say) records the user's values for the
    stock-settings reference, not the parent's (ran after in-process RCCL
    tests, test_bench_contract_single_gpu saw RCCL_UNROLL_FACTOR=4)."""
    env = {"RCCL_UNROLL_FACTOR": "4", "P2P_RCCL_PREV_RCCL_UNROLL_FACTOR": "", "NCCL_DEBUG": "INFO",
           "P2P_RCCL_PREV_NCCL_DEBUG": "=VERSION", "P2P_RCCL_ENV_OWNER": "1", "GPU_MAX_HW_QUEUES": "4"}
    assert bench.user_value("RCCL_UNROLL_FACTOR", env) is None
    assert bench.user_value("NCCL_DEBUG", env) == "VERSION"
    assert bench.user_value("GPU_MAX_HW_QUEUES", env) == "4"
    own = dict(env, P2P_RCCL_ENV_OWNER=str(os.getpid()))  # this process's own settings stand
    assert bench.user_value("RCCL_UNROLL_FACTOR", own) == "4"
    assert bench.user_value("RCCL_UNROLL_FACTOR", {"RCCL_UNROLL_FACTOR": "2"}) == "2"


def test_combine_runs_and_median_ratios():
    """R repeats of a reference-method matrix keep each
    run's mean cell, their median / min / max / spread, and a per-cell median
    matrix; the method ratios come from the medians (not one noisy shot)."""
    from test_nccl_p2p_amd.bench.core import combine_runs, method_ratios, pair_matrix_summary

    def run(v01, v10):
        return pair_matrix_summary({"phases": [{"row": 0, "col": 1, "compat_gbps": 8 * v01, "mismatches": 0},
                                               {"row": 1, "col": 0, "compat_gbps": 8 * v10, "mismatches": 1}]}, 2)

    c = combine_runs([run(50, 70), run(40, 60), run(90, 90), run(45, 55), run(52, 68)], 2)
    assert c["runs"] == [60.0, 50.0, 90.0, 50.0, 60.0]
    assert c["median"] == 60.0 and c["min"] == 50.0 and c["max"] == 90.0 and c["spread"] == round(40 / 60, 4)
    assert c["matrix_gbs"] == [[0.0, 50.0], [68.0, 0.0]] and c["gbs_mean"] == 59.0 and c["gbs_min"] == 50.0
    assert c["cells"] == 2 and c["mismatches"] == 5
    # One GPU: the self cell on the diagonal.
    one = combine_runs([pair_matrix_summary({"phases": [{"row": -1, "col": -1, "compat_gbps": 8 * v,
                                                         "mismatches": 0}]}, 1) for v in (686.7, 751.6, 819.0)], 1)
    assert one["median"] == 751.6 and one["matrix_gbs"] == [[751.6]] and one["gbs_mean"] == 751.6
    # The ratios use the medians: an outlier run moves neither.
    ours = {"uni": combine_runs([run(100, 100), run(120, 120), run(500, 500)], 2)}
    ref = {"uni": combine_runs([run(50, 50), run(10, 10), run(60, 60)], 2)}
    assert method_ratios(ours, ref, 1.0, 2)["method_ratio"]["uni"] == round(120 / 50, 3)
    # Records without repeats still use their mean cell.
    assert method_ratios({"uni": {"gbs_mean": 6.0}}, {"uni": {"gbs_mean": 2.0}}, 1.0, 2)["method_ratio"]["uni"] == 3.0


WATCHDOG_CHILD = r"""
import sys, time
sys.path.insert(0, %r)
from test_nccl_p2p_amd import require_native
from test_nccl_p2p_amd.bench import core
nat = require_native()
nat._push_blocking_abort_hook(120.0)  # an ncclCommAbort that never returns
t0 = time.monotonic()
core.set_start(t0)
dl = core.Deadline(1.0)
rep = core.Reporter(0, 1, None, core.Timeline(t0), dl)
rep.result = {"metric": core.METRIC, "value": 1.0}
core.start_watchdog(dl, rep, nat, {"section": "latency", "skipped": [], "errors": {}})
while True:  # the main thread in Python, outside the engine: the watchdog aborts from its helper
    time.sleep(1.0)
"""


def test_watchdog_ends_the_process_when_the_abort_blocks(native):
    """the watchdog's own abort (abort_if_idle, main thread outside
    the engine) runs on a helper thread with the GIL released, so an abort
    hook that never returns cannot keep the process alive: it prints the line
    and exits at the deadline + ABORT_GRACE_S (+ the linger), not when the
    launcher kills it."""
    import json
    import subprocess
    import time

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    t0 = time.monotonic()
    out = subprocess.run([sys.executable, "-c", WATCHDOG_CHILD % root], capture_output=True, text=True, timeout=60)
    wall = time.monotonic() - t0
    from test_nccl_p2p_amd.bench.core import ABORT_GRACE_S, ABORT_LINGER_S
    assert out.returncode == 0, out.stderr[-2000:]
    assert wall < 1.0 + ABORT_GRACE_S + ABORT_LINGER_S + 15.0, wall
    line = json.loads(out.stdout.strip().splitlines()[-1])
    assert line["deadline_hit"] is True and line["section_errors"] == {"latency": "deadline reached while running"}
    assert "abort from the watchdog (engine idle) still running after" in out.stderr, out.stderr[-2000:]


def test_child_runs_fit_the_slice():
    """The stock-settings child repeats as many runs as the in-process
    reference matrices had, unless the section's slice (less the child's
    start) holds fewer at their measured time per run; at least one."""
    from test_nccl_p2p_amd.bench.core import child_runs

    ref = {"uni": {"runs": [1.0] * 7, "run_s": 0.006}, "bi": {"runs": [1.0] * 3, "run_s": 1.0}}
    # N = 1: 7 runs of 6 ms fit easily.
    assert child_runs(ref, {"uni": 128}, 12.0, 6.0) == {"uni": 7}
    # 6 s left for two modes: 3 s each, 1.2 s per bi run with the margin -> 2 of its 3.
    assert child_runs(ref, {"uni": 128, "bi": 128}, 12.0, 6.0) == {"uni": 7, "bi": 2}
    # No time left: still one run each.
    assert child_runs(ref, {"uni": 128, "bi": 128}, 3.0, 6.0) == {"uni": 1, "bi": 1}
    # Records without run_s (or runs) fall back to one run per mode, bounded the same way.
    assert child_runs({"uni": {}}, {"uni": 8}, 60.0, 6.0) == {"uni": 1}


def test_faults_read_once_and_fire_at_named_points():
    """bench/faults.py reads every P2P_BENCH_* hook once;
    the measured flow only calls its named points."""
    import pytest

    from test_nccl_p2p_amd.bench.faults import Faults

    env = {"P2P_BENCH_FAIL_HEADLINE": "rccl", "P2P_BENCH_FAIL_CANDIDATE": "4,1,tuning",
           "P2P_BENCH_HANG": "candidate:rccl:1,0:stall@1;latency@3"}
    last, first = Faults(3, 4, env), Faults(1, 4, env)
    with pytest.raises(RuntimeError, match="injected headline failure"):
        last.fail_headline("rccl")
    last.fail_headline("ipc")  # other transports: nothing
    with pytest.raises(RuntimeError, match="injected tuning failure"):
        last.candidate_fail(4, 1, "tuning")
    last.candidate_fail(4, 1, "connect")  # that spec names the tuning pass
    first.candidate_fail(4, 1, "tuning")  # only the last rank fails
    assert first.candidate("rccl", 1, 0) == "stall" and last.candidate("rccl", 1, 0) is None
    first.section("latency")  # rank 3's hang, not rank 1's
    first.teardown()
    # Read once: a later change of the environment does not reach the object.
    quiet = Faults(0, 1, {})
    assert quiet.candidate("rccl", 1, 0) is None and quiet.fail_candidate is None
    quiet.fail_headline("rccl")

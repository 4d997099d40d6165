"""Reference-format text: Python printer == reference printf layout, parser
reads it back (also from the native binary's output)."""
from test_nccl_p2p_amd.utils.report import compat_matrix_text, parse_compat, scaling_table

GOLDEN = (
    "Evaluating the Uni-Directional NCCL P2P Bandwidth (Gbps)\n"
    "   D\\D     0      1 \n"
    "     0   0.00 391.53 \n"
    "     1 1234.50   0.00 \n"
    "\n"
    "Evaluating the Bi-Directional NCCL P2P Bandwidth (Gbps)\n"
    "   D\\D     0      1 \n"
    "     0   0.00 391.53 \n"
    "     1 1234.50   0.00 \n"
)


def test_golden():
    m = [[0.0, 391.53], [1234.5, 0.0]]
    assert compat_matrix_text(m, "uni") + compat_matrix_text(m, "bi") == GOLDEN


def test_parse_roundtrip():
    got = parse_compat(GOLDEN)
    assert got["uni"] == [[0.0, 391.53], [1234.5, 0.0]]
    assert got["bi"][1][0] == 1234.5


def test_scaling_table():
    """Round-2 lines: value = mean cell, aggregate_gbs = all flows; the cell
    rate is compared with N = 2 (weak scaling keeps it constant)."""
    rows = [{"n_gpus": 1, "value": 1000.0, "aggregate_gbs": 1000.0},
            {"n_gpus": 2, "value": 100.0, "aggregate_gbs": 200.0, "matrix_gbs_min": 50},
            {"n_gpus": 4, "value": 90.0, "aggregate_gbs": 360.0}]
    t = scaling_table(rows)
    assert "| 4 | 90.0 | 360.0 | 90.0 | 90.0% |" in t and "| 2 | 100.0 | 200.0 | 100.0 | 100.0% |" in t
    assert "| 1 | 1000.0 | 1000.0 | 1000.0 |  |" in t


def test_scaling_table_round1_lines():
    """Round-1 lines carried the aggregate in value and no aggregate_gbs."""
    t = scaling_table([{"n_gpus": 2, "value": 100.0}, {"n_gpus": 4, "value": 200.0}])
    assert "| 4 | 200.0 | 200.0 | 50.0 | 200.0% |" in t


def test_scaling_table_comparisons_and_cli(tmp_path, capsys):
    from test_nccl_p2p_amd.utils.report import main
    rows = [{"metric": "m", "n_gpus": 2, "value": 100.0, "aggregate_gbs": 200.0,
             "reference_semantics": {"cell_gbs_mean": 40.0},
             "extras": {"allpairs_1g": {"aggregate_gbs": 300.0}, "ring_hop": {"hop_us_p50": 3.25}},
             "posting": {"rccl_comms": 4},
             "ipc_transport": {"value_gbs": 110.0, "device_pingpong_p50_us": 1.5, "push": {"value_gbs": 120.0},
                               "relay": {"value_gbs": 150.0, "pair_0_1": [{"bytes": 1, "gbs": 250.5}]}}},
            {"metric": "m", "n_gpus": 8, "value": 95.0, "aggregate_gbs": 760.0, "ipc_transport": {"error": "x"},
             "headline_fallback": {"from": "rccl", "to": "ipc", "error": "e"}},
            {"metric": "m", "n_gpus": 4, "value": None, "error": "headline failed"}]
    t = scaling_table(rows)
    assert "| 2 | 100.0 | 200.0 | 100.0 | 100.0% | 4 |" in t
    assert "| 40.0 | - | 300.0 | 3.25 | 110.0 / 120.0 / - / 150.0 | 250.5 | 1.50 | - |" in t
    # Round-3 lines: the reference method in both direction modes, and the ratios.
    r3 = {"n_gpus": 4, "value": 60.0, "aggregate_gbs": 120.0,
          "reference_semantics": {"uni": {"gbs_mean": 20.0}, "bi": {"gbs_mean": 38.0}},
          "method_ratio": {"uni": 2.5, "bi": 2.4}, "concurrency_ratio": 1.3}
    assert "| 20.0 / 38.0 | 2.5 / 2.4 / 1.3 |" in scaling_table([r3])
    # A fallback line is its own kind: no ratio against the RCCL rows.
    assert "| 8 | 95.0 | 760.0 | 95.0 |  | - |" in t and "- / - / - / - | - | - | rccl -> ipc |" in t
    assert not any(l.startswith("| 4 |") for l in t.splitlines())  # a line without a value is left out
    files = []
    for r in rows:
        f = tmp_path / ("BENCH_%d.json" % r["n_gpus"])
        f.write_text(__import__("json").dumps(r) + "\n")
        files.append(str(f))
    assert main(files) == 0
    out = capsys.readouterr().out
    assert "== scaling" in out and "| 8 | 95.0 |" in out.split("== scaling")[1]


def test_scaling_table_pair_sweep():
    """The N = 2 line's xGMI pair sweep: winner per cell with its gain over
    RCCL on one communicator, corrupt and skipped rows."""
    sw = {"rc": 2, "emulated": None, "best": {
        "bi/33554432": {"row": "rccl-comms4", "cell_gbs": 201.5, "gain": 1.42},
        "uni/1073741824": {"row": "ipc-push", "cell_gbs": 110.25, "gain": None}},
        "corrupt": ["rccl-nchannels_per_peer=8"], "skipped": ["rccl-register=2"],
        "best_rccl": {"bi/33554432": {"row": "rccl-comms4", "cell_gbs": 201.5, "gain": 1.42},
                      "uni/1073741824": {"row": "rccl-proto=Simple", "cell_gbs": 70.0, "gain": 1.05}}}
    t = scaling_table([{"n_gpus": 2, "value": 100.0, "aggregate_gbs": 200.0, "xgmi_pair_sweep": sw},
                       {"n_gpus": 4, "value": 90.0, "aggregate_gbs": 360.0, "xgmi_pair_sweep": None}])
    lines = t.splitlines()
    assert "xGMI pair sweep, 2 GPUs:" in lines
    assert "- bi/33554432: rccl-comms4 201.50 GB/s (1.42x RCCL, 1 communicator)" in lines
    assert "- uni/1073741824: ipc-push 110.25 GB/s" in lines
    assert "- uni/1073741824, best RCCL: rccl-proto=Simple 70.00 GB/s (1.05x)" in lines
    assert not any(l.startswith("- bi/33554432, best RCCL") for l in lines)  # the overall winner already
    assert "- corrupt rows: rccl-nchannels_per_peer=8" in lines and "- skipped rows: rccl-register=2" in lines
    failed = scaling_table([{"n_gpus": 2, "value": 1.0, "xgmi_pair_sweep": {"rc": 1, "error": "no mpirun at x"}}])
    assert "xGMI pair sweep, 2 GPUs: no mpirun at x" in failed


def test_scaling_table_transport_lines():
    """matrix_transport and the RCCL op limits of a multi-GPU line are
    summarised under the table."""
    n = 4
    m = [["self" if a == b else ("P2P" if (a + b) % 3 else "SHM") for b in range(n)] for a in range(n)]
    peers = [{"peer": 0, "transport": "self", "op_channels": 64, "op_limit": 1 << 30},
             {"peer": 1, "transport": "P2P", "op_channels": 8, "op_limit": 128 << 20}]
    r = {"n_gpus": 4, "value": 50.0, "aggregate_gbs": 100.0, "matrix_transport": m,
         "provenance": {"rccl_peers": [{"peers": peers}, None]}}
    t = scaling_table([r])
    assert "RCCL transports, 4 GPUs: P2P 8/12, SHM 4/12; p2p channels per op 8, op limit 128 MiB" in t, t
    assert "WRONG TRANSPORT" not in t
    r["link_check"] = {"direct_xgmi_pairs": 12, "not_p2p": ["0->2 SHM", "2->0 SHM"], "ok": False}
    assert "WRONG TRANSPORT on 2 of 12 direct xGMI pairs: 0->2 SHM, 2->0 SHM" in scaling_table([r])


def test_bench_compat_text_round_trips():
    """A bench line's config-3 matrices print in the reference's exact format
    (GB/s x 8 = Gbps; bi = both directions summed), and parse back."""
    from test_nccl_p2p_amd.utils.report import bench_compat_text, parse_compat
    r = {"n_gpus": 2, "reference_semantics": {"uni": {"matrix_gbs": [[0.0, 48.5], [47.25, 0.0]]},
                                              "bi": {"matrix_gbs": [[0.0, 95.0], [95.0, 0.0]]}}}
    txt = bench_compat_text(r)
    assert txt.startswith("Evaluating the Uni-Directional NCCL P2P Bandwidth (Gbps)\n   D\\D     0      1 \n")
    assert "\nEvaluating the Bi-Directional NCCL P2P Bandwidth (Gbps)\n" in txt
    m = parse_compat(txt)
    assert m["uni"] == [[0.0, 388.0], [378.0, 0.0]] and m["bi"] == [[0.0, 760.0], [760.0, 0.0]]
    assert bench_compat_text({"reference_semantics": None}) == ""


def test_scaling_table_never_mixes_value_kinds():
    """the N = 1 self copy (HBM-bound, no link), the xGMI
    link rows and a fallback line each get a table of their own, and no ratio
    is ever taken across two kinds (1 -> 8 from `value` alone would read as a
    ~40x drop at N = 2)."""
    from test_nccl_p2p_amd.utils.report import FALLBACK, SELF_COPY, XGMI_LINK, value_kind
    rows = [{"n_gpus": 1, "value": 2800.0, "aggregate_gbs": 2800.0, "value_kind": SELF_COPY},
            {"n_gpus": 2, "value": 70.0, "aggregate_gbs": 140.0, "value_kind": XGMI_LINK},
            {"n_gpus": 4, "value": 66.5, "aggregate_gbs": 266.0, "value_kind": XGMI_LINK},
            {"n_gpus": 8, "value": 63.0, "aggregate_gbs": 504.0, "value_kind": XGMI_LINK}]
    t = scaling_table(rows)
    lines = t.splitlines()
    x, s = lines.index("value_kind: " + XGMI_LINK), [i for i, l in enumerate(lines) if l.startswith(
        "value_kind: " + SELF_COPY)][0]
    assert x < s  # the link rows first, the self copy apart below them
    link_rows = [l for l in lines[x:s] if l.startswith("| ") and l[2].isdigit()]
    assert [l.split("|")[1].strip() for l in link_rows] == ["2", "4", "8"]
    assert "| 2 | 70.0 | 140.0 | 70.0 | 100.0% |" in t and "| 4 | 66.5 | 266.0 | 66.5 | 95.0% |" in t
    assert "| 8 | 63.0 | 504.0 | 63.0 | 90.0% |" in t
    # The self-copy row has no ratio at all, and nothing is ever relative to it.
    assert "| 1 | 2800.0 | 2800.0 | 2800.0 |  |" in t and "4000.0%" not in t and "2.5%" not in t
    # Without an N = 2 line of its own kind a row gets no ratio (never one against N = 1).
    t2 = scaling_table([rows[0], rows[3]])
    assert "| 8 | 63.0 | 504.0 | 63.0 |  |" in t2
    fb = {"n_gpus": 2, "value": 90.0, "aggregate_gbs": 180.0, "value_kind": FALLBACK,
          "headline_fallback": {"from": "rccl", "to": "ipc", "error": "e"}}
    t3 = scaling_table([fb, rows[2]])
    assert "| 4 | 66.5 | 266.0 | 66.5 |  |" in t3 and "value_kind: fallback" in t3
    # Lines from before the field are classed from n_gpus and headline_fallback.
    assert value_kind({"n_gpus": 1}) == SELF_COPY and value_kind({"n_gpus": 8}) == XGMI_LINK
    assert value_kind({"n_gpus": 8, "headline_fallback": {"from": "rccl"}}) == FALLBACK


def test_report_cli_reads_repeat_records(tmp_path, capsys):
    """p2p_matrix --repeat --json: the report tool lists each run with its
    index and one summary line per repeats record."""
    import json

    from test_nccl_p2p_amd.utils.report import main, repeat_line

    run = {"type": "run", "mode": "self", "dir": "uni", "bytes": 1 << 25, "iters": 128, "gbs_min": 500.0,
           "gbs_mean": 500.0, "gbs_max": 500.0}
    rep = {"type": "repeats", "mode": "self", "dir": "uni", "bytes": 1 << 25, "runs": [400.0, 500.0, 520.0],
           "median": 500.0, "min": 400.0, "max": 520.0}
    assert repeat_line(rep).endswith("3 runs: GB/s median 500.00 (min 400.00, max 520.00, spread 24.0%)")
    p = tmp_path / "r.json"
    p.write_text("\n".join(json.dumps(x) for x in (dict(run, repeat=0), dict(run, repeat=1), rep)) + "\n")
    assert main([str(p)]) == 0
    out = capsys.readouterr().out
    assert "(run 1)" in out and "(run 0)" not in out and "spread 24.0%" in out

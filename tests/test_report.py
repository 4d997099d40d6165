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
    rows = [{"n_gpus": 1, "value": 1000.0}, {"n_gpus": 2, "value": 100.0, "matrix_gbs_min": 50},
            {"n_gpus": 4, "value": 200.0}]
    t = scaling_table(rows)
    assert "| 4 | 200.0 | 50.0 |" in t and "100.0%" in t


def test_scaling_table_comparisons_and_cli(tmp_path, capsys):
    from test_nccl_p2p_amd.utils.report import main
    rows = [{"metric": "m", "n_gpus": 2, "value": 100.0, "reference_semantics": {"cell_gbs_mean": 40.0},
             "extras": {"allpairs_1g": {"aggregate_gbs": 300.0}},
             "posting": {"rccl_comms": 4},
             "ipc_transport": {"value_gbs": 110.0, "device_pingpong_p50_us": 1.5, "push": {"value_gbs": 120.0},
                               "relay": {"value_gbs": 150.0, "pair_0_1": [{"bytes": 1, "gbs": 250.5}]}}},
            {"metric": "m", "n_gpus": 8, "value": 380.0, "ipc_transport": {"error": "x"}}]
    t = scaling_table(rows)
    assert "| 2 | 100.0 | 50.0 | 4 |" in t
    assert "| 40.0 | 300.0 | - | 110.0 / 120.0 / - / 150.0 | 250.5 | 1.50 |" in t
    assert "| 8 | 380.0 | 47.5 | - |" in t and "95.0%" in t and "- / - / - / - | - |" in t
    files = []
    for r in rows:
        f = tmp_path / ("BENCH_%d.json" % r["n_gpus"])
        f.write_text(__import__("json").dumps(r) + "\n")
        files.append(str(f))
    assert main(files) == 0
    out = capsys.readouterr().out
    assert "== scaling" in out and "| 8 | 380.0 |" in out.split("== scaling")[1]

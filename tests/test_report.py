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

"""Python utilities: statistics parity with the native engine, report CLI,
RCCL environment capture."""
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT
from test_nccl_p2p_amd.utils import rccl_env
from test_nccl_p2p_amd.utils.report import compat_matrix_text, main as report_main, summarize_compat
from test_nccl_p2p_amd.utils.stats import offdiag_summary, percentile, summarize


def test_percentiles_match_native_convention():
    # Same cases as tests/host/test_main.cpp test_stats.
    assert percentile([5, 1, 4, 2, 3], 50) == 3
    assert percentile([1, 2, 3, 4], 50) == 2.5
    assert abs(percentile([1, 2, 3, 4], 90) - 3.7) < 1e-12
    s = summarize([5, 1, 4, 2, 3])
    assert s["n"] == 5 and s["mean"] == 3 and abs(s["stdev"] - 2.5 ** 0.5) < 1e-12
    assert summarize([])["n"] == 0


def test_offdiag_summary():
    m = [[0, 10, 20], [30, 0, 40], [50, 60, 0]]
    s = offdiag_summary(m)
    assert s == {"min": 10, "mean": 35, "max": 60, "cells": 6}


def test_summarize_compat():
    txt = compat_matrix_text([[0, 80.0], [160.0, 0]], "uni")
    out = summarize_compat(txt)
    assert "uni: 2 ranks, GB/s min 10.00 mean 15.00 max 20.00" in out


def test_report_cli(tmp_path, capsys):
    f = tmp_path / "result.txt"
    f.write_text(compat_matrix_text([[0, 8.0], [16.0, 0]], "uni") + compat_matrix_text([[0, 8.0], [8.0, 0]], "bi"))
    j = tmp_path / "bench.jsonl"
    j.write_text(json.dumps({"metric": "m", "n_gpus": 2, "value": 50.0, "aggregate_gbs": 100.0, "matrix_gbs_min": 50,
                             "matrix_gbs_mean": 50, "p50_latency_us": 10}) + "\n")
    assert report_main([str(f), str(j)]) == 0
    out = capsys.readouterr().out
    assert "bi: 2 ranks" in out and "| 2 | 50.0 | 100.0 | 50.0 |" in out


def test_rccl_env_capture(monkeypatch):
    monkeypatch.setenv("NCCL_DEBUG", "WARN")
    monkeypatch.setenv("RCCL_P2P_BATCH_ENABLE", "1")
    env = rccl_env.capture()
    assert env["NCCL_DEBUG"] == "WARN" and env["RCCL_P2P_BATCH_ENABLE"] == "1"
    assert all(k in env for k in rccl_env.P2P_KNOBS)


def test_package_version_and_native(native):
    import test_nccl_p2p_amd

    assert test_nccl_p2p_amd.__version__
    assert test_nccl_p2p_amd.native_available()
    assert "mpirun -n N ./p2p_matrix" in native.usage()


def test_graft_entry_build_is_importable():
    out = subprocess.run([sys.executable, "-c", "import __graft_entry__ as g; print(callable(g.build), callable(g.smoke))"],
                         capture_output=True, text=True, cwd=ROOT, timeout=120)
    assert out.stdout.strip() == "True True"


@pytest.mark.parametrize("argv", [["--dry-run", "--mode", "ring"], ["--help"]])
def test_python_module_cli(native, argv):
    out = subprocess.run([sys.executable, "-m", "test_nccl_p2p_amd"] + argv, capture_output=True, text=True,
                         cwd=ROOT, timeout=120, env=dict(os.environ, RANK="0", WORLD_SIZE="1"))
    assert out.returncode == 0, out.stderr


def test_gate_probe_unsupported_on_cpu(native):
    sess = native.Session(0, 1, transport="host")
    assert json.loads(sess.gate_probe(0.1, True)) == {"supported": False}


def test_chunking_is_rccl_only(native):
    """Session.set_chunk_cap / max_chunk: only the RCCL transport splits
    messages (RCCL's 16 MiB-per-p2p-channel loss); the CPU transports report
    nothing to split and no link report."""
    sess = native.Session(0, 1, transport="host")
    assert sess.set_chunk_cap(16 << 20) is False and sess.max_chunk(0) == 0
    assert sess.link_reports() == "[null]"


def test_child_dies_with_its_parent():
    """utils.proc: a child in a session of its own (out of reach of a kill of
    its parent's process group) that called die_with_parent() is killed by
    the kernel when its parent exits."""
    import psutil
    import time
    child = ("from test_nccl_p2p_amd.utils.proc import die_with_parent; import time; "
             "assert die_with_parent(); time.sleep(120)")
    parent = ("import subprocess, sys, time; from test_nccl_p2p_amd.utils.proc import child_env; "
              "p = subprocess.Popen([sys.executable, '-c', %r], env=child_env(), start_new_session=True, "
              "stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL); "
              "print(p.pid, flush=True); time.sleep(4)" % child)
    out = subprocess.run([sys.executable, "-c", parent], capture_output=True, text=True, cwd=ROOT, timeout=60)
    pid = int(out.stdout.split()[0])
    for _ in range(100):
        try:
            if psutil.Process(pid).status() == psutil.STATUS_ZOMBIE:
                break
        except psutil.NoSuchProcess:
            break
        time.sleep(0.1)
    else:
        os.kill(pid, 9)
        raise AssertionError("the child outlived its parent")


def test_fabric_findings_catch_one_slow_link():
    """a node whose links are alike passes; one slow link,
    a bi cell below its uni cell, a wrong transport or unparsed RCCL lines
    each fail, by name."""
    from test_nccl_p2p_amd.utils.report import fabric_findings

    n = 4
    even = [[0.0 if i == j else 48.0 + (i + j) % 3 for j in range(n)] for i in range(n)]
    uni = [[0.0 if i == j else 390.0 for j in range(n)] for i in range(n)]
    bi = [[0.0 if i == j else 770.0 for j in range(n)] for i in range(n)]
    ok = {"direct_xgmi_pairs": 12, "not_p2p": [], "ok": True}
    assert fabric_findings(even, uni, bi, ok, []) == []
    assert fabric_findings(None, None, None, None, None) == []
    slow = [row[:] for row in even]
    slow[2][1] = 9.5
    f = fabric_findings(slow, uni, bi, ok, [])
    assert len(f) == 1 and f[0].startswith("tournament matrix_gbs: cell 2->1 9.50"), f
    slow_uni = [row[:] for row in uni]
    slow_uni[0][3] = 150.0
    f = fabric_findings(even, slow_uni, bi, ok, [])
    assert len(f) == 1 and "compat uni: cell 0->3" in f[0], f
    low_bi = [row[:] for row in bi]
    low_bi[1][0] = 380.0
    assert fabric_findings(even, uni, low_bi, ok, []) == ["compat bi cell 1<->0 380.00 below its uni cell 390.00"]
    bad = {"direct_xgmi_pairs": 12, "not_p2p": ["0->1 SHM"], "ok": False}
    assert "0->1 SHM" in fabric_findings(even, uni, bi, bad, [])[0]
    assert fabric_findings(even, uni, bi, ok, ["1->3"]) == ["RCCL connection lines not parsed for 1->3"]


def test_fabric_findings_on_the_rehearsals():
    """The matrices the one-GPU rehearsals kept (RCCL over loopback sockets,
    profiles/r5_reh4/, r5_reh8/) pass the rehearsal's bounds; the 8-rank one
    would fail a node's (slow socket pairs, bi below uni), which is why a
    rehearsal asks less."""
    import json

    from test_nccl_p2p_amd.utils.report import fabric_findings

    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from test_multi_gpu import REHEARSAL_MIN_RATIO

    for d, node_ok in (("r5_reh4", True), ("r5_reh8", False)):
        b = json.load(open(os.path.join(ROOT, "profiles", d, "fabric_bench.json")))
        c = json.load(open(os.path.join(ROOT, "profiles", d, "fabric_compat.json")))
        args = (b["matrix_gbs"], c["uni"], c["bi"], b["link_check"], b["unparsed_peers"])
        assert fabric_findings(*args, min_ratio=REHEARSAL_MIN_RATIO, bi_at_least_uni=False) == [], d
        assert (fabric_findings(*args) == []) == node_ok, d


def test_report_reads_the_drivers_pretty_printed_records(tmp_path, capsys):
    """The driver keeps each bench run as a pretty-printed record: an abridged
    `parsed` copy of the line plus the run's stdout tail.  The report tool
    takes the whole line from the tail, and finds every line of a record
    that holds several (one per GPU count)."""
    from test_nccl_p2p_amd.utils.report import bench_lines_in

    def line(n, v):
        return {"metric": "m", "n_gpus": n, "value": v, "aggregate_gbs": v * n, "matrix_gbs_min": v, "steps": 20}

    full = line(1, 2862.9)
    bench = {"n": 1, "rc": 0, "parsed": {"metric": "m", "n_gpus": 1, "value": 2862.9},
             "tail": "noise\n" + json.dumps(full) + "\n---- stderr ----\n"}
    assert bench_lines_in(bench) == [full]
    scale = {"runs": [{"parsed": line(1, 2800.0)}, {"parsed": line(2, 52.0)}, {"parsed": line(8, 50.0)}]}
    assert [r["n_gpus"] for r in bench_lines_in(scale)] == [1, 2, 8]
    assert bench_lines_in({"x": [1, "a", None]}) == []
    f = tmp_path / "SCALE_rNN.json"
    f.write_text(json.dumps(scale, indent=2))
    assert report_main([str(f)]) == 0
    out = capsys.readouterr().out
    assert "| 8 | 50.0 |" in out and "== scaling" in out

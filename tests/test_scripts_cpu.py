"""CPU checks of the operator scripts: the xGMI pair sweep runs end to end on
the host transport (emulated ranks) and refuses a 1-GPU box."""
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT

SWEEP = os.path.join(ROOT, "scripts", "xgmi_pair_sweep.py")


def test_pair_sweep_refuses_one_rank():
    out = subprocess.run([sys.executable, SWEEP, "--np", "1"], capture_output=True, text=True, timeout=60)
    assert out.returncode == 1 and "N >= 2" in out.stderr


def test_pair_sweep_dry_run_lists_every_knob():
    out = subprocess.run([sys.executable, SWEEP, "--np", "8", "--dry-run"], capture_output=True, text=True, timeout=60)
    assert out.returncode == 0, out.stderr
    txt = out.stdout
    for want in ("--comms 8", "NCCL_NCHANNELS_PER_PEER", "NCCL_P2P_NVL_CHUNKSIZE", "NCCL_P2P_NET_CHUNKSIZE",
                 "NCCL_PROTO", "RCCL_P2P_BATCH_ENABLE", "NCCL_P2P_READ_ENABLE", "P2P_RCCL_REGISTER=2",
                 "P2P_RCCL_UNROLL=0", "RCCL_UNROLL_FACTOR=2", "--ipc-engine sdma", "--ipc-engine push",
                 "--ipc-engine relay"):
        assert want in txt, want


@pytest.mark.mpi
def test_pair_sweep_host_emulation(mpirun, host_build, tmp_path):
    out = subprocess.run([sys.executable, SWEEP, "--np", "2", "--emulate", "host", "--sizes", "64K,1M",
                          "--out", str(tmp_path)], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr + out.stdout
    s = json.loads((tmp_path / "summary.json").read_text())
    assert s["failed_row"] is None and s["rows_run"] == 1
    assert set(s["best"]) == {"uni/65536", "uni/1048576", "bi/65536", "bi/1048576"}
    for b in s["best"].values():
        assert b["cell_gbs"] > 0 and b["gain"] == 1.0
    rows = [json.loads(l) for l in (tmp_path / "rows.jsonl").read_text().splitlines()]
    assert all(c["mismatches"] == 0 for r in rows for c in r["cells"].values())


@pytest.mark.mpi
def test_pair_sweep_records_a_corrupt_row_and_goes_on(mpirun, host_build, tmp_path):
    """A row whose bytes fail verification (here injected) is a finding, not a
    fault: it is listed in corrupt_rows, never wins, and the script exits 2."""
    out = subprocess.run([sys.executable, SWEEP, "--np", "2", "--emulate", "host", "--sizes", "64K",
                          "--out", str(tmp_path)], capture_output=True, text=True, timeout=300,
                         env=dict(os.environ, P2P_INJECT_FAULT="corrupt@1"))
    assert out.returncode == 2, out.stderr + out.stdout
    s = json.loads((tmp_path / "summary.json").read_text())
    assert s["failed_row"] is None and s["corrupt_rows"] == ["host"] and s["best"] == {}


def test_node_run_dry_run_and_refusal():
    """scripts/node_run.sh lists its four steps; without >= 2 GPUs it refuses
    (one-GPU boxes have their own scripts)."""
    script = os.path.join(ROOT, "scripts", "node_run.sh")
    out = subprocess.run(["bash", script, "/tmp/p2p_node_dry", "--dry-run"], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    for step in ("multi_gpu_tests", "reference_run", "scaling", "pair_sweep"):
        assert "== %s" % step in out.stdout
    assert "-n 8 ./p2p_matrix" in out.stdout
    out = subprocess.run(["bash", script, "/tmp/p2p_node_real"], capture_output=True, text=True, timeout=120)
    assert out.returncode == 1 and "needs >= 2 visible GPUs" in out.stderr
    # --rehearse: the same steps with 4 ranks on one GPU (profiles/r4_node_rehearsal/)
    out = subprocess.run(["bash", script, "/tmp/p2p_node_dry", "--dry-run", "--rehearse"], capture_output=True,
                         text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    assert "-n 4 ./p2p_matrix" in out.stdout and "--emulate rccl" in out.stdout and "--msgs 32" in out.stdout
    assert "rccl_repro_2gpu" not in out.stdout


@pytest.mark.mpi
def test_pair_sweep_resume_keeps_finished_rows(mpirun, host_build, tmp_path):
    args = [sys.executable, SWEEP, "--np", "2", "--emulate", "host", "--sizes", "64K", "--out", str(tmp_path)]
    first = subprocess.run(args, capture_output=True, text=True, timeout=300)
    assert first.returncode == 0, first.stderr + first.stdout
    again = subprocess.run(args + ["--resume"], capture_output=True, text=True, timeout=300)
    assert again.returncode == 0, again.stderr + again.stdout
    assert "kept from the previous run" in again.stdout
    rows = [json.loads(l) for l in (tmp_path / "rows.jsonl").read_text().splitlines()]
    assert [r["name"] for r in rows] == ["host"]
    assert json.loads((tmp_path / "summary.json").read_text())["rows_run"] == 1


def emulated_tests():
    """Names of the tests marked `emulated` (several ranks on one GPU): on a
    node with >= 2 GPUs conftest skips them, the multi-GPU tier runs the
    same flows across the real GPUs instead."""
    import ast
    import glob

    names = set()
    for path in glob.glob(os.path.join(ROOT, "tests", "test_*.py")):
        for f in ast.parse(open(path).read()).body:
            if isinstance(f, ast.FunctionDef) and any("emulated" in ast.dump(d) for d in f.decorator_list):
                names.add(f.name)
    return names


def measured_single_gpu_tier_s():
    """Duration of the single-GPU tier on a multi-GPU node, from the runs on
    one-GPU MI355X boxes: the final line of every profiles/r<k>*/pytest_gpu*.log
    of the latest round k that has one (a whole tier, not a failed run, run
    with --durations), less
    the `emulated` tests' durations its --durations table lists (skipped on a
    node), worst case."""
    import glob
    import re

    emulated = emulated_tests()
    runs = []
    for path in glob.glob(os.path.join(ROOT, "profiles", "r*", "pytest_gpu*.log")):
        rnd = re.match(r"r(\d+)", os.path.basename(os.path.dirname(path)))
        with open(path) as f:
            lines = [l for l in f.read().splitlines() if l.strip()]
        m = re.search(r"(\d+) passed.* in ([\d.]+)s", lines[-1] if lines else "")
        # Only a log with pytest's --durations table can have the emulated
        # tests taken out; one without it (a plain -q run) is not comparable.
        has_durations = any("slowest" in l and "durations" in l for l in lines)
        if rnd and m and "failed" not in lines[-1] and has_durations:
            skipped_on_node = sum(float(d.group(1)) for d in (re.match(r"([\d.]+)s call\s+\S+::(\w+)", l) for l in lines)
                                  if d and d.group(2) in emulated)
            runs.append((int(rnd.group(1)), float(m.group(2)) - skipped_on_node, path))
    assert runs, "no measured GPU-tier log under profiles/"
    latest = max(r[0] for r in runs)
    return max((r[1], r[2]) for r in runs if r[0] == latest)


def test_multi_gpu_tier_fits_the_driver_step():
    """the driver runs `pytest -m gpu` in one 900 s step.
    The measured single-GPU duration (worst run of the latest round) + every
    multi-GPU test's worst-case budget (the sum of its subprocess limits) ends
    by conftest.SESSION_LIMIT_S, which leaves 60 s for the perf floors; the
    guard in conftest.py applies the same rule per test at run time."""
    import ast

    import conftest

    src = open(os.path.join(ROOT, "tests", "test_multi_gpu.py")).read()
    tree = ast.parse(src)
    tests = [f.name for f in tree.body if isinstance(f, ast.FunctionDef) and f.name.startswith("test_")]
    budget = next(ast.literal_eval(a.value) for a in tree.body
                  if isinstance(a, ast.Assign) and getattr(a.targets[0], "id", "") == "BUDGET_S")
    assert sorted(tests) == sorted(budget), "every multi-GPU test needs a budget"
    single_s, log = measured_single_gpu_tier_s()
    assert single_s + sum(budget.values()) <= conftest.SESSION_LIMIT_S <= 840, (single_s, log, budget)
    # Every subprocess limit in the file is taken from the budget table.
    for f in tree.body:
        if isinstance(f, ast.FunctionDef) and f.name.startswith("test_"):
            for node in ast.walk(f):
                if isinstance(node, ast.keyword) and node.arg == "timeout" and isinstance(node.value, ast.Constant):
                    raise AssertionError("%s: a literal subprocess timeout outside BUDGET_S" % f.name)


def test_gpu_tier_order_puts_floors_last():
    """under the driver's `pytest -x -m gpu`, every
    RCCL correctness test runs before the multi-GPU tier, and the perf floors
    run after everything else."""
    out = subprocess.run([sys.executable, "-m", "pytest", "--collect-only", "-q", "-m", "gpu", "tests"],
                         capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert out.returncode == 0, out.stdout[-3000:] + out.stderr[-3000:]
    ids = [l for l in out.stdout.splitlines() if "::" in l]
    tier = [2 if "test_zz_perf_floors_gpu.py" in i else 1 if "test_multi_gpu.py" in i else 0 for i in ids]
    assert tier == sorted(tier), "collection order mixes the tiers"
    rccl = [n for n, i in enumerate(ids) if "test_rccl_gpu.py" in i or "test_rccl_ranks_gpu.py" in i]
    assert len(rccl) > 30 and max(rccl) < tier.index(1) < tier.index(2)


def test_kernel_overlap_bursts_and_concurrency(tmp_path):
    """scripts/kernel_overlap.py on a hand-made trace: two bursts split at an
    idle gap; in the first, two queues overlap for half of each kernel."""
    rows = [("rcclGenericKernel<4, false>", 1, 0, 100_000), ("rcclGenericKernel<4, false>", 2, 50_000, 150_000),
            ("fill_grid_kernel", 1, 150_000, 4_000_000),  # not matched: does not bridge the gap
            ("rcclGenericKernel<4, false>", 1, 5_000_000, 5_100_000)]
    trace = tmp_path / "t_kernel_trace.csv"
    with open(trace, "w") as f:
        f.write('"Kernel_Name","Queue_Id","Start_Timestamp","End_Timestamp"\n')
        for name, q, s, e in rows:
            f.write('"%s",%d,%d,%d\n' % (name, q, s, e))
    out = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "kernel_overlap.py"), str(trace),
                          "--min-kernels", "1", "--json"], capture_output=True, text=True, check=True)
    first, second = [json.loads(l) for l in out.stdout.splitlines()]
    assert first["kernels"] == 2 and first["queues"] == 2 and first["peak_concurrency"] == 2
    assert first["span_ms"] == 0.15 and first["busy_ms"] == 0.15 and first["busy_fraction"] == 1.0
    assert first["mean_concurrency"] == round(200 / 150, 3)
    assert second["kernels"] == 1 and second["burst"] == 1


def test_every_top_level_script_is_referenced():
    """the top level of scripts/ holds only maintained
    tooling -- each file is referenced by a test, the Makefile, README.md,
    docs/, the package, bench.py or another maintained script; one-shot
    probes live in scripts/probes/."""
    import glob

    sources = []
    for pat in ("tests/*.py", "Makefile", "README.md", "docs/*.md", "bench.py", "__graft_entry__.py",
                "test_nccl_p2p_amd/**/*.py", "scripts/*"):
        sources += [p for p in glob.glob(os.path.join(ROOT, pat), recursive=True) if os.path.isfile(p)]
    texts = {p: open(p, errors="replace").read() for p in sources}
    for path in glob.glob(os.path.join(ROOT, "scripts", "*")):
        if os.path.isdir(path):
            continue
        name = os.path.basename(path)
        refs = [p for p, t in texts.items() if p != path and "scripts/" + name in t]
        assert refs, "scripts/%s is referenced nowhere: move it to scripts/probes/" % name


def test_busy_fraction_union_and_gaps(tmp_path):
    """scripts/busy_fraction.py: overlapping kernels count once, the span runs
    from the first start to the last end, and the idle gaps are the holes
    between busy stretches."""
    sys.path.insert(0, os.path.join(ROOT, "scripts"))
    import busy_fraction

    st = busy_fraction.busy_stats([(0, 10_000), (5_000, 20_000), (30_000, 40_000), (60_000, 70_000)])
    assert st["span_us"] == 70.0 and st["busy_us"] == 40.0 and st["busy_fraction"] == round(40 / 70, 4)
    assert st["kernels"] == 4 and st["idle_gaps"] == 2 and st["idle_gap_p50_us"] == 15.0
    p = tmp_path / "t_kernel_trace.csv"
    p.write_text("Kernel_Name,Start_Timestamp,End_Timestamp\nrcclGenericKernel<4>,100,300\nfill,300,900\n"
                 "rcclGenericKernel<4>,400,500\n")
    assert busy_fraction.read_trace(str(p), "rccl") == [(100, 300), (400, 500)]
    assert busy_fraction.main([str(p), "--json", str(tmp_path / "o.json")]) == 0

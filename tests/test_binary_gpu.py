"""Tier T3: the p2p_matrix executable and bench.py on one MI355X."""
import json
import os
import subprocess
import sys

import pytest

from conftest import MPIRUN, ROOT, ensure_built, free_port
from test_nccl_p2p_amd.utils.report import parse_compat

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def exe():
    ensure_built("gpu")
    return os.path.join(ROOT, "build", "p2p_matrix")


def test_default_run_single_rank_compat(exe):
    out = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr
    m = parse_compat(out.stdout)
    assert m == {"uni": [[0.0]], "bi": [[0.0]]}
    assert "gfx950" in out.stdout


def test_self_sweep_verify(exe, tmp_path):
    js = tmp_path / "r.json"
    out = subprocess.run([exe, "--mode", "self", "--sizes", "4K:256M:4", "-n", "auto", "--verify", "--latency",
                          "--json", str(js), "--verify-impl", "lds"], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr
    runs = [json.loads(l) for l in js.read_text().splitlines()]
    assert sum(1 for r in runs if r["type"] == "run") == 9  # 4K,16K,...,256M
    assert "verification: OK" in out.stdout


@pytest.mark.skipif(not os.path.exists(MPIRUN), reason="no mpirun")
def test_mpirun_one_rank(exe):
    out = subprocess.run([MPIRUN, "-n", "1", exe, "--mode", "pair,self", "--size", "8M", "-n", "8", "--verify"],
                         capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr
    assert "bootstrap mpi" in out.stdout


@pytest.mark.skipif(not os.path.exists(MPIRUN), reason="no mpirun")
def test_reference_invocation_from_repo_root(exe):
    """`make` leaves ./p2p_matrix like the reference's Makefile; the reference
    run line (README.md:5 there) works unchanged and prints the two matrices."""
    out = subprocess.run([MPIRUN, "-n", "1", "./p2p_matrix"], capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert out.returncode == 0, out.stderr
    assert out.stdout.startswith("Evaluating the Uni-Directional NCCL P2P Bandwidth (Gbps)\n   D\\D     0 \n     0   0.00 \n")
    assert "Evaluating the Bi-Directional NCCL P2P Bandwidth (Gbps)" in out.stdout


def test_repeat_self_summary(exe, tmp_path):
    """--repeat 4: the self cell measured four times on the card, summarised
    (median / min / max) and recorded as one repeats record per size."""
    js = tmp_path / "r.json"
    out = subprocess.run([exe, "--mode", "self", "--size", "64M", "-n", "8", "--repeat", "4", "--verify",
                          "--json", str(js)], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr
    assert "== repeats" in out.stdout and "verification: OK" in out.stdout
    recs = [json.loads(l) for l in js.read_text().splitlines()]
    assert sum(1 for r in recs if r["type"] == "run") == 4
    rep = [r for r in recs if r["type"] == "repeats"]
    assert len(rep) == 1 and len(rep[0]["runs"]) == 4
    assert rep[0]["min"] <= rep[0]["median"] <= rep[0]["max"] and rep[0]["min"] > 10


def test_bench_contract_single_gpu():
    out = subprocess.run([sys.executable, "bench.py", "--steps", "6", "--warmup", "2", "--latency-iters", "50"],
                         capture_output=True, text=True, timeout=600, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1
    r = json.loads(lines[0])
    assert r["n_gpus"] == 1 and r["steps"] == 6 and r["value"] > 10
    assert r["verify_mismatches"] == 0 and r["transport"] == "rccl" and r["verify_coverage"] == 1.0
    # The posting the tuning laps chose is never slower than one communicator.
    t = r["posting"]["tuning_ms_per_step"]
    chosen = "comms%d_%s" % (r["posting"]["rccl_comms"], "batch" if r["posting"]["batch"] else "per_message")
    assert t[chosen] <= min(v for k, v in t.items() if k.startswith("comms1_")), t
    # several communicators (4, or 8 with bench.py's 8 hardware queues): ~2x one on the self path
    assert r["posting"]["rccl_comms"] in (4, 8) and r["posting"]["hw_queues"]["GPU_MAX_HW_QUEUES"] == 8, t
    assert isinstance(r["p50_latency_us"], float) and r["p50_latency_us"] > 0
    assert 0 < r["p50_latency_preposted_us"] <= r["p50_latency_us"] * 1.2 + 1.0, r["p50_latency_preposted_us"]
    # The hand-written data plane runs the same self step after the timed
    # region: pull, push and SDMA engines, all verified.
    ipc = r["ipc_transport"]
    assert ipc["verify_mismatches"] == 0 and ipc["value_gbs"] > 0, ipc
    assert ipc["push"]["verify_mismatches"] == 0 and ipc["sdma"]["verify_mismatches"] == 0, ipc
    assert 0 < ipc["device_pingpong_p50_us"] < 50, ipc
    # The reference's methodology twice on the self cell: in this process
    # (RCCL unroll 4, 8 HW queues, INFO log) and in a child with the stock
    # settings, same iterations; both method ratios reported.
    ref, stock = r["reference_semantics"], r["reference_semantics_stock"]
    assert stock["uni"]["iters"] == ref["uni"]["iters"] and stock["uni"]["gbs_mean"] > 0, stock
    assert stock["env"]["P2P_RCCL_UNROLL"] == "0" and stock["env"]["RCCL_UNROLL_FACTOR"] is None, stock
    assert stock["env"]["GPU_MAX_HW_QUEUES"] in (None, "4"), stock
    assert r["method_ratio_stock"]["uni"] > 0 and r["method_ratio"]["uni"] > 0
    # >= 5 runs of each reference-method matrix (in
    # the stock child too), ratios of the medians; the size sweep on the self
    # cell, every size verified; value labelled as the on-GPU self copy.
    for x in (ref, stock, r["pair_serial_events"]):
        assert len(x["uni"]["runs"]) >= 5 and x["uni"]["min"] <= x["uni"]["median"] <= x["uni"]["max"], x
    assert abs(r["method_ratio"]["uni"] - r["pair_serial_events"]["uni"]["median"] / ref["uni"]["median"]) < 0.002
    sw = r["extras"]["self_sweep"]
    assert len(sw) >= 10 and all(p["mismatches"] == 0 and p["gbs"] > 0 for p in sw), sw
    assert r["value_kind"] == "self-copy (on-GPU HBM)"


def test_topology_probe(exe):
    out = subprocess.run([exe, "--topology"], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    assert "GPU link topology" in out.stdout and "visible" in out.stdout


def test_reference_methodology_two_streams(exe):
    # --reference: wall clock, sync per message, no warmup; a receive in a
    # group with a send goes on a second stream (the reference's bi loop,
    # s_1): the self cell's does.  Self path so one GPU suffices.
    out = subprocess.run([exe, "--mode", "self", "--size", "32M", "-n", "16", "--reference", "--verify", "--no-compat"],
                         capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr
    assert "timing=wallclock warmup=0" in out.stdout and "verification: OK" in out.stdout


def test_cli_several_communicators(exe):
    """--comms 4 through the binary: all self-path modes, verified, a size
    sweep that crosses the 1 MiB spreading threshold."""
    out = subprocess.run([exe, "--mode", "self,ring,allpairs", "--sizes", "64K:64M:16", "-n", "6", "--comms", "4",
                          "--verify", "--no-compat"], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-3000:]
    assert "verification: OK" in out.stdout


@pytest.mark.parametrize("comms", ["1", "4"])
def test_cli_fuzz_rccl(exe, comms):
    """--fuzz through the binary on the GPU: random message groups (self pairs
    on one rank, sizes 1 B .. 64 MiB) over one or four communicators."""
    out = subprocess.run([exe, "--mode", "self", "--size", "64M", "-n", "2", "--comms", comms, "--fuzz", "40",
                          "--no-compat"], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-3000:]
    assert "groups of random messages" in out.stdout and "all verified" in out.stdout


def test_cli_rechunks_when_the_warmup_does_not_verify(exe):
    """p2p_matrix --verify under RCCL's 16 MiB-per-p2p-channel loss (one
    channel, the transport's own chunking off): the warmup's deliveries do
    not verify, the run reposts as 16 MiB ops, and the timed iterations
    verify; K = 1 and 4 communicators."""
    env = dict(os.environ, NCCL_MAX_P2P_NCHANNELS="1", P2P_RCCL_MAX_CHUNK="0")
    for comms in ("1", "4"):
        out = subprocess.run([exe, "--mode", "self", "--sizes", "8M,32M", "-n", "4", "--verify", "--no-compat",
                              "--comms", comms], capture_output=True, text=True, timeout=300, env=env)
        assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-2000:]
        assert "verification: OK" in out.stdout
        assert "messages now posted as ops of <= 16 MiB" in out.stderr, out.stderr[-2000:]


def test_bench_drops_a_failing_communicator_candidate():
    """If the 4-communicator candidate fails (injected), bench.py reports it
    in posting.dropped and times the remaining postings (one communicator, or
    eight with bench.py's 8 hardware queues) instead; with one warmup step it
    falls back the same way."""
    for warmup in ("1", "4"):
        out = subprocess.run([sys.executable, "bench.py", "--steps", "4", "--warmup", warmup, "--latency-iters", "20",
                              "--ref-stock", "0"],
                             capture_output=True, text=True, timeout=600, cwd=ROOT,
                             env=dict(os.environ, P2P_BENCH_FAIL_CANDIDATE="4,1"))
        assert out.returncode == 0, out.stderr[-3000:]
        r = json.loads([l for l in out.stdout.splitlines() if l.startswith("{")][0])
        assert r["posting"]["rccl_comms"] in (1, 8) and "injected" in r["posting"]["dropped"]["comms4_batch"]
        assert "comms4_batch" not in r["posting"]["tuning_ms_per_step"]
        assert r["verify_mismatches"] == 0 and r["value"] > 10


def test_bench_chunks_around_rccl_half_delivery():
    """RCCL delivers only the first half of a send/recv whose share of one p2p
    channel exceeds 16 MiB (scripts/rccl_half_repro.cpp).  With one p2p
    channel (NCCL_MAX_P2P_NCHANNELS=1) the transport reads "1 p2p channels"
    from RCCL's INFO log and posts the bench's 32 MiB messages as 16 MiB ops
    by itself (provenance.rccl_peers says so); with its splitting turned off
    (P2P_RCCL_MAX_CHUNK=0) the bench's verified warmup sees the loss, caps the
    ops at 16 MiB, and the timed steps verify; with the fallback off too
    (P2P_RECHUNK=0) the loss reaches the timed check: exit 3."""
    base = [sys.executable, "bench.py", "--steps", "4", "--warmup", "2", "--comms", "1", "--ipc-extra", "0",
            "--ref-iters", "0", "--latency-iters", "20"]
    runs = {}
    for name, extra, rc in (("transport", {}, 0), ("fallback", {"P2P_RCCL_MAX_CHUNK": "0"}, 0),
                            ("off", {"P2P_RCCL_MAX_CHUNK": "0", "P2P_RECHUNK": "0"}, 3)):
        out = subprocess.run(base, capture_output=True, text=True, timeout=600, cwd=ROOT,
                             env=dict(os.environ, NCCL_MAX_P2P_NCHANNELS="1", **extra))
        assert out.returncode == rc, (name, out.stderr[-3000:])
        runs[name] = json.loads([l for l in out.stdout.splitlines() if l.startswith("{")][0])
    for name in ("transport", "fallback"):
        assert runs[name]["verify_mismatches"] == 0 and runs[name]["verify_coverage"] == 1.0, runs[name]
    ch = runs["transport"]["posting"]["chunking"]
    assert ch == {"op_limit_bytes": 16 << 20, "warmup_mismatches": 0, "fallback": None, "cap_bytes": None,
                  "recaptured_graphs": 0}, ch
    peers = runs["transport"]["provenance"]["rccl_peers"][0]
    assert peers["comms"][0]["p2p_channels"] == 1 and peers["op_limit_source"].startswith("rccl INFO log"), peers
    assert peers["peers"][0]["op_channels"] == 1 and peers["peers"][0]["op_limit"] == 16 << 20, peers
    assert runs["transport"]["matrix_transport"] == [["self"]]
    ch = runs["fallback"]["posting"]["chunking"]
    assert ch["warmup_mismatches"] > 0, ch
    assert ch["fallback"] == [{"cap_bytes": 16 << 20, "warmup_mismatches": 0}], ch
    assert ch["op_limit_bytes"] == 16 << 20 and ch["cap_bytes"] == 16 << 20
    ch = runs["off"]["posting"]["chunking"]
    assert ch["fallback"] == "off (P2P_RECHUNK=0)" and runs["off"]["verify_mismatches"] > 0, ch


def test_bench_headline_falls_back_to_ipc():
    """Should RCCL fail on the node (injected on every rank), the timed steps
    run through the IPC data plane and the line names the fallback; the
    metric is RCCL's, so value is null and the IPC number sits beside it."""
    out = subprocess.run([sys.executable, "bench.py", "--steps", "4", "--warmup", "2", "--latency-iters", "20",
                          "--ref-iters", "8", "--ipc-extra", "0"],
                         capture_output=True, text=True, timeout=600, cwd=ROOT,
                         env=dict(os.environ, P2P_BENCH_FAIL_HEADLINE="rccl"))
    assert out.returncode == 0, out.stderr[-3000:]
    r = json.loads([l for l in out.stdout.splitlines() if l.startswith("{")][0])
    assert r["transport"] == "ipc" and r["headline_fallback"]["from"] == "rccl", r.get("headline_fallback")
    assert r["verify_mismatches"] == 0 and r["verify_coverage"] == 1.0
    assert r["value"] is None and r["headline_fallback"]["value_gbs"] > 10, r["headline_fallback"]


@pytest.mark.parametrize("transport", ["rccl", "ipc"])
def test_preposted_latency(exe, tmp_path, transport):
    """--latency-preposted: the self ping-pong posted 16 at a time behind a
    stream gate runs without the host in the loop, so its p50 is at most the
    host-posted one's (plus noise)."""
    js = tmp_path / "l.json"
    out = subprocess.run([exe, "--transport", transport, "--mode", "self", "--size", "4K", "-n", "2",
                          "--latency-preposted", "16", "--latency-iters", "400", "--no-compat", "--json", str(js)],
                         capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-3000:]
    recs = {r["method"]: r for r in (json.loads(l) for l in js.read_text().splitlines()) if r["type"] == "latency"}
    host, pre = recs["host"]["pairs"][0]["one_way_us"], recs["preposted"]["pairs"][0]["one_way_us"]
    assert 0 < pre["p50"] <= host["p50"] * 1.2 + 1.0, (pre, host)
    assert "pre-posted behind a stream gate" in out.stdout


def test_bench_real_rccl_failure_falls_back():
    """A genuine RCCL failure, not an injected one: two ranks on the one GPU
    with no --device, so RCCL refuses the duplicate GPU at communicator init
    on both ranks; the timed steps run through the IPC data plane instead,
    verified, and the line names the RCCL error."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(free_port()), "bench.py", "--gpus", "2", "--steps", "6", "--warmup", "3",
           "--size", "4M", "--msgs", "4", "--sweep", "0", "--extras", "0", "--ref-iters", "0", "--latency-iters", "20",
           "--ipc-extra", "0", "--timeout", "60"]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=600, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-3000:]
    r = json.loads([l for l in out.stdout.splitlines() if l.startswith("{")][0])
    fb = r["headline_fallback"]
    assert r["transport"] == "ipc" and fb["from"] == "rccl" and "ncclCommInitRankConfig" in fb["error"], fb
    assert r["verify_mismatches"] == 0 and r["verify_coverage"] == 1.0 and r["matrix_cells"] == "2/2"
    assert r["value"] is None and fb["value_gbs"] > 0

"""RCCL itself with several ranks on the one GPU of a test box.

RCCL refuses two ranks on one GPU of one host ("Duplicate GPU detected"), so
P2P_RCCL_DISTINCT_HOSTS=1 makes every rank claim a host of its own
(NCCL_HOSTID) and RCCL connects the ranks through its socket network
transport on loopback.  The bytes do not cross xGMI, but every multi-rank
RCCL code path does run: communicator setup across ranks, K communicators
with the (count + src + dst) routing and the sorted launch order, the
tournament / ring / all-pairs schedules, the ring token chain, the latency
matrix, and bench.py's N-rank flow with its communicator candidates.  This is
what the driver's multi-GPU run executes, minus the link.
"""
import json
import os
import re
import subprocess
import sys

import pytest

from conftest import MPIRUN, ROOT, ensure_built, free_port, run_logged

pytestmark = [pytest.mark.gpu]

ENV = dict(os.environ, P2P_RCCL_DISTINCT_HOSTS="1", NCCL_SOCKET_IFNAME="lo", NCCL_IB_DISABLE="1")


@pytest.fixture(scope="module")
def exe():
    ensure_built("gpu")
    return os.path.join(ROOT, "build", "p2p_matrix")


@pytest.mark.skipif(not os.path.exists(MPIRUN), reason="no mpirun")
@pytest.mark.parametrize("comms", ["1", "4"])
def test_cli_four_rccl_ranks_every_mode(exe, tmp_path, comms):
    js = tmp_path / "r.json"
    out = subprocess.run([MPIRUN, "-n", "4", exe, "--device", "0", "--mode", "pair,tournament,ring,allpairs",
                          "--size", "4M", "-n", "4", "--comms", comms, "--verify", "--latency", "--latency-iters", "30",
                          "--latency-preposted", "8",
                          "--json", str(js), "--timeout", "60"],
                         capture_output=True, text=True, timeout=300, env=ENV)
    assert out.returncode == 0, out.stderr[-3000:]
    assert "verification: OK" in out.stdout
    assert out.stdout.startswith("Evaluating the Uni-Directional NCCL P2P Bandwidth (Gbps)")
    recs = [json.loads(l) for l in js.read_text().splitlines()]
    prov = [r for r in recs if r["type"] == "provenance"][0]
    assert prov["env"]["NCCL_HOSTID"].startswith("p2p-emulated-host-")
    assert "ring token latency: 4 rank(s)" in out.stdout
    # The pre-posted ping-pong (stream gates on every rank, released together)
    # ran through RCCL across ranks: every pair has samples.
    pre = [r for r in recs if r["type"] == "latency" and r["method"] == "preposted"]
    assert len(pre) == 1 and len(pre[0]["pairs"]) == 6 and all(p["one_way_us"]["p50"] > 0 for p in pre[0]["pairs"])
    # The CLI re-derives each peer's op limit from RCCL's connection lines
    # after its warm-up; both ends of every pair agree.
    links = [r for r in recs if r["type"] == "links"][0]
    for rep in links["ranks"]:
        assert rep["refinements"] >= 1, rep
        for p in rep["peers"]:
            if p["peer"] != rep["rank"]:
                assert p["op_limit_source"] == "connection lines" and p["op_limit"] == 32 << 20, p
    limit = {(rep["rank"], p["peer"]): p["op_limit"] for rep in links["ranks"] for p in rep["peers"]}
    assert all(limit[(a, b)] == limit[(b, a)] for (a, b) in limit), limit


@pytest.mark.emulated
def test_bench_four_rccl_ranks(tmp_path):
    """bench.py's whole N = 4 flow through RCCL: the five posting candidates
    (1 communicator per message / batched, 2, 4 and 8 communicators), the
    tournament steps with every delivery verified, and every untimed section."""
    out_json = tmp_path / "b.json"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "4", "--master-addr",
           "127.0.0.1", "--master-port", str(free_port()), "bench.py", "--gpus", "4", "--device", "0", "--size", "4M",
           "--msgs", "8", "--sweep-max", "16M", "--allpairs-size", "16M", "--ring-size", "8M", "--ref-iters", "8",
           "--latency-iters", "30", "--ipc-extra", "0", "--timeout", "60", "--json-out", str(out_json)]
    out = run_logged(cmd, 400, "bench_four_rccl_ranks", cwd=ROOT, env=ENV)
    progress = "\n".join(l for l in out.stderr.splitlines() if "bench:" in l or "fatal" in l or "Error" in l)
    assert out.returncode == 0, progress[-3000:]
    r = json.loads(out_json.read_text())
    assert r["transport"] == "rccl" and r["headline_fallback"] is None
    assert r["value_kind"].startswith("emulated: 4 ranks on 1 GPU"), r["value_kind"]
    # The reference-method matrices repeat, in-process and in the stock child.
    for key in ("reference_semantics", "reference_semantics_stock", "pair_serial_events"):
        assert all(len(r[key][d]["runs"]) >= 2 for d in ("uni", "bi")), r[key]
    assert r["verify_mismatches"] == 0 and r["verify_coverage"] == 1.0 and r["matrix_cells"] == "12/12"
    tuned = r["posting"]["tuning_ms_per_step"]
    assert set(tuned) == {"comms1_per_message", "comms1_batch", "comms2_batch", "comms4_batch", "comms8_batch"}, tuned
    assert r["untimed_skipped"] is None and r.get("section_errors") is None
    ex = r["extras"]
    assert ex["allpairs_1g"]["mismatches"] == 0 and ex["ring_256m"]["mismatches"] == 0
    assert ex["ring_hop"]["hop_us_p50"] > 0
    assert all(p["mismatches"] == 0 and p["iter_us_p50"] > 0 for p in ex["pair_sweep_0_1"]), ex["pair_sweep_0_1"]
    lat = r["latency_p50_us_matrix"]
    assert all(lat[a][b] > 0 for a in range(4) for b in range(4) if a != b)
    # BASELINE config 3 by both methods on the reference's serial schedule, uni and bi
    for key in ("reference_semantics", "pair_serial_events"):
        assert r[key]["uni"]["gbs_mean"] > 0 and r[key]["bi"]["gbs_mean"] > 0, r[key]
    assert r["pair_serial_events"]["bi"]["mismatches"] == 0 and r["concurrency_ratio"] > 0
    assert r["method_ratio"]["uni"] > 0 and r["method_ratio"]["bi"] > 0
    # Op limits per peer from RCCL's connection lines after the warm-up
    # (VERDICT r3 item 3): NET peers, 2 channels connected, 32 MiB ops.
    for rep in r["provenance"]["rccl_peers"]:
        assert rep["refinements"] >= 1, rep
        for p in rep["peers"]:
            if p["peer"] == rep["rank"]:
                assert p["op_limit_source"] == "init line", p
            else:
                assert p["op_limit_source"] == "connection lines" and p["channels_connected"] == 2, p
                assert p["op_limit"] == 32 << 20, p
    # Every connected peer's RCCL lines were parsed.
    assert r["unparsed_peers"] == [], r["unparsed_peers"]
    # And every rank keeps a sample of RCCL's real log: version, channel
    # counts, connection lines (here over its socket transport).
    for rep in r["provenance"]["rccl_peers"]:
        sample = rep["log_sample"]
        assert any("RCCL version" in l for l in sample) and any(" via NET" in l for l in sample), sample


@pytest.mark.emulated
def test_bench_deadline_aborts_rccl_inside_and_outside_the_engine(tmp_path):
    """the deadline watchdog gets the RCCL communicators of every
    rank aborted wherever its main thread is.  Rank 1 stalls in Python during
    the first posting candidate (outside the engine: the watchdog aborts them
    from its own thread, abort_if_idle); rank 0, its session's timeout lifted,
    sits in the transport's wait for rank 1's messages (the wait sees the
    request and aborts them on the main thread).  Both end with exit 4
    (nothing measured) and neither crashes."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(free_port()), "bench.py", "--gpus", "2", "--device", "0", "--size", "4M",
           "--msgs", "4", "--ipc-extra", "0", "--timeout", "60", "--deadline", "25"]
    env = dict(ENV, P2P_BENCH_HANG="candidate:rccl:1,0:stall@1;candidate:rccl:1,0:unbounded@0")
    out = run_logged(cmd, 90, "bench_deadline_abort", cwd=ROOT, env=env)
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert out.returncode != 0 and len(lines) == 1, out.stderr[-3000:]
    r = json.loads(lines[0])
    assert r["value"] is None and r["deadline_hit"] is True, r
    assert r["timeline_s"]["open"] == "tuning/comms1_per_message/pass0", r["timeline_s"]
    assert "communicators aborted by the main thread's wait" in out.stderr, out.stderr[-3000:]
    assert "communicators aborted by the watchdog (engine idle)" in out.stderr, out.stderr[-3000:]
    assert "Signal 11" not in out.stderr and "SIGSEGV" not in out.stderr, out.stderr[-3000:]
    # Every rank ended through its watchdog with exit status 4 (nothing measured), or was stopped by
    # torchrun's SIGTERM (-15) once a peer had; none by an exception (1) or a crash.
    codes = re.findall(r"exitcode\s*:\s*(-?\d+)", out.stderr.split("Failures:")[-1])
    assert codes and set(codes) <= {"4", "-15"} and "4" in codes, (codes, out.stderr[-3000:])


@pytest.mark.skipif(not os.path.exists(MPIRUN), reason="no mpirun")
def test_cli_four_rccl_ranks_reference_method(exe):
    """The reference's own methodology through RCCL across ranks: serial
    ordered pairs, host clock, a stream sync per message; uni receives on s_0,
    bi sends on s_0 and receives on s_1 (p2p_matrix.cc:141-267), compat
    matrices on stdout."""
    out = subprocess.run([MPIRUN, "-n", "4", exe, "--device", "0", "--reference", "--size", "4M", "-n", "8", "--verify",
                          "--timeout", "60"], capture_output=True, text=True, timeout=300, env=ENV)
    assert out.returncode == 0, out.stderr[-3000:]
    assert "timing=wallclock warmup=0" in out.stdout and "verification: OK" in out.stdout
    assert "Evaluating the Bi-Directional NCCL P2P Bandwidth (Gbps)" in out.stdout


@pytest.mark.skipif(not os.path.exists(MPIRUN), reason="no mpirun")
@pytest.mark.parametrize("comms", ["1", "4"])
def test_cli_four_rccl_ranks_fuzz(exe, comms):
    """Random message groups across 4 RCCL ranks (random pairs incl. self,
    repeated peers, 1 B .. 4 MiB), every message verified; with 4
    communicators this checks that both ends route every message to the same
    communicator whatever the group's shape."""
    out = subprocess.run([MPIRUN, "-n", "4", exe, "--device", "0", "--mode", "self", "--size", "4M", "-n", "1",
                          "--comms", comms, "--fuzz", "60", "--no-compat", "--timeout", "60"],
                         capture_output=True, text=True, timeout=300, env=ENV)
    assert out.returncode == 0, out.stderr[-3000:]
    assert "all verified" in out.stdout


@pytest.mark.emulated
def test_rccl_teardown_with_a_pending_receive_is_bounded():
    """A session dropped while an RCCL receive is still pending (its peer never
    sends) is torn down within its timeout: the transport's drain aborts the
    communicators instead of waiting on the stream forever, and it runs
    without the GIL, so another Python thread -- bench.py's deadline
    watchdog -- keeps running meanwhile (tests/scripts/teardown_pending.py)."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(free_port()), "tests/scripts/teardown_pending.py"]
    out = run_logged(cmd, 90, "teardown_pending", cwd=ROOT, env=ENV)
    assert out.returncode == 0, out.stderr[-3000:]
    m = re.search(r"TEARDOWN ([0-9.]+) s, ticker ran (\d+) times", out.stdout)
    assert m, out.stdout[-2000:]
    assert 2.5 < float(m.group(1)) < 20 and int(m.group(2)) >= 5, m.group(0)

"""Multi-rank GPU engine on ONE MI355X through the IPC transport: several
processes share the GPU and pull from each other's hipIpc-mapped send
buffers with the gfx950 multi-copy kernel (or SDMA).  Exercises every
schedule, hipEvent timing and device-side verification with N > 1, which the
RCCL transport cannot do on one GPU (duplicate-GPU ranks are refused)."""
import json
import os
import subprocess
import sys

import pytest

from conftest import MPIRUN, ROOT, ensure_built, free_port, run_logged
from test_nccl_p2p_amd.utils.report import parse_compat

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not os.path.exists(MPIRUN), reason="no mpirun")]


@pytest.fixture(scope="module")
def exe():
    ensure_built("gpu")
    return os.path.join(ROOT, "build", "p2p_matrix")


@pytest.mark.parametrize("engine", ["kernel", "sdma", "push"])
def test_two_ranks_all_modes(exe, tmp_path, engine):
    js = tmp_path / "r.json"
    out = subprocess.run([MPIRUN, "-n", "2", exe, "--transport", "ipc", "--ipc-engine", engine, "--device", "0",
                          "--mode", "all", "--sizes", "4K:16M:4", "-n", "6", "--verify", "--latency",
                          "--latency-iters", "50", "--json", str(js), "--timeout", "60"], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-3000:]
    m = parse_compat(out.stdout)
    assert m["uni"][0][1] > 0 and m["bi"][1][0] > 0
    runs = [json.loads(l) for l in js.read_text().splitlines() if '"run"' in l]
    assert len(runs) == 7 * 7  # 7 runs (3 modes x 2 dirs + allpairs) x 7 sizes
    assert all(ph["mismatches"] == 0 for r in runs for ph in r["phases"])


def _device_latency(out_json):
    lines = [json.loads(l) for l in out_json.read_text().splitlines() if '"latency"' in l]
    dev = [l for l in lines if l.get("method") == "device"]
    assert len(dev) == 1
    return dev[0]


def test_device_latency_self(exe, tmp_path):
    """One process: leader and follower are two waves of one workgroup."""
    js = tmp_path / "r.json"
    out = subprocess.run([exe, "--transport", "ipc", "--mode", "self", "--size", "4K", "-n", "2", "--compat-only",
                          "--device-latency", "--latency-size", "4K", "--latency-iters", "500", "--json", str(js)],
                         capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr[-3000:]
    lat = _device_latency(js)
    p = lat["pairs"][0]
    assert lat["bytes"] == 4096 and p["a"] == p["b"] == 0
    assert 0 < p["one_way_us"]["p50"] < 50, p


@pytest.mark.parametrize("nranks", [2, 4])
def test_device_latency_ranks_on_one_gpu(exe, tmp_path, nranks):
    """Several processes on one GPU bounce messages through each other's
    hipIpc-mapped signal pages; every pair of every round reports a time."""
    js = tmp_path / "r.json"
    out = subprocess.run([MPIRUN, "-n", str(nranks), exe, "--transport", "ipc", "--device", "0", "--mode", "ring",
                          "--size", "4K", "-n", "2", "--no-compat", "--device-latency", "--latency-iters", "300",
                          "--json", str(js)], capture_output=True, text=True, timeout=240)
    assert out.returncode == 0, out.stderr[-3000:]
    assert "device-initiated ping-pong" in out.stdout
    lat = _device_latency(js)
    pairs = {(p["a"], p["b"]) for p in lat["pairs"]}
    assert pairs == {(a, b) for a in range(nranks) for b in range(a + 1, nranks)}
    assert all(0 < p["one_way_us"]["p50"] < 100 for p in lat["pairs"]), lat


@pytest.mark.parametrize("engine", ["kernel", "push"])
def test_four_ranks_allpairs_large(exe, engine):
    out = subprocess.run([MPIRUN, "-n", "4", exe, "--transport", "ipc", "--ipc-engine", engine, "--device", "0",
                          "--mode", "allpairs,ring,tournament", "--size", "256M", "-n", "4", "--verify", "--no-compat",
                          "--timeout", "60"],
                         capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-3000:]
    assert "verification: OK" in out.stdout


def test_relay_engine_every_mode(exe, tmp_path):
    """Multi-path relay engine with 4 ranks on one GPU: in pair mode the two
    idle ranks carry two-hop stripes of every message above 1 MiB (their copy
    kernel loads from the sender's mapped buffer and stores into the
    receiver's mapped slot); tournament / ring find no idle links on 4 ranks
    for bi but do for uni; all-pairs stays direct.  Every receive verified."""
    js = tmp_path / "r.json"
    env = dict(os.environ, P2P_RELAY_STATS="1")
    out = subprocess.run([MPIRUN, "-n", "4", exe, "--transport", "ipc", "--ipc-engine", "relay", "--device", "0",
                          "--mode", "all", "--sizes", "64K,2M,1822205,64M", "-n", "4", "--verify", "--no-compat",
                          "--json", str(js), "--timeout", "60"], capture_output=True, text=True, timeout=300, env=env)
    assert out.returncode == 0, out.stderr[-3000:]
    assert "verification: OK" in out.stdout
    runs = [json.loads(l) for l in js.read_text().splitlines() if '"run"' in l]
    assert runs and all(ph["mismatches"] == 0 for r in runs for ph in r["phases"])
    relayed = [int(l.split("relayed ")[1].split()[0]) for l in out.stderr.splitlines() if "relayed" in l]
    assert len(relayed) == 4 and all(b > 0 for b in relayed), out.stderr[-2000:]


def test_relay_pair_cell_with_six_relays(exe):
    """8 ranks on one GPU, one pair cell (0 -> 1) of 32 MiB: the message goes
    out in 7 stripes (direct + 6 relays), verified; wallclock timing too."""
    env = dict(os.environ, P2P_RELAY_STATS="1", P2P_IPC_POOL="1G")
    for timing in ("events", "wallclock"):
        out = subprocess.run([MPIRUN, "-n", "8", exe, "--transport", "ipc", "--ipc-engine", "relay", "--device", "0",
                              "--mode", "pair", "--dir", "bi", "--cells", "0:1", "--size", "32M", "-n", "3", "--verify",
                              "--no-compat", "--timing", timing, "--timeout", "60"],
                             capture_output=True, text=True, timeout=300, env=env)
        assert out.returncode == 0, out.stderr[-3000:]
        assert "verification: OK" in out.stdout
        relayed = {int(l.split("rank ")[1].split()[0]): int(l.split("relayed ")[1].split()[0])
                   for l in out.stderr.splitlines() if " relayed " in l}
        assert sorted(relayed) == list(range(8)), out.stderr[-2000:]
        assert relayed[0] == 0 and relayed[1] == 0 and all(relayed[k] > 0 for k in range(2, 8)), relayed


def test_export_refusal_is_retried(exe):
    """hipIpcGetMemHandle occasionally refuses a fresh block on this stack;
    the transport reallocates and says so.  Injected here: every rank's
    first two exports are refused."""
    env = dict(os.environ, P2P_INJECT_EXPORT_REFUSALS="2")
    out = subprocess.run([MPIRUN, "-n", "2", exe, "--transport", "ipc", "--device", "0", "--mode", "tournament",
                          "--size", "1M", "-n", "4", "--verify", "--no-compat"], capture_output=True, text=True,
                         timeout=300, env=env)
    assert out.returncode == 0, out.stderr[-3000:]
    assert "verification: OK" in out.stdout
    assert out.stderr.count("refused 2 fresh") == 2, out.stderr


def test_corruption_detected_on_gpu(exe):
    env = dict(os.environ, P2P_INJECT_FAULT="corrupt@1:1")
    out = subprocess.run([MPIRUN, "-n", "2", exe, "--transport", "ipc", "--device", "0", "--size", "1M", "-n", "3",
                          "--verify", "--compat-only"], capture_output=True, text=True, timeout=300, env=env)
    assert out.returncode == 2
    assert "VERIFICATION FAILED" in out.stderr


@pytest.mark.parametrize("engine", ["kernel", "push"])
def test_skipped_transfers_detected_on_gpu(exe, engine):
    """P2P_INJECT_FAULT=skip@1: rank 1 moves no payload in the timed
    iterations (pull: its copies are not issued; push: its writes into rank
    0's slots are not issued, the flags still flow, so nothing hangs).  The
    warmup delivered everything, so only the poisoning before timing catches
    it: exit 2.  skip-some@1 drops only every other timed iteration; every
    iteration has a receive generation of its own, so that is caught too.
    The same run without the fault passes."""
    base = [MPIRUN, "-n", "2", exe, "--transport", "ipc", "--ipc-engine", engine, "--device", "0", "--mode",
            "pair,tournament", "--size", "1M", "-n", "4", "-w", "2", "--verify", "--no-compat", "--timeout", "60"]
    for fault in ("skip@1", "skip-some@1"):
        out = subprocess.run(base, capture_output=True, text=True, timeout=300,
                             env=dict(os.environ, P2P_INJECT_FAULT=fault))
        assert out.returncode == 2, (fault, out.stderr[-3000:])
        assert "VERIFICATION FAILED" in out.stderr
    ok = subprocess.run(base, capture_output=True, text=True, timeout=300)
    assert ok.returncode == 0, ok.stderr[-3000:]
    assert "8 of 8 timed deliveries checked" in ok.stdout, ok.stdout[-2000:]


def test_ring_token_chain_on_one_gpu(exe, tmp_path):
    """--mode ring with --latency and --device-latency, 4 processes on one GPU:
    the dependent token chain 0 -> 1 -> 2 -> 3 -> 0, host-posted through the
    push engine's rendezvous and as the one-wave device kernel."""
    js = tmp_path / "r.json"
    out = subprocess.run([MPIRUN, "-n", "4", exe, "--transport", "ipc", "--ipc-engine", "push", "--device", "0",
                          "--mode", "ring", "--dir", "uni", "--size", "64K", "-n", "2", "--no-compat", "--latency",
                          "--device-latency", "--latency-iters", "200", "--json", str(js), "--timeout", "60"],
                         capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-3000:]
    ring = {r["method"]: r for r in (json.loads(l) for l in js.read_text().splitlines()) if r["type"] == "ring_latency"}
    assert set(ring) == {"host", "device"}, ring
    for r in ring.values():
        assert r["nranks"] == 4 and r["laps"] == 50
        assert 0 < r["hop_us"]["p50"] and abs(r["lap_us"]["p50"] / r["hop_us"]["p50"] - 4) < 0.5, r
    assert ring["device"]["hop_us"]["p50"] < ring["host"]["hop_us"]["p50"]


def test_bench_two_ranks_ipc_push():
    """bench.py with the push engine as the headline transport (rendezvous +
    remote writes), graphs off by construction; then the xGMI pair sweep in
    the time left (--xgmi-sweep 1: ranks sharing the GPU, so its IPC rows run
    emulated, each an mpirun job of build/p2p_matrix, verified)."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(free_port()), "bench.py", "--gpus", "2", "--steps", "6", "--warmup", "3",
           "--transport", "ipc:push", "--device", "0", "--latency-iters", "50", "--sweep-max", "64M", "--ipc-extra", "0",
           "--xgmi-sweep", "1", "--xgmi-sweep-sizes", "4M"]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=600, cwd=ROOT)
    progress = "\n".join(l for l in out.stderr.splitlines() if "bench:" in l or "fatal" in l)
    assert out.returncode == 0, progress
    r = json.loads([l for l in out.stdout.splitlines() if l.startswith("{")][0])
    assert r["n_gpus"] == 2 and r["verify_mismatches"] == 0 and r["matrix_cells"] == "2/2" and r["value"] > 0
    assert r["p50_latency_us"] > 0
    sw = r["xgmi_pair_sweep"]
    assert sw["emulated"] == "ipc" and sw["rc"] == 0, sw
    assert sorted(sw["rows"]) == ["ipc-kernel", "ipc-push", "ipc-sdma"], sw
    assert all(row["rc"] == 0 and row["bi/4194304"]["cell_gbs"] > 0 for row in sw["rows"].values()), sw


def test_bench_two_ranks_ipc():
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(free_port()), "bench.py", "--gpus", "2", "--steps", "6", "--warmup", "3",
           "--transport", "ipc", "--device", "0", "--latency-iters", "50"]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=600, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1
    r = json.loads(lines[0])
    assert r["n_gpus"] == 2 and r["verify_mismatches"] == 0 and r["matrix_cells"] == "2/2"
    assert 0 < r["ipc_transport"]["device_pingpong_p50_us"] < 100, r["ipc_transport"]
    push = r["ipc_transport"]["push"]
    assert push["verify_mismatches"] == 0 and push["value_gbs"] > 0, push
    sweep = r["extras"]["pair_sweep_0_1"]
    assert len(sweep) == 11 and sweep[-1]["bytes"] == 4 << 30 and all(p["gbs"] > 0 for p in sweep)


@pytest.mark.emulated
@pytest.mark.parametrize("nranks", [4, 8])
def test_bench_emulated_node(nranks):
    """bench.py at the driver's GPU counts with every rank on the one GPU (IPC
    transport): tournament rounds, all-pairs with N-1 slots, ring, the pair
    sweep, the reference-method matrix and the pull / push comparisons all
    run through the N-rank code paths the 8-GPU scaling run uses."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(nranks),
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), "bench.py", "--gpus", str(nranks),
           "--steps", "14", "--warmup", "7", "--transport", "ipc", "--device", "0", "--sweep-max", "64M",
           "--latency-iters", "100", "--deadline", "560",
           # N ranks share one GPU's memory: 32 messages per step keep every
           # timed step in its own receive slots (128 would cap the generations).
           "--msgs", "32",
           # Child processes for the comparisons would double the processes
           # on the one GPU (8 ranks + 8 children + pytest > the box's 16):
           # isolate them only with 4 ranks.
           "--isolate", "1" if nranks == 4 else "0"]
    out = run_logged(cmd, 600, "bench_emulated_node_%d" % nranks, cwd=ROOT, env=dict(os.environ, P2P_IPC_POOL="1G"))
    progress = "\n".join(l for l in out.stderr.splitlines() if "bench:" in l or "fatal" in l)
    assert out.returncode == 0, progress
    r = json.loads([l for l in out.stdout.splitlines() if l.startswith("{")][0])
    assert r["n_gpus"] == nranks and r["verify_mismatches"] == 0
    assert r["value_kind"] == "emulated: %d ranks on 1 GPU(s), per direction (not xGMI)" % nranks, r["value_kind"]
    assert r["matrix_cells"] == "%d/%d" % (nranks * (nranks - 1), nranks * (nranks - 1))
    m, lat = r["matrix_gbs"], r["latency_p50_us_matrix"]
    assert len(m) == nranks and all(m[a][b] > 0 for a in range(nranks) for b in range(nranks) if a != b)
    assert all(lat[a][b] > 0 for a in range(nranks) for b in range(nranks) if a != b)
    # BASELINE config 3 by both methods on the reference's serial schedule, uni and bi
    for key in ("reference_semantics", "pair_serial_events"):
        assert r[key]["uni"]["gbs_mean"] > 0 and r[key]["bi"]["gbs_mean"] > 0, r[key]
    assert r["pair_serial_events"]["bi"]["mismatches"] == 0 and r["concurrency_ratio"] > 0
    assert r["method_ratio"]["uni"] > 0 and r["method_ratio"]["bi"] > 0
    assert r["extras"]["allpairs_1g"]["aggregate_gbs"] > 0 and r["extras"]["ring_256m"]["aggregate_gbs"] > 0
    assert len(r["extras"]["pair_sweep_0_1"]) == 8  # 4 KiB .. 64 MiB in x4 steps
    ipc = r["ipc_transport"]
    assert ipc["verify_mismatches"] == 0 and ipc["push"]["verify_mismatches"] == 0, ipc
    assert ipc["sdma"]["verify_mismatches"] == 0 and ipc["sdma"]["value_gbs"] > 0, ipc
    assert ipc["device_pingpong_p50_us"] > 0
    dm = ipc["device_latency_p50_us_matrix"]
    assert all(dm[a][b] > 0 and dm[a][b] == dm[b][a] for a in range(nranks) for b in range(nranks) if a != b), dm
    relay = ipc["relay"]
    assert relay["verify_mismatches"] == 0 and relay["value_gbs"] > 0, relay
    assert [p["mismatches"] for p in relay["pair_0_1"]] == [0, 0], relay
    # Every timed delivery verified; value is the mean cell (per flow and
    # direction) and agrees with the matrix of per-step GPU times.
    assert r["verify_coverage"] == 1.0 and ipc["verify_coverage"] == 1.0
    assert abs(r["aggregate_gbs"] - r["flows_per_step"] * r["value"]) < 0.01 * r["aggregate_gbs"]
    assert 0.5 < r["value"] / r["matrix_gbs_mean"] < 1.5, (r["value"], r["matrix_gbs_mean"])
    assert r["extras"]["ring_hop"]["hop_us_p50"] > 0 and ipc["device_ring_hop_p50_us"] > 0
    links = r["provenance"]["rank_links"]
    assert all(links[a][b] == "same-gpu" for a in range(nranks) for b in range(nranks))


@pytest.mark.parametrize("engine", ["kernel", "sdma", "push", "relay"])
def test_fuzz_every_engine(engine):
    """Random groups of verified messages (1 B .. 8 MiB, self messages and
    repeated pairs included) through every IPC engine, 4 processes on one GPU."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "4", "--master-addr",
           "127.0.0.1", "--master-port", str(free_port()), "tests/scripts/fuzz_session.py", "ipc:" + engine, "15"]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=600, cwd=ROOT,
                         env=dict(os.environ, P2P_FUZZ_DEVICE="0", P2P_IPC_POOL="1G"))
    assert out.returncode == 0, out.stderr[-3000:]
    assert "FUZZ ipc:%s mismatches 0" % engine in out.stdout



@pytest.mark.parametrize("engine", ["kernel", "relay"])
def test_cli_fuzz_four_ranks(exe, engine):
    """p2p_matrix --fuzz with 4 processes on the one GPU through the IPC
    transport: random groups (random pairs incl. self, 1 B .. 16 MiB), relay
    stripes through the third and fourth rank."""
    out = subprocess.run([MPIRUN, "-n", "4", exe, "--transport", "ipc", "--ipc-engine", engine, "--device", "0",
                          "--mode", "pair", "--size", "16M", "-n", "2", "--fuzz", "30", "--no-compat",
                          "--timeout", "60"], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-3000:]
    assert "all verified" in out.stdout


def test_xgmi_pair_sweep_emulated():
    """scripts/xgmi_pair_sweep.py end to end on one GPU: two ranks share GPU 0
    through the IPC engines (RCCL rows need distinct GPUs); every row verified
    and a winner per (direction, size) written."""
    import tempfile
    out_dir = tempfile.mkdtemp(prefix="xgmi_sweep_")
    out = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "xgmi_pair_sweep.py"), "--np", "2",
                          "--emulate", "ipc", "--sizes", "4M,32M", "--out", out_dir, "--budget", "150",
                          "--row-timeout", "60"], capture_output=True, text=True, timeout=200)
    assert out.returncode == 0, out.stderr[-3000:] + out.stdout[-3000:]
    s = json.loads(open(os.path.join(out_dir, "summary.json")).read())
    assert s["failed_row"] is None and s["rows_run"] == 3 and not s["rows_skipped"], s
    assert set(s["best"]) == {"uni/4194304", "uni/33554432", "bi/4194304", "bi/33554432"}
    assert all(b["cell_gbs"] > 10 for b in s["best"].values()), s["best"]


def test_push_arena_between_2_and_4_gib():
    """A push receive arena of 2.5 GiB (80 slots of 32 MiB): HIP 7.0's
    hipIpcOpenMemHandle never returns for a block whose size mod 4 GiB is
    2 GiB or more; the transport sizes its exported blocks around that
    (scripts/ipc_open_probe.hip)."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(free_port()), "tests/scripts/step_probe.py", "ipc:push", "tournament",
           "32M", "8", "10", "12"]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=120, cwd=ROOT,
                         env=dict(os.environ, P2P_FUZZ_DEVICE="0", P2P_FUZZ_TIMEOUT="30"))
    assert out.returncode == 0, out.stderr[-3000:]
    # 10 receive generations x 16 messages: every slot of the arena written and verified.
    assert out.stderr.count("driver (depth 10, 2684354560 receive bytes)") == 2, out.stderr[-3000:]
    assert out.stderr.count("'mismatches': 0, 'verified_msgs': 160, 'timed_msgs': 192, 'slots': 160") == 2, \
        out.stderr[-3000:]

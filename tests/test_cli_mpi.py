"""Tier T1: the p2p_matrix application under `mpirun -n N` on the CPU
(host transport), exercising bootstrap, placement, schedules, reporting and
failure handling end to end without a GPU."""
import json
import os
import re
import subprocess

import pytest

from test_nccl_p2p_amd.utils.report import parse_compat

pytestmark = pytest.mark.mpi


def run(mpirun, exe, n, args, env=None, timeout=120):
    e = dict(os.environ)
    e.update(env or {})
    cmd = [mpirun, "-n", str(n), exe] + args
    return subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, env=e)


def test_compat_output_format(mpirun, host_build):
    exe = os.path.join(host_build, "p2p_matrix_host")
    out = run(mpirun, exe, 3, ["--transport", "host", "--size", "64K", "-n", "4", "--compat-only"])
    assert out.returncode == 0, out.stderr
    txt = out.stdout
    assert txt.startswith("Evaluating the Uni-Directional NCCL P2P Bandwidth (Gbps)\n   D\\D     0      1      2 \n")
    assert "\n\nEvaluating the Bi-Directional NCCL P2P Bandwidth (Gbps)\n" in txt
    m = parse_compat(txt)
    for key in ("uni", "bi"):
        mat = m[key]
        assert len(mat) == 3
        for i in range(3):
            assert mat[i][i] == 0.0
            assert all(mat[i][j] > 0 for j in range(3) if j != i)
    # every row line: label "%6d " then 3 cells "%6.02f " (values < 1000 on CPU)
    rows = [l for l in txt.splitlines() if re.match(r"^ {5}\d ", l)]
    assert all(len(l) == 7 * 4 for l in rows)


def test_all_modes_verify_json(mpirun, host_build, tmp_path):
    exe = os.path.join(host_build, "p2p_matrix_host")
    js = tmp_path / "r.json"
    csv = tmp_path / "r.csv"
    out = run(mpirun, exe, 4, ["--transport", "host", "--mode", "all", "--sizes", "4K:16K", "-n", "3",
                               "--verify", "--latency", "--latency-iters", "20", "--json", str(js), "--csv", str(csv)])
    assert out.returncode == 0, out.stderr
    recs = [json.loads(l) for l in js.read_text().splitlines()]
    runs = [r for r in recs if r["type"] == "run"]
    # pair/tournament/ring x {uni,bi} + allpairs once, x 3 sizes
    assert len(runs) == (3 * 2 + 1) * 3
    for r in runs:
        for ph in r["phases"]:
            assert ph["mismatches"] == 0
    lat = [r for r in recs if r["type"] == "latency"][0]
    assert len(lat["pairs"]) == 6
    assert "verification: OK" in out.stdout
    assert csv.read_text().startswith("mode,dir,bytes")


def test_dry_run_and_help(host_build):
    exe = os.path.join(host_build, "p2p_matrix_host")
    out = subprocess.run([exe, "--dry-run", "--mode", "tournament", "--dir", "bi"], capture_output=True, text=True,
                         timeout=60)
    assert out.returncode == 0 and "schedule tournament-bi, 1 ranks" in out.stdout
    h = subprocess.run([exe, "--help"], capture_output=True, text=True, timeout=60)
    assert h.returncode == 0 and "mpirun -n N ./p2p_matrix" in h.stdout
    bad = subprocess.run([exe, "--bogus"], capture_output=True, text=True, timeout=60)
    assert bad.returncode == 1


def test_block_placement_enforced(mpirun, host_build):
    exe = os.path.join(host_build, "p2p_matrix_host")
    base = ["--transport", "host", "--size", "4K", "-n", "2", "--compat-only"]
    ok = subprocess.run([mpirun, "-n", "2", "-env", "P2P_HOSTNAME", "hostA", exe] + base +
                        [":", "-n", "2", "-env", "P2P_HOSTNAME", "hostB", exe] + base,
                        capture_output=True, text=True, timeout=120)
    assert ok.returncode == 0, ok.stderr
    bad = subprocess.run([mpirun, "-n", "1", "-env", "P2P_HOSTNAME", "hostA", exe] + base +
                         [":", "-n", "1", "-env", "P2P_HOSTNAME", "hostB", exe] + base +
                         [":", "-n", "1", "-env", "P2P_HOSTNAME", "hostA", exe] + base +
                         [":", "-n", "1", "-env", "P2P_HOSTNAME", "hostB", exe] + base,
                         capture_output=True, text=True, timeout=120)
    assert bad.returncode != 0
    assert "block placement" in bad.stderr


def test_corruption_detected(mpirun, host_build):
    exe = os.path.join(host_build, "p2p_matrix_host")
    out = run(mpirun, exe, 2, ["--transport", "host", "--size", "64K", "-n", "3", "--verify", "--compat-only"],
              env={"P2P_INJECT_FAULT": "corrupt@1:1"})
    assert out.returncode == 2
    assert "VERIFICATION FAILED" in out.stderr


def test_skipped_transfers_detected(mpirun, host_build):
    """P2P_INJECT_FAULT=skip@1: rank 1's receives silently move no payload in
    the timed iterations (the protocol still runs).  The warmup delivered the
    payload already, so the slots are poisoned again before timing: exit 2."""
    exe = os.path.join(host_build, "p2p_matrix_host")
    for transport in ("host", "shm"):
        out = run(mpirun, exe, 3, ["--transport", transport, "--mode", "pair,tournament", "--size", "64K", "-n", "3",
                                   "-w", "2", "--verify", "--no-compat"], env={"P2P_INJECT_FAULT": "skip@1"})
        assert out.returncode == 2, (transport, out.stderr[-2000:])
        assert "VERIFICATION FAILED" in out.stderr and "moves no payload" in out.stderr
    ok = run(mpirun, exe, 3, ["--transport", "shm", "--mode", "pair", "--size", "64K", "-n", "3", "-w", "2",
                              "--verify", "--no-compat"])
    assert ok.returncode == 0, ok.stderr[-2000:]


def test_every_timed_iteration_is_verified(mpirun, host_build, tmp_path):
    """P2P_INJECT_FAULT=skip-some@1 drops every other timed delivery on rank 1.
    A check of the last delivery per slot would pass (the odd iterations
    delivered); with one receive generation per timed iteration every
    delivery is checked: exit 2, and the JSON reports full coverage.  Under a
    budget that holds only 2 generations the coverage says so (2 of 6)."""
    exe = os.path.join(host_build, "p2p_matrix_host")
    for transport in ("host", "shm"):
        js = tmp_path / ("%s.json" % transport)
        out = run(mpirun, exe, 3, ["--transport", transport, "--mode", "pair,tournament", "--size", "64K", "-n", "6",
                                   "-w", "2", "--verify", "--no-compat", "--json", str(js)],
                  env={"P2P_INJECT_FAULT": "skip-some@1"})
        assert out.returncode == 2, (transport, out.stderr[-2000:])
        assert "every other timed iteration" in out.stderr and "VERIFICATION FAILED" in out.stderr
        runs = [json.loads(l) for l in js.read_text().splitlines() if '"type":"run"' in l]
        assert runs and all(r["verify_coverage"] == 1 and r["timed_msgs"] == r["verified_msgs"] > 0 for r in runs)
        bad = [ph for r in runs for ph in r["phases"] if ph["mismatches"]]
        # rank 1 receives in pair cells (0,1), (2,1) and in tournament phases
        assert bad and all(ph["generations"] == 6 for ph in bad)
    js = tmp_path / "budget.json"
    ok = run(mpirun, exe, 2, ["--transport", "host", "--mode", "pair", "--size", "64K", "-n", "6", "-w", "2",
                              "--verify", "--no-compat", "--json", str(js)], env={"P2P_VERIFY_BUDGET": "300K"})
    assert ok.returncode == 0, ok.stderr[-2000:]
    assert "4 of 12 timed deliveries checked" in ok.stdout
    uni = [json.loads(l) for l in js.read_text().splitlines() if '"type":"run"' in l][0]
    assert abs(uni["verify_coverage"] - 1 / 3) < 1e-6 and uni["verified_msgs"] == 4


def test_default_run_verifies(mpirun, host_build, tmp_path):
    """`mpirun -n N ./p2p_matrix` with no flags verifies
    every timed delivery (outside the timed loop): an injected skip-some
    fault exits 2 without --verify, the JSON carries verify_coverage, the
    compat-only output is the reference's bytes alone, and --no-verify opts
    out (nothing checked, exit 0 despite the fault)."""
    exe = os.path.join(host_build, "p2p_matrix_host")
    for transport in ("host", "shm"):
        js = tmp_path / ("%s.json" % transport)
        out = run(mpirun, exe, 2, ["--transport", transport, "--size", "64K", "-n", "6", "-w", "2", "--json", str(js)],
                  env={"P2P_INJECT_FAULT": "skip-some@1"})
        assert out.returncode == 2, (transport, out.stderr[-2000:])
        assert "VERIFICATION FAILED" in out.stderr and "verification: FAILED" in out.stdout
        runs = [json.loads(l) for l in js.read_text().splitlines() if '"type":"run"' in l]
        assert runs and all(r["verify_coverage"] == 1 for r in runs)
    ok = run(mpirun, exe, 2, ["--transport", "shm", "--size", "64K", "-n", "4", "--compat-only"])
    assert ok.returncode == 0 and "verification" not in ok.stdout
    assert ok.stdout.startswith("Evaluating the Uni-Directional NCCL P2P Bandwidth (Gbps)\n")
    off = run(mpirun, exe, 2, ["--transport", "shm", "--size", "64K", "-n", "6", "-w", "2", "--no-verify"],
              env={"P2P_INJECT_FAULT": "skip-some@1"})
    assert off.returncode == 0 and "verification:" not in off.stdout, off.stderr[-2000:]


def test_json_provenance_and_ring_token(mpirun, host_build, tmp_path):
    """--json starts with the provenance record (knobs, runtime, every rank's
    device and the links between them); --mode ring --latency adds the
    dependent ring token chain."""
    exe = os.path.join(host_build, "p2p_matrix_host")
    js = tmp_path / "r.json"
    out = run(mpirun, exe, 3, ["--transport", "shm", "--mode", "ring", "--size", "16K", "-n", "2", "--latency",
                               "--latency-iters", "60", "--json", str(js), "--no-compat"],
              env={"NCCL_PROTO": "Simple"})
    assert out.returncode == 0, out.stderr[-2000:]
    recs = [json.loads(l) for l in js.read_text().splitlines()]
    prov = recs[0]
    assert prov["type"] == "provenance" and prov["env"]["NCCL_PROTO"] == "Simple"
    assert "GPU_MAX_HW_QUEUES" in prov["env"] and "rccl" in prov["runtime"]
    assert [d["rank"] for d in prov["rank_devices"]] == [0, 1, 2] and len(prov["rank_links"]) == 3
    ring = [r for r in recs if r["type"] == "ring_latency"]
    assert len(ring) == 1 and ring[0]["nranks"] == 3 and ring[0]["laps"] == 20
    assert 0 < ring[0]["hop_us"]["p50"] <= ring[0]["lap_us"]["p50"]
    assert "ring token latency: 3 rank(s)" in out.stdout


def test_dead_rank_does_not_hang(mpirun, host_build):
    exe = os.path.join(host_build, "p2p_matrix_host")
    out = run(mpirun, exe, 3, ["--transport", "host", "--size", "64K", "-n", "3"],
              env={"P2P_INJECT_FAULT": "exit@2:2"}, timeout=120)
    assert out.returncode != 0
    assert "injected fault" in out.stderr


def test_hung_rank_times_out_tcp(host_build):
    """TCP bootstrap (torchrun-style env): a hung rank trips the others' watchdogs."""
    from conftest import free_port

    exe = os.path.join(host_build, "p2p_matrix_host")
    port = free_port()
    procs = []
    for r in range(2):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE="2", MASTER_ADDR="127.0.0.1", P2P_BOOTSTRAP_PORT=str(port),
                   P2P_BOOTSTRAP_TIMEOUT="5", P2P_INJECT_FAULT="hang@1:1")
        procs.append(subprocess.Popen([exe, "--transport", "host", "--size", "4K", "-n", "2", "--timeout", "5"],
                                      env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
    try:
        _, err0 = procs[0].communicate(timeout=90)
        assert procs[0].returncode != 0
        assert "timeout" in err0 or "closed" in err0
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()


def test_resume_and_trace(mpirun, host_build, tmp_path):
    exe = os.path.join(host_build, "p2p_matrix_host")
    js, tr = tmp_path / "r.json", tmp_path / "t.json"
    base = ["--transport", "host", "--sizes", "4K,64K", "-n", "2", "--no-compat", "--json", str(js)]
    first = run(mpirun, exe, 2, base + ["--mode", "pair,ring", "--trace", str(tr)])
    assert first.returncode == 0, first.stderr

    def runs():
        return [json.loads(l) for l in js.read_text().splitlines() if json.loads(l)["type"] == "run"]

    assert len(runs()) == 8  # (pair, ring) x (uni, bi) x 2 sizes
    trace = json.loads(tr.read_text())
    xs = [e for e in trace["traceEvents"] if e["ph"] == "X"]
    assert {e["tid"] for e in xs} == {0, 1} and all(e["dur"] >= 0 for e in xs)
    again = run(mpirun, exe, 2, base + ["--mode", "pair,ring,allpairs", "--resume", "-v"])
    assert again.returncode == 0, again.stderr
    assert len(runs()) == 10  # only the 2 allpairs runs were added
    # Every invocation records its provenance first (the resume appended one).
    assert sum(1 for l in js.read_text().splitlines() if json.loads(l)["type"] == "provenance") == 2
    assert again.stderr.count("resume: skipping") == 8


def test_roctx_library_for_rocprofv3(host_build):
    """P2P_ROCTX=1 loads rocprofiler-sdk's roctx (the one rocprofv3
    --marker-trace records; profiles/r2_tracing/), not the legacy one."""
    exe = os.path.join(host_build, "p2p_matrix_host")
    out = subprocess.run([exe, "--transport", "host", "--mode", "self", "--size", "64K", "-n", "2", "--no-compat"],
                         capture_output=True, text=True, timeout=60, env=dict(os.environ, P2P_ROCTX="1"))
    assert out.returncode == 0, out.stderr
    assert "roctx ranges via librocprofiler-sdk-roctx" in out.stderr, out.stderr


def test_cells_filter(mpirun, host_build):
    exe = os.path.join(host_build, "p2p_matrix_host")
    out = run(mpirun, exe, 3, ["--transport", "host", "--size", "16K", "-n", "2", "--cells", "0-1,2:0",
                               "--compat-only"])
    assert out.returncode == 0, out.stderr
    m = parse_compat(out.stdout)
    for key in ("uni", "bi"):
        nz = {(i, j) for i in range(3) for j in range(3) if m[key][i][j] > 0}
        assert nz == {(0, 1), (2, 0)}


def test_device_latency_needs_one_sided_transport(mpirun, host_build):
    exe = os.path.join(host_build, "p2p_matrix_host")
    out = run(mpirun, exe, 2, ["--transport", "host", "--size", "16K", "-n", "2", "--compat-only", "--device-latency"])
    assert out.returncode != 0
    assert "one-sided transport" in out.stderr + out.stdout


def test_min_gbs_link_check(mpirun, host_build):
    """--min-gbs names every flow below the threshold and exits 3; a threshold
    every link meets passes."""
    exe = os.path.join(host_build, "p2p_matrix_host")
    bad = run(mpirun, exe, 3, ["--transport", "host", "--mode", "tournament", "--dir", "uni", "--size", "64K",
                               "-n", "3", "--no-compat", "--min-gbs", "1e6"])
    assert bad.returncode == 3, bad.stderr
    assert bad.stderr.count("SLOW LINK") == 6 and "LINK CHECK FAILED: 6 flow(s)" in bad.stderr
    ok = run(mpirun, exe, 3, ["--transport", "host", "--mode", "tournament", "--dir", "uni", "--size", "64K",
                              "-n", "3", "--no-compat", "--min-gbs", "1e-6"])
    assert ok.returncode == 0, ok.stderr


def test_shm_transport_all_modes(mpirun, host_build, tmp_path):
    """The shared-memory CPU transport under mpirun: every mode verified, a
    message larger than the 1 MiB ring, and the 4 KiB ping-pong (BASELINE
    config 1's shape) well under the TCP transport's latency."""
    exe = os.path.join(host_build, "p2p_matrix_host")
    js = tmp_path / "r.json"
    out = run(mpirun, exe, 3, ["--transport", "shm", "--mode", "all", "--sizes", "4K,3M", "-n", "3", "--verify",
                               "--latency", "--latency-size", "4K", "--latency-iters", "500", "--json", str(js)])
    assert out.returncode == 0, out.stderr
    assert "verification: OK" in out.stdout and "transport shm" in out.stdout
    recs = [json.loads(l) for l in js.read_text().splitlines()]
    assert all(ph["mismatches"] == 0 for r in recs if r["type"] == "run" for ph in r["phases"])
    lat = [r for r in recs if r["type"] == "latency"][0]
    assert all(0 < p["one_way_us"]["p50"] < 50 for p in lat["pairs"]), lat
    assert not [f for f in os.listdir("/dev/shm") if f.startswith("p2p_shm_")], "segment left in /dev/shm"


def test_fuzz_option(mpirun, host_build, tmp_path):
    """--fuzz N: random verified message groups after the matrices, over the
    TCP and shared-memory transports (csrc/runner.cpp fuzz_transport), with a
    `"type":"fuzz"` JSON line."""
    exe = os.path.join(host_build, "p2p_matrix_host")
    for transport, n in (("host", 2), ("shm", 3)):
        js = tmp_path / ("%s.json" % transport)
        out = run(mpirun, exe, n, ["--transport", transport, "--mode", "pair", "--size", "256K", "-n", "2",
                                   "--fuzz", "12", "--json", str(js)])
        assert out.returncode == 0, out.stderr[-3000:]
        assert "== fuzz: 12 groups of random messages (1 B .. 256K" in out.stdout and "all verified" in out.stdout
        rec = [json.loads(l) for l in js.read_text().splitlines() if '"fuzz"' in l]
        assert rec == [{"type": "fuzz", "rounds": 12, "max_bytes": 262144, "mismatches": 0}]


def test_repeat_runs_summarised(mpirun, host_build, tmp_path):
    """--repeat R (the binary's side of VERDICT r5 item 1): every (mode, dir,
    size) runs R times; the reference matrices print once (the first run, as
    it goes), the repeat summary gives every run's mean cell and their
    median / min / max, and --json keeps each run (with its index) and one
    "repeats" record per configuration."""
    exe = os.path.join(host_build, "p2p_matrix_host")
    js = tmp_path / "rep.json"
    out = run(mpirun, exe, 2, ["--transport", "host", "--size", "64K", "-n", "4", "--repeat", "3", "--json", str(js)])
    assert out.returncode == 0, out.stderr
    assert out.stdout.count("Evaluating the Uni-Directional NCCL P2P Bandwidth (Gbps)") == 1
    assert out.stdout.count("Evaluating the Bi-Directional NCCL P2P Bandwidth (Gbps)") == 1
    assert out.stdout.count("== [pair uni | 64K") == 1  # the extended tables of the first run only
    lines = out.stdout.split("== repeats:")[1].splitlines()
    rows = [l.split() for l in lines if l.strip().startswith("pair")]
    assert [(r[0], r[1], r[3]) for r in rows] == [("pair", "uni", "3"), ("pair", "bi", "3")], lines
    recs = [json.loads(l) for l in js.read_text().splitlines()]
    runs = [r for r in recs if r["type"] == "run"]
    assert sorted((r["dir"], r["repeat"]) for r in runs) == [(d, i) for d in ("bi", "uni") for i in range(3)]
    reps = {r["dir"]: r for r in recs if r["type"] == "repeats"}
    for d in ("uni", "bi"):
        x = reps[d]
        assert len(x["runs"]) == 3 and x["min"] <= x["median"] <= x["max"] and x["median"] == sorted(x["runs"])[1]
    bad = run(mpirun, exe, 1, ["--transport", "host", "--repeat", "0"])
    assert bad.returncode != 0 and "--repeat needs a whole number >= 1" in bad.stderr


@pytest.mark.parametrize("args,msg", [
    (["-n", "0"], "--iters must be >= 1"),
    (["-n", "5x"], "--iters must be >= 1"),
    (["--comms", "0"], "--comms needs a whole number >= 1"),
    (["-w", "-1"], "-w needs a whole number >= 0"),
    (["--warmup=two"], "--warmup needs a whole number >= 0"),
    (["--latency-iters", "0"], "--latency-iters needs a whole number >= 1"),
    (["--fuzz", "-2"], "--fuzz needs a whole number >= 0"),
    (["--timeout", "0"], "--timeout needs a number > 0"),
    (["--device", "-2"], "--device needs a whole number >= -1"),
    (["--min-gbs", "fast"], "--min-gbs needs a number >= 0"),
    (["--iters"], "option --iters needs a value"),
])
def test_cli_rejects_bad_numbers(host_build, args, msg):
    """Numeric options are read whole and range-checked: a typo or a negative
    count exits 1 at the command line with a message naming the option,
    instead of running with an atoi() zero (the reference takes no options)."""
    exe = os.path.join(host_build, "p2p_matrix_host")
    out = subprocess.run([exe, "--transport", "host", "--mode", "self", "--size", "4K"] + args,
                         capture_output=True, text=True, timeout=60)
    assert out.returncode == 1, out.stdout + out.stderr
    assert msg in out.stderr, out.stderr
    assert "verification" not in out.stdout


def test_cli_small_flags(host_build, tmp_path):
    """--version, -v / --verbose, --bootstrap local, --no-warm, --two-streams
    (ignored by the CPU transport) and --key=value spellings."""
    exe = os.path.join(host_build, "p2p_matrix_host")
    v = subprocess.run([exe, "--version"], capture_output=True, text=True, timeout=60)
    assert v.returncode == 0 and v.stdout.startswith("p2p_matrix (MI355X / gfx950, RCCL)")
    js = tmp_path / "r.json"
    out = subprocess.run([exe, "--transport=host", "--bootstrap=local", "--mode=self", "--size=8K", "--iters=3",
                          "--warmup=0", "--no-warm", "--two-streams", "-v", "--timeout=2.5", "--json", str(js)],
                         capture_output=True, text=True, timeout=60)
    assert out.returncode == 0, out.stderr
    assert "bootstrap local" in out.stdout and "verification: OK" in out.stdout
    run_rec = [json.loads(l) for l in js.read_text().splitlines() if '"type":"run"' in l]
    assert len(run_rec) == 1 and run_rec[0]["iters"] == 3 and run_rec[0]["warmup"] == 0


def test_resume_completes_missing_repeats(mpirun, host_build, tmp_path):
    """--resume with --repeat R: a configuration the file holds fewer than R
    runs of runs only the missing repeats (numbered on from the last), one
    with all R is skipped."""
    exe = os.path.join(host_build, "p2p_matrix_host")
    js = tmp_path / "r.json"
    base = ["--transport", "host", "--mode", "self", "--sizes", "4K,64K", "-n", "2", "--no-compat", "--json", str(js)]
    first = run(mpirun, exe, 1, base + ["--repeat", "2"])
    assert first.returncode == 0, first.stderr

    def runs():
        return [(r["bytes"], r["repeat"]) for r in map(json.loads, js.read_text().splitlines()) if r["type"] == "run"]

    assert sorted(runs()) == [(4096, 0), (4096, 1), (65536, 0), (65536, 1)]
    again = run(mpirun, exe, 1, base + ["--repeat", "3", "--resume", "-v"])
    assert again.returncode == 0, again.stderr
    assert sorted(runs()) == [(4096, i) for i in range(3)] + [(65536, i) for i in range(3)]
    done = run(mpirun, exe, 1, base + ["--repeat", "3", "--resume", "-v"])
    assert done.returncode == 0 and done.stderr.count("resume: skipping") == 2 and len(runs()) == 6

"""Tier T3: the RCCL transport on one MI355X (1-rank communicator: self
send/recv through ncclGroupStart/End), through every engine entry point."""
import json
import os
import subprocess
import sys

import pytest
import torch

from conftest import ROOT

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def session(native):
    assert torch.cuda.is_available()
    torch.cuda.set_device(0)
    s = native.Session(0, 1, device=0, transport="rccl", timeout_s=120)
    yield s
    del s


def test_device_desc(session):
    assert "gfx950" in session.device_desc
    assert session.transport == "rccl"


@pytest.mark.parametrize("mode", ["self", "ring", "allpairs", "tournament"])
def test_self_modes_verified(session, mode):
    r = json.loads(session.run(mode=mode, dir="bi", bytes=(4 << 20) + 12, iters=6, warmup=2, verify=True))
    (ph,) = r["phases"]
    assert ph["mismatches"] == 0
    (flow,) = ph["flows"]
    assert flow["src"] == flow["dst"] == 0 and flow["gbs"] > 1.0


def test_pair_mode_single_rank_is_idle_diagonal(session):
    r = json.loads(session.run(mode="pair", dir="uni", bytes=1 << 20, iters=2, warmup=0))
    assert r["phases"] == []  # diagonal only, like the reference's 1-rank run


@pytest.mark.parametrize("timing", ["events", "wallclock"])
def test_timings(session, timing):
    r = json.loads(session.run(mode="self", dir="uni", bytes=32 << 20, iters=16, warmup=2, timing=timing, verify=True))
    ph = r["phases"][0]
    assert ph["mismatches"] == 0 and ph["seconds_per_iter"] > 0
    assert ph["flows"][0]["iter_us"]["n"] == 16


def test_sweep_up_to_1g(session):
    """Verified self send/recv up to 1 GiB, posted as one op each (the op
    limit from RCCL's INFO log is 16 MiB x 64 channels): the transport's own
    chunking must make the verified-warmup fallback unnecessary."""
    for nbytes in [4096, 1 << 20, 64 << 20, 1 << 30]:
        r = json.loads(session.run(mode="self", dir="uni", bytes=nbytes, iters=4, warmup=1, verify=True))
        ph = r["phases"][0]
        assert ph["mismatches"] == 0 and r["verify_coverage"] == 1, ph
        assert not r["rechunked"] and ph["warmup_mismatches"] == 0 and ph["op_bytes"] == 0, ph


def test_latency(session):
    lat = json.loads(session.latency(8, 200, 20))
    (p,) = lat["pairs"]
    assert p["one_way_us"]["n"] == 200 and 0 < p["one_way_us"]["p50"] < 1000


def test_step_driver(native, session):
    d = native.StepDriver(session, "self", "bi", 8 << 20, 4, True)
    d.connect()
    d.run_steps(0, 5)
    d.sync()
    ms = d.step_ms()
    assert len(ms) == 5 and all(m > 0 for m in ms)
    assert d.verify_last() == 0
    assert d.job_bytes_per_step(0) == 4 * (8 << 20)


def test_step_driver_verifies_every_timed_step(native):
    """Every message of every timed step in its own slot: after poison() the
    timed steps refill all of them (coverage 1.0), one or four communicators."""
    for transport in ("rccl", "rccl:4"):
        s = native.Session(0, 1, device=0, transport=transport, timeout_s=120)
        d = native.StepDriver(s, "self", "bi", (4 << 20) + 64, 6, True, True, False, depth=5, salt=3)
        assert d.depth == 5 and d.recv_bytes >= 5 * 6 * ((4 << 20) + 64)
        d.connect()
        d.run_steps(0, 2)
        d.sync()
        d.poison()
        d.run_steps(2, 5)
        d.sync()
        v = d.verify_steps(2, 5)
        assert v["mismatches"] == 0 and v["timed_msgs"] == 30 and v["verified_msgs"] == 30, v
        d.poison()  # nothing ran since: every slot fails
        z = d.verify_steps(2, 5)
        assert z["mismatches"] == z["slots"] * (((4 << 20) + 64) // 4), z
        del d, s


def test_skip_fault_is_caught_rccl():
    """P2P_INJECT_FAULT=skip@0 on the RCCL transport: the timed receives land
    in a sink (the collective still completes); both the run engine (each of
    the 4 timed iterations in a receive generation of its own) and the step
    driver report every timed delivery as missing."""
    code = ("import json\n"
            "from test_nccl_p2p_amd import require_native\n"
            "nat = require_native()\n"
            "s = nat.Session(0, 1, device=0, transport='rccl', timeout_s=60)\n"
            "r = json.loads(s.run(mode='self', dir='uni', bytes=1 << 20, iters=4, warmup=2, verify=True))\n"
            "print('RUN', r['phases'][0]['mismatches'])\n"
            "d = nat.StepDriver(s, 'self', 'bi', 1 << 20, 2, True, True, False, depth=3)\n"
            "d.connect(); d.run_steps(0, 2); d.sync(); d.poison(); d.run_steps(2, 3); d.sync()\n"
            "print('STEPS', d.verify_steps(2, 3)['mismatches'])\n")
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120, cwd=ROOT,
                         env=dict(__import__("os").environ, P2P_INJECT_FAULT="skip@0"))
    assert out.returncode == 0, out.stderr[-3000:]
    words = (1 << 20) // 4
    assert "RUN %d" % (4 * words) in out.stdout and "STEPS %d" % (3 * 2 * words) in out.stdout, out.stdout


def test_skip_some_fault_is_caught_rccl(tmp_path):
    """P2P_INJECT_FAULT=skip-some@0 on the RCCL self path: every other timed
    delivery lands in the sink.  The CLI gives every timed iteration its own
    receive generation, so it exits 2 with full verify_coverage (a check of
    the last delivery per slot would have passed); the step driver reports
    exactly the dropped steps' words."""
    exe = os.path.join(ROOT, "build", "p2p_matrix")
    js = tmp_path / "r.json"
    base = [exe, "--mode", "self", "--size", "1M", "-n", "6", "-w", "2", "--verify", "--no-compat", "--timeout", "60",
            "--json", str(js)]
    out = subprocess.run(base, capture_output=True, text=True, timeout=120,
                         env=dict(os.environ, P2P_INJECT_FAULT="skip-some@0"))
    assert out.returncode == 2, out.stderr[-3000:]
    run = [json.loads(l) for l in js.read_text().splitlines() if '"type":"run"' in l][0]
    assert run["verify_coverage"] == 1 and run["timed_msgs"] == 6, run
    assert run["phases"][0]["mismatches"] == 3 * ((1 << 20) // 4), run["phases"][0]
    links = [json.loads(l) for l in js.read_text().splitlines() if '"type":"links"' in l][0]
    assert links["matrix_transport"] == [["self"]] and links["ranks"][0]["comms"][0]["p2p_channels"] > 0, links
    code = ("from test_nccl_p2p_amd import require_native\n"
            "nat = require_native()\n"
            "s = nat.Session(0, 1, device=0, transport='rccl', timeout_s=60)\n"
            "d = nat.StepDriver(s, 'self', 'bi', 1 << 20, 2, True, True, False, depth=4)\n"
            "d.connect(); d.run_steps(0, 2); d.sync(); d.poison(); d.run_steps(2, 4); d.sync()\n"
            "print('STEPS', d.verify_steps(2, 4)['mismatches'])\n")
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120, cwd=ROOT,
                         env=dict(os.environ, P2P_INJECT_FAULT="skip-some@0"))
    assert out.returncode == 0, out.stderr[-3000:]
    assert "STEPS %d" % (2 * 2 * ((1 << 20) // 4)) in out.stdout, out.stdout


def test_ring_latency_and_provenance(native, session):
    r = json.loads(session.ring_latency(8, 100, 10, False))
    assert r["nranks"] == 1 and r["laps"] == 100 and 0 < r["hop_us"]["p50"] < 1000
    # One runtime for every entry point: the RCCL / HIP this process runs are
    # the files torch loaded (Makefile RUNTIME=torch, build/rt).
    rt = json.loads(native.runtime_json())
    maps = open("/proc/self/maps").read()
    assert rt["rccl"]["library"] in maps and rt["hip"]["library"] in maps, rt
    assert rt["visible_devices"] >= 1
    p = json.loads(session.provenance(0))
    assert p["rank_devices"][0]["pci"] and p["rank_links"] == [["same-gpu"]] and "GPU_MAX_HW_QUEUES" in p["env"]


def test_message_larger_than_4gib(session):
    """size_t counts: the reference's `int msg_size` cannot express this."""
    r = json.loads(session.run(mode="self", dir="uni", bytes=(5 << 30) + 16, iters=2, warmup=1, verify=True))
    ph = r["phases"][0]
    assert ph["mismatches"] == 0 and ph["flows"][0]["gbs"] > 1.0
    # posted as 1 GiB ops by the transport itself, not by the warmup fallback
    assert ph["op_bytes"] == 1 << 30 and ph["warmup_mismatches"] == 0 and not r["rechunked"], ph


@pytest.mark.parametrize("comms", [2, 4, 8])
def test_several_communicators(native, comms):
    """K communicators per rank (messages of >= 1 MiB spread over them, each on
    its own stream, joined back per group): verified step driver, verified
    runs incl. a > 1 GiB message (chunks stay on their message's
    communicator), small-message latency on the first communicator."""
    s = native.Session(0, 1, device=0, transport="rccl:%d" % comms, timeout_s=120)
    assert ("x%d comms" % comms) in s.device_desc
    d = native.StepDriver(s, "self", "bi", 8 << 20, 8, True, True, False)
    d.connect()
    d.run_steps(0, 6)
    d.sync()
    assert len(d.step_ms()) == 6 and d.verify_last() == 0
    del d
    for nbytes in [4096, (4 << 20) + 12, (1 << 30) + 4096]:
        r = json.loads(s.run(mode="self", dir="bi", bytes=nbytes, iters=3, warmup=1, verify=True))
        assert r["phases"][0]["mismatches"] == 0
    lat = json.loads(s.latency(8, 100, 10))
    assert 0 < lat["pairs"][0]["one_way_us"]["p50"] < 1000
    del s


@pytest.mark.parametrize("mode", ["1", "2"])
def test_buffer_registration_knob(native, monkeypatch, mode):
    """P2P_RCCL_REGISTER=1 (ncclCommRegister of every buffer) and =2 (plus
    ncclMemAlloc): verified steps and runs, buffers deregistered and freed
    when the sets go away."""
    monkeypatch.setenv("P2P_RCCL_REGISTER", mode)
    s = native.Session(0, 1, device=0, transport="rccl:2", timeout_s=120)
    d = native.StepDriver(s, "self", "bi", 4 << 20, 4, True, True, False)
    d.connect()
    d.run_steps(0, 4)
    d.sync()
    assert d.verify_last() == 0
    del d
    r = json.loads(s.run(mode="self", dir="bi", bytes=(2 << 20) + 4, iters=3, warmup=1, verify=True))
    assert r["phases"][0]["mismatches"] == 0
    del s


def test_registered_buffers_after_an_abort():
    """A session whose communicators were aborted (the deadline watchdog's
    abort_if_idle) with buffers still registered (P2P_RCCL_REGISTER=1): the
    abort took the registrations with the communicators, so the teardown
    deregisters nothing on them and the process ends cleanly.  In a child:
    abort_if_idle closes the engine for the whole process."""
    code = ("from test_nccl_p2p_amd import require_native\n"
            "nat = require_native()\n"
            "s = nat.Session(0, 1, device=0, transport='rccl:2', timeout_s=60)\n"
            "d = nat.StepDriver(s, 'self', 'bi', 4 << 20, 4, True, True, False)\n"
            "d.connect(); d.run_steps(0, 2); d.sync()\n"
            "print('VERIFY', d.verify_last())\n"
            "print('ABORTED', nat.abort_if_idle(), nat.abort_done())\n"
            "del d, s\n"
            "print('TORN DOWN')\n")
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120, cwd=ROOT,
                         env=dict(os.environ, P2P_RCCL_REGISTER="1"))
    assert out.returncode == 0, out.stderr[-3000:]
    assert "VERIFY 0" in out.stdout and "ABORTED True True" in out.stdout, out.stdout + out.stderr[-2000:]
    assert "TORN DOWN" in out.stdout, out.stderr[-3000:]


@pytest.mark.parametrize("transport,chunk", [("rccl", "0"), ("rccl:4", "0"), ("rccl:4", "1M")])
def test_fuzz_random_groups(native, monkeypatch, transport, chunk):
    """Random groups of self messages (1 B .. 4 MiB, several per group)
    through one or four communicators; with P2P_RCCL_MAX_CHUNK=1M the larger
    messages go out as several chunks on their message's communicator."""
    if chunk != "0":
        monkeypatch.setenv("P2P_RCCL_MAX_CHUNK", chunk)
    s = native.Session(0, 1, device=0, transport=transport, timeout_s=120)
    assert s.fuzz(rounds=30, seed=7, max_bytes=4 << 20) == 0
    del s




@pytest.mark.parametrize("transport", ["rccl", "rccl:4"])
def test_unmatched_receive_is_reported(transport):
    """A receive no send matches ends in an error, not a hang: RCCL rejects a
    lone self receive at ncclGroupEnd ("invalid usage"); the transport
    aborts its communicators and raises.  In a child process: RCCL 2.26 leaves
    thread-local group state behind after a failed ncclGroupEnd, which breaks
    the next communicator created on that thread."""
    code = ("from test_nccl_p2p_amd import require_native\n"
            "s = require_native().Session(0, 1, device=0, transport=%r, timeout_s=5)\n"
            "print('ERR:', s._unmatched_recv(1 << 20))\n"
            "try:\n"
            "    s.run(mode='self', dir='uni', bytes=1 << 20, iters=2, warmup=0)\n"
            "    print('AGAIN: ran')\n"
            "except Exception as e:\n"
            "    print('AGAIN:', e)\n" % transport)
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-3000:]
    assert "ERR: " in out.stdout and ("ncclGroupEnd failed" in out.stdout or "did not finish" in out.stdout), out.stdout
    # the session outlives its aborted communicators; using it
    # again fails with that said, not with RCCL's error on a null communicator.
    assert "AGAIN: " in out.stdout and "on an aborted session" in out.stdout, out.stdout


def test_chunk_sizes_follow_the_channel_knobs():
    """RCCL loses half of an op above 16 MiB per p2p channel, so the
    transport's largest op to itself is 16 MiB x the p2p channels RCCL's INFO
    log reports (64 by default, 4 under NCCL_MAX_P2P_NCHANNELS=4, which RCCL
    caches per process: each setting runs in a process of its own).  With
    the user's own NCCL_DEBUG there is no private log and the round-2 guess
    (64 channels to itself) stands; P2P_RCCL_MAX_CHUNK=0 disables splitting;
    a cap lowers every limit and 0 lifts it again."""
    code = ("import json, test_nccl_p2p_amd as t; n = t.require_native(); "
            "s = n.Session(0, 1, device=0, transport='rccl', timeout_s=60); "
            "a = s.max_chunk(0); ok = s.set_chunk_cap(8 << 20); b = s.max_chunk(0); s.set_chunk_cap(0); "
            "r = json.loads(s.link_reports())[0]; "
            "print(r['op_limit_source'][:9], r['comms'][0]['p2p_channels'], a, ok, b, s.max_chunk(0))")
    for env, src, ch, want in (({}, "rccl INFO", 64, 1 << 30), ({"NCCL_MAX_P2P_NCHANNELS": "4"}, "rccl INFO", 4, 64 << 20),
                               ({"NCCL_DEBUG": "WARN"}, "default (", -1, 1 << 30),
                               ({"P2P_RCCL_MAX_CHUNK": "0"}, "P2P_RCCL_", 64, 0)):
        out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120, cwd=ROOT,
                             env=dict(os.environ, **env))
        assert out.returncode == 0, out.stderr[-2000:]
        line = out.stdout.strip().splitlines()[-1]
        assert line == " ".join([src, str(ch), str(want), "True", str(8 << 20), str(want)]), (env, line)


def test_reference_mode_keeps_rccl_stock_unroll(tmp_path):
    """p2p_matrix --reference runs the reference's methodology on a stock
    RCCL setup: RCCL's own unroll (1 on MI355X), not the unroll 4 the
    default run asks for; RCCL's log says which ran."""
    from conftest import ensure_built
    ensure_built("gpu")
    exe = os.path.join(ROOT, "build", "p2p_matrix")
    got = {}
    for flag in ("--reference", None):
        js = tmp_path / ("r%s.json" % bool(flag))
        cmd = [exe, "--mode", "self", "--size", "4M", "-n", "4", "--no-compat", "--json", str(js), "--timeout", "60"]
        out = subprocess.run(cmd + ([flag] if flag else []), capture_output=True, text=True, timeout=120, cwd=ROOT)
        assert out.returncode == 0, out.stderr[-2000:]
        links = [json.loads(l) for l in js.read_text().splitlines() if '"type":"links"' in l][0]
        got[flag] = links["ranks"][0]["comms"][0]["unroll"]
    assert got == {"--reference": 1, None: 4}, got


def test_rccl_unroll_factor():
    """The transport asks RCCL for unroll-4 kernels (+7% on the bench step,
    +22% on one communicator's step, profiles/r3_unroll/) and RCCL's own log
    confirms it per communicator; P2P_RCCL_UNROLL=0 leaves RCCL's choice (1)
    and a user's RCCL_UNROLL_FACTOR wins; the provenance record holds the
    value in effect.  RCCL reads the variable once per process, so each
    setting runs in a process of its own."""
    code = ("import json, test_nccl_p2p_amd as t; n = t.require_native(); "
            "s = n.Session(0, 1, device=0, transport='rccl', timeout_s=60); "
            "r = json.loads(s.link_reports())[0]; p = json.loads(s.provenance(0)); "
            "print(r['comms'][0]['unroll'], p['env'].get('RCCL_UNROLL_FACTOR'))")
    for env, want in (({}, "4 4"), ({"P2P_RCCL_UNROLL": "0"}, "1 None"), ({"RCCL_UNROLL_FACTOR": "2"}, "2 2")):
        out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120, cwd=ROOT,
                             env=dict(os.environ, **env))
        assert out.returncode == 0, out.stderr[-2000:]
        assert out.stdout.strip().splitlines()[-1] == want, (env, out.stdout)


@pytest.mark.parametrize("transport", ["rccl", "ipc"])
def test_stream_gate_opens_at_its_deadline(native, transport):
    """The pre-posted latency's stream gate: released, it opens at once; never
    released, it opens by itself at its deadline and says so (a host that
    dies between arming and releasing cannot hold the GPU)."""
    sess = native.Session(0, 1, device=0, transport=transport)
    r = json.loads(sess.gate_probe(5.0, True))
    assert r["supported"] and not r["timed_out"] and r["seconds"] < 1.0, r
    r = json.loads(sess.gate_probe(0.3, False))
    assert r["supported"] and r["timed_out"] and 0.25 < r["seconds"] < 5.0, r
    r = json.loads(sess.gate_probe(5.0, True))  # the next gate works normally
    assert not r["timed_out"] and r["seconds"] < 1.0, r
    del sess

"""bench.py --gpus N starts its own N ranks when no launcher set WORLD_SIZE
(VERDICT r4 item 1).  CPU-only: --launch-check runs the launcher plumbing
(child ranks, gloo rendezvous on 127.0.0.1, barrier, per-rank gather, rank 0's
line) without a device; the failure paths are checked too."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _env(**kw):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "MIRSHA_BENCH_DEVICE")}
    env.update(kw)
    return env


def _run(args, **env):
    return subprocess.run([sys.executable, BENCH] + args, env=_env(**env), capture_output=True, text=True,
                          timeout=240)


def test_gpus_2_self_launches_two_ranks():
    r = _run(["--gpus", "2", "--launch-check", "--requests", "1000"])
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 only
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2
    pr = line["per_rank"]
    assert [p["rank"] for p in pr] == [0, 1]
    assert [p["local_rank"] for p in pr] == [0, 1]
    assert len({p["pid"] for p in pr}) == 2 and os.getpid() not in {p["pid"] for p in pr}
    # weak scaling: rank r hashes its own request range
    assert [(p["first_request"], p["requests"]) for p in pr] == [(0, 1000), (1000, 1000)]
    # every rank self-checks its own range; the line ANDs them (verdict r5 item 3a)
    assert [p["self_check"] for p in pr] == [True, True] and line["self_check"] is True
    assert line["distributed"]["backend"] == "gloo"
    assert line["distributed"]["device_identity"]["distinct"] is True


def test_a_failing_rank_check_fails_the_line():
    r = _run(["--gpus", "3", "--launch-check", "--requests", "1010"], MIRSHA_BENCH_CHECK_CORRUPT_RANK="2")
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][0])
    assert [p["self_check"] for p in line["per_rank"]] == [True, True, False]
    assert line["self_check"] is False


def test_gpus_3_self_launches_three_ranks():
    r = _run(["--gpus", "3", "--launch-check", "--requests", "10"])
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][0])
    assert line["n_gpus"] == 3 and len(line["per_rank"]) == 3


def test_gpus_must_match_launcher_world_size():
    r = _run(["--gpus", "2", "--launch-check"], WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    assert r.returncode != 0
    assert "WORLD_SIZE is 1" in r.stderr


def test_more_ranks_than_devices_fails_loudly():
    # no GPU in this container: 0 devices visible
    r = _run(["--gpus", "2", "--steps", "1", "--warmup", "0"])
    assert r.returncode == 2
    assert "device(s) visible" in r.stderr


def test_failing_rank_fails_the_launch():
    # rehearsal knob set (the device count is not checked), but there is no
    # GPU here: every rank dies at its first device call, and so must the launch
    r = _run(["--gpus", "2", "--steps", "1", "--warmup", "0"], MIRSHA_BENCH_DEVICE="0")
    assert r.returncode != 0
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]


def test_sigterm_to_the_launcher_stops_its_ranks():
    """A driver's time limit signals the launching process: its ranks must not
    outlive it (they would keep holding GPUs)."""
    import signal
    import time

    import psutil

    p = subprocess.Popen([sys.executable, BENCH, "--gpus", "2", "--launch-check"],
                         env=_env(MIRSHA_BENCH_CHECK_SLEEP="60"), stdout=subprocess.PIPE, stderr=subprocess.PIPE)
    try:
        parent = psutil.Process(p.pid)
        deadline = time.time() + 60
        kids = []
        while time.time() < deadline and len(kids) < 2:
            kids = parent.children()
            time.sleep(0.2)
        assert len(kids) == 2, kids
        time.sleep(1.0)
        p.send_signal(signal.SIGTERM)
        assert p.wait(timeout=30) == 128 + signal.SIGTERM
        gone, alive = psutil.wait_procs(kids, timeout=30)
        assert not alive, alive
    finally:
        if p.poll() is None:
            p.kill()

"""bench.py's own N-rank launcher: `bench.py --gpus N` without torch.distributed.run starts
the N rank processes itself, before any GPU call; `--dry-launch` makes every rank report its environment and exit
before touching the GPU, so the launcher runs here on CPU."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _run(args, env_extra=None, drop=("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")):
    env = {k: v for k, v in os.environ.items() if k not in drop}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, BENCH] + args, capture_output=True, text=True, timeout=120, env=env)


@pytest.mark.parametrize("n", [2, 4])
def test_self_launch_ranks(n):
    r = _run(["--gpus", str(n), "--dry-launch"])
    assert r.returncode == 0, r.stderr
    lines = [json.loads(ln) for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert sorted(d["rank"] for d in lines) == list(range(n))
    assert all(d["world_size"] == n and d["local_rank"] == d["rank"] for d in lines)
    assert len({d["master"] for d in lines}) == 1 and lines[0]["master"].startswith("127.0.0.1:")


def test_world_size_mismatch_is_an_error():
    r = _run(["--gpus", "2", "--dry-launch"], {"WORLD_SIZE": "3", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode == 2 and "WORLD_SIZE 3" in r.stderr


def test_failing_rank_fails_the_launch():
    r = _run(["--gpus", "3", "--dry-launch"], {"SHUD_BENCH_DRY_FAIL_RANK": "1"})
    assert r.returncode == 5, (r.returncode, r.stderr)


def test_single_gpu_does_not_spawn():
    r = _run(["--gpus", "1", "--dry-launch"])
    assert r.returncode == 0
    d = json.loads(r.stdout.strip())
    assert d["world_size"] == 1 and d["rank"] == 0


def test_hung_rank_is_named_by_its_own_watchdog():
    """A rank that never leaves a phase: its in-rank watchdog (faulthandler, armed per phase at N > 1) exits it after
    the phase's bound (scaled down here), the launcher stops the others and names the rank and the phase."""
    import time
    t0 = time.monotonic()
    r = _run(["--gpus", "3", "--dry-launch"], {"SHUD_BENCH_DRY_HANG_RANK": "1", "SHUD_BENCH_PHASE_SCALE": "0.05"})
    el = time.monotonic() - t0
    assert r.returncode != 0, r.stderr
    assert "rank 1 exited with status 1 in phase 'dry_hang'" in r.stderr, r.stderr[-2000:]
    assert el < 60, el


def test_hung_rank_is_stopped_by_the_launcher():
    """The same hang with the in-rank watchdog off: the launcher's own watchdog (bound + grace) terminates every
    rank, exits 124 and names the stuck rank and phase."""
    import time
    t0 = time.monotonic()
    r = _run(["--gpus", "2", "--dry-launch"], {"SHUD_BENCH_DRY_HANG_RANK": "1", "SHUD_BENCH_PHASE_SCALE": "0.05",
                                                "SHUD_BENCH_RANK_WATCHDOG": "0", "SHUD_BENCH_GRACE_S": "2"})
    el = time.monotonic() - t0
    assert r.returncode == 124, (r.returncode, r.stderr[-2000:])
    assert "watchdog: rank 1 stuck in phase 'dry_hang'" in r.stderr, r.stderr[-2000:]
    assert el < 60, el

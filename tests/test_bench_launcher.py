"""bench.py's own multi-rank launcher (``--gpus N`` without torch.distributed.run): CPU plumbing
check — the children get RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* and form one gloo group."""
import json
import subprocess
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]


def test_bench_spawns_world2_ranks():
    r = subprocess.run([sys.executable, str(REPO / "bench.py"), "--gpus", "2", "--launcher-selftest"],
                       capture_output=True, text=True, timeout=180, cwd=REPO)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out == {"world": 2, "rank_sum": 1.0, "local_rank": 0}


def test_bench_launcher_propagates_failure():
    """A rank that fails makes the launcher fail (and the other rank is not left behind)."""
    r = subprocess.run([sys.executable, str(REPO / "bench.py"), "--gpus", "2", "--launcher-selftest",
                        "--dtype", "nope"], capture_output=True, text=True, timeout=180, cwd=REPO)
    assert r.returncode != 0

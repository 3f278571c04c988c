"""bench.py's own multi-rank launcher (``--gpus N`` without torch.distributed.run): CPU plumbing
check — the children get RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* and form one gloo group."""
import json
import subprocess
import sys
from pathlib import Path

import pytest

REPO = Path(__file__).resolve().parents[1]


@pytest.mark.parametrize("world", [2, 8])
def test_bench_spawns_ranks(world):
    """C3's 2 and C4's 8 ranks from bench.py's own launcher."""
    r = subprocess.run([sys.executable, str(REPO / "bench.py"), "--gpus", str(world), "--launcher-selftest"],
                       capture_output=True, text=True, timeout=240, cwd=REPO)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out == {"world": world, "rank_sum": float(world * (world - 1) // 2), "local_rank": 0}


def test_bench_launcher_propagates_failure():
    """A rank that fails makes the launcher fail (and the other rank is not left behind)."""
    r = subprocess.run([sys.executable, str(REPO / "bench.py"), "--gpus", "2", "--launcher-selftest",
                        "--dtype", "nope"], capture_output=True, text=True, timeout=180, cwd=REPO)
    assert r.returncode != 0


def test_bench_roofline_traffic_comes_from_the_newest_pmc_table():
    """roofline.traffic: conv5's HBM bytes from the newest committed PMC table that has it, whatever template
    argument list the kernel's trace name carries (k_rp_conv3x3_v3<false> since the stamped
    instantiation exists), and null for a non-default shape."""
    sys.path.insert(0, str(REPO))
    import bench
    tables = sorted((REPO / "profiles").glob("*/pmc_traffic.json"))
    assert tables
    got = bench.pmc_traffic(bench.CONV5_KERNEL, True)
    assert got is not None and got[0] > 1e9
    with_conv5 = [str(t.relative_to(REPO)) for t in tables
                  if any(k.split(" grid=")[0].split("<")[0] == bench.CONV5_KERNEL for k in json.loads(t.read_text()))]
    assert got[1] == with_conv5[-1]
    assert bench.pmc_traffic(bench.CONV5_KERNEL, False) is None


def test_bench_roofline_frac_comes_from_the_newest_kernel_trace():
    """roofline.frac (verdict r04 #3): conv5's average duration from the newest committed bench-step
    kernel trace (profiles/*/kernel_stats.csv) that has it, so the line's frac is recomputable from
    profiles/ — 1.4496 TFLOP per launch at the default shape over that average, / 2.5 PF."""
    import csv
    sys.path.insert(0, str(REPO))
    import bench
    got = bench.profile_avg_ns(bench.CONV5_KERNEL, True)
    assert got is not None and got[0] > 1e5
    last = None
    for t in sorted((REPO / "profiles").glob("*/kernel_stats.csv")):
        for row in csv.DictReader(open(t, newline="")):
            if bench.CONV5_KERNEL + "<" in row["Name"] or bench.CONV5_KERNEL + "(" in row["Name"]:
                last = (float(row["AverageNs"]), str(t.relative_to(REPO)))
    assert got[:2] == last
    assert bench.profile_avg_ns(bench.CONV5_KERNEL, False) is None
    frac = bench.CONV5_FLOP_PER_PX * 8 * 480 * 640 / (got[0] * 1e-9) / 1e12 / bench.MFMA_BF16_PEAK_TFLOPS
    assert 0.2 < frac < 1.0

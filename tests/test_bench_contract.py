"""bench.py pieces that need no GPU: the algorithmic byte count the roofline divides by, the
committed rocprof / PMC figures it reads back, and the rank-count checks that must fail before
anything touches a GPU."""
import json
import os
import re
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_algorithmic_bytes_match_survey():
    # 654 B per drone and ctrl step in fp32 (81.75 B per drone*dt), 774 B in f64
    assert bench.alg_bytes_per_drone_step("rpm", 4) == 654
    assert bench.alg_bytes_per_drone_step("rpm", 8) == 774
    assert bench.alg_bytes_per_drone_step("one_d_rpm", 8) == 774 - 3 * 4 - 14 * 3 * 4 - 15 * 3 * 4


def test_committed_profiles_are_read_back():
    """The headline kernel's rocprof figures and PMC traffic come from the newest committed
    summary (profiles/rN_summary.json, highest N), which must hold them."""
    newest = max((f for f in os.listdir(os.path.join(ROOT, "profiles")) if re.fullmatch(r"r\d+_summary\.json", f)),
                 key=lambda f: int(f[1:f.index("_")]))
    name = "gpd::step_kernel_duo<double, 0, true>"
    rp = bench.rocprof_kernel_us(name, 49152, "f64")
    assert rp is not None and rp[1] == "profiles/" + newest
    s = json.load(open(os.path.join(ROOT, rp[1])))
    row = [r for r in s["kernels"] if r["kernel"] == name and "bench" in r["trace"]]
    assert row and row[0]["b2b_launches"] > 0
    assert rp[0] == pytest.approx(row[0]["mean_us"]) and rp[2] == pytest.approx(row[0]["b2b_median_us"])
    tr = bench.pmc_traffic(49152, "f64")
    assert tr is not None and 3.17e6 < tr[0] < 4.5e6          # >= the algorithmic 774 B x 4096
    big = bench.pmc_traffic(1 << 20, "f64")
    assert big is not None and big[0] / (774 * (1 << 20)) < 1.1


def _bench(args, env_extra):
    env = dict(os.environ, **env_extra)
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, capture_output=True, text=True,
                          env=env, timeout=120)


def test_world_size_must_match_gpus():
    r = _bench(["--gpus", "2"], {"WORLD_SIZE": "3", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0 and "WORLD_SIZE=3 but --gpus 2" in (r.stderr + r.stdout)


def test_rccl_needs_the_gpus():
    """--gpus N without a launcher spawns N ranks only when N GPUs are visible for RCCL (none here)."""
    if "WORLD_SIZE" in os.environ:
        pytest.skip("launched under torchrun")
    r = _bench(["--gpus", "2"], {})
    assert r.returncode != 0 and "needs 2 GPUs for RCCL" in (r.stderr + r.stdout)

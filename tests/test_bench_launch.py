"""bench.py --gpus N without a launcher: the launch decision is made before any GPU call,
N > 1 ranks need N devices, and a run that cannot use them exits non-zero instead of reporting a smaller run."""
import os
import subprocess
import sys
from pathlib import Path

import pytest

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))


@pytest.fixture(scope="module")
def bench():
    import bench as b
    return b


def test_launch_plan_single_gpu(bench):
    assert bench.launch_plan(1, {}, 0) == ("run", None)
    assert bench.launch_plan(1, {}, 8) == ("run", None)


def test_launch_plan_spawns_ranks_without_launcher(bench):
    assert bench.launch_plan(8, {}, 8) == ("spawn", 8)
    assert bench.launch_plan(2, {}, 8) == ("spawn", 2)


def test_launch_plan_refuses_missing_devices(bench):
    plan, msg = bench.launch_plan(2, {}, 1)
    assert plan == "error" and "needs 2 GPUs" in msg
    plan, msg = bench.launch_plan(8, {"WORLD_SIZE": "8"}, 1, "nccl")
    assert plan == "error"


def test_launch_plan_under_launcher(bench):
    assert bench.launch_plan(8, {"WORLD_SIZE": "8"}, 8) == ("run", None)
    assert bench.launch_plan(2, {"WORLD_SIZE": "2"}, 1, "gloo") == ("run", None)   # gloo rehearsal on one device
    plan, msg = bench.launch_plan(4, {"WORLD_SIZE": "2"}, 8)
    assert plan == "error" and "WORLD_SIZE=2" in msg


def test_bench_gpus_2_fails_loudly_without_devices():
    # this container has no GPU: --gpus 2 must exit non-zero with the reason, never print a bench line
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, str(REPO / "bench.py"), "--gpus", "2", "--steps", "1"], capture_output=True,
                       text=True, timeout=300, env=env, cwd=REPO)
    if "launching:" in r.stderr:   # a box with >= 2 GPUs: the ranks were started (not this container)
        pytest.skip("devices present")
    assert r.returncode == 2, (r.returncode, r.stderr[-500:])
    assert "needs 2 GPUs" in r.stderr
    assert '"metric"' not in r.stdout

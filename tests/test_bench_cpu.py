"""CPU: bench.py's launcher contract (no GPU needed for these paths)."""
import os
import subprocess
import sys

import msx

REPO = msx.REPO_ROOT


def test_gpus_flag_must_match_the_launcher_world_size():
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    pr = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "4"], env=env,
                        capture_output=True, text=True, timeout=60)
    assert pr.returncode != 0
    assert "WORLD_SIZE=2" in pr.stderr and "--gpus 4" in pr.stderr
    assert pr.stdout == ""


def test_cpu_info_and_median_helpers():
    sys.path.insert(0, REPO)
    import bench
    info = bench.host_cpu_info()
    assert info["nproc"] >= 1 and "model" in info and "numa_nodes" in info
    calls = []
    t, k = bench._median_rate(lambda: calls.append(1), 0, 0.0)
    assert k == 20 and len(calls) == 23 and t >= 0          # 3 warm-ups + 20 timed

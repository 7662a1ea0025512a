"""bench.py launcher contract (CPU): ``--gpus N`` without torchrun spawns N
rank processes and relays rank 0's single JSON line with n_gpus = N."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(extra, env_extra=None):
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT")}
    env.update(env_extra or {})
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--dry-run", "--steps", "3", "--warmup", "1",
                        *extra], capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


def test_self_launch_three_ranks():
    out = _run(["--gpus", "3"])
    assert out["n_gpus"] == 3
    assert out["config"]["parallelism"] == "dp3"
    assert out["config"]["global_batch"] == 3 * 256
    assert out["scaling"] == "weak" and out["higher_is_better"] is True
    for k in ("metric", "value", "unit", "steps", "warmup", "ms_per_step", "vs_baseline", "dtype", "data"):
        assert k in out
    # the InceptionV3 sub-record rides in the same line (BASELINE config 3)
    assert out["models"]["InceptionV3"]["config"]["per_worker_batch"] == 128
    # every rank reports its NUMA placement (utils/numa.py; unbound where sysfs has no KFD GPUs)
    assert [p["rank"] for p in out["placement"]] == [0, 1, 2]
    assert all({"local_rank", "numa", "cpus", "bound"} <= set(p) for p in out["placement"])


def test_single_rank_unchanged():
    out = _run(["--gpus", "1", "--models", "ResNet50"])
    assert out["n_gpus"] == 1 and "models" not in out

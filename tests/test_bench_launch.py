"""bench.py launcher contract: ``--gpus N`` must really run N ranks.

``python bench.py --gpus 2`` without a launcher starts torch.distributed.run as a child
process and reports ``n_gpus: 2`` from a 2-rank process group whose ranks hold identical
weights; ``--gpus 2`` inside a 1-rank job exits non-zero. Runs on CPU (gloo) with the
dry-run MLP model."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _env():
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    env["CUDA_VISIBLE_DEVICES"] = ""
    env["HIP_VISIBLE_DEVICES"] = ""
    env["OMP_NUM_THREADS"] = "2"
    return env


def test_bench_self_launches_n_ranks():
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--model", "mlp",
                        "--steps", "3", "--warmup", "2"], env=_env(), capture_output=True, text=True,
                       timeout=300, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout          # rank 0 only
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["rccl_world"] == 2
    assert out["master_checksum_maxdiff"] == 0.0
    assert out["config"]["parallelism"] == "dp2" and out["config"]["global_batch"] == 2 * out["config"]["per_gpu_batch"]
    assert out["steps"] == 3 and out["ms_per_step"] > 0


def test_bench_refuses_world_mismatch():
    env = _env()
    env["WORLD_SIZE"] = "1"
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--model", "mlp",
                        "--steps", "1", "--warmup", "1"], env=env, capture_output=True, text=True, timeout=120,
                       cwd=ROOT)
    assert p.returncode != 0
    assert "mislabeled" in p.stderr
    assert not [l for l in p.stdout.splitlines() if l.startswith("{")]

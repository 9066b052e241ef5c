"""bench.py driver contract on CPU: ``--gpus N`` with no launcher environment starts N ranks itself
(a child torch.distributed.run), reports ``n_gpus`` = N and a communicator that really spans N
ranks; a launcher/world mismatch fails instead of reporting the wrong rank count."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _env():
    env = dict(os.environ, PYTHONPATH=ROOT, CUDA_VISIBLE_DEVICES="")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    return env


def _json(out):
    lines = [l for l in out.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out[-2000:]
    return json.loads(lines[0])


def test_bench_self_launches_ranks():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--model", "resnet18",
                        "--image-size", "32", "--batch-size", "4", "--steps", "2", "--warmup", "1",
                        "--num-classes", "10", "--watchdog", "300"],
                       capture_output=True, text=True, timeout=600, env=_env(), cwd="/tmp")
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    rec = _json(r.stdout)
    assert rec["n_gpus"] == 2 and rec["steps"] == 2 and rec["warmup"] == 1
    assert rec["config"]["parallelism"] == "dp2" and rec["config"]["global_batch"] == 8
    comm = rec["comm"]
    assert comm["world_check"] == 2 and comm["backend"] == "gloo" and comm["active"]
    # the exposed-communication timing runs on 4 instrumented steps after the timed loop
    assert comm["buckets"] == len(comm["bucket_mb"]) >= 1 and comm["timed_steps"] == 4
    assert comm["exposed_ms"] >= 0 and comm["optimizer_per_bucket"]


def test_bench_refuses_world_mismatch():
    env = _env()
    env.update(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--model", "resnet18",
                        "--image-size", "32", "--batch-size", "2", "--steps", "1", "--warmup", "0",
                        "--num-classes", "10"], capture_output=True, text=True, timeout=300, env=env, cwd="/tmp")
    assert r.returncode != 0
    assert "refusing" in (r.stdout + r.stderr)
    assert not [l for l in r.stdout.splitlines() if l.startswith("{")]

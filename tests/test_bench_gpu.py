"""bench.py on one GPU: the flagship config learns (final loss below ln(num_classes) after the
warm-up + timed steps) and the --graph path captures a real step (its replay is not an empty graph)."""
import json
import math
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(*args, timeout=300):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], capture_output=True, text=True,
                       timeout=timeout, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    return json.loads(lines[-1])


def test_bench_flagship_learns(gpu):
    rec = _bench("--steps", "16", "--warmup", "8", "--infer-images", "0")
    assert rec["metric"] == "resnet50_train_images_per_sec" and rec["n_gpus"] == 1 and rec["steps"] == 16
    assert rec["config"]["global_batch"] == 256 and rec["dtype"] == "bf16"
    loss = rec["config"]["final_loss"]
    assert loss == loss and loss < math.log(rec["config"]["num_classes"]), loss
    assert rec["value"] > 0 and rec["ms_per_step"] > 0


def test_bench_graph_replays_real_step(gpu):
    eager = _bench("--steps", "6", "--warmup", "4", "--batch-size", "64", "--infer-images", "0")
    graph = _bench("--graph", "--steps", "6", "--warmup", "4", "--batch-size", "64", "--infer-images", "0")
    assert graph["config"]["hipgraph"] is True
    loss = graph["config"]["final_loss"]
    assert loss == loss and loss < 1.2 * math.log(1000), loss
    # an empty / partial capture would replay in a fraction of the eager step time
    assert graph["ms_per_step"] > 0.6 * eager["ms_per_step"], (graph["ms_per_step"], eager["ms_per_step"])

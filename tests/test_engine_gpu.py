"""Entry points and engines on the GPU (small configs): hipGraph batch-1 inference, TL training,
text training, checkpoint hand-off — all through the HIP kernels."""
import json
import os
import subprocess
import sys

import pytest
import torch

import pcmp

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(script, *args, timeout=900):
    env = dict(os.environ, PYTHONPATH=ROOT)
    r = subprocess.run([sys.executable, os.path.join(ROOT, script), *args], capture_output=True, text=True,
                       timeout=timeout, env=env)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    return r.stdout


def test_tl_flow_gpu_graph_inference(gpu):
    out = _run("another_neural_net.py", "--model", "resnet50", "--train-size", "256", "--batch-size", "64",
               "--epochs", "1", "--num-images", "20")
    assert "Cuda Device Available" in out and "Inference time is" in out
    rec = json.loads([l for l in out.splitlines() if l.startswith("{")][-1])
    assert rec["batch1_latency"]["graph"] is True


def test_text_bilstm_gpu(gpu):
    out = _run("pytorch_on_language_distr.py", "--model", "bilstm", "--train-size", "256", "--test-size", "64",
               "--epochs", "1")
    assert "Training complete!" in out


def test_text_bert_gpu(gpu):
    out = _run("pytorch_on_language_distr.py", "--model", "bert", "--layers", "2", "--train-size", "128",
               "--test-size", "64", "--epochs", "1")
    assert "  Test took:" in out


def test_graph_predictor_matches_eager(gpu):
    from pcmp.engine.inference import Batch1Predictor
    from pcmp.models.resnet import resnet50
    torch.manual_seed(0)
    m = resnet50(1000).to(gpu).eval()
    x = torch.rand(3, 3, 224, 224)
    p = Batch1Predictor(m, x[:1].to(gpu), use_graph=True)
    with torch.no_grad():
        for i in range(3):
            assert p(x[i:i + 1]) == int(m.forward_logits(x[i:i + 1].to(gpu)).argmax(1))


def test_step_throttle_bounds_inflight(gpu):
    from pcmp.utils.misc import StepThrottle
    dev = torch.device("cuda", 0)
    t = StepThrottle(dev, depth=2)
    a = torch.randn(2048, 2048, device=dev)
    for _ in range(6):
        for _ in range(4):
            a = (a @ a).clamp_(-1, 1)
        t.tick()
        assert t.in_flight <= 2
    torch.cuda.synchronize()
    assert t.in_flight == 2 and torch.isfinite(a).all()

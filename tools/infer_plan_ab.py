"""ResNet-50 batch-1 hipGraph inference latency (p50 over 300 images): round-1 split heuristic
(gemm_plan=0) vs the autotuned small-M plan (gemm_plan=1), each captured fresh, interleaved twice."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import pcmp  # noqa: E402,F401
from pcmp.engine.inference import Batch1Predictor  # noqa: E402
from pcmp.models.resnet import resnet50  # noqa: E402
from pcmp.utils.report import latency_stats  # noqa: E402

from pcmp.ops import _lib  # noqa: E402

assert _lib.load(), _lib.load_error()
dev = torch.device("cuda")
ops = torch.ops.pcmp
torch.manual_seed(0)
m = resnet50(1000).to(dev).eval()
imgs = torch.rand(300, 3, 224, 224)
for rnd in range(2):
    for plan in (0, 1):
        ops.set_knob("gemm_plan", plan)
        pred = Batch1Predictor(m, imgs[:1].to(dev))
        for i in range(20):
            pred(imgs[i:i + 1])
        lat = []
        for i in range(300):
            ts = time.perf_counter()
            pred(imgs[i:i + 1])
            lat.append(time.perf_counter() - ts)
        st = latency_stats(lat)
        print(f"round {rnd} gemm_plan={plan}: p50 {st['p50_ms']:.4f} ms p90 {st['p90_ms']:.4f} p99 {st['p99_ms']:.4f}",
              flush=True)
ops.set_knob("gemm_plan", 1)
print("plans:")
for k in sorted(ops.gemm_plans()):
    print("  ", k)

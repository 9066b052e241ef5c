"""ResNet-50 batch-1 hipGraph inference p50 with the host image in pageable vs pinned memory (the
per-image contract: H2D copy + graph replay + argmax + D2H index), and the bare H2D / D2H costs."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import pcmp  # noqa: E402,F401
from pcmp.engine.inference import Batch1Predictor  # noqa: E402
from pcmp.models.resnet import resnet50  # noqa: E402
from pcmp.ops import _lib  # noqa: E402
from pcmp.utils.report import latency_stats  # noqa: E402

assert _lib.load()
dev = torch.device("cuda")
torch.manual_seed(0)
m = resnet50(1000).to(dev).eval()
imgs = torch.rand(300, 3, 224, 224)
pinned = imgs.pin_memory()
pred = Batch1Predictor(m, imgs[:1].to(dev))
buf = torch.empty(1, 3, 224, 224, device=dev)


def run(src, fn):
    for i in range(20):
        fn(src[i:i + 1])
    lat = []
    for i in range(300):
        ts = time.perf_counter()
        fn(src[i:i + 1])
        lat.append(time.perf_counter() - ts)
    return latency_stats(lat)


def h2d(x):
    buf.copy_(x, non_blocking=True)
    torch.cuda.current_stream().synchronize()


for r in range(2):
    for name, src in (("pageable", imgs), ("pinned", pinned)):
        st = run(src, pred)
        hs = run(src, h2d)
        print(f"round {r} {name}: predict p50 {st['p50_ms']:.4f} ms p90 {st['p90_ms']:.4f}; bare H2D+sync p50 "
              f"{hs['p50_ms']:.4f} ms", flush=True)

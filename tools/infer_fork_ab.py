"""ResNet-50 batch-1 hipGraph inference latency (p50 over 300 pinned images) with the eval-mode
downsample conv on the compute stream (fork off) vs forked onto the side stream (a parallel graph
branch), each captured fresh, interleaved twice; logits of both variants compared."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import pcmp  # noqa: E402,F401
from pcmp.engine.inference import Batch1Predictor  # noqa: E402
from pcmp.models.resnet import resnet50  # noqa: E402
from pcmp.ops import _lib, conv_blocks  # noqa: E402
from pcmp.utils.report import latency_stats  # noqa: E402

assert _lib.load(), _lib.load_error()
dev = torch.device("cuda")
torch.manual_seed(0)
m = resnet50(1000).to(dev).eval()
imgs = torch.rand(300, 3, 224, 224).pin_memory()
outs = {}
for rnd in range(2):
    for rows in (0, 16384 if rnd == 0 else 1 << 30):
        conv_blocks.EVAL_FORK_MAX_ROWS = rows
        pred = Batch1Predictor(m, imgs[:1].to(dev))
        with torch.no_grad():
            outs[rows] = m(imgs[:1].to(dev)).float().cpu()
        for i in range(20):
            pred(imgs[i:i + 1])
        lat = []
        for i in range(300):
            ts = time.perf_counter()
            pred(imgs[i:i + 1])
            lat.append(time.perf_counter() - ts)
        st = latency_stats(lat)
        print(f"round {rnd} fork_rows<={rows}: p50 {st['p50_ms']:.4f} ms p90 {st['p90_ms']:.4f} p99 {st['p99_ms']:.4f}",
              flush=True)
vals = list(outs.values())
print("max |logit diff| fork vs no fork:", max((v - vals[0]).abs().max().item() for v in vals))

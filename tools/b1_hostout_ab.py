"""Batch-1 latency A/B in one process: class-index D2H inside the hipGraph (PCMP_B1_HOST_OUT=1)
against ``.item()`` after the replay (=0), interleaved rounds on the bench's pinned-image loop."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pcmp  # noqa: E402
from pcmp.engine.inference import Batch1Predictor  # noqa: E402
from pcmp.models.resnet import resnet50  # noqa: E402
from pcmp.utils.report import latency_stats  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    m = resnet50(1000).to(dev).eval()
    n = int(os.environ.get("N_IMG", "300"))
    imgs = torch.rand(n, 3, 224, 224, generator=torch.Generator().manual_seed(5)).pin_memory()
    preds = {}
    for arm in ("0", "1"):
        os.environ["PCMP_B1_HOST_OUT"] = arm
        preds[arm] = Batch1Predictor(m, imgs[:1].to(dev), use_graph=True)
    same = all(preds["0"](imgs[i:i + 1]) == preds["1"](imgs[i:i + 1]) for i in range(8))
    print("predictions equal:", same, flush=True)
    for r in range(3):
        for arm in ("0", "1"):
            p = preds[arm]
            for i in range(20):
                p(imgs[i:i + 1])
            lat = []
            for i in range(n):
                ts = time.perf_counter()
                p(imgs[i:i + 1])
                lat.append(time.perf_counter() - ts)
            s = latency_stats(lat)
            print(f"round {r} host_out={arm} p50 {s['p50_ms']:.4f} p90 {s['p90_ms']:.4f} p99 {s['p99_ms']:.4f} ms",
                  flush=True)


if __name__ == "__main__":
    main()

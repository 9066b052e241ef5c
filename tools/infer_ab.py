"""Batch-1 ResNet-50 inference latency A/B in one process, as bench.py measures it (pinned host
images, hipGraph replay + argmax + pinned D2H index): one Batch1Predictor per variant (its warm-up
autotunes the small-M plans under the variant's knobs), interleaved rounds.
Usage: python tools/infer_ab.py --variants 'fix:sk_fix=1;nofix:sk_fix=0' [--rounds 3] [--images 300]"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pcmp  # noqa: E402,F401
from pcmp.engine.inference import Batch1Predictor  # noqa: E402
from pcmp.models.resnet import resnet50  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="fix:sk_fix=1;nofix:sk_fix=0")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--images", type=int, default=300)
    a = ap.parse_args()
    from pcmp.ops import _lib
    assert _lib.load(), _lib.load_error()
    ops = torch.ops.pcmp
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    m = resnet50(1000).to(dev).eval()
    imgs = torch.rand(a.images, 3, 224, 224, generator=torch.Generator().manual_seed(5)).pin_memory()
    variants = []
    for v in a.variants.split(";"):
        name, _, kv = v.partition(":")
        variants.append((name, {k: int(x) for k, x in (i.split("=") for i in filter(None, kv.split(",")))}))
    preds = {}
    for r in range(a.rounds):
        for name, knobs in variants:
            old = {k: ops.set_knob(k, v) for k, v in knobs.items()}
            if name not in preds:
                ops.autotune_clear()   # each variant plans its small-M convs under its own knobs
                preds[name] = Batch1Predictor(m, imgs[:1].to(dev), use_graph=True)
                nfix = sum("+fix" in e for e in ops.gemm_plans())
                print(f"{name}: plans {len(ops.gemm_plans())}, with fixup {nfix}", flush=True)
            pred = preds[name]
            for i in range(20):
                pred(imgs[i:i + 1])
            lat = []
            for i in range(a.images):
                t = time.perf_counter()
                pred(imgs[i:i + 1])
                lat.append(time.perf_counter() - t)
            lat.sort()
            for k, v in old.items():
                ops.set_knob(k, v)
            print(f"round {r} {name:8s} p50 {lat[len(lat) // 2] * 1e3:.4f} ms  p90 {lat[int(len(lat) * 0.9)] * 1e3:.4f} ms",
                  flush=True)


if __name__ == "__main__":
    main()

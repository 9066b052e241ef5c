"""Host-side cost of enqueuing one ResNet training step vs its GPU time (is the step launch-bound?).

Runs W warm-up steps, then times K steps twice: (a) host time to ENQUEUE each step with no device
synchronisation (the GPU queue absorbs the launches), (b) synchronised wall time per step.  If (a)
approaches (b) the step is host-bound and hipGraph capture / fewer launches pay off directly.
Usage (GPU): python tools/host_overhead.py [--model resnet50] [--batch 256]
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
from pcmp.parallel import launch  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--model", default="resnet50")
ap.add_argument("--batch", type=int, default=256)
ap.add_argument("--steps", type=int, default=10)
ap.add_argument("--cprofile", action="store_true", help="cProfile the host side of the timed steps")
a = ap.parse_args()
os.environ.setdefault("PCMP_MAX_INFLIGHT", "0")   # measure enqueue, not the run-ahead throttle
env = launch.init()
ns = argparse.Namespace(model=a.model, num_classes=1000, lr=0.1, image_size=224, batch_size=a.batch,
                        ddp_force=False, grad_dtype=None, sync_bn=False)
step = bench.build_hip(ns, env)
x = torch.rand(a.batch, 3, 224, 224, device=env.device)
y = torch.randint(0, 1000, (a.batch,), device=env.device)
for _ in range(5):
    step(x, y)
torch.cuda.synchronize()
host = []
prof = None
if a.cprofile:
    import cProfile
    prof = cProfile.Profile()
    prof.enable()
t_all = time.perf_counter()
for _ in range(a.steps):
    t = time.perf_counter()
    step(x, y)
    host.append(time.perf_counter() - t)
t_enq = time.perf_counter() - t_all
if prof is not None:
    prof.disable()
torch.cuda.synchronize()
t_tot = time.perf_counter() - t_all
print(f"host enqueue per step: mean {1e3 * sum(host) / len(host):.2f} ms, min {1e3 * min(host):.2f} ms; "
      f"GPU-bound wall per step {1e3 * t_tot / a.steps:.2f} ms (enqueue of all steps {1e3 * t_enq:.1f} ms)")
if prof is not None:
    import pstats
    pstats.Stats(prof).sort_stats("tottime").print_stats(25)

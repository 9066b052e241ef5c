"""Per-step device times of the bench step (diagnosis of the forced-RCCL path, round 6).

python tools/ddp_step_times.py [--timing] <bench.py args...>: builds bench.py's step, runs the warm-up
steps, then --steps steps with one CUDA event after each, and prints every step's ms (no host sync
inside the loop) plus the host enqueue time per step."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
timing = "--timing" in sys.argv
if timing:
    sys.argv.remove("--timing")
import bench  # noqa: E402
import torch  # noqa: E402

args = bench.parse()
from pcmp.parallel import launch  # noqa: E402

env = launch.init(args.local_rank, force_init=args.ddp_force)
B = args.batch_size
x = torch.rand(B, 3, args.image_size, args.image_size, device=env.device)
y = torch.randint(0, args.num_classes, (B,), device=env.device)
step = bench.build_hip(args, env)
for i in range(args.warmup):
    step.opt.set_lr(args.lr * (i + 1) / max(1, args.warmup))
    step(x, y)
if timing and step.ddp is not None:
    step.ddp.time_exposed(True)
torch.cuda.synchronize()
evs, host = [], []
e0 = torch.cuda.Event(enable_timing=True)
e0.record()
for i in range(args.steps):
    t = time.perf_counter()
    step(x, y)
    host.append((time.perf_counter() - t) * 1e3)
    e = torch.cuda.Event(enable_timing=True)
    e.record()
    evs.append(e)
torch.cuda.synchronize()
prev, ms = e0, []
for e in evs:
    ms.append(prev.elapsed_time(e))
    prev = e
print("device ms/step:", " ".join(f"{v:.1f}" for v in ms))
print("host enqueue ms/step:", " ".join(f"{v:.1f}" for v in host))
print(f"mean device {sum(ms) / len(ms):.2f} ms, mean host {sum(host) / len(host):.2f} ms", flush=True)
launch.shutdown()

"""Print the loss curve of N training steps on one fixed synthetic batch (hip vs torch impl)."""
import argparse, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import bench

ap = argparse.ArgumentParser()
ap.add_argument("--impl", default="hip")
ap.add_argument("--steps", type=int, default=20)
ap.add_argument("--batch-size", type=int, default=64)
ap.add_argument("--model", default="resnet50")
ap.add_argument("--lr", type=float, default=0.1)
a = ap.parse_args()
from pcmp.parallel import launch
env = launch.init()
ns = argparse.Namespace(model=a.model, num_classes=1000, lr=a.lr, image_size=224, batch_size=a.batch_size)
step = bench.build_hip(ns, env) if a.impl == "hip" else bench.build_torch(ns, env)
g = torch.Generator(device=env.device).manual_seed(17)
x = torch.rand(a.batch_size, 3, 224, 224, device=env.device, generator=g)
y = torch.randint(0, 1000, (a.batch_size,), device=env.device, generator=g)
out = []
for i in range(a.steps):
    out.append(round(float(step(x, y)), 3))
print(a.impl, out)

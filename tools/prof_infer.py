"""ResNet-50 batch-1 hipGraph inference loop for rocprofv3 (kernel time per image vs latency)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import pcmp  # noqa: E402,F401
from pcmp.engine.inference import Batch1Predictor  # noqa: E402
from pcmp.models.resnet import resnet50  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 50
dev = torch.device("cuda")
torch.manual_seed(0)
m = resnet50(num_classes=10).to(dev).eval()
imgs = torch.rand(n, 3, 224, 224, device=dev)
p = Batch1Predictor(m, imgs[:1], use_graph=True)
for i in range(5):
    p(imgs[i:i + 1])
torch.cuda.synchronize()
lat = []
for i in range(n):
    t = time.perf_counter()
    p(imgs[i:i + 1])
    lat.append(time.perf_counter() - t)
lat.sort()
print(f"batch-1 p50 {1e3 * lat[len(lat) // 2]:.3f} ms over {n} images")

"""ResNet-50 transfer-learning step (the reference's P1 workload, B=64, bf16): eager against one
hipGraph replay (pcmp.engine.graph.GraphedStep), interleaved rounds, plus the host enqueue time of
an eager step (time until the Python call returns, no sync).

Usage: python tools/tl_graph_ab.py [rounds] [iters]
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import pcmp  # noqa: E402,F401
from pcmp.engine.graph import GraphedStep  # noqa: E402
from pcmp.engine.trainer import make_state  # noqa: E402
from pcmp.models.resnet import resnet50_transfer  # noqa: E402
from pcmp.ops import _lib, cross_entropy  # noqa: E402

assert _lib.load(), _lib.load_error()
rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 40
dev = torch.device("cuda")
B = 64
torch.manual_seed(0)
x = torch.rand(B, 3, 224, 224, device=dev)
y = torch.randint(0, 10, (B,), device=dev)
m = resnet50_transfer(10).to(dev).train()
st = make_state(m, "adam", lr=3e-3)
loss_fn = lambda a, b: cross_entropy(m.forward_logits(a), b)  # noqa: E731


def eager():
    st.zero_grad()
    st.backward_step(loss_fn(x, y))


for _ in range(8):
    eager()
torch.cuda.synchronize()
g = GraphedStep(st, loss_fn, [x, y])
for _ in range(4):
    g(x, y)
torch.cuda.synchronize()


def timed(fn):
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / iters * 1e3


def host_ms():
    torch.cuda.synchronize()
    hs = []
    for _ in range(10):
        t = time.perf_counter()
        eager()
        hs.append((time.perf_counter() - t) * 1e3)
        torch.cuda.synchronize()
    hs.sort()
    return hs[len(hs) // 2]


print(f"ResNet-50 TL step B={B}: eager host enqueue p50 {host_ms():.3f} ms")
for r in range(rounds):
    te = timed(eager)
    tg = timed(lambda: g(x, y))
    print(f"round {r + 1}: eager {te:.3f} ms/step ({B / te * 1e3:,.0f} img/s) | graph {tg:.3f} ms/step "
          f"({B / tg * 1e3:,.0f} img/s)", flush=True)

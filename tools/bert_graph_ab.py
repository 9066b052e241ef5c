"""BERT graphed-step A/B (round 6 regression check): GraphedStep timing with the ranged optimizer
step (begin_step/step_range/end_step) vs one whole-arena adam_flat call, interleaved."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import pcmp  # noqa: E402,F401
from pcmp import optim  # noqa: E402
from pcmp.data.synthetic import SyntheticIMDB  # noqa: E402
from pcmp.engine.graph import GraphedStep  # noqa: E402
from pcmp.engine.trainer import make_state  # noqa: E402
from pcmp.models.bert import bert_base  # noqa: E402
from pcmp.ops.kernels import K  # noqa: E402
from pcmp.ops.params import bump_weight_gen  # noqa: E402

dev = torch.device("cuda")
ids, mask, y = SyntheticIMDB(32, 128).get_batch(list(range(32)), dev)
ranged_step = optim.Adam.step


def whole_step(self):
    self.step_t.add_(1.0)
    K.adam_flat(self.flat.master, self.flat.grad, self.m1, self.m2, self.flat.shadow, None, self.lr_t,
                self.grad_scale, self.step_t, self.beta1, self.beta2, self.eps, self.wd, self.decoupled)
    bump_weight_gen()
    self.steps += 1


def run(graph, n=30):
    m = bert_base().to(dev)
    st = make_state(m, "adamw", lr=2e-5, eps=1e-8, clip=1.0)
    if graph:
        g = GraphedStep(st, lambda a, b, c: m(a, None, b, c)[0], [ids, mask, y])
        fn = lambda: g(ids, mask, y)  # noqa: E731
    else:
        def fn():
            st.zero_grad()
            st.backward_step(m(ids, None, mask, y)[0])
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / n * 1e3


for r in range(2):
    for name, impl in (("ranged", ranged_step), ("whole", whole_step)):
        optim.Adam.step = impl
        print(f"round {r} {name}: eager {run(False):.2f} ms, graph {run(True):.2f} ms", flush=True)

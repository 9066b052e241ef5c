"""BERT-base GraphedStep replay vs eager in a fresh process (round 6: the replay ran at half the eager
speed in processes that had not run a ResNet first).  Prints one line; run once per environment."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import pcmp  # noqa: E402,F401
from pcmp.data.synthetic import SyntheticIMDB  # noqa: E402
from pcmp.engine.graph import GraphedStep  # noqa: E402
from pcmp.engine.trainer import make_state  # noqa: E402
from pcmp.models.bert import bert_base  # noqa: E402

dev = torch.device("cuda")
ids, mask, y = SyntheticIMDB(32, 128).get_batch(list(range(32)), dev)


def timeit(fn, n=30):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / n * 1e3


m = bert_base().to(dev)
st = make_state(m, "adamw", lr=2e-5, eps=1e-8, clip=1.0)


def eager():
    st.zero_grad()
    st.backward_step(m(ids, None, mask, y)[0])


te = timeit(eager)
g = GraphedStep(st, lambda a, b, c: m(a, None, b, c)[0], [ids, mask, y])
tg = timeit(lambda: g(ids, mask, y))
print(f"[{os.environ.get('TAGV', '')}] eager {te:.2f} ms, graph {tg:.2f} ms", flush=True)

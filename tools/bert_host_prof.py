"""Host-side (CPU) cost of one eager BERT-base train step: cProfile over N steps with the GPU
queue kept shallow (a sync every step), top functions by total own time.  Usage:
python tools/bert_host_prof.py [steps]"""
import cProfile
import os
import pstats
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pcmp  # noqa: E402,F401
from pcmp.data.synthetic import SyntheticIMDB  # noqa: E402
from pcmp.engine.trainer import make_state  # noqa: E402
from pcmp.models.bert import bert_base  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
dev = torch.device("cuda", 0)
ids, mask, y = SyntheticIMDB(32, 128).get_batch(list(range(32)), dev)
m = bert_base().to(dev)
st = make_state(m, "adamw", lr=2e-5, eps=1e-8, clip=1.0)


def step():
    st.zero_grad()
    st.backward_step(m(ids, None, mask, y)[0])


for _ in range(8):
    step()
torch.cuda.synchronize()
t_host = 0.0
for _ in range(10):
    t0 = time.perf_counter()
    step()
    t_host += time.perf_counter() - t0
    torch.cuda.synchronize()
print(f"host enqueue per step (GPU idle at start): {t_host / 10 * 1e3:.2f} ms", flush=True)
# backward on the calling thread so cProfile sees the autograd Functions' Python
torch.autograd.set_multithreading_enabled(False)
pr = cProfile.Profile()
pr.enable()
for _ in range(steps):
    step()
    torch.cuda.synchronize()
pr.disable()
ps = pstats.Stats(pr)
ps.sort_stats("tottime").print_stats(45)
ps.sort_stats("cumulative").print_stats(40)

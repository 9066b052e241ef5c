"""BERT-base train-step A/B in one process: embedding sum fused into the LayerNorm kernel
(EmbedLayerNormFn) vs the eager torch broadcast (models.bert._EMB_FUSED), interleaved rounds,
B=32 S=128 AdamW + clip (tools/bench_suite.py's bert_train step)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pcmp  # noqa: E402,F401
import pcmp.models.bert as bert  # noqa: E402
from pcmp.data.synthetic import SyntheticIMDB  # noqa: E402
from pcmp.engine.trainer import make_state  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    ids, mask, y = SyntheticIMDB(32, 128).get_batch(list(range(32)), dev)
    torch.manual_seed(0)
    m = bert.bert_base().to(dev)
    st = make_state(m, "adamw", lr=2e-5, eps=1e-8, clip=1.0)

    def step():
        st.zero_grad()
        st.backward_step(m(ids, None, mask, y)[0])

    def timeit(n=40):
        for _ in range(8):
            step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(n):
            step()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / n

    for r in range(3):
        for fused in (False, True):
            bert._EMB_FUSED = fused
            t = timeit()
            print(f"round {r} emb_fused={int(fused)} {32 / t:.1f} samples/s {t * 1e3:.3f} ms/step", flush=True)


if __name__ == "__main__":
    main()

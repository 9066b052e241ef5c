"""BERT-base / BiLSTM train-step knob A/B in one process, interleaved rounds (B=32, S=128, AdamW +
clip 1.0; tools/bench_suite.py's steps).  Usage:
python tools/text_knob_ab.py --variants 'det:emb_atomic=0;atomic:emb_atomic=1' [--models bert,bilstm]"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import pcmp  # noqa: E402,F401
from pcmp.data.synthetic import SyntheticIMDB  # noqa: E402
from pcmp.engine.trainer import make_state  # noqa: E402
from pcmp.ops import _lib, cross_entropy  # noqa: E402


def build(name, dev, ids, mask, y):
    if name == "bert":
        from pcmp.models.bert import bert_base
        m = bert_base().to(dev)
        st = make_state(m, "adamw", lr=2e-5, eps=1e-8, clip=1.0)
        return st, lambda: m(ids, None, mask, y)[0]
    from pcmp.models.bilstm import BiLSTMClassifier
    m = BiLSTMClassifier().to(dev)
    st = make_state(m, "adamw", lr=1e-3, clip=1.0)
    return st, lambda: cross_entropy(m.forward_logits(ids), y)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="det:emb_atomic=0;atomic:emb_atomic=1")
    ap.add_argument("--models", default="bert,bilstm")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--steps", type=int, default=30)
    a = ap.parse_args()
    assert _lib.load(), _lib.load_error()
    ops = torch.ops.pcmp
    dev = torch.device("cuda")
    ids, mask, y = SyntheticIMDB(32, 128).get_batch(list(range(32)), dev)
    variants = []
    for v in a.variants.split(";"):
        name, _, kv = v.partition(":")
        variants.append((name, {k: int(x) for k, x in (i.split("=") for i in filter(None, kv.split(",")))}))
    for model in a.models.split(","):
        st, loss_fn = build(model, dev, ids, mask, y)

        def step():
            st.zero_grad()
            st.backward_step(loss_fn())
        for r in range(a.rounds):
            for name, knobs in variants:
                old = {k: ops.set_knob(k, v) for k, v in knobs.items()}
                for _ in range(5):
                    step()
                torch.cuda.synchronize()
                t = time.perf_counter()
                for _ in range(a.steps):
                    step()
                torch.cuda.synchronize()
                ms = (time.perf_counter() - t) / a.steps * 1e3
                for k, v in old.items():
                    ops.set_knob(k, v)
                print(f"{model} round {r} {name:8s} {ms:7.3f} ms/step  {32 / ms * 1e3:8.1f} samples/s", flush=True)


if __name__ == "__main__":
    main()

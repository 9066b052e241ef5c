"""BERT-base B=32 S=128 train-step A/B in one process (AdamW + clip, tools/bench_suite.py's bert_train
step), interleaved rounds.  Variants are "name:ENV=v,knob=v,...": upper-case keys are environment
variables (e.g. PCMP_WGRAD_STREAM; the side-stream switches are re-read via ops.params.refresh_env), lower-case keys are kernel knobs (set_knob).
GRAPH=1 in a variant replays the step from one captured hipGraph (pcmp.engine.graph.GraphedStep,
captured on the variant's first use).  Also prints the host-side launch time of the eager step
(time to enqueue, no synchronisation) so a launch-bound step shows up.
Usage: python tools/bert_ab.py --variants 'eager:PCMP_WGRAD_STREAM=0;side:' [--rounds 3] [--steps 30]
"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pcmp  # noqa: E402,F401
from pcmp.data.synthetic import SyntheticIMDB  # noqa: E402
from pcmp.engine.trainer import make_state  # noqa: E402
from pcmp.models.bert import bert_base  # noqa: E402
from pcmp.ops import params as _params  # noqa: E402


def parse(spec):
    out = []
    for v in spec.split(";"):
        name, _, kv = v.partition(":")
        env, knobs = {}, {}
        for item in filter(None, kv.split(",")):
            k, val = item.split("=")
            (env if k.isupper() else knobs)[k] = val
        out.append((name, env, knobs))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="serial:PCMP_WGRAD_STREAM=0;side:")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--steps", type=int, default=30)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    ids, mask, y = SyntheticIMDB(32, 128).get_batch(list(range(32)), dev)
    torch.manual_seed(0)
    m = bert_base().to(dev)
    st = make_state(m, "adamw", lr=2e-5, eps=1e-8, clip=1.0)
    ops = torch.ops.pcmp

    def step():
        st.zero_grad()
        loss = m(ids, None, mask, y)[0]
        st.backward_step(loss)
        return loss

    variants = parse(a.variants)
    graphs = {}
    for r in range(a.rounds):
        for name, env, knobs in variants:
            old_env = {k: os.environ.get(k) for k in env}
            os.environ.update(env)
            _params.refresh_env()
            old_k = {k: ops.set_knob(k, int(v)) for k, v in knobs.items()}
            fn = step
            if env.get("GRAPH") == "1":
                if name not in graphs:
                    from pcmp.engine.graph import GraphedStep
                    for _ in range(4):
                        step()
                    graphs[name] = GraphedStep(st, lambda a_, b_, c_: m(a_, None, b_, c_)[0], [ids, mask, y])
                g = graphs[name]
                fn = lambda: g(ids, mask, y)  # noqa: E731
            for _ in range(6):
                fn()
            torch.cuda.synchronize()
            h0 = time.perf_counter()
            fn()
            host_ms = (time.perf_counter() - h0) * 1e3
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.steps):
                loss = fn()
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / a.steps
            for k, v in old_k.items():
                ops.set_knob(k, v)
            for k, v in old_env.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v
            _params.refresh_env()
            print(f"round {r} {name:12s} {32 / dt:8.1f} samples/s {dt * 1e3:7.3f} ms/step "
                  f"host-enqueue {host_ms:6.2f} ms loss {loss.item():.4f}", flush=True)


if __name__ == "__main__":
    main()

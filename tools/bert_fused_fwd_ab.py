"""Same-process A/B of the fused BERT sublayer forward ops (bert_attn_fwd / bert_ffn_fwd: one native
dispatch per sublayer) against issuing the same kernels one op at a time from Python (the round-4
dispatch pattern), interleaved rounds; prints samples/s and the host enqueue time per step.
Usage: python tools/bert_fused_fwd_ab.py [rounds] [steps]"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pcmp  # noqa: E402,F401
from pcmp.data.synthetic import SyntheticIMDB  # noqa: E402
from pcmp.engine.trainer import make_state  # noqa: E402
from pcmp.models.bert import bert_base  # noqa: E402
from pcmp.ops import kernels  # noqa: E402

K = kernels.K
fused = {"attn": K.bert_attn_fwd, "ffn": K.bert_ffn_fwd}


def lin(x, w, bias):
    M, C = x.shape
    return K.conv_fwd(x.view(M, 1, 1, C), w.view(w.shape[0], 1, 1, C), 1, 0, bias, None, False, False)[0].view(M, -1)


def seq_attn(h, ids, wq, bq, wo, bo, g, b, B, S, H, pa, sa, oa, ph, sh, oh, eps, salt=None):
    qkv = lin(h, wq, bq)
    ctx, lse = K.attention_fwd(qkv, ids, B, S, H, pa, sa, oa, salt)
    y = K.layernorm_fwd(lin(ctx, wo, bo), h, g, b, eps, ph, sh, oh, salt)
    return [y[0], qkv, ctx, lse, y[1], y[2], y[3]]


def seq_ffn(h1, w1, b1, w2, b2, g, b, ph, sh, oh, eps, salt=None):
    gu, u = K.linear_gelu_fwd(h1, w1, b1)
    y = K.layernorm_fwd(lin(gu, w2, b2), h1, g, b, eps, ph, sh, oh, salt)
    return [y[0], gu, u, y[1], y[2], y[3]]


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 30
    dev = torch.device("cuda", 0)
    ids, mask, y = SyntheticIMDB(32, 128).get_batch(list(range(32)), dev)
    torch.manual_seed(0)
    m = bert_base().to(dev)
    st = make_state(m, "adamw", lr=2e-5, eps=1e-8, clip=1.0)

    def step():
        st.zero_grad()
        st.backward_step(m(ids, None, mask, y)[0])

    for r in range(rounds):
        for name, (fa, ff) in (("fused", (fused["attn"], fused["ffn"])), ("op-by-op", (seq_attn, seq_ffn))):
            K.bert_attn_fwd, K.bert_ffn_fwd = fa, ff
            for _ in range(5):
                step()
            torch.cuda.synchronize()
            t_host, t0 = 0.0, time.perf_counter()
            for _ in range(steps):
                h0 = time.perf_counter()
                step()
                t_host += time.perf_counter() - h0
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / steps
            print(f"round {r} {name:9s} {32 / dt:8.1f} samples/s  {dt * 1e3:6.3f} ms/step  host-enqueue "
                  f"{t_host / steps * 1e3:5.2f} ms", flush=True)


if __name__ == "__main__":
    main()

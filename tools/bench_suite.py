"""Secondary benchmarks for the BASELINE.json configs beyond the flagship (bench.py):

  resnet18_train   ResNet-18 bf16 training img/s (B=256)             hip vs torch (MIOpen, autocast)
  resnet50_infer   ResNet-50 batch-1 inference latency p50/p90/p99  hip+hipGraph vs torch eager / torch graph
  bilstm_train     BiLSTM text classifier train samples/s (B=32,S=128)  hip vs torch (nn.LSTM packed)
  bert_train       BERT-base train samples/s (B=32,S=128)           hip vs HF transformers (autocast)
One JSON line per measurement.  Usage: python tools/bench_suite.py [names...]
"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import pcmp  # noqa: E402,F401
from pcmp.ops import cross_entropy  # noqa: E402

dev = torch.device("cuda")
HIP_ONLY = os.environ.get("SUITE_HIP_ONLY") == "1"   # skip the stock-PyTorch comparators (clean profiles)


def timeit(fn, warmup=8, iters=30):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / iters


def emit(**kw):
    print(json.dumps(kw), flush=True)


def hip_train_step(model, make_loss, opt="sgd", lr=0.1, **okw):
    from pcmp.engine.trainer import make_state
    st = make_state(model, opt, lr=lr, **okw)

    def step():
        st.zero_grad()
        st.backward_step(make_loss())
    return step


def torch_train_step(model, make_loss, opt):
    def step():
        opt.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            loss = make_loss()
        loss.backward()
        opt.step()
    return step


def resnet18_train():
    from pcmp.models.resnet import resnet18
    from pcmp.models.torch_ref import TorchResNet
    B = 256
    x = torch.rand(B, 3, 224, 224, device=dev)
    y = torch.randint(0, 1000, (B,), device=dev)
    m = resnet18(1000).to(dev)
    t = timeit(hip_train_step(m, lambda: cross_entropy(m.forward_logits(x), y), momentum=0.9))
    emit(bench="resnet18_train", impl="hip", img_s=B / t, ms=t * 1e3, batch=B)
    tm = TorchResNet("resnet18", 1000).to(dev).to(memory_format=torch.channels_last)
    o = torch.optim.SGD(tm.parameters(), lr=0.1, momentum=0.9, fused=True)
    xc = x.contiguous(memory_format=torch.channels_last)
    t = timeit(torch_train_step(tm, lambda: torch.nn.functional.cross_entropy(tm(xc).float(), y), o))
    emit(bench="resnet18_train", impl="torch", img_s=B / t, ms=t * 1e3, batch=B)


def resnet50_tl_train(B=64):
    """The reference's measured workload (BASELINE P1): ResNet-50 transfer learning -- frozen
    backbone with BN in train mode, head Linear(2048,512)-ReLU-Dropout(0.2)-Linear(512,10), Adam 3e-3
    on the head, NLL loss, batch 64 of 224x224 images."""
    from pcmp.models.resnet import resnet50_transfer
    from pcmp.models.torch_ref import TorchResNet
    x = torch.rand(B, 3, 224, 224, device=dev)
    y = torch.randint(0, 10, (B,), device=dev)
    m = resnet50_transfer(10).to(dev).train()
    t = timeit(hip_train_step(m, lambda: cross_entropy(m.forward_logits(x), y), "adam", 3e-3))
    emit(bench="resnet50_tl_train", impl="hip", img_s=B / t, ms=t * 1e3, batch=B, vs_reference_P1a=round(B / t / 1.43, 1))
    head = torch.nn.Sequential(torch.nn.Linear(2048, 512), torch.nn.ReLU(), torch.nn.Dropout(0.2),
                               torch.nn.Linear(512, 10), torch.nn.LogSoftmax(dim=1))
    tm = TorchResNet("resnet50", head=head).to(dev).to(memory_format=torch.channels_last).train()
    for n_, p_ in tm.named_parameters():
        p_.requires_grad_(n_.startswith("fc."))
    o = torch.optim.Adam([p_ for p_ in tm.parameters() if p_.requires_grad], lr=3e-3, fused=True)
    xc = x.contiguous(memory_format=torch.channels_last)
    t = timeit(torch_train_step(tm, lambda: torch.nn.functional.nll_loss(tm(xc).float(), y), o))
    emit(bench="resnet50_tl_train", impl="torch", img_s=B / t, ms=t * 1e3, batch=B)


def resnet50_infer(n=300):
    from pcmp.engine.inference import Batch1Predictor
    from pcmp.models.resnet import resnet50
    from pcmp.models.torch_ref import TorchResNet
    from pcmp.utils.report import latency_stats
    imgs = torch.rand(n, 3, 224, 224)
    m = resnet50(1000).to(dev).eval()

    def run(pred):
        lat = []
        for i in range(n):
            ts = time.perf_counter()
            pred(imgs[i:i + 1])
            lat.append(time.perf_counter() - ts)
        return latency_stats(lat)
    for graph in (True, False):
        p = Batch1Predictor(m, imgs[:1].to(dev), use_graph=graph)
        emit(bench="resnet50_infer_b1", impl="hip" + ("+graph" if graph else ""), **run(p))
    tm = TorchResNet("resnet50", 1000).to(dev).to(memory_format=torch.channels_last).eval()
    static = torch.zeros(1, 3, 224, 224, device=dev).contiguous(memory_format=torch.channels_last)

    @torch.no_grad()
    def eager(x):
        static.copy_(x)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            return int(tm(static).argmax(1).item())
    for _ in range(5):
        eager(imgs[:1])
    emit(bench="resnet50_infer_b1", impl="torch_eager", **run(eager))
    g = torch.cuda.CUDAGraph()
    with torch.no_grad():
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s), torch.autocast("cuda", dtype=torch.bfloat16):
            for _ in range(3):
                out = tm(static).argmax(1)
        torch.cuda.current_stream().wait_stream(s)
        with torch.cuda.graph(g), torch.autocast("cuda", dtype=torch.bfloat16):
            out = tm(static).argmax(1)

    def graphed(x):
        static.copy_(x)
        g.replay()
        return int(out.item())
    emit(bench="resnet50_infer_b1", impl="torch+graph", **run(graphed))


def _text_batch(B=32, S=128):
    from pcmp.data.synthetic import SyntheticIMDB
    ids, mask, y = SyntheticIMDB(B, S).get_batch(list(range(B)), dev)
    return ids, mask, y


def bilstm_train():
    from pcmp.models.bilstm import BiLSTMClassifier, TorchBiLSTM
    ids, mask, y = _text_batch()
    m = BiLSTMClassifier().to(dev)
    t = timeit(hip_train_step(m, lambda: cross_entropy(m.forward_logits(ids), y), "adamw", 1e-3, clip=1.0))
    emit(bench="bilstm_train", impl="hip", samples_s=32 / t, ms=t * 1e3, batch=32)
    tm = TorchBiLSTM().to(dev)
    o = torch.optim.AdamW(tm.parameters(), lr=1e-3)
    t = timeit(torch_train_step(tm, lambda: torch.nn.functional.cross_entropy(tm(ids).float(), y), o))
    emit(bench="bilstm_train", impl="torch", samples_s=32 / t, ms=t * 1e3, batch=32)


def bert_train():
    import transformers
    from pcmp.models.bert import bert_base
    ids, mask, y = _text_batch()
    m = bert_base().to(dev)
    t = timeit(hip_train_step(m, lambda: m(ids, None, mask, y)[0], "adamw", 2e-5, eps=1e-8, clip=1.0))
    emit(bench="bert_train", impl="hip", samples_s=32 / t, ms=t * 1e3, batch=32)
    # the same step replayed from one captured hipGraph (pcmp.engine.graph.GraphedStep)
    from pcmp.engine.graph import GraphedStep
    from pcmp.engine.trainer import make_state
    m2 = bert_base().to(dev)
    st = make_state(m2, "adamw", lr=2e-5, eps=1e-8, clip=1.0)
    g = GraphedStep(st, lambda a, b, c: m2(a, None, b, c)[0], [ids, mask, y])
    t = timeit(lambda: g(ids, mask, y))
    emit(bench="bert_train", impl="hip+hipgraph", samples_s=32 / t, ms=t * 1e3, batch=32)
    if HIP_ONLY:
        return
    hf = transformers.BertForSequenceClassification(transformers.BertConfig(num_labels=2)).to(dev)
    o = torch.optim.AdamW(hf.parameters(), lr=2e-5, eps=1e-8, fused=True)

    def step():
        o.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            loss = hf(ids, attention_mask=mask, labels=y).loss
        loss.backward()
        torch.nn.utils.clip_grad_norm_(hf.parameters(), 1.0)
        o.step()
    t = timeit(step)
    emit(bench="bert_train", impl="torch(HF)", samples_s=32 / t, ms=t * 1e3, batch=32)


if __name__ == "__main__":
    names = sys.argv[1:] or ["resnet18_train", "resnet50_tl_train", "resnet50_infer", "bilstm_train", "bert_train"]
    for n in names:
        try:
            globals()[n]()
        except Exception as e:  # keep going; report the failure
            emit(bench=n, error=repr(e)[:500])

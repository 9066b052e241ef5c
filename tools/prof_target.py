"""Run N training steps of one secondary workload (for rocprofv3):
python tools/prof_target.py bert|bert_graph|bilstm|resnet18|resnet50_f32_tl [steps]
(bert_graph: GraphedStep replays; resnet50_f32_tl: the reference-precision transfer-learning forward,
fp32, train-mode BatchNorm, batch 64 at 224^2, no gradient through the frozen backbone)"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import pcmp  # noqa: E402,F401
from pcmp.ops import cross_entropy  # noqa: E402

dev = torch.device("cuda")
what = sys.argv[1] if len(sys.argv) > 1 else "bert"
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 13
from pcmp.engine.trainer import make_state  # noqa: E402
from pcmp.data.synthetic import SyntheticIMDB  # noqa: E402

if what in ("bert", "bert_graph", "bilstm"):
    ids, mask, y = SyntheticIMDB(32, 128).get_batch(list(range(32)), dev)
    if what in ("bert", "bert_graph"):
        from pcmp.models.bert import bert_base
        m = bert_base().to(dev)
        st = make_state(m, "adamw", lr=2e-5, eps=1e-8, clip=1.0)
        loss_fn = lambda: m(ids, None, mask, y)[0]  # noqa: E731
    else:
        from pcmp.models.bilstm import BiLSTMClassifier
        m = BiLSTMClassifier().to(dev)
        st = make_state(m, "adamw", lr=1e-3, clip=1.0)
        loss_fn = lambda: cross_entropy(m.forward_logits(ids), y)  # noqa: E731
elif what == "resnet50_f32_tl":
    from pcmp.models.resnet import resnet50
    from pcmp.ops import _lib
    _lib.set_precision("fp32")
    m = resnet50(10).to(dev).train()
    x = torch.rand(64, 3, 224, 224, device=dev)
    with torch.no_grad():
        for _ in range(steps):
            m.forward_logits(x)
    torch.cuda.synchronize()
    print("done", what, steps)
    sys.exit(0)
else:
    from pcmp.models.resnet import resnet18
    m = resnet18(1000).to(dev)
    x = torch.rand(256, 3, 224, 224, device=dev)
    y = torch.randint(0, 1000, (256,), device=dev)
    st = make_state(m, "sgd", lr=0.1, momentum=0.9)
    loss_fn = lambda: cross_entropy(m.forward_logits(x), y)  # noqa: E731
if what == "bert_graph":
    from pcmp.engine.graph import GraphedStep
    for _ in range(4):
        st.zero_grad()
        st.backward_step(loss_fn())
    g = GraphedStep(st, lambda a, b, c: m(a, None, b, c)[0], [ids, mask, y])
    for _ in range(steps):
        g(ids, mask, y)
else:
    for _ in range(steps):
        st.zero_grad()
        st.backward_step(loss_fn())
torch.cuda.synchronize()
print("done", what, steps)

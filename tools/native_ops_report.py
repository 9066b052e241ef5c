"""List the non-pcmp (at::native / runtime) GPU kernels of one training step and the Python line
that issued each: torch.profiler over one steady-state step of BERT-base (B=32, S=128, AdamW +
clip) or ResNet-50, kernels grouped by (name, issuing pcmp/model source line).

Usage: python tools/native_ops_report.py [bert|resnet50]
"""
import collections
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pcmp  # noqa: E402,F401


def bert_step():
    from pcmp.data.synthetic import SyntheticIMDB
    from pcmp.engine.trainer import make_state
    from pcmp.models.bert import bert_base
    dev = torch.device("cuda", 0)
    ids, mask, y = SyntheticIMDB(32, 128).get_batch(list(range(32)), dev)
    m = bert_base().to(dev)
    st = make_state(m, "adamw", lr=2e-5, eps=1e-8, clip=1.0)

    def step():
        st.zero_grad()
        st.backward_step(m(ids, None, mask, y)[0])
    return step


def resnet50_step():
    from pcmp.engine.trainer import make_state
    from pcmp.models.resnet import resnet50
    from pcmp.ops import cross_entropy
    dev = torch.device("cuda", 0)
    x = torch.rand(256, 3, 224, 224, device=dev)
    y = torch.randint(0, 1000, (256,), device=dev)
    m = resnet50(1000).to(dev).train()
    st = make_state(m, "sgd", lr=0.02, momentum=0.9)

    def step():
        st.zero_grad()
        st.backward_step(cross_entropy(m.forward_logits(x), y))
    return step


def main():
    which = sys.argv[1] if len(sys.argv) > 1 else "bert"
    step = bert_step() if which == "bert" else resnet50_step()
    for _ in range(4):
        step()
    torch.cuda.synchronize()
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof:
        step()
        torch.cuda.synchronize()
    evs = prof.events()
    total = sum(1 for e in evs if e.device_type.name == "CUDA" and "pcmp" not in e.name)
    # walk the leaf-most aten ops and the non-pcmp kernels each launched
    lines = collections.Counter()
    for e in evs:
        if e.device_type.name != "CPU":
            continue
        kern = [k for k in e.kernels if "pcmp" not in k.name] if hasattr(e, "kernels") else []
        if not kern or not e.name.startswith("aten::"):
            continue
        # only leaf-most aten ops (children launch nothing themselves)
        if any(getattr(ch, "kernels", None) for ch in e.cpu_children):
            continue
        # the leaf op often carries no Python stack: walk up to the first ancestor that has one
        # (and name the ancestor op chain, e.g. aten::zeros > aten::zero_ > aten::fill_)
        anc, chain = e, []
        while anc is not None and not anc.stack:
            chain.append(anc.name)
            anc = anc.cpu_parent
        stack = anc.stack if anc is not None else []
        frames = [f for f in stack if "pcmp" in f or "counterparts_amd" in f or "tools/" in f]
        where = (frames[0] if frames else (stack[0] if stack else "?")) + "  [" + " < ".join(chain[:4]) + "]"
        for k in kern:
            lines[(e.name, k.name[:60], where[-110:])] += 1
    print(f"non-pcmp GPU kernels in one {which} step:")
    for (op, kn, where), n in sorted(lines.items(), key=lambda kv: -kv[1]):
        print(f"  {n:3d}x  {op:28s} {kn:60s}  <- {where}")
    print("non-pcmp GPU kernel events:", total)


if __name__ == "__main__":
    main()

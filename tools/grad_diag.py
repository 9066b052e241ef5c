"""Gradient agreement of the HIP bf16 path, the PyTorch-reference bf16 path (pcmp.ops.ref on GPU)
and stock torch autocast-bf16, each against an fp32 torch.nn ResNet-50 with identical weights."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch, pcmp
from pcmp.ops import _lib, cross_entropy
from pcmp.models.resnet import resnet50
from pcmp.models.torch_ref import TorchResNet
torch.manual_seed(0)
dev = torch.device("cuda")
arch = os.environ.get("ARCH", "resnet50")
from pcmp.models import resnet as R
m = getattr(R, arch)(num_classes=1000).to(dev).train()
B = int(os.environ.get("B", "32")); S = int(os.environ.get("S", "224"))
x = torch.rand(B, 3, S, S, device=dev); y = torch.randint(0, 1000, (B,), device=dev)
state = {k: v.clone() for k, v in m.state_dict().items()}

def tname(n):
    n = n.replace("stem.conv.weight", "conv1.weight").replace("stem.conv.gamma", "bn1.weight").replace("stem.conv.beta", "bn1.bias")
    for i in "123":
        n = n.replace(f"conv{i}.gamma", f"bn{i}.weight").replace(f"conv{i}.beta", f"bn{i}.bias")
    n = n.replace("downsample.weight", "downsample.0.weight").replace("downsample.gamma", "downsample.1.weight").replace("downsample.beta", "downsample.1.bias")
    return n

def to_t(n, g):
    if g.dim() == 4: g = g[..., :3].permute(0, 3, 1, 2) if n.startswith("stem") else g.permute(0, 3, 1, 2)
    if n.startswith("fc."): g = g[:1000]
    return g

res = {}
for be in ("hip", "torch"):
    m.load_state_dict(state); _lib.set_backend(be)
    for p in m.parameters(): p.grad = None
    loss = cross_entropy(m.forward_logits(x), y); loss.backward()
    res[be] = (loss.item(), {tname(n): to_t(n, p.grad.float()) for n, p in m.named_parameters()})
_lib.set_backend("hip")
m.load_state_dict(state)
t = TorchResNet(arch, 1000).to(dev).train().load_from_pcmp(m)
tstate = {k: v.clone() for k, v in t.state_dict().items()}
for mode in ("fp32", "autocast"):
    t.load_state_dict(tstate)
    for p in t.parameters(): p.grad = None
    with torch.autocast("cuda", dtype=torch.bfloat16, enabled=(mode == "autocast")):
        out = t(x); loss = torch.nn.functional.cross_entropy(out.float(), y)
    loss.backward()
    res[mode] = (loss.item(), {n: p.grad.float().clone() for n, p in t.named_parameters()})
print({k: round(v[0], 5) for k, v in res.items()})
ref = res["fp32"][1]
def rel(a, b): return ((a - b).norm() / (b.norm() + 1e-20)).item()
print(f"{'param':40s} {'hip':>8s} {'refbf16':>8s} {'autocast':>8s}")
tot = {k: [] for k in ("hip", "torch", "autocast")}
for n in ref:
    row = []
    for k in ("hip", "torch", "autocast"):
        e = rel(res[k][1][n], ref[n]); tot[k].append(e); row.append(e)
    print(f"{n:40s} {row[0]:8.4f} {row[1]:8.4f} {row[2]:8.4f}")
for k, v in tot.items():
    v = sorted(v); print(k, "median", round(v[len(v)//2], 4), "max", round(v[-1], 4))

import os; os.environ["PCMP_TRACE_OPS"]="1"
import sys; sys.path.insert(0,'/root/repo')
import torch, pcmp
from pcmp.ops import kernels, cross_entropy
from pcmp.models.resnet import resnet50
m = resnet50().train()
x = torch.rand(2,3,224,224); y = torch.randint(0,1000,(2,))
loss = cross_entropy(m.forward_logits(x), y); loss.backward()
B=128
import json
conv = []
for name, a in kernels.TRACE:
    if name == "conv_fwd":
        x, w, s, p = a[0], a[1], a[2], a[3]
        N,H,W,C = x; K,R,S,_ = w; P=(H+2*p-R)//s+1; Q=(W+2*p-S)//s+1
        conv.append(("fwd", N*B*P*Q, K, R*S*C, s, R))
    elif name == "conv_dgrad":
        dy, w, H, W, s, p = a[:6]; N,P,Q,K = dy; K,R,S,C = w
        conv.append(("dgrad", N*B*H*W, C, R*S*K, s, R))
    elif name == "conv_wgrad":
        dy, x = a[0], a[1]; R,S,s = a[3], a[4], a[5]; N,P,Q,K = dy; C = x[3]
        conv.append(("wgrad", K, R*S*C, N*B*P*Q, s, R))
json.dump(conv, open('/tmp/convshapes.json','w'))
print(len(conv)); print(conv[:5])

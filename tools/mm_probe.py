import sys, time, torch
sys.path.insert(0, '/root/repo')
import pcmp
from pcmp.ops import _lib
_lib.load()
ops = torch.ops.pcmp
dev = torch.device('cuda')
def bench(fn, iters=20):
    for _ in range(3): fn()
    torch.cuda.synchronize(); t = time.perf_counter()
    for _ in range(iters): fn()
    torch.cuda.synchronize(); return (time.perf_counter() - t) / iters * 1e6
# 1x1 WGRAD shapes: (N,H,W,C,K)
for (N,H,W,C,K) in [(256,56,56,64,256),(256,56,56,256,64),(256,28,28,128,512),(256,28,28,512,128),(256,14,14,256,1024),(256,14,14,1024,256),(256,7,7,512,2048),(256,7,7,2048,512)]:
    M = N*H*W
    x = torch.randn(M, C, device=dev).to(torch.bfloat16)
    dy = torch.randn(M, K, device=dev).to(torch.bfloat16)
    out = torch.empty(K, 1, 1, C, device=dev)
    t_ours = bench(lambda: ops.conv_wgrad(dy.view(N,H,W,K), x.view(N,H,W,C), out, 1, 1, 1, 0, False))
    t_mm = bench(lambda: torch.mm(dy.t(), x))
    # fwd GEMM: y = x @ w^T  (M x C) (C x K)
    w = torch.randn(K, C, device=dev).to(torch.bfloat16)
    t_fwd_ours = bench(lambda: ops.conv_fwd(x.view(N,H,W,C), w.view(K,1,1,C), 1, 0, None, None, False, False))
    t_fwd_mm = bench(lambda: torch.mm(x, w.t()))
    fl = 2.0*M*C*K
    print(f"M={M:7d} C={C:5d} K={K:5d}  wgrad ours {t_ours:7.1f}us  mm {t_mm:7.1f}us | fwd ours {t_fwd_ours:7.1f}us mm {t_fwd_mm:7.1f}us  ({fl/t_fwd_mm/1e6:.0f} TF mm)", flush=True)

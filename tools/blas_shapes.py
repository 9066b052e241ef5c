"""Run torch.mm (hipBLASLt) on the GEMM shapes of tools/gemm_probe.py a few times, for
rocprofv3 --kernel-trace --stats: the kernel names encode hipBLASLt's tile choice (MT, MI, WG)."""
import torch

SHAPES = [(4096, 4096, 4096), (50176, 256, 2304), (200704, 128, 1152), (12544, 512, 4608),
          (4096, 3072, 768), (4096, 768, 3072), (4096, 2304, 768), (50176, 1024, 256), (200704, 64, 576)]
dev = torch.device("cuda")
for M, N, K in SHAPES:
    A = (torch.rand(M, K, device=dev) * 2 - 1).to(torch.bfloat16)
    B = (torch.rand(N, K, device=dev) * 2 - 1).to(torch.bfloat16)
    for _ in range(3):
        C = torch.mm(A, B.t())
    torch.cuda.synchronize()
    print(M, N, K, flush=True)

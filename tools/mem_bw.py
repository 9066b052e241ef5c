"""HBM bandwidth probe: write-only (fill), read-only (sum), copy and 2-read-1-write streams on
1 GiB bf16 buffers (torch kernels), for the roofline floors of write-heavy conv epilogues."""
import json
import torch


def t(fn, iters=20):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / iters * 1e-3


n = 1 << 29   # 512 Mi bf16 = 1 GiB
a = torch.empty(n, dtype=torch.bfloat16, device="cuda")
b = torch.empty(n, dtype=torch.bfloat16, device="cuda")
c = torch.empty(n, dtype=torch.bfloat16, device="cuda")
a.fill_(1.0); b.fill_(2.0)
nb = n * 2
out = torch.empty((), dtype=torch.float32, device="cuda")
r = {
    "write_TBs": nb / t(lambda: c.fill_(3.0)) / 1e12,
    "read_TBs": nb / t(lambda: torch.sum(a, dim=(0,), dtype=torch.float32, out=out)) / 1e12,
    "copy_TBs": 2 * nb / t(lambda: c.copy_(a)) / 1e12,
    "add_2r1w_TBs": 3 * nb / t(lambda: torch.add(a, b, out=c)) / 1e12,
}
print(json.dumps({k: round(v, 2) for k, v in r.items()}))

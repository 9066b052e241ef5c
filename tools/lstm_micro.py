"""LSTM recurrence micro benchmark: lstm_seq_fwd / lstm_seq_bwd at the BiLSTM config (B=32, S=128,
H=256) per knob variant, us per call and per timestep.  python tools/lstm_micro.py [rounds]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import pcmp  # noqa: E402,F401
from pcmp.ops import _lib  # noqa: E402

assert _lib.load(), _lib.load_error()

ops = torch.ops.pcmp
B, S, H = 32, 128, 256
dev = torch.device("cuda")
torch.manual_seed(0)
ids = torch.randint(1, 1000, (B, S), device=dev)
for i in range(B):
    ids[i, max(1, S - (7 * i) % S):] = 0
gx = (torch.randn(B, S, 2, 4 * H, device=dev) * 0.5).to(torch.bfloat16)
whh = (torch.randn(2, 4 * H, H, device=dev) / H ** 0.5).to(torch.bfloat16)
dh = torch.randn(B, S, 2 * H, device=dev).to(torch.bfloat16)


def timeit(fn, n=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / n * 1e3


rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 3
h, g, c, _ = ops.lstm_seq_fwd(gx, whh, ids)
for r in range(rounds):
    for v in (0, 1, 2):   # 2: v2 forward + partial-exchange backward
        ops.set_knob("lstm_v2", v)
        tf = timeit(lambda: ops.lstm_seq_fwd(gx, whh, ids))
        tb = timeit(lambda: ops.lstm_seq_bwd(dh, g, c, whh, ids))
        print(f"round {r} lstm_v2={v}: fwd {tf:7.1f} us ({tf / S:5.2f} us/step)  bwd {tb:7.1f} us ({tb / S:5.2f} us/step)",
              flush=True)

# phase clocks of workgroup 0 (knob lstm_prof): fraction of the step per phase
ops.set_knob("lstm_prof", 1)
for v, name, fn, phases in (
        (1, "fwd", lambda: ops.lstm_seq_fwd(gx, whh, ids)[3], ["poll", "gather", "MFMA", "cell", "publish"]),
        (1, "bwd", lambda: ops.lstm_seq_bwd(dh, g, c, whh, ids)[1],
         ["cell", "publish", "poll", "A loads + MFMA", "reduce+carry"]),
        (2, "bwd v3", lambda: ops.lstm_seq_bwd(dh, g, c, whh, ids)[1],
         ["cell", "MFMA + publish", "poll", "partials gather", "carry"])):
    ops.set_knob("lstm_v2", v)
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    sync = fn()
    b.record()
    torch.cuda.synchronize()
    us = a.elapsed_time(b) * 1e3
    cyc = sync[4:20].cpu().view(torch.int64)[:len(phases)].tolist()
    tot = sum(cyc)
    print(f"{name}: {us:.1f} us, {tot / S:.0f} clocks/step over the phases; per step: " +
          ", ".join(f"{n} {v / tot * us / S:.2f} us" for n, v in zip(phases, cyc)), flush=True)
ops.set_knob("lstm_prof", 0)
ops.set_knob("lstm_v2", 1)

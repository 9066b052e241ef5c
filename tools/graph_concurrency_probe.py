"""Does a replayed hipGraph run independent branches concurrently?  Two spin kernels on forked
streams (torch.cuda._sleep, one workgroup each): eager vs captured+replayed wall time."""
import time

import torch

N = 20_000_000   # cycles per spin kernel


def fork_join():
    main = torch.cuda.current_stream()
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    s1.wait_stream(main)
    s2.wait_stream(main)
    with torch.cuda.stream(s1):
        torch.cuda._sleep(N)
    with torch.cuda.stream(s2):
        torch.cuda._sleep(N)
    main.wait_stream(s1)
    main.wait_stream(s2)


def one():
    torch.cuda._sleep(N)


def t(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e3


single = t(one)
eager = t(fork_join)
g = torch.cuda.CUDAGraph()
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    fork_join()
torch.cuda.current_stream().wait_stream(s)
with torch.cuda.graph(g):
    fork_join()
graph = t(g.replay)
print(f"one spin kernel {single:.2f} ms; two on forked streams: eager {eager:.2f} ms, hipGraph replay {graph:.2f} ms "
      f"({'concurrent' if graph < 1.5 * single else 'SERIALISED'} in the graph)")

#!/usr/bin/env python3
"""Flagship benchmark: ResNet-50 bf16 training throughput (images/sec) on N MI355X GPUs.

Contract (driver): ``python bench.py --gpus N --steps K --warmup W``; for N>1 launched by
``torch.distributed.run`` with one rank per GPU (RCCL over xGMI).  W untimed warm-up steps,
then EXACTLY K timed steps bracketed by barrier + device synchronize on both sides; the step
time is the MAX over ranks; rank 0 prints ONE JSON line.  ``value`` is the whole-job aggregate
(images/sec summed over all GPUs, weak scaling: per-GPU batch fixed).

What a timed step contains (nothing skipped): synthetic Imagenette-shaped batch [B,3,224,224]
fp32 NCHW on device -> fused NCHW->NHWC/bf16 conversion -> full ResNet-50 forward (53 conv+BN,
16 bottlenecks, 1000-way fc) -> fused softmax cross-entropy -> full backward (dgrad + wgrad of
every conv, BN backward) with bucketed RCCL all-reduce overlapped with backward (N>1) -> fused
flat SGD-momentum update of all 25.6 M params (+ bf16 shadow refresh).

``--impl torch`` runs the self-baseline: the same model on stock PyTorch-ROCm (MIOpen convs,
channels_last, bf16 autocast, torch DDP, torch fused SGD).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

BASELINE_IMG_PER_SEC = 1.43  # ResNet-50 TL training throughput (7,576 img / 5314.1 s)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch-size", type=int, default=256, help="per-GPU batch")
    ap.add_argument("--model", default="resnet50")
    ap.add_argument("--impl", default="hip", choices=["hip", "torch"])
    ap.add_argument("--image-size", type=int, default=224)
    ap.add_argument("--num-classes", type=int, default=1000)
    ap.add_argument("--lr", type=float, default=0.1)
    ap.add_argument("--profile", default=None, help="write a torch.profiler chrome trace here")
    ap.add_argument("--sync-bn", action="store_true", help="BatchNorm statistics over all ranks (SyncBN)")
    ap.add_argument("--graph", action="store_true",
                    help="capture the whole training step (forward, backward, optimizer) as one hipGraph "
                         "after warm-up and replay it (hip impl, one rank)")
    ap.add_argument("--local_rank", "--local-rank", type=int, default=None)
    return ap.parse_args()


def graph_step(step, x, y):
    """Capture one full training step into a hipGraph (static x / y / parameters / optimizer state)
    and return a replay function.  Autotuning is finished by then (warm-up) and never runs while a
    graph is captured; the WGRAD / downsample side stream joins the capture through events."""
    main = torch.cuda.current_stream()
    s = torch.cuda.Stream()
    s.wait_stream(main)
    with torch.cuda.stream(s):
        for _ in range(2):
            step(x, y)
    main.wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        loss = step(x, y)

    def replay(x_, y_):
        assert x_ is x and y_ is y, "graph replay needs the captured input tensors"
        g.replay()
        return loss

    return replay


def build_hip(args, env):
    import pcmp
    from pcmp.models import resnet
    from pcmp.optim import SGD
    from pcmp.ops import cross_entropy
    from pcmp.parallel.ddp import DistributedDataParallel
    from pcmp.utils.flat import FlatParams
    from pcmp.utils.misc import StepThrottle

    torch.manual_seed(1234)
    model = getattr(resnet, args.model)(num_classes=args.num_classes).to(env.device).train()
    if getattr(args, "sync_bn", False) and env.world_size > 1:
        from pcmp.parallel.ddp import convert_sync_batchnorm
        convert_sync_batchnorm(model)
    flat = FlatParams(model.parameters())
    opt = SGD(flat, lr=args.lr, momentum=0.9, weight_decay=5e-5)
    ddp = DistributedDataParallel(model, flat) if env.world_size > 1 else None
    if ddp is not None:
        opt.set_grad_scale(ddp.grad_scale())

    # host run-ahead bound (PCMP_MAX_INFLIGHT steps): keeps the caching allocator's footprint at a
    # few steps' worth instead of growing with every step the host gets ahead of the GPU
    throttle = StepThrottle(env.device)

    def step(x, y):
        opt.zero_grad()
        logits = model.forward_logits(x)
        loss = cross_entropy(logits, y)
        loss.backward()
        if ddp is not None:
            ddp.finish_gradient_sync()
        opt.step()
        throttle.tick()
        return loss

    return step


def build_torch(args, env):
    import pcmp  # noqa: F401
    from pcmp.models.torch_ref import TorchResNet

    torch.manual_seed(1234)
    model = TorchResNet(args.model, args.num_classes).to(env.device).to(memory_format=torch.channels_last).train()
    if getattr(args, "sync_bn", False) and env.world_size > 1:
        model = torch.nn.SyncBatchNorm.convert_sync_batchnorm(model)
    if env.world_size > 1:
        model = torch.nn.parallel.DistributedDataParallel(model, device_ids=[env.local_rank], bucket_cap_mb=32)
    opt = torch.optim.SGD(model.parameters(), lr=args.lr, momentum=0.9, weight_decay=5e-5, fused=True)
    crit = torch.nn.CrossEntropyLoss()

    def step(x, y):
        opt.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            out = model(x.contiguous(memory_format=torch.channels_last))
            loss = crit(out.float(), y)
        loss.backward()
        opt.step()
        return loss

    return step


def main():
    args = parse()
    import pcmp
    from pcmp.parallel import launch

    env = launch.init(args.local_rank)
    if env.world_size != args.gpus and env.is_main:
        print(f"[bench] note: --gpus {args.gpus} but WORLD_SIZE={env.world_size}", file=sys.stderr)
    if env.device.type == "cuda":
        torch.backends.cudnn.benchmark = True
    B = args.batch_size
    g = torch.Generator(device=env.device).manual_seed(17 + env.rank)
    x = torch.rand(B, 3, args.image_size, args.image_size, device=env.device, generator=g)
    y = torch.randint(0, args.num_classes, (B,), device=env.device, generator=g)

    step = build_hip(args, env) if args.impl == "hip" else build_torch(args, env)

    def sync():
        if env.device.type == "cuda":
            torch.cuda.synchronize()
        launch.barrier()
        if env.device.type == "cuda":
            torch.cuda.synchronize()

    for i in range(args.warmup):
        loss = step(x, y)
    graphed = bool(args.graph and args.impl == "hip" and env.world_size == 1 and env.device.type == "cuda")
    if graphed:
        step = graph_step(step, x, y)
        loss = step(x, y)
    sync()
    prof = None
    if args.profile and env.is_main:
        prof = torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CPU,
                                                  torch.profiler.ProfilerActivity.CUDA])
        prof.__enter__()
    t0 = time.perf_counter()
    for i in range(args.steps):
        loss = step(x, y)
    sync()
    dt = time.perf_counter() - t0
    if prof is not None:
        prof.__exit__(None, None, None)
        prof.export_chrome_trace(args.profile)
    t = torch.tensor([dt], dtype=torch.float64, device=env.device)
    if env.world_size > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dt = float(t.item())
    ms = dt / args.steps * 1e3
    img_s = B * env.world_size * args.steps / dt
    final_loss = float(loss.float().item())
    if os.environ.get("PCMP_MEMSTATS") == "1" and env.device.type == "cuda" and env.is_main:
        ms_ = torch.cuda.memory_stats(env.device)
        print(f"[bench] mem peak {ms_.get('allocated_bytes.all.peak', 0) / 2**30:.1f} GiB reserved "
              f"{ms_.get('reserved_bytes.all.peak', 0) / 2**30:.1f} GiB alloc_retries "
              f"{ms_.get('num_alloc_retries', 0)} device_allocs {ms_.get('num_device_alloc', 0)} "
              f"device_frees {ms_.get('num_device_free', 0)}", file=sys.stderr, flush=True)
    if env.is_main:
        rec = {
            "metric": "resnet50_train_images_per_sec" if args.model == "resnet50" else f"{args.model}_train_images_per_sec",
            "value": round(img_s, 2),
            "unit": "images/s",
            "n_gpus": env.world_size,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": round(img_s / BASELINE_IMG_PER_SEC, 1),
            "dtype": "bf16",
            "data": "synthetic",
            "config": {"model": args.model, "global_batch": B * env.world_size, "per_gpu_batch": B,
                       "image_size": args.image_size, "num_classes": args.num_classes,
                       "seq_len": None, "parallelism": f"dp{env.world_size}", "impl": args.impl,
                       "optimizer": "sgd_momentum", "final_loss": round(final_loss, 4),
                       "hipgraph": graphed},
        }
        print(json.dumps(rec), flush=True)
    launch.shutdown()


if __name__ == "__main__":
    main()

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

After the timed region (outside it) every rank also measures ResNet-50 batch-1 inference latency
on the trained model (eval mode, BN folded, whole forward replayed from one hipGraph, per image:
H2D copy of a host image + replay + argmax + D2H index, the reference's predict_image contract,
SURVEY E1) and rank 0 reports ``inference_p50_ms`` / ``inference_p99_ms`` — the second half of
BASELINE.json's metric.  ``--infer-images 0`` skips it.

``--ddp-force`` initialises the ``nccl`` (RCCL) process group and issues every gradient bucket's
all-reduce even at one rank, so the multi-GPU communication path runs on a one-GPU box;
``--grad-dtype bf16`` all-reduces bf16 gradient copies (half the xGMI bytes).

``--gpus N`` without a launcher (no ``WORLD_SIZE`` in the environment) starts ``torch.distributed.run``
with N ranks as a CHILD process before anything touches the GPU, waits for it and exits with its
status: a ``--gpus 8`` run never reports a one-GPU number.  Under a launcher, ``--gpus`` must equal
``WORLD_SIZE`` or the run fails.  The JSON line proves the communicator's size (``comm.world_check``
= an all-reduce of ones over the process group) and reports the gradient buckets and the exposed
(non-overlapped) all-reduce time per step (``comm.exposed_ms``: from the compute stream reaching
the end of backward to the last bucket's collective and optimizer update finishing, CUDA events,
mean over 4 instrumented steps run AFTER the timed loop -- the timing events cost step time).

The learning rate ramps linearly over the warm-up steps to ``--lr`` and stays constant in the timed
steps (no per-step host work in the timed region); ``final_loss`` (the loss of the last timed step on
the fixed synthetic batch) then sits below ln(num_classes), a cheap numerics sanity signal.

``vs_baseline`` is null: the reference publishes no full-network training number (its only
training figure, BASELINE.md P1a = 1.43 img/s, is frozen-backbone transfer learning on a CPU
Colab runtime), so no like-for-like ratio exists.  The stock PyTorch-ROCm self-baseline of the same
step (MIOpen, ``--impl torch``) is a builder-measured figure in BASELINE.md, not part of this line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
# before the HIP runtime initialises: importing pcmp raises GPU_MAX_HW_QUEUES to >= 8, one hardware
# queue per stream (compute, WGRAD side, DDP comm, RCCL) instead of the pool's exported 4 shared
# round-robin (pcmp/__init__.py)
import pcmp  # noqa: E402,F401

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


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
    ap.add_argument("--lr", type=float, default=0.02,
                    help="peak SGD lr, reached by a linear ramp over the warm-up steps")
    ap.add_argument("--profile", default=None, help="write a torch.profiler chrome trace here")
    ap.add_argument("--sync-bn", action="store_true", help="BatchNorm statistics over all ranks (SyncBN)")
    ap.add_argument("--graph", action="store_true",
                    help="capture the whole training step (forward, backward, optimizer) as one hipGraph "
                         "after warm-up and replay it (hip impl, one rank)")
    ap.add_argument("--ddp-force", action="store_true",
                    help="RCCL process group + bucket all-reduces even at one rank (exercises the comm path)")
    ap.add_argument("--opt-after-join", action="store_true",
                    help="DDP: one whole-arena SGD update after the last all-reduce instead of the per-bucket "
                         "update as each all-reduce completes (the A/B baseline of the per-bucket optimizer)")
    ap.add_argument("--grad-dtype", default=None, choices=["fp32", "bf16"],
                    help="gradient all-reduce dtype (default fp32, exact)")
    ap.add_argument("--infer-images", type=int, default=200,
                    help="batch-1 inference latency images measured after the timed loop (0 = skip)")
    ap.add_argument("--watchdog", type=float, default=None,
                    help="abort (exit 3) if a step makes no progress for this many seconds (0 = off; "
                         "default 300 when N > 1, so a hung collective fails the job promptly "
                         "instead of waiting out the 600 s RCCL timeout; off at N = 1)")
    ap.add_argument("--master-port", type=int, default=0, help="self-launch rendezvous port (0 = pick a free one)")
    ap.add_argument("--local_rank", "--local-rank", type=int, default=None)
    return ap.parse_args()


def _free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def self_launch(args) -> int | None:
    """``--gpus N`` (N > 1) with no launcher environment: run this script under
    ``torch.distributed.run`` with N ranks as a child process and return its exit status.  Must run
    before anything initialises the HIP runtime (no exec from a GPU-initialised process)."""
    if args.gpus <= 1 or "WORLD_SIZE" in os.environ or "LOCAL_RANK" in os.environ:
        return None
    import subprocess
    port = args.master_port or _free_port()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__), *sys.argv[1:]]
    print(f"[bench] --gpus {args.gpus} without a launcher: starting {args.gpus} ranks under torch.distributed.run "
          f"(127.0.0.1:{port})", file=sys.stderr, flush=True)
    return subprocess.call(cmd)


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
    # thread-local capture: the RCCL watchdog thread's event queries must not break it
    with torch.cuda.graph(g, capture_error_mode="thread_local"):
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
    use_ddp = env.world_size > 1 or (args.ddp_force and env.backend is not None)
    ddp = DistributedDataParallel(model, flat, force=args.ddp_force, grad_dtype=args.grad_dtype) if use_ddp else None
    if ddp is not None and args.opt_after_join:
        opt.set_grad_scale(ddp.grad_scale())

    # host run-ahead bound (PCMP_MAX_INFLIGHT steps): keeps the caching allocator's footprint at a
    # few steps' worth instead of growing with every step the host gets ahead of the GPU
    throttle = StepThrottle(env.device)

    # the step's compute stream runs at high queue priority, so the command processor dispatches its
    # critical-path (DGRAD / BN chain) workgroups ahead of the WGRAD side stream's when CUs free up:
    # 12,213-12,283 -> 12,392-12,409 img/s in 3 interleaved rounds (profiles/r3_prio_pf2_ab.txt);
    # PCMP_STEP_PRIO=0 runs it on the default stream
    # PriorityStream.step orders the step after the caller's stream (set_lr's device write, the
    # input batch) and the caller's stream after the step, every step; it stays on the capturing
    # stream during a hipGraph capture (--graph), so the captured graph holds the whole step
    from pcmp.utils.misc import PriorityStream
    prio = PriorityStream(env.device)

    def step_body(x, y):
        opt.zero_grad()
        logits = model.forward_logits(x)
        loss = cross_entropy(logits, y)
        loss.backward()
        if ddp is not None and not args.opt_after_join:
            ddp.finish_gradient_sync(opt=opt)   # per-bucket SGD as each all-reduce completes
        else:
            if ddp is not None:
                ddp.finish_gradient_sync()
            opt.step()
        throttle.tick()
        return loss

    def step(x, y):
        with prio.step(x, y):
            return step_body(x, y)

    step.model = model
    step.ddp = ddp
    step.opt = opt
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


def batch1_latency(model, args, env):
    """Per-image batch-1 latency of the trained model (outside the timed training region)."""
    from pcmp.engine.inference import Batch1Predictor
    from pcmp.utils.report import latency_stats

    n = args.infer_images
    # host images in pinned (page-locked) memory, as a serving input queue / DataLoader(pin_memory=True)
    # would hold them: the per-image H2D copy is then a direct DMA (20 vs 35 us for a 224^2 fp32 image,
    # profiles/r2_infer_plan_ab.txt)
    imgs = torch.rand(n, 3, args.image_size, args.image_size, generator=torch.Generator().manual_seed(5)).pin_memory()
    torch.cuda.synchronize()
    pred = Batch1Predictor(model, imgs[:1].to(env.device), use_graph=True)
    for i in range(min(20, n)):
        pred(imgs[i:i + 1])
    lat = []
    for i in range(n):
        ts = time.perf_counter()
        pred(imgs[i:i + 1])
        lat.append(time.perf_counter() - ts)
    model.train()
    return latency_stats(lat)


def main():
    args = parse()
    rc = self_launch(args)
    if rc is not None:
        sys.exit(rc)
    import pcmp
    from pcmp.parallel import launch
    from pcmp.utils.misc import Watchdog

    env = launch.init(args.local_rank, force_init=args.ddp_force)
    if env.world_size != args.gpus:
        raise SystemExit(f"[bench] --gpus {args.gpus} but the job has WORLD_SIZE={env.world_size} ranks: refusing to "
                         f"report a {env.world_size}-rank number as {args.gpus} GPUs")
    if args.watchdog is None:
        args.watchdog = 300.0 if env.world_size > 1 else 0.0
    wd = Watchdog(args.watchdog, abort=True).start() if args.watchdog > 0 else None
    # the communicator really spans WORLD_SIZE ranks: all-reduce of ones over the process group
    world_check = 1
    if dist.is_initialized():
        one = torch.ones(1, device=env.device)
        dist.all_reduce(one)
        world_check = int(one.item())
    if env.device.type == "cuda":
        torch.backends.cudnn.benchmark = True
    B = args.batch_size
    g = torch.Generator(device=env.device).manual_seed(17 + env.rank)
    x = torch.rand(B, 3, args.image_size, args.image_size, device=env.device, generator=g)
    y = torch.randint(0, args.num_classes, (B,), device=env.device, generator=g)

    step = build_hip(args, env) if args.impl == "hip" else build_torch(args, env)
    hip_model = getattr(step, "model", None)

    def sync():
        if env.device.type == "cuda":
            torch.cuda.synchronize()
        launch.barrier()
        if env.device.type == "cuda":
            torch.cuda.synchronize()

    opt = getattr(step, "opt", None)
    ddp = getattr(step, "ddp", None)
    ramp = max(1, args.warmup)
    for i in range(args.warmup):
        if opt is not None:
            opt.set_lr(args.lr * (i + 1) / ramp)
        loss = step(x, y)
        if wd is not None:
            wd.kick(i, "warmup")
    if env.world_size > 1:
        # every shape is planned by now: all ranks take rank 0's autotuned kernels
        from pcmp.parallel.ddp import sync_autotune
        sync_autotune()
    if opt is not None:
        opt.set_lr(args.lr)
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
        if wd is not None:
            wd.kick(args.warmup + i, "timed")
    sync()
    dt = time.perf_counter() - t0
    comm = {"backend": env.backend, "world_check": world_check}
    if ddp is not None and not graphed:
        # the exposed-communication / per-bucket timeline instrumentation (timing events on the
        # compute, comm and timeline streams) runs on extra steps AFTER the timed loop: inside it,
        # it slowed the forced-RCCL step 18.6 -> 28.0 ms (profiles/r6_rccl_steps.txt)
        ddp.time_exposed(True)
        for _ in range(4):
            step(x, y)           # final_loss stays the last TIMED step's
        sync()
        comm.update(ddp.comm_report())
        comm["comm_timing_steps"] = "4 extra steps after the timed loop"
        ddp.time_exposed(False)
    if prof is not None:
        prof.__exit__(None, None, None)
        prof.export_chrome_trace(args.profile)
    # per-rank spread (a straggler shows here); the reported step time is the MAX over ranks
    from pcmp.parallel.ddp import step_time_spread
    spread = step_time_spread(dt)
    comm["rank_ms_per_step"] = {"min": round(spread["min_s"] / args.steps * 1e3, 3),
                                "max": round(spread["max_s"] / args.steps * 1e3, 3),
                                "slowest_rank": spread["slowest_rank"]}
    dt = spread["max_s"]
    infer = None
    if args.infer_images > 0 and hip_model is not None and env.device.type == "cuda":
        infer = batch1_latency(hip_model, args, env)
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
            "vs_baseline": None,
            "dtype": "bf16" if (env.device.type == "cuda" or args.impl == "torch") else "fp32",
            "data": "synthetic",
            "config": {"model": args.model, "global_batch": B * env.world_size, "per_gpu_batch": B,
                       "image_size": args.image_size, "num_classes": args.num_classes,
                       "seq_len": None, "parallelism": f"dp{env.world_size}", "impl": args.impl,
                       "optimizer": "sgd_momentum", "final_loss": round(final_loss, 4),
                       "hipgraph": graphed, "ddp_force": bool(args.ddp_force),
                       "grad_allreduce_dtype": args.grad_dtype or "fp32", "lr": args.lr,
                       "lr_warmup_steps": ramp if opt is not None else 0},
            "comm": comm,
        }
        if infer is not None:
            rec["inference_p50_ms"] = round(infer["p50_ms"], 4)
            rec["inference_p99_ms"] = round(infer["p99_ms"], 4)
            rec["inference_config"] = {"model": args.model, "batch": 1, "image_size": args.image_size,
                                       "images": infer["n"], "hipgraph": True, "bn_folded": True,
                                       "host_input": "pinned", "conv_plan": "autotuned small-M",
                                       "per_image": "h2d copy + graph replay + argmax + d2h index"}
        print(json.dumps(rec), flush=True)
    if wd is not None:
        wd.stop()
    launch.shutdown()


if __name__ == "__main__":
    main()

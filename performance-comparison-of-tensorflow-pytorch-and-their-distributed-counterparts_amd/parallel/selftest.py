"""Multi-process DDP self-tests (CPU/gloo or GPU/RCCL) used by tests/ and tools/.

``ddp_equivalence_worker``: every rank trains the same model on its shard of a global batch with
the framework's flat-bucket DDP; the gradient after all-reduce averaging must equal the
single-process gradient on the concatenated batch, and parameters must stay identical across
ranks after several optimizer steps ("DDP grads == single-process grads on the
concatenated batch").
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist


def _build(kind, seed=0):
    torch.manual_seed(seed)
    if kind == "mlp":
        from ..models.layers import MLPHead
        return MLPHead(64, 128, 5, p=0.0)
    if kind == "bilstm":
        from ..models.bilstm import BiLSTMClassifier
        return BiLSTMClassifier(300, 32, 32, 1, 2, 0.0)
    if kind == "resnet_syncbn":
        from ..models.resnet import resnet18
        return resnet18(num_classes=10)
    raise ValueError(kind)


def _batch(kind, n, seed=1):
    g = torch.Generator().manual_seed(seed)
    if kind == "mlp":
        return torch.randn(n, 64, generator=g), torch.randint(0, 5, (n,), generator=g)
    if kind == "resnet_syncbn":
        return torch.rand(n, 3, 32, 32, generator=g), torch.randint(0, 10, (n,), generator=g)
    ids = torch.randint(1, 300, (n, 10), generator=g)
    ids[::3, 6:] = 0
    return ids, torch.randint(0, 2, (n,), generator=g)


def _loss(model, kind, x, y):
    from ..ops import cross_entropy
    return cross_entropy(model.forward_logits(x), y)


def ddp_equivalence_worker(rank, world, port, out_dir, kind="mlp", bucket_mb=0.01, device="cpu", grad_dtype=None):
    """``device='cuda'``: every rank runs the HIP kernels on cuda:0 (one-GPU rehearsal) and the
    gradient buckets are CUDA tensors all-reduced by gloo; tolerances cover bf16 compute."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from .. import optim
    from ..utils.flat import FlatParams
    from .ddp import DistributedDataParallel
    dev = torch.device(device)
    if dev.type == "cuda":
        torch.cuda.set_device(0)
    model = _build(kind, seed=rank).to(dev)      # different init per rank: DDP must broadcast rank 0's
    if kind == "resnet_syncbn":
        # BN statistics over both shards == the single-process full batch: gradients match exactly
        from .ddp import convert_sync_batchnorm
        convert_sync_batchnorm(model)
    flat = FlatParams(model.parameters(), shadow_dtype=None if dev.type == "cpu" else torch.bfloat16)
    ddp = DistributedDataParallel(model, flat, bucket_cap_mb=bucket_mb, first_bucket_mb=bucket_mb / 4,
                                  grad_dtype=grad_dtype)
    opt = optim.SGD(flat, lr=0.05, momentum=0.9)
    opt.set_grad_scale(ddp.grad_scale())
    N = 8 * world
    x, y = _batch(kind, N)
    x, y = x.to(dev), y.to(dev)
    if dev.type == "cuda" and x.is_floating_point() and kind != "resnet_syncbn":
        x = x.to(torch.bfloat16)                 # GPU activations are bf16 (ResNet converts its fp32 images)
    shard = slice(rank * 8, (rank + 1) * 8)
    # reference: single-process gradient on the full batch with rank 0's initial weights
    ref = _build(kind, seed=0).to(dev)
    rflat = FlatParams(ref.parameters(), shadow_dtype=flat.shadow.dtype if flat.shadow is not None else None)
    rflat.zero_grad()
    _loss(ref, kind, x, y).backward()
    ref_grad = rflat.grad.clone()
    opt.zero_grad()
    _loss(model, kind, x[shard], y[shard]).backward()
    ddp.finish_gradient_sync()
    avg = flat.grad * ddp.grad_scale()
    if grad_dtype == "bf16":     # bf16 all-reduce: each rank's shard gradient rounded to 8 mantissa bits
        ok_grad = bool((avg - ref_grad).norm() <= 2e-2 * ref_grad.norm() + 1e-6)
    elif dev.type == "cpu" and kind == "resnet_syncbn":   # deep net: compare relative to the gradient norm
        ok_grad = bool((avg - ref_grad).norm() <= 1e-4 * ref_grad.norm())
    elif dev.type == "cpu":
        ok_grad = torch.allclose(avg, ref_grad, atol=1e-5, rtol=1e-4)
    else:   # bf16 compute: compare at the bf16 noise level relative to the gradient norm
        ok_grad = bool((avg - ref_grad).norm() <= 2e-2 * ref_grad.norm() + 1e-6)
    for _ in range(3):
        opt.step()
        opt.zero_grad()
        _loss(model, kind, x[shard], y[shard]).backward()
        ddp.finish_gradient_sync()
    gathered = [torch.zeros_like(flat.master) for _ in range(world)]
    dist.all_gather(gathered, flat.master)
    ok_sync = all(torch.equal(gathered[0], g) for g in gathered)
    if kind == "resnet_syncbn":   # SyncBN: identical running statistics on every rank
        rm = torch.cat([b.flatten().float() for n_, b in model.named_buffers() if "running" in n_])
        grm = [torch.zeros_like(rm) for _ in range(world)]
        dist.all_gather(grm, rm)
        ok_sync = ok_sync and all(torch.equal(grm[0], g) for g in grm)
    torch.save({"ok_grad": ok_grad, "ok_sync": ok_sync, "nbuckets": len(ddp.buckets),
                "maxdiff": float((avg - ref_grad).abs().max())}, os.path.join(out_dir, f"rank{rank}.pt"))
    if dev.type == "cuda":
        torch.cuda.synchronize()
    dist.destroy_process_group()


def per_bucket_opt_worker(rank, world, port, out_dir, opt_name="sgd", clip=None, kind="bilstm", bucket_mb=0.01):
    """The optimizer issued per bucket inside ``finish_gradient_sync(opt=...)`` against the same
    model trained with the join + ONE whole-arena update (``opt.step()``): with plain updates the
    parameters must be bitwise equal after several steps (the same elementwise kernel over
    sub-ranges); with global-norm clipping (two-phase sum of squares) equal to fp32 rounding of the
    coefficient.  ``kind='bilstm'`` at ``bucket_mb=0.01`` also splits the embedding table (the
    largest parameter) into several bucket chunks."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from .. import optim
    from ..utils.flat import FlatParams
    from .ddp import DistributedDataParallel
    x, y = _batch(kind, 8 * world)
    shard = slice(rank * 8, (rank + 1) * 8)
    masters, nchunks = [], 0
    for per_bucket in (False, True):
        model = _build(kind, seed=rank)
        flat = FlatParams(model.parameters(), shadow_dtype=None)
        ddp = DistributedDataParallel(model, flat, bucket_cap_mb=bucket_mb, first_bucket_mb=bucket_mb / 4,
                                      last_bucket_mb=bucket_mb / 4, split_param_mb=bucket_mb)
        nchunks = max(len(v) for v in ddp._bucket_of.values())
        kw = {"momentum": 0.9} if opt_name == "sgd" else {"weight_decay": 0.01}
        opt = optim.build(opt_name, flat, lr=0.05 if opt_name == "sgd" else 1e-3, **kw)
        for _ in range(3):
            opt.zero_grad()
            _loss(model, kind, x[shard], y[shard]).backward()
            if per_bucket:
                ddp.finish_gradient_sync(opt=opt, clip=clip)
            else:
                ddp.finish_gradient_sync()
                sc = ddp.grad_scale()
                if clip is not None:
                    opt.clip_grad_norm(clip, pre_scale=sc, post_scale=sc)
                else:
                    opt.set_grad_scale(sc)
                opt.step()
        masters.append(flat.master.clone())
    a, b = masters
    torch.save({"bitwise": bool(torch.equal(a, b)), "maxdiff": float((a - b).abs().max()),
                "scale": float(a.abs().max()), "nchunks": nchunks},
               os.path.join(out_dir, f"pb{rank}.pt"))
    dist.destroy_process_group()


def bucket_timeline_worker(rank, world, port, out, device="cpu"):
    """Two-step data-parallel run with the per-bucket timeline on (tests/test_ddp_cpu.py,
    tests/test_ddp_gpu.py): saves comm_report() plus whether average_buffers() made the per-rank
    BatchNorm running means equal to their mean.  ``device='cuda'``: both ranks share cuda:0 and
    all-reduce CUDA buckets over gloo (the one-GPU rehearsal of the comm-stream overlap)."""
    from .. import optim
    from ..utils.flat import FlatParams
    from .ddp import DistributedDataParallel
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device(device)
    if dev.type == "cuda":
        torch.cuda.set_device(0)
    model = _build("resnet_syncbn", seed=rank).to(dev)      # plain per-rank BatchNorm (no SyncBN)
    flat = FlatParams(model.parameters(), shadow_dtype=None if dev.type == "cpu" else torch.bfloat16)
    ddp = DistributedDataParallel(model, flat, bucket_cap_mb=1.0, first_bucket_mb=0.25, last_bucket_mb=0.25)
    opt = optim.SGD(flat, lr=0.01)
    opt.set_grad_scale(ddp.grad_scale())
    x, y = _batch("resnet_syncbn", 8, seed=10 + rank)       # different data per rank
    x, y = x.to(dev), y.to(dev)
    ddp.time_exposed(True)
    for _ in range(2):
        opt.zero_grad()
        _loss(model, "resnet_syncbn", x, y).backward()
        ddp.finish_gradient_sync()
        opt.step()
    rep = ddp.comm_report()
    rm = [b.detach().cpu().clone() for n_, b in model.named_buffers() if "running_mean" in n_]
    gathered = [None] * world
    dist.all_gather_object(gathered, rm)
    ddp.average_buffers()
    after = [b.detach().cpu().clone() for n_, b in model.named_buffers() if "running_mean" in n_]
    all_after = [None] * world
    dist.all_gather_object(all_after, after)
    mean_before = [sum(g[i] for g in gathered) / world for i in range(len(rm))]
    torch.save({"rep": rep, "differ_before": any(not torch.equal(a, b) for a, b in zip(gathered[0], gathered[1])),
                "equal_after": all(torch.equal(a, b) for a, b in zip(all_after[0], all_after[1])),
                "is_mean": all(torch.allclose(a, m, rtol=1e-5, atol=1e-6) for a, m in zip(after, mean_before))},
               os.path.join(out, f"tl{rank}.pt"))
    if dev.type == "cuda":
        torch.cuda.synchronize()
    dist.destroy_process_group()


def rccl_force_check(kind: str = "resnet18", grad_dtype: str = "fp32", steps: int = 3) -> dict:
    """One-GPU exercise of the RCCL data-parallel path (run in its own process).

    Initialises the ``nccl`` process group at world size 1 and wraps the model in the framework's
    DDP with ``force=True`` so every bucket's all-reduce is issued through RCCL from the comm
    stream, ordered by events after the compute and WGRAD streams.  The all-reduced gradient of a
    one-rank job is the local gradient, so with fp32 buckets it must be BIT-identical to the same
    backward without DDP; with bf16 buckets it must equal the bf16 rounding of it.  Parameters after
    ``steps`` SGD steps with and without DDP must match the same way."""
    from ..models import resnet
    from ..ops import cross_entropy
    from .. import optim
    from ..utils.flat import FlatParams
    from . import launch
    from .ddp import DistributedDataParallel

    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    env = launch.init(force_init=True)
    assert env.backend == "nccl", env
    dev = env.device
    g = torch.Generator(device=dev).manual_seed(3)
    x = torch.rand(16, 3, 64, 64, device=dev, generator=g)
    y = torch.randint(0, 10, (16,), device=dev, generator=g)

    def run(use_ddp):
        torch.manual_seed(0)
        model = getattr(resnet, kind)(num_classes=10).to(dev).train()
        flat = FlatParams(model.parameters())
        ddp = DistributedDataParallel(model, flat, force=True, grad_dtype=grad_dtype,
                                      bucket_cap_mb=2.0, first_bucket_mb=0.5, last_bucket_mb=0.5) if use_ddp else None
        opt = optim.SGD(flat, lr=0.01, momentum=0.9)
        grads = []
        for _ in range(steps):
            opt.zero_grad()
            cross_entropy(model.forward_logits(x), y).backward()
            if ddp is not None:     # per-bucket SGD on the comm stream as each all-reduce completes
                ddp.finish_gradient_sync(opt=opt)
                grads.append(flat.grad.clone())
            else:
                grads.append(flat.grad.clone())
                opt.step()
        torch.cuda.synchronize()
        return grads, flat.master.clone(), (len(ddp.buckets) if ddp else 0)

    ref_g, ref_p, _ = run(False)
    got_g, got_p, nb = run(True)
    if grad_dtype == "bf16":
        first = ref_g[0].to(torch.bfloat16).float()
        ok_grad = bool(torch.equal(got_g[0], first))
        ok_param = bool(((got_p - ref_p).norm() <= 1e-2 * ref_p.norm()).item())
    else:
        ok_grad = all(torch.equal(a, b) for a, b in zip(ref_g, got_g))
        ok_param = bool(torch.equal(ref_p, got_p))
    res = {"ok_grad": ok_grad, "ok_param": ok_param, "nbuckets": nb, "backend": env.backend,
           "maxdiff": float((got_g[0] - ref_g[0]).abs().max())}
    launch.shutdown()
    return res


if __name__ == "__main__":
    import json
    import sys
    kind = sys.argv[1] if len(sys.argv) > 1 else "resnet18"
    gd = sys.argv[2] if len(sys.argv) > 2 else "fp32"
    print(json.dumps(rccl_force_check(kind, gd)), flush=True)

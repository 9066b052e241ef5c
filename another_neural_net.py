#!/usr/bin/env python3
"""Distributed image transfer-learning script (reference: another_neural_net.py).

Reference behaviour: rank bootstrap (--local_rank, process group), device report,
80/20 split of the Imagenette train folder with distributed sampling (batch 64), then
``resnet50(...)`` or ``vgg16(...)``: ImageNet backbone frozen, new MLP head, NLL loss, Adam,
3 epochs with per-epoch eval ("Epoch e/E.. Train loss.. Test loss.. Test accuracy.."), VGG early
stopping, "Training time per epoch is X seconds", then batch-1 inference over ~1000/world random
images ("Inference time is X seconds").

MI355X-native: one process per GPU (torchrun or the legacy launcher), RCCL process group,
HIP-kernel model, flat fused Adam, gradient-synchronised DDP (the reference's replicas never
synchronised), hipGraph batch-1 inference with p50/p90/p99, synthetic Imagenette-shaped data by
default (``--data-dir`` reads a real ImageFolder).  ``--preset mlp-cpu`` runs the 2-layer MLP head
standalone on random IMDB-shaped token tensors on the CPU (BASELINE.json config 1).

Launch:  torchrun --nproc-per-node 8 --master-addr 127.0.0.1 another_neural_net.py --model resnet50
         python -m torch.distributed.launch --nproc_per_node=4 ... another_neural_net.py  (legacy)
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import torch  # noqa: E402

import pcmp  # noqa: E402,F401
from pcmp.engine import cli  # noqa: E402


def main(argv=None):
    ap = cli.common_parser(__doc__.splitlines()[0])
    ap.add_argument("--model", choices=["resnet50", "vgg16", "resnet18", "mlp"], default=None)
    ap.add_argument("--train-size", type=int, default=9469, help="images in the (synthetic) train folder")
    ap.add_argument("--image-size", type=int, default=224)
    ap.add_argument("--num-images", type=int, default=None, help="batch-1 inference images (reference: 1000)")
    ap.add_argument("--print-every", type=int, default=1)
    ap.add_argument("--full-train", action="store_true", help="train the whole network (not transfer learning)")
    ap.add_argument("--no-graph", action="store_true")
    args = ap.parse_args(argv)
    cli.apply_preset(args, dict(model="vgg16", epochs=3, batch_size=64, num_images=1000, full_train=False))
    env = cli.setup(args)
    from pcmp.parallel.launch import device_report
    from pcmp.utils.report import rprint
    device_report(env.local_rank, printer=rprint)
    with cli.run_context(args, env):
        if args.model == "mlp":
            return run_mlp_cpu(args, env)
        return run_image(args, env)


def build_image_model(args, device):
    from pcmp.models import resnet, vgg
    if args.model == "vgg16":
        m = vgg.vgg16(10) if args.full_train else vgg.vgg16_transfer(10)
        opt = dict(optimizer="adam", lr=args.lr or 1e-3)           # Adam(model.parameters()) default lr
    else:
        arch = getattr(resnet, args.model)
        if args.full_train:
            m = arch(10)
            opt = dict(optimizer="sgd", lr=args.lr or 0.1, momentum=0.9, weight_decay=5e-5)
        else:
            m = resnet.resnet50_transfer(10)
            opt = dict(optimizer="adam", lr=args.lr or 0.003)      # Adam(model.fc.parameters(), lr=0.003)
    cli.load_pretrained(m, getattr(args, "weights", None))   # models.resnet50(pretrained=True) (:95, :244)
    return m.to(device), opt


def run_image(args, env):
    from pcmp.data.synthetic import BatchLoader, SyntheticImages
    from pcmp.engine.inference import infer_batch1
    from pcmp.engine.trainer import make_state, train_image_classifier
    from pcmp.parallel.sampler import ShardedSampler
    from pcmp.utils.report import rprint
    dev = env.device
    if args.data_dir:
        from pcmp.data.imagefolder import ImageFolder, load_split_train_test
        trainloader, testloader = load_split_train_test(args.data_dir, 0.2, args.batch_size, env.distributed, dev)
        infer_ds = ImageFolder(args.data_dir)
    else:
        ds = SyntheticImages(args.train_size, 10, args.image_size, seed=args.seed, device=dev)
        idx = torch.randperm(len(ds), generator=torch.Generator().manual_seed(args.seed)).tolist()
        split = int(0.2 * len(ds))
        trainloader = BatchLoader(ds, args.batch_size, ShardedSampler(idx[split:]), dev)
        testloader = BatchLoader(ds, args.batch_size, ShardedSampler(idx[:split]), dev)
        infer_ds = ds
    model, optkw = build_image_model(args, dev)
    state = make_state(model, distributed=env.distributed, **optkw)
    early = 1 if args.model == "vgg16" else None
    t_train = train_image_classifier(state, trainloader, testloader, args.epochs, args.print_every,
                                     early_stopping_patience=early, verbose_steps=args.verbose,
                                     reference_compat=args.reference_compat)
    # ---- batch-1 inference over ~num_images/world random images (E1)
    n = max(1, args.num_images // env.world_size)
    idx = torch.randperm(len(infer_ds), generator=torch.Generator().manual_seed(args.seed + env.rank))[:n].tolist()
    images, labels = infer_ds.get_batch(idx, "cpu")
    total, stats, _ = infer_batch1(model, images.float() / 255.0 if images.dtype == torch.uint8 else images,
                                   labels, dev, use_graph=not args.no_graph, print_every_image=args.verbose)
    cli.write_json(args, {"script": "another_neural_net", "model": args.model, "world_size": env.world_size,
                          "train_seconds": t_train, "history": state.history, "inference_total_s": total,
                          "batch1_latency": stats, "data": "real" if args.data_dir else "synthetic"})
    return 0


def run_mlp_cpu(args, env):
    """BASELINE config 1: the 2-layer MLP head on random IMDB-shaped token tensors, CPU.

    Train on a sharded 2,048-review split and evaluate on a held-out 512-review split (indices
    2048..2559 of the same synthetic corpus, so labels follow the same class signatures); the
    epoch line reports the held-out loss / accuracy, summed over ranks."""
    from pcmp.data.synthetic import BatchLoader, SyntheticIMDB
    from pcmp.engine.trainer import make_state
    from pcmp.models.layers import MLPHead
    from pcmp.ops import cross_entropy
    from pcmp.parallel.metrics import all_reduce_sum
    from pcmp.parallel.sampler import ShardedSampler
    from pcmp.utils.report import epoch_line, rprint, training_time_line
    n_train, n_test = 2048, 512
    ds = SyntheticIMDB(n=n_train + n_test, seed=args.seed)
    model = MLPHead(128, 512, 2, 0.2).to(env.device)
    state = make_state(model, "adam", lr=args.lr or 3e-3, distributed=env.distributed)
    loader = BatchLoader(ds, args.batch_size, ShardedSampler(list(range(n_train))), env.device)
    test_loader = BatchLoader(ds, args.batch_size, ShardedSampler(list(range(n_train, n_train + n_test)), shuffle=False),
                              env.device)

    def feats(ids):
        return (ids.float() / ds.VOCAB).to(env.device)

    t1 = time.time()
    for epoch in range(args.epochs):
        loader.set_epoch(epoch)
        model.train()
        tot, n = 0.0, 0
        for ids, mask, y in loader:
            state.zero_grad()
            loss = cross_entropy(model.forward_logits(feats(ids)), y)
            state.backward_step(loss)
            tot += float(loss.detach())
            n += 1
        model.eval()
        te_loss, te_correct, te_n, te_batches = 0.0, 0, 0, 0
        with torch.no_grad():
            for ids, mask, y in test_loader:
                z = model.forward_logits(feats(ids))
                te_loss += float(cross_entropy(z, y))
                te_correct += int((z.argmax(1) == y).sum())
                te_n += y.numel()
                te_batches += 1
        s = all_reduce_sum([tot, n, te_loss, te_batches, te_correct, te_n])
        rprint(epoch_line(epoch + 1, args.epochs, s[0] / max(1, s[1]), s[2] / max(1, s[3]), s[4] / max(1, s[5])))
    dt = time.time() - t1
    rprint(training_time_line(dt))
    cli.write_json(args, {"script": "another_neural_net", "preset": "mlp-cpu", "train_seconds": dt,
                          "test_loss": s[2] / max(1, s[3]), "test_accuracy": s[4] / max(1, s[5])})
    return 0

if __name__ == "__main__":
    sys.exit(main())

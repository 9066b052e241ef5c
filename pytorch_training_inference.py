#!/usr/bin/env python3
"""Single-process image notebook flow (reference: pytorch_training_inference_on_image.ipynb).

Cells reproduced (BASELINE P1-P4):
  ResNet-50: load/split data (bs 64) -> frozen ImageNet backbone + MLP head, NLLLoss, Adam(3e-3)
  -> 1 epoch (print_every=10) + eval -> "Saving Model" -> reload -> ``eval()`` -> batch-1
  inference over 1000 random images -> "Inference time is X seconds" (P1/P3);
  VGG16: frozen backbone + head, Adam, 1 epoch with early stopping (best checkpoint) -> reload ->
  batch-1 inference over 1000 images (P4).
MI355X-native: HIP-kernel models, fused Adam, hipGraph batch-1 inference (p50/p90/p99 reported),
state_dict-based model hand-off (``save_model``/``load_model``), synthetic Imagenette-shaped data
unless ``--data-dir``.
"""
import os
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import torch  # noqa: E402

import pcmp  # noqa: E402,F401
from pcmp.engine import cli  # noqa: E402


def main(argv=None):
    ap = cli.common_parser(__doc__.splitlines()[0])
    ap.add_argument("--models", default="resnet50,vgg16")
    ap.add_argument("--train-size", type=int, default=9469)
    ap.add_argument("--image-size", type=int, default=224)
    ap.add_argument("--num-images", type=int, default=1000)
    ap.add_argument("--print-every", type=int, default=10)
    ap.add_argument("--save-dir", default=None)
    args = ap.parse_args(argv)
    cli.apply_preset(args, dict(epochs=1, batch_size=64))
    env = cli.setup(args)
    from pcmp.data.synthetic import BatchLoader, SyntheticImages
    from pcmp.engine.inference import infer_batch1
    from pcmp.engine.trainer import make_state, train_image_classifier
    from pcmp.models import resnet, vgg
    from pcmp.utils.checkpoint import load_model, save_model
    from pcmp.utils.report import rprint

    dev = env.device
    if args.data_dir:
        from pcmp.data.imagefolder import ImageFolder, load_split_train_test
        trainloader, testloader = load_split_train_test(args.data_dir, 0.2, args.batch_size, False, dev)
        infer_ds = ImageFolder(args.data_dir)
    else:
        ds = SyntheticImages(args.train_size, 10, args.image_size, seed=args.seed, device=dev)
        idx = torch.randperm(len(ds), generator=torch.Generator().manual_seed(args.seed)).tolist()
        split = int(0.2 * len(ds))
        trainloader = BatchLoader(ds, args.batch_size, device=dev, indices=idx[split:], shuffle=True)
        testloader = BatchLoader(ds, args.batch_size, device=dev, indices=idx[:split], shuffle=True)
        infer_ds = ds
    rprint([f"class_{i}" for i in range(10)] if not args.data_dir else infer_ds.classes)
    save_dir = args.save_dir or tempfile.mkdtemp(prefix="pcmp_nb_")
    records = {}
    with cli.run_context(args, env):
        for name in args.models.split(","):
            if name == "resnet50":
                spec = {"builder": "pcmp.models.resnet:resnet50_transfer", "kwargs": {"num_classes": 10}}
                model = cli.load_pretrained(resnet.resnet50_transfer(10), args.weights).to(dev)   # nb :389
                state = make_state(model, "adam", lr=args.lr or 0.003)
                early = None
            else:
                spec = {"builder": "pcmp.models.vgg:vgg16_transfer", "kwargs": {"num_classes": 10}}
                model = cli.load_pretrained(vgg.vgg16_transfer(10), args.weights_vgg).to(dev)   # nb :1968
                state = make_state(model, "adam", lr=args.lr or 1e-3)
                early = 1
            path = os.path.join(save_dir, f"{name}_model.pt")
            t = train_image_classifier(state, trainloader, testloader, args.epochs, args.print_every,
                                       early_stopping_patience=early, save_fn=lambda m: save_model(path, m, spec),
                                       reference_compat=args.reference_compat)
            model = load_model(path).to(dev).eval()
            n = args.num_images
            ii = torch.randperm(len(infer_ds), generator=torch.Generator().manual_seed(args.seed + 1))[:n].tolist()
            example = torch.zeros(1, 3, args.image_size, args.image_size)
            # get_random_images(1000) runs INSIDE the timed region, as in the reference (nb :891-905)
            total, stats, _ = infer_batch1(model, None, None, dev, fetch=lambda: infer_ds.get_batch(ii, "cpu"),
                                           example=example)
            records[name] = {"train_seconds": t, "history": state.history, "inference_total_s": total, "batch1_latency": stats}
    cli.write_json(args, {"script": "pytorch_training_inference", "results": records,
                          "data": "real" if args.data_dir else "synthetic"})
    return 0


if __name__ == "__main__":
    sys.exit(main())

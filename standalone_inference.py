#!/usr/bin/env python3
"""Framework-comparison batch-1 inference (references: Standalone_Inference_Imagenette_trial.ipynb,
DeepLearning_standalone_trial.ipynb).

Reference: for {TF, PyTorch} x {ResNet-50, VGG16} with ImageNet-pretrained
classifiers, loop over the 3,925 Imagenette val images (``get_image_paths``), preprocess, predict,
print the top label, and time the loop ("Inference Time is: X seconds"); plus a single-image
sanity prediction with top-k softmax percentages.  All four timing cells were interrupted, so no
reference numbers exist (BASELINE P6).

Here there is ONE backend (HIP kernels); the "TF/Keras" column is the Keras-semantics variant of
the same framework (ResNet50 v1 stride placement, caffe-style ``preprocess_input``) and the
"PyTorch" column the torchvision-topology models with ``ToTensor`` inputs.  Weights are random
(no downloads), so labels are meaningless; timing is what is compared.  Every model is run in
``eval()`` under ``no_grad`` with a hipGraph-replayed batch-1 forward (the reference forgot both,
SURVEY §0.2-4/6).
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
    ap.add_argument("--models", default="pt-resnet50,pt-vgg16,keras-resnet50,keras-vgg16")
    ap.add_argument("--num-images", type=int, default=3925, help="Imagenette2 val size")
    ap.add_argument("--image-size", type=int, default=224)
    ap.add_argument("--print-labels", action="store_true")
    args = ap.parse_args(argv)
    cli.apply_preset(args, {})
    env = cli.setup(args)
    from pcmp.data.synthetic import SyntheticImages
    from pcmp.engine.inference import Batch1Predictor, predict_topk
    from pcmp.models import resnet, vgg
    from pcmp.models.keras_resnet import preprocess_input_caffe
    from pcmp.utils import report as R
    from pcmp.utils.misc import watchdog_kick

    dev = env.device
    paths = None
    if args.data_dir:
        # the reference loads + preprocesses every image INSIDE its timed loop
        # (Standalone_Inference_Imagenette_trial.ipynb:98-107,165-188): host JPEG decode, then the
        # resize / ToTensor on the device (resize_image kernel) when a GPU is used
        from pcmp.data.imagefolder import get_image_paths, preprocess_single
        paths = get_image_paths(args.data_dir)[: args.num_images]
        images = preprocess_single(paths[0], args.image_size, dev)   # example for graph capture
        images = images.cpu() if images.is_cuda else images
    else:
        ds = SyntheticImages(args.num_images, 10, args.image_size, seed=args.seed)
        images, _ = ds.get_batch(list(range(args.num_images)), "cpu")
        R.rprint(args.num_images)
    with cli.run_context(args, env):
        results = {}
        for name in args.models.split(","):
            fam, arch = name.split("-")
            model = (resnet.ResNet("resnet50", 1000, variant="keras" if fam == "keras" else "torchvision")
                     if arch == "resnet50" else vgg.vgg16(1000))
            wpath = args.weights if arch == "resnet50" else args.weights_vgg
            if fam == "pt":
                cli.load_pretrained(model, wpath)   # models.resnet50 / vgg16(pretrained=True)
            model = model.to(dev).eval()
            pre = (lambda x: preprocess_input_caffe(x.permute(0, 2, 3, 1) * 255.0)) if fam == "keras" else (lambda x: x)
            # single-image sanity prediction (E3)
            top = predict_topk(model, pre(images[:1]).to(dev), None, 5 if fam == "pt" else 3)
            R.rprint(R.label_probability_line(top[0][0], round(top[0][1], 2)))
            predictor = Batch1Predictor(model, pre(images[:1]).to(dev))
            lat = []
            t = time.time()
            n_img = len(paths) if paths is not None else images.shape[0]
            for i in range(n_img):
                watchdog_kick("inference")
                ts = time.perf_counter()
                xi = preprocess_single(paths[i], args.image_size, dev) if paths is not None else images[i:i + 1]
                idx = predictor(pre(xi))
                lat.append(time.perf_counter() - ts)
                if args.print_labels:
                    R.rprint(idx)
            total = time.time() - t
            R.rprint(R.standalone_inference_line(total))
            results[name] = {"total_s": total, **R.latency_stats(lat)}
    cli.write_json(args, {"script": "standalone_inference", "n_images": len(paths) if paths is not None else int(images.shape[0]),
                          "results": results,
                          "weights": args.weights or args.weights_vgg or "random-init", "data": "real" if args.data_dir else "synthetic"})
    return 0


if __name__ == "__main__":
    sys.exit(main())

#!/usr/bin/env python3
"""Keras/TensorFlow counterpart (reference: resnet.py) on the single HIP path.

Reference: ImageDataGenerator(rescale=1/255).flow_from_directory(
batch 64, 224x224, categorical), ResNet50(weights='imagenet', include_top=False) -> Flatten ->
Dense(10, softmax), compile(SGD(lr=0.001), categorical_crossentropy, accuracy), fit(epochs=5,
validation_data=val), then a timed ``model.evaluate(val)`` printing "the inference takes X
seconds" (the reference crashes there: ``time`` is never imported).
The backbone is fully fine-tuned (not frozen), as in the reference.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import torch  # noqa: E402

import pcmp  # noqa: E402,F401
from pcmp.engine import cli  # noqa: E402


def main(argv=None):
    ap = cli.common_parser(__doc__.splitlines()[0])
    ap.add_argument("--train-size", type=int, default=9469)
    ap.add_argument("--val-size", type=int, default=3925)
    ap.add_argument("--image-size", type=int, default=224)
    args = ap.parse_args(argv)
    cli.apply_preset(args, dict(epochs=5, batch_size=64))
    env = cli.setup(args)
    from pcmp.data.synthetic import BatchLoader, SyntheticImages
    from pcmp.engine.trainer import keras_evaluate, keras_fit, make_state
    from pcmp.models.keras_resnet import KerasResNet50TL
    from pcmp.parallel.sampler import ShardedSampler
    dev = env.device
    if args.data_dir:
        # ImageDataGenerator(rescale=1./255).flow_from_directory(<dir>/train|val, batch 64, 224x224,
        # categorical, shuffle=True) (resnet.py:10-16): uint8 batches, /255 on the device
        from pcmp.data.imagefolder import flow_from_directory
        train = flow_from_directory(os.path.join(args.data_dir, "train"), args.image_size, args.batch_size,
                                    dev, env.distributed)
        val = flow_from_directory(os.path.join(args.data_dir, "val"), args.image_size, args.batch_size,
                                  dev, env.distributed)
        num_classes = len(train.ds.classes)
    else:
        tr = SyntheticImages(args.train_size, 10, args.image_size, seed=args.seed)
        va = SyntheticImages(args.val_size, 10, args.image_size, seed=args.seed + 1)
        train = BatchLoader(tr, args.batch_size, ShardedSampler(len(tr), shuffle=True), dev)
        val = BatchLoader(va, args.batch_size, ShardedSampler(len(va), shuffle=True), dev)
        num_classes = 10
    x0, y0 = next(iter(train))
    print(len(x0), tuple(x0[0].permute(1, 2, 0).shape), (len(y0), num_classes))
    model = KerasResNet50TL(num_classes, image_size=args.image_size).to(dev)
    state = make_state(model, "sgd", lr=args.lr or 0.001, distributed=env.distributed)
    with cli.run_context(args, env):
        hist = keras_fit(state, train, val, args.epochs)
        loss, acc = keras_evaluate(model, val, timed=True)
    cli.write_json(args, {"script": "resnet.py (keras counterpart)", "history": hist, "val_loss": loss,
                          "val_accuracy": acc, "data": "real" if args.data_dir else "synthetic"})
    return 0


if __name__ == "__main__":
    sys.exit(main())

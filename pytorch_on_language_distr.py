#!/usr/bin/env python3
"""Distributed text classification (reference: pytorch_on_language_distr.py).

Reference flow: read "IMDB Dataset.csv" (HTML tags stripped), first 10,000 reviews
for train / next 2,500 for test, BERT tokenizer encode(max_length=128) -> pad_sequences(post) ->
attention masks -> train_test_split(random_state=2020, test_size=0.1) -> DistributedSampler ->
batch 32 -> BertForSequenceClassification(num_labels=2), AdamW(lr=2e-5, eps=1e-8), linear schedule
(no warm-up, 3 epochs), clip_grad_norm 1.0, seed 42; per-epoch "Average training loss" /
"Training epcoh took" / validation accuracy; final test accuracy + "Test took".

MI355X-native: ``--model bilstm`` (north-star BiLSTM encoder, default) or ``--model bert``
(reference-faithful BERT-base) on HIP kernels; RCCL DDP with gradient synchronisation (the
reference's DDP line is commented out, so its ranks never synchronised); the text pipeline runs
natively (``torch.ops.pcmp.text_encode``); synthetic IMDB-shaped data unless ``--csv`` is given
(the reference's imdb.zip is a missing blob here).
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import torch  # noqa: E402

import pcmp  # noqa: E402,F401
from pcmp.engine import cli
from pcmp.ops.kernels import FP32_REF_OPS  # noqa: E402


def main(argv=None):
    ap = cli.common_parser(__doc__.splitlines()[0])
    ap.add_argument("--model", choices=["bilstm", "bert"], default=None)
    ap.add_argument("--csv", default=None, help="IMDB Dataset.csv (review,sentiment)")
    ap.add_argument("--vocab", default=None, help="BERT vocab.txt (else built from the corpus)")
    ap.add_argument("--max-len", type=int, default=128)
    ap.add_argument("--train-size", type=int, default=10000)
    ap.add_argument("--test-size", type=int, default=2500)
    ap.add_argument("--layers", type=int, default=None, help="override encoder depth (tests)")
    ap.add_argument("--print-batches", action="store_true", help="reference's per-step print(batch)")
    ap.add_argument("--graph", action="store_true",
                    help="replay each training step from one captured hipGraph (single GPU process)")
    args = ap.parse_args(argv)
    cli.apply_preset(args, dict(model="bilstm", epochs=3, batch_size=32))
    env = cli.setup(args)
    from pcmp.data.imdb import TensorTextDataset, train_val_split
    from pcmp.data.synthetic import BatchLoader, SyntheticIMDB
    from pcmp.engine.trainer import make_state, test_text, train_text_classifier
    from pcmp.optim import linear_schedule_with_warmup
    from pcmp.parallel.sampler import ShardedSampler
    from pcmp.utils import report as R

    dev = env.device
    if args.csv:
        from pcmp.data import imdb
        texts, labels = imdb.read_files(args.csv)
        (tr_t, tr_y), (te_t, te_y) = imdb.split_reference(texts, labels)
        R.rprint(R.LOADING_TOKENIZER)
        vocab = imdb.load_vocab(args.vocab) if args.vocab else imdb.build_vocab(list(tr_t))
        R.rprint(R.padding_token_line("[PAD]", 0))
        ids, mask = imdb.encode(list(tr_t), vocab, args.max_len)
        tids, tmask = imdb.encode(list(te_t), vocab, args.max_len)
        (a, am, al), (b, bm, bl) = train_val_split(ids.numpy(), list(tr_y), mask.numpy())
        train_ds, val_ds = TensorTextDataset(a, am, al), TensorTextDataset(b, bm, bl)
        test_ds = TensorTextDataset(tids, tmask, list(te_y))
    else:
        full = SyntheticIMDB(args.train_size + args.test_size, args.max_len, seed=args.seed)
        ids, mask, y = full.get_batch(list(range(len(full))), "cpu")
        ntr = args.train_size
        (a, am, al), (b, bm, bl) = train_val_split(ids[:ntr].numpy(), y[:ntr].numpy(), mask[:ntr].numpy())
        train_ds, val_ds = TensorTextDataset(a, am, al), TensorTextDataset(b, bm, bl)
        test_ds = TensorTextDataset(ids[ntr:], mask[ntr:], y[ntr:])
    bs = args.batch_size
    train_loader = BatchLoader(train_ds, bs, ShardedSampler(len(train_ds)), dev)
    val_loader = BatchLoader(val_ds, bs, ShardedSampler(len(val_ds)), dev)
    test_loader = BatchLoader(test_ds, bs, ShardedSampler(len(test_ds)), dev)

    if args.model == "bert":
        from pcmp.models.bert import BertConfig, BertForSequenceClassification
        cfg = BertConfig(num_labels=2)
        if args.layers:
            cfg.num_hidden_layers = args.layers
        model = cli.load_pretrained(BertForSequenceClassification(cfg), args.weights).to(dev)   # from_pretrained (:155)
        lr = args.lr or 2e-5
    else:
        from pcmp.models.bilstm import BiLSTMClassifier
        model = BiLSTMClassifier(num_layers=args.layers or 2).to(dev)
        lr = args.lr or 1e-3
    state = make_state(model, "adamw", lr=lr, eps=1e-8, distributed=env.distributed, clip=1.0)
    total_steps = len(train_loader) * args.epochs
    state.sched = linear_schedule_with_warmup(state.opt, 0, total_steps)
    t0 = time.time()
    with cli.run_context(args, env):
        times = train_text_classifier(state, train_loader, val_loader, args.epochs, print_batches=args.print_batches,
                                      graph=args.graph and not env.distributed)
        acc = test_text(model, test_loader)
    cli.write_json(args, {"script": "pytorch_on_language_distr", "model": args.model, "world_size": env.world_size,
                          "epoch_seconds": times, "train_loss": state.history["train_loss"], "test_accuracy": acc,
                          "samples_per_sec": len(train_ds) * args.epochs / max(1e-9, sum(times)),
                          "total_seconds": time.time() - t0, "data": "real" if args.csv else "synthetic",
                          "dtype": args.dtype,
                          "fp32_reference_ops": sorted(FP32_REF_OPS) if args.dtype == "fp32" else []})
    if model.__class__.__name__ == "BiLSTMClassifier":
        from pcmp.ops.rnn import check_errors
        check_errors()
    return 0


if __name__ == "__main__":
    sys.exit(main())

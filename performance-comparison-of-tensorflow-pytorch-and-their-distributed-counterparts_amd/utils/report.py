"""Report strings and metrics.

Every human-readable line the reference prints is reproduced verbatim here (including its
typos: "Capablity", "epcoh"), so a user diffing logs sees the same lines; a machine-readable
JSON record is emitted alongside (``emit_json``).  Only rank 0 prints unless asked otherwise.
"""
from __future__ import annotations

import datetime
import json
import sys

import numpy as np
import torch


def is_main() -> bool:
    import torch.distributed as dist
    return not dist.is_initialized() or dist.get_rank() == 0


def rprint(*a, all_ranks=False, **kw):
    if all_ranks or is_main():
        print(*a, **kw, flush=True)


# ----------------------------------------------------------------------------- G2 / G3 / G4
def format_time(elapsed: float) -> str:
    """pytorch_on_language_distr.py:196-204 — rounds to whole seconds, 'h:mm:ss'."""
    return str(datetime.timedelta(seconds=int(round(elapsed))))


def flat_accuracy(preds, labels) -> float:
    """pytorch_on_language_distr.py:188-191 (numpy argmax accuracy)."""
    preds = np.asarray(preds)
    labels = np.asarray(labels)
    pred_flat = np.argmax(preds, axis=1).flatten()
    labels_flat = labels.flatten()
    return np.sum(pred_flat == labels_flat) / len(labels_flat)


def top1_accuracy(logps: torch.Tensor, labels: torch.Tensor) -> float:
    """another_neural_net.py:150-153: exp -> topk(1) -> equals -> mean over a CPU FloatTensor."""
    ps = torch.exp(logps.float())
    top_p, top_class = ps.topk(1, dim=1)
    equals = top_class == labels.view(*top_class.shape)
    return torch.mean(equals.type(torch.FloatTensor)).item()


# ----------------------------------------------------------------------------- Appendix A
def epoch_line(epoch, epochs, train_loss, test_loss, test_acc) -> str:
    return (f"Epoch {epoch}/{epochs}.. "
            f"Train loss: {train_loss:.3f}.. "
            f"Test loss: {test_loss:.3f}.. "
            f"Test accuracy: {test_acc:.3f}")


def training_time_line(seconds) -> str:
    return "Training time per epoch is {} seconds".format(seconds)


def inference_time_line(seconds) -> str:
    return "Inference time is {} seconds".format(seconds)


def standalone_inference_line(seconds) -> str:
    return "Inference Time is: {} seconds".format(seconds)


def keras_inference_line(seconds) -> str:
    return "the inference takes {} seconds".format(seconds)


def label_probability_line(label, pct) -> str:
    return "the label is {} with {}% probability".format(label, pct)


TRAINLOADER_DONE = "trainloader done"
SAVING_MODEL = "Saving Model"
EARLY_STOPPING = "Early stopping!"
LOADING_TOKENIZER = "Loading BERT tokenizer..."
TRAINING = "Training..."
RUNNING_VALIDATION = "Running Validation..."
TRAINING_COMPLETE = "Training complete!"
PRINTED_BATCH = "Printed batch"
NO_GPU = "No GPU. switching to CPU"


def padding_token_line(tok, tid) -> str:
    return '\nPadding token: "{:}", ID: {:}'.format(tok, tid)


def text_epoch_header(epoch_i, epochs) -> str:
    return "======== Epoch {:} / {:} ========".format(epoch_i + 1, epochs)


def batch_progress_line(step, total, elapsed) -> str:
    return "  Batch {:>5,}  of  {:>5,}.    Elapsed: {:}.".format(step, total, elapsed)


def avg_train_loss_line(v) -> str:
    return "  Average training loss: {0:.2f}".format(v)


def epoch_took_line(t) -> str:
    return "  Training epcoh took: {:}".format(t)


def val_accuracy_line(v) -> str:
    return "  Accuracy: {0:.2f}".format(v)


def val_took_line(t) -> str:
    return "  Validation took: {:}".format(t)


def test_accuracy_line(v) -> str:
    return "  Accuracy: {0:.4f}".format(v)


def test_took_line(t) -> str:
    return "  Test took: {:}".format(t)


# ----------------------------------------------------------------------------- JSON metrics
def latency_stats(lat_s) -> dict:
    a = np.asarray(lat_s, dtype=np.float64) * 1e3
    if a.size == 0:
        return {}
    return {"p50_ms": float(np.percentile(a, 50)), "p90_ms": float(np.percentile(a, 90)),
            "p99_ms": float(np.percentile(a, 99)), "mean_ms": float(a.mean()), "n": int(a.size)}


def emit_json(record: dict, stream=None, all_ranks=False):
    if all_ranks or is_main():
        print(json.dumps(record, default=float), file=stream or sys.stdout, flush=True)

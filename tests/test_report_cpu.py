"""Golden-string tests for every Appendix A report line."""
import numpy as np
import torch

import pcmp  # noqa: F401
from pcmp.utils import report as R


def test_image_strings():
    assert R.epoch_line(1, 3, 2.5551, 0.0551, 0.979) == "Epoch 1/3.. Train loss: 2.555.. Test loss: 0.055.. Test accuracy: 0.979"
    assert R.training_time_line(5314.126418352127) == "Training time per epoch is 5314.126418352127 seconds"
    assert R.inference_time_line(246.6539294719696) == "Inference time is 246.6539294719696 seconds"
    assert R.standalone_inference_line(1.5) == "Inference Time is: 1.5 seconds"
    assert R.keras_inference_line(2.0) == "the inference takes 2.0 seconds"
    assert R.label_probability_line("Indian_elephant", 51.4) == "the label is Indian_elephant with 51.4% probability"
    assert R.TRAINLOADER_DONE == "trainloader done"
    assert R.SAVING_MODEL == "Saving Model"
    assert R.EARLY_STOPPING == "Early stopping!"
    assert R.NO_GPU == "No GPU. switching to CPU"


def test_text_strings():
    assert R.text_epoch_header(0, 3) == "======== Epoch 1 / 3 ========"
    assert R.batch_progress_line(40, 282, "0:00:12") == "  Batch    40  of    282.    Elapsed: 0:00:12."
    assert R.batch_progress_line(1200, 2000, "1:00:00") == "  Batch 1,200  of  2,000.    Elapsed: 1:00:00."
    assert R.avg_train_loss_line(0.4567) == "  Average training loss: 0.46"
    assert R.epoch_took_line("0:01:02") == "  Training epcoh took: 0:01:02"
    assert R.val_accuracy_line(0.8765) == "  Accuracy: 0.88"
    assert R.val_took_line("0:00:05") == "  Validation took: 0:00:05"
    assert R.test_accuracy_line(0.87654) == "  Accuracy: 0.8765"
    assert R.test_took_line("0:00:07") == "  Test took: 0:00:07"
    assert R.padding_token_line("[PAD]", 0) == '\nPadding token: "[PAD]", ID: 0'
    assert R.LOADING_TOKENIZER == "Loading BERT tokenizer..."
    assert R.TRAINING_COMPLETE == "Training complete!"


def test_format_time_and_accuracy():
    assert R.format_time(0.4) == "0:00:00"
    assert R.format_time(3661.6) == "1:01:02"
    preds = np.array([[0.1, 0.9], [0.8, 0.2], [0.3, 0.7]])
    assert R.flat_accuracy(preds, np.array([1, 0, 0])) == 2 / 3
    logp = torch.log_softmax(torch.tensor([[0.0, 2.0], [3.0, 0.0]]), 1)
    assert R.top1_accuracy(logp, torch.tensor([1, 1])) == 0.5


def test_latency_stats():
    s = R.latency_stats([0.001] * 98 + [0.01, 0.02])
    assert abs(s["p50_ms"] - 1.0) < 1e-9 and s["n"] == 100 and s["p99_ms"] > 9.0


def test_device_report_cpu_and_seeding():
    import random

    import numpy as np
    import torch

    from pcmp.parallel.launch import device_report
    from pcmp.utils.misc import seed_everything
    out = []
    dev = device_report(0, printer=lambda *a: out.append(" ".join(str(x) for x in a)))
    if not torch.cuda.is_available():
        assert out == ["No GPU. switching to CPU"] and dev.type == "cpu"
    seed_everything(42)
    a = (random.random(), float(np.random.rand()), float(torch.rand(1)))
    seed_everything(42)
    assert a == (random.random(), float(np.random.rand()), float(torch.rand(1)))

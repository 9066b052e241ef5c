"""Engine / entry points / checkpoint / text pipeline on CPU (tiny synthetic configs)."""
import json
import os
import subprocess
import sys

import pytest
import torch

import pcmp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(script, *args, timeout=600):
    env = dict(os.environ, PYTHONPATH=ROOT, CUDA_VISIBLE_DEVICES="")
    r = subprocess.run([sys.executable, os.path.join(ROOT, script), "--device", "cpu", *args], capture_output=True,
                       text=True, timeout=timeout, env=env)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    return r.stdout


def _last_json(out):
    for line in reversed(out.strip().splitlines()):
        if line.startswith("{"):
            return json.loads(line)
    raise AssertionError("no JSON record")


def test_another_neural_net_resnet_tl():
    out = _run("another_neural_net.py", "--model", "resnet50", "--train-size", "24", "--image-size", "64",
               "--batch-size", "8", "--epochs", "1", "--num-images", "3")
    assert "No GPU. switching to CPU" in out
    assert "trainloader done" in out and "Epoch 1/1.. Train loss:" in out
    assert "Training time per epoch is" in out and "Inference time is" in out
    rec = _last_json(out)
    assert rec["batch1_latency"]["n"] == 3 and "p50_ms" in rec["batch1_latency"]


def test_mlp_cpu_preset():
    out = _run("another_neural_net.py", "--preset", "mlp-cpu")
    assert "Training time per epoch is" in out


def test_text_bert_entrypoint():
    out = _run("pytorch_on_language_distr.py", "--model", "bert", "--layers", "1", "--train-size", "40",
               "--test-size", "16", "--epochs", "1", "--batch-size", "8")
    for s in ("======== Epoch 1 / 1 ========", "Training...", "  Average training loss:", "  Training epcoh took:",
              "Running Validation...", "  Validation took:", "Training complete!", "  Test took:"):
        assert s in out, s


def test_keras_counterpart_entrypoint():
    out = _run("resnet.py", "--train-size", "8", "--val-size", "8", "--image-size", "64", "--batch-size", "8",
               "--epochs", "1")
    assert "the inference takes" in out


def test_notebook_flow_save_reload_infer(tmp_path):
    out = _run("pytorch_training_inference.py", "--models", "resnet50", "--train-size", "24", "--image-size", "64",
               "--batch-size", "8", "--num-images", "2", "--save-dir", str(tmp_path))
    assert "Saving Model" in out and "Inference time is" in out
    assert (tmp_path / "resnet50_model.pt").exists()


def test_standalone_inference_entrypoint():
    out = _run("standalone_inference.py", "--models", "pt-resnet50,keras-resnet50", "--num-images", "2",
               "--image-size", "64")
    assert out.count("Inference Time is:") == 2


def test_checkpoint_roundtrip(tmp_path):
    from pcmp.models.resnet import resnet18
    from pcmp.optim import SGD
    from pcmp.utils.checkpoint import load_checkpoint, load_model, save_checkpoint, save_model
    from pcmp.utils.flat import FlatParams
    m = resnet18(10)
    flat = FlatParams(m.parameters(), shadow_dtype=None)
    opt = SGD(flat, lr=0.01, momentum=0.9)
    from pcmp.ops import cross_entropy
    cross_entropy(m.forward_logits(torch.rand(4, 3, 32, 32)), torch.tensor([0, 1, 2, 3])).backward()
    opt.step()
    save_checkpoint(str(tmp_path / "c.pt"), m, opt, epoch=3)
    m2 = resnet18(10)
    flat2 = FlatParams(m2.parameters(), shadow_dtype=None)
    opt2 = SGD(flat2, lr=0.5, momentum=0.9)
    ep, _ = load_checkpoint(str(tmp_path / "c.pt"), m2, opt2)
    assert ep == 3 and opt2.lr == 0.01 and torch.equal(flat.master, flat2.master) and torch.equal(opt.mom, opt2.mom)
    save_model(str(tmp_path / "m.pt"), m, {"builder": "pcmp.models.resnet:resnet18", "kwargs": {"num_classes": 10}})
    m3 = load_model(str(tmp_path / "m.pt")).eval()
    m.eval()
    x = torch.rand(1, 3, 32, 32)
    assert torch.allclose(m.forward_logits(x), m3.forward_logits(x))


def test_native_text_pipeline_matches_python():
    from pcmp.data import imdb
    texts = ["This movie was GREAT!!<br /><br />Loved it, 10/10.", "bad.", "Unseenwordxyz and the end",
             "a " * 300, ""]
    vocab = imdb.build_vocab(texts + ["movie great loved the end and a bad"], size=400)
    ids_n, m_n = imdb.encode(texts, vocab, 16)
    ids_p, m_p = imdb.encode(texts, vocab, 16, force_python=True)
    assert torch.equal(ids_n, ids_p) and torch.equal(m_n, m_p)
    assert ids_n[0, 0].item() == 101 and (ids_n[3] > 0).all()        # [CLS] ... truncated to 16
    assert ids_n[1].tolist()[:4] == [101, vocab.index("bad"), vocab.index("."), 102]
    assert ids_n[4].tolist()[:3] == [101, 102, 0]
    assert torch.equal(m_n, (ids_n > 0).long())


def test_rm_tags_and_csv_reader(tmp_path):
    from pcmp.data import imdb
    assert imdb.rm_tags("a<br />b<i>c</i>") == "a b c "
    p = tmp_path / "IMDB Dataset.csv"
    p.write_text('review,sentiment\n"Good <br/>film",positive\n"Awful",negative\n')
    texts, labels = imdb.read_files(str(p))
    assert list(labels) == [1, 0] and "<" not in texts[0]


def test_synthetic_datasets_shapes():
    from pcmp.data.synthetic import BatchLoader, SyntheticIMDB, SyntheticImages
    ds = SyntheticImages(100, 10, 32)
    x, y = ds.get_batch([0, 5, 7])
    assert x.shape == (3, 3, 32, 32) and 0 <= x.min() and x.max() <= 1 and y.max() < 10
    assert torch.equal(ds.labels(torch.tensor([5])), ds.labels(torch.tensor([5])))
    t = SyntheticIMDB(50)
    ids, mask, lab = t.get_batch(list(range(50)))
    assert ids.shape == (50, 128) and (ids[:, 0] == 101).all() and torch.equal(mask, (ids > 0).long())
    assert len(BatchLoader(ds, 32)) == 4


def test_label_tables_and_decode():
    from pcmp.data.labels import decode_topk, imagenette_labels, parse_label_table
    txt = "{0: 'tench, Tinca tinca',\n 1: 'goldfish, Carassius auratus',\n 2: \"great white shark\"}"
    assert parse_label_table(txt) == ["tench, Tinca tinca", "goldfish, Carassius auratus", "great white shark"]
    assert parse_label_table("a\nb\n\nc\n") == ["a", "b", "c"]
    labels = imagenette_labels()
    assert len(labels) == 10
    logits = torch.tensor([[0.0, 5.0, 1.0]])
    top = decode_topk(logits, ["x", "y", "z"], k=2)
    assert [t[0] for t in top[0]] == [1, 2] and top[0][0][1] == "y"
    assert abs(sum(torch.softmax(logits, -1)[0].tolist()) - 1) < 1e-6


def test_phase_timer_wiring(monkeypatch):
    """PCMP_PHASE_TIMES=1 brackets data / forward / backward / optimizer phases."""
    monkeypatch.setenv("PCMP_PHASE_TIMES", "1")
    monkeypatch.setenv("PCMP_PHASE_WARMUP", "0")
    import torch
    from pcmp.engine.trainer import make_state, train_image_classifier
    from pcmp.models.layers import MLPHead

    torch.manual_seed(0)
    m = MLPHead(16, 32, 4, p=0.0)
    st = make_state(m, "sgd", lr=0.1)
    assert st.timer is not None
    data = [(torch.randn(8, 16), torch.randint(0, 4, (8,))) for _ in range(3)]
    lines = []
    train_image_classifier(st, data, data[:1], epochs=1, printer=lambda *a: lines.append(" ".join(map(str, a))))
    ph = st.history["phases"]
    for k in ("data", "forward", "backward", "optimizer"):
        assert k in ph and ph[k]["host_s_total"] >= 0.0
    assert any(l.startswith("[phase times") for l in lines)


def test_step_throttle_noop_on_cpu(monkeypatch):
    from pcmp.utils.misc import StepThrottle
    t = StepThrottle("cpu", depth=2)
    for _ in range(5):
        t.tick()
    assert t.in_flight == 0
    monkeypatch.setenv("PCMP_MAX_INFLIGHT", "0")
    assert StepThrottle("cpu").depth == 0


def test_train_state_has_throttle():
    from pcmp.engine.trainer import make_state
    from pcmp.utils.misc import StepThrottle
    m = torch.nn.Linear(4, 2)
    st = make_state(m, "sgd", lr=0.1)
    assert isinstance(st.throttle, StepThrottle)
    loss = m(torch.randn(3, 4)).square().mean()
    st.zero_grad()
    st.backward_step(loss)
    assert st.throttle.in_flight == 0      # CPU: no events


def test_synthetic_labels_are_balanced_and_lengths_vary():
    """The synthetic datasets must carry every class (a degenerate hash once gave every image
    class 2 and every review label 0 and length 128, which made any accuracy check vacuous)."""
    from pcmp.data.synthetic import SyntheticImages, SyntheticIMDB
    y = SyntheticImages(9469, 10, 32, seed=42).labels(torch.arange(9469))
    counts = torch.bincount(y, minlength=10).float()
    assert counts.min() > 0.8 * counts.mean() and counts.max() < 1.2 * counts.mean()
    t = SyntheticIMDB(12500, seed=42)
    lab = torch.bincount(t.labels(torch.arange(12500)), minlength=2).float()
    assert abs(lab[0] / lab.sum() - 0.5) < 0.05
    L = t.lengths(torch.arange(12500))
    frac_full = (L == 128).float().mean()
    assert 0.7 < frac_full < 0.8 and int(L.min()) < 20
    # labels are a pure function of (seed, index): any shard / order sees the same labelled set
    d = SyntheticImages(100, 10, 32, seed=7)
    assert torch.equal(d.labels(torch.tensor([5, 17, 3])), d.labels(torch.arange(100))[[5, 17, 3]])


def test_mlp_cpu_reports_held_out_metrics():
    out = _run("another_neural_net.py", "--preset", "mlp-cpu", "--epochs", "2")
    rec = _last_json(out)
    assert "test_accuracy" in rec and 0.0 <= rec["test_accuracy"] <= 1.0
    assert out.count("Epoch ") == 2


def test_dtype_fp32_stays_on_hip_backend():
    """--dtype fp32 (the reference's precision) keeps the HIP backend: fp32 kernels of csrc/f32.hip
    (image ops) and csrc/text_f32.hip (text encoders); no op runs the PyTorch reference."""
    from pcmp.ops import _lib
    from pcmp.ops.kernels import FP32_REF_OPS
    assert len(FP32_REF_OPS) == 0
    try:
        _lib.set_precision("fp32")
        assert _lib.backend() == "hip" and _lib.precision() == "fp32"
        assert _lib.default_compute_dtype(torch.device("cuda", 0)) == torch.float32
        from pcmp.models.resnet import resnet18
        m = resnet18(num_classes=10)
        assert m._cdtype(torch.device("cuda", 0)) == torch.float32
    finally:
        _lib.set_precision("bf16")
        _lib.set_backend("hip")
    assert _lib.default_compute_dtype(torch.device("cuda", 0)) == torch.bfloat16
    assert _lib.default_compute_dtype(torch.device("cpu")) == torch.float32


def test_dtype_flag_on_entrypoint():
    out = _run("another_neural_net.py", "--preset", "mlp-cpu", "--dtype", "fp32")
    assert "Training time per epoch is" in out


def test_watchdog_fires_and_is_kicked():
    import io
    import time as _t
    from pcmp.utils.misc import Watchdog, watchdog_kick
    buf = io.StringIO()
    with Watchdog(0.4, abort=False, stream=buf) as wd:
        for _ in range(5):
            watchdog_kick("train_step")
            _t.sleep(0.05)
        assert wd.state["step"] == 5 and wd.state["phase"] == "train_step"
        _t.sleep(1.6)      # no kicks: the watchdog reports the stall with the last step/phase
    assert "[watchdog] no progress" in buf.getvalue() and "step=5 phase=train_step" in buf.getvalue()
    watchdog_kick("after")  # no active watchdog: a no-op


def test_watchdog_abort_reached_on_stream_without_fd():
    """A StringIO stream has no fileno (faulthandler refuses it): the stacks are still written and
    the abort is still reached."""
    import io
    import threading
    import time as _t
    from pcmp.utils.misc import Watchdog
    buf = io.StringIO()
    fired = threading.Event()
    codes = []
    wd = Watchdog(0.3, abort=True, stream=buf)
    wd._exit = lambda code: (codes.append(code), fired.set(), wd._stop.set())
    with wd:
        assert fired.wait(5.0)
    assert codes == [3]
    out = buf.getvalue()
    assert "[watchdog] no progress" in out and "most recent call last" in out


def test_profile_and_watchdog_flags_on_entrypoint(tmp_path):
    trace = tmp_path / "trace.json"
    _run("another_neural_net.py", "--preset", "mlp-cpu", "--watchdog", "120", "--profile", str(trace))
    assert trace.exists() and trace.stat().st_size > 0
    json.loads(trace.read_text())


def test_keras_flow_from_directory(tmp_path):
    import numpy as np
    from PIL import Image
    for split in ("train", "val"):
        for c in ("cat", "dog", "eel"):
            d = tmp_path / split / c
            d.mkdir(parents=True)
            for i in range(2):
                Image.fromarray((np.random.rand(20, 30, 3) * 255).astype(np.uint8)).save(d / f"{i}.JPEG")
    from pcmp.data.imagefolder import flow_from_directory
    it = flow_from_directory(str(tmp_path / "train"), 32, 4, None)
    xs = [x for x, _ in it]
    assert len(it.ds) == 6 and it.ds.classes == ["cat", "dog", "eel"]
    assert xs[0].dtype == torch.uint8 and tuple(xs[0].shape[1:]) == (3, 32, 32)
    out = _run("resnet.py", "--data-dir", str(tmp_path), "--image-size", "32", "--batch-size", "4", "--epochs", "1")
    assert "Found 6 images belonging to 3 classes." in out and "the inference takes" in out
    assert _last_json(out)["data"] == "real"


def test_hw_queue_floor():
    """The pool exports GPU_MAX_HW_QUEUES=4: pcmp raises it to 8 (forced-RCCL step 24.9 -> 22.2 ms),
    keeps a larger inherited value, and PCMP_HW_QUEUES pins it exactly (clamped to 1..32)."""
    import pcmp
    for env, want in (({"GPU_MAX_HW_QUEUES": "4"}, 8), ({}, 8), ({"GPU_MAX_HW_QUEUES": "16"}, 16),
                      ({"GPU_MAX_HW_QUEUES": "4", "PCMP_HW_QUEUES": "4"}, 4),
                      ({"PCMP_HW_QUEUES": "99"}, 32), ({"GPU_MAX_HW_QUEUES": "x"}, 8)):
        e = dict(env)
        assert pcmp.ensure_hw_queues(e) == want
        assert e["GPU_MAX_HW_QUEUES"] == str(want)


def test_weights_flag_loads_torchvision_resnet(tmp_path):
    """--weights PATH on the TL entry point: the torchvision-layout backbone is read with
    torch.load(weights_only=True) and loaded before training (another_neural_net.py:95)."""
    from pcmp.models.torch_ref import TorchResNet
    path = tmp_path / "resnet50.pth"
    torch.save(TorchResNet("resnet50", 1000).state_dict(), path)
    out = _run("another_neural_net.py", "--model", "resnet50", "--train-size", "16", "--image-size", "32",
               "--batch-size", "8", "--epochs", "1", "--num-images", "2", "--weights", str(path))
    assert f"loaded pretrained weights from {path}" in out and "Training time per epoch is" in out

"""Training engine (D1-D11) on flat parameters, fused optimizers and RCCL DDP.

Loops mirror the reference's, with its report strings (Appendix A) on rank 0:
  * ``train_image_classifier`` — the ResNet-50 / VGG16 transfer-learning loops (D6/D7/D8):
    per step zero_grad/forward/NLL(=fused CE)/backward/step; an eval pass every
    ``print_every`` epochs with exp->topk accuracy; "Epoch e/E.. Train loss.. Test loss.. Test
    accuracy.." lines; optional VGG early stopping on validation loss with best-model restore;
    ``torch.save``-style hand-off via ``save_path``; "Training time per epoch is X seconds"
    (the reference's wall time over ALL epochs incl. eval, despite the wording).
  * ``train_text_classifier`` / ``evaluate_text`` — the BERT loop (D9/D10/E4): AdamW(2e-5,
    eps 1e-8) + linear schedule without warm-up, clip_grad_norm 1.0, progress line every 40
    steps, average-loss / epoch-time lines, validation accuracy = mean of per-batch
    ``flat_accuracy``; works for the BiLSTM and BERT models alike.
  * ``keras_fit`` / ``keras_evaluate`` — resnet.py's ``model.fit(train, epochs, validation_data)``
    / timed ``model.evaluate`` (D11/E5) with categorical cross-entropy and SGD(lr=1e-3).
Differences from the reference are deliberate and switchable with ``reference_compat``:
losses are accumulated on device (no per-step ``.item()`` sync), the printed "Train loss" is the
true mean (the reference divides the epoch's loss sum by ``print_every``), the
VGG loop zeroes gradients (§0.2-2).  ``reference_compat=True`` reproduces the printed values.
"""
from __future__ import annotations

import contextlib
import os
import time
from dataclasses import dataclass, field

import torch

from .. import optim as pcmp_optim
from ..ops.functions import cross_entropy
from ..ops.kernels import argmax_rows
from ..parallel.ddp import DistributedDataParallel
from ..parallel.metrics import all_reduce_max, all_reduce_sum
from ..utils import report as R
from ..utils.checkpoint import BestCheckpoint
from ..utils.flat import FlatParams
from ..utils.misc import PriorityStream, StepThrottle, roctx_range, watchdog_kick
from ..utils.timer import PhaseTimer


@dataclass
class TrainState:
    model: torch.nn.Module
    flat: FlatParams
    opt: object
    ddp: DistributedDataParallel | None = None
    sched: object = None
    clip: float | None = None
    history: dict = field(default_factory=lambda: {"train_loss": [], "test_loss": [], "test_acc": []})
    timer: PhaseTimer | None = None   # per-phase device time, PCMP_PHASE_TIMES=1
    throttle: StepThrottle | None = None   # host run-ahead bound (allocator footprint)
    prio: PriorityStream | None = None     # high-priority compute stream for the step
    steps_done: int = 0

    def phase(self, name):
        """Phase bracket: HIP-event device time + a roctx range for rocprofv3 (when timing)."""
        if self.timer is None:
            return contextlib.nullcontext()
        stack = contextlib.ExitStack()
        stack.enter_context(roctx_range(name))
        stack.enter_context(self.timer.phase(name))
        return stack

    def zero_grad(self):
        self.opt.zero_grad()

    def backward_step(self, loss):
        with self.phase("backward"):
            loss.backward()
        if self.ddp is not None:
            # join of the bucket all-reduces overlapped with backward, and the optimizer step issued
            # per bucket as each all-reduce completes (two-phase clip when clipping)
            with self.phase("comm+optimizer"):
                self.ddp.finish_gradient_sync(opt=self.opt, clip=self.clip)
        else:
            with self.phase("optimizer"):
                if self.clip is not None:
                    self.opt.clip_grad_norm(self.clip)
                else:
                    self.opt.set_grad_scale(None)
                self.opt.step()
        if self.sched is not None:
            self.sched.step()
        if self.timer is not None:
            self.timer.step()
        if self.throttle is not None:
            self.throttle.tick()
        self.steps_done += 1
        if self.steps_done == 1:
            # every shape of a full batch has been planned in this first step: all ranks take rank
            # 0's kernels (shapes first seen later are synced at the epoch ends, end_epoch)
            self.end_epoch()
        watchdog_kick("train_step")

    def end_epoch(self):
        """Re-sync the autotuned kernel tables over the ranks when any rank planned new shapes."""
        if self.ddp is not None and self.ddp.world > 1:
            from ..parallel.ddp import sync_autotune_if_grown
            sync_autotune_if_grown(self.ddp.pg)

    def before_eval(self):
        """Every rank evaluates with the ranks' mean BatchNorm running statistics (DDP)."""
        if self.ddp is not None and self.ddp.world > 1:
            self.ddp.average_buffers()

    def phase_report(self, printer=None):
        """Summarise the per-phase device times into ``history['phases']`` (and print one line)."""
        if self.timer is None:
            return None
        summ = self.timer.summary()
        self.history["phases"] = summ
        if printer is not None:
            parts = [f"{k} {v.get('device_ms_mean', 0.0):.3f} ms" for k, v in summ.items()]
            printer("[phase times, device mean per step] " + ", ".join(parts))
        return summ


def make_state(model, optimizer="sgd", lr=0.1, distributed=False, clip=None, shadow_dtype=None, **opt_kw):
    """Flatten trainable params (bf16 shadows on GPU), build the fused optimizer and DDP."""
    params = [p for p in model.parameters() if p.requires_grad]
    dev = params[0].device
    if shadow_dtype is None:   # bf16 weight shadows feed the bf16 kernels; none in fp32 parity mode
        from ..ops import _lib
        shadow_dtype = torch.bfloat16 if _lib.default_compute_dtype(dev) == torch.bfloat16 else None
    flat = FlatParams(params, shadow_dtype=shadow_dtype)
    opt = pcmp_optim.build(optimizer, flat, lr=lr, **opt_kw)
    ddp = DistributedDataParallel(model, flat) if distributed else None
    timer = PhaseTimer(warmup_steps=int(os.environ.get("PCMP_PHASE_WARMUP", "2"))) \
        if os.environ.get("PCMP_PHASE_TIMES") == "1" else None
    return TrainState(model, flat, opt, ddp, clip=clip, timer=timer, throttle=StepThrottle(dev),
                      prio=PriorityStream(dev))


def _logits(model, x):
    return model.forward_logits(x) if hasattr(model, "forward_logits") else model(x)


# ---------------------------------------------------------------------------------- images
@torch.no_grad()
def evaluate_images(model, loader, reference_compat=False):
    """Eval pass: mean NLL per batch and exp->topk(1) accuracy averaged over batches (G4)."""
    model.eval() if not reference_compat else None
    loss_sum, acc_sum, nb = 0.0, 0.0, 0
    dev = None
    losses, accs = [], []
    for x, y in loader:
        watchdog_kick("eval")
        z = _logits(model, x)
        logp = torch.log_softmax(z.float(), dim=1)
        losses.append(torch.nn.functional.nll_loss(logp, y))
        accs.append((argmax_rows(logp) == y).float().mean())
        nb += 1
    if nb:
        loss_sum = float(torch.stack(losses).sum())
        acc_sum = float(torch.stack(accs).sum())
    model.train()
    s = all_reduce_sum([loss_sum, acc_sum, nb])
    nbt = max(1.0, s[2])
    return s[0] / nbt, s[1] / nbt


def train_image_classifier(state: TrainState, trainloader, testloader, epochs=1, print_every=1,
                           early_stopping_patience=None, save_fn=None, verbose_steps=False,
                           reference_compat=False, printer=R.rprint):
    model = state.model
    model.train()
    t1 = time.time()
    best = BestCheckpoint("min") if early_stopping_patience else None
    epochs_no_improve = 0
    steps = 0
    running = torch.zeros((), dtype=torch.float64, device=state.flat.device)
    n_in_window = 0
    for epoch in range(epochs):
        if hasattr(trainloader, "set_epoch") and not reference_compat:
            trainloader.set_epoch(epoch)
        it = iter(trainloader)
        while True:
            with state.phase("data"):
                batch = next(it, None)
            if batch is None:
                break
            x, y = batch
            steps += 1
            if verbose_steps:
                printer(steps)
            with (state.prio.step(x, y) if state.prio is not None else contextlib.nullcontext()):
                state.zero_grad()
                with state.phase("forward"):
                    loss = cross_entropy(_logits(model, x), y)
                state.backward_step(loss)
                running += loss.detach().double()
            n_in_window += 1
        printer(R.TRAINLOADER_DONE)
        state.end_epoch()
        if (epoch % print_every) == 0 or epoch == epochs - 1:
            state.before_eval()
            test_loss, test_acc = evaluate_images(model, testloader, reference_compat)
            tot = all_reduce_sum([float(running), n_in_window])
            train_loss = tot[0] / print_every if reference_compat else tot[0] / max(1.0, tot[1])
            state.history["train_loss"].append(train_loss)
            state.history["test_loss"].append(test_loss)
            state.history["test_acc"].append(test_acc)
            printer(R.epoch_line(epoch + 1, epochs, train_loss, test_loss, test_acc))
            running.zero_()
            n_in_window = 0
            if best is not None:
                if best.update(test_loss, model):
                    epochs_no_improve = 0
                    if save_fn is not None:
                        printer(R.SAVING_MODEL)
                        save_fn(model)
                else:
                    epochs_no_improve += 1
                    if epochs_no_improve >= early_stopping_patience:
                        printer(R.EARLY_STOPPING)
                        best.restore(model)
                        break
    if save_fn is not None and best is None:
        printer(R.SAVING_MODEL)
        save_fn(model)
    elapsed = all_reduce_max(time.time() - t1)
    printer(R.training_time_line(elapsed))
    state.phase_report(printer)
    return elapsed


# ---------------------------------------------------------------------------------- text
def train_text_classifier(state: TrainState, train_loader, val_loader=None, epochs=3, print_batches=False,
                          progress_every=40, printer=R.rprint, graph=False):
    """The reference's BERT / text training loop (pytorch_on_language_distr.py:219-335).  ``graph``:
    replay each full-size batch's step from one captured hipGraph (:class:`pcmp.engine.graph.
    GraphedStep`; single process, GPU); other batch shapes run eagerly."""
    model = state.model
    times = []
    graphed = None
    use_graph = bool(graph) and state.ddp is None and state.flat.device.type == "cuda"

    def loss_of(ids, mask, labels):
        return model(ids, None, mask, labels)[0] if _is_bert(model) else cross_entropy(
            model.forward_logits(ids, mask), labels)
    for epoch_i in range(epochs):
        printer("")
        printer(R.text_epoch_header(epoch_i, epochs))
        printer(R.TRAINING)
        t0 = time.time()
        if hasattr(train_loader, "set_epoch"):
            train_loader.set_epoch(epoch_i)
        total = torch.zeros((), dtype=torch.float64, device=state.flat.device)
        n = 0
        model.train()
        nsteps = len(train_loader)
        for step, batch in enumerate(train_loader):
            if print_batches:
                printer(R.PRINTED_BATCH)
                printer(batch)
            if step % progress_every == 0 and not step == 0:
                printer(R.batch_progress_line(step, nsteps, R.format_time(time.time() - t0)))
            ids, mask, labels = batch
            if use_graph and graphed is None:
                from .graph import GraphedStep
                graphed = GraphedStep(state, loss_of, [ids, mask, labels])
            if graphed is not None and graphed.matches(ids, mask, labels):
                loss = graphed(ids, mask, labels)
                total += loss.double()
                n += 1
                watchdog_kick("train_step")
                continue
            state.zero_grad()
            with state.phase("forward"):
                loss = loss_of(ids, mask, labels)
            total += loss.detach().double()
            n += 1
            state.backward_step(loss)
        state.end_epoch()
        avg = all_reduce_sum([float(total), n])
        avg_train_loss = avg[0] / max(1.0, avg[1])
        state.history["train_loss"].append(avg_train_loss)
        printer("")
        printer(R.avg_train_loss_line(avg_train_loss))
        took = all_reduce_max(time.time() - t0)
        times.append(took)
        printer(R.epoch_took_line(R.format_time(took)))
        if val_loader is not None:
            printer("")
            printer(R.RUNNING_VALIDATION)
            t0 = time.time()
            acc = evaluate_text(model, val_loader)
            printer(R.val_accuracy_line(acc))
            printer(R.val_took_line(R.format_time(time.time() - t0)))
    printer("")
    printer(R.TRAINING_COMPLETE)
    state.phase_report(printer)
    return times


def _is_bert(model):
    from ..models.bert import BertForSequenceClassification
    m = model.module if hasattr(model, "module") else model
    return isinstance(m, BertForSequenceClassification)


@torch.no_grad()
def evaluate_text(model, loader):
    """Mean over batches of flat_accuracy (pytorch_on_language_distr.py:296-333)."""
    model.eval()
    accs = []
    for ids, mask, labels in loader:
        watchdog_kick("eval")
        z = model.forward_logits(ids, mask)
        accs.append((argmax_rows(z) == labels).float().mean())
    model.train()
    s = all_reduce_sum([float(torch.stack(accs).sum()) if accs else 0.0, len(accs)])
    return s[0] / max(1.0, s[1])


def test_text(model, loader, printer=R.rprint):
    """E4: 'Accuracy: {:.4f}' + 'Test took: h:mm:ss'."""
    t0 = time.time()
    acc = evaluate_text(model, loader)
    printer(R.test_accuracy_line(acc))
    printer(R.test_took_line(R.format_time(time.time() - t0)))
    return acc


# ---------------------------------------------------------------------------------- keras
def keras_fit(state: TrainState, train, val=None, epochs=5, printer=R.rprint):
    """model.fit(train, epochs, validation_data=val) with categorical CE (resnet.py:24-25)."""
    from ..models.keras_resnet import categorical_crossentropy
    hist = []
    for e in range(epochs):
        t0 = time.time()
        tot, correct, n = 0.0, 0.0, 0
        for x, y in train:
            onehot = torch.nn.functional.one_hot(y, state.model.num_classes).float()
            state.zero_grad()
            z = state.model.forward_logits(x)
            loss = categorical_crossentropy(z, onehot)
            state.backward_step(loss)
            tot += float(loss) * y.numel()
            correct += float((argmax_rows(z) == y).sum())
            n += y.numel()
        rec = {"epoch": e + 1, "loss": tot / max(1, n), "accuracy": correct / max(1, n), "time_s": time.time() - t0}
        if val is not None:
            rec["val_loss"], rec["val_accuracy"] = keras_evaluate(state.model, val, timed=False)
        printer(f"Epoch {e + 1}/{epochs} - {rec['time_s']:.0f}s - loss: {rec['loss']:.4f} - accuracy: "
                f"{rec['accuracy']:.4f}" + (f" - val_loss: {rec['val_loss']:.4f} - val_accuracy: "
                                             f"{rec['val_accuracy']:.4f}" if val is not None else ""))
        hist.append(rec)
    return hist


@torch.no_grad()
def keras_evaluate(model, val, timed=True, printer=R.rprint):
    t1 = time.time()
    model.eval()
    tot, correct, n = 0.0, 0.0, 0
    for x, y in val:
        watchdog_kick("eval")
        z = model.forward_logits(x).float()
        tot += float(torch.nn.functional.cross_entropy(z, y, reduction="sum"))
        correct += float((argmax_rows(z) == y).sum())
        n += y.numel()
    model.train()
    if timed:
        printer(R.keras_inference_line(time.time() - t1))
    return tot / max(1, n), correct / max(1, n)

"""Whole-training-step hipGraph capture (HIP graphs instead of a tracing compiler).

A pcmp training step (forward, loss, backward, gradient clipping, fused optimizer update) is a
fixed sequence of kernel launches for fixed input shapes.  :class:`GraphedStep` records that
sequence once into a hipGraph and replays it: the host then issues one graph launch per step
instead of several hundred kernel launches through the Python autograd engine.  For launch-bound
models this removes the host from the critical path -- BERT-base trains ~400 small kernels per
step and idled 26 % of the trace between them in eager mode (profiles/r2_rocprof_bert_no_hipblaslt.txt).

What makes a replayed step equal to an eager one:
  * every planner / autotune decision is taken in the eager warm-up steps before capture (the
    kernels never autotune while a capture is active);
  * dropout: the captured kernels read a device-side salt (``dropout_rng.salt``) that the captured
    step itself increments, so each replay draws fresh masks (arguments are frozen at capture);
  * the learning-rate schedule runs OUTSIDE the graph between replays (``opt.set_lr`` writes the
    device scalar the captured optimizer kernel reads); Adam's step count and the clipping
    coefficient already live on the device;
  * the warm-up steps' parameter / optimizer / buffer updates are undone (snapshot and restore),
    so training with a graph starts from the same state as without.

Reference: the reference's BERT loop (pytorch_on_language_distr.py:244-275) calls zero_grad /
forward / backward / clip / step / scheduler.step per batch; :meth:`GraphedStep.__call__` is that
body for one batch.  Inputs of another shape (an epoch's last partial batch) run eagerly.
"""
from __future__ import annotations

import torch

from ..ops.functions import dropout_rng
from ..ops.params import bump_weight_gen


class GraphedStep:
    def __init__(self, state, loss_fn, example_inputs, warmup: int = 2):
        """``state``: a :class:`pcmp.engine.trainer.TrainState` (single process: no DDP);
        ``loss_fn(*inputs)`` -> scalar loss (the forward + loss of one batch);
        ``example_inputs``: device tensors of the shapes to capture for."""
        assert state.ddp is None, "GraphedStep: collectives are not captured (single-process steps only)"
        self.state = state
        self.loss_fn = loss_fn
        self.static = [t.detach().clone() for t in example_inputs]
        self.shapes = [tuple(t.shape) for t in self.static]
        self.device = self.static[0].device
        self.salt = torch.zeros(1, dtype=torch.int64, device=self.device)
        self.replays = 0
        snap = self._snapshot()
        sched, state.sched = state.sched, None     # the schedule runs outside the graph
        timer, state.timer = state.timer, None     # per-phase event timing is an eager-mode tool
        try:
            side = torch.cuda.Stream(self.device)
            side.wait_stream(torch.cuda.current_stream(self.device))
            with torch.cuda.stream(side):
                for _ in range(max(1, warmup)):
                    self._body()
            torch.cuda.current_stream(self.device).wait_stream(side)
            torch.cuda.synchronize(self.device)
            self._restore(snap)
            self.graph = torch.cuda.CUDAGraph()
            prev = dropout_rng.salt
            dropout_rng.salt = self.salt
            try:
                with torch.cuda.graph(self.graph, capture_error_mode="thread_local"):   # see inference.py
                    self.loss = self._body()
                    self.salt.add_(1)
            finally:
                dropout_rng.salt = prev
        finally:
            state.sched = sched
            state.timer = timer

    # ------------------------------------------------------------------------------------------
    def _body(self):
        st = self.state
        st.zero_grad()
        loss = self.loss_fn(*self.static)
        st.backward_step(loss)
        return loss.detach()

    def _snapshot(self):
        st = self.state
        ts = [st.flat.master]
        if st.flat.shadow is not None:
            ts.append(st.flat.shadow)
        ts += list(st.opt._state().values())
        ts += [b for b in st.model.buffers()]
        return [(t, t.detach().clone()) for t in ts]

    @staticmethod
    def _restore(snap):
        with torch.no_grad():
            for t, c in snap:
                t.copy_(c)

    def matches(self, *inputs) -> bool:
        return all(tuple(t.shape) == s for t, s in zip(inputs, self.shapes))

    def __call__(self, *inputs):
        """One training step on ``inputs`` (copied into the captured buffers); returns the loss
        (a device tensor, valid until the next call)."""
        for s, t in zip(self.static, inputs):
            s.copy_(t, non_blocking=True)
        self.graph.replay()
        self.replays += 1
        bump_weight_gen()          # the captured optimizer moved the weights (derived caches key on it)
        st = self.state
        if st.sched is not None:
            st.sched.step()
        if st.throttle is not None:
            st.throttle.tick()
        return self.loss

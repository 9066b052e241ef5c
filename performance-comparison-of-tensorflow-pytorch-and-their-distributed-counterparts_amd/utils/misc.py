"""Seeding, profiling hooks (§5.1) and a hang watchdog (§5.3)."""
from __future__ import annotations

import contextlib
import faulthandler
import os
import random
import sys
import threading
import time

import numpy as np
import torch


def seed_everything(seed: int = 42):
    """pytorch_on_language_distr.py:210-217 — random, numpy, torch, cuda seeds (+ dropout RNG)."""
    random.seed(seed)
    np.random.seed(seed)
    torch.manual_seed(seed)
    if torch.cuda.is_available():
        torch.cuda.manual_seed_all(seed)
    from ..ops.functions import dropout_rng
    dropout_rng.reseed(seed)


@contextlib.contextmanager
def roctx_range(name: str):
    """Named range visible to rocprofv3 (--marker-trace) / torch.profiler; no-op on CPU."""
    pushed = False
    if torch.cuda.is_available():
        try:
            torch.cuda.nvtx.range_push(name)
            pushed = True
        except Exception:
            pushed = False
    try:
        yield
    finally:
        if pushed:
            torch.cuda.nvtx.range_pop()


@contextlib.contextmanager
def chrome_trace(path: str | None):
    """``--profile PATH``: torch.profiler (ROCm activity via roctracer) -> Chrome trace."""
    if not path:
        yield None
        return
    acts = [torch.profiler.ProfilerActivity.CPU]
    if torch.cuda.is_available():
        acts.append(torch.profiler.ProfilerActivity.CUDA)
    with torch.profiler.profile(activities=acts, record_shapes=False) as prof:
        yield prof
    prof.export_chrome_trace(path)


class Watchdog:
    """Dumps the current step/phase and all Python stacks if no ``kick()`` for ``timeout_s``,
    then (optionally) aborts the process so a dead rank does not hang the job."""

    def __init__(self, timeout_s: float = 600.0, abort: bool = False, stream=sys.stderr):
        self.timeout = timeout_s
        self.abort = abort
        self.stream = stream
        self.last = time.monotonic()
        self.state = {"step": -1, "phase": "init"}
        self._stop = threading.Event()
        self._t = threading.Thread(target=self._run, daemon=True)

    def start(self):
        self._t.start()
        return self

    def kick(self, step=None, phase=None):
        self.last = time.monotonic()
        if step is not None:
            self.state["step"] = step
        if phase is not None:
            self.state["phase"] = phase

    def stop(self):
        self._stop.set()

    def _run(self):
        while not self._stop.wait(min(5.0, self.timeout / 4)):
            if time.monotonic() - self.last > self.timeout:
                print(f"[watchdog] no progress for {self.timeout:.0f}s at step={self.state['step']} "
                      f"phase={self.state['phase']} (rank {os.environ.get('RANK', '0')})", file=self.stream, flush=True)
                faulthandler.dump_traceback(file=self.stream)
                if self.abort:
                    os._exit(3)
                self.last = time.monotonic()

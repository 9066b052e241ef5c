"""Device-accurate timers.

The reference times whole phases with ``time.time()`` and no device synchronisation (G1). We keep
that wall-clock number (it is what the report strings print) and add:
  * ``PhaseTimer`` — per-phase device time from HIP events (data / forward / backward / comm /
    optimizer), warm-up exclusion, per-step summaries;
  * ``sync_time()`` — wall time with a device synchronize fence (what a clean throughput
    number needs).
"""
from __future__ import annotations

import contextlib
import time
from collections import defaultdict

import torch


def synchronize(device=None):
    if torch.cuda.is_available() and (device is None or torch.device(device).type == "cuda"):
        torch.cuda.synchronize(device)


def sync_time(device=None) -> float:
    synchronize(device)
    return time.perf_counter()


class PhaseTimer:
    """``with timer.phase("forward"): ...`` records HIP events; ``summary()`` syncs once."""

    def __init__(self, enabled=True, warmup_steps=0, device=None):
        self.enabled = enabled and torch.cuda.is_available()
        self.warmup = warmup_steps
        self.step_idx = 0
        self.events = defaultdict(list)
        self.cpu = defaultdict(float)
        self.device = device

    @contextlib.contextmanager
    def phase(self, name):
        if self.step_idx < self.warmup:
            yield
            return
        t0 = time.perf_counter()
        if self.enabled:
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            try:
                yield
            finally:
                e.record()
                self.events[name].append((s, e))
                self.cpu[name] += time.perf_counter() - t0
        else:
            try:
                yield
            finally:
                self.cpu[name] += time.perf_counter() - t0

    def step(self):
        self.step_idx += 1

    def summary(self) -> dict:
        out = {}
        if self.enabled:
            synchronize()
            for k, evs in self.events.items():
                ms = [s.elapsed_time(e) for s, e in evs]
                out[k] = {"device_ms_total": sum(ms), "device_ms_mean": sum(ms) / max(1, len(ms)), "n": len(ms)}
        for k, v in self.cpu.items():
            out.setdefault(k, {})["host_s_total"] = v
        return out

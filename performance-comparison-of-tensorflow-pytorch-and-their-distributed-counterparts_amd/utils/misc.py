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


_ACTIVE_WATCHDOG = None


def watchdog_kick(phase: str | None = None) -> None:
    """Progress heartbeat from the training / eval / inference loops (no-op without ``--watchdog``)."""
    wd = _ACTIVE_WATCHDOG
    if wd is not None:
        wd.kick(wd.state["step"] + 1, phase)


class Watchdog:
    """Dumps the current step/phase and all Python stacks if no ``kick()`` for ``timeout_s``,
    then (optionally) aborts the process so a dead rank does not hang the job.

    The reference's runs that hung were stopped by hand (``KeyboardInterrupt``,
    Standalone_Inference_Imagenette_trial.ipynb:119-120); ``--watchdog SECONDS`` on every entry
    point starts one of these (``abort=True`` under DDP: a rank stuck in a collective exits with
    status 3, and the launcher tears the job down instead of hanging).  The engine loops kick it
    through :func:`watchdog_kick` once per step / batch / image."""

    def __init__(self, timeout_s: float = 600.0, abort: bool = False, stream=sys.stderr):
        self.timeout = timeout_s
        self.abort = abort
        self.stream = stream
        self.last = time.monotonic()
        self.state = {"step": 0, "phase": "init"}   # step = kicks so far
        self._stop = threading.Event()
        self._t = threading.Thread(target=self._run, daemon=True)
        self._exit = os._exit            # replaceable in tests

    def start(self):
        global _ACTIVE_WATCHDOG
        self.last = time.monotonic()
        self._t.start()
        _ACTIVE_WATCHDOG = self
        return self

    def kick(self, step=None, phase=None):
        self.last = time.monotonic()
        if step is not None:
            self.state["step"] = step
        if phase is not None:
            self.state["phase"] = phase

    def stop(self):
        global _ACTIVE_WATCHDOG
        self._stop.set()
        if _ACTIVE_WATCHDOG is self:
            _ACTIVE_WATCHDOG = None

    def __enter__(self):
        return self.start()

    def __exit__(self, *exc):
        self.stop()
        return False

    def _run(self):
        while not self._stop.wait(min(5.0, self.timeout / 4)):
            if time.monotonic() - self.last > self.timeout:
                print(f"[watchdog] no progress for {self.timeout:.0f}s at step={self.state['step']} "
                      f"phase={self.state['phase']} (rank {os.environ.get('RANK', '0')})", file=self.stream, flush=True)
                try:
                    _dump_stacks(self.stream)
                except Exception as e:   # never let a reporting failure skip the abort below
                    try:
                        print(f"[watchdog] stack dump failed: {e!r}", file=sys.__stderr__, flush=True)
                    except Exception:
                        pass
                if self.abort:
                    self._exit(3)
                self.last = time.monotonic()


def _dump_stacks(stream) -> None:
    """All Python thread stacks to ``stream``: faulthandler when the stream has a real file
    descriptor (works even with the GIL held by a stuck thread), else formatted frames (StringIO,
    pytest capture, notebook streams, which have no ``fileno``)."""
    try:
        stream.fileno()
        has_fd = True
    except (AttributeError, OSError, ValueError):
        has_fd = False
    if has_fd:
        stream.flush()
        faulthandler.dump_traceback(file=stream)
        return
    import traceback
    for tid, frame in sys._current_frames().items():
        stream.write(f"Thread 0x{tid:x} (most recent call last):\n")
        stream.write("".join(traceback.format_stack(frame)))
    stream.flush()


def _env_int(name: str, default: int) -> int:
    """Integer environment knob; a malformed value warns and falls back instead of raising deep
    inside a training loop."""
    raw = os.environ.get(name)
    if raw is None or raw.strip() == "":
        return default
    try:
        return int(raw)
    except ValueError:
        print(f"[pcmp] ignoring {name}={raw!r} (not an integer); using {default}", file=sys.stderr)
        return default


class StepThrottle:
    """Bounds how many training steps the host may enqueue ahead of the GPU.

    Nothing in a pcmp step synchronises the host (losses stay on device), so the host, which needs
    8-15 ms to enqueue a ResNet-50 step that takes the GPU 22 ms, runs further and further ahead.
    Every tensor freed on the host while its kernels are still queued (and every ``record_stream``
    on the WGRAD side stream) keeps its block out of the caching allocator until the GPU catches
    up, so the allocator keeps reserving fresh segments: 83 GiB reserved for a 10.7 GiB peak at
    B=256, 221 GiB at B=1024 (``profiles/r1_alloc_ab.txt``), a few steps away from the 288 GB of
    HBM.  ``tick()`` after each step records an event on the current stream and, once more than
    ``depth`` steps are in flight, waits for the oldest; with depth 2 the GPU still always has a
    whole step queued.  ``PCMP_MAX_INFLIGHT`` overrides the depth (0 disables).  No-op on CPU.

    The bound is on run-ahead, not on fragmentation: at depth 2 the allocator still reserves about
    3.4x the live peak (B=256: 36.9 GiB reserved for a 10.7 GiB peak; B=1024: 145 GiB for 41.5 GiB,
    ``profiles/r1_throttle_ab.txt``) because blocks recorded on the WGRAD side stream and the
    comm stream are reusable only once those streams pass them.  Depth 1 cuts B=256 to 25.9 GiB
    at unchanged throughput (``profiles/r1_inflight_depth_ab.txt``); depth 2 stays the default as
    margin for slower or contended hosts (8 ranks enqueueing on one node).  The wait uses a
    blocking event, so a throttled rank sleeps instead of spinning a core that the data loader
    and RCCL's proxy threads need."""

    def __init__(self, device=None, depth: int | None = None):
        if depth is None:
            depth = _env_int("PCMP_MAX_INFLIGHT", 2)
        self.depth = max(0, int(depth))
        self.device = torch.device(device) if device is not None else None
        self._events = []

    def tick(self) -> None:
        if self.depth <= 0 or self.device is None or self.device.type != "cuda":
            return
        if torch.cuda.is_current_stream_capturing():
            return
        ev = torch.cuda.Event(blocking=True)
        ev.record(torch.cuda.current_stream(self.device))
        self._events.append(ev)
        while len(self._events) > self.depth:
            self._events.pop(0).synchronize()

    @property
    def in_flight(self) -> int:
        return len(self._events)


class PriorityStream:
    """High-priority HIP stream for a training step's compute work.

    The conv WGRADs (and the downsample branch) run on a side stream concurrently with the
    DGRAD / BatchNorm chain, which is the critical path of a ResNet step.  Issuing the step itself
    on a high-priority queue makes the command processor dispatch the critical path's workgroups
    first whenever CUs free up: ResNet-50 B=256 +1.2 % (profiles/r3_prio_pf2_ab.txt).
    ``with ps.step(x, y):`` runs a step on it (the inputs, produced on the caller's stream, are
    waited for and recorded on it; the caller's stream waits for the step at the end).  No-op on
    CPU or with ``PCMP_STEP_PRIO=0``."""

    def __init__(self, device=None):
        dev = torch.device(device) if device is not None else None
        on = dev is not None and dev.type == "cuda" and os.environ.get("PCMP_STEP_PRIO", "1") == "1"
        self.stream = torch.cuda.Stream(dev, priority=-1) if on else None

    @contextlib.contextmanager
    def step(self, *tensors):
        if self.stream is None or torch.cuda.is_current_stream_capturing():
            yield
            return
        cur = torch.cuda.current_stream(self.stream.device)
        self.stream.wait_stream(cur)
        for t in tensors:
            if isinstance(t, torch.Tensor) and t.is_cuda:
                t.record_stream(self.stream)
        with torch.cuda.stream(self.stream):
            yield
        cur.wait_stream(self.stream)


"""Data-parallel gradient synchronisation over RCCL (xGMI), bucketed and overlapped with backward.

Reference: the reference's DDP wrap is commented out (pytorch_on_language_distr.py:220-221), so
its "distributed" runs are independent replicas.  This module is the gradient-
synchronised data parallelism the north star asks for:

* gradients live in ONE flat fp32 buffer (:class:`pcmp.utils.flat.FlatParams`, reverse
  registration order), so a bucket is a contiguous slice — the all-reduce runs in place on it,
  no pack/unpack copies;
* the wgrad kernels announce each finished parameter (``p._grad_ready_hook``); when the last
  parameter of a bucket is written, the bucket's ``all_reduce(SUM, async_op=True)`` is issued.
  ProcessGroupNCCL (RCCL on ROCm) orders its internal stream after the compute stream at the
  moment of the call, so the collective overlaps with the remaining backward kernels;
* buckets are launched strictly in index order on every rank (collective order must match);
* bucket sizing for 7 point-to-point xGMI links per MI355X: a small first bucket (default 4 MB)
  so communication starts early in backward, then 32 MB buckets so each of RCCL's per-link
  channel chunks stays >= ~256 KB at world 8, and a small LAST bucket (default
  4 MB): the last bucket's all-reduce cannot overlap anything (it waits for the stem's gradient,
  the end of backward), so only a few MB stay exposed instead of up to a whole 32 MB bucket;
* a parameter larger than a bucket (BERT's 23.4 M-element word embedding: 94 MB fp32) is split
  into bucket-sized chunks (``split_param_mb``, default max(bucket, 8 MB)), each its own bucket, so its all-reduce streams in pieces instead of one
  94 MB collective that nothing after it can overlap;
* the optimizer runs PER BUCKET (``finish_gradient_sync(opt=...)``): each bucket's slice of the flat
  arena is updated by the fused optimizer kernel on the comm stream as soon as that bucket's
  all-reduce completes, overlapping the later buckets' collectives, instead of one update after the
  last bucket.  With global-norm clipping the sum of squares is the per-bucket part (two-phase clip:
  per-bucket partial sums as the collectives complete, then one coefficient and one update);
* the 1/world averaging is folded into the optimizer kernel's gradient scale (no extra pass);
* initial parameters and buffers are broadcast from rank 0 (DDP constructor semantics);
  ``broadcast_buffers="forward"`` (or ``True``) re-broadcasts the buffers (BatchNorm running
  statistics) from rank 0 at every forward as torch DDP does, as ONE coalesced broadcast per dtype;
  the default ``"init"`` broadcasts them at construction only (running statistics do not enter a
  training-mode forward) and :meth:`average_buffers` all-reduces them before an evaluation, so a
  per-rank eval aggregated by ``parallel/metrics.py`` uses one set of statistics.

Stream ordering (MI355X: compute stream + WGRAD side stream + RCCL's internal stream):

* every gradient-ready hook notes the HIP stream that wrote the gradient (the conv WGRADs run on
  the side stream, BN gamma/beta and Linear grads on the compute stream);
* when a bucket completes, an event is recorded on each stream that contributed to it and a
  dedicated COMM stream waits on exactly those events; the collective is issued with the comm
  stream current, so RCCL's stream orders after the comm stream only.  The compute stream never
  waits for the WGRAD stream (or for communication) before the end of backward;
* ``finish_gradient_sync`` makes the comm stream wait for every collective and the compute
  stream wait for the comm stream once, right before the optimizer;
* ``grad_dtype=torch.bfloat16`` all-reduces a bf16 copy of each bucket (cast on the comm stream,
  half the xGMI bytes) and casts the sum back into the fp32 gradient; fp32 (default) is exact;
* ``force=True`` (``PCMP_DDP_FORCE=1``) issues every bucket's collective even at world size 1,
  so the RCCL path (process group, comm stream, events, casts) runs on a one-GPU box.
"""
from __future__ import annotations

import collections
import contextlib
import os
import time

import torch
import torch.distributed as dist

from ..ops.kernels import K
from ..ops.ref import sumsq_blocks as _sumsq_blocks
from ..utils.flat import FlatParams


class _Bucket:
    __slots__ = ("index", "start", "end", "params", "pending", "work", "launched", "streams", "events", "t_launch",
                 "part_off")

    def __init__(self, index, start, end, params):
        self.index, self.start, self.end, self.params = index, start, end, params
        self.part_off = 0       # first row of this bucket's sum-of-squares partials (two-phase clip)
        self.pending = len(params)
        self.work = None
        self.launched = False
        self.streams = {}       # stream id -> stream that wrote a gradient of this bucket this step
        self.events = {}        # stream id -> reusable event (recorded when the bucket launches)
        self.t_launch = None    # timing: comm-stream event (GPU) / host seconds (CPU) at launch


def plan_segments(sizes, max_elems, quantum=1024):
    """Per-parameter segments (param index, lo, hi) in arena order: a slice larger than ``max_elems``
    is split into equal chunks (multiples of ``quantum`` elements: vector-aligned sub-slices for the
    fused optimizer kernels), every other slice is one segment."""
    segs = []
    for i, n in enumerate(sizes):
        if max_elems > 0 and n > max_elems:
            k = -(-n // max_elems)
            step = -(-(-(-n // k)) // quantum) * quantum
            lo = 0
            while lo < n:
                hi = min(n, lo + step)
                segs.append((i, lo, hi))
                lo = hi
        else:
            segs.append((i, 0, n))
    return segs


def plan_buckets(sizes, first_bucket_elems, bucket_elems, last_bucket_elems=0):
    """Greedy contiguous bucketing of consecutive slices -> list of [i0, i1) param index ranges.
    With ``last_bucket_elems`` the trailing slices (the last gradients backward produces) are split
    off first into a tail bucket of about that size."""
    tail = None
    if last_bucket_elems > 0 and len(sizes) > 1:
        acc, j = 0, len(sizes)
        while j > 1 and acc < last_bucket_elems:
            j -= 1
            acc += sizes[j]
        if acc < sum(sizes):
            tail, sizes = (j, len(sizes)), sizes[:j]
    out = _plan_greedy(sizes, first_bucket_elems, bucket_elems)
    if tail is not None:
        out.append(tail)
    return out


def _plan_greedy(sizes, first_bucket_elems, bucket_elems):
    out, i0, acc = [], 0, 0
    cap = first_bucket_elems
    for i, n in enumerate(sizes):
        acc += n
        if acc >= cap:
            out.append((i0, i + 1))
            i0, acc, cap = i + 1, 0, bucket_elems
    if i0 < len(sizes):
        out.append((i0, len(sizes)))
    return out


class DistributedDataParallel(torch.nn.Module):
    TIMED_STEPS_KEPT = 256   # time_exposed keeps the most recent timed steps' events

    def __init__(self, module: torch.nn.Module, flat: FlatParams, process_group=None, bucket_cap_mb: float = 32.0,
                 first_bucket_mb: float = 4.0, broadcast_buffers: bool | str = "init", average: bool = True,
                 last_bucket_mb: float = 4.0, force: bool | None = None, grad_dtype: torch.dtype | str | None = None,
                 split_param_mb: float | None = None):
        super().__init__()
        self.module = module
        self.flat = flat
        self.pg = process_group
        self.world = dist.get_world_size(process_group) if dist.is_initialized() else 1
        self.average = average
        self.require_sync = True
        if force is None:
            force = os.environ.get("PCMP_DDP_FORCE") == "1"
        # collectives are issued when there is a peer, or when forced (one-GPU exercise of RCCL)
        self.active = dist.is_initialized() and (self.world > 1 or bool(force))
        self.grad_dtype = _parse_dtype(grad_dtype if grad_dtype is not None
                                       else os.environ.get("PCMP_DDP_GRAD_DTYPE"))
        self._comm_stream = None
        self._lowp = None
        if self.active and flat.grad.is_cuda:
            # one comm stream per DDP instance; high priority so its short cast kernels and RCCL's
            # stream hand-offs are not queued behind long conv grids
            self._comm_stream = torch.cuda.Stream(flat.grad.device, priority=-1)
            if self.grad_dtype != torch.float32:
                self._lowp = torch.empty(flat.grad.numel(), dtype=self.grad_dtype, device=flat.grad.device)
        elif self.grad_dtype != torch.float32 and self.active:
            self._lowp = torch.empty(flat.grad.numel(), dtype=self.grad_dtype, device=flat.grad.device)
        esz = flat.grad.element_size()
        sizes = []
        offs = flat.offsets + [flat.numel]
        for i in range(len(flat.params)):
            sizes.append(offs[i + 1] - offs[i])
        cap = int(bucket_cap_mb * 2 ** 20 / esz)
        # parameters above max(bucket, 8 MB) are chunked (never into collectives smaller than 8 MB
        # unless asked: a tiny test bucket must not turn every conv filter into dozens of buckets)
        split = int((split_param_mb if split_param_mb is not None else max(bucket_cap_mb, 8.0)) * 2 ** 20 / esz)
        segs = plan_segments(sizes, split)
        ranges = plan_buckets([hi - lo for _, lo, hi in segs], int(first_bucket_mb * 2 ** 20 / esz), cap,
                              int(last_bucket_mb * 2 ** 20 / esz))
        self.buckets = []
        self._bucket_of = {}     # id(param) -> the buckets holding (a chunk of) its gradient
        nparts = 0
        for bi, (s0, s1) in enumerate(ranges):
            pis = sorted({segs[k][0] for k in range(s0, s1)})
            ps = [flat.params[i] for i in pis]
            b = _Bucket(bi, offs[segs[s0][0]] + segs[s0][1], offs[segs[s1 - 1][0]] + segs[s1 - 1][2], ps)
            b.part_off = nparts
            nparts += _sumsq_blocks(b.end - b.start)
            self.buckets.append(b)
            for p in ps:
                self._bucket_of.setdefault(id(p), []).append(b)
        self._nparts = nparts
        self._parts = None       # sum-of-squares partial rows of every bucket (two-phase clip)
        self._scale_t = None     # device scalar 1/world (optimizer gradient scale)
        self._opt_in_tail = False   # the optimizer ran per bucket inside finish_gradient_sync
        for p in flat.params:
            p._grad_ready_hook = self._on_grad_ready
        self._next_launch = 0
        self._timing = False
        # per step: (compute-done event, comm-done event) or host seconds / [(bucket, launch, done)]
        # events (GPU) or seconds vs finish (CPU); the last TIMED_STEPS_KEPT steps (time_exposed)
        self._exposed = collections.deque(maxlen=self.TIMED_STEPS_KEPT)
        self._timeline = collections.deque(maxlen=self.TIMED_STEPS_KEPT)
        self._tl_stream = None
        self._ev_ref = None
        if broadcast_buffers is True:
            broadcast_buffers = "forward"
        if broadcast_buffers not in (False, "init", "forward"):
            raise ValueError(f"broadcast_buffers: True / 'forward', 'init' or False, not {broadcast_buffers!r}")
        self.buffer_mode = broadcast_buffers
        if self.world > 1:
            self._broadcast_state(broadcast_buffers is not False)

    # ------------------------------------------------------------------------------------------
    def time_exposed(self, on: bool = True):
        """Record, per step, how long the optimizer waits for communication after backward: from
        the compute stream reaching ``finish_gradient_sync`` to the last collective (and its bf16
        cast-back) finishing on the comm stream.  CUDA events (no host sync); host seconds on CPU."""
        self._timing = bool(on)
        # the most recent timed steps only (each holds CUDA events until comm_report): a long timed
        # run keeps a bounded number of events alive
        self._exposed = collections.deque(maxlen=self.TIMED_STEPS_KEPT)
        self._timeline = collections.deque(maxlen=self.TIMED_STEPS_KEPT)
        if on and self._comm_stream is not None and self._tl_stream is None:
            self._tl_stream = torch.cuda.Stream(self.flat.grad.device)

    def comm_report(self) -> dict:
        """Bucket plan + exposed communication time (mean/max ms over the timed steps) + a per-bucket
        timeline: when each bucket's all-reduce was launched and when it completed, in ms relative
        to the end of backward (the compute stream reaching ``finish_gradient_sync``; negative =
        before it), averaged over the timed steps, with the bytes each bucket moves."""
        esz = self.flat.grad.element_size()
        wsz = torch.tensor([], dtype=self.grad_dtype).element_size()
        rep = {"active": bool(self.active), "world": self.world, "buckets": len(self.buckets),
               "bucket_mb": [round((b.end - b.start) * esz / 2 ** 20, 2) for b in self.buckets],
               "grad_allreduce_dtype": str(self.grad_dtype).replace("torch.", ""),
               # exposed_ms then spans end of backward -> last bucket's update (comm + optimizer tail)
               "optimizer_per_bucket": bool(self._opt_in_tail)}
        vals = []
        for e in self._exposed:
            if isinstance(e, tuple):
                e[1].synchronize()
                vals.append(max(0.0, e[0].elapsed_time(e[1])))
            else:
                vals.append(e * 1e3)
        if vals:
            rep["exposed_ms"] = round(sum(vals) / len(vals), 4)
            rep["exposed_ms_max"] = round(max(vals), 4)
            rep["timed_steps"] = len(vals)
        acc = {}
        for step in self._timeline:
            for bi, lt, dt in step:
                a = acc.setdefault(bi, [0.0, 0.0, 0])
                a[0] += lt
                a[1] += dt
                a[2] += 1
        if acc:
            rep["bucket_timeline"] = [
                {"bucket": bi, "bytes": (self.buckets[bi].end - self.buckets[bi].start) * wsz,
                 "launch_ms": round(a[0] / a[2], 4), "done_ms": round(a[1] / a[2], 4)}
                for bi, a in sorted(acc.items())]
        return rep

    # ------------------------------------------------------------------------------------------
    def _broadcast_state(self, buffers: bool):
        src = dist.get_global_rank(self.pg, 0) if self.pg is not None else 0
        dist.broadcast(self.flat.master, src, group=self.pg)
        self.flat.refresh_shadows()
        if buffers:
            self.sync_buffers()

    def _buffer_groups(self):
        groups = {}
        for b in self.module.buffers():
            if b.is_floating_point() or b.dtype in (torch.int64, torch.int32):
                groups.setdefault((b.dtype, b.device), []).append(b)
        return groups

    def sync_buffers(self):
        """Broadcast every buffer from rank 0: one coalesced broadcast per (dtype, device)."""
        if self.world <= 1:
            return
        src = dist.get_global_rank(self.pg, 0) if self.pg is not None else 0
        for bufs in self._buffer_groups().values():
            flat = torch._utils._flatten_dense_tensors(bufs)
            dist.broadcast(flat, src, group=self.pg)
            for b, v in zip(bufs, torch._utils._unflatten_dense_tensors(flat, bufs)):
                b.copy_(v)

    def average_buffers(self):
        """All-reduce the floating buffers (BatchNorm running mean / variance) to their mean over the
        ranks and broadcast the integer ones (batch counters) from rank 0: every rank then evaluates
        with the same statistics.  Call before an evaluation; the trainers do."""
        if self.world <= 1:
            return
        src = dist.get_global_rank(self.pg, 0) if self.pg is not None else 0
        for (dt, _), bufs in self._buffer_groups().items():
            flat = torch._utils._flatten_dense_tensors(bufs)
            if flat.is_floating_point():
                dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=self.pg)
                flat.div_(self.world)
            else:
                dist.broadcast(flat, src, group=self.pg)
            for b, v in zip(bufs, torch._utils._unflatten_dense_tensors(flat, bufs)):
                b.copy_(v)

    def forward(self, *a, **kw):
        self._reset()
        if self.buffer_mode == "forward" and self.world > 1 and torch.is_grad_enabled():
            self.sync_buffers()
        return self.module(*a, **kw)

    def _reset(self):
        for b in self.buckets:
            b.pending = len(b.params)
            b.work = None
            b.launched = False
            b.streams.clear()
        self._next_launch = 0

    @contextlib.contextmanager
    def no_sync(self):
        """Gradient accumulation window: buckets are not all-reduced."""
        old = self.require_sync
        self.require_sync = False
        try:
            yield
        finally:
            self.require_sync = old

    # ------------------------------------------------------------------------------------------
    def _on_grad_ready(self, p):
        bs = self._bucket_of.get(id(p))
        if bs is None:
            return
        done = False
        for b in bs:
            if self._comm_stream is not None:
                s = torch.cuda.current_stream(p.device)
                b.streams[s.cuda_stream] = s
                if self._timing and self._ev_ref is None:    # the step's first gradient: time origin
                    self._ev_ref = torch.cuda.Event(enable_timing=True)
                    self._ev_ref.record(s)
            b.pending -= 1
            done = done or b.pending == 0
        if done:
            self._launch_ready()

    def _launch_ready(self):
        while self._next_launch < len(self.buckets) and self.buckets[self._next_launch].pending <= 0:
            self._launch(self.buckets[self._next_launch])
            self._next_launch += 1

    def _launch(self, b: _Bucket):
        b.launched = True
        if not self.active or not self.require_sync:
            return
        view = self.flat.grad[b.start:b.end]
        cs = self._comm_stream
        if cs is None:                                   # CPU tensors (gloo)
            if self._timing:
                b.t_launch = time.perf_counter()
            if self._lowp is not None:
                low = self._lowp[b.start:b.end]
                low.copy_(view)
                b.work = dist.all_reduce(low, op=dist.ReduceOp.SUM, group=self.pg, async_op=True)
            else:
                b.work = dist.all_reduce(view, op=dist.ReduceOp.SUM, group=self.pg, async_op=True)
            return
        # order the collective after exactly the streams that wrote this bucket's gradients
        streams = b.streams or {0: torch.cuda.current_stream(view.device)}
        for key, s in streams.items():
            ev = b.events.get(key)
            if ev is None:
                ev = b.events[key] = torch.cuda.Event()
            ev.record(s)
            cs.wait_event(ev)
        if self._timing:
            b.t_launch = torch.cuda.Event(enable_timing=True)
            b.t_launch.record(cs)                        # every gradient of the bucket written
        with torch.cuda.stream(cs):
            if self._lowp is not None:
                low = self._lowp[b.start:b.end]
                low.copy_(view)                          # fp32 -> bf16 on the comm stream
                b.work = dist.all_reduce(low, op=dist.ReduceOp.SUM, group=self.pg, async_op=True)
            else:
                b.work = dist.all_reduce(view, op=dist.ReduceOp.SUM, group=self.pg, async_op=True)

    def _opt_scale(self):
        """Device scalar 1/world for the optimizer's gradient scale (None when it is 1)."""
        if self.grad_scale() == 1.0:
            return None
        if self._scale_t is None:
            self._scale_t = torch.tensor([self.grad_scale()], dtype=torch.float32, device=self.flat.device)
        return self._scale_t

    def _step_whole(self, opt, clip):
        """The optimizer step after a join without collectives: clip + one update over the arena."""
        norm = None
        if clip is not None:
            s = self.grad_scale()
            norm = opt.clip_grad_norm(clip, pre_scale=s, post_scale=s)
        else:
            opt.grad_scale = self._opt_scale()
        opt.step()
        return norm

    def finish_gradient_sync(self, opt=None, clip: float | None = None):
        """Call after ``loss.backward()``: launches buckets whose params produced no gradient
        (their slices hold zeros from ``zero_grad``), then joins every outstanding all-reduce.
        GPU: the comm stream waits for RCCL, casts low-precision sums back into the fp32 arena,
        and the compute stream waits for the comm stream once; the host never blocks.

        ``opt`` (a :mod:`pcmp.optim` flat optimizer): the optimizer step is issued HERE, per bucket
        on the comm stream -- each bucket's slice is updated as soon as its all-reduce completes,
        while later buckets are still in flight (after the end of backward: the updated weights
        must not be read by a backward kernel still queued).  ``clip``: global-norm clipping in
        two phases (per-bucket partial sums of squares as the collectives complete, then one
        coefficient and one update).  The caller must NOT call ``opt.step()`` again; returns the
        pre-clip norm (device scalar) when ``clip`` is given."""
        issued = self.active and self.require_sync
        if opt is not None and not issued:
            self._finish_join()
            return self._step_whole(opt, clip)
        return self._finish_join(opt, clip)

    def _finish_join(self, opt=None, clip=None):
        cs = self._comm_stream
        timing = self._timing and self.active and self.require_sync
        main = torch.cuda.current_stream(cs.device) if cs is not None else None
        if (timing or opt is not None) and cs is not None:
            ev_a = torch.cuda.Event(enable_timing=timing)
            ev_a.record(main)
        if opt is not None:
            self._opt_in_tail = True
        t0 = time.perf_counter()
        for b in self.buckets:
            b.pending = 0
        self._launch_ready()
        ctx = torch.cuda.stream(cs) if cs is not None else contextlib.nullcontext()
        line = []
        norm = None
        with ctx:
            if opt is not None:
                if cs is not None:
                    cs.wait_event(ev_a)       # every backward kernel that reads the weights is done
                opt.grad_scale = self._opt_scale()
                opt.begin_step()
                if clip is not None and self._parts is None:
                    self._parts = torch.zeros(self._nparts, dtype=torch.float32, device=self.flat.device)
            for b in self.buckets:
                if b.work is not None:
                    if timing and cs is not None and b.t_launch is not None:
                        # completion on a stream of its own: the comm stream is still queued behind
                        # later buckets' input waits, the timeline stream only behind this collective
                        with torch.cuda.stream(self._tl_stream):
                            b.work.wait()
                            ev_d = torch.cuda.Event(enable_timing=True)
                            ev_d.record(self._tl_stream)
                        line.append((b.index, b.t_launch, ev_d))
                    b.work.wait()
                    if timing and cs is None and b.t_launch is not None:
                        line.append((b.index, b.t_launch - t0, time.perf_counter() - t0))
                    if self._lowp is not None:
                        self.flat.grad[b.start:b.end].copy_(self._lowp[b.start:b.end])
                    b.work = None
                b.t_launch = None
                if opt is not None:
                    if clip is not None:
                        K.grad_sumsq_parts(self.flat.grad[b.start:b.end], self._parts, b.part_off)
                    else:
                        opt.step_range(b.start, b.end)
            if opt is not None:
                if clip is not None:
                    s = self.grad_scale()
                    norm, coef = K.clip_coef_parts(self._parts, s, clip, s)
                    opt.grad_scale = coef
                    opt.step_range(0, self.flat.numel)
                    if cs is not None:
                        norm.record_stream(main)      # the caller reads it on the compute stream
                opt.end_step()
            if timing and cs is not None:
                ev_b = torch.cuda.Event(enable_timing=True)
                ev_b.record(cs)
                self._exposed.append((ev_a, ev_b))
        if timing and cs is None:
            self._exposed.append(time.perf_counter() - t0)
            self._timeline.append([(bi, lt * 1e3, dt * 1e3) for bi, lt, dt in line])
        elif timing and line and self._ev_ref is not None:
            self._timeline.append(_EventLine(self._ev_ref, ev_a, line))
        self._ev_ref = None
        if cs is not None:
            main.wait_stream(cs)
        self._reset()
        return norm

    def grad_scale(self) -> float:
        return 1.0 / self.world if (self.average and self.world > 1) else 1.0


class _EventLine:
    """One step's GPU bucket timeline, resolved to ms relative to end of backward when iterated."""

    def __init__(self, ev_ref, ev_end, line):
        self.ev_ref, self.ev_end, self.line = ev_ref, ev_end, line

    def __iter__(self):
        self.ev_end.synchronize()
        end = self.ev_ref.elapsed_time(self.ev_end)
        for bi, ev_l, ev_d in self.line:
            ev_d.synchronize()
            yield bi, self.ev_ref.elapsed_time(ev_l) - end, self.ev_ref.elapsed_time(ev_d) - end


def _parse_dtype(d) -> torch.dtype:
    if d is None or d == "" or d == "fp32" or d == "float32" or d == torch.float32:
        return torch.float32
    if d in ("bf16", "bfloat16", torch.bfloat16):
        return torch.bfloat16
    raise ValueError(f"unsupported DDP gradient all-reduce dtype: {d!r} (fp32 or bf16)")


def convert_sync_batchnorm(module: torch.nn.Module, process_group=None) -> torch.nn.Module:
    """SyncBN option ("per-rank batch statistics, as DDP's default; make SyncBN an
    option"): every fused conv+BN layer of ``module`` computes its training-mode batch statistics,
    and its backward reduction, over all ranks of ``process_group`` (default: the world) with one
    fp64 all-reduce of the per-channel sums each way.  Running statistics are then identical on
    every rank.  Returns ``module`` (modified in place), like torch.nn.SyncBatchNorm.convert_sync_batchnorm."""
    from ..models.layers import ConvBN
    for m in module.modules():
        if isinstance(m, ConvBN):
            m.sync_group = process_group if process_group is not None else True
    return module



def sync_autotune(process_group=None) -> int:
    """Make every rank run rank 0's autotuned kernel choices.

    The conv / GEMM planner (``plan_gemm``) and the WGRAD split-K tuner (``wgrad_nsplit``) time
    their candidates on each rank's own GPU the first time a shape is seen.  Timing noise lets
    ranks pick different kernels, and in data parallelism the slowest rank gates every step (and
    a different split count changes the gradient's summation order).  Call this once after the
    first (warm-up) step, when every shape has been planned: rank 0's tables are broadcast and
    loaded over every rank's own (``torch.ops.pcmp.autotune_table`` / ``autotune_load``).
    Returns the number of entries applied on this rank (0 at world size 1 or without the native
    library)."""
    if not dist.is_initialized() or dist.get_world_size(process_group) <= 1:
        return 0
    from ..ops import _lib
    have = _lib.load()
    table = [list(torch.ops.pcmp.autotune_table()) if have else []]
    src = dist.get_global_rank(process_group, 0) if process_group is not None else 0
    dist.broadcast_object_list(table, src=src, group=process_group)
    if not have or not table[0]:
        return 0
    return int(torch.ops.pcmp.autotune_load(table[0]))


_SYNCED_SIZE = [-1]   # THIS rank's plan-table size right after the last sync


def sync_autotune_if_grown(process_group=None) -> int:
    """Run :func:`sync_autotune` again when ANY rank planned shapes after the last sync (a last
    partial batch, other text batch shapes, the first eval batches): each rank compares its table
    with its own size right after the last sync, and one MAX all-reduce of the growth decides, so
    every rank takes the same branch -- growth on a rank that is not the largest is seen too.
    Called at epoch ends by the training loops; returns the entries applied (0 when nothing grew)."""
    if not dist.is_initialized() or dist.get_world_size(process_group) <= 1:
        return 0
    from ..ops import _lib
    have = _lib.load()
    n = len(torch.ops.pcmp.autotune_table()) if have else 0
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend(process_group) == "nccl" \
        else torch.device("cpu")
    t = torch.tensor([n - _SYNCED_SIZE[0]], dtype=torch.int64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=process_group)
    if int(t.item()) <= 0:
        return 0
    applied = sync_autotune(process_group)
    # remembered AFTER the merge: rank 0's entries now count as this rank's own, so the next epoch
    # does not see them as growth (no redundant second sync)
    _SYNCED_SIZE[0] = len(torch.ops.pcmp.autotune_table()) if have else 0
    return applied


def step_time_spread(seconds: float, process_group=None) -> dict:
    """Per-rank wall time of a timed region -> {min, max, mean, argmax rank} over all ranks (one
    small all-gather).  The bench reports MAX (the job's pace) but a straggler is only visible in
    the spread."""
    if not dist.is_initialized() or dist.get_world_size(process_group) <= 1:
        return {"min_s": seconds, "max_s": seconds, "mean_s": seconds, "slowest_rank": 0}
    world = dist.get_world_size(process_group)
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend(process_group) == "nccl" \
        else torch.device("cpu")
    t = torch.tensor([float(seconds)], dtype=torch.float64, device=dev)
    out = [torch.zeros_like(t) for _ in range(world)]
    dist.all_gather(out, t, group=process_group)
    v = [float(x.item()) for x in out]
    return {"min_s": min(v), "max_s": max(v), "mean_s": sum(v) / world, "slowest_rank": int(max(range(world), key=v.__getitem__))}

"""Fused conv+BN(+ReLU) block executors with hand-scheduled backward.

A whole residual block (BasicBlock / Bottleneck, with or without a downsample branch) or the
ResNet stem is ONE autograd node.  Its forward runs the implicit-GEMM conv kernels (BN partial
statistics emitted by the conv epilogue), the BN finalize kernel and the fused
``bn_apply`` (scale/shift + residual branch + ReLU).  Its backward is scheduled by hand so that:
  * the block tail's ReLU mask, the BN backward of the last conv AND of the downsample branch
    share one reduction pass and one apply pass;
  * the identity-path gradient and the downsample dgrad are added inside the dgrad epilogue
    of the first conv (no separate add kernel, no autograd accumulation);
  * every weight gradient is written by the wgrad kernel straight into the flat DDP bucket
    (``pcmp.ops.params.emit_grad``) and announced to the data-parallel engine immediately.

Reference parity: torchvision ResNet-50 Bottleneck (conv1x1-bn-relu-conv3x3(stride)-bn-relu-
conv1x1-bn (+downsample conv1x1/s + bn) -> add -> relu), printed at
pytorch_training_inference_on_image.ipynb:454-626; BasicBlock for the ResNet-18 north-star slice;
stem conv7x7/2-bn-relu-maxpool3x3/2 (:455-458).
"""
from __future__ import annotations

import os
import weakref

import torch
import torch.distributed as dist

from . import params as _params
from .kernels import K
from .params import compute_weight, compute_weight_t, emit_grad, sink_or_temp


def _sync_group(L):
    """SyncBN process group of a BN layer (``True`` = default group), or None when not syncing."""
    g = getattr(L, "sync_group", None)
    if g is None or not dist.is_available() or not dist.is_initialized():
        return None
    return g


def _global_sums(part, count, group):
    """SyncBN: per-tile partials [T,2,C] -> fp64 sums over every rank's batch [1,2,C] and the global
    element count (ranks hold equal per-rank batches, as DistributedSampler shards guarantee)."""
    grp = None if group is True else group
    s = part.double().sum(0, keepdim=True)
    dist.all_reduce(s, group=grp)
    return s, count * dist.get_world_size(grp)


class _Act:
    """The activation y = relu(scale*z + shift) of a BatchNorm, left unmaterialised: the 1x1 conv that
    consumes it forms y while staging its operand (``in_scale`` / ``in_shift`` of ``conv_fwd``, and
    of that conv's ``conv_wgrad`` in backward), so the forward ``bn_apply`` pass (read z, write y)
    never runs.  The ReLU mask the backward needs is recomputed from z already."""

    __slots__ = ("z", "scale", "shift")

    def __init__(self, z, scale, shift):
        self.z, self.scale, self.shift = z, scale, shift

    @property
    def shape(self):
        return self.z.shape


def _act_fold_ok(L, z) -> bool:
    """Should relu(BN(z)) feeding conv ``L`` stay folded?  GPU bf16: 1x1 stride-1 convs with C % 64 ==
    0, and only the memory-bound shapes whose conv already runs on the register-staged kernel (short
    reductions of layers 1-2: >= PCMP_ACT_FOLD_MINROWS rows, default 150k; ResNet-50 layer 2 at B=256
    has 200,704).  GPU fp32 only with PCMP_ACT_FOLD_F32=1 (every conv with C % 16 == 0): the fp32
    32x32x2 kernel then applies relu(scale * z + shift) to its A operand while staging it (BN
    coefficients read once per wave with scalar loads).  With the single-stage LDS main loop the
    staging sits between the two barriers of a K-step and the fold loses: TL forward 8.41 ms off vs
    8.90 ms on, same box (profiles/r5_f32_nbuf_fold_tl_ab.txt)."""
    import os
    if os.environ.get("PCMP_ACT_FOLD", "1") == "0" or not z.is_cuda:
        return False
    if z.dtype == torch.float32:
        return os.environ.get("PCMP_ACT_FOLD_F32", "0") == "1" and z.shape[-1] % 16 == 0
    if z.dtype != torch.bfloat16:
        return False
    if not (L.R == 1 and L.S == 1 and L.stride == 1 and z.shape[-1] % 64 == 0 and z.shape[-1] <= 128):
        return False
    try:
        minrows = int(os.environ.get("PCMP_ACT_FOLD_MINROWS", "150000"))
    except ValueError:
        minrows = 150000
    return z.numel() // z.shape[-1] >= minrows


def _act_args(x):
    """(x, in_scale, in_shift) for a conv_fwd / conv_wgrad operand."""
    if isinstance(x, _Act):
        return x.z, x.scale, x.shift
    return x, None, None


def _conv_bn_train(x, L, dtype, w=None, stride=None, pad=None):
    """conv (+stats) -> finalize.  Returns c, mean, invstd, scale, shift.  (``w``/``stride``/``pad``
    override the layer's: the space-to-depth stem; ``x`` may be an :class:`_Act`.)"""
    if w is None:
        w = compute_weight(L.weight, dtype)
    xz, isc, ish = _act_args(x)
    if isc is None:
        c, part = K.conv_fwd(xz, w, L.stride if stride is None else stride, L.pad if pad is None else pad, None, None,
                             False, True)
    else:
        c, part = K.conv_fwd(xz, w, L.stride if stride is None else stride, L.pad if pad is None else pad, None, None,
                             False, True, isc, ish)
    count = c.numel() // c.shape[-1]
    grp = _sync_group(L)
    if grp is not None:   # SyncBN: batch statistics over all ranks
        part, count = _global_sums(part, count, grp)
    track = L.track_running_stats
    mean, invstd, scale, shift = K.bn_finalize(part, count, L.gamma, L.beta,
                                               L.running_mean if track else None,
                                               L.running_var if track else None, L.momentum, L.eps)
    return c, mean, invstd, scale, shift


def _folded(L, dtype):
    """Inference-time BN folding: conv(x, W) * scale + shift == conv(x, W * scale) + shift.

    The folded compute weight (from the fp32 master) and the fp32 bias are cached on the layer,
    keyed on the global weight generation (bumped by optimizer steps and training-mode forwards
    that move the running statistics) plus the tensors' own version counters (bumped by
    ``load_state_dict`` / in-place edits), so eval forwards after the first are pure conv launches
    (bias + residual + ReLU fused in the conv epilogue, no BN apply pass).
    """
    key = (_params.WEIGHT_GEN[0], L.weight._version, L.gamma._version, L.beta._version,
           L.running_mean._version, L.running_var._version, dtype, L.weight.device)
    f = getattr(L, "_fold", None)
    if f is None or f[0] != key:
        scale, shift = K.bn_eval_coeff(L.gamma.detach(), L.beta.detach(), L.running_mean, L.running_var, L.eps)
        w = (L.weight.detach().float() * scale.view(-1, 1, 1, 1)).to(dtype).contiguous()
        f = (key, w, shift.float().contiguous())
        L._fold = f
    return f[1], f[2]


def _conv_bn_eval(x, L, dtype, relu, resid=None):
    """Eval-mode conv + BN (folded) (+ residual) (+ ReLU): one conv launch."""
    w, b = _folded(L, dtype)
    return K.conv_fwd(x, w, L.stride, L.pad, b, resid, relu, False)[0]


class _Fold:
    """The input gradient dz = k1*g + k2*x + k3 of a BatchNorm, left unmaterialised.

    Its consumers -- the DGRAD and the WGRAD of the 1x1 stride-1 conv that produced the BN's input
    -- form dz while they stage the operand (``fold_x`` / ``fold_coef`` of ``conv_dgrad_bnr`` and
    ``conv_wgrad``), so the ``bn_bwd_apply`` pass (read g and x, write dz) and the two reads of dz
    never run: on the DGRAD chain one extra read of x replaces three memory passes."""

    __slots__ = ("g", "x", "coef")

    def __init__(self, g, x, coef):
        self.g, self.x, self.coef = g, x, coef


def _fold_enabled() -> bool:
    import os
    return os.environ.get("PCMP_DZ_FOLD", "1") != "0"


def _fold_min_rows() -> int:
    import os
    try:
        return int(os.environ.get("PCMP_DZ_FOLD_MINROWS", "400000"))
    except ValueError:
        return 400000


def _fold_ok(L, g) -> bool:
    """Should the BN-backward output feeding conv ``L`` stay folded?  1x1 stride-1 convs whose channel
    count fits the kernels' block-uniform tap walk; on the GPU only the bf16 HIP kernels fold, and
    only for the memory-bound layer-1 shapes (>= PCMP_DZ_FOLD_MINROWS rows, default 400k: ResNet-50
    layer 1 at B=256 has 802,816).  Per shape (tools/fold_micro.py, profiles/r3_fold_micro.txt) the
    fold saves 33-107 us of the DGRAD chain there, and costs more than it saves from layer 2 on: the
    folded GEMMs run on the register-staged kernel instead of the LDS-DMA ones, and the folded WGRAD
    reads g and x (the side stream is not free: folding every shape cost 5 % of the step)."""
    if not _fold_enabled() or not (L.R == 1 and L.S == 1 and L.stride == 1 and g.shape[-1] % 64 == 0):
        return False
    if g.is_cuda and (g.dtype != torch.bfloat16 or g.numel() // g.shape[-1] < _fold_min_rows()):
        return False
    return True


def _stem_tail_mode(t) -> bool:
    import os
    return t.is_cuda and t.dtype == torch.bfloat16 and _fold_enabled() and os.environ.get("PCMP_STEM_TAIL", "1") != "0"


def _mat(dh):
    """Materialise a folded BN-backward output (paths whose kernel cannot fold)."""
    if isinstance(dh, _Fold):
        return K.bn_bwd_apply(dh.g, None, dh.x, dh.coef, None, None, False)[0]
    return dh


def _fold_args(dh):
    """(dy, fold_x, fold_coef) for a DGRAD / WGRAD op."""
    if isinstance(dh, _Fold):
        return dh.g, dh.x, dh.coef
    return dh, None, None


def _bn_backward(dy, ymask, x, mean, invstd, L, x2=None, mean2=None, invstd2=None, L2=None, want_g=False,
                 parts=None, fold=False):
    """Backward of one BN (or two BNs sharing the incoming gradient) -> list of dx (+g).

    ``parts`` = reduction partials already produced by a dgrad epilogue (``conv_dgrad_bnr``; then
    ``dy`` is the masked gradient and ``ymask`` is None) -- skips the separate reduction pass.
    ``fold``: the first BN's dx is returned as a :class:`_Fold` (not applied); a second BN's dx is
    still applied."""
    if parts is None:
        parts = K.bn_bwd_reduce(dy, ymask, x, mean, invstd, x2, mean2, invstd2)
    count = x.numel() // x.shape[-1]

    def finalize(part, Lk, mu, isd, gout, bout, acc):
        grp = _sync_group(Lk)
        if grp is None:
            return K.bn_bwd_finalize(part, count, Lk.gamma, mu, isd, gout, bout, acc)
        # SyncBN: dgamma/dbeta from this rank's sums (DDP averages them, as torch SyncBatchNorm);
        # the input-gradient coefficients from the sums over every rank's batch
        K.bn_bwd_finalize(part, count, Lk.gamma, mu, isd, gout, bout, acc)
        gsum, gcount = _global_sums(part, count, grp)
        return K.bn_bwd_finalize(gsum, gcount, Lk.gamma, mu, isd, None, None, False)

    gout, acc, fin = sink_or_temp(L.gamma)
    bout, bacc, bfin = sink_or_temp(L.beta)
    coef = finalize(parts[0], L, mean, invstd, gout, bout, acc or bacc)
    grads = {L.gamma: fin(), L.beta: bfin()}
    coef2 = None
    if x2 is not None:
        gout2, acc2, fin2 = sink_or_temp(L2.gamma)
        bout2, bacc2, bfin2 = sink_or_temp(L2.beta)
        coef2 = finalize(parts[1], L2, mean2, invstd2, gout2, bout2, acc2 or bacc2)
        grads[L2.gamma] = fin2()
        grads[L2.beta] = bfin2()
    if fold:
        assert ymask is None and not want_g, "fold: dy must already be the masked gradient"
        rest = list(K.bn_bwd_apply(dy, None, x2, coef2, None, None, False)) if x2 is not None else []
        return [_Fold(dy, x, coef)] + rest, grads
    outs = K.bn_bwd_apply(dy, ymask, x, coef, x2, coef2, want_g)
    return outs, grads


def _fused_conv_bwd(L, dh, a, st, grads):
    """The layer-1 conv3 backward as ONE kernel (``conv1x1_bwd_fused``, csrc/bwd_fused.h): its DGRAD with
    the previous BN's reduction AND its WGRAD, reading dz (or its BatchNorm-backward fold g, x) and the
    folded input relu(BN(z)) once instead of once per GEMM (the layer is HBM-bound; the separate
    side-stream WGRAD re-read 1.15 KB per pixel).  Returns conv_dgrad_bnr's [g, part] (the weight
    gradient is emitted here), or None where the shape / path does not apply.  PCMP_BWD_FUSED=0: off."""
    if os.environ.get("PCMP_BWD_FUSED", "1") == "0" or not isinstance(a, _Act):
        return None
    if not (L.R == 1 and L.S == 1 and L.stride == 1 and L.pad == 0):
        return None
    g, fx, fc = _fold_args(dh)
    if not (g.is_cuda and g.dtype == torch.bfloat16 and g.shape[-1] == 256 and a.z.shape[-1] == 64
            and (g.numel() // 256) % 32 == 0):
        return None
    w = L.weight
    if not w.requires_grad:
        return None
    wt = compute_weight_t(w, g.dtype)
    if wt is None:   # no flat arena: transpose the (small) compute weight here
        wc = compute_weight(w, g.dtype)
        wt = wc.reshape(wc.shape[0], -1).t().contiguous()
    mean, istd = st
    res = []

    def fill(out, acc):
        res.append(K.conv1x1_bwd_fused(g, fx, fc, wt, a.z, a.scale, a.shift, mean, istd, out, acc))

    grads[w] = emit_grad(w, fill)
    return res[0]


def _bnr_ok(L):
    """Fused dgrad+BN-reduce needs every input pixel produced by an epilogue (stride-2 sub-pixel
    classes without taps would be skipped)."""
    return L.stride == 1 or (L.stride == 2 and L.R >= 2 and L.S >= 2)


def _wgrad(L, dy, x, grads, fill=None):
    """Weight gradient of layer ``L`` (``fill(out, accumulate)`` overrides the plain conv WGRAD)."""
    w = L.weight
    g, fx, fc = _fold_args(dy)
    xz, isc, ish = _act_args(x)
    keep = tuple(t for t in (g, xz, fx, fc, isc, ish) if t is not None)
    if fill is None:
        if fx is None and isc is None:
            def fill(out, acc):
                K.conv_wgrad(g, xz, out, L.R, L.S, L.stride, L.pad, acc)
        else:
            def fill(out, acc):
                K.conv_wgrad(g, xz, out, L.R, L.S, L.stride, L.pad, acc, fx, fc, isc, ish)
    if g.is_cuda and w.requires_grad and getattr(w, "main_grad", None) is not None and _params.side_stream_enabled():
        # into the flat gradient buffer on the WGRAD stream, concurrent with this layer's DGRAD
        _params.run_on_side(lambda: emit_grad(w, fill), keep)
        grads[w] = None
        return
    grads[w] = emit_grad(w, fill)


# ---- space-to-depth stem --------------------------------------------------------------------------
# On the GPU the 7x7/2 (pad 3) stem conv runs as a 4x4/1 unpadded conv over the 2x2 space-to-depth
# image S[n,i,j,(dy*2+dx)*4+c] = X[n,c,2i+dy-3,2j+dx-3] (``K.image_to_s2d``) with the 7x7 filter
# embedded in an 8x8 one: a 256-deep GEMM reduction (4 full K-tiles) instead of 7*7*8 = 392 (7
# K-tiles, 5 of every 8 input channels padding), same products, same output.  PCMP_STEM_S2D=0
# keeps the direct 7x7 conv (A/B runs).
S2D_CH = 16


def stem_s2d_wanted(device) -> bool:
    import os
    return device.type == "cuda" and os.environ.get("PCMP_STEM_S2D", "1") != "0"


def stem_s2d_enabled(x, L) -> bool:
    return (x.dtype in (torch.bfloat16, torch.float32) and L.R == 7 and L.S == 7 and L.stride == 2 and
            x.shape[-1] in (8, S2D_CH) and stem_s2d_wanted(x.device))


def s2d_weight(w):
    """[Co,7,7,Cp>=4] stem filter -> [Co,4,4,16] filter of the space-to-depth conv."""
    co = w.shape[0]
    w8 = torch.nn.functional.pad(w[..., :4], (0, 0, 0, 1, 0, 1))           # [Co,8,8,4], r = 2r'+dy
    return w8.reshape(co, 4, 2, 4, 2, 4).permute(0, 1, 3, 2, 4, 5).reshape(co, 4, 4, S2D_CH).contiguous()


def s2d_weight_grad(g4):
    """[Co,4,4,16] gradient of the space-to-depth filter -> [Co,7,7,4] gradient of the 7x7 filter."""
    co = g4.shape[0]
    return g4.reshape(co, 4, 4, 2, 2, 4).permute(0, 1, 3, 2, 4, 5).reshape(co, 8, 8, 4)[:, :7, :7, :]


def s2d_input_grad(gs, H, W, pad, cpad):
    """Gradient w.r.t. the space-to-depth image -> gradient w.r.t. the [N,H,W,cpad] stem input."""
    N, Hs, Ws, _ = gs.shape
    g = gs.reshape(N, Hs, Ws, 2, 2, 4).permute(0, 1, 3, 2, 4, 5).reshape(N, 2 * Hs, 2 * Ws, 4)
    g = g[:, pad:pad + H, pad:pad + W, :]
    return torch.nn.functional.pad(g, (0, cpad - 4)).contiguous()


def _folded_s2d(L, dtype):
    w, b = _folded(L, dtype)
    f = getattr(L, "_fold_s2d", None)
    if f is None or f[0] is not w:
        f = (w, s2d_weight(w))
        L._fold_s2d = f
    return f[1], b


class _TailBN:
    """The BatchNorm(s) feeding a residual block's output ``out = relu(bn3(c3) + shortcut)``,
    published by the block's training forward so that the NEXT block's backward can fuse their
    backward reduction into its final dgrad epilogue (``conv_dgrad_bnr`` with ``ymask = out``).
    The next block hands back the masked gradient ``g`` and the partials; this block's backward
    then skips its own reduction pass.  The masked gradient equals d(out) on the support of the
    ReLU, which is all this block's backward consumes."""

    __slots__ = ("out_ptr", "out_shape", "c", "mean", "invstd", "cd", "meand", "invstdd", "g_ptr", "parts",
                 "mbits", "__weakref__")

    def __init__(self, out, c, mean, invstd, cd, meand, invstdd, mbits=None):
        self.out_ptr, self.out_shape = out.data_ptr(), tuple(out.shape)
        self.mbits = mbits   # out > 0 as bits (1 byte / 8 channels): the next block's dgrad mask
        self.c, self.mean, self.invstd = c, mean, invstd
        self.cd, self.meand, self.invstdd = cd, meand, invstdd
        self.g_ptr = None
        self.parts = None


_LAST_TAIL = [lambda: None]   # weakref to the most recently published _TailBN


def _link_prev_tail(x):
    st = _LAST_TAIL[0]()
    if st is not None and st.out_ptr == x.data_ptr() and st.out_shape == tuple(x.shape):
        return st
    return None


def _dgrad_into_prev(dh, w, H, W, L, resid, x, prev, resid_sub=False):
    """dx = dgrad(dh) + resid, masked by x > 0, with prev's BN reduction fused in the epilogue
    (``resid_sub``: resid is a 1x1 stride-2 downsample's compact DGRAD, added at even pixels)."""
    mask = None if prev.mbits is not None else x
    g, fx, fc = _fold_args(dh)
    r = K.conv_dgrad_bnr(g, w, H, W, L.stride, L.pad, resid, mask, prev.c, prev.mean, prev.invstd,
                         prev.cd, prev.meand, prev.invstdd, None, None, compute_weight_t(L.weight, g.dtype),
                         prev.mbits, fx, fc, resid_sub)
    prev.parts = r[1:]
    prev.g_ptr = r[0].data_ptr()
    return r[0]


# PCMP_COMPACT_DOWN=0: the downsample DGRAD writes the dense zero-filled [N, H, W, C] gradient (A/B)
_COMPACT_DOWN = os.environ.get("PCMP_COMPACT_DOWN", "1") != "0"


def _compact_down_dgrad_ok(dcd, down, H, W) -> bool:
    return (down.R == 1 and down.S == 1 and down.stride == 2 and down.pad == 0 and H % 2 == 0 and W % 2 == 0
            and dcd.dtype == torch.bfloat16 and dcd.shape[1] * 2 == H and dcd.shape[2] * 2 == W)


def _compact_down_dgrad(dcd, down, H, W):
    """A 1x1 stride-2 pad-0 downsample's DGRAD is nonzero only at the even pixels (2i, 2j) of its
    [N, H, W, C] input gradient, where it is a plain stride-1 1x1 DGRAD of dcd: computed compact
    ([N, H/2, W/2, C]) it needs no zero fill of the other 3/4, and the conv1 DGRAD that adds it
    (``conv_dgrad_bnr(..., resid_sub=True)``) reads a quarter of the bytes."""
    wd = compute_weight(down.weight, dcd.dtype)
    wdt = compute_weight_t(down.weight, dcd.dtype)
    if wdt is not None:   # 1x1 stride 2: the class-blocked layout holds class (0, 0) only = [C][1][1][K]
        wdt = wdt.view(wd.shape[3], 1, 1, wd.shape[0])
    return K.conv_dgrad(dcd, wd, dcd.shape[1], dcd.shape[2], 1, 0, None, wdt)


def _side_branch_ok(t, L) -> bool:
    """Independent branch of a block on the side stream (GPU; not with SyncBN, whose statistics
    all-reduce runs on the compute stream).  PCMP_DOWN_STREAM=0 keeps it on the compute stream."""
    import os
    return (t.is_cuda and _params.side_stream_enabled() and _sync_group(L) is None and
            os.environ.get("PCMP_DOWN_STREAM", "1") != "0")


# Output pixels (N*P*Q) up to which an eval-mode downsample conv is forked onto the side stream.
# Off: in the captured batch-1 graph the parallel branch costs ~93 us of fork/join per image
# (p50 0.479 -> 0.572 ms, profiles/r2_infer_fork_ab.txt, tools/infer_fork_ab.py).
EVAL_FORK_MAX_ROWS = 0


def _eval_fork_ok(x, L) -> bool:
    P = (x.shape[1] + 2 * L.pad - L.R) // L.stride + 1
    Q = (x.shape[2] + 2 * L.pad - L.S) // L.stride + 1
    return _side_branch_ok(x, L) and x.shape[0] * P * Q <= EVAL_FORK_MAX_ROWS


class ResidualBlockFn(torch.autograd.Function):
    """out = relu( BN_L(conv_L(...relu(BN_1(conv_1(x)))...)) + shortcut(x) )."""

    @staticmethod
    def forward(ctx, x, blk, *params):
        dtype = x.dtype
        main, down = blk.main_layers(), blk.down_layer()
        if not blk.training:
            # small inference batches: the downsample conv's few workgroups run next to the main
            # branch on the side stream (kept as a parallel branch when the forward is graph-captured)
            efork = None
            if down is not None and _eval_fork_ok(x, down):
                efork = _params.fork_side(lambda: _conv_bn_eval(x, down, dtype, False), (x,))
            h = x
            for L in main[:-1]:
                h = _conv_bn_eval(h, L, dtype, True)
            if efork is not None:
                r = _params.join_side(*efork)
            else:
                r = _conv_bn_eval(x, down, dtype, False) if down is not None else x
            return _conv_bn_eval(h, main[-1], dtype, True, r)

        _params.WEIGHT_GEN[0] += 1      # running statistics move in training mode
        # the downsample conv (+ BN statistics / finalize) is independent of the main branch: it runs
        # on the side stream, concurrently with conv1..convL
        dfork = None
        if down is not None and any(ctx.needs_input_grad) and _side_branch_ok(x, down):
            dfork = _params.fork_side(lambda: _conv_bn_train(x, down, dtype), (x,))
        acts, cs, stats, coefs = [x], [], [], []
        h = x
        for i, L in enumerate(main):
            c, mean, invstd, sc, sh = _conv_bn_train(h, L, dtype)
            cs.append(c)
            stats.append((mean, invstd))
            coefs.append((sc, sh))
            if i < len(main) - 1:
                if _act_fold_ok(main[i + 1], c):   # the next (1x1) conv forms relu(BN(c)) itself
                    h = _Act(c, sc, sh)
                else:
                    h = K.bn_apply(c, sc, sh, None, None, None, True)
                acts.append(h)
            else:
                last = (sc, sh)
        # the block output's ReLU mask as bits, for the next block's fused dgrad epilogue
        mbits = (torch.empty(cs[-1].numel() // 8, dtype=torch.uint8, device=x.device)
                 if any(ctx.needs_input_grad) and cs[-1].shape[-1] % 8 == 0 else None)
        if down is not None:
            if dfork is not None:
                cd, meand, invstdd, scd, shd = _params.join_side(*dfork)
            else:
                cd, meand, invstdd, scd, shd = _conv_bn_train(x, down, dtype)
            out = K.bn_apply(cs[-1], last[0], last[1], cd, scd, shd, True, mbits)
        else:
            cd = meand = invstdd = None
            out = K.bn_apply(cs[-1], last[0], last[1], x, None, None, True, mbits)
        if any(ctx.needs_input_grad):
            ctx.prev_tail = _link_prev_tail(x) if ctx.needs_input_grad[0] else None
            tail = _TailBN(out, cs[-1], stats[-1][0], stats[-1][1], cd, meand, invstdd, mbits)
            _LAST_TAIL[0] = weakref.ref(tail)
            ctx.tail = tail
            ctx.save_for_backward(x, out)
            ctx.main = main
            ctx.down = down
            ctx.acts = acts[1:]          # intermediates only; x and out go through save_for_backward
            ctx.cs = cs
            ctx.stats = stats
            ctx.coefs = coefs
            ctx.dstate = (cd, meand, invstdd)
            ctx.params = params
            ctx.saved_ok = True
        else:
            ctx.saved_ok = False
        return out

    @staticmethod
    def backward(ctx, dout):
        assert ctx.saved_ok, "ResidualBlockFn.backward without saved state"
        main, down = ctx.main, ctx.down
        x, out = ctx.saved_tensors
        acts, cs, stats = [x] + ctx.acts, ctx.cs, ctx.stats
        cd, meand, invstdd = ctx.dstate
        dout = dout.contiguous()
        H, W = x.shape[1], x.shape[2]
        grads = {}
        Ll = main[-1]
        mean, invstd = stats[-1]
        tail = ctx.tail
        fused = tail.parts is not None and tail.g_ptr == dout.data_ptr()
        parts = tail.parts if fused else None
        mask = None if fused else out          # a fused dout is already masked by out > 0
        tail.parts = None
        # the last conv's dz stays folded into its DGRAD / WGRAD (needs the masked gradient dout)
        fold_tail = fused and _fold_ok(Ll, dout)
        if down is not None:
            outs, gr = _bn_backward(dout, mask, cs[-1], mean, invstd, Ll, cd, meand, invstdd, down, parts=parts,
                                    fold=fold_tail)
            dh, dcd = outs[0], outs[1]
            gid = None
        elif fused:
            outs, gr = _bn_backward(dout, None, cs[-1], mean, invstd, Ll, parts=parts, fold=fold_tail)
            dh, gid = outs[0], dout
            dcd = None
        else:
            outs, gr = _bn_backward(dout, out, cs[-1], mean, invstd, Ll, want_g=True)
            dh, gid = outs[0], outs[1]
            dcd = None
        grads.update(gr)
        need_dx = ctx.needs_input_grad[0]
        dx = None
        # downsample dgrad (the shortcut's input gradient, added in conv1's dgrad epilogue) on the side
        # stream, concurrently with the main branch's backward chain
        prev0 = ctx.prev_tail if (need_dx and _bnr_ok(main[0])) else None
        tfork = None
        t_sub = False
        if down is not None and prev0 is not None and _side_branch_ok(dcd, down):
            wd = compute_weight(down.weight, dcd.dtype)
            wdt = compute_weight_t(down.weight, dcd.dtype)
            # the consumer (the main branch's first DGRAD) takes the compact form only at stride 1
            t_sub = _COMPACT_DOWN and main[0].stride == 1 and _compact_down_dgrad_ok(dcd, down, H, W)
            if t_sub:
                tfork = _params.fork_side(lambda: _compact_down_dgrad(dcd, down, H, W), (dcd, wd))
            else:
                tfork = _params.fork_side(lambda: K.conv_dgrad(dcd, wd, H, W, down.stride, down.pad, None, wdt),
                                          (dcd, wd, wdt))
        for i in range(len(main) - 1, -1, -1):
            L = main[i]
            r_fused = _fused_conv_bwd(L, dh, acts[i], stats[i - 1], grads) if (i > 0 and _bnr_ok(L)) else None
            if r_fused is None:
                _wgrad(L, dh, acts[i], grads)
            dtype = _fold_args(dh)[0].dtype
            wcomp = compute_weight(L.weight, dtype)
            wt = compute_weight_t(L.weight, dtype)
            if i > 0:
                Hi, Wi = acts[i].shape[1], acts[i].shape[2]
                m_prev, is_prev = stats[i - 1]
                if _bnr_ok(L):
                    # dgrad epilogue applies the previous ReLU mask and emits that BN's reduction
                    # the ReLU mask of acts[i] = relu(cs[i-1] * scale + shift) is recomputed from cs[i-1]
                    sc_prev, sh_prev = ctx.coefs[i - 1]
                    g, fx, fc = _fold_args(dh)
                    if r_fused is not None:
                        r = r_fused
                    else:
                        r = K.conv_dgrad_bnr(g, wcomp, Hi, Wi, L.stride, L.pad, None, None, cs[i - 1],
                                             m_prev, is_prev, None, None, None, sc_prev, sh_prev, wt, None, fx, fc)
                    # conv1's dz folds when every consumer can: its WGRAD, and its DGRAD only on the
                    # fused into-previous-block path
                    fold = (i - 1 == 0 and _fold_ok(main[0], r[0]) and (not need_dx or prev0 is not None))
                    outs, gr = _bn_backward(r[0], None, cs[i - 1], m_prev, is_prev, main[i - 1], parts=r[1:],
                                            fold=fold)
                else:
                    da = K.conv_dgrad(_mat(dh), wcomp, Hi, Wi, L.stride, L.pad, None, wt)
                    ai = acts[i]
                    if isinstance(ai, _Act):   # (never for ResNet v1.5: folded inputs feed 1x1 stride-1 convs)
                        ai = K.bn_apply(ai.z, ai.scale, ai.shift, None, None, None, True)
                    outs, gr = _bn_backward(da, ai, cs[i - 1], m_prev, is_prev, main[i - 1])
                grads.update(gr)
                dh = outs[0]
            else:
                prev = ctx.prev_tail if (need_dx and _bnr_ok(L)) else None
                if down is not None:
                    _wgrad(down, dcd, acts[0], grads)
                    if need_dx:
                        wd = compute_weight(down.weight, dtype)
                        wdt = compute_weight_t(down.weight, dtype)
                        if prev is not None:
                            if tfork is not None:
                                t = _params.join_side(*tfork)
                            else:
                                t = K.conv_dgrad(dcd, wd, H, W, down.stride, down.pad, None, wdt)
                                t_sub = False
                            dx = _dgrad_into_prev(dh, wcomp, H, W, L, t, x, prev, t_sub)
                        else:
                            t = K.conv_dgrad(_mat(dh), wcomp, H, W, L.stride, L.pad, None, wt)
                            dx = K.conv_dgrad(dcd, wd, H, W, down.stride, down.pad, t, wdt)
                elif need_dx:
                    if prev is not None:
                        dx = _dgrad_into_prev(dh, wcomp, H, W, L, gid, x, prev)
                    else:
                        dx = K.conv_dgrad(_mat(dh), wcomp, H, W, L.stride, L.pad, gid, wt)
        # free saved activations early
        ctx.acts = ctx.cs = ctx.dstate = ctx.coefs = None
        ctx.prev_tail = ctx.tail = None
        pgrads = tuple(grads.get(p) for p in ctx.params)
        return (dx, None) + pgrads


class StemFn(torch.autograd.Function):
    """y = maxpool3x3/2( relu( BN( conv7x7/2(x) ) ) ): conv (+BN statistics) -> finalize -> pooling with
    the BN + ReLU applied in its prologue; backward = one fused pooling/mask/BN-reduction pass, the
    BN-backward apply, WGRAD."""

    @staticmethod
    def forward(ctx, x, stem, *params):
        L = stem.conv
        dtype = x.dtype
        s2d = stem_s2d_enabled(x, L)
        xin = x
        if s2d and x.shape[-1] != S2D_CH:   # NHWC input padded to 8 channels
            x = K.image_to_s2d(x, L.pad, 1.0, None, None, True)
        if not stem.training:
            if s2d:
                w4, b = _folded_s2d(L, dtype)
                c = K.conv_fwd(x, w4, 1, 0, b, None, True, False)[0]
            else:
                c = _conv_bn_eval(x, L, dtype, True)
            return K.maxpool_fwd(c, 3, 2, 1, False)[0]
        _params.WEIGHT_GEN[0] += 1
        if s2d:
            c, mean, invstd, sc, sh = _conv_bn_train(x, L, dtype, s2d_weight(compute_weight(L.weight, dtype)), 1, 0)
        else:
            c, mean, invstd, sc, sh = _conv_bn_train(x, L, dtype)
        # BN + ReLU fused into the pooling prologue: the normalised activation is never stored
        y, idx = K.maxpool_fwd(c, 3, 2, 1, True, sc, sh)
        if any(ctx.needs_input_grad):
            ctx.save_for_backward(x)
            ctx.state = (c, sc, sh, idx, mean, invstd)
            ctx.s2d = (tuple(xin.shape) if xin is not x else None) if s2d else False
            ctx.stem = stem
            ctx.params = params
        else:
            ctx.state = None
        return y

    @staticmethod
    def backward(ctx, dy):
        (x,) = ctx.saved_tensors
        c, sc, sh, idx, mean, invstd = ctx.state
        L = ctx.stem.conv
        grads = {}
        # pooling backward + ReLU mask (recomputed from c) + BN-backward partials in one pass
        r = K.maxpool_bwd_bnr(dy.contiguous(), idx, c, mean, invstd, sc, sh, 3, 2, 1)
        # The stem's WGRAD is the last GEMM of the step: nothing on the compute stream can overlap it
        # (profiles/r3_step_tail.txt: the compute stream idled ~315 us waiting for it on the side stream).
        # Tail mode (PCMP_STEM_TAIL, default on, GPU): when the WGRAD is the BN gradient's only
        # consumer (no input gradient), the BN-backward apply is folded into it, and it runs on the
        # compute stream with its autotuned split count (a lone GEMM wants the whole chip, not the
        # side stream's fixed 384-workgroup target).
        tail = _stem_tail_mode(c) and not ctx.needs_input_grad[0] and c.shape[-1] % 8 == 0
        outs, gr = _bn_backward(r[0], None, c, mean, invstd, L, parts=r[1:], fold=tail)
        grads.update(gr)
        dc = outs[0]
        g_, fx, fc = _fold_args(dc)
        if ctx.s2d is False:
            if tail:
                grads[L.weight] = emit_grad(L.weight, lambda out, acc: K.conv_wgrad(
                    g_, x, out, L.R, L.S, L.stride, L.pad, acc, fx, fc))
            else:
                _wgrad(L, dc, x, grads)
        else:
            def fill(out, acc):
                g4 = torch.empty(out.shape[0], 4, 4, S2D_CH, dtype=torch.float32, device=out.device)
                K.conv_wgrad(g_, x, g4, 4, 4, 1, 0, False, fx, fc)
                g = s2d_weight_grad(g4)
                if acc:
                    out[..., :4].add_(g)
                else:
                    out[..., :4].copy_(g)
                    out[..., 4:].zero_()
            if tail:
                grads[L.weight] = emit_grad(L.weight, fill)
            else:
                _wgrad(L, dc, x, grads, fill)
        dx = None
        if ctx.needs_input_grad[0]:
            if ctx.s2d is False:
                dx = K.conv_dgrad(dc, compute_weight(L.weight, dc.dtype), x.shape[1], x.shape[2], L.stride, L.pad,
                                  None, compute_weight_t(L.weight, dc.dtype))
            else:
                dx = K.conv_dgrad(dc, s2d_weight(compute_weight(L.weight, dc.dtype)), x.shape[1], x.shape[2], 1, 0,
                                  None, None)
                if ctx.s2d is not None:   # input was the 8-channel NHWC image
                    N, H, W, cp = ctx.s2d
                    dx = s2d_input_grad(dx, H, W, L.pad, cp)
        ctx.state = None
        return (dx, None) + tuple(grads.get(p) for p in ctx.params)


class ConvBiasActFn(torch.autograd.Function):
    """y = act(conv(x, W) + b) -- VGG16 conv3x3+bias+ReLU and the Keras-style biased convs."""

    @staticmethod
    def forward(ctx, x, conv, weight, bias):
        w = compute_weight(weight, x.dtype)
        y = K.conv_fwd(x, w, conv.stride, conv.pad, bias.float() if bias is not None else None, None,
                       conv.relu, False)[0]
        if any(ctx.needs_input_grad):
            ctx.save_for_backward(x, y)
            ctx.conv = conv
            ctx.weight, ctx.bias = weight, bias
        return y

    @staticmethod
    def backward(ctx, dy):
        x, y = ctx.saved_tensors
        conv, weight, bias = ctx.conv, ctx.weight, ctx.bias
        dy = dy.contiguous()
        if conv.relu:
            dy = K.relu_bwd(dy, y)
        gw = emit_grad(weight, lambda out, acc: K.conv_wgrad(dy, x, out, conv.R, conv.S, conv.stride, conv.pad, acc))
        gb = emit_grad(bias, lambda out, acc: K.colsum(dy, out, acc)) if bias is not None else None
        dx = None
        if ctx.needs_input_grad[0]:
            dx = K.conv_dgrad(dy, compute_weight(weight, dy.dtype), x.shape[1], x.shape[2], conv.stride, conv.pad,
                              None, compute_weight_t(weight, dy.dtype))
        return dx, None, gw, gb


class MaxPoolFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, k, s, pad):
        need = ctx.needs_input_grad[0]
        r = K.maxpool_fwd(x, k, s, pad, need)
        if need:
            ctx.save_for_backward(r[1])
            ctx.cfg = (x.shape[1], x.shape[2], k, s, pad)
        return r[0]

    @staticmethod
    def backward(ctx, dy):
        (idx,) = ctx.saved_tensors
        H, W, k, s, pad = ctx.cfg
        return K.maxpool_bwd(dy.contiguous(), idx, H, W, k, s, pad), None, None, None


class GapFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        ctx.hw = (x.shape[1], x.shape[2])
        return K.gap_fwd(x)

    @staticmethod
    def backward(ctx, dy):
        return K.gap_bwd(dy.contiguous(), *ctx.hw)

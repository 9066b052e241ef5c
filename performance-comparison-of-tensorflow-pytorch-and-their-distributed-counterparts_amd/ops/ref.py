"""PyTorch reference implementations of every native op (same signatures and return
conventions as ``torch.ops.pcmp.*``).

They run the CPU plumbing config, the CPU test-suite, and serve as the fp32 reference that the
HIP kernels are checked against on the GPU (``tests/test_kernels_gpu.py``).  Math is done in
fp32 and cast to the activation dtype, mirroring the kernels' fp32 accumulation.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F


def _nchw(x):
    return x.float().permute(0, 3, 1, 2)


def _nhwc(x):
    return x.permute(0, 2, 3, 1)


# ------------------------------------------------------------------------------ convolution
def fold_act(z, scale, shift):
    """y = relu(scale*z + shift) per channel (bn_apply's output), rounded to z's dtype: the operand a
    BatchNorm-forward fold (``in_scale`` / ``in_shift``) forms while staging instead of reading it."""
    return torch.relu(z.float() * scale.float() + shift.float()).to(z.dtype)


def conv_fwd(x, w, stride, pad, bias=None, resid=None, relu=False, want_stats=False, in_scale=None, in_shift=None):
    if in_scale is not None:
        x = fold_act(x, in_scale, in_shift)
    y = _nhwc(F.conv2d(_nchw(x), _nchw(w), None, stride, pad))
    if bias is not None:
        y = y + bias.float()
    if resid is not None:
        y = y + resid.float().reshape(y.shape)
    if relu:
        y = torch.relu(y)
    y = y.to(x.dtype).contiguous()
    if want_stats:
        yr = y.float().reshape(-1, y.shape[-1])
        return [y, torch.stack([yr.sum(0), (yr * yr).sum(0)]).unsqueeze(0)]
    return [y]


def conv_dgrad(dy, w, H, W, stride, pad, resid=None, wt=None):
    if wt is not None:   # the pre-transposed weight must agree with w (checked, then unused)
        if wt.dim() == 1:    # class-blocked stride-2 form of the flat arena: same elements, other order
            assert wt.numel() == w.numel(), "conv_dgrad: class-blocked wt must hold w.numel() elements"
        else:
            assert wt.shape == (w.shape[3], w.shape[1], w.shape[2], w.shape[0]), "conv_dgrad: wt must be [C,R,S,K]"
    N, K, R, S, C = dy.shape[0], w.shape[0], w.shape[1], w.shape[2], w.shape[3]
    dx = torch.nn.grad.conv2d_input((N, C, H, W), _nchw(w), _nchw(dy), stride=stride, padding=pad)
    dx = _nhwc(dx)
    if resid is not None:
        dx = dx + resid.float().reshape(dx.shape)
    return dx.to(dy.dtype).contiguous()


def fold_dz(g, x, coef):
    """dz = k1*g + k2*x + k3 per channel (bn_bwd_apply's output), rounded to g's dtype: the operand a
    BatchNorm-backward fold (``fold_x`` / ``fold_coef``) forms while staging instead of reading it."""
    C = g.shape[-1]
    c = coef.float().reshape(3, C)
    return (c[0] * g.float() + c[1] * x.float() + c[2]).to(g.dtype)


def expand_sub_resid(r, H, W):
    """[N, ceil(H/2), ceil(W/2), C] sub-sampled residual -> [N, H, W, C], zero off the (2i, 2j) pixels."""
    full = torch.zeros(r.shape[0], H, W, r.shape[-1], dtype=r.dtype, device=r.device)
    full[:, 0::2, 0::2] = r
    return full


def conv_dgrad_bnr(dy, w, H, W, stride, pad, resid, ymask, x, mean, invstd, x2=None, mean2=None, invstd2=None,
                   mscale=None, mshift=None, wt=None, ymask_bits=None, fold_x=None, fold_coef=None, resid_sub=False):
    if resid_sub and resid is not None:
        resid = expand_sub_resid(resid, H, W)
    if fold_x is not None:
        dy = fold_dz(dy, fold_x, fold_coef)
    if ymask_bits is not None:                    # mask as bits (bn_apply mbits)
        ymask = unpack_mask_bits(ymask_bits, x.shape)
    elif ymask is None and mscale is not None:    # mask recomputed from x: relu(x * scale + shift) > 0
        ymask = (x.float() * mscale + mshift).reshape(x.shape)
    g = _masked(conv_dgrad(dy, w, H, W, stride, pad, resid, wt), ymask).to(dy.dtype).contiguous()
    return [g] + bn_bwd_reduce(g, None, x, mean, invstd, x2, mean2, invstd2)


def conv_wgrad(dy, x, out, R, S, stride, pad, accumulate, fold_x=None, fold_coef=None, in_scale=None, in_shift=None):
    if fold_x is not None:
        dy = fold_dz(dy, fold_x, fold_coef)
    if in_scale is not None:
        x = fold_act(x, in_scale, in_shift)
    K, C = dy.shape[-1], x.shape[-1]
    dw = torch.nn.grad.conv2d_weight(_nchw(x), (K, C, R, S), _nchw(dy), stride=stride, padding=pad)
    dw = _nhwc(dw).reshape(out.shape).to(out.dtype)
    if accumulate:
        out.add_(dw)
    else:
        out.copy_(dw)


def conv1x1_bwd_fused(g, fold_x, fold_coef, wt, z, scale, shift, mean, invstd, dw, accumulate):
    """Fused 1x1 conv backward (csrc/bwd_fused.h): the DGRAD + BN-reduce of the input BN (mask
    recomputed from z) and the WGRAD against relu(scale * z + shift), from the same dz."""
    dz = fold_dz(g, fold_x, fold_coef) if fold_x is not None else g
    K, C = dz.shape[-1], z.shape[-1]
    w = wt.reshape(C, K).t().contiguous().reshape(K, 1, 1, C)
    r = conv_dgrad_bnr(dz, w, z.shape[1], z.shape[2], 1, 0, None, None, z, mean, invstd, None, None, None,
                       scale, shift)
    conv_wgrad(dz, z, dw, 1, 1, 1, 0, accumulate, None, None, scale, shift)
    return r


# ------------------------------------------------------------------------------ batchnorm
def bn_partials(x):
    xr = x.float().reshape(-1, x.shape[-1])
    return torch.stack([xr.sum(0), (xr * xr).sum(0)]).unsqueeze(0)


def bn_finalize(part, count, gamma, beta, running_mean, running_var, momentum, eps):
    s = part.double().sum(0)
    mean = s[0] / count
    var = (s[1] / count - mean * mean).clamp_min(0)
    invstd = (1.0 / torch.sqrt(var + eps)).float()
    mean = mean.float()
    g = gamma.float() if gamma is not None else torch.ones_like(mean)
    b = beta.float() if beta is not None else torch.zeros_like(mean)
    scale = g * invstd
    shift = b - mean * scale
    if running_mean is not None:
        unbiased = var * count / (count - 1) if count > 1 else var
        running_mean.mul_(1 - momentum).add_(momentum * mean)
        running_var.mul_(1 - momentum).add_(momentum * unbiased.float())
    return [mean, invstd, scale, shift]


def bn_eval_coeff(gamma, beta, running_mean, running_var, eps):
    invstd = torch.rsqrt(running_var.float() + eps)
    g = gamma.float() if gamma is not None else torch.ones_like(invstd)
    b = beta.float() if beta is not None else torch.zeros_like(invstd)
    scale = g * invstd
    return [scale, b - running_mean.float() * scale]


_BIT_WEIGHTS = {}


def pack_mask_bits(y):
    """uint8 [numel/8]: bit e of byte i = y.flatten()[8i+e] > 0 (the backward ReLU mask)."""
    w = _BIT_WEIGHTS.get(y.device)
    if w is None:
        w = _BIT_WEIGHTS[y.device] = (2 ** torch.arange(8, device=y.device)).to(torch.int32)
    return ((y.reshape(-1, 8).float() > 0).to(torch.int32) * w).sum(1).to(torch.uint8)


def unpack_mask_bits(bits, shape):
    b = bits.to(torch.int32).reshape(-1, 1) >> torch.arange(8, device=bits.device).to(torch.int32)
    return (b & 1).to(torch.float32).reshape(shape)


def bn_apply(x, scale, shift, x2=None, scale2=None, shift2=None, relu=False, mbits=None):
    y = x.float() * scale + shift
    if x2 is not None:
        y = y + (x2.float() * scale2 + shift2 if scale2 is not None else x2.float())
    if relu:
        y = torch.relu(y)
    y = y.to(x.dtype)
    if mbits is not None:
        mbits.copy_(pack_mask_bits(y))
    return y


def _masked(dy, ymask):
    g = dy.float()
    if ymask is not None:
        g = torch.where(ymask.float() > 0, g, torch.zeros_like(g))
    return g


def bn_bwd_reduce(dy, ymask, x, mean, invstd, x2=None, mean2=None, invstd2=None):
    C = x.shape[-1]
    g = _masked(dy, ymask).reshape(-1, C)
    xh = (x.float().reshape(-1, C) - mean) * invstd
    out = [torch.stack([g.sum(0), (g * xh).sum(0)]).unsqueeze(0)]
    if x2 is not None:
        xh2 = (x2.float().reshape(-1, C) - mean2) * invstd2
        out.append(torch.stack([g.sum(0), (g * xh2).sum(0)]).unsqueeze(0))
    return out


def bn_bwd_finalize(part, count, gamma, mean, invstd, dgamma, dbeta, accumulate):
    s = part.double().sum(0)
    sg, sgx = s[0], s[1]
    if dgamma is not None:
        (dgamma.add_ if accumulate else dgamma.copy_)(sgx.float())
    if dbeta is not None:
        (dbeta.add_ if accumulate else dbeta.copy_)(sg.float())
    g = gamma.double() if gamma is not None else torch.ones_like(sg)
    is_ = invstd.double()
    k1 = g * is_
    k2 = -(g * is_ * is_ * sgx / count)
    k3 = -(g * is_ * sg / count) - k2 * mean.double()
    return torch.stack([k1, k2, k3]).float()


def bn_bwd_apply(dy, ymask, x, coef, x2=None, coef2=None, want_g=False):
    g = _masked(dy, ymask)
    out = [(coef[0] * g + coef[1] * x.float() + coef[2]).to(dy.dtype)]
    if x2 is not None:
        out.append((coef2[0] * g + coef2[1] * x2.float() + coef2[2]).to(dy.dtype))
    if want_g:
        out.append(g.to(dy.dtype))
    return out


# ------------------------------------------------------------------------------ pooling
def maxpool_fwd(x, k, s, pad, want_idx, scale=None, shift=None):
    if scale is not None:     # fused BN + ReLU prologue
        x = torch.relu(x.float() * scale + shift).to(x.dtype)
    N, H, W, C = x.shape
    y, gidx = F.max_pool2d(_nchw(x), k, s, pad, return_indices=True)
    P, Q = y.shape[2], y.shape[3]
    yo = _nhwc(y).to(x.dtype).contiguous()
    if not want_idx:
        return [yo]
    hh = torch.div(gidx, W, rounding_mode="floor")
    ww = gidx - hh * W
    p = torch.arange(P, device=x.device).view(1, 1, P, 1)
    q = torch.arange(Q, device=x.device).view(1, 1, 1, Q)
    local = (hh - (p * s - pad)) * k + (ww - (q * s - pad))
    return [yo, _nhwc(local).to(torch.uint8).contiguous()]


def maxpool_bwd(dy, idx, H, W, k, s, pad):
    N, P, Q, C = dy.shape
    loc = idx.long().permute(0, 3, 1, 2)
    r = torch.div(loc, k, rounding_mode="floor")
    c = loc - r * k
    p = torch.arange(P, device=dy.device).view(1, 1, P, 1)
    q = torch.arange(Q, device=dy.device).view(1, 1, 1, Q)
    gidx = (p * s - pad + r) * W + (q * s - pad + c)
    dx = torch.zeros(N, C, H * W, dtype=torch.float32, device=dy.device)
    dx.scatter_add_(2, gidx.reshape(N, C, -1), _nchw(dy).reshape(N, C, -1))
    return _nhwc(dx.view(N, C, H, W)).to(dy.dtype).contiguous()


def maxpool_bwd_bnr(dy, idx, cx, mean, invstd, scale, shift, k, s, pad):
    """Stem backward: g = maxpool_bwd(dy) masked by relu(cx * scale + shift) > 0, plus the BN-backward
    partials [1, 2, C] = (sum g, sum g * (cx - mean) * invstd)."""
    g = maxpool_bwd(dy, idx, cx.shape[1], cx.shape[2], k, s, pad)
    g = _masked(g, (cx.float() * scale + shift)).to(dy.dtype).contiguous()
    return [g] + bn_bwd_reduce(g, None, cx, mean, invstd)


def gap_fwd(x):
    N, C = x.shape[0], x.shape[-1]
    return x.float().reshape(N, -1, C).mean(1).to(x.dtype)


def gap_bwd(dy, H, W):
    N, C = dy.shape
    return (dy.float() / (H * W)).view(N, 1, 1, C).expand(N, H, W, C).to(dy.dtype).contiguous()


def nchw_to_nhwc_f32(x, cpad, scale):
    h = x.float().permute(0, 2, 3, 1) * scale
    return F.pad(h, (0, cpad - h.shape[-1])).contiguous()


def resize_image(x, Ho, Wo, mode, cpad, scale, mean=None, stdv=None):
    """PIL bilinear resize of uint8 [N,H,W,C] images (the device kernel's reference)."""
    import numpy as np
    from PIL import Image
    outs = []
    for im in x.cpu().numpy():
        pim = Image.fromarray(im[..., 0] if im.shape[-1] == 1 else im)
        r = np.asarray(pim.resize((int(Wo), int(Ho)), Image.BILINEAR), dtype=np.uint8)
        outs.append(torch.from_numpy(r.reshape(int(Ho), int(Wo), -1).copy()))
    u = torch.stack(outs).to(x.device)                       # [N, Ho, Wo, C]
    if mode == 0:
        return u.permute(0, 3, 1, 2).contiguous()
    v = u.float() * scale
    if mean is not None:
        C = v.shape[-1]
        v = (v - mean[:C].float().to(v.device)) / stdv[:C].float().to(v.device)
    v = F.pad(v, (0, cpad - v.shape[-1]))
    return v.to(torch.bfloat16 if mode == 1 else torch.float32).contiguous()


# ------------------------------------------------------------------------------ loss
def softmax_xent(logits, labels, want_logp, want_grad, grad_scale, ignore_index):
    z = logits.float()
    logp = torch.log_softmax(z, dim=1)
    B, V = z.shape
    out = []
    if labels is not None:
        valid = (labels != ignore_index) & (labels >= 0) & (labels < V)
        lab = torch.where(valid, labels, torch.zeros_like(labels))
        loss_rows = torch.where(valid, -logp.gather(1, lab.view(-1, 1)).squeeze(1), torch.zeros(B, device=z.device))
    else:
        valid = torch.zeros(B, dtype=torch.bool, device=z.device)
        lab = torch.zeros(B, dtype=torch.long, device=z.device)
        loss_rows = torch.zeros(B, device=z.device)
    out.append(loss_rows)
    if want_logp:
        out.append(logp)
    if want_grad:
        g = torch.softmax(z, dim=1)
        g[torch.arange(B, device=z.device), lab] -= 1.0
        g = torch.where(valid.view(-1, 1), g * grad_scale, torch.zeros_like(g))
        out.append(g.to(logits.dtype))
    return out


def loss_mean(loss_rows, labels, V, ignore_index):
    valid = ((labels != ignore_index) & (labels >= 0) & (labels < V)).sum().float()
    return torch.stack([loss_rows.float().sum() / valid.clamp_min(1.0), valid])


def xent_grad_scale(dl, gout, valid):
    return (dl.float() * (gout.float().reshape(-1)[0] / valid.float().reshape(-1)[0].clamp_min(1.0))).to(dl.dtype)


def log_softmax_bwd(g, logp):
    gf = g.float()
    return (gf - torch.exp(logp.float()) * gf.sum(1, keepdim=True)).to(g.dtype)


# ------------------------------------------------------------------------------ dropout RNG
_M64 = (1 << 64) - 1


def _s64(v):
    v &= _M64
    return v - (1 << 64) if v >= (1 << 63) else v


def _lsr(z, k):
    # logical shift right on int64 two's-complement values
    return (z >> k) & ((1 << (64 - k)) - 1)


def _lowbias32(x):
    m32 = 0xFFFFFFFF
    x = torch.bitwise_xor(x, x >> 16)
    x = (x * 0x7FEB352D) & m32
    x = torch.bitwise_xor(x, x >> 15)
    x = (x * 0x846CA68B) & m32
    return torch.bitwise_xor(x, x >> 16)


def hash_uniform(seed: int, idx: torch.Tensor) -> torch.Tensor:
    """Bit-exact torch port of ``uniform01`` in csrc/common.h: lowbias32(lo32(idx) ^
    lowbias32(hi32(idx) ^ key)), key = the 64-bit seed folded to 32 bits."""
    m32 = 0xFFFFFFFF
    seed &= _M64
    key = (seed & m32) ^ (((seed >> 32) * 0x9E3779B9) & m32)
    i = idx.long()
    inner = _lowbias32(torch.bitwise_xor(_lsr(i, 32) & m32, key))
    x = _lowbias32(torch.bitwise_xor(i & m32, inner))
    return (x >> 8).float() * (1.0 / 16777216.0)


def _salted(seed, salt):
    if salt is None:
        return seed
    return (seed + int(salt.reshape(-1)[0].item()) * 0x9E3779B97F4A7C15) & _M64


def dropout(x, p, seed, offset, salt=None):
    seed = _salted(seed, salt)
    idx = torch.arange(x.numel(), device=x.device, dtype=torch.int64) + offset
    keep = hash_uniform(seed, idx).view(x.shape) >= p
    return torch.where(keep, x.float() / (1.0 - p), torch.zeros((), device=x.device)).to(x.dtype)


# ------------------------------------------------------------------------------ misc
def relu_bwd(dy, y):
    return torch.where(y.float() > 0, dy, torch.zeros_like(dy))


def colsum(x, out, accumulate):
    s = x.float().reshape(-1, x.shape[-1]).sum(0)
    if accumulate:
        out.add_(s)
    else:
        out.copy_(s)


def nchw_to_nhwc(x, cpad, scale, mean=None, stdv=None):
    y = x.float() * scale
    if mean is not None:
        y = (y - mean.view(1, -1, 1, 1)) / stdv.view(1, -1, 1, 1)
    y = y.permute(0, 2, 3, 1)
    if cpad > y.shape[-1]:
        y = F.pad(y, (0, cpad - y.shape[-1]))
    return y.to(torch.bfloat16).contiguous()


def image_to_s2d_f32(x, pad, scale):
    """csrc/elementwise.hip image_to_s2d_f32: image_to_s2d of an NCHW f32 / u8 image, fp32 out."""
    return image_to_s2d(x.float(), pad, scale, None, None, False, keep_f32=True)


def image_to_s2d(x, pad, scale, mean=None, stdv=None, nhwc=False, keep_f32=False):
    """Stem space-to-depth (csrc/elementwise.hip image_to_s2d_kernel):
    S[n,i,j,(dy*2+dx)*4+c] = X[n,c,2i+dy-pad,2j+dx-pad] (zero outside / c >= Cin); bf16 out, except
    fp32 NHWC in -> fp32 out (the fp32 stem)."""
    if nhwc:
        h = x.float()[..., :4]
    else:
        h = x.float() * scale
        if mean is not None:
            h = (h - mean.view(1, -1, 1, 1)) / stdv.view(1, -1, 1, 1)
        h = h.permute(0, 2, 3, 1)
    N, H, W, C = h.shape
    Hs, Ws = (H + 2 * pad + 1) // 2, (W + 2 * pad + 1) // 2
    h = F.pad(h, (0, 4 - C, pad, 2 * Ws - W - pad, pad, 2 * Hs - H - pad))
    h = h.reshape(N, Hs, 2, Ws, 2, 4).permute(0, 1, 3, 2, 4, 5).reshape(N, Hs, Ws, 16)
    if keep_f32 or (nhwc and x.dtype == torch.float32):   # fp32 path: fp32 out
        return h.contiguous()
    return h.to(torch.bfloat16).contiguous()


# ------------------------------------------------------------------------------ optimizers
def sgd_flat(w, g, mom, shadow, mask, lr, gscale, momentum, dampening, wd, nesterov, first_step):
    gs = gscale.float() if gscale is not None else 1.0
    d = g * gs + wd * w
    if momentum != 0:
        if first_step:
            mom.copy_(d)
        else:
            mom.mul_(momentum).add_(d, alpha=1 - dampening)
        d = d + momentum * mom if nesterov else mom
    upd = lr * d
    if mask is not None:
        upd = upd * mask.to(upd.dtype)
    w.sub_(upd)
    if shadow is not None:
        shadow.copy_(w.to(shadow.dtype))


def adam_flat(w, g, m1, m2, shadow, mask, lr, gscale, step, beta1, beta2, eps, wd, decoupled):
    gs = gscale.float() if gscale is not None else 1.0
    t = float(step)
    on = mask.bool() if mask is not None else None
    gv = g * gs
    w_new = w * (1 - lr * wd) if decoupled else w.clone()
    if not decoupled:
        gv = gv + wd * w
    m1_new = beta1 * m1 + (1 - beta1) * gv
    m2_new = beta2 * m2 + (1 - beta2) * gv * gv
    bc1 = 1 - beta1 ** t
    bc2 = 1 - beta2 ** t
    denom = m2_new.sqrt() / (bc2 ** 0.5) + eps
    w_new = w_new - (lr / bc1) * m1_new / denom
    if on is not None:
        w_new = torch.where(on, w_new, w)
        m1_new = torch.where(on, m1_new, m1)
        m2_new = torch.where(on, m2_new, m2)
    w.copy_(w_new)
    m1.copy_(m1_new)
    m2.copy_(m2_new)
    if shadow is not None:
        shadow.copy_(w.to(shadow.dtype))


def grad_clip_coef(g, pre_scale, max_norm, post_scale):
    norm = g.double().pow(2).sum().sqrt().float() * pre_scale
    c = torch.clamp(max_norm / (norm + 1e-6), max=1.0) if max_norm > 0 else torch.ones_like(norm)
    return [norm.reshape(()), (c * post_scale).reshape(())]


def sumsq_blocks(n):
    """Partial-sum rows grad_sumsq_parts writes for an n-element slice (csrc/optim.hip flat_grid)."""
    return max(1, min(2048, (n // 4 + 255) // 256))


def grad_sumsq_parts(g, part, offset):
    nb = sumsq_blocks(g.numel())
    part[offset:offset + nb] = 0.0
    part[offset] = g.double().pow(2).sum().float()


def clip_coef_parts(part, pre_scale, max_norm, post_scale):
    norm = part.double().sum().sqrt().float() * pre_scale
    c = torch.clamp(max_norm / (norm + 1e-6), max=1.0) if max_norm > 0 else torch.ones_like(norm)
    return [norm.reshape(()), (c * post_scale).reshape(())]


def cast_to_bf16(x, y):
    y.copy_(x.to(y.dtype))


def wt_transpose_multi(src, dst, desc, blocks):
    """dst[C][T][K] = src[K][tap(t)][C] for every entry described by desc rows (src_off, dst_off, K,
    T, C, first_block, S, RS, r0, s0, step, subS), tap(t) = (r0 + step*(t // subS))*S + s0 +
    step*(t % subS) -- the batched DGRAD weight transpose (whole filters and stride-2 classes)."""
    for so, do, K, T, C, _, S, RS, r0, s0, step, subS in desc.tolist():
        taps = [(r0 + step * (t // subS)) * S + s0 + step * (t % subS) for t in range(T)]
        w = src[so:so + K * RS * C].view(K, RS, C)[:, taps, :]
        dst[do:do + K * T * C].copy_(w.permute(2, 1, 0).reshape(-1))


# ------------------------------------------------------------------------------ text / LSTM
def embedding_fwd(ids, W):
    return W[ids]


def embedding_bwd(ids, dy, dW, padding_idx, accumulate):
    if not accumulate:
        dW.zero_()
    E = dW.shape[-1]
    idf = ids.reshape(-1)
    g = dy.reshape(-1, E).float()
    keep = idf != padding_idx
    dW.index_add_(0, idf[keep], g[keep])


def masked_mean_fwd(x, ids):
    m = (ids > 0).float().unsqueeze(-1)
    cnt = m.sum(1).clamp_min(1.0)
    return ((x.float() * m).sum(1) / cnt).to(x.dtype)


def masked_mean_bwd(dy, ids, S):
    m = (ids > 0).float().unsqueeze(-1)
    cnt = m.sum(1, keepdim=True).clamp_min(1.0)
    return (dy.float().unsqueeze(1) * m / cnt).to(dy.dtype)


def lstm_seq_fwd(gx, whh, ids):
    """Reference recurrence with packed-sequence masking (state carried at padded steps)."""
    B, S, _, G4 = gx.shape
    H = G4 // 4
    dev = gx.device
    hout = torch.zeros(B, S, 2 * H, dtype=whh.dtype, device=dev)
    gates = torch.zeros(B, S, 2, 4 * H, dtype=torch.float32, device=dev)
    cst = torch.zeros(B, S, 2, H, dtype=torch.float32, device=dev)
    valid = ids > 0
    for d in range(2):
        W = whh[d].float()
        h = torch.zeros(B, H, device=dev)
        hq = torch.zeros(B, H, device=dev)  # compute-dtype rounded h used by the recurrence
        c = torch.zeros(B, H, device=dev)
        order = range(S) if d == 0 else range(S - 1, -1, -1)
        for t in order:
            pre = gx[:, t, d].float() + hq @ W.t()
            i, f, g, o = pre.split(H, dim=1)
            i, f, g, o = torch.sigmoid(i), torch.sigmoid(f), torch.tanh(g), torch.sigmoid(o)
            cn = f * c + i * g
            hn = o * torch.tanh(cn)
            v = valid[:, t].unsqueeze(1)
            c = torch.where(v, cn, c)
            h = torch.where(v, hn, h)
            hq = h.to(whh.dtype).float()
            gates[:, t, d] = torch.cat([i, f, g, o], 1)
            cst[:, t, d] = c
            hout[:, t, d * H:(d + 1) * H] = h.to(whh.dtype)
    return [hout, gates, cst, torch.zeros(4, dtype=torch.int32, device=dev)]


def lstm_seq_bwd(dhout, gates, cst, whh, ids):
    B, S, _, G4 = gates.shape
    H = G4 // 4
    dev = gates.device
    dgates = torch.zeros(B, S, 2, G4, dtype=whh.dtype, device=dev)
    valid = ids > 0
    for d in range(2):
        W = whh[d].float()
        dh_carry = torch.zeros(B, H, device=dev)
        dc = torch.zeros(B, H, device=dev)
        order = range(S - 1, -1, -1) if d == 0 else range(S)
        for t in order:
            tprev = t - 1 if d == 0 else t + 1
            i, f, g, o = gates[:, t, d].split(H, dim=1)
            c = cst[:, t, d]
            cprev = cst[:, tprev, d] if 0 <= tprev < S else torch.zeros_like(c)
            dh = dhout[:, t, d * H:(d + 1) * H].float() + dh_carry
            tc = torch.tanh(c)
            dcn = dc + dh * o * (1 - tc * tc)
            dgo = dh * tc * o * (1 - o)
            dgi = dcn * g * i * (1 - i)
            dgg = dcn * i * (1 - g * g)
            dgf = dcn * cprev * f * (1 - f)
            dg = torch.cat([dgi, dgf, dgg, dgo], 1)
            v = valid[:, t].unsqueeze(1)
            dg = torch.where(v, dg, torch.zeros_like(dg))
            dgq = dg.to(whh.dtype)
            dgates[:, t, d] = dgq
            dc = torch.where(v, dcn * f, dc)
            dh_carry = torch.where(v, dgq.float() @ W, dh)
    return [dgates, torch.zeros(4, dtype=torch.int32, device=dev)]


# ------------------------------------------------------------------------------ transformer
def layernorm_fwd(x, r, g, b, eps, p=0.0, seed=0, offset=0, salt=None):
    xf = x.float()
    if p > 0:
        idx = torch.arange(x.numel(), device=x.device, dtype=torch.int64) + offset
        keep = hash_uniform(_salted(seed, salt), idx).view(x.shape) >= p
        xf = torch.where(keep, xf / (1.0 - p), torch.zeros((), device=x.device))
    xs = xf + r.float() if r is not None else xf
    if r is not None or p > 0:
        xs = xs.to(x.dtype).float()
    mean = xs.mean(-1)
    var = ((xs - mean.unsqueeze(-1)) ** 2).mean(-1)
    rstd = torch.rsqrt(var + eps)
    y = (xs - mean.unsqueeze(-1)) * rstd.unsqueeze(-1) * g + b
    D = x.shape[-1]
    return [y.to(x.dtype), xs.to(x.dtype), mean.reshape(-1), rstd.reshape(-1)]


def embed_layernorm_fwd(x, pos, tt, g, b, eps):
    """csrc/transformer.hip embed_layernorm_fwd: LN(x + pos[row % S] + tt), the sum rounded once."""
    D = x.shape[-1]
    S = pos.numel() // D
    xs = (x.float().reshape(-1, S, D) + pos.float().reshape(1, S, D) + tt.float().reshape(1, 1, D)).reshape(x.shape)
    xs = xs.to(x.dtype).float()
    mean = xs.mean(-1)
    var = ((xs - mean.unsqueeze(-1)) ** 2).mean(-1)
    rstd = torch.rsqrt(var + eps)
    y = (xs - mean.unsqueeze(-1)) * rstd.unsqueeze(-1) * g + b
    return [y.to(x.dtype), xs.to(x.dtype), mean.reshape(-1), rstd.reshape(-1)]


def layernorm_bwd(dy, xs, mean, rstd, g, dg, db, accumulate):
    D = xs.shape[-1]
    dyf = dy.float().reshape(-1, D)
    xh = (xs.float().reshape(-1, D) - mean.view(-1, 1)) * rstd.view(-1, 1)
    gy = dyf * g
    dx = rstd.view(-1, 1) * (gy - gy.mean(-1, keepdim=True) - xh * (gy * xh).mean(-1, keepdim=True))
    if dg is not None:
        (dg.add_ if accumulate else dg.copy_)((dyf * xh).sum(0))
    if db is not None:
        (db.add_ if accumulate else db.copy_)(dyf.sum(0))
    return dx.reshape(xs.shape).to(dy.dtype)


def layernorm_bwd_fused(dy, xs, mean, rstd, g, dg, db, dbias, accmask, p, seed, offset, salt=None):
    """Reference of csrc/transformer.hip ln_bwd_fused_kernel: [dx, dxd] plus dgamma / dbeta /
    dbias (column sums of dy*xhat, dy, dxd) written or accumulated (bit w of accmask)."""
    D = xs.shape[-1]
    dyf = dy.float().reshape(-1, D)
    xh = (xs.float().reshape(-1, D) - mean.view(-1, 1)) * rstd.view(-1, 1)
    gy = dyf * g
    dx = (rstd.view(-1, 1) * (gy - gy.mean(-1, keepdim=True) - xh * (gy * xh).mean(-1, keepdim=True))).to(dy.dtype)
    dxd = dropout(dx, p, seed, offset, salt) if p > 0 else dx
    for w, (out, val) in enumerate(((dg, (dyf * xh).sum(0)), (db, dyf.sum(0)), (dbias, dxd.float().sum(0)))):
        if out is not None:
            (out.add_ if (accmask >> w) & 1 else out.copy_)(val)
    return [dx.reshape(xs.shape), dxd.reshape(xs.shape)]


def linear_gelu_fwd(x, w, bias=None):
    u = x.float() @ w.float().t()
    if bias is not None:
        u = u + bias.float()
    u = u.to(x.dtype)
    return [F.gelu(u.float()).to(x.dtype), u]


def linear_dgrad_gelu(dy, w, u, wt=None):
    uf = u.float()
    cdf = 0.5 * (1 + torch.erf(uf * 0.7071067811865476))
    pdf = 0.3989422804014327 * torch.exp(-0.5 * uf * uf)
    return ((dy.float() @ w.float()) * (cdf + uf * pdf)).to(dy.dtype)


def gelu_fwd(x):
    return F.gelu(x.float()).to(x.dtype)


def gelu_bwd(dy, x):
    xf = x.float()
    cdf = 0.5 * (1 + torch.erf(xf * 0.7071067811865476))
    pdf = 0.3989422804014327 * torch.exp(-0.5 * xf * xf)
    return (dy.float() * (cdf + xf * pdf)).to(dy.dtype)


def tanh_fwd(x):
    return torch.tanh(x.float()).to(x.dtype)


def tanh_bwd(dy, y):
    return (dy.float() * (1 - y.float() ** 2)).to(dy.dtype)


def add_bf16(a, b):
    return (a.float() + b.float()).to(a.dtype)


def _attn_prep(qkv, ids, B, S, H):
    D = qkv.shape[-1] // 3
    t = qkv.float().view(B, S, 3, H, D // H)
    q, k, v = t[:, :, 0].transpose(1, 2), t[:, :, 1].transpose(1, 2), t[:, :, 2].transpose(1, 2)  # [B,H,S,d]
    bias = torch.zeros(B, 1, 1, S, device=qkv.device)
    if ids is not None:
        bias = torch.where((ids > 0).view(B, 1, 1, S), bias, torch.full_like(bias, -1e30))
    return q, k, v, bias, D


def _attn_drop(B, H, S, p, seed, offset, device):
    if p <= 0:
        return None
    idx = torch.arange(B * H * S * S, device=device, dtype=torch.int64) + offset
    keep = hash_uniform(seed, idx).view(B, H, S, S) >= p
    return keep.float() / (1.0 - p)


def attention_fwd(qkv, ids, B, S, H, p_drop, seed, offset, salt=None):
    seed = _salted(seed, salt)
    q, k, v, bias, D = _attn_prep(qkv, ids, B, S, H)
    s = q @ k.transpose(-1, -2) * 0.125 + bias
    lse = torch.logsumexp(s, -1)
    P = torch.exp(s - lse.unsqueeze(-1))
    dm = _attn_drop(B, H, S, p_drop, seed, offset, qkv.device)
    if dm is not None:
        P = P * dm
    P = P.to(qkv.dtype).float()
    ctx = (P @ v).transpose(1, 2).reshape(B * S, D)
    return [ctx.to(qkv.dtype), lse.reshape(B * H, S)]


def attention_bwd(dctx, qkv, ctx, lse, ids, B, S, H, p_drop, seed, offset, salt=None):
    seed = _salted(seed, salt)
    q, k, v, bias, D = _attn_prep(qkv, ids, B, S, H)
    d = D // H
    dO = dctx.float().view(B, S, H, d).transpose(1, 2)
    O = ctx.float().view(B, S, H, d).transpose(1, 2)
    s = q @ k.transpose(-1, -2) * 0.125 + bias
    P = torch.exp(s - lse.view(B, H, S, 1))
    dm = _attn_drop(B, H, S, p_drop, seed, offset, qkv.device)
    Pd = P * dm if dm is not None else P
    dV = Pd.to(qkv.dtype).float().transpose(-1, -2) @ dO
    dPd = dO @ v.transpose(-1, -2)
    dP = dPd * dm if dm is not None else dPd
    Dd = (dO * O).sum(-1, keepdim=True)
    dS = (P * (dP - Dd)).to(qkv.dtype).float()
    dQ = dS @ k * 0.125
    dK = dS.transpose(-1, -2) @ q * 0.125
    out = torch.stack([dQ, dK, dV], 2)  # [B,H,3,S,d]
    return out.permute(0, 3, 2, 1, 4).reshape(B * S, 3 * D).to(qkv.dtype)


def topk_rows(x, k, want_values):
    """Row-wise top-k of the last dim: larger first, ties to the smaller index, NaN above numbers
    (csrc/elementwise.hip topk_rows_kernel)."""
    xf = x.float().reshape(-1, x.shape[-1])
    v, i = torch.sort(xf, dim=-1, descending=True, stable=True)
    v, i = v[:, :k].contiguous(), i[:, :k].contiguous()
    return [v, i] if want_values else [i]


_SM_GOLD, _SM_M1, _SM_M2 = 0x9E3779B97F4A7C15, 0xBF58476D1CE4E5B9, 0x94D049BB133111EB


def _splitmix64(z):
    import numpy as np
    with np.errstate(over="ignore"):
        z = z + np.uint64(_SM_GOLD)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(_SM_M1)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(_SM_M2)
        return z ^ (z >> np.uint64(31))


def synth_images(labels, color, freq, S, seed, noise):
    """data/synthetic.py image formula with the counter-based noise of synth_images_kernel."""
    import math

    import numpy as np
    B, C = labels.numel(), color.shape[1]
    y = labels.long().cpu()
    step = np.float32(2 * math.pi) / np.float32(S - 1)
    t = torch.arange(S, dtype=torch.float32) * float(step)
    fy, fx = freq[y, 0].float().cpu(), freq[y, 1].float().cpu()
    pat = torch.sin(fy.view(B, 1, 1) * t.view(1, S, 1)) * torch.cos(fx.view(B, 1, 1) * t.view(1, 1, S))
    key = _splitmix64(np.array([seed & (2 ** 64 - 1)], dtype=np.uint64))[0]
    n = np.arange(B * C * S * S, dtype=np.uint64)
    u = (_splitmix64(key ^ n) >> np.uint64(40)).astype(np.float32) * np.float32(1.0 / 16777216.0)
    u = torch.from_numpy(u).view(B, C, S, S)
    x = 0.5 * color[y].float().cpu().view(B, C, 1, 1) + 0.25 * (pat.unsqueeze(1) + 1.0) * 0.5 + noise * u
    return x.clamp_(0.0, 1.0).to(labels.device)


# ------------------------------------------------------------------------------ fused BERT sublayers
def _linear(x, w, bias):
    M, C = x.shape
    N = w.shape[0]
    return conv_fwd(x.reshape(M, 1, 1, C), w.reshape(N, 1, 1, C), 1, 0, bias)[0].reshape(M, N)


def bert_attn_fwd(h, ids, wq, bq, wo, bo, g, b, B, S, H, p_attn, seed_a, off_a, p_hid, seed_h, off_h, eps,
                  salt=None):
    """csrc/transformer.hip bert_attn_fwd: [h1, qkv, ctx, lse, xs, mean, rstd] of
    h1 = LayerNorm(h + dropout(attn_out(attention(qkv(h)))))."""
    qkv = _linear(h, wq, bq)
    ctx, lse = attention_fwd(qkv, ids, B, S, H, p_attn, seed_a, off_a, salt)
    a = _linear(ctx, wo, bo)
    y, xs, mean, rstd = layernorm_fwd(a, h, g, b, eps, p_hid, seed_h, off_h, salt)
    return [y, qkv, ctx, lse, xs, mean, rstd]


def bert_ffn_fwd(h1, w1, b1, w2, b2, g, b, p_hid, seed_h, off_h, eps, salt=None):
    """csrc/transformer.hip bert_ffn_fwd: [h2, gelu(u), u, xs, mean, rstd] of
    h2 = LayerNorm(h1 + dropout(ffn2(gelu(ffn1(h1)))))."""
    gu, u = linear_gelu_fwd(h1, w1, b1)
    f = _linear(gu, w2, b2)
    y, xs, mean, rstd = layernorm_fwd(f, h1, g, b, eps, p_hid, seed_h, off_h, salt)
    return [y, gu, u, xs, mean, rstd]

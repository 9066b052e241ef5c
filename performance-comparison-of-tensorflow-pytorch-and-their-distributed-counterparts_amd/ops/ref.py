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
def conv_fwd(x, w, stride, pad, bias=None, resid=None, relu=False, want_stats=False):
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


def conv_dgrad(dy, w, H, W, stride, pad, resid=None):
    N, K, R, S, C = dy.shape[0], w.shape[0], w.shape[1], w.shape[2], w.shape[3]
    dx = torch.nn.grad.conv2d_input((N, C, H, W), _nchw(w), _nchw(dy), stride=stride, padding=pad)
    dx = _nhwc(dx)
    if resid is not None:
        dx = dx + resid.float().reshape(dx.shape)
    return dx.to(dy.dtype).contiguous()


def conv_wgrad(dy, x, out, R, S, stride, pad, accumulate):
    K, C = dy.shape[-1], x.shape[-1]
    dw = torch.nn.grad.conv2d_weight(_nchw(x), (K, C, R, S), _nchw(dy), stride=stride, padding=pad)
    dw = _nhwc(dw).reshape(out.shape).to(out.dtype)
    if accumulate:
        out.add_(dw)
    else:
        out.copy_(dw)


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


def bn_apply(x, scale, shift, x2=None, scale2=None, shift2=None, relu=False):
    y = x.float() * scale + shift
    if x2 is not None:
        y = y + (x2.float() * scale2 + shift2 if scale2 is not None else x2.float())
    if relu:
        y = torch.relu(y)
    return y.to(x.dtype)


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
def maxpool_fwd(x, k, s, pad, want_idx):
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


def gap_fwd(x):
    N, C = x.shape[0], x.shape[-1]
    return x.float().reshape(N, -1, C).mean(1).to(x.dtype)


def gap_bwd(dy, H, W):
    N, C = dy.shape
    return (dy.float() / (H * W)).view(N, 1, 1, C).expand(N, H, W, C).to(dy.dtype).contiguous()


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


# ------------------------------------------------------------------------------ dropout RNG
_M64 = (1 << 64) - 1


def _s64(v):
    v &= _M64
    return v - (1 << 64) if v >= (1 << 63) else v


def _lsr(z, k):
    # logical shift right on int64 two's-complement values
    return (z >> k) & ((1 << (64 - k)) - 1)


def hash_uniform(seed: int, idx: torch.Tensor) -> torch.Tensor:
    """Bit-exact torch port of ``uniform01`` in csrc/common.h (splitmix64 finaliser)."""
    z = torch.bitwise_xor(torch.tensor(_s64(seed), dtype=torch.int64, device=idx.device),
                          idx.long() * _s64(0x9E3779B97F4A7C15))
    z = torch.bitwise_xor(z, _lsr(z, 30)) * _s64(0xBF58476D1CE4E5B9)
    z = torch.bitwise_xor(z, _lsr(z, 27)) * _s64(0x94D049BB133111EB)
    z = torch.bitwise_xor(z, _lsr(z, 31))
    u32 = z & 0xFFFFFFFF
    return (u32 >> 8).float() * (1.0 / 16777216.0)


def dropout(x, p, seed, offset):
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


def cast_to_bf16(x, y):
    y.copy_(x.to(y.dtype))

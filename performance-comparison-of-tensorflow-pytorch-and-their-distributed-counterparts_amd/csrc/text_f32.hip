// fp32 kernels of the text encoders (the reference's precision: its BERT fine-tune runs fp32 end to
// end with no autocast, /root/reference/pytorch_on_language_distr.py:151-161,258-275).  The op
// wrappers in transformer.hip / rnn.hip / igemm.hip call these when their activations are fp32
// (``--dtype fp32``), so the fp32 text path runs on HIP kernels like the fp32 image path (f32.hip).
//
// Semantics are those of ops/ref.py (the CPU reference) evaluated in fp32: LayerNorm (+ residual,
// + dropout), embedding LayerNorm, erf-GELU / tanh, attention with additive padding mask and
// attention-probability dropout, embedding gather / scatter-add, masked mean pooling, and the
// BiLSTM recurrence with packed-sequence masking (state carried at padded steps).  Dropout masks
// use the same counter hash (uniform01) and element indexing as the bf16 kernels.
//
// These kernels favour simple, exact fp32 arithmetic over peak speed: the bf16 kernels carry the
// throughput path; this path exists for reference-precision parity runs.
#include "common.h"
#include "embed.h"
#include "f32.h"

#include <vector>

namespace pcmp {
namespace f32 {

static int tgrid(int64_t n, int threads = 256) {
  return (int)std::max<int64_t>(1, std::min<int64_t>(16384, (n + threads - 1) / threads));
}

// ------------------------------------------------------------------------------- elementwise
// mode 0: erf-GELU, 1: tanh
__global__ void act_fwd_f32_kernel(const float* __restrict__ x, float* __restrict__ y, int64_t n, int mode) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    y[i] = mode == 0 ? gelu_erf(x[i]) : tanhf(x[i]);
}
// mode 0: dy * gelu'(x); 1: dy * (1 - y^2)
__global__ void act_bwd_f32_kernel(const float* __restrict__ dy, const float* __restrict__ xy, float* __restrict__ dx,
                                   int64_t n, int mode) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const float v = xy[i];
    dx[i] = dy[i] * (mode == 0 ? dgelu_erf(v) : 1.f - v * v);
  }
}
__global__ void add_f32_kernel(const float* __restrict__ a, const float* __restrict__ b, float* __restrict__ y,
                               int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    y[i] = a[i] + b[i];
}

at::Tensor act_fwd(const at::Tensor& x, int mode) {
  PCMP_CHECK_CUDA(x); PCMP_CHECK_F32(x);
  auto xc = x.contiguous();
  auto y = at::empty_like(xc);
  if (xc.numel() == 0) return y;
  hipLaunchKernelGGL(act_fwd_f32_kernel, dim3(tgrid(xc.numel())), dim3(256), 0, cur_stream(), ptr<float>(xc),
                     ptr<float>(y), xc.numel(), mode);
  PCMP_LAUNCH_CHECK();
  return y;
}
at::Tensor act_bwd(const at::Tensor& dy, const at::Tensor& xy, int mode) {
  PCMP_CHECK_F32(dy); PCMP_CHECK_F32(xy);
  auto dyc = dy.contiguous(), xc = xy.contiguous();
  TORCH_CHECK(dyc.numel() == xc.numel(), "act_bwd: shapes");
  auto dx = at::empty_like(xc);
  if (xc.numel() == 0) return dx;
  hipLaunchKernelGGL(act_bwd_f32_kernel, dim3(tgrid(xc.numel())), dim3(256), 0, cur_stream(), ptr<float>(dyc),
                     ptr<float>(xc), ptr<float>(dx), xc.numel(), mode);
  PCMP_LAUNCH_CHECK();
  return dx;
}
at::Tensor add(const at::Tensor& a, const at::Tensor& b) {
  PCMP_CHECK_F32(a); PCMP_CHECK_F32(b);
  auto ac = a.contiguous(), bc = b.contiguous();
  TORCH_CHECK(ac.numel() == bc.numel(), "add: shapes");
  auto y = at::empty_like(ac);
  if (ac.numel() == 0) return y;
  hipLaunchKernelGGL(add_f32_kernel, dim3(tgrid(ac.numel())), dim3(256), 0, cur_stream(), ptr<float>(ac), ptr<float>(bc),
                     ptr<float>(y), ac.numel());
  PCMP_LAUNCH_CHECK();
  return y;
}

// ------------------------------------------------------------------------------- LayerNorm
// One wave per row.  xs = drop(x) + r (+ pos[row % S] + tt for the embedding form), stored when it
// differs from x; mean / rstd over xs; y = (xs - mean) * rstd * g + b.
__global__ void __launch_bounds__(256) ln_fwd_f32_kernel(const float* __restrict__ x, const float* __restrict__ r,
                                                          const float* __restrict__ g, const float* __restrict__ b,
                                                          float* __restrict__ y, float* __restrict__ xs_out,
                                                          float* __restrict__ mean, float* __restrict__ rstd, int M,
                                                          int D, float eps, float p, uint64_t seed, uint64_t offset,
                                                          const int64_t* salt, int S, const float* __restrict__ tt) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= M) return;
  const float* xr = x + (size_t)row * D;
  const float* rr = r ? (S > 0 ? r + (size_t)(row % S) * D : r + (size_t)row * D) : nullptr;
  const uint64_t sd = dropout_seed(seed, salt);
  const float* src = xr;
  float sum = 0.f;
  if (xs_out) {
    float* xo = xs_out + (size_t)row * D;
    for (int i = lane; i < D; i += 64) {
      float v = xr[i];
      if (p > 0.f) v = uniform01(sd, offset + (uint64_t)row * D + i) >= p ? v / (1.f - p) : 0.f;
      if (rr) v += rr[i];
      if (tt) v += tt[i];
      xo[i] = v;
      sum += v;
    }
    src = xo;
  } else {
    for (int i = lane; i < D; i += 64) sum += xr[i];
  }
  const float mu = warp_sum(sum) / D;
  float sq = 0.f;
  for (int i = lane; i < D; i += 64) {
    const float d = src[i] - mu;
    sq += d * d;
  }
  const float rs = rsqrtf(warp_sum(sq) / D + eps);
  float* yr = y + (size_t)row * D;
  for (int i = lane; i < D; i += 64) yr[i] = (src[i] - mu) * rs * g[i] + b[i];
  if (lane == 0) {
    mean[row] = mu;
    rstd[row] = rs;
  }
}

std::vector<at::Tensor> layernorm_fwd(const at::Tensor& x, const c10::optional<at::Tensor>& r, const at::Tensor& g,
                                      const at::Tensor& b, double eps, double p, int64_t seed, int64_t offset,
                                      const c10::optional<at::Tensor>& salt) {
  PCMP_CHECK_F32(x); PCMP_CHECK_CONTIG(x); PCMP_CHECK_F32(g); PCMP_CHECK_F32(b);
  const int D = x.size(-1);
  const int M = x.numel() / D;
  TORCH_CHECK(p >= 0.0 && p < 1.0, "layernorm: dropout p in [0, 1)");
  const bool hr = r.has_value() && r->defined();
  at::Tensor rc;
  if (hr) {
    rc = r->contiguous();
    PCMP_CHECK_F32(rc);
    TORCH_CHECK(rc.numel() == x.numel(), "layernorm: residual shape");
  }
  auto y = at::empty_like(x);
  at::Tensor xs = (hr || p > 0.0) ? at::empty_like(x) : x;
  auto mean = at::empty({M}, x.options()), rstd = at::empty({M}, x.options());
  if (M == 0) return {y, xs, mean, rstd};
  hipLaunchKernelGGL(ln_fwd_f32_kernel, dim3(ceil_div(M, 4)), dim3(256), 0, cur_stream(), ptr<float>(x),
                     hr ? ptr<float>(rc) : nullptr, ptr<float>(g), ptr<float>(b), ptr<float>(y),
                     (hr || p > 0.0) ? ptr<float>(xs) : nullptr, ptr<float>(mean), ptr<float>(rstd), M, D, (float)eps,
                     (float)p, (uint64_t)seed, (uint64_t)offset, p > 0.0 ? salt_ptr(salt) : nullptr, 0, nullptr);
  PCMP_LAUNCH_CHECK();
  return {y, xs, mean, rstd};
}

std::vector<at::Tensor> embed_layernorm_fwd(const at::Tensor& x, const at::Tensor& pos, const at::Tensor& tt,
                                            const at::Tensor& g, const at::Tensor& b, double eps) {
  PCMP_CHECK_F32(x); PCMP_CHECK_CONTIG(x); PCMP_CHECK_F32(pos); PCMP_CHECK_CONTIG(pos);
  PCMP_CHECK_F32(tt); PCMP_CHECK_CONTIG(tt); PCMP_CHECK_F32(g); PCMP_CHECK_F32(b);
  const int D = x.size(-1);
  const int M = x.numel() / D;
  TORCH_CHECK(pos.numel() % D == 0 && pos.numel() > 0, "embed_layernorm: pos must be [S, D]");
  const int S = pos.numel() / D;
  TORCH_CHECK(M % S == 0 && tt.numel() == D, "embed_layernorm: rows must be a multiple of S, tt [D]");
  auto y = at::empty_like(x), xs = at::empty_like(x);
  auto mean = at::empty({M}, x.options()), rstd = at::empty({M}, x.options());
  if (M == 0) return {y, xs, mean, rstd};
  hipLaunchKernelGGL(ln_fwd_f32_kernel, dim3(ceil_div(M, 4)), dim3(256), 0, cur_stream(), ptr<float>(x),
                     ptr<float>(pos), ptr<float>(g), ptr<float>(b), ptr<float>(y), ptr<float>(xs), ptr<float>(mean),
                     ptr<float>(rstd), M, D, (float)eps, 0.f, (uint64_t)0, (uint64_t)0, nullptr, S, ptr<float>(tt));
  PCMP_LAUNCH_CHECK();
  return {y, xs, mean, rstd};
}

// LayerNorm backward (+ dropout of dx): one wave per row, LN_RPB rows per block; per-block column
// partials of dy*xhat, dy, dxd -> part[block][np][D], reduced by col_reduce_f32_kernel (fixed order).
constexpr int LN_RPB = 16;
__global__ void __launch_bounds__(256) ln_bwd_f32_kernel(const float* __restrict__ dy, const float* __restrict__ xs,
                                                          const float* __restrict__ mean,
                                                          const float* __restrict__ rstd, const float* __restrict__ g,
                                                          float* __restrict__ dx, float* __restrict__ dxd,
                                                          float* __restrict__ part, int M, int D, int np, float p,
                                                          uint64_t seed, uint64_t offset, const int64_t* salt) {
  extern __shared__ float sp[];   // [4 waves][np][D]
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  float* mine = sp + (size_t)w * np * D;
  for (int i = lane; i < np * D; i += 64) mine[i] = 0.f;
  const uint64_t sd = dropout_seed(seed, salt);
  for (int rr = w; rr < LN_RPB; rr += 4) {
    const int row = blockIdx.x * LN_RPB + rr;
    if (row >= M) break;
    const float* dyr = dy + (size_t)row * D;
    const float* xr = xs + (size_t)row * D;
    const float mu = mean[row], rs = rstd[row];
    float s1 = 0.f, s2 = 0.f;
    for (int i = lane; i < D; i += 64) {
      const float xh = (xr[i] - mu) * rs;
      const float gy = dyr[i] * g[i];
      s1 += gy;
      s2 += gy * xh;
      mine[i] += dyr[i] * xh;
      mine[D + i] += dyr[i];
    }
    s1 = warp_sum(s1) / D;
    s2 = warp_sum(s2) / D;
    for (int i = lane; i < D; i += 64) {
      const float xh = (xr[i] - mu) * rs;
      const float v = rs * (dyr[i] * g[i] - s1 - xh * s2);
      dx[(size_t)row * D + i] = v;
      if (dxd != dx) {
        const float vd = uniform01(sd, offset + (uint64_t)row * D + i) >= p ? v / (1.f - p) : 0.f;
        dxd[(size_t)row * D + i] = vd;
        if (np == 3) mine[2 * D + i] += vd;
      } else if (np == 3) {
        mine[2 * D + i] += v;
      }
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < np * D; i += blockDim.x) {
    float s = 0.f;
    for (int ww = 0; ww < 4; ++ww) s += sp[(size_t)ww * np * D + i];
    part[(size_t)blockIdx.x * np * D + i] = s;
  }
}

// out_w[d] (+)= sum_t part[t][w][d]  (bit w of accmask: accumulate)
__global__ void col_reduce_f32_kernel(const float* __restrict__ part, int T, int np, int D, float* o0, float* o1,
                                      float* o2, int accmask) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= np * D) return;
  const int w = i / D, d = i - w * D;
  float* o = w == 0 ? o0 : (w == 1 ? o1 : o2);
  if (!o) return;
  float s = 0.f;
  for (int t = 0; t < T; ++t) s += part[((size_t)t * np + w) * D + d];
  o[d] = ((accmask >> w) & 1) ? o[d] + s : s;
}

std::vector<at::Tensor> layernorm_bwd_fused(const at::Tensor& dy, const at::Tensor& xs, const at::Tensor& mean,
                                            const at::Tensor& rstd, const at::Tensor& g,
                                            const c10::optional<at::Tensor>& dg, const c10::optional<at::Tensor>& db,
                                            const c10::optional<at::Tensor>& dbias, int64_t accmask, double p,
                                            int64_t seed, int64_t offset, const c10::optional<at::Tensor>& salt) {
  PCMP_CHECK_F32(xs); PCMP_CHECK_CONTIG(xs); PCMP_CHECK_F32(g); PCMP_CHECK_F32(mean); PCMP_CHECK_F32(rstd);
  auto dyc = dy.contiguous();
  PCMP_CHECK_F32(dyc);
  const int D = xs.size(-1);
  const int M = xs.numel() / D;
  TORCH_CHECK(dyc.numel() == xs.numel() && mean.numel() == M && rstd.numel() == M && g.numel() == D,
              "layernorm_bwd (fp32): shapes");
  TORCH_CHECK(p >= 0.0 && p < 1.0, "layernorm_bwd (fp32): dropout p in [0, 1)");
  auto dx = at::empty_like(xs);
  at::Tensor dxd = p > 0.0 ? at::empty_like(xs) : dx;
  float* outs[3] = {nullptr, nullptr, nullptr};
  const c10::optional<at::Tensor>* ts[3] = {&dg, &db, &dbias};
  for (int w = 0; w < 3; ++w) {
    if (ts[w]->has_value() && (*ts[w])->defined()) {
      PCMP_CHECK_F32(**ts[w]); PCMP_CHECK_CONTIG(**ts[w]);
      TORCH_CHECK((*ts[w])->numel() == D, "layernorm_bwd (fp32): gradient output size");
      outs[w] = ptr<float>(**ts[w]);
    }
  }
  if (M == 0) return {dx, dxd};
  const int np = outs[2] ? 3 : 2;
  TORCH_CHECK((size_t)4 * np * D * sizeof(float) <= 160 * 1024, "layernorm_bwd (fp32): D too large");
  const int T = ceil_div(M, LN_RPB);
  auto part = at::empty({T, np, D}, mean.options());
  auto st = cur_stream();
  PCMP_ALLOW_BIG_LDS(ln_bwd_f32_kernel);
  hipLaunchKernelGGL(ln_bwd_f32_kernel, dim3(T), dim3(256), (size_t)4 * np * D * sizeof(float), st, ptr<float>(dyc),
                     ptr<float>(xs), ptr<float>(mean), ptr<float>(rstd), ptr<float>(g), ptr<float>(dx),
                     ptr<float>(dxd), ptr<float>(part), M, D, np, (float)p, (uint64_t)seed, (uint64_t)offset,
                     p > 0.0 ? salt_ptr(salt) : nullptr);
  PCMP_LAUNCH_CHECK();
  if (outs[0] || outs[1] || outs[2]) {
    hipLaunchKernelGGL(col_reduce_f32_kernel, dim3(ceil_div(np * D, 256)), dim3(256), 0, st, ptr<float>(part), T, np, D,
                       outs[0], outs[1], outs[2], (int)accmask);
    PCMP_LAUNCH_CHECK();
  }
  return {dx, dxd};
}

at::Tensor layernorm_bwd(const at::Tensor& dy, const at::Tensor& xs, const at::Tensor& mean, const at::Tensor& rstd,
                         const at::Tensor& g, const c10::optional<at::Tensor>& dg, const c10::optional<at::Tensor>& db,
                         bool accumulate) {
  return layernorm_bwd_fused(dy, xs, mean, rstd, g, dg, db, c10::nullopt, accumulate ? 3 : 0, 0.0, 0, 0,
                             c10::nullopt)[0];
}

// ------------------------------------------------------------------------------- attention
// qkv [B*S][3D] (q | k | v, head h at columns h*64..), ctx [B*S][D], lse [B*H][S]; scale 1/8;
// additive mask -1e30 on padded keys (ids == 0); probability dropout index ((b*H+h)*S+q)*S+key.
constexpr int AD32 = 64;
__global__ void __launch_bounds__(256) attn_fwd_f32_kernel(const float* __restrict__ qkv, const int64_t* __restrict__ ids,
                                                            float* __restrict__ ctx, float* __restrict__ lse, int B,
                                                            int S, int H, float p, uint64_t seed, uint64_t offset,
                                                            const int64_t* salt) {
  extern __shared__ float sm[];
  float* sK = sm;                  // [S][64]
  float* sV = sm + S * AD32;       // [S][64]
  float* sB = sV + S * AD32;       // [S] key bias
  const int bh = blockIdx.x, b = bh / H, h = bh % H;
  const int D = H * AD32, D3 = 3 * D;
  const float* base = qkv + (size_t)b * S * D3;
  for (int i = threadIdx.x; i < S * AD32; i += blockDim.x) {
    const int key = i / AD32, d = i % AD32;
    sK[i] = base[(size_t)key * D3 + D + h * AD32 + d];
    sV[i] = base[(size_t)key * D3 + 2 * D + h * AD32 + d];
  }
  for (int key = threadIdx.x; key < S; key += blockDim.x)
    sB[key] = (ids && ids[(size_t)b * S + key] <= 0) ? -1e30f : 0.f;
  __syncthreads();
  const uint64_t sd = dropout_seed(seed, salt);
  for (int q = threadIdx.x; q < S; q += blockDim.x) {
    float qv[AD32];
#pragma unroll
    for (int d = 0; d < AD32; ++d) qv[d] = base[(size_t)q * D3 + h * AD32 + d];
    float m = -INFINITY, l = 0.f;
    for (int key = 0; key < S; ++key) {
      float s = 0.f;
#pragma unroll
      for (int d = 0; d < AD32; ++d) s += qv[d] * sK[key * AD32 + d];
      s = s * 0.125f + sB[key];
      const float mn = fmaxf(m, s);
      l = l * __expf(m - mn) + __expf(s - mn);
      m = mn;
    }
    const float ls = m + __logf(l);
    float acc[AD32];
#pragma unroll
    for (int d = 0; d < AD32; ++d) acc[d] = 0.f;
    const uint64_t rowidx = offset + ((uint64_t)bh * S + q) * S;
    for (int key = 0; key < S; ++key) {
      float s = 0.f;
#pragma unroll
      for (int d = 0; d < AD32; ++d) s += qv[d] * sK[key * AD32 + d];
      float pr = __expf(s * 0.125f + sB[key] - ls);
      if (p > 0.f) pr = uniform01(sd, rowidx + key) >= p ? pr / (1.f - p) : 0.f;
#pragma unroll
      for (int d = 0; d < AD32; ++d) acc[d] += pr * sV[key * AD32 + d];
    }
    float* o = ctx + ((size_t)b * S + q) * D + h * AD32;
#pragma unroll
    for (int d = 0; d < AD32; ++d) o[d] = acc[d];
    lse[(size_t)bh * S + q] = ls;
  }
}

// backward pass 1 (one thread per query): P, dP, dS rows -> scratch Pd / dS [B*H][S][S]; dQ
__global__ void __launch_bounds__(256) attn_bwd_q_f32_kernel(const float* __restrict__ qkv,
                                                              const int64_t* __restrict__ ids,
                                                              const float* __restrict__ dctx,
                                                              const float* __restrict__ ctx,
                                                              const float* __restrict__ lse, float* __restrict__ Pd,
                                                              float* __restrict__ dS, float* __restrict__ dqkv, int B,
                                                              int S, int H, float p, uint64_t seed, uint64_t offset,
                                                              const int64_t* salt) {
  extern __shared__ float sm[];
  float* sK = sm;
  float* sV = sm + S * AD32;
  float* sB = sV + S * AD32;
  const int bh = blockIdx.x, b = bh / H, h = bh % H;
  const int D = H * AD32, D3 = 3 * D;
  const float* base = qkv + (size_t)b * S * D3;
  for (int i = threadIdx.x; i < S * AD32; i += blockDim.x) {
    const int key = i / AD32, d = i % AD32;
    sK[i] = base[(size_t)key * D3 + D + h * AD32 + d];
    sV[i] = base[(size_t)key * D3 + 2 * D + h * AD32 + d];
  }
  for (int key = threadIdx.x; key < S; key += blockDim.x)
    sB[key] = (ids && ids[(size_t)b * S + key] <= 0) ? -1e30f : 0.f;
  __syncthreads();
  const uint64_t sd = dropout_seed(seed, salt);
  for (int q = threadIdx.x; q < S; q += blockDim.x) {
    float qv[AD32], dov[AD32];
    float Dd = 0.f;
#pragma unroll
    for (int d = 0; d < AD32; ++d) {
      qv[d] = base[(size_t)q * D3 + h * AD32 + d];
      dov[d] = dctx[((size_t)b * S + q) * D + h * AD32 + d];
      Dd += dov[d] * ctx[((size_t)b * S + q) * D + h * AD32 + d];
    }
    const float ls = lse[(size_t)bh * S + q];
    float dq[AD32];
#pragma unroll
    for (int d = 0; d < AD32; ++d) dq[d] = 0.f;
    const uint64_t rowidx = offset + ((uint64_t)bh * S + q) * S;
    float* pdr = Pd + ((size_t)bh * S + q) * S;
    float* dsr = dS + ((size_t)bh * S + q) * S;
    for (int key = 0; key < S; ++key) {
      float s = 0.f, dpd = 0.f;
#pragma unroll
      for (int d = 0; d < AD32; ++d) {
        s += qv[d] * sK[key * AD32 + d];
        dpd += dov[d] * sV[key * AD32 + d];
      }
      const float P = __expf(s * 0.125f + sB[key] - ls);
      float dm = 1.f;
      if (p > 0.f) dm = uniform01(sd, rowidx + key) >= p ? 1.f / (1.f - p) : 0.f;
      const float ds = P * (dpd * dm - Dd);
      pdr[key] = P * dm;
      dsr[key] = ds;
#pragma unroll
      for (int d = 0; d < AD32; ++d) dq[d] += ds * sK[key * AD32 + d];
    }
    float* o = dqkv + ((size_t)b * S + q) * D3 + h * AD32;
#pragma unroll
    for (int d = 0; d < AD32; ++d) o[d] = dq[d] * 0.125f;
  }
}

// backward pass 2 (one thread per key): dV = Pd^T dO, dK = dS^T Q / 8
__global__ void __launch_bounds__(256) attn_bwd_kv_f32_kernel(const float* __restrict__ qkv,
                                                               const float* __restrict__ dctx,
                                                               const float* __restrict__ Pd,
                                                               const float* __restrict__ dS, float* __restrict__ dqkv,
                                                               int B, int S, int H) {
  extern __shared__ float sm[];
  float* sQ = sm;               // [S][64]
  float* sO = sm + S * AD32;    // dO [S][64]
  const int bh = blockIdx.x, b = bh / H, h = bh % H;
  const int D = H * AD32, D3 = 3 * D;
  for (int i = threadIdx.x; i < S * AD32; i += blockDim.x) {
    const int q = i / AD32, d = i % AD32;
    sQ[i] = qkv[((size_t)b * S + q) * D3 + h * AD32 + d];
    sO[i] = dctx[((size_t)b * S + q) * D + h * AD32 + d];
  }
  __syncthreads();
  for (int key = threadIdx.x; key < S; key += blockDim.x) {
    float dk[AD32], dv[AD32];
#pragma unroll
    for (int d = 0; d < AD32; ++d) dk[d] = dv[d] = 0.f;
    for (int q = 0; q < S; ++q) {
      const float pd = Pd[((size_t)bh * S + q) * S + key];
      const float ds = dS[((size_t)bh * S + q) * S + key];
#pragma unroll
      for (int d = 0; d < AD32; ++d) {
        dv[d] += pd * sO[q * AD32 + d];
        dk[d] += ds * sQ[q * AD32 + d];
      }
    }
    float* o = dqkv + ((size_t)b * S + key) * D3 + h * AD32;
#pragma unroll
    for (int d = 0; d < AD32; ++d) {
      o[D + d] = dk[d] * 0.125f;
      o[2 * D + d] = dv[d];
    }
  }
}

static size_t attn_f32_smem(int S) { return ((size_t)2 * S * AD32 + S) * sizeof(float); }

std::vector<at::Tensor> attention_fwd(const at::Tensor& qkv, const c10::optional<at::Tensor>& ids, int64_t B,
                                      int64_t S, int64_t H, double p_drop, int64_t seed, int64_t offset,
                                      const c10::optional<at::Tensor>& salt) {
  PCMP_CHECK_F32(qkv); PCMP_CHECK_CONTIG(qkv);
  const int D3 = qkv.size(-1), D = D3 / 3;
  TORCH_CHECK(D == H * AD32, "attention (fp32): head dim must be 64");
  TORCH_CHECK(S >= 1 && S <= 256, "attention (fp32): S <= 256");
  TORCH_CHECK(qkv.numel() == B * S * D3, "attention (fp32): qkv shape");
  auto ctx = at::empty({B * S, D}, qkv.options());
  auto lse = at::empty({B * H, S}, qkv.options());
  at::Tensor idc;
  if (ids.has_value() && ids->defined()) idc = ids->contiguous();
  if (B * H == 0) return {ctx, lse};
  PCMP_ALLOW_BIG_LDS(attn_fwd_f32_kernel);
  hipLaunchKernelGGL(attn_fwd_f32_kernel, dim3(B * H), dim3(std::min<int64_t>(256, (S + 63) / 64 * 64)),
                     attn_f32_smem(S), cur_stream(), ptr<float>(qkv), idc.defined() ? idc.data_ptr<int64_t>() : nullptr,
                     ptr<float>(ctx), ptr<float>(lse), (int)B, (int)S, (int)H, (float)p_drop, (uint64_t)seed,
                     (uint64_t)offset, p_drop > 0.0 ? salt_ptr(salt) : nullptr);
  PCMP_LAUNCH_CHECK();
  return {ctx, lse};
}

at::Tensor attention_bwd(const at::Tensor& dctx, const at::Tensor& qkv, const at::Tensor& ctx, const at::Tensor& lse,
                         const c10::optional<at::Tensor>& ids, int64_t B, int64_t S, int64_t H, double p_drop,
                         int64_t seed, int64_t offset, const c10::optional<at::Tensor>& salt) {
  PCMP_CHECK_F32(qkv); PCMP_CHECK_CONTIG(qkv); PCMP_CHECK_F32(ctx); PCMP_CHECK_CONTIG(ctx); PCMP_CHECK_F32(lse);
  auto dc = dctx.contiguous();
  PCMP_CHECK_F32(dc);
  const int D3 = qkv.size(-1), D = D3 / 3;
  TORCH_CHECK(D == H * AD32 && S >= 1 && S <= 256, "attention_bwd (fp32): head dim 64, S <= 256");
  TORCH_CHECK(qkv.numel() == B * S * D3 && dc.numel() == B * S * D && ctx.numel() == B * S * D &&
              lse.numel() == B * H * S, "attention_bwd (fp32): shapes");
  auto dqkv = at::empty_like(qkv);
  if (B * H == 0) return dqkv;
  at::Tensor idc;
  if (ids.has_value() && ids->defined()) idc = ids->contiguous();
  auto Pd = at::empty({B * H, S, S}, qkv.options());
  auto dS = at::empty({B * H, S, S}, qkv.options());
  const dim3 blk(std::min<int64_t>(256, (S + 63) / 64 * 64));
  auto st = cur_stream();
  PCMP_ALLOW_BIG_LDS(attn_bwd_q_f32_kernel);
  hipLaunchKernelGGL(attn_bwd_q_f32_kernel, dim3(B * H), blk, attn_f32_smem(S), st, ptr<float>(qkv),
                     idc.defined() ? idc.data_ptr<int64_t>() : nullptr, ptr<float>(dc), ptr<float>(ctx),
                     ptr<float>(lse), ptr<float>(Pd), ptr<float>(dS), ptr<float>(dqkv), (int)B, (int)S, (int)H,
                     (float)p_drop, (uint64_t)seed, (uint64_t)offset, p_drop > 0.0 ? salt_ptr(salt) : nullptr);
  PCMP_LAUNCH_CHECK();
  PCMP_ALLOW_BIG_LDS(attn_bwd_kv_f32_kernel);
  hipLaunchKernelGGL(attn_bwd_kv_f32_kernel, dim3(B * H), blk, (size_t)2 * S * AD32 * sizeof(float), st,
                     ptr<float>(qkv), ptr<float>(dc), ptr<float>(Pd), ptr<float>(dS), ptr<float>(dqkv), (int)B, (int)S,
                     (int)H);
  PCMP_LAUNCH_CHECK();
  return dqkv;
}

// ------------------------------------------------------------------------------- embedding / pooling
__global__ void embedding_fwd_f32_kernel(const int64_t* __restrict__ ids, const float* __restrict__ W,
                                         float* __restrict__ out, int64_t rows, int E) {
  const int64_t n = rows * E;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / E;
    out[i] = W[ids[r] * E + (i - r * E)];
  }
}
__global__ void embedding_bwd_f32_kernel(const int64_t* __restrict__ ids, const float* __restrict__ dy,
                                         float* __restrict__ dW, int64_t rows, int E, int64_t padding_idx) {
  const int64_t n = rows * E;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / E;
    const int64_t id = ids[r];
    if (id != padding_idx) atomicAdd(dW + id * E + (i - r * E), dy[i]);
  }
}

at::Tensor embedding_fwd(const at::Tensor& ids, const at::Tensor& W) {
  PCMP_CHECK_CUDA(ids); PCMP_CHECK_F32(W); PCMP_CHECK_CONTIG(W);
  TORCH_CHECK(ids.scalar_type() == at::kLong, "ids int64");
  const int E = W.size(1);
  auto idc = ids.contiguous();
  auto sizes = idc.sizes().vec();
  sizes.push_back(E);
  auto out = at::empty(sizes, W.options());
  const int64_t rows = idc.numel();
  if (rows == 0) return out;
  hipLaunchKernelGGL(embedding_fwd_f32_kernel, dim3(tgrid(rows * E)), dim3(256), 0, cur_stream(),
                     idc.data_ptr<int64_t>(), ptr<float>(W), ptr<float>(out), rows, E);
  PCMP_LAUNCH_CHECK();
  return out;
}

void embedding_bwd(const at::Tensor& ids, const at::Tensor& dy, at::Tensor dW, int64_t padding_idx, bool accumulate) {
  PCMP_CHECK_F32(dy); PCMP_CHECK_F32(dW); PCMP_CHECK_CONTIG(dW);
  auto idc = ids.contiguous();
  auto dyc = dy.contiguous();
  const int E = dW.size(-1);
  if (!accumulate) dW.zero_();
  const int64_t rows = idc.numel();
  if (rows == 0) return;
  if (kn_emb_atomic.get()) {
    hipLaunchKernelGGL(embedding_bwd_f32_kernel, dim3(tgrid(rows * E)), dim3(256), 0, cur_stream(),
                       idc.data_ptr<int64_t>(), ptr<float>(dyc), ptr<float>(dW), rows, E, padding_idx);
  } else {   // deterministic segmented reduction (rnn.hip embedding_bwd_seg_kernel)
    embedding_bwd_det<float>(idc, ptr<float>(dyc), ptr<float>(dW), dW.size(0), E, padding_idx, cur_stream());
  }
  PCMP_LAUNCH_CHECK();
}

__global__ void masked_mean_fwd_f32_kernel(const float* __restrict__ x, const int64_t* __restrict__ ids, int S, int D,
                                           float* __restrict__ y) {
  const int b = blockIdx.x;
  int cnt = 0;
  for (int s = 0; s < S; ++s) cnt += ids[(size_t)b * S + s] > 0;
  const float inv = 1.f / (float)max(cnt, 1);
  for (int d = threadIdx.x; d < D; d += blockDim.x) {
    float acc = 0.f;
    for (int s = 0; s < S; ++s)
      if (ids[(size_t)b * S + s] > 0) acc += x[((size_t)b * S + s) * D + d];
    y[(size_t)b * D + d] = acc * inv;
  }
}
__global__ void masked_mean_bwd_f32_kernel(const float* __restrict__ dy, const int64_t* __restrict__ ids, int S, int D,
                                           float* __restrict__ dx) {
  const int b = blockIdx.x;
  int cnt = 0;
  for (int s = 0; s < S; ++s) cnt += ids[(size_t)b * S + s] > 0;
  const float inv = 1.f / (float)max(cnt, 1);
  for (int i = threadIdx.x; i < S * D; i += blockDim.x) {
    const int s = i / D, d = i % D;
    dx[(size_t)b * S * D + i] = ids[(size_t)b * S + s] > 0 ? dy[(size_t)b * D + d] * inv : 0.f;
  }
}

at::Tensor masked_mean_fwd(const at::Tensor& x, const at::Tensor& ids) {
  PCMP_CHECK_F32(x); PCMP_CHECK_CONTIG(x);
  const int B = x.size(0), S = x.size(1), D = x.size(2);
  auto y = at::empty({B, D}, x.options());
  auto idc = ids.contiguous();
  if (B == 0) return y;
  hipLaunchKernelGGL(masked_mean_fwd_f32_kernel, dim3(B), dim3(256), 0, cur_stream(), ptr<float>(x),
                     idc.data_ptr<int64_t>(), S, D, ptr<float>(y));
  PCMP_LAUNCH_CHECK();
  return y;
}

at::Tensor masked_mean_bwd(const at::Tensor& dy, const at::Tensor& ids, int64_t S) {
  PCMP_CHECK_F32(dy);
  const int B = dy.size(0), D = dy.size(1);
  auto dx = at::empty({B, S, D}, dy.options());
  auto idc = ids.contiguous();
  auto dyc = dy.contiguous();
  if (B == 0) return dx;
  hipLaunchKernelGGL(masked_mean_bwd_f32_kernel, dim3(B), dim3(256), 0, cur_stream(), ptr<float>(dyc),
                     idc.data_ptr<int64_t>(), (int)S, D, ptr<float>(dx));
  PCMP_LAUNCH_CHECK();
  return dx;
}

// ------------------------------------------------------------------------------- BiLSTM recurrence
// One workgroup per (direction, block of LR sequences): it owns every hidden unit of those rows,
// so the recurrence needs no inter-workgroup exchange.  Thread j = hidden unit j (H <= 1024).
// Forward: pre[b][g*H+j] = gx + sum_k h[b][k] W[g*H+j][k], read through the transposed copy
// Wt[dir][k][g*H+j] (coalesced over j).  Backward: dh_rec[b][j] = sum_r dg[b][r] W[r][j].
constexpr int LR = 4;

__global__ void lstm_transpose_f32_kernel(const float* __restrict__ w, float* __restrict__ wt, int R, int C) {
  // w [2][R][C] -> wt [2][C][R]
  const int64_t n = 2ll * R * C;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t d = i / ((int64_t)R * C), rem = i - d * R * C;
    const int c = (int)(rem / R), r = (int)(rem - (int64_t)c * R);
    wt[i] = w[d * R * C + (int64_t)r * C + c];
  }
}

__device__ __forceinline__ float sigm_f32(float x) { return 1.f / (1.f + expf(-x)); }

__global__ void lstm_fwd_f32_kernel(const float* __restrict__ gx, const float* __restrict__ wt,
                                    const int64_t* __restrict__ ids, float* __restrict__ hout,
                                    float* __restrict__ gates, float* __restrict__ cst, int B, int S, int H) {
  extern __shared__ float sh[];   // [LR][H]
  const int nrb = (B + LR - 1) / LR;
  const int dir = blockIdx.x / nrb, b0 = (blockIdx.x % nrb) * LR;
  const int j = threadIdx.x;
  const int G4 = 4 * H;
  const float* W = wt + (size_t)dir * H * G4;
  float c[LR], h[LR];
#pragma unroll
  for (int r = 0; r < LR; ++r) {
    c[r] = h[r] = 0.f;
    sh[r * H + j] = 0.f;
  }
  __syncthreads();
  for (int step = 0; step < S; ++step) {
    const int t = dir == 0 ? step : S - 1 - step;
    float acc[LR][4];
#pragma unroll
    for (int r = 0; r < LR; ++r) {
      const int b = b0 + r;
#pragma unroll
      for (int g = 0; g < 4; ++g)
        acc[r][g] = b < B ? gx[(((size_t)b * S + t) * 2 + dir) * G4 + g * H + j] : 0.f;
    }
    for (int k = 0; k < H; ++k) {
      float w[4];
#pragma unroll
      for (int g = 0; g < 4; ++g) w[g] = W[(size_t)k * G4 + g * H + j];
#pragma unroll
      for (int r = 0; r < LR; ++r) {
        const float hk = sh[r * H + k];
#pragma unroll
        for (int g = 0; g < 4; ++g) acc[r][g] += hk * w[g];
      }
    }
    __syncthreads();   // every thread has read h_{t-1} from LDS
#pragma unroll
    for (int r = 0; r < LR; ++r) {
      const int b = b0 + r;
      if (b >= B) continue;
      const float ig = sigm_f32(acc[r][0]), fg = sigm_f32(acc[r][1]), gg = tanhf(acc[r][2]), og = sigm_f32(acc[r][3]);
      if (ids[(size_t)b * S + t] > 0) {
        c[r] = fg * c[r] + ig * gg;
        h[r] = og * tanhf(c[r]);
      }
      const size_t gb = (((size_t)b * S + t) * 2 + dir) * G4;
      gates[gb + j] = ig;
      gates[gb + H + j] = fg;
      gates[gb + 2 * H + j] = gg;
      gates[gb + 3 * H + j] = og;
      cst[(((size_t)b * S + t) * 2 + dir) * H + j] = c[r];
      hout[((size_t)b * S + t) * 2 * H + dir * H + j] = h[r];
      sh[r * H + j] = h[r];
    }
    __syncthreads();
  }
}

__global__ void lstm_bwd_f32_kernel(const float* __restrict__ dhout, const float* __restrict__ gates,
                                    const float* __restrict__ cst, const float* __restrict__ whh,
                                    const int64_t* __restrict__ ids, float* __restrict__ dgates, int B, int S, int H) {
  extern __shared__ float sdg[];   // [LR][4H]
  const int nrb = (B + LR - 1) / LR;
  const int dir = blockIdx.x / nrb, b0 = (blockIdx.x % nrb) * LR;
  const int j = threadIdx.x;
  const int G4 = 4 * H;
  const float* W = whh + (size_t)dir * G4 * H;   // [4H][H]
  float dc[LR], dhc[LR];
#pragma unroll
  for (int r = 0; r < LR; ++r) dc[r] = dhc[r] = 0.f;
  for (int step = 0; step < S; ++step) {
    const int t = dir == 0 ? S - 1 - step : step;
    const int tp = dir == 0 ? t - 1 : t + 1;
    bool valid[LR];
    float dh[LR];
#pragma unroll
    for (int r = 0; r < LR; ++r) {
      const int b = b0 + r;
      valid[r] = false;
      dh[r] = 0.f;
      float dg4[4] = {0.f, 0.f, 0.f, 0.f};
      if (b < B) {
        valid[r] = ids[(size_t)b * S + t] > 0;
        dh[r] = dhout[((size_t)b * S + t) * 2 * H + dir * H + j] + dhc[r];
        if (valid[r]) {
          const size_t gb = (((size_t)b * S + t) * 2 + dir) * G4;
          const float ig = gates[gb + j], fg = gates[gb + H + j], gg = gates[gb + 2 * H + j], og = gates[gb + 3 * H + j];
          const float cc = cst[(((size_t)b * S + t) * 2 + dir) * H + j];
          const float cp = (tp >= 0 && tp < S) ? cst[(((size_t)b * S + tp) * 2 + dir) * H + j] : 0.f;
          const float tc = tanhf(cc);
          const float dcn = dc[r] + dh[r] * og * (1.f - tc * tc);
          dg4[3] = dh[r] * tc * og * (1.f - og);
          dg4[0] = dcn * gg * ig * (1.f - ig);
          dg4[2] = dcn * ig * (1.f - gg * gg);
          dg4[1] = dcn * cp * fg * (1.f - fg);
          dc[r] = dcn * fg;
        }
        const size_t gb = (((size_t)b * S + t) * 2 + dir) * G4;
#pragma unroll
        for (int g = 0; g < 4; ++g) dgates[gb + g * H + j] = dg4[g];
      }
#pragma unroll
      for (int g = 0; g < 4; ++g) sdg[r * G4 + g * H + j] = dg4[g];
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < LR; ++r) {
      if (valid[r]) {
        float s = 0.f;
        for (int q = 0; q < G4; ++q) s += sdg[r * G4 + q] * W[(size_t)q * H + j];
        dhc[r] = s;
      } else {
        dhc[r] = dh[r];
      }
    }
    __syncthreads();
  }
}

std::vector<at::Tensor> lstm_seq_fwd(const at::Tensor& gx, const at::Tensor& whh, const at::Tensor& ids) {
  PCMP_CHECK_F32(gx); PCMP_CHECK_CONTIG(gx); PCMP_CHECK_F32(whh); PCMP_CHECK_CONTIG(whh);
  const int B = gx.size(0), S = gx.size(1), H = whh.size(2);
  TORCH_CHECK(H >= 1 && H <= 1024 && gx.size(2) == 2 && gx.size(3) == 4 * H, "lstm_seq_fwd (fp32): shapes, H <= 1024");
  auto idc = ids.contiguous();
  auto hout = at::empty({B, S, 2 * H}, whh.options());
  auto gates = at::empty({B, S, 2, 4 * H}, gx.options());
  auto cst = at::empty({B, S, 2, H}, gx.options());
  auto sync = at::zeros({4}, gx.options().dtype(at::kInt));
  if (B == 0 || S == 0) return {hout, gates, cst, sync};
  auto wt = at::empty({2, H, 4 * H}, whh.options());
  auto st = cur_stream();
  hipLaunchKernelGGL(lstm_transpose_f32_kernel, dim3(tgrid(wt.numel())), dim3(256), 0, st, ptr<float>(whh),
                     ptr<float>(wt), 4 * H, H);
  PCMP_LAUNCH_CHECK();
  PCMP_ALLOW_BIG_LDS(lstm_fwd_f32_kernel);
  hipLaunchKernelGGL(lstm_fwd_f32_kernel, dim3(2 * ceil_div(B, LR)), dim3(H), (size_t)LR * H * sizeof(float), st,
                     ptr<float>(gx), ptr<float>(wt), idc.data_ptr<int64_t>(), ptr<float>(hout), ptr<float>(gates),
                     ptr<float>(cst), B, S, H);
  PCMP_LAUNCH_CHECK();
  return {hout, gates, cst, sync};
}

std::vector<at::Tensor> lstm_seq_bwd(const at::Tensor& dhout, const at::Tensor& gates, const at::Tensor& cst,
                                     const at::Tensor& whh, const at::Tensor& ids) {
  PCMP_CHECK_F32(gates); PCMP_CHECK_F32(cst); PCMP_CHECK_F32(whh); PCMP_CHECK_CONTIG(whh);
  const int B = gates.size(0), S = gates.size(1), H = whh.size(2);
  TORCH_CHECK(H >= 1 && H <= 1024, "lstm_seq_bwd (fp32): H <= 1024");
  auto idc = ids.contiguous();
  auto dh = dhout.contiguous();
  PCMP_CHECK_F32(dh);
  auto gc = gates.contiguous(), cc = cst.contiguous();
  auto dgates = at::empty({B, S, 2, 4 * H}, whh.options());
  auto sync = at::zeros({4}, gates.options().dtype(at::kInt));
  if (B == 0 || S == 0) return {dgates, sync};
  TORCH_CHECK((size_t)LR * 4 * H * sizeof(float) <= 64 * 1024, "lstm_seq_bwd (fp32): LDS");
  PCMP_ALLOW_BIG_LDS(lstm_bwd_f32_kernel);
  hipLaunchKernelGGL(lstm_bwd_f32_kernel, dim3(2 * ceil_div(B, LR)), dim3(H), (size_t)LR * 4 * H * sizeof(float),
                     cur_stream(), ptr<float>(dh), ptr<float>(gc), ptr<float>(cc), ptr<float>(whh),
                     idc.data_ptr<int64_t>(), ptr<float>(dgates), B, S, H);
  PCMP_LAUNCH_CHECK();
  return {dgates, sync};
}

// ------------------------------------------------------------------------------- Linear + GELU
// u = x w^T + bias (fp32 GEMM of f32.hip), y = gelu(u): returns [y, u]
std::vector<at::Tensor> linear_gelu_fwd(const at::Tensor& x, const at::Tensor& w, const c10::optional<at::Tensor>& bias) {
  TORCH_CHECK(x.dim() == 2 && w.dim() == 2 && x.size(1) == w.size(1), "linear_gelu_fwd: x [M, C], w [N, C]");
  const int64_t M = x.size(0), C = x.size(1), N = w.size(0);
  auto u = f32::conv_fwd(x.contiguous().view({M, 1, 1, C}), w.contiguous().view({N, 1, 1, C}), 1, 0, bias,
                         c10::nullopt, false, false)[0].view({M, N});
  return {act_fwd(u, 0), u};
}

// dx = (dy w) * gelu'(u)
at::Tensor linear_dgrad_gelu(const at::Tensor& dy, const at::Tensor& w, const at::Tensor& u) {
  TORCH_CHECK(dy.dim() == 2 && w.dim() == 2 && u.dim() == 2 && dy.size(1) == w.size(0) && u.size(1) == w.size(1),
              "linear_dgrad_gelu: dy [M, N], w [N, C], u [M, C]");
  const int64_t M = dy.size(0), N = w.size(0), C = w.size(1);
  auto g = f32::conv_dgrad(dy.contiguous().view({M, 1, 1, N}), w.contiguous().view({N, 1, 1, C}), 1, 1, 1, 0,
                           c10::nullopt).view({M, C});
  return act_bwd(g, u, 0);
}

}  // namespace f32
}  // namespace pcmp

// BERT-base kernels: LayerNorm (+fused residual add), GELU(erf), tanh, bf16 add, and a fused
// multi-head attention forward/backward for short sequences (S <= 128, head dim 64).
//
// Reference parity: BertForSequenceClassification("bert-base-uncased") of
// pytorch_on_language_distr.py:151-161 — 12 layers, hidden 768, 12 heads, FFN 3072 GELU(erf),
// LayerNorm eps 1e-12, dropout 0.1 on embeddings / attention probs / hidden states,
// additive attention mask from ``attention_mask``.
//
// Attention (S=128, d=64): one workgroup per (batch, head); Q/K/V of the head are staged in LDS
// straight from the fused QKV projection output [B*S, 3*768] (no head-split transposes), the
// 128x128 score tile never leaves the CU.  Forward: each of the 4 waves owns 32 query rows:
// S = Q K^T on MFMA, row softmax (masked, scaled) reduced across the 16-lane column groups,
// log-sum-exp saved, hash-RNG dropout, P V on MFMA, output written head-interleaved [B*S, 768].
// Backward (FlashAttention-2 style, key-parallel): each wave owns 32 keys, recomputes P^T from
// Q, K and the saved LSE, computes dV += Pd^T dO, dP^T = V dO^T, dS^T = P^T (dP^T - D) and
// dK = dS^T Q on MFMA; dQ = dS K is taken after the waves exchange dS^T through LDS.
#include "common.h"
#include "f32.h"

namespace pcmp {

__device__ __forceinline__ void ldv8(const __bf16* p, float* v) {
  const u16x8 u = *reinterpret_cast<const u16x8*>(p);
#pragma unroll
  for (int e = 0; e < 8; ++e) v[e] = bf2f(u[e]);
}
__device__ __forceinline__ void stv8(__bf16* p, const float* v) {
  u16x8 u;
#pragma unroll
  for (int e = 0; e < 8; ++e) u[e] = f2bf(v[e]);
  *reinterpret_cast<u16x8*>(p) = u;
}
static Knob kn_ln_blocks("ln_blocks", 256);
static Knob kn_ln_rpb("ln_rpb", 8);
static int egrid(int64_t n) { return (int)std::max<int64_t>(1, std::min<int64_t>(4096, (n + 255) / 256)); }

// ------------------------------------------------------------------------------- LayerNorm
// one wave per row; y = LN(drop(x) [+ r]) * g + b ; saves xs = drop(x) + r (when r given or p > 0),
// mean, rstd.  drop: the dropout of the sublayer output (hidden_dropout_prob) with the mask of
// dropout_kernel on x's flat index, so BERT's dropout -> residual add -> LayerNorm is one pass.
__global__ void layernorm_fwd_kernel(const __bf16* __restrict__ x, const __bf16* __restrict__ r,
                                     const float* __restrict__ g, const float* __restrict__ b, __bf16* __restrict__ y,
                                     __bf16* __restrict__ xs, float* __restrict__ mean_out,
                                     float* __restrict__ rstd_out, int M, int D, float eps, float p,
                                     uint64_t seed0, uint64_t off, const int64_t* __restrict__ salt,
                                     int rper = 0, const __bf16* __restrict__ r2 = nullptr) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const int rrow = rper ? row % rper : row;
  if (row >= M) return;
  const int DV = D / 8;
  constexpr int MAXV = 4;  // D <= 64*8*4 = 2048
  float v[MAXV][8];
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < MAXV; ++k) {
    const int cv = lane + 64 * k;
    if (cv < DV) {
      ldv8(x + (size_t)row * D + cv * 8, v[k]);
      if (p > 0.f) {
        const uint64_t seed = dropout_seed(seed0, salt);
        const float scale = 1.f / (1.f - p);
        const uint64_t i0 = off + (uint64_t)row * D + cv * 8;
#pragma unroll
        for (int e = 0; e < 8; ++e) v[k][e] = uniform01(seed, i0 + e) >= p ? v[k][e] * scale : 0.f;
      }
      if (xs) {
        float w[8], w2[8];
        if (r) ldv8(r + (size_t)rrow * D + cv * 8, w);
        if (r2) ldv8(r2 + cv * 8, w2);
#pragma unroll
        for (int e = 0; e < 8; ++e) {   // (x + r) + r2: the lane-dense kernel's order
          v[k][e] += r ? w[e] : 0.f;
          if (r2) v[k][e] += w2[e];
        }
        // keep the bf16-rounded sum so backward sees exactly the normalised values
        u16x8 u;
#pragma unroll
        for (int e = 0; e < 8; ++e) { u[e] = f2bf(v[k][e]); v[k][e] = bf2f(u[e]); }
        if (xs) *reinterpret_cast<u16x8*>(xs + (size_t)row * D + cv * 8) = u;
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) s += v[k][e];
    }
  }
  const float mu = warp_sum(s) / D;
  float q = 0.f;
#pragma unroll
  for (int k = 0; k < MAXV; ++k)
    if (lane + 64 * k < DV)
#pragma unroll
      for (int e = 0; e < 8; ++e) { const float d = v[k][e] - mu; q += d * d; }
  const float rs = rsqrtf(warp_sum(q) / D + eps);
#pragma unroll
  for (int k = 0; k < MAXV; ++k) {
    const int cv = lane + 64 * k;
    if (cv < DV) {
      float o[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = (v[k][e] - mu) * rs * g[cv * 8 + e] + b[cv * 8 + e];
      stv8(y + (size_t)row * D + cv * 8, o);
    }
  }
  if (lane == 0) { mean_out[row] = mu; rstd_out[row] = rs; }
}


// LayerNorm forward for D = 256*KC (BERT: 768), the layout of ln_bwd_fused_kernel: lane owns
// columns 256k + 4*lane (8-byte loads / stores, every lane busy), gamma / beta as float4, one row per
// wave, 4 rows per block.  Same math and outputs as layernorm_fwd_kernel.
template <int KC>
__global__ void __launch_bounds__(256) ln_fwd_kernel(const __bf16* __restrict__ x, const __bf16* __restrict__ r,
                                                     const float* __restrict__ g, const float* __restrict__ b,
                                                     __bf16* __restrict__ y, __bf16* __restrict__ xs,
                                                     float* __restrict__ mean_out, float* __restrict__ rstd_out, int M,
                                                     float eps, float p, uint64_t seed0, uint64_t off,
                                                     const int64_t* __restrict__ salt, int rper = 0,
                                                     const __bf16* __restrict__ r2 = nullptr) {
  constexpr int D = 256 * KC;
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= M) return;
  // rper > 0: r has rper rows, row i adds r[i % rper] (BERT's position rows broadcast over the
  // batch); r2: one more [D] row added to every row (the token-type row)
  const int rrow = rper ? row % rper : row;
  float v[KC][4];
  uint2 xv[KC], rv[KC], r2v[KC];
#pragma unroll
  for (int k = 0; k < KC; ++k) {
    const size_t o = (size_t)row * D + 256 * k + 4 * lane;
    xv[k] = *reinterpret_cast<const uint2*>(x + o);
    if (r) rv[k] = *reinterpret_cast<const uint2*>(r + (size_t)rrow * D + 256 * k + 4 * lane);
    if (r2) r2v[k] = *reinterpret_cast<const uint2*>(r2 + 256 * k + 4 * lane);
  }
  const bool drop = p > 0.f;
  const uint64_t seed = drop ? dropout_seed(seed0, salt) : 0;
  const float scale = drop ? 1.f / (1.f - p) : 1.f;
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < KC; ++k) {
    v[k][0] = __uint_as_float(xv[k].x << 16); v[k][1] = __uint_as_float(xv[k].x & 0xffff0000u);
    v[k][2] = __uint_as_float(xv[k].y << 16); v[k][3] = __uint_as_float(xv[k].y & 0xffff0000u);
    if (drop) {
      const uint64_t i0 = off + (uint64_t)row * D + 256 * k + 4 * lane;
#pragma unroll
      for (int e = 0; e < 4; ++e) v[k][e] = uniform01(seed, i0 + e) >= p ? v[k][e] * scale : 0.f;
    }
    if (xs) {
      if (r) {
        v[k][0] += __uint_as_float(rv[k].x << 16); v[k][1] += __uint_as_float(rv[k].x & 0xffff0000u);
        v[k][2] += __uint_as_float(rv[k].y << 16); v[k][3] += __uint_as_float(rv[k].y & 0xffff0000u);
      }
      if (r2) {
        v[k][0] += __uint_as_float(r2v[k].x << 16); v[k][1] += __uint_as_float(r2v[k].x & 0xffff0000u);
        v[k][2] += __uint_as_float(r2v[k].y << 16); v[k][3] += __uint_as_float(r2v[k].y & 0xffff0000u);
      }
      // keep the bf16-rounded sum so backward sees exactly the normalised values
      const uint2 u = uint2{f2bf2(v[k][0], v[k][1]), f2bf2(v[k][2], v[k][3])};
      *reinterpret_cast<uint2*>(xs + (size_t)row * D + 256 * k + 4 * lane) = u;
      v[k][0] = __uint_as_float(u.x << 16); v[k][1] = __uint_as_float(u.x & 0xffff0000u);
      v[k][2] = __uint_as_float(u.y << 16); v[k][3] = __uint_as_float(u.y & 0xffff0000u);
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) s += v[k][e];
  }
  const float mu = warp_sum(s) * (1.f / D);
  float q = 0.f;
#pragma unroll
  for (int k = 0; k < KC; ++k)
#pragma unroll
    for (int e = 0; e < 4; ++e) { const float d = v[k][e] - mu; q += d * d; }
  const float rs = rsqrtf(warp_sum(q) * (1.f / D) + eps);
#pragma unroll
  for (int k = 0; k < KC; ++k) {
    const f32x4 g4 = *reinterpret_cast<const f32x4*>(g + 256 * k + 4 * lane);
    const f32x4 b4 = *reinterpret_cast<const f32x4*>(b + 256 * k + 4 * lane);
    float o[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) o[e] = (v[k][e] - mu) * rs * g4[e] + b4[e];
    *reinterpret_cast<uint2*>(y + (size_t)row * D + 256 * k + 4 * lane) = uint2{f2bf2(o[0], o[1]), f2bf2(o[2], o[3])};
  }
  if (lane == 0) { mean_out[row] = mu; rstd_out[row] = rs; }
}

// dx = rstd * (gy - mean(gy) - xhat * mean(gy * xhat)), gy = dy * gamma; per-block partial
// dgamma/dbeta into part[blockIdx][2][D]
__global__ void layernorm_bwd_kernel(const __bf16* __restrict__ dy, const __bf16* __restrict__ xs,
                                     const float* __restrict__ mean, const float* __restrict__ rstd,
                                     const float* __restrict__ g, __bf16* __restrict__ dx, float* __restrict__ part,
                                     int M, int D, int rows_per_block) {
  extern __shared__ float sh[];  // [4 waves][2][D]
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int DV = D / 8;
  constexpr int MAXV = 4;
  float dg[MAXV][8], db[MAXV][8];
#pragma unroll
  for (int k = 0; k < MAXV; ++k)
#pragma unroll
    for (int e = 0; e < 8; ++e) { dg[k][e] = 0.f; db[k][e] = 0.f; }
  const int r0 = blockIdx.x * rows_per_block, r1 = min(M, r0 + rows_per_block);
  for (int row = r0 + wid; row < r1; row += 4) {
    const float mu = mean[row], rs = rstd[row];
    float gy[MAXV][8], xh[MAXV][8];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int k = 0; k < MAXV; ++k) {
      const int cv = lane + 64 * k;
      if (cv < DV) {
        float dv[8], xv[8];
        ldv8(dy + (size_t)row * D + cv * 8, dv);
        ldv8(xs + (size_t)row * D + cv * 8, xv);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          xh[k][e] = (xv[e] - mu) * rs;
          gy[k][e] = dv[e] * g[cv * 8 + e];
          s1 += gy[k][e];
          s2 += gy[k][e] * xh[k][e];
          dg[k][e] += dv[e] * xh[k][e];
          db[k][e] += dv[e];
        }
      }
    }
    s1 = warp_sum(s1) / D;
    s2 = warp_sum(s2) / D;
#pragma unroll
    for (int k = 0; k < MAXV; ++k) {
      const int cv = lane + 64 * k;
      if (cv < DV) {
        float o[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] = rs * (gy[k][e] - s1 - xh[k][e] * s2);
        stv8(dx + (size_t)row * D + cv * 8, o);
      }
    }
  }
#pragma unroll
  for (int k = 0; k < MAXV; ++k) {
    const int cv = lane + 64 * k;
    if (cv < DV)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        sh[(wid * 2 + 0) * D + cv * 8 + e] = dg[k][e];
        sh[(wid * 2 + 1) * D + cv * 8 + e] = db[k][e];
      }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 2 * D; i += blockDim.x) {
    const int which = i / D, c = i % D;
    float s = 0.f;
    for (int w = 0; w < 4; ++w) s += sh[(w * 2 + which) * D + c];
    part[(size_t)blockIdx.x * 2 * D + i] = s;
  }
}


// Fused LayerNorm backward for D = 256*KC (BERT: 768): lane owns columns 256k + 4*lane (8-byte
// loads, every lane busy -- the one-vector-per-lane layout above idles half the lanes at D = 768),
// gamma in registers, 8 rows per block (2 per wave) so a CU holds 8+ waves of independent rows.
// Besides dx (the gradient of the LayerNorm input x + r, which is also the residual's gradient) it
// emits the gradient of the dropped branch, dxd = dx * keep / (1 - p) (the mask of the forward's
// fused dropout regenerated from the same counter), and per-block partial column sums
// part[blk][np][D] of (dy * xhat, dy, dxd): dgamma, dbeta and -- np = 3 -- the bias gradient of
// the Linear whose output was dropped (BERT's attention-output / FFN-down projections), so the
// backward of dropout + bias + residual + LayerNorm is this kernel and one column reduction.
template <int KC>
__global__ void __launch_bounds__(256) ln_bwd_fused_kernel(
    const __bf16* __restrict__ dy, const __bf16* __restrict__ xs, const float* __restrict__ mean,
    const float* __restrict__ rstd, const float* __restrict__ g, __bf16* __restrict__ dx, __bf16* __restrict__ dxd,
    float* __restrict__ part, int M, int rows_per_block, int np, float p, uint64_t seed0, uint64_t off,
    const int64_t* __restrict__ salt) {
  constexpr int D = 256 * KC;
  __shared__ f32x4 red[4][3][D / 4];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  float gg[KC][4], adg[KC][4], adb[KC][4], abi[KC][4];
#pragma unroll
  for (int k = 0; k < KC; ++k) {
    const f32x4 t = *reinterpret_cast<const f32x4*>(g + 256 * k + 4 * lane);
#pragma unroll
    for (int e = 0; e < 4; ++e) { gg[k][e] = t[e]; adg[k][e] = 0.f; adb[k][e] = 0.f; abi[k][e] = 0.f; }
  }
  const bool drop = p > 0.f;
  const uint64_t seed = drop ? dropout_seed(seed0, salt) : 0;
  const float scale = drop ? 1.f / (1.f - p) : 1.f;
  const int r0 = blockIdx.x * rows_per_block, r1 = min(M, r0 + rows_per_block);
  for (int row = r0 + wid; row < r1; row += 4) {
    uint2 dv[KC], xv[KC];
#pragma unroll
    for (int k = 0; k < KC; ++k) {
      const size_t o = (size_t)row * D + 256 * k + 4 * lane;
      dv[k] = *reinterpret_cast<const uint2*>(dy + o);
      xv[k] = *reinterpret_cast<const uint2*>(xs + o);
    }
    const float mu = mean[row], rs = rstd[row];
    float gy[KC][4], xh[KC][4];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int k = 0; k < KC; ++k) {
      const float d4[4] = {__uint_as_float(dv[k].x << 16), __uint_as_float(dv[k].x & 0xffff0000u),
                           __uint_as_float(dv[k].y << 16), __uint_as_float(dv[k].y & 0xffff0000u)};
      const float x4[4] = {__uint_as_float(xv[k].x << 16), __uint_as_float(xv[k].x & 0xffff0000u),
                           __uint_as_float(xv[k].y << 16), __uint_as_float(xv[k].y & 0xffff0000u)};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        xh[k][e] = (x4[e] - mu) * rs;
        gy[k][e] = d4[e] * gg[k][e];
        s1 += gy[k][e];
        s2 += gy[k][e] * xh[k][e];
        adg[k][e] += d4[e] * xh[k][e];
        adb[k][e] += d4[e];
      }
    }
    s1 = warp_sum(s1) * (1.f / D);
    s2 = warp_sum(s2) * (1.f / D);
#pragma unroll
    for (int k = 0; k < KC; ++k) {
      const size_t o = (size_t)row * D + 256 * k + 4 * lane;
      float v[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = rs * (gy[k][e] - s1 - xh[k][e] * s2);
      const uint2 ov = uint2{f2bf2(v[0], v[1]), f2bf2(v[2], v[3])};
      *reinterpret_cast<uint2*>(dx + o) = ov;
      // branch gradient from the bf16 dx (what a separate dropout kernel would read)
      float b4[4] = {__uint_as_float(ov.x << 16), __uint_as_float(ov.x & 0xffff0000u),
                     __uint_as_float(ov.y << 16), __uint_as_float(ov.y & 0xffff0000u)};
      if (drop) {
        const uint64_t i0 = off + (uint64_t)o;
#pragma unroll
        for (int e = 0; e < 4; ++e) b4[e] = uniform01(seed, i0 + e) >= p ? b4[e] * scale : 0.f;
        const uint2 bv = uint2{f2bf2(b4[0], b4[1]), f2bf2(b4[2], b4[3])};
        if (dxd) *reinterpret_cast<uint2*>(dxd + o) = bv;
        b4[0] = __uint_as_float(bv.x << 16); b4[1] = __uint_as_float(bv.x & 0xffff0000u);
        b4[2] = __uint_as_float(bv.y << 16); b4[3] = __uint_as_float(bv.y & 0xffff0000u);
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) abi[k][e] += b4[e];
    }
  }
#pragma unroll
  for (int k = 0; k < KC; ++k) {
    red[wid][0][64 * k + lane] = f32x4{adg[k][0], adg[k][1], adg[k][2], adg[k][3]};
    red[wid][1][64 * k + lane] = f32x4{adb[k][0], adb[k][1], adb[k][2], adb[k][3]};
    if (np > 2) red[wid][2][64 * k + lane] = f32x4{abi[k][0], abi[k][1], abi[k][2], abi[k][3]};
  }
  __syncthreads();
  for (int i = threadIdx.x; i < np * (D / 4); i += blockDim.x) {
    const int which = i / (D / 4), c = i - which * (D / 4);
    const f32x4 t = (red[0][which][c] + red[1][which][c]) + (red[2][which][c] + red[3][which][c]);
    reinterpret_cast<f32x4*>(part + ((size_t)blockIdx.x * np + which) * D)[c] = t;
  }
}

// out_w[d] (+)= sum_t part[t][w][d] for w < np (outputs o0, o1, o2; null skips; bit w of accmask
// accumulates).  Block = 16 column quads x 16 row groups: ~T/16 rows per thread, deterministic.
__global__ void __launch_bounds__(256) col_reduce3_kernel(const float* __restrict__ part, int T, int np, int D,
                                                          float* __restrict__ o0, float* __restrict__ o1,
                                                          float* __restrict__ o2, int accmask) {
  __shared__ f32x4 sh[16][17];
  const int L4 = np * D / 4;
  const int cq = threadIdx.x & 15, rg = threadIdx.x >> 4;
  const int q = blockIdx.x * 16 + cq;
  f32x4 s = {0.f, 0.f, 0.f, 0.f};
  if (q < L4) {
    const f32x4* p4 = reinterpret_cast<const f32x4*>(part);
    int t = rg;
    for (; t + 48 < T; t += 64) {
      const f32x4 a = p4[(size_t)t * L4 + q], b = p4[(size_t)(t + 16) * L4 + q];
      const f32x4 c = p4[(size_t)(t + 32) * L4 + q], d = p4[(size_t)(t + 48) * L4 + q];
      s += (a + b) + (c + d);
    }
    for (; t < T; t += 16) s += p4[(size_t)t * L4 + q];
  }
  sh[rg][cq] = s;
  __syncthreads();
  if (rg == 0 && q < L4) {
#pragma unroll
    for (int r = 1; r < 16; ++r) s += sh[r][cq];
    const int which = q / (D / 4), c = q - which * (D / 4);
    float* o = which == 0 ? o0 : (which == 1 ? o1 : o2);
    if (o) {
      f32x4* o4 = reinterpret_cast<f32x4*>(o) + c;
      if ((accmask >> which) & 1) s += *o4;
      *o4 = s;
    }
  }
}
// ------------------------------------------------------------------------------- activations
// gelu_erf / dgelu_erf: common.h

// mode 0: gelu, 1: tanh ; y = f(x)
__global__ void act_fwd_kernel(const __bf16* __restrict__ x, __bf16* __restrict__ y, int64_t nv, int mode) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nv; i += (int64_t)gridDim.x * blockDim.x) {
    float v[8];
    ldv8(x + i * 8, v);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = mode == 0 ? gelu_fast(v[e]) : tanhf(v[e]);
    stv8(y + i * 8, v);
  }
}
// gelu: dx = dy * gelu'(x) (x = pre-activation) ; tanh: dx = dy * (1 - y^2) (y = output)
__global__ void act_bwd_kernel(const __bf16* __restrict__ dy, const __bf16* __restrict__ xy, __bf16* __restrict__ dx,
                               int64_t nv, int mode) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nv; i += (int64_t)gridDim.x * blockDim.x) {
    float g[8], v[8];
    ldv8(dy + i * 8, g);
    ldv8(xy + i * 8, v);
#pragma unroll
    for (int e = 0; e < 8; ++e) g[e] *= mode == 0 ? dgelu_fast(v[e]) : (1.f - v[e] * v[e]);
    stv8(dx + i * 8, g);
  }
}

__global__ void add_bf16_kernel(const __bf16* __restrict__ a, const __bf16* __restrict__ b, __bf16* __restrict__ y,
                                int64_t nv) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nv; i += (int64_t)gridDim.x * blockDim.x) {
    float u[8], v[8];
    ldv8(a + i * 8, u);
    ldv8(b + i * 8, v);
#pragma unroll
    for (int e = 0; e < 8; ++e) u[e] += v[e];
    stv8(y + i * 8, u);
  }
}

// ------------------------------------------------------------------------------- attention
constexpr int AD = 64;     // head dim
constexpr int AS = 128;    // max sequence (LDS budget)
constexpr int ASP = AS + 8;  // padded LDS row (bf16 elements) for [*][S] tiles
constexpr int ADP = AD + 8;  // padded LDS row for [*][d] tiles

struct AttnParams {
  const __bf16* qkv;     // [B*S][3*D]  (q | k | v, head h at cols h*64)
  const int64_t* ids;    // [B][S] key mask = ids > 0 (nullptr: no mask)
  __bf16* out;           // fwd: ctx [B*S][D]
  float* lse;            // [B*H][S]
  const __bf16* dout;    // bwd: dctx [B*S][D]
  const __bf16* o;       // bwd: ctx
  __bf16* dqkv;          // bwd: [B*S][3*D]
  int B, S, H, D;
  float scale, p_drop;
  uint64_t seed, offset;
  const int64_t* salt;   // optional per-replay RNG salt (hipGraph-captured steps), see dropout_seed()
};

// bf16 fragment (8 consecutive k) from an LDS row-major tile: X[row][k0..k0+7]
__device__ __forceinline__ bf16x8 frag_row(const __bf16* X, int ld, int row, int k0) {
  return *reinterpret_cast<const bf16x8*>(X + row * ld + k0);
}

// bf16 fragment of X^T for an LDS tile stored row-major X[k][m] (ld elements per row): M/N index
// mbase + (lane & 15), reduction indices k0 + 8*(lane >> 4) .. +7 (k0 a multiple of 32), read with
// two ds_read_b64_tr_b16 (each lane addresses 4 consecutive m of one k row; the 16-lane groups
// transpose) -- no transposed copy of the tile and no per-element LDS gathers.
__device__ __forceinline__ bf16x8 frag_tr(const __bf16* X, int ld, int k0, int mbase) {
  typedef short s16x4 __attribute__((ext_vector_type(4)));
  typedef __attribute__((address_space(3))) s16x4 lds_s16x4_t;
  const int lane = threadIdx.x & 63;
  const int row = k0 + 8 * (lane >> 4) + ((lane >> 2) & 3), col = mbase + (lane & 3) * 4;
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t*)(X + row * ld + col));
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t*)(X + (row + 4) * ld + col));
  return __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
}

__device__ __forceinline__ float drop_scale(const AttnParams& p, int bh, int q, int k) {
  if (p.p_drop <= 0.f) return 1.f;
  const uint64_t idx = ((uint64_t)bh * p.S + q) * p.S + k;
  return uniform01(dropout_seed(p.seed, p.salt), p.offset + idx) >= p.p_drop ? 1.f / (1.f - p.p_drop) : 0.f;
}



// Forward, register-resident design (default): block = 4 waves x 16 queries of one (batch, head),
// grid = B*H*ceil(S/64) (768 workgroups at B=32, S=128: 3 per CU instead of 1.5).  Each wave
// computes S^T = K Q^T on MFMA with K and Q fragments loaded straight from the QKV projection
// output (16-byte row reads; no LDS), so the C layout leaves every lane with one query's scores
// for 4 keys per key tile: the softmax reduces in registers plus two cross-group shuffles, and P
// never leaves the registers -- O^T = V^T P^T takes P^T as the B operand in the same layout when
// the 32-key MFMA reduction runs over the permuted key order (32c + 4g + i, 32c + 16 + 4g + i),
// which the V^T A operand matches through ds_read_b64_tr_b16 reads of V staged row-major in LDS.
// O^T's C layout gives each lane 4 consecutive head dims of one query: 8-byte output stores.
__device__ __forceinline__ bf16x8 frag_tr_perm(const __bf16* X, int ld, int kbase, int mbase) {
  typedef short s16x4 __attribute__((ext_vector_type(4)));
  typedef __attribute__((address_space(3))) s16x4 lds_s16x4_t;
  const int lane = threadIdx.x & 63;
  const int row = kbase + 4 * (lane >> 4) + ((lane >> 2) & 3), col = mbase + (lane & 3) * 4;
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t*)(X + row * ld + col));
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t*)(X + (row + 16) * ld + col));
  return __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
}

template <int NT>   // key tiles of 16 (S = 16 * NT, NT even)
__global__ void __launch_bounds__(256) attention_fwd2_kernel(const AttnParams p) {
  constexpr int S = 16 * NT;
  constexpr int QB = (S + 63) / 64;
  __shared__ __attribute__((aligned(16))) __bf16 sV[S * ADP];
  __shared__ __attribute__((aligned(16))) float sMask[S];
  const int bh = blockIdx.x / QB, qb = blockIdx.x - bh * QB;
  const int b = bh / p.H, h = bh - b * p.H;
  const int D3 = 3 * p.D;
  const __bf16* base = p.qkv + (size_t)b * S * D3 + h * AD;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, fr = lane & 15, g = lane >> 4;
  const int q0 = qb * 64 + w * 16;
  const bool act = q0 < S;
  // S^T = K Q^T: A = K rows (keys), B = Q^T (lane: query q0 + fr, dims 8g..8g+7 of each 32-dim step)
  f32x4 st[NT];
#pragma unroll
  for (int j = 0; j < NT; ++j) st[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  if (act) {
    bf16x8 qf[2];
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) qf[kk] = *reinterpret_cast<const bf16x8*>(base + (size_t)(q0 + fr) * D3 + kk * 32 + 8 * g);
#pragma unroll
    for (int j = 0; j < NT; ++j)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        const bf16x8 kf = *reinterpret_cast<const bf16x8*>(base + p.D + (size_t)(16 * j + fr) * D3 + kk * 32 + 8 * g);
        st[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf, qf[kk], st[j], 0, 0, 0);
      }
  }
  for (int i = tid; i < S * (AD / 8); i += 256) {
    const int sr = i >> 3, c8 = i & 7;
    *reinterpret_cast<uint4*>(sV + sr * ADP + c8 * 8) =
        *reinterpret_cast<const uint4*>(base + 2 * p.D + (size_t)sr * D3 + c8 * 8);
  }
  for (int sr = tid; sr < S; sr += 256) sMask[sr] = (p.ids && p.ids[(size_t)b * S + sr] <= 0) ? -1e30f : 0.f;
  __syncthreads();
  if (!act) return;
  // softmax over keys for query q = q0 + fr; lane holds keys 16j + 4g + e
  const int q = q0 + fr;
  float mx = -INFINITY;
#pragma unroll
  for (int j = 0; j < NT; ++j) {
    const f32x4 mk = *reinterpret_cast<const f32x4*>(sMask + 16 * j + 4 * g);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float v = st[j][e] * p.scale + mk[e];
      st[j][e] = v;
      mx = fmaxf(mx, v);
    }
  }
  mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
  mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
  float sum = 0.f;
#pragma unroll
  for (int j = 0; j < NT; ++j)
#pragma unroll
    for (int e = 0; e < 4; ++e) { const float ev = __expf(st[j][e] - mx); st[j][e] = ev; sum += ev; }
  sum += __shfl_xor(sum, 16, 64);
  sum += __shfl_xor(sum, 32, 64);
  const float inv = 1.f / sum;
  if (g == 0) p.lse[(size_t)bh * S + q] = mx + __logf(sum);
  // P^T B operands per 32-key chunk c: slots i < 4 -> key 32c + 4g + i, i >= 4 -> 32c + 16 + 4g + i - 4
  bf16x8 pb[NT / 2];
#pragma unroll
  for (int c = 0; c < NT / 2; ++c) {
    unsigned pk[4];
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {
      const int j = 2 * c + hh;
      float v[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = st[j][e] * inv * drop_scale(p, bh, q, 16 * j + 4 * g + e);
      pk[2 * hh] = f2bf2(v[0], v[1]);
      pk[2 * hh + 1] = f2bf2(v[2], v[3]);
    }
    pb[c] = __builtin_bit_cast(bf16x8, uint4{pk[0], pk[1], pk[2], pk[3]});
  }
  // O^T[d][q] = V^T P^T over the permuted key order
  __bf16* orow = p.out + ((size_t)b * S + q) * p.D + h * AD;
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    f32x4 o = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int c = 0; c < NT / 2; ++c)
      o = __builtin_amdgcn_mfma_f32_16x16x32_bf16(frag_tr_perm(sV, ADP, 32 * c, 16 * t), pb[c], o, 0, 0, 0);
    *reinterpret_cast<uint2*>(orow + 16 * t + 4 * g) = uint2{f2bf2(o[0], o[1]), f2bf2(o[2], o[3])};
  }
}


// Backward, register-resident design (default): block = one (batch, head), one wave per 16-key
// tile (8 waves at S = 128).  Each wave computes S and dPd = dO V^T for its keys over all queries
// (C layout: lane = one key, 4 queries per query tile), so P, dS = P (dP - D) stay in registers and
// feed dV^T = dO^T Pd and dK^T = Q^T dS directly as B operands over the permuted query order (the
// forward's trick; dO^T / Q^T come from ds_read_b64_tr_b16 reads of dO / Q staged row-major).
// dS^T goes to LDS once (8-byte stores); after one barrier each wave takes dQ^T = K^T dS^T for 16
// queries with both operands from transpose reads.  dK, dV, dQ leave as 8-byte stores.
template <int NT>
__global__ void __launch_bounds__(512) attention_bwd2_kernel(const AttnParams p) {
  constexpr int S = 16 * NT;
  constexpr int TP = S + 8;   // dS^T row pitch (bf16)
  __shared__ __attribute__((aligned(16))) __bf16 sQ[S * ADP];
  __shared__ __attribute__((aligned(16))) __bf16 sK[S * ADP];
  __shared__ __attribute__((aligned(16))) __bf16 sdO[S * ADP];
  __shared__ __attribute__((aligned(16))) __bf16 sT[S * TP];
  __shared__ __attribute__((aligned(16))) float sL[S];
  __shared__ __attribute__((aligned(16))) float sDd[S];
  __shared__ float sMask[S];
  const int bh = blockIdx.x, b = bh / p.H, h = bh - (bh / p.H) * p.H;
  const int D3 = 3 * p.D;
  const __bf16* base = p.qkv + (size_t)b * S * D3 + h * AD;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, fr = lane & 15, g = lane >> 4;
  // stage Q, K, dO row-major; D[q] = rowsum(dO * O) over the 8 lanes that hold row q's chunks
  for (int i = tid; i < S * (AD / 8); i += NT * 64) {
    const int r = i >> 3, c8 = i & 7;
    const uint4 qv = *reinterpret_cast<const uint4*>(base + (size_t)r * D3 + c8 * 8);
    const uint4 kv = *reinterpret_cast<const uint4*>(base + p.D + (size_t)r * D3 + c8 * 8);
    const size_t orow = ((size_t)b * S + r) * p.D + h * AD + c8 * 8;
    const uint4 dv = *reinterpret_cast<const uint4*>(p.dout + orow);
    float a[8], c[8];
    ldv8(p.o + orow, a);
    *reinterpret_cast<uint4*>(sQ + r * ADP + c8 * 8) = qv;
    *reinterpret_cast<uint4*>(sK + r * ADP + c8 * 8) = kv;
    *reinterpret_cast<uint4*>(sdO + r * ADP + c8 * 8) = dv;
    const unsigned short* du = reinterpret_cast<const unsigned short*>(&dv);
    float dot = 0.f;
#pragma unroll
    for (int e = 0; e < 8; ++e) { c[e] = bf2f(du[e]); dot += a[e] * c[e]; }
    dot += __shfl_xor(dot, 1, 64);
    dot += __shfl_xor(dot, 2, 64);
    dot += __shfl_xor(dot, 4, 64);
    if (c8 == 0) sDd[r] = dot;
  }
  for (int r = tid; r < S; r += NT * 64) {
    sL[r] = p.lse[(size_t)bh * S + r];
    sMask[r] = (p.ids && p.ids[(size_t)b * S + r] <= 0) ? -1e30f : 0.f;
  }
  __syncthreads();
  const int key = 16 * w + fr;
  // S = Q K^T and dPd = dO V^T for this wave's keys: C[q][key], A = Q / dO rows, B = K / V rows
  f32x4 sc[NT], dp[NT];
  {
    bf16x8 kb[2], vb[2];
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      kb[kk] = frag_row(sK, ADP, key, kk * 32 + 8 * g);
      vb[kk] = *reinterpret_cast<const bf16x8*>(base + 2 * p.D + (size_t)key * D3 + kk * 32 + 8 * g);
    }
#pragma unroll
    for (int i = 0; i < NT; ++i) {
      sc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
      dp[i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        sc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(frag_row(sQ, ADP, 16 * i + fr, kk * 32 + 8 * g), kb[kk], sc[i], 0, 0, 0);
        dp[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(frag_row(sdO, ADP, 16 * i + fr, kk * 32 + 8 * g), vb[kk], dp[i], 0, 0, 0);
      }
    }
  }
  // P = exp(s * scale + mask - lse), Pd = P * drop, dS = P * (dPd * drop - D) * scale  (q = 16i + 4g + e)
  const float mk = sMask[key];
#pragma unroll
  for (int i = 0; i < NT; ++i) {
    const f32x4 l4 = *reinterpret_cast<const f32x4*>(sL + 16 * i + 4 * g);
    const f32x4 d4 = *reinterpret_cast<const f32x4*>(sDd + 16 * i + 4 * g);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int q = 16 * i + 4 * g + e;
      const float pr = __expf(sc[i][e] * p.scale + mk - l4[e]);
      const float dsc = drop_scale(p, bh, q, key);
      sc[i][e] = pr * dsc;                                      // Pd
      dp[i][e] = pr * (dp[i][e] * dsc - d4[e]) * p.scale;      // dS (scaled)
    }
  }
  // B operands over the permuted query order: slots i < 4 -> q = 32c + 4g + i, else 32c + 16 + 4g + i - 4
  auto pack = [&](const f32x4* v, int c) {
    return __builtin_bit_cast(bf16x8, uint4{f2bf2(v[2 * c][0], v[2 * c][1]), f2bf2(v[2 * c][2], v[2 * c][3]),
                                            f2bf2(v[2 * c + 1][0], v[2 * c + 1][1]),
                                            f2bf2(v[2 * c + 1][2], v[2 * c + 1][3])});
  };
  bf16x8 pbv[NT / 2], dsb[NT / 2];
#pragma unroll
  for (int c = 0; c < NT / 2; ++c) { pbv[c] = pack(sc, c); dsb[c] = pack(dp, c); }
  // dS^T -> LDS [key][q] (lane: row key, 4 consecutive queries per tile)
#pragma unroll
  for (int i = 0; i < NT; ++i)
    *reinterpret_cast<uint2*>(sT + key * TP + 16 * i + 4 * g) = uint2{f2bf2(dp[i][0], dp[i][1]), f2bf2(dp[i][2], dp[i][3])};
  // dV^T = dO^T Pd, dK^T = Q^T dS: C[d][key]; lane stores 4 consecutive d of its key
  __bf16* krow = p.dqkv + ((size_t)b * S + key) * D3 + p.D + h * AD;
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    f32x4 dv = f32x4{0.f, 0.f, 0.f, 0.f}, dk = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int c = 0; c < NT / 2; ++c) {
      dv = __builtin_amdgcn_mfma_f32_16x16x32_bf16(frag_tr_perm(sdO, ADP, 32 * c, 16 * t), pbv[c], dv, 0, 0, 0);
      dk = __builtin_amdgcn_mfma_f32_16x16x32_bf16(frag_tr_perm(sQ, ADP, 32 * c, 16 * t), dsb[c], dk, 0, 0, 0);
    }
    *reinterpret_cast<uint2*>(krow + 16 * t + 4 * g) = uint2{f2bf2(dk[0], dk[1]), f2bf2(dk[2], dk[3])};
    *reinterpret_cast<uint2*>(krow + p.D + 16 * t + 4 * g) = uint2{f2bf2(dv[0], dv[1]), f2bf2(dv[2], dv[3])};
  }
  __syncthreads();
  // dQ^T = K^T dS^T for queries 16w .. 16w+15: A = K^T (transpose reads of K), B = dS^T rows
  const int q = 16 * w + fr;
  __bf16* qrow = p.dqkv + ((size_t)b * S + q) * D3 + h * AD;
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    f32x4 dq = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int c = 0; c < NT / 2; ++c)
      dq = __builtin_amdgcn_mfma_f32_16x16x32_bf16(frag_tr(sK, ADP, 32 * c, 16 * t), frag_tr(sT, TP, 32 * c, 16 * w),
                                                   dq, 0, 0, 0);
    *reinterpret_cast<uint2*>(qrow + 16 * t + 4 * g) = uint2{f2bf2(dq[0], dq[1]), f2bf2(dq[2], dq[3])};
  }
}


// ------------------------------------------------------------------------------- host
std::vector<at::Tensor> layernorm_fwd(const at::Tensor& x, const c10::optional<at::Tensor>& r, const at::Tensor& g,
                                      const at::Tensor& b, double eps, double p, int64_t seed, int64_t offset,
                                      const c10::optional<at::Tensor>& salt) {
  if (x.scalar_type() == at::kFloat) return f32::layernorm_fwd(x, r, g, b, eps, p, seed, offset, salt);
  PCMP_CHECK_BF16(x); PCMP_CHECK_CONTIG(x); PCMP_CHECK_F32(g); PCMP_CHECK_F32(b);
  const int D = x.size(-1);
  const int M = x.numel() / D;
  TORCH_CHECK(D % 8 == 0 && D <= 2048, "layernorm: D % 8 and <= 2048");
  auto y = at::empty_like(x);
  const bool hr = r.has_value() && r->defined();
  TORCH_CHECK(p >= 0.0 && p < 1.0, "layernorm: dropout p in [0, 1)");
  at::Tensor xs = (hr || p > 0.0) ? at::empty_like(x) : x;
  auto f32 = x.options().dtype(at::kFloat);
  auto mean = at::empty({M}, f32), rstd = at::empty({M}, f32);
  if (D % 256 == 0 && D <= 1024) {   // lane-dense kernel; the generic one below for other widths
    const __bf16* rp = hr ? ptr<__bf16>(*r) : nullptr;
    __bf16* xsp = (hr || p > 0.0) ? ptr<__bf16>(xs) : nullptr;
    const int64_t* sp = p > 0.0 ? salt_ptr(salt) : nullptr;
#define PCMP_LNF(KC)                                                                                            \
  hipLaunchKernelGGL(ln_fwd_kernel<KC>, dim3(ceil_div(M, 4)), dim3(256), 0, cur_stream(), ptr<__bf16>(x), rp,   \
                     ptr<float>(g), ptr<float>(b), ptr<__bf16>(y), xsp, ptr<float>(mean), ptr<float>(rstd), M,  \
                     (float)eps, (float)p, (uint64_t)seed, (uint64_t)offset, sp)
    switch (D / 256) {
      case 1: PCMP_LNF(1); break;
      case 2: PCMP_LNF(2); break;
      case 3: PCMP_LNF(3); break;
      default: PCMP_LNF(4); break;
    }
#undef PCMP_LNF
    PCMP_LAUNCH_CHECK();
    return {y, xs, mean, rstd};
  }
  hipLaunchKernelGGL(layernorm_fwd_kernel, dim3(ceil_div(M, 4)), dim3(256), 0, cur_stream(), ptr<__bf16>(x),
                     hr ? ptr<__bf16>(*r) : nullptr, ptr<float>(g), ptr<float>(b), ptr<__bf16>(y),
                     (hr || p > 0.0) ? ptr<__bf16>(xs) : nullptr, ptr<float>(mean), ptr<float>(rstd), M, D, (float)eps,
                     (float)p, (uint64_t)seed, (uint64_t)offset, p > 0.0 ? salt_ptr(salt) : nullptr);
  PCMP_LAUNCH_CHECK();
  return {y, xs, mean, rstd};
}

// BERT embedding sum + LayerNorm in one pass: y = LN(x + pos[row % S] + tt) with x [M, D] (the
// gathered word rows), pos [S, D] (position rows, broadcast over the batch), tt [D] (token-type
// row); returns [y, xs, mean, rstd] like layernorm_fwd (xs = the bf16-rounded sum).
std::vector<at::Tensor> embed_layernorm_fwd(const at::Tensor& x, const at::Tensor& pos, const at::Tensor& tt,
                                            const at::Tensor& g, const at::Tensor& b, double eps) {
  if (x.scalar_type() == at::kFloat) return f32::embed_layernorm_fwd(x, pos, tt, g, b, eps);
  PCMP_CHECK_BF16(x); PCMP_CHECK_CONTIG(x); PCMP_CHECK_BF16(pos); PCMP_CHECK_CONTIG(pos);
  PCMP_CHECK_BF16(tt); PCMP_CHECK_CONTIG(tt); PCMP_CHECK_F32(g); PCMP_CHECK_F32(b);
  const int D = x.size(-1);
  const int M = x.numel() / D;
  TORCH_CHECK(D % 8 == 0 && D <= 2048, "embed_layernorm: D % 8 and <= 2048");
  TORCH_CHECK(pos.numel() % D == 0 && pos.numel() > 0, "embed_layernorm: pos must be [S, D]");
  const int S = pos.numel() / D;
  TORCH_CHECK(M % S == 0, "embed_layernorm: rows must be a multiple of S");
  TORCH_CHECK(tt.numel() == D && g.numel() == D && b.numel() == D, "embed_layernorm: tt / gamma / beta must be [D]");
  auto y = at::empty_like(x), xs = at::empty_like(x);
  auto f32 = x.options().dtype(at::kFloat);
  auto mean = at::empty({M}, f32), rstd = at::empty({M}, f32);
  if (D % 256 == 0 && D <= 1024) {
#define PCMP_ELNF(KC)                                                                                            \
  hipLaunchKernelGGL(ln_fwd_kernel<KC>, dim3(ceil_div(M, 4)), dim3(256), 0, cur_stream(), ptr<__bf16>(x),        \
                     ptr<__bf16>(pos), ptr<float>(g), ptr<float>(b), ptr<__bf16>(y), ptr<__bf16>(xs),           \
                     ptr<float>(mean), ptr<float>(rstd), M, (float)eps, 0.f, (uint64_t)0, (uint64_t)0, nullptr,  \
                     S, ptr<__bf16>(tt))
    switch (D / 256) {
      case 1: PCMP_ELNF(1); break;
      case 2: PCMP_ELNF(2); break;
      case 3: PCMP_ELNF(3); break;
      default: PCMP_ELNF(4); break;
    }
#undef PCMP_ELNF
  } else {
    hipLaunchKernelGGL(layernorm_fwd_kernel, dim3(ceil_div(M, 4)), dim3(256), 0, cur_stream(), ptr<__bf16>(x),
                       ptr<__bf16>(pos), ptr<float>(g), ptr<float>(b), ptr<__bf16>(y), ptr<__bf16>(xs),
                       ptr<float>(mean), ptr<float>(rstd), M, D, (float)eps, 0.f, (uint64_t)0, (uint64_t)0, nullptr, S,
                       ptr<__bf16>(tt));
  }
  PCMP_LAUNCH_CHECK();
  return {y, xs, mean, rstd};
}

// returns dx; dgamma/dbeta written (or accumulated) into the given fp32 tensors when defined
std::vector<at::Tensor> layernorm_bwd_fused(const at::Tensor& dy, const at::Tensor& xs, const at::Tensor& mean,
                                            const at::Tensor& rstd, const at::Tensor& g,
                                            const c10::optional<at::Tensor>& dg, const c10::optional<at::Tensor>& db,
                                            const c10::optional<at::Tensor>& dbias, int64_t accmask, double p,
                                            int64_t seed, int64_t offset, const c10::optional<at::Tensor>& salt);

at::Tensor layernorm_bwd(const at::Tensor& dy, const at::Tensor& xs, const at::Tensor& mean, const at::Tensor& rstd,
                         const at::Tensor& g, const c10::optional<at::Tensor>& dg, const c10::optional<at::Tensor>& db,
                         bool accumulate) {
  if (xs.scalar_type() == at::kFloat) return f32::layernorm_bwd(dy, xs, mean, rstd, g, dg, db, accumulate);
  const int D = xs.size(-1);
  if (D % 256 == 0 && D <= 1024)   // the lane-dense kernel (no dropout, no bias output)
    return layernorm_bwd_fused(dy, xs, mean, rstd, g, dg, db, c10::nullopt, accumulate ? 3 : 0, 0.0, 0, 0,
                               c10::nullopt)[0];
  auto dyc = dy.contiguous();
  const int M = xs.numel() / D;
  auto dx = at::empty_like(xs);
  const int target_blocks = std::max(1, kn_ln_blocks.get());   // knob ln_blocks (A/B runs)
  const int rpb = std::max(4, ceil_div(M, target_blocks));
  const int T = ceil_div(M, rpb);
  auto part = at::empty({T, 2, D}, mean.options());
  hipLaunchKernelGGL(layernorm_bwd_kernel, dim3(T), dim3(256), (size_t)8 * D * sizeof(float), cur_stream(),
                     ptr<__bf16>(dyc), ptr<__bf16>(xs), ptr<float>(mean), ptr<float>(rstd), ptr<float>(g),
                     ptr<__bf16>(dx), ptr<float>(part), M, D, rpb);
  PCMP_LAUNCH_CHECK();
  // dgamma / dbeta reduced straight into their (flat-gradient) destinations
  float* dgp = nullptr;
  float* dbp = nullptr;
  for (auto [t, d] : {std::make_pair(&dg, &dgp), std::make_pair(&db, &dbp)}) {
    if (t->has_value() && (*t)->defined()) {
      PCMP_CHECK_F32(**t); PCMP_CHECK_CONTIG(**t);
      TORCH_CHECK((*t)->numel() == D, "layernorm_bwd: dgamma/dbeta size");
      *d = ptr<float>(**t);
    }
  }
  if (dgp || dbp) launch_col_reduce(ptr<float>(part), T, 2 * D, dgp, accumulate, cur_stream(), dbp, D);
  return dx;
}


// Fused backward of drop(x) + r -> LayerNorm (see ln_bwd_fused_kernel): returns [dx, dxd] (dxd is
// dx itself when p == 0); dgamma / dbeta / dbias reduced into the given fp32 tensors, bit w of
// accmask accumulating into output w.  D must be a multiple of 256 (<= 1024).
std::vector<at::Tensor> layernorm_bwd_fused(const at::Tensor& dy, const at::Tensor& xs, const at::Tensor& mean,
                                            const at::Tensor& rstd, const at::Tensor& g,
                                            const c10::optional<at::Tensor>& dg, const c10::optional<at::Tensor>& db,
                                            const c10::optional<at::Tensor>& dbias, int64_t accmask, double p,
                                            int64_t seed, int64_t offset, const c10::optional<at::Tensor>& salt) {
  if (xs.scalar_type() == at::kFloat)
    return f32::layernorm_bwd_fused(dy, xs, mean, rstd, g, dg, db, dbias, accmask, p, seed, offset, salt);
  PCMP_CHECK_BF16(xs); PCMP_CHECK_CONTIG(xs); PCMP_CHECK_F32(g); PCMP_CHECK_F32(mean); PCMP_CHECK_F32(rstd);
  auto dyc = dy.contiguous();
  PCMP_CHECK_BF16(dyc);
  const int D = xs.size(-1);
  const int M = xs.numel() / D;
  TORCH_CHECK(dyc.numel() == xs.numel() && mean.numel() == M && rstd.numel() == M && g.numel() == D,
              "layernorm_bwd_fused: shapes");
  TORCH_CHECK(D % 256 == 0 && D <= 1024, "layernorm_bwd_fused: D must be a multiple of 256 (<= 1024)");
  TORCH_CHECK(p >= 0.0 && p < 1.0, "layernorm_bwd_fused: dropout p in [0, 1)");
  auto dx = at::empty_like(xs);
  at::Tensor dxd = p > 0.0 ? at::empty_like(xs) : dx;
  float* outs[3] = {nullptr, nullptr, nullptr};
  const c10::optional<at::Tensor>* ts[3] = {&dg, &db, &dbias};
  for (int w = 0; w < 3; ++w) {
    if (ts[w]->has_value() && (*ts[w])->defined()) {
      PCMP_CHECK_F32(**ts[w]); PCMP_CHECK_CONTIG(**ts[w]);
      TORCH_CHECK((*ts[w])->numel() == D, "layernorm_bwd_fused: gradient output size");
      outs[w] = ptr<float>(**ts[w]);
    }
  }
  const int np = outs[2] ? 3 : 2;
  const int rpb = std::max(4, kn_ln_rpb.get());   // knob ln_rpb: rows per block (A/B runs)
  const int T = ceil_div(M, rpb);
  auto part = at::empty({T, np, D}, mean.options());
  auto st = cur_stream();
  const float pf = (float)p;
  const int64_t* sp = p > 0.0 ? salt_ptr(salt) : nullptr;
#define PCMP_LNB(KC)                                                                                            \
  hipLaunchKernelGGL(ln_bwd_fused_kernel<KC>, dim3(T), dim3(256), 0, st, ptr<__bf16>(dyc), ptr<__bf16>(xs),    \
                     ptr<float>(mean), ptr<float>(rstd), ptr<float>(g), ptr<__bf16>(dx),                       \
                     p > 0.0 ? ptr<__bf16>(dxd) : nullptr, ptr<float>(part), M, rpb, np, pf, (uint64_t)seed,   \
                     (uint64_t)offset, sp)
  switch (D / 256) {
    case 1: PCMP_LNB(1); break;
    case 2: PCMP_LNB(2); break;
    case 3: PCMP_LNB(3); break;
    default: PCMP_LNB(4); break;
  }
#undef PCMP_LNB
  PCMP_LAUNCH_CHECK();
  if (outs[0] || outs[1] || outs[2]) {
    hipLaunchKernelGGL(col_reduce3_kernel, dim3(ceil_div(np * D / 4, 16)), dim3(256), 0, st, ptr<float>(part), T, np,
                       D, outs[0], outs[1], outs[2], (int)accmask);
    PCMP_LAUNCH_CHECK();
  }
  return {dx, dxd};
}

static at::Tensor act_fwd(const at::Tensor& x, int mode) {
  if (x.scalar_type() == at::kFloat) return f32::act_fwd(x, mode);
  PCMP_CHECK_BF16(x); PCMP_CHECK_CONTIG(x);
  TORCH_CHECK(x.numel() % 8 == 0, "activation numel % 8");
  auto y = at::empty_like(x);
  hipLaunchKernelGGL(act_fwd_kernel, dim3(egrid(x.numel() / 8)), dim3(256), 0, cur_stream(), ptr<__bf16>(x),
                     ptr<__bf16>(y), x.numel() / 8, mode);
  PCMP_LAUNCH_CHECK();
  return y;
}
static at::Tensor act_bwd(const at::Tensor& dy, const at::Tensor& xy, int mode) {
  if (xy.scalar_type() == at::kFloat) return f32::act_bwd(dy, xy, mode);
  auto dyc = dy.contiguous();
  auto dx = at::empty_like(xy);
  hipLaunchKernelGGL(act_bwd_kernel, dim3(egrid(xy.numel() / 8)), dim3(256), 0, cur_stream(), ptr<__bf16>(dyc),
                     ptr<__bf16>(xy), ptr<__bf16>(dx), xy.numel() / 8, mode);
  PCMP_LAUNCH_CHECK();
  return dx;
}
at::Tensor gelu_fwd(const at::Tensor& x) { return act_fwd(x, 0); }
at::Tensor gelu_bwd(const at::Tensor& dy, const at::Tensor& x) { return act_bwd(dy, x, 0); }
at::Tensor tanh_fwd(const at::Tensor& x) { return act_fwd(x, 1); }
at::Tensor tanh_bwd(const at::Tensor& dy, const at::Tensor& y) { return act_bwd(dy, y, 1); }

at::Tensor add_bf16(const at::Tensor& a, const at::Tensor& b) {
  if (a.scalar_type() == at::kFloat) return f32::add(a, b);
  PCMP_CHECK_BF16(a); PCMP_CHECK_BF16(b);
  auto ac = a.contiguous(), bc = b.contiguous();
  TORCH_CHECK(ac.numel() == bc.numel() && ac.numel() % 8 == 0, "add_bf16: shapes");
  auto y = at::empty_like(ac);
  hipLaunchKernelGGL(add_bf16_kernel, dim3(egrid(ac.numel() / 8)), dim3(256), 0, cur_stream(), ptr<__bf16>(ac),
                     ptr<__bf16>(bc), ptr<__bf16>(y), ac.numel() / 8);
  PCMP_LAUNCH_CHECK();
  return y;
}


// qkv [B*S][3D] bf16 -> [ctx [B*S][D] bf16, lse [B*H][S] f32]
std::vector<at::Tensor> attention_fwd(const at::Tensor& qkv, const c10::optional<at::Tensor>& ids, int64_t B,
                                      int64_t S, int64_t H, double p_drop, int64_t seed, int64_t offset,
                                      const c10::optional<at::Tensor>& salt) {
  if (qkv.scalar_type() == at::kFloat) return f32::attention_fwd(qkv, ids, B, S, H, p_drop, seed, offset, salt);
  PCMP_CHECK_BF16(qkv); PCMP_CHECK_CONTIG(qkv);
  const int D3 = qkv.size(-1), D = D3 / 3;
  TORCH_CHECK(D == H * AD, "attention: head dim must be 64");
  TORCH_CHECK(S % 32 == 0 && S <= AS, "attention: S must be a multiple of 32 and <= 128");
  TORCH_CHECK(qkv.numel() == B * S * D3, "attention: qkv shape");
  auto ctx = at::empty({B * S, D}, qkv.options());
  auto lse = at::empty({B * H, S}, qkv.options().dtype(at::kFloat));
  at::Tensor idc;
  if (ids.has_value() && ids->defined()) idc = ids->contiguous();
  AttnParams p{ptr<__bf16>(qkv), idc.defined() ? idc.data_ptr<int64_t>() : nullptr, ptr<__bf16>(ctx), ptr<float>(lse),
               nullptr, nullptr, nullptr, (int)B, (int)S, (int)H, D, 0.125f, (float)p_drop, (uint64_t)seed,
               (uint64_t)offset, salt_ptr(salt)};
  const int nt = (int)S / 16;
  const dim3 grid((unsigned)(B * H * ((S + 63) / 64)));
  switch (nt) {
    case 2: hipLaunchKernelGGL(attention_fwd2_kernel<2>, grid, dim3(256), 0, cur_stream(), p); break;
    case 4: hipLaunchKernelGGL(attention_fwd2_kernel<4>, grid, dim3(256), 0, cur_stream(), p); break;
    case 6: hipLaunchKernelGGL(attention_fwd2_kernel<6>, grid, dim3(256), 0, cur_stream(), p); break;
    default: hipLaunchKernelGGL(attention_fwd2_kernel<8>, grid, dim3(256), 0, cur_stream(), p); break;
  }
  PCMP_LAUNCH_CHECK();
  return {ctx, lse};
}

at::Tensor attention_bwd(const at::Tensor& dctx, const at::Tensor& qkv, const at::Tensor& ctx, const at::Tensor& lse,
                         const c10::optional<at::Tensor>& ids, int64_t B, int64_t S, int64_t H, double p_drop,
                         int64_t seed, int64_t offset, const c10::optional<at::Tensor>& salt) {
  if (qkv.scalar_type() == at::kFloat)
    return f32::attention_bwd(dctx, qkv, ctx, lse, ids, B, S, H, p_drop, seed, offset, salt);
  PCMP_CHECK_BF16(qkv); PCMP_CHECK_CONTIG(qkv); PCMP_CHECK_BF16(ctx); PCMP_CHECK_CONTIG(ctx); PCMP_CHECK_F32(lse);
  auto dc = dctx.contiguous();
  const int D3 = qkv.size(-1), D = D3 / 3;
  TORCH_CHECK(D == H * AD, "attention_bwd: head dim must be 64");
  TORCH_CHECK(S % 32 == 0 && S <= AS, "attention_bwd: S must be a multiple of 32 and <= 128");
  TORCH_CHECK(qkv.numel() == B * S * D3 && dc.numel() == B * S * D && ctx.numel() == B * S * D &&
              lse.numel() == B * H * S, "attention_bwd: shapes");
  auto dqkv = at::empty_like(qkv);
  at::Tensor idc;
  if (ids.has_value() && ids->defined()) idc = ids->contiguous();
  AttnParams p{ptr<__bf16>(qkv), idc.defined() ? idc.data_ptr<int64_t>() : nullptr, nullptr, ptr<float>(lse),
               ptr<__bf16>(dc), ptr<__bf16>(ctx), ptr<__bf16>(dqkv), (int)B, (int)S, (int)H, D, 0.125f,
               (float)p_drop, (uint64_t)seed, (uint64_t)offset, salt_ptr(salt)};
  switch ((int)S / 16) {
    case 2: hipLaunchKernelGGL(attention_bwd2_kernel<2>, dim3(B * H), dim3(128), 0, cur_stream(), p); break;
    case 4: hipLaunchKernelGGL(attention_bwd2_kernel<4>, dim3(B * H), dim3(256), 0, cur_stream(), p); break;
    case 6: hipLaunchKernelGGL(attention_bwd2_kernel<6>, dim3(B * H), dim3(384), 0, cur_stream(), p); break;
    default: hipLaunchKernelGGL(attention_bwd2_kernel<8>, dim3(B * H), dim3(512), 0, cur_stream(), p); break;
  }
  PCMP_LAUNCH_CHECK();
  return dqkv;
}

// ---- fused BERT sublayer forwards: one op dispatch per post-LN sublayer (the eager step is host-
// bound on slow hosts: every Python -> C++ op call costs ~10 us of enqueue, profiles/r5_bert_host.txt).
// Same kernels and order as the op-by-op BertAttentionBlockFn / BertFFNBlockFn forwards
// (ops/transformer.py); the dropout seeds / offsets come from the Python RNG as before.
std::vector<at::Tensor> conv_fwd(const at::Tensor& x, const at::Tensor& w, int64_t stride, int64_t pad,
                                 const c10::optional<at::Tensor>& bias, const c10::optional<at::Tensor>& resid,
                                 bool relu, bool want_stats, const c10::optional<at::Tensor>& in_scale,
                                 const c10::optional<at::Tensor>& in_shift);
std::vector<at::Tensor> linear_gelu_fwd(const at::Tensor& x, const at::Tensor& w, const c10::optional<at::Tensor>& bias);

static at::Tensor linear_fwd(const at::Tensor& x, const at::Tensor& w, const at::Tensor& bias) {
  const int64_t M = x.size(0), C = x.size(1), N = w.size(0);
  return conv_fwd(x.view({M, 1, 1, C}), w.view({N, 1, 1, C}), 1, 0, bias, c10::nullopt, false, false, c10::nullopt,
                  c10::nullopt)[0].view({M, N});
}

// h1 = LayerNorm(h + dropout(attn_out(attention(qkv(h)))))  -> [h1, qkv, ctx, lse, xs, mean, rstd]
std::vector<at::Tensor> bert_attn_fwd(const at::Tensor& h, const c10::optional<at::Tensor>& ids, const at::Tensor& wq,
                                      const at::Tensor& bq, const at::Tensor& wo, const at::Tensor& bo,
                                      const at::Tensor& g, const at::Tensor& b, int64_t B, int64_t S, int64_t H,
                                      double p_attn, int64_t seed_a, int64_t off_a, double p_hid, int64_t seed_h,
                                      int64_t off_h, double eps, const c10::optional<at::Tensor>& salt) {
  at::Tensor qkv = linear_fwd(h, wq, bq);
  auto at_ = attention_fwd(qkv, ids, B, S, H, p_attn, seed_a, off_a, salt);
  at::Tensor a = linear_fwd(at_[0], wo, bo);
  auto ln = layernorm_fwd(a, h, g, b, eps, p_hid, seed_h, off_h, salt);
  return {ln[0], qkv, at_[0], at_[1], ln[1], ln[2], ln[3]};
}

// h2 = LayerNorm(h1 + dropout(ffn2(gelu(ffn1(h1)))))  -> [h2, g, u, xs, mean, rstd]
std::vector<at::Tensor> bert_ffn_fwd(const at::Tensor& h1, const at::Tensor& w1, const at::Tensor& b1,
                                     const at::Tensor& w2, const at::Tensor& b2, const at::Tensor& g,
                                     const at::Tensor& b, double p_hid, int64_t seed_h, int64_t off_h, double eps,
                                     const c10::optional<at::Tensor>& salt) {
  auto gu = linear_gelu_fwd(h1, w1, b1);
  at::Tensor f = linear_fwd(gu[0], w2, b2);
  auto ln = layernorm_fwd(f, h1, g, b, eps, p_hid, seed_h, off_h, salt);
  return {ln[0], gu[0], gu[1], ln[1], ln[2], ln[3]};
}

}  // namespace pcmp

TORCH_LIBRARY_FRAGMENT(pcmp, m) {
  m.def("bert_attn_fwd(Tensor h, Tensor? ids, Tensor wq, Tensor bq, Tensor wo, Tensor bo, Tensor g, Tensor b, int B, "
        "int S, int H, float p_attn, int seed_a, int off_a, float p_hid, int seed_h, int off_h, float eps, "
        "Tensor? salt=None) -> Tensor[]",
        &pcmp::bert_attn_fwd);
  m.def("bert_ffn_fwd(Tensor h1, Tensor w1, Tensor b1, Tensor w2, Tensor b2, Tensor g, Tensor b, float p_hid, "
        "int seed_h, int off_h, float eps, Tensor? salt=None) -> Tensor[]",
        &pcmp::bert_ffn_fwd);
  m.def("layernorm_fwd(Tensor x, Tensor? r, Tensor g, Tensor b, float eps, float p=0., int seed=0, int offset=0, "
        "Tensor? salt=None) -> Tensor[]", &pcmp::layernorm_fwd);
  m.def("layernorm_bwd_fused(Tensor dy, Tensor xs, Tensor mean, Tensor rstd, Tensor g, Tensor(a!)? dg, "
        "Tensor(b!)? db, Tensor(c!)? dbias, int accmask, float p, int seed, int offset, Tensor? salt=None) -> Tensor[]",
        &pcmp::layernorm_bwd_fused);
  m.def("layernorm_bwd(Tensor dy, Tensor xs, Tensor mean, Tensor rstd, Tensor g, Tensor(a!)? dg, Tensor(b!)? db, "
        "bool accumulate) -> Tensor",
        &pcmp::layernorm_bwd);
  m.def("embed_layernorm_fwd(Tensor x, Tensor pos, Tensor tt, Tensor g, Tensor b, float eps) -> Tensor[]",
        &pcmp::embed_layernorm_fwd);
  m.def("gelu_fwd(Tensor x) -> Tensor", &pcmp::gelu_fwd);
  m.def("gelu_bwd(Tensor dy, Tensor x) -> Tensor", &pcmp::gelu_bwd);
  m.def("tanh_fwd(Tensor x) -> Tensor", &pcmp::tanh_fwd);
  m.def("tanh_bwd(Tensor dy, Tensor y) -> Tensor", &pcmp::tanh_bwd);
  m.def("add_bf16(Tensor a, Tensor b) -> Tensor", &pcmp::add_bf16);
  m.def("attention_fwd(Tensor qkv, Tensor? ids, int B, int S, int H, float p_drop, int seed, int offset, "
        "Tensor? salt=None) -> Tensor[]",
        &pcmp::attention_fwd);
  m.def("attention_bwd(Tensor dctx, Tensor qkv, Tensor ctx, Tensor lse, Tensor? ids, int B, int S, int H, float p_drop, "
        "int seed, int offset, Tensor? salt=None) -> Tensor",
        &pcmp::attention_bwd);
}

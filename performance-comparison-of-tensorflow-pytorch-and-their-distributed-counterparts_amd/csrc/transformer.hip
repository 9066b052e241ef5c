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
static int egrid(int64_t n) { return (int)std::max<int64_t>(1, std::min<int64_t>(4096, (n + 255) / 256)); }

// ------------------------------------------------------------------------------- LayerNorm
// one wave per row; y = LN(x [+ r]) * g + b ; saves xs = x + r (when r given), mean, rstd.
__global__ void layernorm_fwd_kernel(const __bf16* __restrict__ x, const __bf16* __restrict__ r,
                                     const float* __restrict__ g, const float* __restrict__ b, __bf16* __restrict__ y,
                                     __bf16* __restrict__ xs, float* __restrict__ mean_out,
                                     float* __restrict__ rstd_out, int M, int D, float eps) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
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
      if (r) {
        float w[8];
        ldv8(r + (size_t)row * D + cv * 8, w);
#pragma unroll
        for (int e = 0; e < 8; ++e) v[k][e] += w[e];
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

// column reduction of partials [T][L] -> out[L] (fp32 result, fp64 accumulation); accumulate opt.
// ------------------------------------------------------------------------------- activations
__device__ __forceinline__ float gelu_erf(float x) { return 0.5f * x * (1.f + erff(x * 0.70710678118654752f)); }
__device__ __forceinline__ float dgelu_erf(float x) {
  const float cdf = 0.5f * (1.f + erff(x * 0.70710678118654752f));
  const float pdf = 0.3989422804014327f * __expf(-0.5f * x * x);
  return cdf + x * pdf;
}

// mode 0: gelu, 1: tanh ; y = f(x)
__global__ void act_fwd_kernel(const __bf16* __restrict__ x, __bf16* __restrict__ y, int64_t nv, int mode) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nv; i += (int64_t)gridDim.x * blockDim.x) {
    float v[8];
    ldv8(x + i * 8, v);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = mode == 0 ? gelu_erf(v[e]) : tanhf(v[e]);
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
    for (int e = 0; e < 8; ++e) g[e] *= mode == 0 ? dgelu_erf(v[e]) : (1.f - v[e] * v[e]);
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

// stage rows [S][64] of a qkv section into LDS (row-major, padded) and optionally transposed
__device__ __forceinline__ void stage_head(const __bf16* src, int ldsrc, int S, __bf16* dst, __bf16* dstT) {
  for (int i = threadIdx.x; i < S * (AD / 8); i += blockDim.x) {
    const int s = i / (AD / 8), c8 = i % (AD / 8);
    const uint4 v = *reinterpret_cast<const uint4*>(src + (size_t)s * ldsrc + c8 * 8);
    if (dst) *reinterpret_cast<uint4*>(dst + s * ADP + c8 * 8) = v;
    if (dstT) {
      const unsigned short* u = reinterpret_cast<const unsigned short*>(&v);
#pragma unroll
      for (int e = 0; e < 8; ++e) reinterpret_cast<unsigned short*>(dstT)[(c8 * 8 + e) * ASP + s] = u[e];
    }
  }
}

__global__ void __launch_bounds__(256) attention_fwd_kernel(const AttnParams p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int bh = blockIdx.x, b = bh / p.H, h = bh % p.H;
  const int S = p.S, D3 = 3 * p.D;
  __bf16* sQ = reinterpret_cast<__bf16*>(smem);          // [S][ADP]
  __bf16* sK = sQ + AS * ADP;                             // [S][ADP]
  __bf16* sVt = sK + AS * ADP;                            // [AD][ASP]
  __bf16* sP = sVt + AD * ASP;                            // [4 waves][32][ASP]
  float* sMask = reinterpret_cast<float*>(sP + 4 * 32 * ASP);  // [S]
  const __bf16* base = p.qkv + (size_t)b * S * D3 + h * AD;
  stage_head(base, D3, S, sQ, nullptr);
  stage_head(base + p.D, D3, S, sK, nullptr);
  stage_head(base + 2 * p.D, D3, S, nullptr, sVt);
  for (int s = threadIdx.x; s < S; s += blockDim.x)
    sMask[s] = (p.ids && p.ids[(size_t)b * S + s] <= 0) ? -1e30f : 0.f;
  __syncthreads();
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int NT = S / 16;  // key tiles (<= 8)
  {
    const int q0 = w * 32;
    const bool act = q0 < S;  // all waves reach the barrier below
    f32x4 acc[2][8];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0, 0, 0, 0};
    __bf16* P = sP + w * 32 * ASP;
    if (act) {
#pragma unroll
    for (int kk = 0; kk < AD; kk += 32) {
      const int k0 = kk + 8 * (lane >> 4);
      bf16x8 a0 = frag_row(sQ, ADP, q0 + (lane & 15), k0), a1 = frag_row(sQ, ADP, q0 + 16 + (lane & 15), k0);
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (j < NT) {
          const bf16x8 bb = frag_row(sK, ADP, j * 16 + (lane & 15), k0);
          acc[0][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, bb, acc[0][j], 0, 0, 0);
          acc[1][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, bb, acc[1][j], 0, 0, 0);
        }
    }
    // softmax over keys for rows (i, e): row = q0 + 16i + 4*(lane>>4) + e ; key = 16j + (lane&15)
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float mx = -INFINITY;
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (j < NT) {
            const float v = acc[i][j][e] * p.scale + sMask[j * 16 + (lane & 15)];
            acc[i][j][e] = v;
            mx = fmaxf(mx, v);
          }
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) mx = fmaxf(mx, __shfl_xor(mx, o, 64));
        float sum = 0.f;
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (j < NT) { const float ev = __expf(acc[i][j][e] - mx); acc[i][j][e] = ev; sum += ev; }
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) sum += __shfl_xor(sum, o, 64);
        const float inv = 1.f / sum;
        const int rl = 16 * i + 4 * (lane >> 4) + e;
        const int q = q0 + rl;
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (j < NT) {
            const int key = j * 16 + (lane & 15);
            const float pv = acc[i][j][e] * inv * drop_scale(p, bh, q, key);
            reinterpret_cast<unsigned short*>(P)[rl * ASP + key] = f2bf(pv);
          }
        if ((lane & 15) == 0) p.lse[(size_t)bh * S + q] = mx + __logf(sum);
      }
    }
    __syncthreads();
    if (!act) return;
    // O[32][64] = P[32][S] V[S][64] ; B fragment from V^T rows
    f32x4 o[2][4];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) o[i][j] = f32x4{0, 0, 0, 0};
    for (int kk = 0; kk < S; kk += 32) {
      const int k0 = kk + 8 * (lane >> 4);
      const bf16x8 a0 = frag_row(P, ASP, lane & 15, k0), a1 = frag_row(P, ASP, 16 + (lane & 15), k0);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const bf16x8 bb = frag_row(sVt, ASP, j * 16 + (lane & 15), k0);
        o[0][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, bb, o[0][j], 0, 0, 0);
        o[1][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, bb, o[1][j], 0, 0, 0);
      }
    }
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int q = q0 + 16 * i + 4 * (lane >> 4) + e;
          const int d = 16 * j + (lane & 15);
          reinterpret_cast<unsigned short*>(p.out)[((size_t)b * S + q) * p.D + h * AD + d] = f2bf(o[i][j][e]);
        }
  }
}

__global__ void __launch_bounds__(256) attention_bwd_kernel(const AttnParams p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int bh = blockIdx.x, b = bh / p.H, h = bh % p.H;
  const int S = p.S, D3 = 3 * p.D;
  // Q, K, V, dO row-major; their transposed operands are read with frag_tr
  __bf16* sQ = reinterpret_cast<__bf16*>(smem);   // [S][ADP]
  __bf16* sK = sQ + AS * ADP;                      // [S][ADP]
  __bf16* sV = sK + AS * ADP;                      // [S][ADP]
  __bf16* sdO = sV + AS * ADP;                     // [S][ADP]
  __bf16* sT = sdO + AS * ADP;                     // [S keys][ASP] : Pd^T then dS^T tiles (wave w: keys 32w..)
  float* sL = reinterpret_cast<float*>(sT + AS * ASP);  // lse [S]
  float* sDd = sL + AS;                                  // D [S]
  float* sMask = sDd + AS;                               // [S]
  const __bf16* base = p.qkv + (size_t)b * S * D3 + h * AD;
  stage_head(base, D3, S, sQ, nullptr);
  stage_head(base + p.D, D3, S, sK, nullptr);
  stage_head(base + 2 * p.D, D3, S, sV, nullptr);
  stage_head(p.dout + (size_t)b * S * p.D + h * AD, p.D, S, sdO, nullptr);
  for (int s = threadIdx.x; s < S; s += blockDim.x) {
    sL[s] = p.lse[(size_t)bh * S + s];
    sMask[s] = (p.ids && p.ids[(size_t)b * S + s] <= 0) ? -1e30f : 0.f;
    // D = rowsum(dO * O)
    float acc = 0.f;
    const __bf16* orow = p.o + ((size_t)b * S + s) * p.D + h * AD;
    const __bf16* drow = p.dout + ((size_t)b * S + s) * p.D + h * AD;
    for (int d = 0; d < AD; d += 8) {
      float a[8], c[8];
      ldv8(orow + d, a);
      ldv8(drow + d, c);
#pragma unroll
      for (int e = 0; e < 8; ++e) acc += a[e] * c[e];
    }
    sDd[s] = acc;
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int NT = S / 16;
  const int kw0 = w * 32;           // this wave's keys
  const bool active = kw0 < S;
  __bf16* T = sT + kw0 * ASP;       // [32 keys][ASP]
  f32x4 dk[2][4], dv[2][4];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) { dk[i][j] = f32x4{0, 0, 0, 0}; dv[i][j] = f32x4{0, 0, 0, 0}; }
  f32x4 sacc[2][8], pacc[2][8];
  if (active) {
    // S^T[key][q] = K_w Q^T ; dP^T[key][q] = V_w dO^T
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) { sacc[i][j] = f32x4{0, 0, 0, 0}; pacc[i][j] = f32x4{0, 0, 0, 0}; }
#pragma unroll
    for (int kk = 0; kk < AD; kk += 32) {
      const int k0 = kk + 8 * (lane >> 4);
      const bf16x8 ka0 = frag_row(sK, ADP, kw0 + (lane & 15), k0), ka1 = frag_row(sK, ADP, kw0 + 16 + (lane & 15), k0);
      const bf16x8 va0 = frag_row(sV, ADP, kw0 + (lane & 15), k0), va1 = frag_row(sV, ADP, kw0 + 16 + (lane & 15), k0);
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (j < NT) {
          const bf16x8 qb = frag_row(sQ, ADP, j * 16 + (lane & 15), k0);
          const bf16x8 ob = frag_row(sdO, ADP, j * 16 + (lane & 15), k0);
          sacc[0][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ka0, qb, sacc[0][j], 0, 0, 0);
          sacc[1][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ka1, qb, sacc[1][j], 0, 0, 0);
          pacc[0][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(va0, ob, pacc[0][j], 0, 0, 0);
          pacc[1][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(va1, ob, pacc[1][j], 0, 0, 0);
        }
    }
    // P^T = exp(S^T*scale + mask[key] - lse[q]); write Pd^T (dropout applied) to T; dS^T kept in sacc
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int kl = 16 * i + 4 * (lane >> 4) + e;
        const int key = kw0 + kl;
        const float mk = sMask[key];
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (j < NT) {
            const int q = j * 16 + (lane & 15);
            const float pr = __expf(sacc[i][j][e] * p.scale + mk - sL[q]);
            const float ds = drop_scale(p, bh, q, key);
            reinterpret_cast<unsigned short*>(T)[kl * ASP + q] = f2bf(pr * ds);
            const float dP = pacc[i][j][e] * ds;
            sacc[i][j][e] = pr * (dP - sDd[q]);  // dS^T (unscaled)
          }
      }
    __builtin_amdgcn_s_waitcnt(0);
  }
  __syncthreads();
  if (active) {
    // dV[key][d] = sum_q Pd^T[key][q] dO[q][d]  : A = T rows (k = q), B from dO^T rows
    for (int kk = 0; kk < S; kk += 32) {
      const int k0 = kk + 8 * (lane >> 4);
      const bf16x8 a0 = frag_row(T, ASP, lane & 15, k0), a1 = frag_row(T, ASP, 16 + (lane & 15), k0);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const bf16x8 bb = frag_tr(sdO, ADP, kk, j * 16);
        dv[0][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, bb, dv[0][j], 0, 0, 0);
        dv[1][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, bb, dv[1][j], 0, 0, 0);
      }
    }
  }
  __syncthreads();
  if (active) {
    // overwrite T with dS^T (bf16)
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int kl = 16 * i + 4 * (lane >> 4) + e;
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (j < NT) reinterpret_cast<unsigned short*>(T)[kl * ASP + j * 16 + (lane & 15)] = f2bf(sacc[i][j][e]);
      }
  }
  __syncthreads();
  if (active) {
    // dK[key][d] = sum_q dS^T[key][q] Q[q][d] * scale : A = T rows, B from Q^T rows
    for (int kk = 0; kk < S; kk += 32) {
      const int k0 = kk + 8 * (lane >> 4);
      const bf16x8 a0 = frag_row(T, ASP, lane & 15, k0), a1 = frag_row(T, ASP, 16 + (lane & 15), k0);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const bf16x8 bb = frag_tr(sQ, ADP, kk, j * 16);
        dk[0][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, bb, dk[0][j], 0, 0, 0);
        dk[1][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, bb, dk[1][j], 0, 0, 0);
      }
    }
    // write dK, dV
    __bf16* dst = p.dqkv + (size_t)b * S * D3 + h * AD;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int key = kw0 + 16 * i + 4 * (lane >> 4) + e;
          const int d = 16 * j + (lane & 15);
          reinterpret_cast<unsigned short*>(dst)[(size_t)key * D3 + p.D + d] = f2bf(dk[i][j][e] * p.scale);
          reinterpret_cast<unsigned short*>(dst)[(size_t)key * D3 + 2 * p.D + d] = f2bf(dv[i][j][e]);
        }
  }
  // dQ[q][d] = sum_key dS[q][key] K[key][d] * scale ; wave w takes queries 32w.. ; A[q][key] = dS^T[key][q]
  if (active) {
    const int q0 = w * 32;
    f32x4 dq[2][4];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) dq[i][j] = f32x4{0, 0, 0, 0};
    for (int kk = 0; kk < S; kk += 32) {
      const bf16x8 a0 = frag_tr(sT, ASP, kk, q0), a1 = frag_tr(sT, ASP, kk, q0 + 16);
      bf16x8 bb[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) bb[j] = frag_tr(sK, ADP, kk, j * 16);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        dq[0][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, bb[j], dq[0][j], 0, 0, 0);
        dq[1][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, bb[j], dq[1][j], 0, 0, 0);
      }
    }
    __bf16* dst = p.dqkv + (size_t)b * S * D3 + h * AD;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int q = q0 + 16 * i + 4 * (lane >> 4) + e;
          const int d = 16 * j + (lane & 15);
          reinterpret_cast<unsigned short*>(dst)[(size_t)q * D3 + d] = f2bf(dq[i][j][e] * p.scale);
        }
  }
}

// ------------------------------------------------------------------------------- host
std::vector<at::Tensor> layernorm_fwd(const at::Tensor& x, const c10::optional<at::Tensor>& r, const at::Tensor& g,
                                      const at::Tensor& b, double eps) {
  PCMP_CHECK_BF16(x); PCMP_CHECK_CONTIG(x); PCMP_CHECK_F32(g); PCMP_CHECK_F32(b);
  const int D = x.size(-1);
  const int M = x.numel() / D;
  TORCH_CHECK(D % 8 == 0 && D <= 2048, "layernorm: D % 8 and <= 2048");
  auto y = at::empty_like(x);
  const bool hr = r.has_value() && r->defined();
  at::Tensor xs = hr ? at::empty_like(x) : x;
  auto f32 = x.options().dtype(at::kFloat);
  auto mean = at::empty({M}, f32), rstd = at::empty({M}, f32);
  hipLaunchKernelGGL(layernorm_fwd_kernel, dim3(ceil_div(M, 4)), dim3(256), 0, cur_stream(), ptr<__bf16>(x),
                     hr ? ptr<__bf16>(*r) : nullptr, ptr<float>(g), ptr<float>(b), ptr<__bf16>(y),
                     hr ? ptr<__bf16>(xs) : nullptr, ptr<float>(mean), ptr<float>(rstd), M, D, (float)eps);
  PCMP_LAUNCH_CHECK();
  return {y, xs, mean, rstd};
}

// returns dx; dgamma/dbeta written (or accumulated) into the given fp32 tensors when defined
at::Tensor layernorm_bwd(const at::Tensor& dy, const at::Tensor& xs, const at::Tensor& mean, const at::Tensor& rstd,
                         const at::Tensor& g, const c10::optional<at::Tensor>& dg, const c10::optional<at::Tensor>& db,
                         bool accumulate) {
  auto dyc = dy.contiguous();
  const int D = xs.size(-1);
  const int M = xs.numel() / D;
  auto dx = at::empty_like(xs);
  static const int target_blocks = [] {   // PCMP_LN_BLOCKS overrides (A/B runs)
    const char* e = std::getenv("PCMP_LN_BLOCKS");
    return e ? std::max(1, std::atoi(e)) : 256;
  }();
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

static at::Tensor act_fwd(const at::Tensor& x, int mode) {
  PCMP_CHECK_BF16(x); PCMP_CHECK_CONTIG(x);
  TORCH_CHECK(x.numel() % 8 == 0, "activation numel % 8");
  auto y = at::empty_like(x);
  hipLaunchKernelGGL(act_fwd_kernel, dim3(egrid(x.numel() / 8)), dim3(256), 0, cur_stream(), ptr<__bf16>(x),
                     ptr<__bf16>(y), x.numel() / 8, mode);
  PCMP_LAUNCH_CHECK();
  return y;
}
static at::Tensor act_bwd(const at::Tensor& dy, const at::Tensor& xy, int mode) {
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
  PCMP_CHECK_BF16(a); PCMP_CHECK_BF16(b);
  auto ac = a.contiguous(), bc = b.contiguous();
  TORCH_CHECK(ac.numel() == bc.numel() && ac.numel() % 8 == 0, "add_bf16: shapes");
  auto y = at::empty_like(ac);
  hipLaunchKernelGGL(add_bf16_kernel, dim3(egrid(ac.numel() / 8)), dim3(256), 0, cur_stream(), ptr<__bf16>(ac),
                     ptr<__bf16>(bc), ptr<__bf16>(y), ac.numel() / 8);
  PCMP_LAUNCH_CHECK();
  return y;
}

static size_t attn_fwd_smem() { return ((size_t)2 * AS * ADP + AD * ASP + 4 * 32 * ASP) * 2 + AS * 4; }
static size_t attn_bwd_smem() { return ((size_t)4 * AS * ADP + AS * ASP) * 2 + 3 * AS * 4; }

// qkv [B*S][3D] bf16 -> [ctx [B*S][D] bf16, lse [B*H][S] f32]
std::vector<at::Tensor> attention_fwd(const at::Tensor& qkv, const c10::optional<at::Tensor>& ids, int64_t B,
                                      int64_t S, int64_t H, double p_drop, int64_t seed, int64_t offset,
                                      const c10::optional<at::Tensor>& salt) {
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
  hipLaunchKernelGGL(attention_fwd_kernel, dim3(B * H), dim3(256), attn_fwd_smem(), cur_stream(), p);
  PCMP_LAUNCH_CHECK();
  return {ctx, lse};
}

at::Tensor attention_bwd(const at::Tensor& dctx, const at::Tensor& qkv, const at::Tensor& ctx, const at::Tensor& lse,
                         const c10::optional<at::Tensor>& ids, int64_t B, int64_t S, int64_t H, double p_drop,
                         int64_t seed, int64_t offset, const c10::optional<at::Tensor>& salt) {
  PCMP_CHECK_BF16(qkv);
  auto dc = dctx.contiguous();
  const int D3 = qkv.size(-1), D = D3 / 3;
  auto dqkv = at::empty_like(qkv);
  at::Tensor idc;
  if (ids.has_value() && ids->defined()) idc = ids->contiguous();
  AttnParams p{ptr<__bf16>(qkv), idc.defined() ? idc.data_ptr<int64_t>() : nullptr, nullptr, ptr<float>(lse),
               ptr<__bf16>(dc), ptr<__bf16>(ctx), ptr<__bf16>(dqkv), (int)B, (int)S, (int)H, D, 0.125f,
               (float)p_drop, (uint64_t)seed, (uint64_t)offset, salt_ptr(salt)};
  hipLaunchKernelGGL(attention_bwd_kernel, dim3(B * H), dim3(256), attn_bwd_smem(), cur_stream(), p);
  PCMP_LAUNCH_CHECK();
  return dqkv;
}

}  // namespace pcmp

TORCH_LIBRARY_FRAGMENT(pcmp, m) {
  m.def("layernorm_fwd(Tensor x, Tensor? r, Tensor g, Tensor b, float eps) -> Tensor[]", &pcmp::layernorm_fwd);
  m.def("layernorm_bwd(Tensor dy, Tensor xs, Tensor mean, Tensor rstd, Tensor g, Tensor(a!)? dg, Tensor(b!)? db, "
        "bool accumulate) -> Tensor",
        &pcmp::layernorm_bwd);
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

// BatchNorm2d (NHWC, bf16 activations, fp32 statistics) for CDNA4.
//
// Replaces the BatchNorm2d(+ReLU)(+residual add) layers of torchvision ResNet-50
// (pytorch_training_inference_on_image.ipynb:454-626; SURVEY.md §2.4.1 "BatchNorm2d ... fused
// with ReLU, and with residual add+ReLU at the block tail").  Train mode uses batch statistics
// and updates running stats with momentum (running_var unbiased), eval mode uses running stats.
//
// Forward is split into three memory passes at most:
//   1. per-block column partial sums (fused into the producing conv's epilogue, or
//      bn_partials_kernel when the producer is not ours),
//   2. bn_finalize_kernel: fp64 reduction of the partials -> mean/invstd, per-channel scale/shift,
//      running-stat update,
//   3. bn_apply_kernel: y = act(x*scale+shift [+ x2*scale2+shift2 | + res]) with 16-B vectors.
// Backward: bn_bwd_reduce_kernel (g = dy*(y>0) recomputed, partial sums of g and g*xhat for up
// to two BN layers that share g -- the bottleneck tail and its downsample branch), then
// bn_bwd_finalize_kernel (dgamma/dbeta into the flat gradient buffer, per-channel dx
// coefficients), then bn_bwd_apply_kernel dx = k1*g + k2*x + k3 (optionally also writing g for
// the identity path).
#include "common.h"
#include "f32.h"

#include <mutex>
#include <unordered_map>

namespace pcmp {

struct RowMap {
  int CV;    // 8-channel vectors per row
  int tpr;   // threads per row
  int rpp;   // rows per pass
  int vpt;   // vectors per thread per row
};
static RowMap make_rowmap(int C) {
  RowMap r;
  r.CV = C / 8;
  r.tpr = r.CV < 256 ? r.CV : 256;
  r.rpp = 256 / r.tpr;
  r.vpt = r.CV / r.tpr;
  return r;
}

__device__ __forceinline__ void load8(const __bf16* p, float* v) {
  const u16x8 u = *reinterpret_cast<const u16x8*>(p);
#pragma unroll
  for (int e = 0; e < 8; ++e) v[e] = bf2f(u[e]);
}
__device__ __forceinline__ void store8(__bf16* p, const float* v) {
  u16x8 u;
#pragma unroll
  for (int e = 0; e < 8; ++e) u[e] = f2bf(v[e]);
  *reinterpret_cast<u16x8*>(p) = u;
}

// ---- forward partial statistics of x (used when the producer did not emit them) ----------
__global__ void bn_partials_kernel(const __bf16* __restrict__ x, float* __restrict__ part, int M, int C,
                                   int rows_per_block, RowMap rm) {
  extern __shared__ float sh[];  // [rpp][2][C]
  const int tid = threadIdx.x;
  const int tr = tid / rm.tpr, tc = tid % rm.tpr;
  const int r0 = blockIdx.x * rows_per_block;
  const int r1 = min(M, r0 + rows_per_block);
  for (int k = 0; k < rm.vpt; ++k) {
    const int cv = tc + k * rm.tpr;
    float s1[8] = {0}, s2[8] = {0};
    for (int r = r0 + tr; r < r1; r += rm.rpp) {
      float v[8];
      load8(x + (size_t)r * C + cv * 8, v);
#pragma unroll
      for (int e = 0; e < 8; ++e) { s1[e] += v[e]; s2[e] += v[e] * v[e]; }
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      sh[(tr * 2 + 0) * C + cv * 8 + e] = s1[e];
      sh[(tr * 2 + 1) * C + cv * 8 + e] = s2[e];
    }
  }
  __syncthreads();
  for (int i = tid; i < 2 * C; i += blockDim.x) {
    float s = 0.f;
    for (int r = 0; r < rm.rpp; ++r) s += sh[r * 2 * C + i];
    part[(size_t)blockIdx.x * 2 * C + i] = s;
  }
}

// ---- stage-1 column reduction of partials: part [T][L] f32 -> red [G][L] f64 ----------------
// grid (ceil(L/64), G), 256 threads = 64 columns x 4 row lanes; each block sums `rpb` rows.
__global__ void partials_reduce_kernel(const float* __restrict__ part, int T, int L, int rpb,
                                       double* __restrict__ red) {
  __shared__ double sh[4][64];
  const int col = blockIdx.x * 64 + (threadIdx.x & 63);
  const int g = threadIdx.x >> 6;
  const int r0 = blockIdx.y * rpb, r1 = min(T, r0 + rpb);
  // 8 independent loads in flight per thread (a dependent add chain would expose one global-load
  // latency per row: this launch-boundary reduction is latency-bound, not bandwidth-bound)
  double s8[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (col < L) {
    int r = r0 + g;
    for (; r + 28 < r1; r += 32) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = part[(size_t)(r + 4 * u) * L + col];
#pragma unroll
      for (int u = 0; u < 8; ++u) s8[u] += v[u];
    }
    for (; r < r1; r += 4) s8[0] += part[(size_t)r * L + col];
  }
  const double s = ((s8[0] + s8[1]) + (s8[2] + s8[3])) + ((s8[4] + s8[5]) + (s8[6] + s8[7]));
  sh[g][threadIdx.x & 63] = s;
  __syncthreads();
  if (g == 0 && col < L) red[(size_t)blockIdx.y * L + col] = s + sh[1][threadIdx.x] + sh[2][threadIdx.x] + sh[3][threadIdx.x];
}

// per-channel finalize math, shared by the two-launch and the fused (last-arriver) paths
struct FinFwd {
  double count;
  const float* gamma; const float* beta;
  float* rmean; float* rvar;
  float momentum, eps;
  float* mean_out; float* invstd_out; float* scale_out; float* shift_out;
};
__device__ __forceinline__ void bn_finalize_channel(int c, double s1, double s2, const FinFwd& a) {
  const double mean = s1 / a.count;
  double var = s2 / a.count - mean * mean;
  if (var < 0) var = 0;
  const float invstd = (float)(1.0 / sqrt(var + (double)a.eps));
  a.mean_out[c] = (float)mean;
  a.invstd_out[c] = invstd;
  const float gm = a.gamma ? a.gamma[c] : 1.f, bt = a.beta ? a.beta[c] : 0.f;
  a.scale_out[c] = gm * invstd;
  a.shift_out[c] = bt - (float)mean * gm * invstd;
  if (a.rmean) {
    const double unbiased = a.count > 1 ? var * a.count / (a.count - 1) : var;
    a.rmean[c] = (1.f - a.momentum) * a.rmean[c] + a.momentum * (float)mean;
    a.rvar[c] = (1.f - a.momentum) * a.rvar[c] + a.momentum * (float)unbiased;
  }
}

struct FinBwd {
  double count;
  const float* gamma; const float* mean; const float* invstd;
  float* dgamma_out; float* dbeta_out;
  int accumulate;
  float* coef;
  int C;
};
__device__ __forceinline__ void bn_bwd_finalize_channel(int c, double sg, double sgx, const FinBwd& a) {
  const float dbeta = (float)sg, dgamma = (float)sgx;
  if (a.dgamma_out) a.dgamma_out[c] = a.accumulate ? a.dgamma_out[c] + dgamma : dgamma;
  if (a.dbeta_out) a.dbeta_out[c] = a.accumulate ? a.dbeta_out[c] + dbeta : dbeta;
  const float gm = a.gamma ? a.gamma[c] : 1.f;
  const float is = a.invstd[c], mu = a.mean[c];
  const float k1 = gm * is;
  const float k2 = -(float)(gm * (double)is * is * sgx / a.count);
  const float k3 = -(float)(gm * (double)is * sg / a.count) - k2 * mu;
  a.coef[c] = k1;
  a.coef[a.C + c] = k2;
  a.coef[2 * a.C + c] = k3;
}

// ---- one-launch finalize for up to a few hundred partial rows -------------------------------
// The GEMM epilogues emit one partial row per BM-row tile: 98-392 rows for ResNet-50's layer-3/4
// BatchNorms at B=256.  1024 threads = 64 channels x 16 row lanes (8 loads in flight per thread),
// the lanes summed in fixed order: ONE launch where the two-stage path (partials_reduce_kernel into
// <= 64 fp64 rows + the finalize) takes two -- ~100 launches per ResNet-50 step, each a ~5 us
// dependent kernel boundary on the compute stream.  (Round 4's single-launch alternative, a last-
// arriver ticket over stage-1 blocks, paid an agent-scope release per block: -3.2 %, removed.)
template <typename PT, bool BWD, typename FA>
__global__ __launch_bounds__(1024) void bn_finalize_wide_kernel(const PT* __restrict__ part, int T, int C, FA fa) {
  __shared__ double sh[2][16][64];
  const int j = threadIdx.x & 63, g = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + j;
  double s1 = 0, s2 = 0;
  if (c < C) {
    int t = g;
    for (; t + 48 < T; t += 64) {
      PT a[4], b[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        a[u] = part[(size_t)(t + 16 * u) * 2 * C + c];
        b[u] = part[(size_t)(t + 16 * u) * 2 * C + C + c];
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) { s1 += a[u]; s2 += b[u]; }
    }
    for (; t < T; t += 16) {
      s1 += part[(size_t)t * 2 * C + c];
      s2 += part[(size_t)t * 2 * C + C + c];
    }
  }
  sh[0][g][j] = s1;
  sh[1][g][j] = s2;
  __syncthreads();
  if (g == 0 && c < C) {
    for (int k = 1; k < 16; ++k) { s1 += sh[0][k][j]; s2 += sh[1][k][j]; }
    if constexpr (BWD) bn_bwd_finalize_channel(c, s1, s2, fa);
    else bn_finalize_channel(c, s1, s2, fa);
  }
}

// (Round 5's one-launch last-arriver finalize for > 512 partial rows -- sc1 write-through hand-off
// without release / acquire, off by default and 0.1-0.4 % slower in the step, profiles/
// r5_bn_lastblock_ab.txt -- was removed in round 6: its correctness rested on ISA-level ordering
// arguments, not on the memory model.  Above bn_wide_rows the two-launch path runs.)

// ---- finalize: partials [T][2][C] -> mean, invstd, scale, shift; running stats update --------
// block = 256 threads handles 64 channels (4 row-groups of partials).
template <typename PT>
__global__ void bn_finalize_kernel(const PT* __restrict__ part, int T, int C, double count,
                                   const float* __restrict__ gamma, const float* __restrict__ beta,
                                   float* __restrict__ rmean, float* __restrict__ rvar, float momentum,
                                   float eps, float* __restrict__ mean_out, float* __restrict__ invstd_out,
                                   float* __restrict__ scale_out, float* __restrict__ shift_out) {
  __shared__ double sh[2][4][64];
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  const int g = threadIdx.x >> 6;
  double s1 = 0, s2 = 0;
  if (c < C) {
    int t = g;
    for (; t + 12 < T; t += 16) {   // 4 rows x 2 sums of independent loads in flight
      PT a[4], b[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        a[u] = part[(size_t)(t + 4 * u) * 2 * C + c];
        b[u] = part[(size_t)(t + 4 * u) * 2 * C + C + c];
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) { s1 += a[u]; s2 += b[u]; }
    }
    for (; t < T; t += 4) {
      s1 += part[(size_t)t * 2 * C + c];
      s2 += part[(size_t)t * 2 * C + C + c];
    }
  }
  sh[0][g][threadIdx.x & 63] = s1;
  sh[1][g][threadIdx.x & 63] = s2;
  __syncthreads();
  if (g == 0 && c < C) {
    for (int k = 1; k < 4; ++k) { s1 += sh[0][k][threadIdx.x]; s2 += sh[1][k][threadIdx.x]; }
    bn_finalize_channel(c, s1, s2, FinFwd{count, gamma, beta, rmean, rvar, momentum, eps, mean_out, invstd_out,
                                          scale_out, shift_out});
  }
}

// eval-mode coefficients from running statistics
__global__ void bn_eval_coeff_kernel(int C, const float* __restrict__ gamma, const float* __restrict__ beta,
                                     const float* __restrict__ rmean, const float* __restrict__ rvar,
                                     float eps, float* __restrict__ scale_out, float* __restrict__ shift_out) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const float invstd = rsqrtf(rvar[c] + eps);
  const float gm = gamma ? gamma[c] : 1.f, bt = beta ? beta[c] : 0.f;
  scale_out[c] = gm * invstd;
  shift_out[c] = bt - rmean[c] * gm * invstd;
}

// ---- apply: y = act(x*sc+sh [+ x2*sc2+sh2 | + res]) ------------------------------------------
__global__ void bn_apply_kernel(const __bf16* __restrict__ x, const float* __restrict__ sc,
                                const float* __restrict__ shf, const __bf16* __restrict__ x2,
                                const float* __restrict__ sc2, const float* __restrict__ shf2,
                                __bf16* __restrict__ y, int64_t nvec, int CV, int relu,
                                uint8_t* __restrict__ mbits) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nvec;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int cv = (int)(i % CV);
    float v[8];
    load8(x + i * 8, v);
    const f32x4 a0 = reinterpret_cast<const f32x4*>(sc)[cv * 2], a1 = reinterpret_cast<const f32x4*>(sc)[cv * 2 + 1];
    const f32x4 b0 = reinterpret_cast<const f32x4*>(shf)[cv * 2], b1 = reinterpret_cast<const f32x4*>(shf)[cv * 2 + 1];
    const float a[8] = {a0[0], a0[1], a0[2], a0[3], a1[0], a1[1], a1[2], a1[3]};
    const float b[8] = {b0[0], b0[1], b0[2], b0[3], b1[0], b1[1], b1[2], b1[3]};
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = v[e] * a[e] + b[e];
    if (x2) {
      float w[8];
      load8(x2 + i * 8, w);
      if (sc2) {
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] += w[e] * sc2[cv * 8 + e] + shf2[cv * 8 + e];
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] += w[e];
      }
    }
    if (relu) {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = fmaxf(v[e], 0.f);
    }
    u16x8 u;
#pragma unroll
    for (int e = 0; e < 8; ++e) u[e] = f2bf(v[e]);
    *reinterpret_cast<u16x8*>(y + i * 8) = u;
    if (mbits) {   // bit e = stored y[e] > 0 (sign clear, nonzero): the backward ReLU mask
      unsigned bits = 0;
#pragma unroll
      for (int e = 0; e < 8; ++e) bits |= ((u[e] & 0x8000u) == 0 && (u[e] & 0x7fffu) != 0) ? (1u << e) : 0u;
      mbits[i] = (uint8_t)bits;
    }
  }
}

// ---- backward reduce: partial sums of g and g*xhat (g = dy * (y>0) when y given) -------------
// Up to two BN layers (x/mean/invstd and x2/mean2/invstd2) that share the same g.
__global__ void bn_bwd_reduce_kernel(const __bf16* __restrict__ dy, const __bf16* __restrict__ ymask,
                                     const __bf16* __restrict__ x, const float* __restrict__ mean,
                                     const float* __restrict__ invstd, const __bf16* __restrict__ x2,
                                     const float* __restrict__ mean2, const float* __restrict__ invstd2,
                                     float* __restrict__ part, float* __restrict__ part2, int M, int C,
                                     int rows_per_block, RowMap rm) {
  extern __shared__ float sh[];  // [rpp][4][C]
  const int tid = threadIdx.x;
  const int tr = tid / rm.tpr, tc = tid % rm.tpr;
  const int r0 = blockIdx.x * rows_per_block;
  const int r1 = min(M, r0 + rows_per_block);
  const int NS = x2 ? 4 : 2;
  for (int k = 0; k < rm.vpt; ++k) {
    const int cv = tc + k * rm.tpr;
    float sg[8] = {0}, sgx[8] = {0}, sgx2[8] = {0};
    float mu[8], is[8], mu2[8], is2[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      mu[e] = mean[cv * 8 + e]; is[e] = invstd[cv * 8 + e];
      mu2[e] = x2 ? mean2[cv * 8 + e] : 0.f; is2[e] = x2 ? invstd2[cv * 8 + e] : 0.f;
    }
    for (int r = r0 + tr; r < r1; r += rm.rpp) {
      const size_t o = (size_t)r * C + cv * 8;
      float g[8], xv[8];
      load8(dy + o, g);
      if (ymask) {
        const u16x8 ym = *reinterpret_cast<const u16x8*>(ymask + o);
#pragma unroll
        for (int e = 0; e < 8; ++e) g[e] = (bf2f(ym[e]) > 0.f) ? g[e] : 0.f;
      }
      load8(x + o, xv);
#pragma unroll
      for (int e = 0; e < 8; ++e) { sg[e] += g[e]; sgx[e] += g[e] * (xv[e] - mu[e]) * is[e]; }
      if (x2) {
        load8(x2 + o, xv);
#pragma unroll
        for (int e = 0; e < 8; ++e) sgx2[e] += g[e] * (xv[e] - mu2[e]) * is2[e];
      }
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      sh[(tr * NS + 0) * C + cv * 8 + e] = sg[e];
      sh[(tr * NS + 1) * C + cv * 8 + e] = sgx[e];
      if (x2) sh[(tr * NS + 3) * C + cv * 8 + e] = sgx2[e];
    }
  }
  __syncthreads();
  for (int i = tid; i < 2 * C; i += blockDim.x) {
    const int which = i / C, c = i % C;
    float s = 0.f;
    for (int r = 0; r < rm.rpp; ++r) s += sh[(r * NS + which) * C + c];
    part[(size_t)blockIdx.x * 2 * C + i] = s;
    if (x2) {
      float s2 = 0.f;
      const int w2 = which == 0 ? 0 : 3;
      for (int r = 0; r < rm.rpp; ++r) s2 += sh[(r * NS + w2) * C + c];
      part2[(size_t)blockIdx.x * 2 * C + i] = s2;
    }
  }
}

// partials [T][2][C] -> dgamma/dbeta (written/accumulated into dgamma_out/dbeta_out, optional) and
// per-channel dx coefficients coef[3][C]: dx = k1*g + k2*x + k3
template <typename PT>
__global__ void bn_bwd_finalize_kernel(const PT* __restrict__ part, int T, int C, double count,
                                       const float* __restrict__ gamma, const float* __restrict__ mean,
                                       const float* __restrict__ invstd, float* __restrict__ dgamma_out,
                                       float* __restrict__ dbeta_out, int accumulate, float* __restrict__ coef) {
  __shared__ double sh[2][4][64];
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  const int g = threadIdx.x >> 6;
  double sg = 0, sgx = 0;
  if (c < C) {
    int t = g;
    for (; t + 12 < T; t += 16) {   // 4 rows x 2 sums of independent loads in flight
      PT a[4], b[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        a[u] = part[(size_t)(t + 4 * u) * 2 * C + c];
        b[u] = part[(size_t)(t + 4 * u) * 2 * C + C + c];
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) { sg += a[u]; sgx += b[u]; }
    }
    for (; t < T; t += 4) {
      sg += part[(size_t)t * 2 * C + c];
      sgx += part[(size_t)t * 2 * C + C + c];
    }
  }
  sh[0][g][threadIdx.x & 63] = sg;
  sh[1][g][threadIdx.x & 63] = sgx;
  __syncthreads();
  if (g == 0 && c < C) {
    for (int k = 1; k < 4; ++k) { sg += sh[0][k][threadIdx.x]; sgx += sh[1][k][threadIdx.x]; }
    bn_bwd_finalize_channel(c, sg, sgx, FinBwd{count, gamma, mean, invstd, dgamma_out, dbeta_out, accumulate, coef, C});
  }
}

// dx = k1*g + k2*x + k3 (g = dy*(y>0) if ymask); optional second BN (x2, coef2 -> dx2) sharing g;
// optional g_out (bf16) for the identity path of a residual block.
__global__ void bn_bwd_apply_kernel(const __bf16* __restrict__ dy, const __bf16* __restrict__ ymask,
                                    const __bf16* __restrict__ x, const float* __restrict__ coef,
                                    __bf16* __restrict__ dx, const __bf16* __restrict__ x2,
                                    const float* __restrict__ coef2, __bf16* __restrict__ dx2,
                                    __bf16* __restrict__ g_out, int64_t nvec, int CV) {
  const int C = CV * 8;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nvec;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int cv = (int)(i % CV);
    float g[8], xv[8], o[8];
    load8(dy + i * 8, g);
    if (ymask) {
      const u16x8 ym = *reinterpret_cast<const u16x8*>(ymask + i * 8);
#pragma unroll
      for (int e = 0; e < 8; ++e) g[e] = (bf2f(ym[e]) > 0.f) ? g[e] : 0.f;
    }
    if (g_out) store8(g_out + i * 8, g);
    load8(x + i * 8, xv);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int c = cv * 8 + e;
      o[e] = coef[c] * g[e] + coef[C + c] * xv[e] + coef[2 * C + c];
    }
    store8(dx + i * 8, o);
    if (x2) {
      load8(x2 + i * 8, xv);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int c = cv * 8 + e;
        o[e] = coef2[c] * g[e] + coef2[C + c] * xv[e] + coef2[2 * C + c];
      }
      store8(dx2 + i * 8, o);
    }
  }
}

// ---- v2 apply kernels (default): fixed channel group per thread, one wave of the whole tensor ---
// The grid's thread count T is a multiple of CV = C/8 (CV divides 256), so the 8-channel group
// i % CV of a thread is the same at every step of its walk: the per-channel coefficients are
// loaded ONCE into registers (v1 re-read them and did a 64-bit modulo per vector).  Measured
// (tools/ew_micro.py, profiles/r2_ew_apply_ab.txt, ResNet-50 B=256 shapes, in-process A/B): the
// best schedule is ONE 16-B vector per operand per thread over a grid that covers the tensor
// (U = 1, no block cap): 6.0-7.0 TB/s, 8 % less time than v1's 4096-block grid-stride loop and
// bitwise identical to it; U = 2/4 independent loads per thread or capped grids (2048-16384
// blocks) were slower, non-temporal stores made no difference.  Full groups of U run without
// bounds checks (a per-element guard would make hipcc wait vmcnt(0) per load); the tail is one
// guarded pass.
static Knob kn_bn_apply_v("bn_apply_v", 2);
static Knob kn_ew_unroll("ew_unroll", 1);
static Knob kn_ew_blocks("ew_blocks", 1 << 30);
static Knob kn_ew_nt("ew_nt", 0);   // 1: non-temporal (streaming) output stores

__device__ __forceinline__ void coef8(const float* p, int cv, float* d) {
  const f32x4 a0 = reinterpret_cast<const f32x4*>(p)[cv * 2], a1 = reinterpret_cast<const f32x4*>(p)[cv * 2 + 1];
  d[0] = a0[0]; d[1] = a0[1]; d[2] = a0[2]; d[3] = a0[3];
  d[4] = a1[0]; d[5] = a1[1]; d[6] = a1[2]; d[7] = a1[3];
}

// X2: 0 none, 1 plain residual add, 2 second BN branch (x2*sc2+sh2)
__device__ __forceinline__ void st16(__bf16* p, const u16x8& u, bool nt) {
  if (nt) __builtin_nontemporal_store(u, reinterpret_cast<u16x8*>(p));
  else *reinterpret_cast<u16x8*>(p) = u;
}
__device__ __forceinline__ void st8f(__bf16* p, const float* v, bool nt) {
  u16x8 u;
#pragma unroll
  for (int e = 0; e < 8; ++e) u[e] = f2bf(v[e]);
  st16(p, u, nt);
}

template <int U, int X2, bool RELU, bool MB, bool NT = false>
__global__ void __launch_bounds__(256) bn_apply_v2_kernel(const __bf16* __restrict__ x, const float* __restrict__ sc,
                                                          const float* __restrict__ shf, const __bf16* __restrict__ x2,
                                                          const float* __restrict__ sc2, const float* __restrict__ shf2,
                                                          __bf16* __restrict__ y, int nvec, int CV,
                                                          uint8_t* __restrict__ mbits) {
  const int T = gridDim.x * 256;
  const int tid = blockIdx.x * 256 + threadIdx.x;
  const int cv = tid % CV;
  float a[8], b[8], a2[8], b2[8];
  coef8(sc, cv, a);
  coef8(shf, cv, b);
  if constexpr (X2 == 2) { coef8(sc2, cv, a2); coef8(shf2, cv, b2); }
  auto body = [&](const u16x8& xv, const u16x8& wv, int i) {
    float v[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      v[e] = bf2f(xv[e]) * a[e] + b[e];
      if constexpr (X2 == 1) v[e] += bf2f(wv[e]);
      if constexpr (X2 == 2) v[e] += bf2f(wv[e]) * a2[e] + b2[e];
      if constexpr (RELU) v[e] = fmaxf(v[e], 0.f);
    }
    u16x8 u;
#pragma unroll
    for (int e = 0; e < 8; ++e) u[e] = f2bf(v[e]);
    st16(y + (size_t)i * 8, u, NT);
    if constexpr (MB) {
      unsigned bits = 0;
#pragma unroll
      for (int e = 0; e < 8; ++e) bits |= ((u[e] & 0x8000u) == 0 && (u[e] & 0x7fffu) != 0) ? (1u << e) : 0u;
      mbits[i] = (uint8_t)bits;
    }
  };
  int base = tid;
  for (; base + (U - 1) * T < nvec; base += U * T) {
    u16x8 xv[U], wv[U];
#pragma unroll
    for (int k = 0; k < U; ++k) xv[k] = *reinterpret_cast<const u16x8*>(x + (size_t)(base + k * T) * 8);
    if constexpr (X2 != 0) {
#pragma unroll
      for (int k = 0; k < U; ++k) wv[k] = *reinterpret_cast<const u16x8*>(x2 + (size_t)(base + k * T) * 8);
    }
#pragma unroll
    for (int k = 0; k < U; ++k) body(xv[k], wv[k], base + k * T);
  }
  for (int i = base; i < nvec; i += T) {
    const u16x8 xv = *reinterpret_cast<const u16x8*>(x + (size_t)i * 8);
    u16x8 wv{};
    if constexpr (X2 != 0) wv = *reinterpret_cast<const u16x8*>(x2 + (size_t)i * 8);
    body(xv, wv, i);
  }
}

template <int U, bool MASK, bool TWO, bool G, bool NT = false>
__global__ void __launch_bounds__(256) bn_bwd_apply_v2_kernel(const __bf16* __restrict__ dy, const __bf16* __restrict__ ymask,
                                                              const __bf16* __restrict__ x, const float* __restrict__ coef,
                                                              __bf16* __restrict__ dx, const __bf16* __restrict__ x2,
                                                              const float* __restrict__ coef2, __bf16* __restrict__ dx2,
                                                              __bf16* __restrict__ g_out, int nvec, int CV) {
  const int T = gridDim.x * 256;
  const int tid = blockIdx.x * 256 + threadIdx.x;
  const int cv = tid % CV;
  const int C = CV * 8;
  float k1[8], k2[8], k3[8], q1[8], q2[8], q3[8];
  coef8(coef, cv, k1); coef8(coef + C, cv, k2); coef8(coef + 2 * C, cv, k3);
  if constexpr (TWO) { coef8(coef2, cv, q1); coef8(coef2 + C, cv, q2); coef8(coef2 + 2 * C, cv, q3); }
  auto body = [&](const u16x8& gv, const u16x8& mv, const u16x8& xv, const u16x8& x2v, int i) {
    float g[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      g[e] = bf2f(gv[e]);
      if constexpr (MASK) g[e] = bf2f(mv[e]) > 0.f ? g[e] : 0.f;
    }
    if constexpr (G) {
      if constexpr (MASK) st8f(g_out + (size_t)i * 8, g, NT);
      else st16(g_out + (size_t)i * 8, gv, NT);
    }
    float o[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = k1[e] * g[e] + k2[e] * bf2f(xv[e]) + k3[e];
    st8f(dx + (size_t)i * 8, o, NT);
    if constexpr (TWO) {
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = q1[e] * g[e] + q2[e] * bf2f(x2v[e]) + q3[e];
      st8f(dx2 + (size_t)i * 8, o, NT);
    }
  };
  auto ld = [](const __bf16* p, int i) { return *reinterpret_cast<const u16x8*>(p + (size_t)i * 8); };
  int base = tid;
  for (; base + (U - 1) * T < nvec; base += U * T) {
    u16x8 gv[U], mv[U], xv[U], x2v[U];
#pragma unroll
    for (int k = 0; k < U; ++k) gv[k] = ld(dy, base + k * T);
    if constexpr (MASK) {
#pragma unroll
      for (int k = 0; k < U; ++k) mv[k] = ld(ymask, base + k * T);
    }
#pragma unroll
    for (int k = 0; k < U; ++k) xv[k] = ld(x, base + k * T);
    if constexpr (TWO) {
#pragma unroll
      for (int k = 0; k < U; ++k) x2v[k] = ld(x2, base + k * T);
    }
#pragma unroll
    for (int k = 0; k < U; ++k) body(gv[k], mv[k], xv[k], x2v[k], base + k * T);
  }
  for (int i = base; i < nvec; i += T) {
    u16x8 mv{}, x2v{};
    if constexpr (MASK) mv = ld(ymask, i);
    if constexpr (TWO) x2v = ld(x2, i);
    body(ld(dy, i), mv, ld(x, i), x2v, i);
  }
}

// grid for the v2 kernels: a multiple of 8 blocks (so the thread count is a multiple of CV <= 256)
static int ew2_blocks(int64_t nvec, int U) {
  const int cap = std::max(8, kn_ew_blocks.get() / 8 * 8);
  const int need = ceil_div(nvec, 256 * (int64_t)U);
  return std::max(8, std::min(cap, ceil_div(need, 8) * 8));
}
static bool ew2_ok(int CV, int64_t nvec) { return kn_bn_apply_v.get() == 2 && 256 % CV == 0 && nvec < (1ll << 31); }

template <int U>
static void launch_bn_apply_v2(const __bf16* x, const float* sc, const float* sh, const __bf16* x2, const float* sc2,
                               const float* sh2, __bf16* y, int64_t nvec, int CV, bool relu, uint8_t* mb,
                               hipStream_t st) {
  const int blocks = ew2_blocks(nvec, U);
  const int x2m = x2 ? (sc2 ? 2 : 1) : 0;
#define PCMP_BNA(X2, R, M)                                                                                      \
  do {                                                                                                        \
    if (kn_ew_nt.get())                                                                                       \
      hipLaunchKernelGGL((bn_apply_v2_kernel<U, X2, R, M, true>), dim3(blocks), dim3(256), 0, st, x, sc, sh, x2, \
                         sc2, sh2, y, (int)nvec, CV, mb);                                                     \
    else                                                                                                      \
      hipLaunchKernelGGL((bn_apply_v2_kernel<U, X2, R, M, false>), dim3(blocks), dim3(256), 0, st, x, sc, sh, x2, \
                         sc2, sh2, y, (int)nvec, CV, mb);                                                     \
  } while (0)
  if (x2m == 0) {
    if (relu) { if (mb) PCMP_BNA(0, true, true); else PCMP_BNA(0, true, false); }
    else { if (mb) PCMP_BNA(0, false, true); else PCMP_BNA(0, false, false); }
  } else if (x2m == 1) {
    if (relu) { if (mb) PCMP_BNA(1, true, true); else PCMP_BNA(1, true, false); }
    else { if (mb) PCMP_BNA(1, false, true); else PCMP_BNA(1, false, false); }
  } else {
    if (relu) { if (mb) PCMP_BNA(2, true, true); else PCMP_BNA(2, true, false); }
    else { if (mb) PCMP_BNA(2, false, true); else PCMP_BNA(2, false, false); }
  }
#undef PCMP_BNA
  PCMP_LAUNCH_CHECK();
}

template <int U>
static void launch_bn_bwd_apply_v2(const __bf16* dy, const __bf16* ym, const __bf16* x, const float* coef, __bf16* dx,
                                   const __bf16* x2, const float* coef2, __bf16* dx2, __bf16* g, int64_t nvec, int CV,
                                   hipStream_t st) {
  const int blocks = ew2_blocks(nvec, U);
#define PCMP_BBA(M, TW, G)                                                                                       \
  do {                                                                                                         \
    if (kn_ew_nt.get())                                                                                        \
      hipLaunchKernelGGL((bn_bwd_apply_v2_kernel<U, M, TW, G, true>), dim3(blocks), dim3(256), 0, st, dy, ym, x, coef, \
                         dx, x2, coef2, dx2, g, (int)nvec, CV);                                               \
    else                                                                                                       \
      hipLaunchKernelGGL((bn_bwd_apply_v2_kernel<U, M, TW, G, false>), dim3(blocks), dim3(256), 0, st, dy, ym, x,  \
                         coef, dx, x2, coef2, dx2, g, (int)nvec, CV);                                          \
  } while (0)
  const bool m = ym != nullptr, tw = x2 != nullptr, gg = g != nullptr;
  if (m) {
    if (tw) { if (gg) PCMP_BBA(true, true, true); else PCMP_BBA(true, true, false); }
    else { if (gg) PCMP_BBA(true, false, true); else PCMP_BBA(true, false, false); }
  } else {
    if (tw) { if (gg) PCMP_BBA(false, true, true); else PCMP_BBA(false, true, false); }
    else { if (gg) PCMP_BBA(false, false, true); else PCMP_BBA(false, false, false); }
  }
#undef PCMP_BBA
  PCMP_LAUNCH_CHECK();
}

// ------------------------------------------------------------------------------------------------
static int rows_per_block_for(int M, const RowMap& rm, int target_blocks = 2048) {
  int rpb = std::max(rm.rpp, ceil_div(M, target_blocks));
  rpb = ceil_div(rpb, rm.rpp) * rm.rpp;
  return rpb;
}

static void check_act(const at::Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kBFloat16 && t.is_contiguous(), name,
              ": contiguous bf16 GPU tensor expected");
  TORCH_CHECK(t.size(-1) % 8 == 0, name, ": channels must be a multiple of 8");
}

// x: [..., C] bf16 -> partial stats [T][2][C]
at::Tensor bn_partials(const at::Tensor& x) {
  if (x.scalar_type() == at::kFloat) return f32::bn_partials(x);
  check_act(x, "bn_partials");
  const int C = x.size(-1);
  const int M = x.numel() / C;
  const RowMap rm = make_rowmap(C);
  const int rpb = rows_per_block_for(M, rm);
  const int T = ceil_div(M, rpb);
  auto part = at::empty({T, 2, C}, x.options().dtype(at::kFloat));
  const size_t shm = (size_t)rm.rpp * 2 * C * sizeof(float);
  hipLaunchKernelGGL(bn_partials_kernel, dim3(T), dim3(256), shm, cur_stream(), ptr<__bf16>(x),
                     ptr<float>(part), M, C, rpb, rm);
  PCMP_LAUNCH_CHECK();
  return part;
}

// Reduce [T][2][C] f32 partials to at most ~64 rows of f64 when T is large (parallel stage 1).
static at::Tensor reduce_partials(const at::Tensor& part, int& T_out) {
  const int T = part.size(0), L = 2 * part.size(2);
  if (T <= 64) { T_out = T; return at::Tensor(); }
  const int rpb = std::max(16, ceil_div(T, 64));
  const int G = ceil_div(T, rpb);
  auto red = at::empty({G, L}, part.options().dtype(at::kDouble));
  hipLaunchKernelGGL(partials_reduce_kernel, dim3(ceil_div(L, 64), G), dim3(256), 0, cur_stream(), ptr<float>(part),
                     T, L, rpb, ptr<double>(red));
  PCMP_LAUNCH_CHECK();
  T_out = G;
  return red;
}

// Partial-row count up to which the finalize is one wide launch (knob bn_wide_rows; <= 64 rows the
// 256-thread finalize reads them directly, above bn_wide_rows the two-stage path runs).
static Knob kn_bn_wide_rows("bn_wide_rows", 512);
template <bool BWD, typename FA>
static bool wide_finalize(const at::Tensor& part, const FA& fa) {
  const int T = part.size(0), C = part.size(2);
  if (T <= 64) return false;
  if (T <= kn_bn_wide_rows.get()) {
    hipLaunchKernelGGL((bn_finalize_wide_kernel<float, BWD, FA>), dim3(ceil_div(C, 64)), dim3(1024), 0, cur_stream(),
                       ptr<float>(part), T, C, fa);
    PCMP_LAUNCH_CHECK();
    return true;
  }
  return false;
}

// partials -> (mean, invstd, scale, shift) ; updates running stats in place when given.
std::vector<at::Tensor> bn_finalize(const at::Tensor& part, int64_t count, const c10::optional<at::Tensor>& gamma,
                                    const c10::optional<at::Tensor>& beta,
                                    const c10::optional<at::Tensor>& running_mean,
                                    const c10::optional<at::Tensor>& running_var, double momentum, double eps) {
  const int T = part.size(0), C = part.size(2);
  auto opts = part.options().dtype(at::kFloat);
  auto out = at::empty({4, C}, opts);
  if (part.scalar_type() == at::kDouble) {   // pre-reduced (e.g. all-reduced SyncBN) fp64 sums
    TORCH_CHECK(part.is_contiguous(), "bn_finalize: contiguous partials");
    hipLaunchKernelGGL(bn_finalize_kernel<double>, dim3(ceil_div(C, 64)), dim3(256), 0, cur_stream(), ptr<double>(part),
                       T, C, (double)count, optr<float>(gamma), optr<float>(beta), optr<float>(running_mean),
                       optr<float>(running_var), (float)momentum, (float)eps, ptr<float>(out) + 0 * C,
                       ptr<float>(out) + 1 * C, ptr<float>(out) + 2 * C, ptr<float>(out) + 3 * C);
    PCMP_LAUNCH_CHECK();
    return {out[0], out[1], out[2], out[3]};
  }
  PCMP_CHECK_F32(part);
  TORCH_CHECK(part.is_contiguous(), "bn_finalize: contiguous partials");
  if (wide_finalize<false>(part, FinFwd{(double)count, optr<float>(gamma), optr<float>(beta), optr<float>(running_mean),
                                         optr<float>(running_var), (float)momentum, (float)eps, ptr<float>(out) + 0 * C,
                                         ptr<float>(out) + 1 * C, ptr<float>(out) + 2 * C, ptr<float>(out) + 3 * C}))
    return {out[0], out[1], out[2], out[3]};
  int T2;
  at::Tensor red = reduce_partials(part, T2);
  if (red.defined())
    hipLaunchKernelGGL(bn_finalize_kernel<double>, dim3(ceil_div(C, 64)), dim3(256), 0, cur_stream(), ptr<double>(red),
                       T2, C, (double)count, optr<float>(gamma), optr<float>(beta), optr<float>(running_mean),
                       optr<float>(running_var), (float)momentum, (float)eps, ptr<float>(out) + 0 * C,
                       ptr<float>(out) + 1 * C, ptr<float>(out) + 2 * C, ptr<float>(out) + 3 * C);
  else
    hipLaunchKernelGGL(bn_finalize_kernel<float>, dim3(ceil_div(C, 64)), dim3(256), 0, cur_stream(), ptr<float>(part),
                       T, C, (double)count, optr<float>(gamma), optr<float>(beta), optr<float>(running_mean),
                       optr<float>(running_var), (float)momentum, (float)eps, ptr<float>(out) + 0 * C,
                       ptr<float>(out) + 1 * C, ptr<float>(out) + 2 * C, ptr<float>(out) + 3 * C);
  PCMP_LAUNCH_CHECK();
  return {out[0], out[1], out[2], out[3]};
}

std::vector<at::Tensor> bn_eval_coeff(const c10::optional<at::Tensor>& gamma, const c10::optional<at::Tensor>& beta,
                                      const at::Tensor& running_mean, const at::Tensor& running_var, double eps) {
  const int C = running_mean.numel();
  auto out = at::empty({2, C}, running_mean.options());
  hipLaunchKernelGGL(bn_eval_coeff_kernel, dim3(ceil_div(C, 256)), dim3(256), 0, cur_stream(), C,
                     optr<float>(gamma), optr<float>(beta), ptr<float>(running_mean), ptr<float>(running_var),
                     (float)eps, ptr<float>(out), ptr<float>(out) + C);
  PCMP_LAUNCH_CHECK();
  return {out[0], out[1]};
}

static int ew_blocks(int64_t nvec) { return (int)std::min<int64_t>(4096, (nvec + 255) / 256); }

at::Tensor bn_apply(const at::Tensor& x, const at::Tensor& scale, const at::Tensor& shift,
                    const c10::optional<at::Tensor>& x2, const c10::optional<at::Tensor>& scale2,
                    const c10::optional<at::Tensor>& shift2, bool relu, const c10::optional<at::Tensor>& mbits) {
  if (x.scalar_type() == at::kFloat) return f32::bn_apply(x, scale, shift, x2, scale2, shift2, relu, mbits);
  check_act(x, "bn_apply");
  const int C = x.size(-1);
  auto y = at::empty_like(x);
  const int64_t nvec = x.numel() / 8;
  const __bf16* x2p = nullptr;
  if (x2.has_value() && x2->defined()) {
    check_act(*x2, "bn_apply x2");
    TORCH_CHECK(x2->numel() == x.numel(), "bn_apply: x2 shape");
    x2p = ptr<__bf16>(*x2);
  }
  uint8_t* mb = nullptr;
  if (mbits.has_value() && mbits->defined()) {
    TORCH_CHECK(mbits->scalar_type() == at::kByte && mbits->is_contiguous() && mbits->numel() == nvec,
                "bn_apply: mbits must be contiguous uint8 with one byte per 8 elements");
    mb = mbits->data_ptr<uint8_t>();
  }
  if (ew2_ok(C / 8, nvec)) {
    const int U = kn_ew_unroll.get();
    auto f = U >= 8 ? &launch_bn_apply_v2<8> : (U == 2 ? &launch_bn_apply_v2<2> : (U == 1 ? &launch_bn_apply_v2<1> : &launch_bn_apply_v2<4>));
    f(ptr<__bf16>(x), ptr<float>(scale), ptr<float>(shift), x2p, optr<float>(scale2), optr<float>(shift2),
      ptr<__bf16>(y), nvec, C / 8, relu, mb, cur_stream());
    return y;
  }
  hipLaunchKernelGGL(bn_apply_kernel, dim3(ew_blocks(nvec)), dim3(256), 0, cur_stream(), ptr<__bf16>(x),
                     ptr<float>(scale), ptr<float>(shift), x2p, optr<float>(scale2), optr<float>(shift2),
                     ptr<__bf16>(y), nvec, C / 8, (int)relu, mb);
  PCMP_LAUNCH_CHECK();
  return y;
}

// returns partials for BN1 (and BN2 when x2 given)
std::vector<at::Tensor> bn_bwd_reduce(const at::Tensor& dy, const c10::optional<at::Tensor>& ymask,
                                      const at::Tensor& x, const at::Tensor& mean, const at::Tensor& invstd,
                                      const c10::optional<at::Tensor>& x2, const c10::optional<at::Tensor>& mean2,
                                      const c10::optional<at::Tensor>& invstd2) {
  if (dy.scalar_type() == at::kFloat) return f32::bn_bwd_reduce(dy, ymask, x, mean, invstd, x2, mean2, invstd2);
  check_act(dy, "bn_bwd dy");
  check_act(x, "bn_bwd x");
  const int C = x.size(-1);
  const int M = x.numel() / C;
  const RowMap rm = make_rowmap(C);
  const int rpb = rows_per_block_for(M, rm);
  const int T = ceil_div(M, rpb);
  auto part = at::empty({T, 2, C}, x.options().dtype(at::kFloat));
  const bool two = x2.has_value() && x2->defined();
  at::Tensor part2 = two ? at::empty({T, 2, C}, part.options()) : at::Tensor();
  const size_t shm = (size_t)rm.rpp * (two ? 4 : 2) * C * sizeof(float);
  hipLaunchKernelGGL(bn_bwd_reduce_kernel, dim3(T), dim3(256), shm, cur_stream(), ptr<__bf16>(dy),
                     optr<__bf16>(ymask), ptr<__bf16>(x), ptr<float>(mean), ptr<float>(invstd),
                     two ? ptr<__bf16>(*x2) : nullptr, optr<float>(mean2), optr<float>(invstd2), ptr<float>(part),
                     two ? ptr<float>(part2) : nullptr, M, C, rpb, rm);
  PCMP_LAUNCH_CHECK();
  if (two) return {part, part2};
  return {part};
}

// returns coef [3][C]; writes dgamma/dbeta into the given fp32 buffers (flat grad views)
at::Tensor bn_bwd_finalize(const at::Tensor& part, int64_t count, const c10::optional<at::Tensor>& gamma,
                           const at::Tensor& mean, const at::Tensor& invstd,
                           const c10::optional<at::Tensor>& dgamma, const c10::optional<at::Tensor>& dbeta,
                           bool accumulate) {
  const int T = part.size(0), C = part.size(2);
  auto coef = at::empty({3, C}, part.options().dtype(at::kFloat));
  if (part.scalar_type() == at::kDouble) {   // pre-reduced (e.g. all-reduced SyncBN) fp64 sums
    TORCH_CHECK(part.is_contiguous(), "bn_bwd_finalize: contiguous partials");
    hipLaunchKernelGGL(bn_bwd_finalize_kernel<double>, dim3(ceil_div(C, 64)), dim3(256), 0, cur_stream(),
                       ptr<double>(part), T, C, (double)count, optr<float>(gamma), ptr<float>(mean), ptr<float>(invstd),
                       optr<float>(dgamma), optr<float>(dbeta), (int)accumulate, ptr<float>(coef));
    PCMP_LAUNCH_CHECK();
    return coef;
  }
  PCMP_CHECK_F32(part);
  TORCH_CHECK(part.is_contiguous(), "bn_bwd_finalize: contiguous partials");
  if (wide_finalize<true>(part, FinBwd{(double)count, optr<float>(gamma), ptr<float>(mean), ptr<float>(invstd),
                                        optr<float>(dgamma), optr<float>(dbeta), (int)accumulate, ptr<float>(coef), C}))
    return coef;
  int T2;
  at::Tensor red = reduce_partials(part, T2);
  if (red.defined())
    hipLaunchKernelGGL(bn_bwd_finalize_kernel<double>, dim3(ceil_div(C, 64)), dim3(256), 0, cur_stream(),
                       ptr<double>(red), T2, C, (double)count, optr<float>(gamma), ptr<float>(mean), ptr<float>(invstd),
                       optr<float>(dgamma), optr<float>(dbeta), (int)accumulate, ptr<float>(coef));
  else
    hipLaunchKernelGGL(bn_bwd_finalize_kernel<float>, dim3(ceil_div(C, 64)), dim3(256), 0, cur_stream(),
                       ptr<float>(part), T, C, (double)count, optr<float>(gamma), ptr<float>(mean), ptr<float>(invstd),
                       optr<float>(dgamma), optr<float>(dbeta), (int)accumulate, ptr<float>(coef));
  PCMP_LAUNCH_CHECK();
  return coef;
}

// returns [dx] (+ dx2) (+ g)
std::vector<at::Tensor> bn_bwd_apply(const at::Tensor& dy, const c10::optional<at::Tensor>& ymask,
                                     const at::Tensor& x, const at::Tensor& coef,
                                     const c10::optional<at::Tensor>& x2, const c10::optional<at::Tensor>& coef2,
                                     bool want_g) {
  if (dy.scalar_type() == at::kFloat) return f32::bn_bwd_apply(dy, ymask, x, coef, x2, coef2, want_g);
  check_act(dy, "bn_bwd_apply dy");
  const int C = x.size(-1);
  auto dx = at::empty_like(x);
  const bool two = x2.has_value() && x2->defined();
  at::Tensor dx2 = two ? at::empty_like(*x2) : at::Tensor();
  at::Tensor g = want_g ? at::empty_like(dy) : at::Tensor();
  const int64_t nvec = x.numel() / 8;
  if (ew2_ok(C / 8, nvec)) {
    const int U = kn_ew_unroll.get();
    auto f = U >= 8 ? &launch_bn_bwd_apply_v2<8> : (U == 2 ? &launch_bn_bwd_apply_v2<2> : (U == 1 ? &launch_bn_bwd_apply_v2<1> : &launch_bn_bwd_apply_v2<4>));
    f(ptr<__bf16>(dy), optr<__bf16>(ymask), ptr<__bf16>(x), ptr<float>(coef), ptr<__bf16>(dx),
      two ? ptr<__bf16>(*x2) : nullptr, optr<float>(coef2), two ? ptr<__bf16>(dx2) : nullptr,
      want_g ? ptr<__bf16>(g) : nullptr, nvec, C / 8, cur_stream());
    std::vector<at::Tensor> r{dx};
    if (two) r.push_back(dx2);
    if (want_g) r.push_back(g);
    return r;
  }
  hipLaunchKernelGGL(bn_bwd_apply_kernel, dim3(ew_blocks(nvec)), dim3(256), 0, cur_stream(), ptr<__bf16>(dy),
                     optr<__bf16>(ymask), ptr<__bf16>(x), ptr<float>(coef), ptr<__bf16>(dx),
                     two ? ptr<__bf16>(*x2) : nullptr, optr<float>(coef2), two ? ptr<__bf16>(dx2) : nullptr,
                     want_g ? ptr<__bf16>(g) : nullptr, nvec, C / 8);
  PCMP_LAUNCH_CHECK();
  std::vector<at::Tensor> r{dx};
  if (two) r.push_back(dx2);
  if (want_g) r.push_back(g);
  return r;
}

}  // namespace pcmp

TORCH_LIBRARY_FRAGMENT(pcmp, m) {
  m.def("bn_partials(Tensor x) -> Tensor", &pcmp::bn_partials);
  m.def("bn_finalize(Tensor part, int count, Tensor? gamma, Tensor? beta, Tensor(a!)? running_mean, "
        "Tensor(b!)? running_var, float momentum, float eps) -> Tensor[]",
        &pcmp::bn_finalize);
  m.def("bn_eval_coeff(Tensor? gamma, Tensor? beta, Tensor running_mean, Tensor running_var, float eps) -> Tensor[]",
        &pcmp::bn_eval_coeff);
  m.def("bn_apply(Tensor x, Tensor scale, Tensor shift, Tensor? x2, Tensor? scale2, Tensor? shift2, bool relu, "
        "Tensor(a!)? mbits=None) -> Tensor",
        &pcmp::bn_apply);
  m.def("bn_bwd_reduce(Tensor dy, Tensor? ymask, Tensor x, Tensor mean, Tensor invstd, Tensor? x2, Tensor? mean2, "
        "Tensor? invstd2) -> Tensor[]",
        &pcmp::bn_bwd_reduce);
  m.def("bn_bwd_finalize(Tensor part, int count, Tensor? gamma, Tensor mean, Tensor invstd, Tensor(a!)? dgamma, "
        "Tensor(b!)? dbeta, bool accumulate) -> Tensor",
        &pcmp::bn_bwd_finalize);
  m.def("bn_bwd_apply(Tensor dy, Tensor? ymask, Tensor x, Tensor coef, Tensor? x2, Tensor? coef2, bool want_g) -> Tensor[]",
        &pcmp::bn_bwd_apply);
}

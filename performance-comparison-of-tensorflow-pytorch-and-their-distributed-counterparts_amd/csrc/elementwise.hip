// Pooling, loss, dropout, activation-backward, bias-gradient and input-conversion kernels (NHWC,
// bf16, 16-B vectors over channels).
//
// Reference parity:
//   * MaxPool2d(3,2,1) of the ResNet stem and the 5 MaxPool2d(2,2) of VGG16
//     (pytorch_training_inference_on_image.ipynb:458,1991-2041)
//   * AdaptiveAvgPool2d(1) (ResNet) — global average pool
//   * LogSoftmax(dim=1) + NLLLoss of the transfer heads (another_neural_net.py:108-113,250-257)
//     and CrossEntropy of BertForSequenceClassification — one fused row kernel
//   * Dropout(0.2/0.4/0.5/0.1) — counter-based hash RNG, mask regenerated in backward
//   * ToTensor/normalise of the image pipeline — fused NCHW f32/u8 -> NHWC bf16
//     with zero channel padding to a multiple of 8 (the stem conv's MFMA K granularity)
#include <type_traits>
#include "common.h"
#include "f32.h"

#include <climits>
#include <mutex>
#include <string>
#include <vector>

namespace pcmp {

__device__ __forceinline__ void ld8(const __bf16* p, float* v) {
  const u16x8 u = *reinterpret_cast<const u16x8*>(p);
#pragma unroll
  for (int e = 0; e < 8; ++e) v[e] = bf2f(u[e]);
}
__device__ __forceinline__ void st8(__bf16* p, const float* v) {
  u16x8 u;
#pragma unroll
  for (int e = 0; e < 8; ++e) u[e] = f2bf(v[e]);
  *reinterpret_cast<u16x8*>(p) = u;
}
static int grid_for(int64_t n, int block = 256, int cap = 4096) {
  return (int)std::max<int64_t>(1, std::min<int64_t>(cap, (n + block - 1) / block));
}

// ---------------------------------------------------------------- max pool (NHWC) -------------
// y[n,p,q,c] = max over window; idx[n,p,q,c] = argmax position inside the window (uint8)
// Optional fused BatchNorm(+ReLU) prologue (sc/sh non-null): the pooled value is
// bf16(relu(x * sc + sh)), exactly what a separate bn_apply would have stored -- the stem's
// normalised activation is never written (ResNet stem: conv -> BN -> ReLU -> maxpool).
__global__ void maxpool_fwd_kernel(const __bf16* __restrict__ x, __bf16* __restrict__ y,
                                   uint8_t* __restrict__ idx, int N, int H, int W, int C, int P, int Q,
                                   int k, int s, int pad, const float* __restrict__ sc,
                                   const float* __restrict__ sh) {
  const int CV = C / 8;
  const int64_t total = (int64_t)N * P * Q * CV;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int cv = i % CV;
    int64_t t = i / CV;
    const int q = t % Q; t /= Q;
    const int p = t % P;
    const int n = t / P;
    float best[8], a[8], b[8];
    int bi[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      best[e] = -INFINITY; bi[e] = 0;
      a[e] = sc ? sc[cv * 8 + e] : 1.f;
      b[e] = sc ? sh[cv * 8 + e] : 0.f;
    }
    for (int r = 0; r < k; ++r) {
      const int h = p * s - pad + r;
      if ((unsigned)h >= (unsigned)H) continue;
      for (int c = 0; c < k; ++c) {
        const int w = q * s - pad + c;
        if ((unsigned)w >= (unsigned)W) continue;
        float v[8];
        ld8(x + (((size_t)n * H + h) * W + w) * C + cv * 8, v);
        if (sc) {
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = bf2f(f2bf(fmaxf(v[e] * a[e] + b[e], 0.f)));
        }
#pragma unroll
        for (int e = 0; e < 8; ++e)
          if (v[e] > best[e] || (v[e] != v[e])) { best[e] = v[e]; bi[e] = r * k + c; }
      }
    }
    st8(y + i * 8, best);
    if (idx) {
      uint64_t packed = 0;
#pragma unroll
      for (int e = 0; e < 8; ++e) packed |= (uint64_t)(bi[e] & 0xff) << (8 * e);
      *reinterpret_cast<uint64_t*>(idx + i * 8) = packed;
    }
  }
}

// The ResNet stem's 3x3 / stride-2 / pad-1 pooling (B=256: 411 MB in, 154 MB out), one thread per
// (output pixel, 8-channel vector), 32-bit index math, all nine window loads issued before any is
// consumed (out-of-image taps read a clamped in-image address and are skipped in the fold).  The
// generic kernel above spends its time in 64-bit divisions and a data-dependent tap loop that
// serialises the loads: 212 us -> see profiles/r2_pool_ab.txt.  Fold order, NaN and tie handling
// are the generic kernel's, so values and argmax indices are identical.
__global__ void __launch_bounds__(256) maxpool3s2_fwd_kernel(const __bf16* __restrict__ x, __bf16* __restrict__ y,
                                                             uint8_t* __restrict__ idx, unsigned total, int H, int W,
                                                             int CV, int P, int Q, const float* __restrict__ sc,
                                                             const float* __restrict__ sh) {
  const unsigned i = blockIdx.x * 256u + threadIdx.x;
  if (i >= total) return;
  const unsigned cv = i % (unsigned)CV, pix = i / (unsigned)CV;
  const unsigned q = pix % (unsigned)Q, t = pix / (unsigned)Q;
  const unsigned p = t % (unsigned)P, n = t / (unsigned)P;
  const int C = CV * 8;
  u16x8 raw[9];
  bool ok[9];
#pragma unroll
  for (int r = 0; r < 3; ++r) {
    const int h = 2 * (int)p - 1 + r;
    const bool hok = (unsigned)h < (unsigned)H;
    const int hc = hok ? h : 0;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const int w = 2 * (int)q - 1 + c;
      const bool wok = (unsigned)w < (unsigned)W;
      ok[r * 3 + c] = hok && wok;
      raw[r * 3 + c] = *reinterpret_cast<const u16x8*>(x + ((n * H + hc) * W + (wok ? w : 0)) * (unsigned)C + cv * 8);
    }
  }
  float best[8], a[8], b[8];
  int bi[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    best[e] = -INFINITY; bi[e] = 0;
    a[e] = sc ? sc[cv * 8 + e] : 1.f;
    b[e] = sc ? sh[cv * 8 + e] : 0.f;
  }
#pragma unroll
  for (int j = 0; j < 9; ++j) {
    if (!ok[j]) continue;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float v = bf2f(raw[j][e]);
      if (sc) v = bf2f(f2bf(fmaxf(v * a[e] + b[e], 0.f)));
      if (v > best[e] || (v != v)) { best[e] = v; bi[e] = j; }
    }
  }
  st8(y + (size_t)i * 8, best);
  if (idx) {
    uint64_t packed = 0;
#pragma unroll
    for (int e = 0; e < 8; ++e) packed |= (uint64_t)(bi[e] & 0xff) << (8 * e);
    *reinterpret_cast<uint64_t*>(idx + (size_t)i * 8) = packed;
  }
}

// gather-form backward: dx[n,h,w,c] = sum of dy over the windows whose argmax is (h,w)
__global__ void maxpool_bwd_kernel(const __bf16* __restrict__ dy, const uint8_t* __restrict__ idx,
                                   __bf16* __restrict__ dx, int N, int H, int W, int C, int P, int Q,
                                   int k, int s, int pad) {
  const int CV = C / 8;
  const int64_t total = (int64_t)N * H * W * CV;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int cv = i % CV;
    int64_t t = i / CV;
    const int w = t % W; t /= W;
    const int h = t % H;
    const int n = t / H;
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    // candidate output rows p with p*s - pad <= h <= p*s - pad + k - 1
    const int p_lo = max(0, (h + pad - k + s) / s), p_hi = min(P - 1, (h + pad) / s);
    const int q_lo = max(0, (w + pad - k + s) / s), q_hi = min(Q - 1, (w + pad) / s);
    for (int p = p_lo; p <= p_hi; ++p) {
      const int r = h - (p * s - pad);
      if (r < 0 || r >= k) continue;
      for (int q = q_lo; q <= q_hi; ++q) {
        const int c = w - (q * s - pad);
        if (c < 0 || c >= k) continue;
        const size_t o = (((size_t)n * P + p) * Q + q) * C + cv * 8;
        const uint64_t packed = *reinterpret_cast<const uint64_t*>(idx + o);
        float g[8];
        ld8(dy + o, g);
        const int pos = r * k + c;
#pragma unroll
        for (int e = 0; e < 8; ++e)
          if ((int)((packed >> (8 * e)) & 0xff) == pos) acc[e] += g[e];
      }
    }
    st8(dx + i * 8, acc);
  }
}

// Stem backward fused: gather-form maxpool backward + ReLU mask recomputed from the pre-BN input
// c (relu(c * sc + sh) > 0) + the BatchNorm-backward partial sums of that BN, per block of rows:
// writes g = bf16(sum of dy over the windows whose argmax is the pixel) * mask and part [T][2][C]
// = (sum g, sum g * (c - mean) * invstd).  Replaces maxpool_bwd + bn_bwd_reduce (which re-read the
// gradient and the normalised activation).  Block = 256 threads = rpp pixel rows x tpr channel
// vectors (C/8 <= 256).  K3S2: the stem's 3x3 / stride-2 / pad-1 window, where input pixel (h, w)
// lies in output rows p = h/2 .. (h+1)/2 and columns q = w/2 .. (w+1)/2 (1-4 windows, r and c
// always in range): the candidate loads are issued together, branch-free, and folded in the
// generic kernel's (p, q) order, so the sums are bitwise the same.
template <bool K3S2>
__global__ void __launch_bounds__(256) maxpool_bwd_bnr_kernel(const __bf16* __restrict__ dy, const uint8_t* __restrict__ idx,
                                       const __bf16* __restrict__ cx, const float* __restrict__ mean,
                                       const float* __restrict__ invstd, const float* __restrict__ sc,
                                       const float* __restrict__ sh, __bf16* __restrict__ g_out,
                                       float* __restrict__ part, int N, int H, int W, int C, int P, int Q, int k,
                                       int s, int pad, int rows_per_block) {
  extern __shared__ float red[];   // [rpp][2][C]
  const int CV = C / 8;
  const int tpr = CV, rpp = 256 / CV;
  const int tid = threadIdx.x;
  const int tr = tid / tpr, cv = tid % tpr;
  const int M = N * H * W;
  const int r0 = blockIdx.x * rows_per_block, r1 = min(M, r0 + rows_per_block);
  float sg[8] = {0, 0, 0, 0, 0, 0, 0, 0}, sgx[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  float mu[8], is[8], a[8], b[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    mu[e] = mean[cv * 8 + e]; is[e] = invstd[cv * 8 + e];
    a[e] = sc[cv * 8 + e]; b[e] = sh[cv * 8 + e];
  }
  if (tr < rpp) {
#pragma unroll 2
    for (int row = r0 + tr; row < r1; row += rpp) {
      const int w = (unsigned)row % (unsigned)W;
      const int t = (unsigned)row / (unsigned)W;
      const int h = (unsigned)t % (unsigned)H;
      const int n = (unsigned)t / (unsigned)H;
      float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
      if constexpr (K3S2) {
        const int p0 = h >> 1, q0 = w >> 1;
        const int p1 = min(P - 1, (h + 1) >> 1), q1 = min(Q - 1, (w + 1) >> 1);
        const int pp[4] = {p0, p0, p1, p1}, qq[4] = {q0, q1, q0, q1};
        const bool use[4] = {true, q1 != q0, p1 != p0, p1 != p0 && q1 != q0};
        uint64_t pk[4];
        u16x8 gv[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const unsigned o = (((unsigned)n * P + pp[j]) * Q + qq[j]) * (unsigned)C + cv * 8;
          pk[j] = *reinterpret_cast<const uint64_t*>(idx + o);
          gv[j] = *reinterpret_cast<const u16x8*>(dy + o);
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          if (!use[j]) continue;
          const int pos = (h - (2 * pp[j] - 1)) * 3 + (w - (2 * qq[j] - 1));
#pragma unroll
          for (int e = 0; e < 8; ++e)
            if ((int)((pk[j] >> (8 * e)) & 0xff) == pos) acc[e] += bf2f(gv[j][e]);
        }
      } else {
      const int p_lo = max(0, (h + pad - k + s) / s), p_hi = min(P - 1, (h + pad) / s);
      const int q_lo = max(0, (w + pad - k + s) / s), q_hi = min(Q - 1, (w + pad) / s);
      for (int p = p_lo; p <= p_hi; ++p) {
        const int r = h - (p * s - pad);
        if (r < 0 || r >= k) continue;
        for (int q = q_lo; q <= q_hi; ++q) {
          const int c = w - (q * s - pad);
          if (c < 0 || c >= k) continue;
          const size_t o = (((size_t)n * P + p) * Q + q) * C + cv * 8;
          const uint64_t packed = *reinterpret_cast<const uint64_t*>(idx + o);
          float gg[8];
          ld8(dy + o, gg);
          const int pos = r * k + c;
#pragma unroll
          for (int e = 0; e < 8; ++e)
            if ((int)((packed >> (8 * e)) & 0xff) == pos) acc[e] += gg[e];
        }
      }
      }
      const size_t oi = (size_t)row * C + cv * 8;
      float xv[8];
      ld8(cx + oi, xv);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float gr = bf2f(f2bf(acc[e]));
        acc[e] = (xv[e] * a[e] + b[e] > 0.f) ? gr : 0.f;
        sg[e] += acc[e];
        sgx[e] += acc[e] * (xv[e] - mu[e]) * is[e];
      }
      st8(g_out + oi, acc);
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      red[(tr * 2 + 0) * C + cv * 8 + e] = sg[e];
      red[(tr * 2 + 1) * C + cv * 8 + e] = sgx[e];
    }
  }
  __syncthreads();
  for (int i = tid; i < 2 * C; i += blockDim.x) {
    const int which = i / C, c = i % C;
    float t = 0.f;
    for (int r = 0; r < rpp; ++r) t += red[(r * 2 + which) * C + c];
    part[(size_t)blockIdx.x * 2 * C + i] = t;
  }
}

// Stem backward fused, 2x2-quad form (even H, W; 3x3 / stride-2 / pad-1 window): a thread owns the
// input pixels (2a + dh, 2b + dw) of one quad x 8 channels.  The four pixels share the pooled
// windows (a, b), (a, b+1), (a+1, b), (a+1, b+1), so those are loaded once per quad (4 dy + 4 argmax
// loads for 4 pixels instead of 4 per pixel); each pixel folds its windows in the per-pixel kernel's
// order, so g is bitwise that kernel's; the partial sums come in another order (knob pool_quad).
__global__ void __launch_bounds__(256) maxpool_bwd_bnr_quad_kernel(
    const __bf16* __restrict__ dy, const uint8_t* __restrict__ idx, const __bf16* __restrict__ cx,
    const float* __restrict__ mean, const float* __restrict__ invstd, const float* __restrict__ sc,
    const float* __restrict__ sh, __bf16* __restrict__ g_out, float* __restrict__ part, int N, int H, int W, int C,
    int P, int Q, int quads_per_block) {
  extern __shared__ float red[];   // [rpp][2][C]
  const int CV = C / 8;
  const int tpr = CV, rpp = 256 / CV;
  const int tid = threadIdx.x;
  const int tr = tid / tpr, cv = tid % tpr;
  const int H2 = H >> 1, W2 = W >> 1;
  const int MQ = N * H2 * W2;
  const int r0 = blockIdx.x * quads_per_block, r1 = min(MQ, r0 + quads_per_block);
  float sg[8] = {0, 0, 0, 0, 0, 0, 0, 0}, sgx[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  float mu[8], is[8], a[8], b[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    mu[e] = mean[cv * 8 + e]; is[e] = invstd[cv * 8 + e];
    a[e] = sc[cv * 8 + e]; b[e] = sh[cv * 8 + e];
  }
  if (tr < rpp) {
    for (int qd = r0 + tr; qd < r1; qd += rpp) {
      const int qb = (unsigned)qd % (unsigned)W2;
      const int t = (unsigned)qd / (unsigned)W2;
      const int qa = (unsigned)t % (unsigned)H2;
      const int n = (unsigned)t / (unsigned)H2;
      const int pa1 = min(P - 1, qa + 1), qb1 = min(Q - 1, qb + 1);
      const int pp[4] = {qa, qa, pa1, pa1}, qq[4] = {qb, qb1, qb, qb1};
      uint64_t pk[4];
      u16x8 gv[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const unsigned o = (((unsigned)n * P + pp[j]) * Q + qq[j]) * (unsigned)C + cv * 8;
        pk[j] = *reinterpret_cast<const uint64_t*>(idx + o);
        gv[j] = *reinterpret_cast<const u16x8*>(dy + o);
      }
      float xv[4][8];
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        const int h = 2 * qa + (d >> 1), w = 2 * qb + (d & 1);
        ld8(cx + ((size_t)((unsigned)n * H + h) * W + w) * C + cv * 8, xv[d]);
      }
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        const int dh = d >> 1, dw = d & 1;
        const int h = 2 * qa + dh, w = 2 * qb + dw;
        // this pixel's windows, in the per-pixel kernel's (p0, q0), (p0, q1), (p1, q0), (p1, q1) order:
        // p1 = min(P-1, (h+1)/2) is qa+1 only for odd h, q1 likewise
        const int p1 = dh ? pa1 : qa, q1 = dw ? qb1 : qb;
        const bool use[4] = {true, q1 != qb, p1 != qa, p1 != qa && q1 != qb};
        const int jj[4] = {0, dw ? 1 : 0, dh ? 2 : 0, (dh && dw) ? 3 : 0};
        float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          if (!use[k]) continue;
          const int j = jj[k];
          const int pos = (h - (2 * pp[j] - 1)) * 3 + (w - (2 * qq[j] - 1));
#pragma unroll
          for (int e = 0; e < 8; ++e)
            if ((int)((pk[j] >> (8 * e)) & 0xff) == pos) acc[e] += bf2f(gv[j][e]);
        }
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float gr = bf2f(f2bf(acc[e]));
          acc[e] = (xv[d][e] * a[e] + b[e] > 0.f) ? gr : 0.f;
          sg[e] += acc[e];
          sgx[e] += acc[e] * (xv[d][e] - mu[e]) * is[e];
        }
        st8(g_out + ((size_t)((unsigned)n * H + h) * W + w) * C + cv * 8, acc);
      }
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      red[(tr * 2 + 0) * C + cv * 8 + e] = sg[e];
      red[(tr * 2 + 1) * C + cv * 8 + e] = sgx[e];
    }
  }
  __syncthreads();
  for (int i = tid; i < 2 * C; i += blockDim.x) {
    const int which = i / C, c = i % C;
    float t = 0.f;
    for (int r = 0; r < rpp; ++r) t += red[(r * 2 + which) * C + c];
    part[(size_t)blockIdx.x * 2 * C + i] = t;
  }
}

// ---------------------------------------------------------------- global average pool ----------
// x [N, HW, C] -> y [N, C]  (one block per (n, 64*8-channel slab))
__global__ void gap_fwd_kernel(const __bf16* __restrict__ x, __bf16* __restrict__ y, int HW, int C) {
  const int n = blockIdx.y;
  const int CV = C / 8;
  const int cv = blockIdx.x * 64 + (threadIdx.x & 63);
  const int g = threadIdx.x >> 6;  // 4 row groups
  __shared__ float sh[4][64][8];
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (cv < CV) {
    for (int r = g; r < HW; r += 4) {
      float v[8];
      ld8(x + ((size_t)n * HW + r) * C + cv * 8, v);
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] += v[e];
    }
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) sh[g][threadIdx.x & 63][e] = acc[e];
  __syncthreads();
  if (g == 0 && cv < CV) {
    const float inv = 1.f / HW;
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] = (acc[e] + sh[1][threadIdx.x][e] + sh[2][threadIdx.x][e] + sh[3][threadIdx.x][e]) * inv;
    st8(y + (size_t)n * C + cv * 8, acc);
  }
}

__global__ void gap_bwd_kernel(const __bf16* __restrict__ dy, __bf16* __restrict__ dx, int N, int HW, int C) {
  const int CV = C / 8;
  const int64_t total = (int64_t)N * HW * CV;
  const float inv = 1.f / HW;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int cv = i % CV;
    const int n = (int)(i / ((int64_t)HW * CV));
    float v[8];
    ld8(dy + (size_t)n * C + cv * 8, v);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] *= inv;
    st8(dx + i * 8, v);
  }
}

// ---------------------------------------------------------------- softmax cross-entropy --------
// one wave per row: logits [B][V] (bf16 or f32) -> logp (f32, optional), dlogits (bf16/f32,
// optional, = (softmax - onehot) * grad_scale), per-row loss (f32) -> loss_rows[B]
template <typename T>
__device__ __forceinline__ float ldv(const T* p, int i);
template <>
__device__ __forceinline__ float ldv<float>(const float* p, int i) { return p[i]; }
template <>
__device__ __forceinline__ float ldv<__bf16>(const __bf16* p, int i) {
  return bf2f(reinterpret_cast<const unsigned short*>(p)[i]);
}

template <typename T>
__global__ void xent_kernel(const T* __restrict__ logits, const int64_t* __restrict__ labels, int B, int V,
                            float* __restrict__ logp, T* __restrict__ dlogits, float* __restrict__ loss_rows,
                            float grad_scale, int ignore_index) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (row >= B) return;
  const T* z = logits + (size_t)row * V;
  float mx = -INFINITY;
  for (int i = lane; i < V; i += 64) mx = fmaxf(mx, ldv<T>(z, i));
  mx = warp_max(mx);
  float se = 0.f;
  for (int i = lane; i < V; i += 64) se += __expf(ldv<T>(z, i) - mx);
  se = warp_sum(se);
  const float lse = mx + __logf(se);
  const int64_t y = labels ? labels[row] : -1;
  const bool valid = labels && y != ignore_index && y >= 0 && y < V;
  if (logp)
    for (int i = lane; i < V; i += 64) logp[(size_t)row * V + i] = ldv<T>(z, i) - lse;
  if (dlogits) {
    for (int i = lane; i < V; i += 64) {
      float g = valid ? (__expf(ldv<T>(z, i) - lse) - (i == y ? 1.f : 0.f)) * grad_scale : 0.f;
      if constexpr (std::is_same<T, float>::value) dlogits[(size_t)row * V + i] = g;
      else reinterpret_cast<unsigned short*>(dlogits)[(size_t)row * V + i] = f2bf(g);
    }
  }
  if (lane == 0 && loss_rows) loss_rows[row] = valid ? (lse - ldv<T>(z, (int)y)) : 0.f;
}


// ---------------------------------------------------------------- loss mean / grad scale --------
// mean over valid rows of the per-row losses (one workgroup, fixed summation order: deterministic):
// out[0] = sum(loss_rows) / max(1, valid), out[1] = valid (row count whose label is not ignored).
// Replaces the sum / count / clamp / divide torch launches of the cross-entropy forward.
__global__ __launch_bounds__(256) void loss_mean_kernel(const float* __restrict__ loss_rows,
                                                        const int64_t* __restrict__ labels, int B, int V,
                                                        int ignore_index, float* __restrict__ out) {
  __shared__ float sh[2][4];
  float s = 0.f, c = 0.f;
  for (int i = threadIdx.x; i < B; i += 256) {
    s += loss_rows[i];
    const int64_t y = labels[i];
    c += (y != ignore_index && y >= 0 && y < V) ? 1.f : 0.f;
  }
  s = warp_sum(s);
  c = warp_sum(c);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) { sh[0][w] = s; sh[1][w] = c; }
  __syncthreads();
  if (threadIdx.x == 0) {
    const float ts = (sh[0][0] + sh[0][1]) + (sh[0][2] + sh[0][3]);
    const float tc = (sh[1][0] + sh[1][1]) + (sh[1][2] + sh[1][3]);
    out[0] = ts / fmaxf(tc, 1.f);
    out[1] = tc;
  }
}

// dl * (gout[0] / max(1, valid[0])): the cross-entropy backward's upstream-gradient scale on device
template <typename T>
__global__ __launch_bounds__(256) void xent_grad_scale_kernel(const T* __restrict__ dl, const float* __restrict__ gout,
                                                              const float* __restrict__ valid, T* __restrict__ out,
                                                              int64_t n) {
  const float sc = gout[0] / fmaxf(valid[0], 1.f);
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    if constexpr (std::is_same<T, float>::value) out[i] = dl[i] * sc;
    else reinterpret_cast<unsigned short*>(out)[i] = f2bf(bf2f(reinterpret_cast<const unsigned short*>(dl)[i]) * sc);
  }
}

// log-softmax backward: dz = g - exp(logp) * sum_row(g); one wave per row, logp fp32, g/dz T
template <typename T>
__global__ __launch_bounds__(256) void log_softmax_bwd_kernel(const T* __restrict__ g, const float* __restrict__ logp,
                                                              T* __restrict__ dz, int B, int V) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= B) return;
  const T* gr = g + (size_t)row * V;
  const float* lr = logp + (size_t)row * V;
  float sg = 0.f;
  for (int i = lane; i < V; i += 64) sg += ldv<T>(gr, i);
  sg = warp_sum(sg);
  for (int i = lane; i < V; i += 64) {
    const float v = ldv<T>(gr, i) - __expf(lr[i]) * sg;
    if constexpr (std::is_same<T, float>::value) dz[(size_t)row * V + i] = v;
    else reinterpret_cast<unsigned short*>(dz)[(size_t)row * V + i] = f2bf(v);
  }
}

// ---------------------------------------------------------------- dropout ----------------------
// y = x * keep / (1-p), keep = uniform(seed, offset+i) >= p ; same call in backward on dy.
__global__ void dropout_kernel(const __bf16* __restrict__ x, __bf16* __restrict__ y, int64_t n, float p,
                               uint64_t seed0, uint64_t offset, const int64_t* __restrict__ salt) {
  const float scale = 1.f / (1.f - p);
  const uint64_t seed = dropout_seed(seed0, salt);
  const int64_t nv = n / 8;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nv;
       i += (int64_t)gridDim.x * blockDim.x) {
    float v[8];
    ld8(x + i * 8, v);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = uniform01(seed, offset + i * 8 + e) >= p ? v[e] * scale : 0.f;
    st8(y + i * 8, v);
  }
}

// ---------------------------------------------------------------- relu backward ----------------
__global__ void relu_bwd_kernel(const __bf16* __restrict__ dy, const __bf16* __restrict__ y,
                                __bf16* __restrict__ dx, int64_t nv) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nv;
       i += (int64_t)gridDim.x * blockDim.x) {
    const u16x8 g = reinterpret_cast<const u16x8*>(dy)[i];
    const u16x8 v = reinterpret_cast<const u16x8*>(y)[i];
    u16x8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = bf2f(v[e]) > 0.f ? g[e] : (unsigned short)0;
    reinterpret_cast<u16x8*>(dx)[i] = o;
  }
}

// ---------------------------------------------------------------- column sums (bias grad) -------
// x [M][C] bf16 -> out[C] f32 (+= if accumulate). grid.x over 64-vector column slabs,
// grid.y over row chunks -> partial f32 atomics (few rows chunks; deterministic when grid.y==1)
// Column sums of a bf16 [M][C] matrix (bias gradients): stage 1 writes per-chunk partial sums
// part[chunk][C] (grid = column blocks x row chunks, sized to fill the GPU), stage 2 reduces the
// chunks deterministically (launch_col_reduce).
__global__ void colsum_partial_kernel(const __bf16* __restrict__ x, float* __restrict__ part, int M, int C,
                                      int rows_per_chunk) {
  const int CV = C / 8;
  const int cv = blockIdx.x * 64 + (threadIdx.x & 63);
  const int g = threadIdx.x >> 6;
  __shared__ float sh[4][64][9];
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  const int r0 = blockIdx.y * rows_per_chunk, r1 = min(M, r0 + rows_per_chunk);
  if (cv < CV) {
    for (int r = r0 + g; r < r1; r += 4) {
      float v[8];
      ld8(x + (size_t)r * C + cv * 8, v);
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] += v[e];
    }
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) sh[g][threadIdx.x & 63][e] = acc[e];
  __syncthreads();
  if (g == 0 && cv < CV) {
    float v[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = acc[e] + sh[1][threadIdx.x][e] + sh[2][threadIdx.x][e] + sh[3][threadIdx.x][e];
    f32x4* o = reinterpret_cast<f32x4*>(part + (size_t)blockIdx.y * C + cv * 8);
    o[0] = f32x4{v[0], v[1], v[2], v[3]};
    o[1] = f32x4{v[4], v[5], v[6], v[7]};
  }
}

// out[l] (+)= sum_t part[t][l]: block = 64 column quads x 4 row groups, float4 loads
// columns [0, L1) go to out, [L1, L) to out2 (a null destination skips its columns)
__global__ void col_reduce_kernel(const float* __restrict__ part, int T, int L, float* __restrict__ out,
                                  int accumulate, float* __restrict__ out2, int L1) {
  const int L4 = L / 4;
  const int q = blockIdx.x * 64 + (threadIdx.x & 63);
  const int g = threadIdx.x >> 6;
  __shared__ f32x4 sh[4][64];
  f32x4 s = {0.f, 0.f, 0.f, 0.f};
  if (q < L4) {
    const f32x4* p4 = reinterpret_cast<const f32x4*>(part);
    int t = g;
    for (; t + 12 < T; t += 16) {
      const f32x4 a = p4[(size_t)t * L4 + q], b = p4[(size_t)(t + 4) * L4 + q];
      const f32x4 c = p4[(size_t)(t + 8) * L4 + q], d = p4[(size_t)(t + 12) * L4 + q];
      s += (a + b) + (c + d);
    }
    for (; t < T; t += 4) s += p4[(size_t)t * L4 + q];
  }
  sh[g][threadIdx.x & 63] = s;
  __syncthreads();
  if (g == 0 && q < L4) {
    s = (sh[0][threadIdx.x] + sh[1][threadIdx.x]) + (sh[2][threadIdx.x] + sh[3][threadIdx.x]);
    const int L14 = L1 / 4;
    f32x4* o = q < L14 ? reinterpret_cast<f32x4*>(out) + q : (out2 ? reinterpret_cast<f32x4*>(out2) + (q - L14) : nullptr);
    if (q < L14 && !out) o = nullptr;
    if (o) {
      if (accumulate) s += *o;
      *o = s;
    }
  }
}

void launch_col_reduce(const float* part, int T, int L, float* out, bool accumulate, hipStream_t st, float* out2,
                       int L1) {
  if (L1 < 0) L1 = L;
  TORCH_CHECK(L % 4 == 0 && L1 % 4 == 0, "col_reduce: L % 4");
  hipLaunchKernelGGL(col_reduce_kernel, dim3(ceil_div(L / 4, 64)), dim3(256), 0, st, part, T, L, out,
                     (int)accumulate, out2, L1);
  PCMP_LAUNCH_CHECK();
}

// ---------------------------------------------------------------- input conversion -------------
// x: [N, Cin, H, W] (f32 or u8) -> y: [N, H, W, Cpad] bf16, y = (x*scale - mean[c]) / std[c]
template <typename T>
__global__ void nchw_to_nhwc_kernel(const T* __restrict__ x, __bf16* __restrict__ y, int N, int Cin, int HW,
                                    int Cpad, float scale, const float* __restrict__ mean,
                                    const float* __restrict__ stdv) {
  const int64_t total = (int64_t)N * HW;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int n = i / HW, hw = i % HW;
    for (int c0 = 0; c0 < Cpad; c0 += 8) {
      float v[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int c = c0 + e;
        if (c < Cin) {
          float a = (float)x[((size_t)n * Cin + c) * HW + hw] * scale;
          if (mean) a = (a - mean[c]) / stdv[c];
          v[e] = a;
        } else {
          v[e] = 0.f;
        }
      }
      st8(y + (size_t)i * Cpad + c0, v);
    }
  }
}


// fp32 variant of the input conversion (the reference-precision path, ``--dtype fp32``)
template <typename T>
__global__ void nchw_to_nhwc_f32_kernel(const T* __restrict__ x, float* __restrict__ y, int N, int Cin, int HW,
                                        int Cpad, float scale) {
  const int64_t total = (int64_t)N * HW * Cpad;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int c = i % Cpad;
    const int64_t r = i / Cpad;
    const int n = r / HW, hw = r % HW;
    y[i] = c < Cin ? (float)x[((size_t)n * Cin + c) * HW + hw] * scale : 0.f;
  }
}


// ---------------------------------------------------------------- device image resize -----------
// PIL-exact bilinear (antialiased) resize of uint8 HWC images on the device: SURVEY §2.4.6 /
// B6 — the reference's per-image ``Resize((224,224))`` + ``ToTensor`` (another_neural_net.py:170-187;
// nb :847-862) without the host PIL resize.  Same algorithm as Pillow's ImagingResample for 8-bit
// images: separable triangle filter with support max(1, in/out), coefficients computed in double
// (no fma contraction) and rounded to 22-bit fixed point, horizontal pass first with a clipped
// uint8 intermediate, then the vertical pass.  Output either a CHW uint8 image (bit-identical to
// PIL's) or, fused, the model input: NHWC with channels padded to cpad, (v*scale - mean)/std, in
// bf16 or fp32.
constexpr int RS_PREC = 22;
constexpr int RS_MAXK = 64;   // taps per output pixel (support <= 31.5: downscale ratios up to 31x)

__device__ __forceinline__ int resize_coeffs(int xx, int in_size, int out_size, int* kint) {
#pragma clang fp contract(off)
  const double scale = (double)in_size / (double)out_size;
  const double filterscale = scale < 1.0 ? 1.0 : scale;
  const double support = 1.0 * filterscale;
  const double center = ((double)xx + 0.5) * scale;
  const double ss = 1.0 / filterscale;
  int xmin = (int)(center - support + 0.5);
  if (xmin < 0) xmin = 0;
  int xmax = (int)(center + support + 0.5);
  if (xmax > in_size) xmax = in_size;
  xmax -= xmin;
  if (xmax > RS_MAXK) xmax = RS_MAXK;
  auto tri = [&](int x) {   // Pillow's bilinear_filter at tap x
    double t = ((double)(x + xmin) - center + 0.5) * ss;
    if (t < 0.0) t = -t;
    return t < 1.0 ? 1.0 - t : 0.0;
  };
  double ww = 0.0;
  for (int x = 0; x < xmax; ++x) ww += tri(x);
  for (int x = 0; x < xmax; ++x) {
    const double w = tri(x);
    const double k = ww != 0.0 ? w / ww : w;
    kint[x] = (int)(k * (double)(1 << RS_PREC) + (k < 0.0 ? -0.5 : 0.5));
  }
  return (xmin << 8) | xmax;   // xmax <= 64 fits 8 bits
}

__device__ __forceinline__ unsigned char clip8(int v) {
  if (v >= (1 << RS_PREC << 8)) return 255;
  if (v <= 0) return 0;
  return (unsigned char)(v >> RS_PREC);
}

// horizontal pass: src [N][H][W][C] u8 -> tmp [N][H][Wo][C] u8 (one thread per output pixel, all C)
__global__ __launch_bounds__(256) void resize_h_kernel(const unsigned char* __restrict__ src,
                                                       unsigned char* __restrict__ tmp, int N, int H, int W, int C,
                                                       int Wo) {
  const int64_t total = (int64_t)N * H * Wo;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
    const int xo = t % Wo;
    const int64_t row = t / Wo;   // n*H + y
    int k[RS_MAXK];
    const int b = resize_coeffs(xo, W, Wo, k);
    const int xmin = b >> 8, nt = b & 255;
    const unsigned char* s = src + (size_t)row * W * C;
    for (int c = 0; c < C; ++c) {
      int acc = 1 << (RS_PREC - 1);
      for (int x = 0; x < nt; ++x) acc += (int)s[(size_t)(xmin + x) * C + c] * k[x];
      tmp[((size_t)row * Wo + xo) * C + c] = clip8(acc);
    }
  }
}

// vertical pass: tmp [N][H][Wo][C] -> out.  MODE 0: CHW u8 image [N][C][Ho][Wo]; MODE 1/2: NHWC
// [N][Ho][Wo][cpad] bf16 / fp32 of (v*scale - mean[c]) / std[c] (zero in the padded channels).
template <int MODE>
__global__ __launch_bounds__(256) void resize_v_kernel(const unsigned char* __restrict__ tmp, void* __restrict__ out,
                                                       int N, int H, int Wo, int C, int Ho, int cpad, float scale,
                                                       const float* __restrict__ mean, const float* __restrict__ stdv) {
  const int64_t total = (int64_t)N * Ho * Wo;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
    const int xo = t % Wo;
    const int yo = (t / Wo) % Ho;
    const int n = t / ((int64_t)Wo * Ho);
    int k[RS_MAXK];
    const int b = resize_coeffs(yo, H, Ho, k);
    const int ymin = b >> 8, nt = b & 255;
    const int cmax = MODE == 0 ? C : cpad;
    for (int c = 0; c < cmax; ++c) {
      float v = 0.f;
      unsigned char u = 0;
      if (c < C) {
        int acc = 1 << (RS_PREC - 1);
        for (int y = 0; y < nt; ++y) acc += (int)tmp[(((size_t)n * H + ymin + y) * Wo + xo) * C + c] * k[y];
        u = clip8(acc);
        v = (float)u * scale;
        if (mean) v = (v - mean[c]) / stdv[c];
      }
      if constexpr (MODE == 0) {
        reinterpret_cast<unsigned char*>(out)[(((size_t)n * C + c) * Ho + yo) * Wo + xo] = u;
      } else if constexpr (MODE == 1) {
        reinterpret_cast<unsigned short*>(out)[(((size_t)n * Ho + yo) * Wo + xo) * cpad + c] = f2bf(v);
      } else {
        reinterpret_cast<float*>(out)[(((size_t)n * Ho + yo) * Wo + xo) * cpad + c] = v;
      }
    }
  }
}

// Stem space-to-depth.  A 7x7 / stride-2 / pad-p convolution over X equals a 4x4 / stride-1 /
// unpadded convolution over S[n][i][j][(dy*2+dx)*4 + c] = X[n][c][2i+dy-p][2j+dx-p] (zero outside
// the image and for c >= Cin) with the 7x7 filter embedded in an 8x8 one (ops/conv_blocks.py
// s2d_weight): the GEMM reduction shrinks from 7*7*8 (Cin padded to 8 for 16-B chunks) to
// 4*4*16 = 256, four full K-tiles, and every 16-B chunk still holds one tap's channels.
// One thread per S pixel (16 channels = two 16-B stores).  NHWC: X is [N,H,W,Cs] (the 8-channel
// padded stem input; bf16, or fp32 for the fp32 path, TO = float) instead of [N,Cin,H,W] f32/u8.
template <typename T, bool NHWC, typename TO = __bf16>
__global__ void image_to_s2d_kernel(const T* __restrict__ x, TO* __restrict__ y, int N, int Cin, int H, int W,
                                    int Cs, int Hs, int Ws, int pad, float scale, const float* __restrict__ mean,
                                    const float* __restrict__ stdv) {
  const int64_t total = (int64_t)N * Hs * Ws;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    int j, i, n;
    if (total < INT_MAX) {   // 32-bit index math (64-bit division is a long VALU sequence)
      const unsigned u = (unsigned)t, r = u / (unsigned)Ws;
      j = u - r * (unsigned)Ws; i = r % (unsigned)Hs; n = r / (unsigned)Hs;
    } else {
      j = t % Ws;
      const int64_t r = t / Ws;
      i = r % Hs; n = r / Hs;
    }
    float v[16];
#pragma unroll
    for (int d = 0; d < 4; ++d) {
      const int h = 2 * i + (d >> 1) - pad, w = 2 * j + (d & 1) - pad;
      const bool ok = (unsigned)h < (unsigned)H && (unsigned)w < (unsigned)W;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        float a = 0.f;
        if (ok && c < Cin) {
          if constexpr (NHWC) {
            a = (float)x[(((size_t)n * H + h) * W + w) * Cs + c];
          } else {
            a = (float)x[(((size_t)n * Cin + c) * H + h) * W + w] * scale;
            if (mean) a = (a - mean[c]) / stdv[c];
          }
        }
        v[d * 4 + c] = a;
      }
    }
    if constexpr (std::is_same<TO, float>::value) {
#pragma unroll
      for (int q = 0; q < 4; ++q)
        *reinterpret_cast<float4*>(y + t * 16 + 4 * q) = make_float4(v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]);
    } else {
      st8(y + t * 16, v);
      st8(y + t * 16 + 8, v + 8);
    }
  }
}

// ---------------------------------------------------------------- host ---------------------------
// specialised 3x3 / stride-2 / pad-1 pooling kernels (32-bit indexing); knob pool3s2=0 -> generic
static Knob kn_pool3s2("pool3s2", 1);

static Knob kn_pool_quad("pool_quad", 1);   // stem pooling backward over 2x2 input quads
static bool pool3s2_ok(const at::Tensor& x, int64_t k, int64_t s, int64_t pad) {
  return kn_pool3s2.get() && k == 3 && s == 2 && pad == 1 && x.numel() < (int64_t)INT_MAX;
}

std::vector<at::Tensor> maxpool_fwd(const at::Tensor& x, int64_t k, int64_t s, int64_t pad, bool want_idx,
                                    const c10::optional<at::Tensor>& scale, const c10::optional<at::Tensor>& shift) {
  if (x.scalar_type() == at::kFloat) return f32::maxpool_fwd(x, k, s, pad, want_idx, scale, shift);
  PCMP_CHECK_CUDA(x); PCMP_CHECK_BF16(x); PCMP_CHECK_CONTIG(x);
  const bool bn = scale.has_value() && scale->defined();
  if (bn) {
    PCMP_CHECK_F32(*scale);
    TORCH_CHECK(shift.has_value() && shift->defined() && scale->numel() == x.size(3) && shift->numel() == x.size(3),
                "maxpool_fwd: fused BN needs per-channel scale and shift");
  }
  const int N = x.size(0), H = x.size(1), W = x.size(2), C = x.size(3);
  TORCH_CHECK(C % 8 == 0 && k * k <= 255, "maxpool: C%8 / k");
  const int P = (H + 2 * pad - k) / s + 1, Q = (W + 2 * pad - k) / s + 1;
  auto y = at::empty({N, P, Q, C}, x.options());
  at::Tensor idx = want_idx ? at::empty({N, P, Q, C}, x.options().dtype(at::kByte)) : at::Tensor();
  const int64_t total = (int64_t)N * P * Q * (C / 8);
  if (pool3s2_ok(x, k, s, pad)) {
    hipLaunchKernelGGL(maxpool3s2_fwd_kernel, dim3((unsigned)ceil_div(total, 256)), dim3(256), 0, cur_stream(),
                       ptr<__bf16>(x), ptr<__bf16>(y), want_idx ? ptr<uint8_t>(idx) : nullptr, (unsigned)total, H, W,
                       C / 8, P, Q, bn ? ptr<float>(*scale) : nullptr, bn ? ptr<float>(*shift) : nullptr);
  } else {
    hipLaunchKernelGGL(maxpool_fwd_kernel, dim3(grid_for(total)), dim3(256), 0, cur_stream(), ptr<__bf16>(x),
                       ptr<__bf16>(y), want_idx ? ptr<uint8_t>(idx) : nullptr, N, H, W, C, P, Q, (int)k, (int)s,
                       (int)pad, bn ? ptr<float>(*scale) : nullptr, bn ? ptr<float>(*shift) : nullptr);
  }
  PCMP_LAUNCH_CHECK();
  if (want_idx) return {y, idx};
  return {y};
}

at::Tensor maxpool_bwd(const at::Tensor& dy, const at::Tensor& idx, int64_t H, int64_t W, int64_t k, int64_t s,
                       int64_t pad) {
  if (dy.scalar_type() == at::kFloat) return f32::maxpool_bwd(dy, idx, H, W, k, s, pad);
  PCMP_CHECK_BF16(dy); PCMP_CHECK_CONTIG(dy);
  const int N = dy.size(0), P = dy.size(1), Q = dy.size(2), C = dy.size(3);
  auto dx = at::empty({N, H, W, C}, dy.options());
  const int64_t total = (int64_t)N * H * W * (C / 8);
  hipLaunchKernelGGL(maxpool_bwd_kernel, dim3(grid_for(total)), dim3(256), 0, cur_stream(), ptr<__bf16>(dy),
                     ptr<uint8_t>(idx), ptr<__bf16>(dx), N, (int)H, (int)W, C, P, Q, (int)k, (int)s, (int)pad);
  PCMP_LAUNCH_CHECK();
  return dx;
}

// fused stem backward (see maxpool_bwd_bnr_kernel): returns [g, part]
std::vector<at::Tensor> maxpool_bwd_bnr(const at::Tensor& dy, const at::Tensor& idx, const at::Tensor& cx,
                                        const at::Tensor& mean, const at::Tensor& invstd, const at::Tensor& scale,
                                        const at::Tensor& shift, int64_t k, int64_t s, int64_t pad) {
  if (dy.scalar_type() == at::kFloat) return f32::maxpool_bwd_bnr(dy, idx, cx, mean, invstd, scale, shift, k, s, pad);
  PCMP_CHECK_BF16(dy); PCMP_CHECK_CONTIG(dy); PCMP_CHECK_BF16(cx); PCMP_CHECK_CONTIG(cx);
  TORCH_CHECK(idx.scalar_type() == at::kByte && idx.is_contiguous() && idx.numel() == dy.numel(), "maxpool_bwd_bnr: idx");
  const int N = dy.size(0), P = dy.size(1), Q = dy.size(2), C = dy.size(3);
  const int H = cx.size(1), W = cx.size(2);
  TORCH_CHECK(cx.size(0) == N && cx.size(3) == C && C % 8 == 0 && C / 8 <= 256 && 256 % (C / 8) == 0,
              "maxpool_bwd_bnr: channel layout");
  for (const at::Tensor* t : {&mean, &invstd, &scale, &shift}) {
    PCMP_CHECK_F32(*t);
    TORCH_CHECK(t->numel() == C, "maxpool_bwd_bnr: per-channel vectors");
  }
  const int M = N * H * W, rpp = 256 / (C / 8);
  auto g = at::empty_like(cx);
  if (kn_pool_quad.get() && pool3s2_ok(cx, k, s, pad) && H % 2 == 0 && W % 2 == 0 && P == H / 2 && Q == W / 2) {
    const int MQ = M / 4;
    int qpb = std::max(rpp, ceil_div(MQ, 2048));
    qpb = ceil_div(qpb, rpp) * rpp;
    const int T = ceil_div(MQ, qpb);
    auto part = at::empty({T, 2, C}, cx.options().dtype(at::kFloat));
    hipLaunchKernelGGL(maxpool_bwd_bnr_quad_kernel, dim3(T), dim3(256), (size_t)rpp * 2 * C * sizeof(float),
                       cur_stream(), ptr<__bf16>(dy), ptr<uint8_t>(idx), ptr<__bf16>(cx), ptr<float>(mean),
                       ptr<float>(invstd), ptr<float>(scale), ptr<float>(shift), ptr<__bf16>(g), ptr<float>(part), N,
                       H, W, C, P, Q, qpb);
    PCMP_LAUNCH_CHECK();
    return {g, part};
  }
  int rpb = std::max(rpp, ceil_div(M, 2048));
  rpb = ceil_div(rpb, rpp) * rpp;
  const int T = ceil_div(M, rpb);
  auto part = at::empty({T, 2, C}, cx.options().dtype(at::kFloat));
  auto kfn = pool3s2_ok(cx, k, s, pad) && P == (H - 1) / 2 + 1 && Q == (W - 1) / 2 + 1 ? &maxpool_bwd_bnr_kernel<true>
                                                                                     : &maxpool_bwd_bnr_kernel<false>;
  hipLaunchKernelGGL(kfn, dim3(T), dim3(256), (size_t)rpp * 2 * C * sizeof(float), cur_stream(),
                     ptr<__bf16>(dy), ptr<uint8_t>(idx), ptr<__bf16>(cx), ptr<float>(mean), ptr<float>(invstd),
                     ptr<float>(scale), ptr<float>(shift), ptr<__bf16>(g), ptr<float>(part), N, H, W, C, P, Q,
                     (int)k, (int)s, (int)pad, rpb);
  PCMP_LAUNCH_CHECK();
  return {g, part};
}

at::Tensor gap_fwd(const at::Tensor& x) {
  if (x.scalar_type() == at::kFloat) return f32::gap_fwd(x);
  PCMP_CHECK_BF16(x); PCMP_CHECK_CONTIG(x);
  const int N = x.size(0), C = x.size(-1);
  const int HW = x.numel() / ((int64_t)N * C);
  TORCH_CHECK(C % 8 == 0, "gap: C%8");
  auto y = at::empty({N, C}, x.options());
  dim3 grid(ceil_div(C / 8, 64), N);
  hipLaunchKernelGGL(gap_fwd_kernel, grid, dim3(256), 0, cur_stream(), ptr<__bf16>(x), ptr<__bf16>(y), HW, C);
  PCMP_LAUNCH_CHECK();
  return y;
}

at::Tensor gap_bwd(const at::Tensor& dy, int64_t H, int64_t W) {
  if (dy.scalar_type() == at::kFloat) return f32::gap_bwd(dy, H, W);
  PCMP_CHECK_BF16(dy); PCMP_CHECK_CONTIG(dy);
  const int N = dy.size(0), C = dy.size(1);
  auto dx = at::empty({N, H, W, C}, dy.options());
  const int64_t total = (int64_t)N * H * W * (C / 8);
  hipLaunchKernelGGL(gap_bwd_kernel, dim3(grid_for(total)), dim3(256), 0, cur_stream(), ptr<__bf16>(dy),
                     ptr<__bf16>(dx), N, (int)(H * W), C);
  PCMP_LAUNCH_CHECK();
  return dx;
}

// returns [loss_rows(f32 [B]), logp(f32) if want_logp, dlogits if want_grad]
std::vector<at::Tensor> softmax_xent(const at::Tensor& logits, const c10::optional<at::Tensor>& labels,
                                     bool want_logp, bool want_grad, double grad_scale, int64_t ignore_index) {
  PCMP_CHECK_CUDA(logits); PCMP_CHECK_CONTIG(logits);
  TORCH_CHECK(logits.dim() == 2, "softmax_xent: [B,V] logits");
  const int B = logits.size(0), V = logits.size(1);
  auto f32 = logits.options().dtype(at::kFloat);
  auto loss_rows = at::empty({B}, f32);
  at::Tensor logp = want_logp ? at::empty({B, V}, f32) : at::Tensor();
  at::Tensor dl = want_grad ? at::empty_like(logits) : at::Tensor();
  const int64_t* lab = nullptr;
  if (labels.has_value() && labels->defined()) {
    TORCH_CHECK(labels->scalar_type() == at::kLong, "labels must be int64");
    lab = labels->data_ptr<int64_t>();
  }
  dim3 grid(ceil_div(B, 4)), block(256);
  if (logits.scalar_type() == at::kFloat) {
    hipLaunchKernelGGL(xent_kernel<float>, grid, block, 0, cur_stream(), ptr<float>(logits), lab, B, V,
                       want_logp ? ptr<float>(logp) : nullptr, want_grad ? ptr<float>(dl) : nullptr,
                       ptr<float>(loss_rows), (float)grad_scale, (int)ignore_index);
  } else {
    PCMP_CHECK_BF16(logits);
    hipLaunchKernelGGL(xent_kernel<__bf16>, grid, block, 0, cur_stream(), ptr<__bf16>(logits), lab, B, V,
                       want_logp ? ptr<float>(logp) : nullptr, want_grad ? ptr<__bf16>(dl) : nullptr,
                       ptr<float>(loss_rows), (float)grad_scale, (int)ignore_index);
  }
  PCMP_LAUNCH_CHECK();
  std::vector<at::Tensor> r{loss_rows};
  if (want_logp) r.push_back(logp);
  if (want_grad) r.push_back(dl);
  return r;
}


at::Tensor loss_mean(const at::Tensor& loss_rows, const at::Tensor& labels, int64_t V, int64_t ignore_index) {
  PCMP_CHECK_CUDA(loss_rows); PCMP_CHECK_F32(loss_rows); PCMP_CHECK_CONTIG(loss_rows); PCMP_CHECK_CONTIG(labels);
  TORCH_CHECK(labels.scalar_type() == at::kLong && labels.numel() == loss_rows.numel(), "loss_mean: int64 labels [B]");
  auto out = at::empty({2}, loss_rows.options());
  hipLaunchKernelGGL(loss_mean_kernel, dim3(1), dim3(256), 0, cur_stream(), ptr<float>(loss_rows),
                     labels.data_ptr<int64_t>(), (int)loss_rows.numel(), (int)V, (int)ignore_index, ptr<float>(out));
  PCMP_LAUNCH_CHECK();
  return out;
}

at::Tensor xent_grad_scale(const at::Tensor& dl, const at::Tensor& gout, const at::Tensor& valid) {
  PCMP_CHECK_CUDA(dl); PCMP_CHECK_CONTIG(dl); PCMP_CHECK_F32(gout); PCMP_CHECK_F32(valid);
  auto out = at::empty_like(dl);
  const int64_t n = dl.numel();
  if (n == 0) return out;
  const int grid = (int)std::min<int64_t>(ceil_div(n, (int64_t)256), 4096);
  if (dl.scalar_type() == at::kFloat)
    hipLaunchKernelGGL(xent_grad_scale_kernel<float>, dim3(grid), dim3(256), 0, cur_stream(), ptr<float>(dl),
                       ptr<float>(gout), ptr<float>(valid), ptr<float>(out), n);
  else {
    PCMP_CHECK_BF16(dl);
    hipLaunchKernelGGL(xent_grad_scale_kernel<__bf16>, dim3(grid), dim3(256), 0, cur_stream(), ptr<__bf16>(dl),
                       ptr<float>(gout), ptr<float>(valid), ptr<__bf16>(out), n);
  }
  PCMP_LAUNCH_CHECK();
  return out;
}

at::Tensor log_softmax_bwd(const at::Tensor& g, const at::Tensor& logp) {
  PCMP_CHECK_CUDA(g); PCMP_CHECK_CONTIG(g); PCMP_CHECK_F32(logp); PCMP_CHECK_CONTIG(logp);
  TORCH_CHECK(g.dim() == 2 && logp.sizes() == g.sizes(), "log_softmax_bwd: g, logp [B,V]");
  const int B = g.size(0), V = g.size(1);
  auto dz = at::empty_like(g);
  if (B == 0) return dz;
  if (g.scalar_type() == at::kFloat)
    hipLaunchKernelGGL(log_softmax_bwd_kernel<float>, dim3(ceil_div(B, 4)), dim3(256), 0, cur_stream(), ptr<float>(g),
                       ptr<float>(logp), ptr<float>(dz), B, V);
  else {
    PCMP_CHECK_BF16(g);
    hipLaunchKernelGGL(log_softmax_bwd_kernel<__bf16>, dim3(ceil_div(B, 4)), dim3(256), 0, cur_stream(),
                       ptr<__bf16>(g), ptr<float>(logp), ptr<__bf16>(dz), B, V);
  }
  PCMP_LAUNCH_CHECK();
  return dz;
}

at::Tensor dropout(const at::Tensor& x, double p, int64_t seed, int64_t offset, const c10::optional<at::Tensor>& salt) {
  if (x.scalar_type() == at::kFloat) return f32::dropout(x, p, seed, offset, salt);
  PCMP_CHECK_BF16(x); PCMP_CHECK_CONTIG(x);
  TORCH_CHECK(x.numel() % 8 == 0, "dropout: numel % 8");
  auto y = at::empty_like(x);
  hipLaunchKernelGGL(dropout_kernel, dim3(grid_for(x.numel() / 8)), dim3(256), 0, cur_stream(), ptr<__bf16>(x),
                     ptr<__bf16>(y), x.numel(), (float)p, (uint64_t)seed, (uint64_t)offset, salt_ptr(salt));
  PCMP_LAUNCH_CHECK();
  return y;
}

at::Tensor relu_bwd(const at::Tensor& dy, const at::Tensor& y) {
  if (dy.scalar_type() == at::kFloat) return f32::relu_bwd(dy, y);
  PCMP_CHECK_BF16(dy); PCMP_CHECK_CONTIG(dy); PCMP_CHECK_CONTIG(y);
  TORCH_CHECK(dy.numel() % 8 == 0, "relu_bwd: numel % 8");
  auto dx = at::empty_like(dy);
  hipLaunchKernelGGL(relu_bwd_kernel, dim3(grid_for(dy.numel() / 8)), dim3(256), 0, cur_stream(),
                     ptr<__bf16>(dy), ptr<__bf16>(y), ptr<__bf16>(dx), dy.numel() / 8);
  PCMP_LAUNCH_CHECK();
  return dx;
}

void colsum(const at::Tensor& x, at::Tensor out, bool accumulate) {
  if (x.scalar_type() == at::kFloat) return f32::colsum(x, out, accumulate);
  PCMP_CHECK_BF16(x); PCMP_CHECK_CONTIG(x); PCMP_CHECK_F32(out); PCMP_CHECK_CONTIG(out);
  const int C = x.size(-1);
  const int M = x.numel() / C;
  TORCH_CHECK(C % 8 == 0 && out.numel() == C, "colsum: shapes");
  const int colblocks = ceil_div(C / 8, 64);
  const int chunks = std::max(1, std::min({ceil_div(512, colblocks), ceil_div(M, 16), 256}));
  const int rpc = ceil_div(M, chunks);
  const int T = ceil_div(M, rpc);
  auto part = at::empty({T, C}, out.options());
  hipLaunchKernelGGL(colsum_partial_kernel, dim3(colblocks, T), dim3(256), 0, cur_stream(), ptr<__bf16>(x),
                     ptr<float>(part), M, C, rpc);
  PCMP_LAUNCH_CHECK();
  launch_col_reduce(ptr<float>(part), T, C, ptr<float>(out), accumulate, cur_stream());
}

at::Tensor nchw_to_nhwc(const at::Tensor& x, int64_t cpad, double scale, const c10::optional<at::Tensor>& mean,
                        const c10::optional<at::Tensor>& stdv) {
  PCMP_CHECK_CUDA(x); PCMP_CHECK_CONTIG(x);
  const int N = x.size(0), Cin = x.size(1), H = x.size(2), W = x.size(3);
  TORCH_CHECK(cpad % 8 == 0 && cpad >= Cin, "nchw_to_nhwc: cpad");
  auto y = at::empty({N, H, W, cpad}, x.options().dtype(at::kBFloat16));
  const int64_t total = (int64_t)N * H * W;
  if (x.scalar_type() == at::kFloat) {
    hipLaunchKernelGGL(nchw_to_nhwc_kernel<float>, dim3(grid_for(total)), dim3(256), 0, cur_stream(),
                       ptr<float>(x), ptr<__bf16>(y), N, Cin, H * W, (int)cpad, (float)scale, optr<float>(mean),
                       optr<float>(stdv));
  } else {
    TORCH_CHECK(x.scalar_type() == at::kByte, "nchw_to_nhwc: f32 or u8 input");
    hipLaunchKernelGGL(nchw_to_nhwc_kernel<uint8_t>, dim3(grid_for(total)), dim3(256), 0, cur_stream(),
                       ptr<uint8_t>(x), ptr<__bf16>(y), N, Cin, H * W, (int)cpad, (float)scale, optr<float>(mean),
                       optr<float>(stdv));
  }
  PCMP_LAUNCH_CHECK();
  return y;
}


at::Tensor nchw_to_nhwc_f32(const at::Tensor& x, int64_t cpad, double scale) {
  PCMP_CHECK_CUDA(x); PCMP_CHECK_CONTIG(x);
  const int N = x.size(0), Cin = x.size(1), H = x.size(2), W = x.size(3);
  TORCH_CHECK(cpad % 4 == 0 && cpad >= Cin, "nchw_to_nhwc_f32: cpad");
  auto y = at::empty({N, H, W, cpad}, x.options().dtype(at::kFloat));
  const int64_t total = (int64_t)N * H * W * cpad;
  if (total == 0) return y;
  const int grid = (int)std::min<int64_t>(ceil_div(total, (int64_t)256), 8192);
  if (x.scalar_type() == at::kFloat)
    hipLaunchKernelGGL(nchw_to_nhwc_f32_kernel<float>, dim3(grid), dim3(256), 0, cur_stream(), ptr<float>(x),
                       ptr<float>(y), N, Cin, H * W, (int)cpad, (float)scale);
  else {
    TORCH_CHECK(x.scalar_type() == at::kByte, "nchw_to_nhwc_f32: f32 or u8 input");
    hipLaunchKernelGGL(nchw_to_nhwc_f32_kernel<uint8_t>, dim3(grid), dim3(256), 0, cur_stream(), ptr<uint8_t>(x),
                       ptr<float>(y), N, Cin, H * W, (int)cpad, (float)scale);
  }
  PCMP_LAUNCH_CHECK();
  return y;
}


// x: uint8 [N, H, W, C] (decoded HWC images, C <= 4).  mode 0: PIL-exact resize -> uint8 [N, C, Ho, Wo];
// mode 1 / 2: fused model input, NHWC [N, Ho, Wo, cpad] bf16 / fp32 = (u8 * scale - mean) / std.
at::Tensor resize_image(const at::Tensor& x, int64_t Ho, int64_t Wo, int64_t mode, int64_t cpad, double scale,
                        const c10::optional<at::Tensor>& mean, const c10::optional<at::Tensor>& stdv) {
  PCMP_CHECK_CUDA(x); PCMP_CHECK_CONTIG(x);
  TORCH_CHECK(x.scalar_type() == at::kByte && x.dim() == 4 && x.size(3) <= 4, "resize_image: uint8 [N,H,W,C<=4]");
  TORCH_CHECK(mode >= 0 && mode <= 2 && Ho > 0 && Wo > 0, "resize_image: mode / size");
  const int N = x.size(0), H = x.size(1), W = x.size(2), C = x.size(3);
  TORCH_CHECK((double)H / Ho <= 31.0 && (double)W / Wo <= 31.0, "resize_image: downscale ratio above 31");
  if (mode) TORCH_CHECK(cpad >= C, "resize_image: cpad < channels");
  if (mean.has_value() && mean->defined()) {
    PCMP_CHECK_F32(*mean); PCMP_CHECK_F32(*stdv);
    TORCH_CHECK(mean->numel() >= C && stdv->numel() >= C, "resize_image: mean/std");
  }
  auto tmp = at::empty({N, H, Wo, C}, x.options());
  at::Tensor out;
  if (mode == 0) out = at::empty({N, C, Ho, Wo}, x.options());
  else out = at::empty({N, Ho, Wo, cpad}, x.options().dtype(mode == 1 ? at::kBFloat16 : at::kFloat));
  if (N == 0) return out;
  const int64_t th = (int64_t)N * H * Wo, tv = (int64_t)N * Ho * Wo;
  hipLaunchKernelGGL(resize_h_kernel, dim3((int)std::min<int64_t>(ceil_div(th, (int64_t)256), 4096)), dim3(256), 0,
                     cur_stream(), ptr<unsigned char>(x), ptr<unsigned char>(tmp), N, H, W, C, (int)Wo);
  PCMP_LAUNCH_CHECK();
  const dim3 gv((int)std::min<int64_t>(ceil_div(tv, (int64_t)256), 4096));
  const float* mp = optr<float>(mean);
  const float* sp = optr<float>(stdv);
#define PCMP_RV(M) hipLaunchKernelGGL(resize_v_kernel<M>, gv, dim3(256), 0, cur_stream(), ptr<unsigned char>(tmp), \
                                      out.data_ptr(), N, H, (int)Wo, C, (int)Ho, (int)cpad, (float)scale, mp, sp)
  if (mode == 0) PCMP_RV(0); else if (mode == 1) PCMP_RV(1); else PCMP_RV(2);
#undef PCMP_RV
  PCMP_LAUNCH_CHECK();
  return out;
}

// fp32 form for the fp32 (reference-precision) stem: NCHW f32 / u8 images -> [N, Hs, Ws, 16] fp32 in
// one pass (no 8-channel NHWC intermediate)
at::Tensor image_to_s2d_f32(const at::Tensor& x, int64_t pad, double scale) {
  PCMP_CHECK_CUDA(x); PCMP_CHECK_CONTIG(x);
  TORCH_CHECK(x.dim() == 4 && x.size(1) <= 4 && pad >= 0, "image_to_s2d_f32: NCHW input, at most 4 channels");
  const int N = x.size(0), Cin = x.size(1), H = x.size(2), W = x.size(3);
  const int Hs = (H + 2 * pad + 1) / 2, Ws = (W + 2 * pad + 1) / 2;
  auto y = at::empty({N, Hs, Ws, 16}, x.options().dtype(at::kFloat));
  const int64_t total = (int64_t)N * Hs * Ws;
  if (x.scalar_type() == at::kFloat) {
    hipLaunchKernelGGL((image_to_s2d_kernel<float, false, float>), dim3(grid_for(total, 256, INT_MAX)), dim3(256), 0,
                       cur_stream(), ptr<float>(x), ptr<float>(y), N, Cin, H, W, 0, Hs, Ws, (int)pad, (float)scale,
                       nullptr, nullptr);
  } else {
    TORCH_CHECK(x.scalar_type() == at::kByte, "image_to_s2d_f32: f32 or u8 NCHW input");
    hipLaunchKernelGGL((image_to_s2d_kernel<uint8_t, false, float>), dim3(grid_for(total, 256, INT_MAX)), dim3(256),
                       0, cur_stream(), ptr<uint8_t>(x), ptr<float>(y), N, Cin, H, W, 0, Hs, Ws, (int)pad,
                       (float)scale, nullptr, nullptr);
  }
  PCMP_LAUNCH_CHECK();
  return y;
}

at::Tensor image_to_s2d(const at::Tensor& x, int64_t pad, double scale, const c10::optional<at::Tensor>& mean,
                        const c10::optional<at::Tensor>& stdv, bool nhwc) {
  PCMP_CHECK_CUDA(x); PCMP_CHECK_CONTIG(x);
  TORCH_CHECK(x.dim() == 4, "image_to_s2d: 4-D input");
  const int N = x.size(0);
  const int Cin = nhwc ? std::min<int>(4, x.size(3)) : x.size(1);
  const int H = nhwc ? x.size(1) : x.size(2), W = nhwc ? x.size(2) : x.size(3);
  const int Cs = nhwc ? x.size(3) : 0;
  TORCH_CHECK(Cin <= 4 && pad >= 0, "image_to_s2d: at most 4 input channels");
  const int Hs = (H + 2 * pad + 1) / 2, Ws = (W + 2 * pad + 1) / 2;
  const bool f32 = nhwc && x.scalar_type() == at::kFloat;   // fp32 path: fp32 in, fp32 out
  auto y = at::empty({N, Hs, Ws, 16}, x.options().dtype(f32 ? at::kFloat : at::kBFloat16));
  const int64_t total = (int64_t)N * Hs * Ws;
  if (f32) {
    hipLaunchKernelGGL((image_to_s2d_kernel<float, true, float>), dim3(grid_for(total, 256, INT_MAX)), dim3(256), 0,
                       cur_stream(), ptr<float>(x), ptr<float>(y), N, Cin, H, W, Cs, Hs, Ws, (int)pad, 1.f, nullptr,
                       nullptr);
  } else if (nhwc) {
    PCMP_CHECK_BF16(x);
    hipLaunchKernelGGL((image_to_s2d_kernel<__bf16, true>), dim3(grid_for(total, 256, INT_MAX)), dim3(256), 0, cur_stream(),
                       ptr<__bf16>(x), ptr<__bf16>(y), N, Cin, H, W, Cs, Hs, Ws, (int)pad, 1.f, nullptr, nullptr);
  } else if (x.scalar_type() == at::kFloat) {
    hipLaunchKernelGGL((image_to_s2d_kernel<float, false>), dim3(grid_for(total, 256, INT_MAX)), dim3(256), 0, cur_stream(),
                       ptr<float>(x), ptr<__bf16>(y), N, Cin, H, W, 0, Hs, Ws, (int)pad, (float)scale,
                       optr<float>(mean), optr<float>(stdv));
  } else {
    TORCH_CHECK(x.scalar_type() == at::kByte, "image_to_s2d: f32 or u8 NCHW input");
    hipLaunchKernelGGL((image_to_s2d_kernel<uint8_t, false>), dim3(grid_for(total, 256, INT_MAX)), dim3(256), 0, cur_stream(),
                       ptr<uint8_t>(x), ptr<__bf16>(y), N, Cin, H, W, 0, Hs, Ws, (int)pad, (float)scale,
                       optr<float>(mean), optr<float>(stdv));
  }
  PCMP_LAUNCH_CHECK();
  return y;
}

// ---- row-wise top-k / argmax: one wave per row ----------------------------------------------
// Replaces torch.argmax / torch.topk on logits (batch-1 prediction, top-1/top-5 accuracy).  Each
// lane keeps its own sorted top-KM of the columns it strides over (lane, lane+64, ...), then k
// rounds of a 64-lane butterfly pick the best head and its lane pops it.  Order: larger value
// first, ties to the smaller column (torch.argmax's first-occurrence rule); NaN ranks above every
// number, as in torch.
__device__ __forceinline__ bool topk_better(float a, int ia, float b, int ib) {
  const bool na = a != a, nb = b != b;
  if (na != nb) return na;
  if (na) return ia < ib;
  return a > b || (a == b && ia < ib);
}
__device__ __forceinline__ float load_f(const float* p) { return *p; }
__device__ __forceinline__ float load_f(const __bf16* p) { return (float)*p; }

template <typename T, int KM>
__global__ __launch_bounds__(256) void topk_rows_kernel(const T* __restrict__ x, int B, int C, int64_t ld, int k,
                                                        float* __restrict__ vals, int64_t* __restrict__ idx) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= B) return;
  const T* xr = x + (size_t)row * ld;
  float v[KM];
  int ix[KM];
#pragma unroll
  for (int q = 0; q < KM; ++q) { v[q] = -INFINITY; ix[q] = INT_MAX; }
  for (int j = lane; j < C; j += 64) {
    float cv = load_f(xr + j);
    int ci = j;
#pragma unroll
    for (int q = 0; q < KM; ++q)
      if (topk_better(cv, ci, v[q], ix[q])) {
        const float tv = v[q]; const int ti = ix[q];
        v[q] = cv; ix[q] = ci; cv = tv; ci = ti;
      }
  }
  for (int r = 0; r < k; ++r) {
    float bv = v[0];
    int bi = ix[0];
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
      const float ov = __shfl_xor(bv, off);
      const int oi = __shfl_xor(bi, off);
      if (topk_better(ov, oi, bv, bi)) { bv = ov; bi = oi; }
    }
    if (lane == 0) {
      if (vals) vals[(size_t)row * k + r] = bv;
      idx[(size_t)row * k + r] = bi;
    }
    if (ix[0] == bi) {   // the winning lane pops its head
#pragma unroll
      for (int q = 0; q + 1 < KM; ++q) { v[q] = v[q + 1]; ix[q] = ix[q + 1]; }
      v[KM - 1] = -INFINITY; ix[KM - 1] = INT_MAX;
    }
  }
}

std::vector<at::Tensor> topk_rows(const at::Tensor& x, int64_t k, bool want_values) {
  PCMP_CHECK_CUDA(x);
  TORCH_CHECK(x.dim() == 2 && x.numel() > 0 && x.stride(1) == 1, "topk_rows: non-empty [B, C] rows with unit column stride");
  const int C = x.size(1);
  const int B = x.size(0);
  const int64_t ld = x.stride(0);
  TORCH_CHECK(k >= 1 && k <= 8 && k <= C, "topk_rows: 1 <= k <= min(8, C)");
  auto idx = at::empty({B, k}, x.options().dtype(at::kLong));
  at::Tensor vals = want_values ? at::empty({B, k}, x.options().dtype(at::kFloat)) : at::Tensor();
  float* vp = want_values ? ptr<float>(vals) : nullptr;
  const dim3 grid(ceil_div(B, 4)), block(256);
  const int kk = (int)k;
  if (x.scalar_type() == at::kFloat) {
    const float* xp = x.data_ptr<float>();
    if (k == 1) hipLaunchKernelGGL((topk_rows_kernel<float, 1>), grid, block, 0, cur_stream(), xp, B, C, ld, 1, vp, ptr<int64_t>(idx));
    else hipLaunchKernelGGL((topk_rows_kernel<float, 8>), grid, block, 0, cur_stream(), xp, B, C, ld, kk, vp, ptr<int64_t>(idx));
  } else {
    TORCH_CHECK(x.scalar_type() == at::kBFloat16, "topk_rows: f32 or bf16 input");
    const __bf16* xp = reinterpret_cast<const __bf16*>(x.data_ptr());
    if (k == 1) hipLaunchKernelGGL((topk_rows_kernel<__bf16, 1>), grid, block, 0, cur_stream(), xp, B, C, ld, 1, vp, ptr<int64_t>(idx));
    else hipLaunchKernelGGL((topk_rows_kernel<__bf16, 8>), grid, block, 0, cur_stream(), xp, B, C, ld, kk, vp, ptr<int64_t>(idx));
  }
  PCMP_LAUNCH_CHECK();
  if (want_values) return {vals, idx};
  return {idx};
}

// ---- synthetic image batch (data/synthetic.py SyntheticImages on the GPU) ----------------------
// x[b,c,i,j] = clamp(0.5*color[y_b,c] + 0.25*(sin(fy*t_i)*cos(fx*t_j) + 1)*0.5 + noise*u, 0, 1),
// t = linspace(0, 2*pi, S), u a counter-based uniform (splitmix64 of (seed, element index)): one
// launch instead of ~10 torch ops, four contiguous pixels per thread (16-B stores).
__device__ __forceinline__ uint64_t splitmix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
__global__ __launch_bounds__(256) void synth_images_kernel(const int64_t* __restrict__ labels,
                                                           const float* __restrict__ color,
                                                           const float* __restrict__ freq, int B, int C, int S,
                                                           int K, uint64_t seed, float noise, float* __restrict__ out) {
  const int S4 = S / 4;
  const int64_t total = (int64_t)B * C * S * S4;
  const float step = 6.283185307179586f / (float)(S - 1);
  const uint64_t key = splitmix64(seed);
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
    const int j4 = t % S4;
    int64_t r = t / S4;
    const int i = r % S; r /= S;
    const int c = r % C;
    const int b = r / C;
    const int y = (int)min(max(labels[b], (int64_t)0), (int64_t)(K - 1));   // out-of-range labels clamp, never read OOB
    const float fy = freq[2 * y], fx = freq[2 * y + 1];
    const float base = 0.5f * color[y * C + c];
    const float sy = sinf(fy * (i * step));
    float o[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int j = 4 * j4 + e;
      const uint64_t h = splitmix64(key ^ (uint64_t)(4 * t + e));
      const float u = (float)(h >> 40) * (1.0f / 16777216.0f);
      const float val = base + 0.25f * (sy * cosf(fx * (j * step)) + 1.f) * 0.5f + noise * u;
      o[e] = fminf(fmaxf(val, 0.f), 1.f);
    }
    *reinterpret_cast<float4*>(out + 4 * t) = make_float4(o[0], o[1], o[2], o[3]);
  }
}

at::Tensor synth_images(const at::Tensor& labels, const at::Tensor& color, const at::Tensor& freq, int64_t S,
                        int64_t seed, double noise) {
  PCMP_CHECK_CUDA(labels); PCMP_CHECK_CONTIG(labels); PCMP_CHECK_F32(color); PCMP_CHECK_F32(freq);
  PCMP_CHECK_CONTIG(color); PCMP_CHECK_CONTIG(freq);
  TORCH_CHECK(labels.scalar_type() == at::kLong && labels.dim() == 1, "synth_images: int64 labels [B]");
  TORCH_CHECK(color.dim() == 2 && freq.dim() == 2 && freq.size(1) == 2 && freq.size(0) == color.size(0),
              "synth_images: color [K,C], freq [K,2]");
  TORCH_CHECK(S >= 4 && S % 4 == 0, "synth_images: image size must be a multiple of 4");
  TORCH_CHECK(color.size(0) >= 1, "synth_images: at least one class");
  const int B = labels.size(0), C = color.size(1);
  auto out = at::empty({B, C, S, S}, color.options());
  if (B == 0) return out;
  const int64_t total = (int64_t)B * C * S * (S / 4);
  const int grid = (int)std::min<int64_t>(ceil_div(total, (int64_t)256), 8192);
  hipLaunchKernelGGL(synth_images_kernel, dim3(grid), dim3(256), 0, cur_stream(), ptr<int64_t>(labels),
                     ptr<float>(color), ptr<float>(freq), B, C, (int)S, (int)color.size(0), (uint64_t)seed, (float)noise, ptr<float>(out));
  PCMP_LAUNCH_CHECK();
  return out;
}

}  // namespace pcmp

namespace pcmp {
static std::vector<Knob*>& knob_registry() {
  static std::vector<Knob*> r;
  return r;
}
static std::mutex& knob_mutex() {
  static std::mutex m;
  return m;
}
Knob::Knob(const char* n, int dflt) : name(n), value(dflt) {
  std::lock_guard<std::mutex> g(knob_mutex());
  knob_registry().push_back(this);
}
// returns the previous value; unknown names raise
int64_t set_knob(const std::string& name, int64_t v) {
  std::lock_guard<std::mutex> g(knob_mutex());
  for (Knob* k : knob_registry())
    if (name == k->name) return k->value.exchange((int)v);
  TORCH_CHECK(false, "set_knob: unknown knob ", name);
  return 0;
}
std::vector<std::string> list_knobs() {
  std::lock_guard<std::mutex> g(knob_mutex());
  std::vector<std::string> r;
  for (Knob* k : knob_registry()) r.push_back(std::string(k->name) + "=" + std::to_string(k->get()));
  return r;
}
}  // namespace pcmp

TORCH_LIBRARY_FRAGMENT(pcmp, m) {
  m.def("set_knob(str name, int value) -> int", &pcmp::set_knob);
  m.def("list_knobs() -> str[]", &pcmp::list_knobs);
  m.def("maxpool_fwd(Tensor x, int k, int s, int pad, bool want_idx, Tensor? scale=None, Tensor? shift=None) -> Tensor[]",
        &pcmp::maxpool_fwd);
  m.def("maxpool_bwd_bnr(Tensor dy, Tensor idx, Tensor cx, Tensor mean, Tensor invstd, Tensor scale, Tensor shift, "
        "int k, int s, int pad) -> Tensor[]",
        &pcmp::maxpool_bwd_bnr);
  m.def("maxpool_bwd(Tensor dy, Tensor idx, int H, int W, int k, int s, int pad) -> Tensor", &pcmp::maxpool_bwd);
  m.def("gap_fwd(Tensor x) -> Tensor", &pcmp::gap_fwd);
  m.def("gap_bwd(Tensor dy, int H, int W) -> Tensor", &pcmp::gap_bwd);
  m.def("softmax_xent(Tensor logits, Tensor? labels, bool want_logp, bool want_grad, float grad_scale, "
        "int ignore_index) -> Tensor[]",
        &pcmp::softmax_xent);
  m.def("loss_mean(Tensor loss_rows, Tensor labels, int V, int ignore_index) -> Tensor", &pcmp::loss_mean);
  m.def("xent_grad_scale(Tensor dl, Tensor gout, Tensor valid) -> Tensor", &pcmp::xent_grad_scale);
  m.def("log_softmax_bwd(Tensor g, Tensor logp) -> Tensor", &pcmp::log_softmax_bwd);
  m.def("dropout(Tensor x, float p, int seed, int offset, Tensor? salt=None) -> Tensor", &pcmp::dropout);
  m.def("relu_bwd(Tensor dy, Tensor y) -> Tensor", &pcmp::relu_bwd);
  m.def("colsum(Tensor x, Tensor(a!) out, bool accumulate) -> ()", &pcmp::colsum);
  m.def("nchw_to_nhwc(Tensor x, int cpad, float scale, Tensor? mean, Tensor? stdv) -> Tensor", &pcmp::nchw_to_nhwc);
  m.def("nchw_to_nhwc_f32(Tensor x, int cpad, float scale) -> Tensor", &pcmp::nchw_to_nhwc_f32);
  m.def("resize_image(Tensor x, int Ho, int Wo, int mode, int cpad, float scale, Tensor? mean, Tensor? stdv) -> Tensor",
        &pcmp::resize_image);
  m.def("image_to_s2d(Tensor x, int pad, float scale, Tensor? mean, Tensor? stdv, bool nhwc) -> Tensor", &pcmp::image_to_s2d);
  m.def("image_to_s2d_f32(Tensor x, int pad, float scale) -> Tensor", &pcmp::image_to_s2d_f32);
  m.def("topk_rows(Tensor x, int k, bool want_values) -> Tensor[]", &pcmp::topk_rows);
  m.def("synth_images(Tensor labels, Tensor color, Tensor freq, int S, int seed, float noise) -> Tensor", &pcmp::synth_images);
}

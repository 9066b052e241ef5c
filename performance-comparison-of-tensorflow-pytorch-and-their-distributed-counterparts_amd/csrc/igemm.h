// Implicit-GEMM convolution / linear kernels on CDNA4 MFMA (v_mfma_f32_16x16x32_bf16).
//
// One kernel template covers the three GEMMs of a convolution (and of a Linear layer, which is
// a 1x1 conv over [M,1,1,Cin]):
//   FWD   : Y[m=(n,p,q)][co]      = sum_{k=(r,s,ci)}  X[n,p*st-pad+r,q*st-pad+s,ci] * W[co][r][s][ci]
//   DGRAD : dX[m=(n,h,w)][ci]     = sum_{k=(r,s,co)} dY[n,(h+pad-r)/st,(w+pad-s)/st,co] * Wt[ci][r][s][co]
//   WGRAD : dW[co][j=(r,s,ci)]    = sum_{m=(n,p,q)}  dY[m][co] * X[n,p*st-pad+r,q*st-pad+s,ci]   (split-K)
// Layouts: activations NHWC bf16, weights KRSC bf16, accumulation fp32.
//
// Reference parity: these replace the cuDNN/MKL-DNN convolutions and Linear layers executed by
// torchvision ResNet-50 / VGG16 and the HF BERT / transfer heads in the reference
// (another_neural_net.py:95-112,244-255;
// pytorch_training_inference_on_image.ipynb:454-635).
//
// Structure (cdna_hip_programming.md §5): 256 threads = 4 waves (2x2), block tile BMxBN, BK=64,
// register-staged double-buffered LDS (global loads for tile t+1 are issued before the MFMAs of
// tile t and written to the other LDS buffer after them: one barrier per K-step), XOR-swizzled
// LDS images (ds_read_b128 row reads for FWD/DGRAD; ds_read_b64_tr_b16 transposed reads for
// WGRAD whose operands are both reduction-index-major), XCD-aware bijective block remap, and an
// LDS-staged epilogue that writes 16-byte coalesced rows and emits per-column BatchNorm partial
// statistics of the stored (bf16-rounded) output.
#pragma once
#include "common.h"
#include "f32.h"

#include <algorithm>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

namespace pcmp {

// ----------------------------------------------------------------------------------------------
// Fast unsigned division by a runtime-invariant divisor (round-up multiply method), n < 2^31.
struct FastDiv {
  uint32_t d, m, s;
};
static FastDiv make_fastdiv(uint32_t d) {
  FastDiv f;
  f.d = d;
  uint32_t s = 0;
  while ((1ull << s) < d) ++s;
  f.s = s;
  f.m = (uint32_t)(((1ull << 32) * ((1ull << s) - d)) / d + 1);
  return f;
}
__device__ __forceinline__ uint32_t fdiv(uint32_t n, const FastDiv& f) {
  return (__umulhi(n, f.m) + n) >> f.s;
}

enum IgemmMode { MODE_FWD = 0, MODE_DGRAD = 1, MODE_WGRAD = 2 };

struct IgemmParams {
  const __bf16* a;    // FWD: x[N,H,W,C]; DGRAD: dy[N,P,Q,K]; WGRAD: dy[N,P,Q,K]
  const __bf16* b;    // FWD: w[K][R][S][C]; DGRAD: wt[C][R][S][K]; WGRAD: x[N,H,W,C]
  void* out;          // FWD/DGRAD: bf16 [gm][gn]; WGRAD: f32 [split][gm][gn]
  const float* bias;  // FWD: [gn] (optional)
  const __bf16* resid;  // FWD/DGRAD: bf16 [gm][gn] added before activation (optional); act 3: u
  __bf16* aux;          // act 2: bf16 [gm][gn] pre-activation output u (GELU's backward operand)
  float* stats;       // FWD/DGRAD: [gridM][2][gn] per-block column sum / sum of squares (optional)
  int gm, gn, gk;
  int N, H, W, C, K, R, S, P, Q, stride, pad;
  FastDiv fd_PQ, fd_Q, fd_HW, fd_W;
  // DGRAD decode: rows m -> (n, hh, ww) over [N][dH][dW]; h = hh*ostep + oph (sub-pixel class)
  int dH, dW, offy, offx, sub, oph, opw;
  int relu;         // epilogue activation: 0 none, 1 ReLU, 2 GELU (u = acc + bias -> aux, out = gelu(u)),
                    // 3 GELU backward (out = acc * gelu'(u), u read through resid; BERT FFN)
  unsigned a_bytes, b_bytes;   // buffer-resource extents of a / b (hardware OOB -> zero)
  int ksplit;       // K elements per split (multiple of BK)
  int nsplit;
  int tiles_m, tiles_n;
  float alpha;
  int accumulate;   // WGRAD with nsplit==1: out += result
  // DGRAD fused BatchNorm-backward reduction (bn_x != null): the epilogue stores
  // g = dgrad(+resid) * (bn_mask > 0) and writes per-tile partials [tiles_m][2][gn] of
  // (sum g, sum g*xhat) to stats (and of (sum g, sum g*xhat2) to stats2 for a second BN sharing g).
  const __bf16* bn_mask;
  const __bf16* bn_x;
  const float* bn_mean;
  const float* bn_istd;
  const __bf16* bn_x2;
  const float* bn_mean2;
  const float* bn_istd2;
  float* stats2;
  // mask recomputed from bn_x instead of read: relu(bn_x * bn_msc + bn_msh) > 0 (the forward BN
  // apply of an intermediate layer); used when bn_mask is null
  const float* bn_msc;
  const float* bn_msh;
  // mask as bits (1 byte per 8 channels, written by the forward bn_apply of a block output): used
  // instead of bn_mask -- 1/16 of the bytes of the bf16 tensor
  const uint8_t* bn_mbits;
  int stats_cap;   // BM-row tiles the stats / stats2 buffers hold (host-side bounds check)
  // BatchNorm-backward fold (register-staged DGRAD / WGRAD of 1x1 stride-1 convs, fold_x != null):
  // the dy operand is dz = k1*g + k2*x + k3, computed while the tile is staged from g (= a),
  // x (= fold_x, same layout and extent as a) and per-channel coefficients fold_coef[3][K]
  // (bn_bwd_finalize's k1 | k2 | k3), rounded to bf16 exactly as bn_bwd_apply rounds its output.
  // The bn_bwd_apply pass that would write dz (and the two reads of it) never runs.
  const __bf16* fold_x;
  const float* fold_coef;
  int fold_lds;   // DGRAD / FWD: byte offset of the block's LDS copy of the fold coefficients
  // BatchNorm-forward fold (act_sc != null): the activation operand -- FWD's A (x), WGRAD's B (x) --
  // is y = relu(act_sc[c] * z + act_sh[c]) formed while staging from the pre-BN tensor z, instead
  // of the bn_apply pass that would write y (register-staged kernel; FWD: 1x1 stride-1 convs)
  const float* act_sc;
  const float* act_sh;
  // DGRAD (stride 1): the residual is sub-sampled -- resid is [N][rs_H2][rs_W2][gn] and adds at
  // output pixels (2i, 2j) only (a 1x1 stride-2 downsample's DGRAD, which is zero elsewhere)
  int resid_sub, rs_H2, rs_W2;
};

// y = relu(a*z + b) of one 16-B chunk (8 channels), bf16-rounded as bn_apply rounds; 0 for an
// invalid row / padding
__device__ __forceinline__ uint4 fold_act(uint4 z, const float* a, const float* b, bool ok) {
  const u16x8 zv = __builtin_bit_cast(u16x8, z);
  u16x8 o;
#pragma unroll
  for (int e = 0; e < 8; ++e) o[e] = ok ? f2bf(fmaxf(bf2f(zv[e]) * a[e] + b[e], 0.f)) : (unsigned short)0;
  return __builtin_bit_cast(uint4, o);
}

// dz = k1*g + k2*x + k3 of one 16-B chunk (8 channels), bf16-rounded; 0 for an invalid row
__device__ __forceinline__ uint4 fold_dz(uint4 g, uint4 x, const float* k1, const float* k2, const float* k3,
                                         bool ok) {
  const u16x8 gv = __builtin_bit_cast(u16x8, g), xv = __builtin_bit_cast(u16x8, x);
  u16x8 o;
#pragma unroll
  for (int e = 0; e < 8; ++e) o[e] = ok ? f2bf(k1[e] * bf2f(gv[e]) + k2[e] * bf2f(xv[e]) + k3[e]) : (unsigned short)0;
  return __builtin_bit_cast(uint4, o);
}

constexpr int BK = 64;
constexpr int NT = 256;

// DGRAD + BN-backward-reduce epilogue: register-ring depth of its resid / x / mask loads (2 = one
// step ahead, round 1; 4 = three steps ahead).  A/B knob (tools/gemm_knob_ab.py).
inline Knob kn_wgrad_m32("wgrad_m32", 1);   // WGRAD on 32x32x16 MFMAs (igemm_kernel M32; profiles/r4_wgrad_m32_ab.txt)
inline Knob kn_epi_depth("epi_depth", 4);   // measured: profiles/r2_epilogue_depth_ab.txt
// the dual BN-reduce epilogue (EPI_BNR2) at depth 4 needs 256 VGPRs and spills; depth 2 fits and
// is 0-6 % faster (profiles/r2_bnr2_ab.txt)
inline Knob kn_epi_depth_bnr2("epi_depth_bnr2", 2);

// XCD-aware bijective remap (cdna_hip_programming.md §5 "XCD swizzle must be bijective"):
// consecutive logical tiles land on the same XCD so they share its L2.
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  if (nwg <= 8) return bid;
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  const int base = (xcd < r) ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + (bid >> 3);
}

// Row-read LDS image for FWD/DGRAD operands: [rows][BK] bf16, 128-B rows, 16-B chunks swizzled
// chunk ^ (row & 7) -> conflict-free ds_read_b128 for the 16x16x32 fragment pattern.
__device__ __forceinline__ int rr_off(int row, int chunk) {  // byte offset
  return row * (BK * 2) + ((chunk ^ (row & 7)) << 4);
}

// Transposed-read LDS image for WGRAD operands: [BK rows (reduction)][COLS] bf16.
// 16x16x32 reads (M32 = false): a 32-lane LDS cycle of ds_read_b64_tr_b16 covers 8 rows x 32 B, so 8
// distinct even XOR masks spread the rows' 32-B pairs over the 64 banks.  32x32x16 reads (M32): a
// 32-lane cycle covers 4 rows x 64 B (rows rowb..rowb+3, 32 columns), so the row's 64-B group is XOR-
// shifted by a multiple of 4 chunks: (row & 3) for >= 256-B rows, ((row >> 1) & 1) for 128-B rows,
// whose odd rows already sit on the other 32 banks.  (Round 4 used the 16x16x32 masks for the 32x32
// reads: rows 0/1 and 2/3 collided, 33 % of the WGRAD kernel's LDS cycles were bank conflicts --
// SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE, profiles/r5_wgrad_pmc.txt.)  The 16-B row writes (8 lanes
// per row and cycle) stay conflict-free under either mapping.
template <int COLS, bool M32 = false>
__device__ __forceinline__ int tr_off(int row, int col) {  // byte offset of element (row,col), col%4==0 ok
  constexpr int RB = COLS * 2;  // row bytes
  int x;
  if constexpr (M32) {
    if constexpr (RB >= 256) x = 4 * (row & 3);
    else if constexpr (RB == 128) x = 4 * ((row >> 1) & 1);
    else x = 0;
  } else {
    int f;
    if constexpr (RB >= 256) {
      f = (row & 3) | (((row >> 3) & 1) << 2);            // 8 distinct 32-B slots per half-wave
    } else if constexpr (RB == 128) {
      f = ((row >> 1) & 1) | (((row >> 3) & 1) << 1);
    } else {
      f = 0;
    }
    x = 2 * f;
  }
  const int chunk = (col >> 3) ^ x;  // 16-B chunk, XOR keeps 32-B pairs intact
  return row * RB + (chunk << 4) + ((col & 7) << 1);
}

// Buffer resource over a whole tensor: loads at out-of-range byte offsets return ZERO (hardware
// range check), which implements conv zero-padding and tile tails without selects or branches.
constexpr unsigned kOOB = 0x80000000u;
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ uint4 bload16(__amdgpu_buffer_rsrc_t r, unsigned voff) {
  typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));
  const u32x4_t v = __builtin_amdgcn_raw_buffer_load_b128(r, (int)voff, 0, 0);
  return uint4{v[0], v[1], v[2], v[3]};
}

// LDS row rho of the B tile holds output channel chan_perm(rho): within each group of 32 rows,
// rho = 16jj + 4q + e  ->  8q + 4jj + e  (so MFMA tile pair (2jp, 2jp+1), lane group q, element e
// maps to channel 32jp + 8q + 4jj + e).
template <bool PAIR>
__device__ __forceinline__ int chan_perm(int rho) {
  if constexpr (!PAIR) return rho;
  return (rho & ~31) | (((rho >> 2) & 3) << 3) | (((rho >> 4) & 1) << 2) | (rho & 3);
}

// UNIF: the A source channel count (C for FWD, K for DGRAD) is a multiple of BK, so the 8 16-B
// chunks of a K-step share one filter tap (r,s) and a block-uniform channel base c0: per K-step
// the address update is one uniform scalar offset plus one add per row.
// Epilogue variants (FWD/DGRAD): plain store, + BatchNorm partial statistics of the stored output
// (FWD training), + fused BatchNorm-backward reduction (DGRAD; BNR2: two BNs share the gradient).
// EPI_GELU: the plain epilogue plus the GELU forward / backward activations (act 2 / 3, the BERT FFN
// Linear GEMMs) -- its own instantiations, so the conv kernels' plain epilogue carries no GELU code
enum { EPI_PLAIN = 0, EPI_STATS = 1, EPI_BNR = 2, EPI_BNR2 = 3, EPI_GELU = 4 };

// FWD/DGRAD epilogue shared by the 4-wave and 8-wave kernels.  acc[j][i] holds the D^T fragment of
// MFMA column tile j (4 output channels, PAIR-permuted) x row tile i (16 pixels).
__device__ __forceinline__ void lds_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}
template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
// workgroup barrier for LDS data only: raw s_barrier after an explicit lgkmcnt(0) -- unlike
// __syncthreads() it does not drain LDS-DMA loads still in flight (cdna_hip_programming.md §5)
__device__ __forceinline__ void lds_sync() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  lds_barrier();
}

// sum over the 16 lanes of a DPP row (quad xor-1, quad xor-2, half-row mirror, row mirror): every
// lane of the row ends with the row's sum
template <int CTRL>
__device__ __forceinline__ float dpp_mov(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float row16_sum(float v) {
  v += dpp_mov<0xB1>(v);    // quad_perm(1,0,3,2)
  v += dpp_mov<0x4E>(v);    // quad_perm(2,3,0,1)
  v += dpp_mov<0x141>(v);   // row_half_mirror
  v += dpp_mov<0x140>(v);   // row_mirror
  return v;
}


// SHRED: the epilogue scratch is the fixed region at `smem` (the halo kernel keeps its next tile's
// halo in the rest of LDS): column sums by DPP row reductions, LDS-only barriers
template <int MODE, int BM, int BN, int WM, int WN, int EPI, int NTHR, int EPD = 2, bool SHRED = false>
__device__ __forceinline__ void igemm_epilogue_fd(const IgemmParams& p, f32x4 (&acc)[BN / WN / 16][BM / WM / 16],
                                                  char* smem, int tid, int m0, int n0, int tile_m, int split) {
  constexpr int WTM = BM / WM, WTN = BN / WN;
  constexpr int TM = WTM / 16, TN = WTN / 16;
  constexpr bool PAIR = (TN % 2 == 0);
  const int lane = tid & 63, wid = tid >> 6;
  const int wr = wid / WN, wc = wid % WN;
  const int fr = lane & 15, fq = lane >> 4;
  {
    // lane holds 4 channels chan(j) .. chan(j)+3 per MFMA column tile j of pixel m = m0 + wr*WTM + 16i + fr
    auto chan = [&](int j) {   // channel offset inside the BN tile of acc[j][*][0]
      return PAIR ? wc * WTN + (j >> 1) * 32 + fq * 8 + (j & 1) * 4 : wc * WTN + j * 16 + fq * 4;
    };
    if (p.nsplit > 1) {
      // split-K: raw fp32 partials; the epilogue runs in the reduction kernel
      float* ws = reinterpret_cast<float*>(p.out) + (size_t)split * p.gm * p.gn;
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int m = m0 + wr * WTM + i * 16 + fr;
        if (m >= p.gm) continue;
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int n = n0 + chan(j);
          if (n < p.gn) *reinterpret_cast<f32x4*>(ws + (size_t)m * p.gn + n) = acc[j][i];
        }
      }
      return;   // the split partials are reduced (+ epilogue) by splitk_epilogue_kernel
    }
    __bf16* out = reinterpret_cast<__bf16*>(p.out);
    constexpr int VW = PAIR ? 8 : 4;          // channels per store
    constexpr int NV = TN * 4 / VW;           // stores per pixel row
    constexpr int NP = VW / 2;                // packed bf16 pairs per store
    constexpr bool stats = EPI == EPI_STATS;
    constexpr bool bnr = MODE == MODE_DGRAD && (EPI == EPI_BNR || EPI == EPI_BNR2);
    constexpr bool bnr2 = MODE == MODE_DGRAD && EPI == EPI_BNR2;
    constexpr int NS = bnr2 ? 3 : 2;          // per-channel sums kept
    // GELU forward / backward epilogues (act 2 / 3) exist only in the EPI_GELU instantiations (the
    // Linear GEMMs); compiling them out elsewhere keeps the conv kernels' epilogue code and register
    // budget untouched
    constexpr bool GELU = EPI == EPI_GELU && !SHRED;
    float sm[NS][TN][4];
#pragma unroll
    for (int k = 0; k < NS; ++k)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e) sm[k][j][e] = 0.f;
    const bool has_res = p.resid != nullptr;
    const bool has_mb = bnr && p.bn_mbits != nullptr;
    const bool has_mk = bnr && !has_mb && p.bn_mask != nullptr;
    const bool mfx = bnr && !has_mb && !has_mk && p.bn_msc != nullptr;   // ReLU mask recomputed from x
    // output row offsets of the TM pixel-row groups (rrows: the residual's, -1 = no residual term)
    size_t orows[TM];
    int rrows[MODE == MODE_DGRAD ? TM : 1];
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int m = m0 + wr * WTM + i * 16 + fr;
      size_t orow = m < p.gm ? m : 0;
      if constexpr (MODE == MODE_DGRAD) {
        rrows[i] = (int)orow;
        if ((p.sub || p.resid_sub) && m < p.gm) {
          const int n = fdiv(m, p.fd_HW);
          const int rem = m - n * p.dH * p.dW;
          const int hh = fdiv(rem, p.fd_W);
          const int ww = rem - hh * p.dW;
          if (p.sub) orow = ((size_t)n * p.H + 2 * hh + p.oph) * p.W + 2 * ww + p.opw;
          else rrows[i] = ((hh | ww) & 1) ? -1 : (n * p.rs_H2 + (hh >> 1)) * p.rs_W2 + (ww >> 1);
        }
      }
      orows[i] = orow;
    }
    // Stores walk (i outer, v inner: the two 64-B halves of a pixel's 128-B channel run are stored
    // back to back); the resid / mask / x operand loads of step t+EPD-1 are issued before the math
    // of step t (an EPD-slot register ring: EPD-1 steps of HBM loads in flight per thread).
    constexpr int D = EPD;
    unsigned rvA[D][NP], mkA[D][NP], xvA[D][NP], xv2A[D][NP], mbA[D];
    auto issue = [&](int t, int b) {
      const int i = t / NV, v = t % NV;
      const int m = m0 + wr * WTM + i * 16 + fr;
      const int n = n0 + chan(v * (VW / 4));
      const bool ok = m < p.gm && n < p.gn;
      const size_t o = orows[i] * p.gn + (ok ? n : 0);
      auto ldv = [&](unsigned* d, const __bf16* src) {
        if constexpr (VW == 8) {
          const uint4 t4 = ok ? *reinterpret_cast<const uint4*>(src + o) : uint4{0, 0, 0, 0};
          d[0] = t4.x; d[1] = t4.y; d[2] = t4.z; d[3] = t4.w;
        } else {
          const uint2 t2 = ok ? *reinterpret_cast<const uint2*>(src + o) : uint2{0, 0};
          d[0] = t2.x; d[1] = t2.y;
        }
      };
      if (has_res) {
        if constexpr (MODE == MODE_DGRAD) {
          if (p.resid_sub) {   // sub-sampled residual: zero where rrows < 0
            const bool okr = ok && rrows[i] >= 0;
            const size_t ro = (size_t)(okr ? rrows[i] : 0) * p.gn + (ok ? n : 0);
            if constexpr (VW == 8) {
              const uint4 t4 = okr ? *reinterpret_cast<const uint4*>(p.resid + ro) : uint4{0, 0, 0, 0};
              rvA[b][0] = t4.x; rvA[b][1] = t4.y; rvA[b][2] = t4.z; rvA[b][3] = t4.w;
            } else {
              const uint2 t2 = okr ? *reinterpret_cast<const uint2*>(p.resid + ro) : uint2{0, 0};
              rvA[b][0] = t2.x; rvA[b][1] = t2.y;
            }
          } else {
            ldv(rvA[b], p.resid);
          }
        } else {
          ldv(rvA[b], p.resid);
        }
      }
      if constexpr (bnr) {
        if (has_mb) {   // o is a multiple of VW: the store's channels are bits (o & 7) .. +VW-1 of byte o/8
          const unsigned byte = ok ? p.bn_mbits[o >> 3] : 0u;
          mbA[b] = VW == 8 ? byte : ((byte >> (o & 4)) & 0xfu);
        }
        if (has_mk) ldv(mkA[b], p.bn_mask);
        ldv(xvA[b], p.bn_x);
        if constexpr (bnr2) ldv(xv2A[b], p.bn_x2);
      }
    };
    if (has_res || bnr) {
#pragma unroll
      for (int d = 0; d < D - 1; ++d)
        if (d < NV * TM) issue(d, d);
    }
    // per-channel coefficient tables of the tile's BN columns, staged once in LDS (stage buffers
    // are dead; the column-sum scratch that reuses this space is written after a barrier)
    float* ctab = reinterpret_cast<float*>(smem);
    const bool has_bias = MODE == MODE_FWD && p.bias != nullptr;
    if (bnr || has_bias) {
      for (int idx = tid; idx < BN; idx += NTHR) {
        const int c = min(n0 + idx, p.gn - 1);
        if (has_bias) ctab[idx] = p.bias[c];
        if constexpr (bnr) {
          const float is = p.bn_istd[c];
          ctab[0 * BN + idx] = is;
          ctab[1 * BN + idx] = -p.bn_mean[c] * is;
          ctab[2 * BN + idx] = mfx ? p.bn_msc[c] : 0.f;
          ctab[3 * BN + idx] = mfx ? p.bn_msh[c] : 0.f;
          if constexpr (bnr2) {
            const float is2 = p.bn_istd2[c];
            ctab[4 * BN + idx] = is2;
            ctab[5 * BN + idx] = -p.bn_mean2[c] * is2;
          }
        }
      }
      if constexpr (SHRED) lds_sync(); else __syncthreads();
    }
    auto ldt = [&](float* d, int tab, int j0) {
#pragma unroll
      for (int e4 = 0; e4 < VW; e4 += 4) {
        const f32x4 t4 = *reinterpret_cast<const f32x4*>(ctab + tab * BN + chan(j0) + e4);
        d[e4] = t4[0]; d[e4 + 1] = t4[1]; d[e4 + 2] = t4[2]; d[e4 + 3] = t4[3];
      }
    };
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int m = m0 + wr * WTM + i * 16 + fr;
#pragma unroll
      for (int v = 0; v < NV; ++v) {
        const int t = i * NV + v, b = t % D;
        if ((has_res || bnr) && t + D - 1 < NV * TM) issue(t + D - 1, (t + D - 1) % D);
        const int j0 = v * (VW / 4);
        const int n = n0 + chan(j0);
        if (m >= p.gm || n >= p.gn) continue;
        const size_t o = orows[i] * p.gn + n;
        float bias[VW], ka[VW], kb[VW], ka2[VW], kb2[VW], msc[VW], msh[VW];
        if (has_bias) ldt(bias, 0, j0);
        else {
#pragma unroll
          for (int e = 0; e < VW; ++e) bias[e] = 0.f;
        }
        if constexpr (bnr) {
          ldt(ka, 0, j0); ldt(kb, 1, j0);
          if (mfx) { ldt(msc, 2, j0); ldt(msh, 3, j0); }
          if constexpr (bnr2) { ldt(ka2, 4, j0); ldt(kb2, 5, j0); }
        }
        unsigned ov[NP], av[NP];
#pragma unroll
        for (int q = 0; q < NP; ++q) {
          const int j = j0 + (q >> 1), e0 = (q & 1) * 2, ce = 2 * q;   // ce: channel within the store
          float x0 = acc[j][i][e0] + bias[ce];
          float x1 = acc[j][i][e0 + 1] + bias[ce + 1];
          if (has_res) {
            const float r0 = __uint_as_float(rvA[b][q] << 16), r1 = __uint_as_float(rvA[b][q] & 0xffff0000u);
            if (GELU && p.relu == 3) { x0 *= dgelu_fast(r0); x1 *= dgelu_fast(r1); }
            else { x0 += r0; x1 += r1; }
          }
          if constexpr (GELU) {
            if (p.relu == 1) { x0 = fmaxf(x0, 0.f); x1 = fmaxf(x1, 0.f); }
            else if (p.relu == 2) {   // u (bf16) -> aux; out = gelu(u) as the separate kernel would
              const unsigned uu = f2bf2(x0, x1);
              av[q] = uu;
              x0 = gelu_fast(__uint_as_float(uu << 16));
              x1 = gelu_fast(__uint_as_float(uu & 0xffff0000u));
            }
          } else if (p.relu) { x0 = fmaxf(x0, 0.f); x1 = fmaxf(x1, 0.f); }
          unsigned u = f2bf2(x0, x1);
          if constexpr (bnr) {
            const float xa = __uint_as_float(xvA[b][q] << 16), xb = __uint_as_float(xvA[b][q] & 0xffff0000u);
            // g = round(dgrad) masked by the forward ReLU output (> 0: sign clear and nonzero)
            if (has_mb) {
              const unsigned bits = mbA[b] >> ce;
              u &= ((bits & 1u) ? 0x0000ffffu : 0u) | ((bits & 2u) ? 0xffff0000u : 0u);
            } else if (has_mk) {
              const unsigned y = mkA[b][q];
              const unsigned keep = (((y & 0x8000u) == 0 && (y & 0x7fffu) != 0) ? 0x0000ffffu : 0u) |
                                    (((y & 0x80000000u) == 0 && (y & 0x7fff0000u) != 0) ? 0xffff0000u : 0u);
              u &= keep;
            } else if (mfx) {
              const float z0 = fmaf(xa, msc[ce], msh[ce]);
              const float z1 = fmaf(xb, msc[ce + 1], msh[ce + 1]);
              u &= (z0 > 0.f ? 0x0000ffffu : 0u) | (z1 > 0.f ? 0xffff0000u : 0u);
            }
            const float r0 = __uint_as_float(u << 16), r1 = __uint_as_float(u & 0xffff0000u);
            sm[0][j][e0] += r0; sm[0][j][e0 + 1] += r1;
            sm[1][j][e0] += r0 * fmaf(xa, ka[ce], kb[ce]);
            sm[1][j][e0 + 1] += r1 * fmaf(xb, ka[ce + 1], kb[ce + 1]);
            if constexpr (bnr2) {
              sm[2][j][e0] += r0 * fmaf(__uint_as_float(xv2A[b][q] << 16), ka2[ce], kb2[ce]);
              sm[2][j][e0 + 1] += r1 * fmaf(__uint_as_float(xv2A[b][q] & 0xffff0000u), ka2[ce + 1], kb2[ce + 1]);
            }
          } else if constexpr (stats) {
            const float r0 = __uint_as_float(u << 16), r1 = __uint_as_float(u & 0xffff0000u);
            sm[0][j][e0] += r0; sm[0][j][e0 + 1] += r1;
            sm[1][j][e0] += r0 * r0; sm[1][j][e0 + 1] += r1 * r1;
          }
          ov[q] = u;
        }
        if constexpr (VW == 8) *reinterpret_cast<uint4*>(out + o) = *reinterpret_cast<const uint4*>(ov);
        else *reinterpret_cast<uint2*>(out + o) = *reinterpret_cast<const uint2*>(ov);
        if constexpr (GELU) {
          if (p.relu == 2) {
            if constexpr (VW == 8) *reinterpret_cast<uint4*>(p.aux + o) = *reinterpret_cast<const uint4*>(av);
            else *reinterpret_cast<uint2*>(p.aux + o) = *reinterpret_cast<const uint2*>(av);
          }
        }
      }
    }
    if constexpr (stats || bnr) {
      float* red;   // [WM][NS][BN] per-wave-row partial column sums
      if constexpr (SHRED) {
        red = reinterpret_cast<float*>(smem) + 6 * BN;   // after the coefficient rows
#pragma unroll
        for (int k = 0; k < NS; ++k)
#pragma unroll
          for (int j = 0; j < TN; ++j) {
            f32x4 v;
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = row16_sum(sm[k][j][e]);
            if (fr == 0) *reinterpret_cast<f32x4*>(red + (wr * NS + k) * BN + chan(j)) = v;
          }
        lds_sync();
      } else {
      // Column sums over the tile's pixels: each wave transposes its lanes' partial sums through
      // LDS ([16 pixel rows][NS][WTN], padded rows) and every lane then sums 16 values for its
      // (k, channel) pairs -- ~3 LDS ops per value instead of a 4-step cross-lane reduction.
      constexpr int RS = NS * WTN + 4;
      float* tb = reinterpret_cast<float*>(smem) + wid * 16 * RS;
      red = reinterpret_cast<float*>(smem) + (NTHR / 64) * 16 * RS;   // [WM][NS][BN]
      __syncthreads();   // stage buffers are dead from here on
#pragma unroll
      for (int k = 0; k < NS; ++k)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          *reinterpret_cast<f32x4*>(tb + fr * RS + k * WTN + chan(j) - wc * WTN) =
              f32x4{sm[k][j][0], sm[k][j][1], sm[k][j][2], sm[k][j][3]};
      __syncthreads();
#pragma unroll
      for (int idx = lane; idx < NS * WTN; idx += 64) {
        const int k = idx / WTN, ch = idx - k * WTN;
        float t = 0.f;
#pragma unroll
        for (int r = 0; r < 16; ++r) t += tb[r * RS + k * WTN + ch];
        red[(wr * NS + k) * BN + wc * WTN + ch] = t;
      }
      __syncthreads();
      }
      float* st = p.stats + (size_t)tile_m * 2 * p.gn;
      float* st2 = bnr2 ? p.stats2 + (size_t)tile_m * 2 * p.gn : nullptr;
      for (int i = tid; i < BN; i += NTHR) {
        const int c = n0 + i;
        if (c < p.gn) {
          float t[NS];
#pragma unroll
          for (int k = 0; k < NS; ++k) {
            t[k] = 0.f;
#pragma unroll
            for (int w = 0; w < WM; ++w) t[k] += red[(w * NS + k) * BN + i];
          }
          st[c] = t[0];
          st[p.gn + c] = t[1];
          if constexpr (bnr2) {
            st2[c] = t[0];
            st2[p.gn + c] = t[2];
          }
        }
      }
    }
  }
}

// FOLD (bitmask): 1 = the A operand is formed while staging -- DGRAD / WGRAD: dz of the BatchNorm-
// backward fold (fold_x, fold_coef); FWD: relu(a*z + b) of the BatchNorm-forward fold (act_sc/sh);
// 2 = WGRAD's B operand (x) is relu(a*z + b) (act_sc / act_sh)
// M32 (WGRAD only): the MFMAs are v_mfma_f32_32x32x16_bf16 on 32x32 sub-tiles of the wave tile
// (fragments from the same k-major LDS image through ds_read_b64_tr_b16, one 16-lane group per
// (16-column half, 8-deep k half)): half the MFMA instructions, same LDS bytes (knob wgrad_m32)
template <int MODE, int BM, int BN, int WM, int WN, bool UNIF, int EPI, int EPD = 2, int NTHR = NT, int FOLD = 0,
          bool M32_ = false>
__global__ void __launch_bounds__(NTHR, NTHR == NT ? 2 : 1) igemm_kernel(const IgemmParams p) {
  constexpr int WTM = BM / WM, WTN = BN / WN;   // wave tile
  constexpr int TM = WTM / 16, TN = WTN / 16;   // 16x16 MFMA tiles per wave
  constexpr int A_BYTES = BM * BK * 2, B_BYTES = BN * BK * 2;
  constexpr int STAGE = A_BYTES + B_BYTES;
  constexpr int NVA = BM * BK / 8 / NTHR;  // 16-B vectors per thread per stage
  constexpr int NVB = BN * BK / 8 / NTHR;
  static_assert(NVA >= 1 && NVB >= 1, "tile too small");
  static_assert(WM * WN == NTHR / 64, "one wave tile per wave");
  constexpr bool FA = (FOLD & 1) != 0, FB = (FOLD & 2) != 0;
  constexpr bool FAX = FA && MODE != MODE_FWD;   // A fold reading a second tensor (dz = f(g, x))
  static_assert(!FA || MODE == MODE_WGRAD || UNIF, "fold: FWD / DGRAD need the block-uniform walk");
  static_assert(!FB || MODE == MODE_WGRAD, "fold: B-operand fold is WGRAD only");
  static_assert(NVA <= 32 && NVB <= 32, "fold: row-valid bits");

  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid / WN, wc = wid % WN;

  // ---- tile coordinates ---------------------------------------------------------------------
  const int nwg = gridDim.x;
  const int lin = xcd_remap(blockIdx.x, nwg);
  const int tiles_mn = p.tiles_m * p.tiles_n;
  const int split = lin / tiles_mn;
  const int t = lin - split * tiles_mn;
  const int tile_n = t % p.tiles_n;
  const int tile_m = t / p.tiles_n;
  const int m0 = tile_m * BM, n0 = tile_n * BN;
  const int kbeg = split * p.ksplit;
  const int kend = min(p.gk, kbeg + p.ksplit);
  const int nk = (kend - kbeg + BK - 1) / BK;

  // FWD/DGRAD compute D^T tiles (weights as the MFMA A operand) so each lane ends up holding 4
  // consecutive output channels of one pixel -> direct 8-byte stores, no LDS staging.
  // PAIR: output-channel permutation inside each 32-channel group of the B (weight) tile so that a
  // lane's two MFMA column tiles 2jp, 2jp+1 hold 8 CONSECUTIVE channels -> 16-B epilogue stores.
  constexpr bool PAIR = MODE != MODE_WGRAD && (TN % 2 == 0);
  constexpr int AT0 = (MODE == MODE_WGRAD) ? TM : TN;
  constexpr int AT1 = (MODE == MODE_WGRAD) ? TN : TM;
  f32x4 acc[AT0][AT1];
#pragma unroll
  for (int i = 0; i < AT0; ++i)
#pragma unroll
    for (int j = 0; j < AT1; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  constexpr bool M32 = M32_ && MODE == MODE_WGRAD;
  static_assert(!M32 || (WTM % 32 == 0 && WTN % 32 == 0), "M32: 32-multiple wave tiles");
  constexpr int TM32 = M32 ? WTM / 32 : 1, TN32 = M32 ? WTN / 32 : 1;
  f32x16 acc32[TM32][TN32];
#pragma unroll
  for (int i = 0; i < TM32; ++i)
#pragma unroll
    for (int j = 0; j < TN32; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc32[i][j][r] = 0.f;

  uint4 ra[NVA], rb[NVB];

  const __amdgpu_buffer_rsrc_t rsA = make_rsrc(p.a, p.a_bytes);
  const __amdgpu_buffer_rsrc_t rsB = make_rsrc(p.b, p.b_bytes);
  // BatchNorm-backward fold: x chunks beside the g chunks, row-valid bits, channel of the stage
  uint4 rx[FAX ? NVA : 1];
  unsigned fold_ok = 0, fold_okb = 0;
  int fold_chan = 0;
  const __amdgpu_buffer_rsrc_t rsX = make_rsrc(FAX ? p.fold_x : p.a, p.a_bytes);

  // ---- per-thread loader state ----------------------------------------------------------------
  const int lchunk = tid & 7;
  const int lrow = tid >> 3;
  int a_off[NVA];            // FWD/DGRAD: element offset of row's (tap 0) base; WGRAD unused
  int a_y[NVA], a_x[NVA];    // bounds coordinates (invalid rows get a huge negative a_y)
  int b_off[NVB];            // FWD/DGRAD: n*gk (or -1 for n >= gn)
  constexpr int CPR_A = BM / 8, CPR_B = BN / 8;
  int wa_col = 0, wb_col = 0;
  int wb_r = 0, wb_s = 0, wb_c = 0, wb_ok = 0;
  int kr = 0, ks = 0, kc = 0;     // tap / channel state (uniform when UNIF)
  const int CIN = (MODE == MODE_FWD) ? p.C : p.K;

  if constexpr (MODE != MODE_WGRAD) {
#pragma unroll
    for (int i = 0; i < NVA; ++i) {
      const int m = m0 + lrow + (NTHR / 8) * i;
      const bool v = m < p.gm;
      const int mm = v ? m : 0;
      if constexpr (MODE == MODE_FWD) {
        const int n = fdiv(mm, p.fd_PQ);
        const int rem = mm - n * p.P * p.Q;
        const int pp = fdiv(rem, p.fd_Q);
        const int qq = rem - pp * p.Q;
        const int yv = pp * p.stride - p.pad;
        a_y[i] = v ? yv : -(1 << 28);
        a_x[i] = qq * p.stride - p.pad;
        a_off[i] = ((n * p.H + yv) * p.W + a_x[i]) * p.C;
      } else {
        const int n = fdiv(mm, p.fd_HW);
        const int rem = mm - n * p.dH * p.dW;
        const int hh = fdiv(rem, p.fd_W);
        const int ww = rem - hh * p.dW;
        const int yv = hh + p.offy;
        a_y[i] = v ? yv : -(1 << 28);
        a_x[i] = ww + p.offx;
        a_off[i] = ((n * p.P + yv) * p.Q + a_x[i]) * p.K;
      }
    }
#pragma unroll
    for (int i = 0; i < NVB; ++i) {
      const int n = n0 + chan_perm<PAIR>(lrow + (NTHR / 8) * i);
      b_off[i] = n < p.gn ? n * p.gk : -1;
    }
    if constexpr (UNIF) {
      kc = kbeg % CIN;
      const int rs = kbeg / CIN;
      ks = rs % p.S;
      kr = rs / p.S;
    } else {
      const int k = kbeg + lchunk * 8;
      kc = k % CIN;
      const int rs = k / CIN;
      ks = rs % p.S;
      kr = rs / p.S;
    }
  } else {
    wa_col = (tid % CPR_A) * 8;
    wb_col = (tid % CPR_B) * 8;
    const int j = n0 + wb_col;
    wb_ok = j < p.gn;
    const int jj = wb_ok ? j : 0;
    wb_c = jj % p.C;
    const int rs = jj / p.C;
    wb_s = rs % p.S;
    wb_r = rs / p.S;
  }
  // WGRAD operand walks, advanced incrementally by BK reduction rows per K-step (no per-step
  // divisions / 32-bit multiplies: those made the loader VALU-bound, profiles/r1_pmc_mix.txt):
  //   A' row m: element offset m*K + co;
  //   B' row m = (n, pp, qq): im2col base ((n*H + pp*st)*W + qq*st)*C, kept with ps = pp*st and
  //   qs = qq*st; +BK rows = (+dn, +dp, +dq) with at most one carry into pp and one into n.
  int wa_off[MODE == MODE_WGRAD ? NVA : 1];
  int wb_off[MODE == MODE_WGRAD ? NVB : 1], wb_ps[MODE == MODE_WGRAD ? NVB : 1], wb_qs[MODE == MODE_WGRAD ? NVB : 1];
  int wg_dqs = 0, wg_Qs = 0, wg_dps = 0, wg_Ps = 0, wg_A0 = 0, wg_A1 = 0, wg_A2 = 0, wb_coloff = 0;
  if constexpr (MODE == MODE_WGRAD) {
    const int st = p.stride;
    const int dq = BK % p.Q, dp = (BK / p.Q) % p.P, dn = BK / (p.P * p.Q);
    wg_dqs = dq * st; wg_Qs = p.Q * st; wg_dps = dp * st; wg_Ps = p.P * st;
    const int WC = p.W * p.C;
    wg_A0 = dq * st * p.C + dp * st * WC + dn * p.H * WC;
    wg_A1 = st * WC - p.Q * st * p.C;
    wg_A2 = p.H * WC - p.P * st * WC;
    wb_coloff = ((wb_r - p.pad) * p.W + (wb_s - p.pad)) * p.C + wb_c;
#pragma unroll
    for (int i = 0; i < NVA; ++i) {
      const int row = (tid + NTHR * i) / CPR_A;
      wa_off[i] = (kbeg + row) * p.K + m0 + wa_col;
    }
#pragma unroll
    for (int i = 0; i < NVB; ++i) {
      const int row = (tid + NTHR * i) / CPR_B;
      const int m = min(kbeg + row, p.gk);   // rows past gk are masked; keep the decomposition in range
      const int n = fdiv(m, p.fd_PQ);
      const int rem = m - n * p.P * p.Q;
      const int pp = fdiv(rem, p.fd_Q);
      const int qq = rem - pp * p.Q;
      wb_ps[i] = pp * st;
      wb_qs[i] = qq * st;
      wb_off[i] = ((n * p.H + pp * st) * p.W + qq * st) * p.C;
    }
  }

  // fold coefficients: WGRAD -- the thread's 8 output channels m0 + wa_col .. +7 are fixed, so
  // their k1/k2/k3 live in registers; DGRAD -- the stage's reduction channels change per K-step, so
  // the block copies fold_coef [3][K] into LDS once (after every buffer the kernel uses)
  float wk1[MODE == MODE_WGRAD && FA ? 8 : 1], wk2[MODE == MODE_WGRAD && FA ? 8 : 1],
      wk3[MODE == MODE_WGRAD && FA ? 8 : 1];
  float bsc[FB ? 8 : 1], bsh[FB ? 8 : 1];   // WGRAD B fold: the thread's 8 input channels are fixed
  if constexpr (FB) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const f32x4 a = wb_ok ? *reinterpret_cast<const f32x4*>(p.act_sc + wb_c + 4 * h) : f32x4{0.f, 0.f, 0.f, 0.f};
      const f32x4 b = wb_ok ? *reinterpret_cast<const f32x4*>(p.act_sh + wb_c + 4 * h) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int e = 0; e < 4; ++e) { bsc[4 * h + e] = a[e]; bsh[4 * h + e] = b[e]; }
    }
  }
  if constexpr (FA) {
    if constexpr (MODE == MODE_WGRAD) {
      const int co = m0 + wa_col;
      const bool cok = co < p.gm;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const f32x4 a = cok ? *reinterpret_cast<const f32x4*>(p.fold_coef + co + 4 * h) : f32x4{0.f, 0.f, 0.f, 0.f};
        const f32x4 b = cok ? *reinterpret_cast<const f32x4*>(p.fold_coef + p.gm + co + 4 * h) : f32x4{0.f, 0.f, 0.f, 0.f};
        const f32x4 c = cok ? *reinterpret_cast<const f32x4*>(p.fold_coef + 2 * p.gm + co + 4 * h) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int e = 0; e < 4; ++e) { wk1[4 * h + e] = a[e]; wk2[4 * h + e] = b[e]; wk3[4 * h + e] = c[e]; }
      }
    } else if constexpr (MODE == MODE_DGRAD) {
      f32x4* dst = reinterpret_cast<f32x4*>(smem + p.fold_lds);
      for (int i = tid; i < 3 * p.K / 4; i += NTHR) dst[i] = reinterpret_cast<const f32x4*>(p.fold_coef)[i];
      __syncthreads();
    } else {   // FWD: [scale | shift] of the C input channels
      f32x4* dst = reinterpret_cast<f32x4*>(smem + p.fold_lds);
      const int nv = p.C / 4;
      for (int i = tid; i < 2 * nv; i += NTHR)
        dst[i] = i < nv ? reinterpret_cast<const f32x4*>(p.act_sc)[i] : reinterpret_cast<const f32x4*>(p.act_sh)[i - nv];
      __syncthreads();
    }
  }

  auto load_stage = [&](int kt) {
    const int k0 = kbeg + kt * BK;
    if constexpr (MODE != MODE_WGRAD) {
      int tap, chan;
      if constexpr (UNIF) {
        chan = kc + lchunk * 8;
        if constexpr (MODE == MODE_FWD) tap = (kr * p.W + ks) * p.C;
        else tap = -(kr * p.Q + ks) * p.K;
      } else {
        chan = kc;
        if constexpr (MODE == MODE_FWD) tap = (kr * p.W + ks) * p.C;
        else tap = -(kr * p.Q + ks) * p.K;
      }
      const bool kok = UNIF ? true : (k0 + lchunk * 8 < kend);
      if constexpr (FA) fold_chan = chan;   // 1x1: the reduction index is the channel
#pragma unroll
      for (int i = 0; i < NVA; ++i) {
        bool ok;
        if constexpr (MODE == MODE_FWD) {
          ok = (unsigned)(a_y[i] + kr) < (unsigned)p.H && (unsigned)(a_x[i] + ks) < (unsigned)p.W;
        } else {
          if (p.stride != 1 && !p.sub) {
            // generic strided dgrad (not used for stride 2: sub-pixel classes) -- exact checks
            const int ph = a_y[i] - kr, pw = a_x[i] - ks;
            ok = ph >= 0 && pw >= 0 && (ph % p.stride) == 0 && (pw % p.stride) == 0 &&
                 ph / p.stride < p.P && pw / p.stride < p.Q;
          } else {
            ok = (unsigned)(a_y[i] - kr) < (unsigned)p.P && (unsigned)(a_x[i] - ks) < (unsigned)p.Q;
          }
        }
        ok = ok && kok;
        const unsigned voff = ok ? (unsigned)(a_off[i] + tap + chan) * 2u : kOOB;
        ra[i] = bload16(rsA, voff);
        if constexpr (FA) {
          if constexpr (FAX) rx[i] = bload16(rsX, voff);
          fold_ok = ok ? (fold_ok | (1u << i)) : (fold_ok & ~(1u << i));
        }
      }
      const int kk = k0 + lchunk * 8;
#pragma unroll
      for (int i = 0; i < NVB; ++i) {
        const bool ok = b_off[i] >= 0 && kk < kend;
        rb[i] = bload16(rsB, ok ? (unsigned)(b_off[i] + kk) * 2u : kOOB);
      }
      // advance (r,s,c) by BK
      if constexpr (UNIF) {
        kc += BK;
        if (kc >= CIN) {
          kc = 0;
          if (++ks == p.S) { ks = 0; ++kr; }
        }
      } else {
        kc += BK;
        while (kc >= CIN) {
          kc -= CIN;
          if (++ks == p.S) { ks = 0; ++kr; }
        }
      }
    } else {
      // A': rows = reduction index m, cols = output channel co (dy rows are contiguous in co)
      const bool co_ok = m0 + wa_col < p.gm;
#pragma unroll
      for (int i = 0; i < NVA; ++i) {
        const int row = (tid + NTHR * i) / CPR_A;
        const bool ok = co_ok && k0 + row < kend;
        ra[i] = bload16(rsA, ok ? (unsigned)wa_off[i] * 2u : kOOB);
        if constexpr (FA) {
          rx[i] = bload16(rsX, ok ? (unsigned)wa_off[i] * 2u : kOOB);
          fold_ok = ok ? (fold_ok | (1u << i)) : (fold_ok & ~(1u << i));
        }
        wa_off[i] += BK * p.K;
      }
      // B': rows = m, cols = j=(r,s,c): im2col gather of x (a specialised linear walk for 1x1
      // stride-1 convs measured neutral in the step, profiles/r5_wgrad_experiments.txt)
#pragma unroll
      for (int i = 0; i < NVB; ++i) {
        const int row = (tid + NTHR * i) / CPR_B;
        const int yy = wb_ps[i] - p.pad + wb_r;
        const int xx = wb_qs[i] - p.pad + wb_s;
        const bool ok = wb_ok && k0 + row < kend && (unsigned)yy < (unsigned)p.H && (unsigned)xx < (unsigned)p.W;
        rb[i] = bload16(rsB, ok ? (unsigned)(wb_off[i] + wb_coloff) * 2u : kOOB);
        if constexpr (FB) fold_okb = ok ? (fold_okb | (1u << i)) : (fold_okb & ~(1u << i));
        // advance the walk by BK rows
        int qs = wb_qs[i] + wg_dqs;
        const bool c1 = qs >= wg_Qs;
        qs -= c1 ? wg_Qs : 0;
        int ps = wb_ps[i] + wg_dps + (c1 ? p.stride : 0);
        const bool c2 = ps >= wg_Ps;
        ps -= c2 ? wg_Ps : 0;
        wb_qs[i] = qs;
        wb_ps[i] = ps;
        wb_off[i] += wg_A0 + (c1 ? wg_A1 : 0) + (c2 ? wg_A2 : 0);
      }
    }
  };

  auto store_stage = [&](int buf) {
    char* sA = smem + buf * STAGE;
    char* sB = sA + A_BYTES;
    if constexpr (FB) {
#pragma unroll
      for (int i = 0; i < NVB; ++i) rb[i] = fold_act(rb[i], bsc, bsh, (fold_okb >> i) & 1u);
    }
    if constexpr (FA && MODE == MODE_FWD) {
      const float* cf = reinterpret_cast<const float*>(smem + p.fold_lds) + fold_chan;
      float a[8], b[8];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const f32x4 u = *reinterpret_cast<const f32x4*>(cf + 4 * h);
        const f32x4 v = *reinterpret_cast<const f32x4*>(cf + p.C + 4 * h);
#pragma unroll
        for (int e = 0; e < 4; ++e) { a[4 * h + e] = u[e]; b[4 * h + e] = v[e]; }
      }
#pragma unroll
      for (int i = 0; i < NVA; ++i) ra[i] = fold_act(ra[i], a, b, (fold_ok >> i) & 1u);
    }
    if constexpr (FAX) {
      if constexpr (MODE == MODE_WGRAD) {
#pragma unroll
        for (int i = 0; i < NVA; ++i) ra[i] = fold_dz(ra[i], rx[i], wk1, wk2, wk3, (fold_ok >> i) & 1u);
      } else {
        const float* cf = reinterpret_cast<const float*>(smem + p.fold_lds) + fold_chan;
        float k1[8], k2[8], k3[8];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const f32x4 a = *reinterpret_cast<const f32x4*>(cf + 4 * h);
          const f32x4 b = *reinterpret_cast<const f32x4*>(cf + p.K + 4 * h);
          const f32x4 c = *reinterpret_cast<const f32x4*>(cf + 2 * p.K + 4 * h);
#pragma unroll
          for (int e = 0; e < 4; ++e) { k1[4 * h + e] = a[e]; k2[4 * h + e] = b[e]; k3[4 * h + e] = c[e]; }
        }
#pragma unroll
        for (int i = 0; i < NVA; ++i) ra[i] = fold_dz(ra[i], rx[i], k1, k2, k3, (fold_ok >> i) & 1u);
      }
    }
    if constexpr (MODE != MODE_WGRAD) {
#pragma unroll
      for (int i = 0; i < NVA; ++i)
        *reinterpret_cast<uint4*>(sA + rr_off(lrow + (NTHR / 8) * i, lchunk)) = ra[i];
#pragma unroll
      for (int i = 0; i < NVB; ++i)
        *reinterpret_cast<uint4*>(sB + rr_off(lrow + (NTHR / 8) * i, lchunk)) = rb[i];
    } else {
#pragma unroll
      for (int i = 0; i < NVA; ++i) {
        const int v = tid + NTHR * i;
        *reinterpret_cast<uint4*>(sA + tr_off<BM, M32>(v / CPR_A, wa_col)) = ra[i];
      }
#pragma unroll
      for (int i = 0; i < NVB; ++i) {
        const int v = tid + NTHR * i;
        *reinterpret_cast<uint4*>(sB + tr_off<BN, M32>(v / CPR_B, wb_col)) = rb[i];
      }
    }
  };

  typedef short s16x4 __attribute__((ext_vector_type(4)));
  typedef __attribute__((address_space(3))) s16x4 lds_s16x4_t;
  typedef short s16x8 __attribute__((ext_vector_type(8)));

  auto compute_stage = [&](int buf) {
    const char* sA = smem + buf * STAGE;
    const char* sB = sA + A_BYTES;
    if constexpr (M32) {
      // lane group g = lane >> 4 reads columns 16 * (g & 1) .. +15 of a 32-column slice at k rows
      // 8 * (g >> 1) .. +7 of the 16-deep step: lane l ends with column (l & 31), k 8 * (l >> 5) .. +7
      const int g = lane >> 4, q = (lane >> 2) & 3, pc = (lane & 3) * 4;
#pragma unroll
      for (int kq = 0; kq < BK / 16; ++kq) {
        const int rowb = kq * 16 + 8 * (g >> 1) + q;
        bf16x8 fa[TM32], fb[TN32];
#pragma unroll
        for (int i = 0; i < TM32; ++i) {
          const int col = wr * WTM + i * 32 + 16 * (g & 1) + pc;
          s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t*)(sA + tr_off<BM, true>(rowb, col)));
          s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t*)(sA + tr_off<BM, true>(rowb + 4, col)));
          fa[i] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
        }
#pragma unroll
        for (int j = 0; j < TN32; ++j) {
          const int col = wc * WTN + j * 32 + 16 * (g & 1) + pc;
          s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t*)(sB + tr_off<BN, true>(rowb, col)));
          s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t*)(sB + tr_off<BN, true>(rowb + 4, col)));
          fb[j] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
        }
#pragma unroll
        for (int i = 0; i < TM32; ++i)
#pragma unroll
          for (int j = 0; j < TN32; ++j)
            acc32[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i], fb[j], acc32[i][j], 0, 0, 0);
      }
      return;
    }
#pragma unroll
    for (int kk = 0; kk < BK / 32; ++kk) {
      bf16x8 fa[TM], fb[TN];
      if constexpr (MODE != MODE_WGRAD) {
        const int chunk = kk * 4 + (lane >> 4);
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          const int row = wr * WTM + i * 16 + (lane & 15);
          fa[i] = *reinterpret_cast<const bf16x8*>(sA + rr_off(row, chunk));
        }
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int row = wc * WTN + j * 16 + (lane & 15);
          fb[j] = *reinterpret_cast<const bf16x8*>(sB + rr_off(row, chunk));
        }
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
          for (int i = 0; i < TM; ++i)
            acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[j], fa[i], acc[j][i], 0, 0, 0);
      } else {
        const int g = lane >> 4, q = (lane >> 2) & 3, pc = (lane & 3) * 4;
        const int rowb = kk * 32 + 8 * g + q;
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          const int col = wr * WTM + i * 16 + pc;
          s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t*)(sA + tr_off<BM>(rowb, col)));
          s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t*)(sA + tr_off<BM>(rowb + 4, col)));
          fa[i] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
        }
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int col = wc * WTN + j * 16 + pc;
          s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t*)(sB + tr_off<BN>(rowb, col)));
          s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t*)(sB + tr_off<BN>(rowb + 4, col)));
          fb[j] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
        }
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
      }
    }
  };

  // ---- main loop: register-staged double buffer, one barrier per K-step ------------------------
  if (nk > 0) {
    load_stage(0);
    store_stage(0);
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
      const int cur = kt & 1;
      if (kt + 1 < nk) load_stage(kt + 1);
      compute_stage(cur);
      if (kt + 1 < nk) store_stage(cur ^ 1);
      __syncthreads();
    }
  }

  // ---- epilogue -------------------------------------------------------------------------------
  const int fr = lane & 15, fq = lane >> 4;
  if constexpr (M32) {
    // 32x32 accumulator: column (lane & 31), register r -> row 8 * (r / 4) + 4 * (lane >> 5) + r % 4
    float* out = reinterpret_cast<float*>(p.out) + (size_t)split * p.gm * p.gn;
#pragma unroll
    for (int i = 0; i < TM32; ++i)
#pragma unroll
      for (int j = 0; j < TN32; ++j) {
        const int col = n0 + wc * WTN + j * 32 + (lane & 31);
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = m0 + wr * WTM + i * 32 + 8 * (r >> 2) + 4 * (lane >> 5) + (r & 3);
          if (row < p.gm && col < p.gn) {
            float v = acc32[i][j][r] * p.alpha;
            float* dst = out + (size_t)row * p.gn + col;
            if (p.accumulate) v += *dst;
            *dst = v;
          }
        }
      }
    return;
  } else if constexpr (MODE == MODE_WGRAD) {
    float* out = reinterpret_cast<float*>(p.out) + (size_t)split * p.gm * p.gn;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int col = n0 + wc * WTN + j * 16 + fr;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int row = m0 + wr * WTM + i * 16 + fq * 4 + e;
          if (row < p.gm && col < p.gn) {
            float v = acc[i][j][e] * p.alpha;
            float* dst = out + (size_t)row * p.gn + col;
            if (p.accumulate) v += *dst;
            *dst = v;
          }
        }
      }
    return;
  } else {
    igemm_epilogue_fd<MODE, BM, BN, WM, WN, EPI, NTHR, EPD>(p, acc, smem, tid, m0, n0, tile_m, split);
  }
}

// ------------------------------------------------------------------------------------------------
// LDS-DMA kernel for FWD/DGRAD GEMMs with the block-uniform tap walk.  Two instantiations:
//   8 waves, BM = 256 x BN = 256 (2x4 waves, 128x64 wave tiles), 1 block per CU -- large grids;
//   4 waves, BM x BN = 128x128 / 256x64 (64x64 wave tiles), 2 blocks per CU -- everything else.
// Operand tiles are staged global -> LDS by buffer_load ... lds (LDS-DMA: no VGPR round trip and no
// ds_write -- the register-staged kernel's 16-B LDS stores transfer at ~79 B/clk/CU, a third of the
// ds_read_b128 rate -- and hardware zero-fill for padding / tails through the buffer range check);
// the XOR swizzle of the row-read image is applied to the per-lane SOURCE chunk and undone on the
// ds_read (cdna_hip_programming.md §5.4 rule 21).  Each K-tile (BK = 64) is computed in four
// phases, one output quadrant per phase; during phase p of tile t the p-th half-tile of tile t+1
// is DMA'd into the other LDS buffer, and counted s_waitcnt vmcnt(N) waits retire exactly the
// half-tile the next phase reads, so operand loads stay in flight across the barriers instead of
// draining every K-step.  Half-tile issue order (A0, B0, B1, A1) follows the quadrant order
// (0,0) (0,1) (1,1) (1,0) of the consumer.
constexpr int NT8 = 512;
constexpr int BM8 = 256;


// Schedule: early prefetch -- each half-tile of tile t+2 is DMA'd into the buffer being read as soon
// as its tile-t half has been consumed (4-7 phases of lead, one counted vmcnt per K-tile; +0.7 % on
// the ResNet-50 step over the lock-step 4-phase schedule, profiles/r3_prio_pf2_ab.txt; the lock-step
// and wave-row-staggered schedules were removed in round 4)
template <int MODE, int BM, int BN, int WM, int WN, int NTHR, int MINB, int EPI, int EPD = 2>
__global__ void __launch_bounds__(NTHR, MINB) igemm_dma_kernel(const IgemmParams p) {
  constexpr int NW = NTHR / 64;
  constexpr int WTM = BM / WM, WTN = BN / WN;
  constexpr int TM = WTM / 16, TN = WTN / 16;
  constexpr int TMH = TM / 2, TNH = TN / 2;     // fragments per quadrant
  constexpr int A_BYTES = BM * BK * 2, B_BYTES = BN * BK * 2;
  constexpr int STAGE = A_BYTES + B_BYTES;
  constexpr int NA = BM / 16 / NW;              // LDS-DMA instructions (8 rows each) per wave per A half-tile
  constexpr int NB = BN / 16 / NW;              // ... per B half-tile
  constexpr int AH = WTM / 2, BH = WTN / 2;     // rows of one wave-row / wave-column segment of a half
  static_assert(MODE != MODE_WGRAD, "FWD/DGRAD only");
  static_assert(WM * WN == NW, "one wave tile per wave");
  static_assert(NA >= 1 && NB >= 1 && NA * NW * 16 == BM && NB * NW * 16 == BN, "loader slots");
  static_assert(AH % 8 == 0 && BH % 8 == 0 && TM % 2 == 0 && TN % 2 == 0, "quadrants");
  static_assert(WTN % 32 == 0, "PAIR channel permutation works on 32-row groups");

  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid / WN, wc = wid % WN;

  const int lin = xcd_remap(blockIdx.x, gridDim.x);
  // split-K (plain GEMMs with too few tiles to fill the chip): consecutive blocks on one XCD take
  // the splits of one tile; each split writes raw fp32 partials reduced by splitk_epilogue_kernel
  const int tiles_mn = p.tiles_m * p.tiles_n;
  const int split = lin / tiles_mn;
  const int tl = lin - split * tiles_mn;
  const int tile_n = tl % p.tiles_n;
  const int tile_m = tl / p.tiles_n;
  const int m0 = tile_m * BM, n0 = tile_n * BN;
  const int kbeg = split * p.ksplit;
  const int nk = (min(p.gk, kbeg + p.ksplit) - kbeg) / BK;

  f32x4 acc[TN][TM];
#pragma unroll
  for (int j = 0; j < TN; ++j)
#pragma unroll
    for (int i = 0; i < TM; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};

  const __amdgpu_buffer_rsrc_t rsA = make_rsrc(p.a, p.a_bytes);
  const __amdgpu_buffer_rsrc_t rsB = make_rsrc(p.b, p.b_bytes);

  // ---- loader slots: each DMA instruction writes 8 consecutive LDS rows (1 KB); lane -> (row
  // base + lane/8, chunk position lane%8) and loads global chunk (lane%8) ^ (row & 7)
  const int gch = (lane & 7) ^ (lane >> 3);
  int a_off[2][NA], a_y[2][NA], a_x[2][NA], a_lds[2][NA];
  int b_off[2][NB], b_lds[2][NB];
#pragma unroll
  for (int mh = 0; mh < 2; ++mh)
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      const int h0 = wid * (8 * NA) + i * 8;                 // first half-row of this instruction
      const int row0 = (h0 / AH) * WTM + mh * AH + h0 % AH;  // logical (= LDS) row of lane 0
      a_lds[mh][i] = row0 * (BK * 2);
      const int m = m0 + row0 + (lane >> 3);
      const bool v = m < p.gm;
      const int mm = v ? m : 0;
      if constexpr (MODE == MODE_FWD) {
        const int n = fdiv(mm, p.fd_PQ);
        const int rem = mm - n * p.P * p.Q;
        const int pp = fdiv(rem, p.fd_Q);
        const int qq = rem - pp * p.Q;
        const int yv = pp * p.stride - p.pad;
        a_y[mh][i] = v ? yv : -(1 << 28);
        a_x[mh][i] = qq * p.stride - p.pad;
        a_off[mh][i] = ((n * p.H + yv) * p.W + a_x[mh][i]) * p.C + gch * 8;
      } else {
        const int n = fdiv(mm, p.fd_HW);
        const int rem = mm - n * p.dH * p.dW;
        const int hh = fdiv(rem, p.fd_W);
        const int ww = rem - hh * p.dW;
        const int yv = hh + p.offy;
        a_y[mh][i] = v ? yv : -(1 << 28);
        a_x[mh][i] = ww + p.offx;
        a_off[mh][i] = ((n * p.P + yv) * p.Q + a_x[mh][i]) * p.K + gch * 8;
      }
    }
#pragma unroll
  for (int nh = 0; nh < 2; ++nh)
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      const int h0 = wid * (8 * NB) + i * 8;
      const int rho0 = (h0 / BH) * WTN + nh * BH + h0 % BH;
      b_lds[nh][i] = A_BYTES + rho0 * (BK * 2);
      const int n = n0 + chan_perm<true>(rho0 + (lane >> 3));
      b_off[nh][i] = n < p.gn ? n * p.gk + gch * 8 : -1;
    }

  // uniform tap / channel state of the next K-tile to load (C or K is a multiple of BK)
  const int CIN = (MODE == MODE_FWD) ? p.C : p.K;
  int kc = kbeg % CIN, k0 = kbeg;
  int ks = (kbeg / CIN) % p.S, kr = (kbeg / CIN) / p.S;
  auto issue_a = [&](int mh, int buf) {
    int tap;
    if constexpr (MODE == MODE_FWD) tap = (kr * p.W + ks) * p.C + kc;
    else tap = -(kr * p.Q + ks) * p.K + kc;
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      bool ok;
      if constexpr (MODE == MODE_FWD)
        ok = (unsigned)(a_y[mh][i] + kr) < (unsigned)p.H && (unsigned)(a_x[mh][i] + ks) < (unsigned)p.W;
      else
        ok = (unsigned)(a_y[mh][i] - kr) < (unsigned)p.P && (unsigned)(a_x[mh][i] - ks) < (unsigned)p.Q;
      const unsigned voff = ok ? (unsigned)(a_off[mh][i] + tap) * 2u : kOOB;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsA, (__attribute__((address_space(3))) void*)(smem + buf * STAGE + a_lds[mh][i]),
                                               16, voff, 0, 0, 0);
    }
  };
  auto issue_b = [&](int nh, int buf) {
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      const unsigned voff = b_off[nh][i] >= 0 ? (unsigned)(b_off[nh][i] + k0) * 2u : kOOB;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsB, (__attribute__((address_space(3))) void*)(smem + buf * STAGE + b_lds[nh][i]),
                                               16, voff, 0, 0, 0);
    }
  };
  auto advance = [&]() {
    k0 += BK;
    kc += BK;
    if (kc >= CIN) {
      kc = 0;
      if (++ks == p.S) { ks = 0; ++kr; }
    }
  };

  bf16x8 fa[TMH][2], fb[2][TNH][2];
  auto read_a = [&](int mh, int buf) {
    const char* sA = smem + buf * STAGE;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int i = 0; i < TMH; ++i) {
        const int row = wr * WTM + mh * AH + i * 16 + (lane & 15);
        fa[i][kk] = *reinterpret_cast<const bf16x8*>(sA + rr_off(row, kk * 4 + (lane >> 4)));
      }
  };
  auto read_b = [&](int nh, int buf) {
    const char* sB = smem + buf * STAGE + A_BYTES;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int j = 0; j < TNH; ++j) {
        const int row = wc * WTN + nh * BH + j * 16 + (lane & 15);
        fb[nh][j][kk] = *reinterpret_cast<const bf16x8*>(sB + rr_off(row, kk * 4 + (lane >> 4)));
      }
  };
  auto mma = [&](int mh, int nh) {
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int j = 0; j < TNH; ++j)
#pragma unroll
        for (int i = 0; i < TMH; ++i)
          acc[nh * TNH + j][mh * TMH + i] =
              __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[nh][j][kk], fa[i][kk], acc[nh * TNH + j][mh * TMH + i], 0, 0, 0);
  };

  // per-tile tap state (the halves of tiles t+1 and t+2 are in flight together)
  struct KS { int k0, kc, ks, kr; };
  auto adv = [&](KS st) {
    st.k0 += BK; st.kc += BK;
    if (st.kc >= CIN) { st.kc = 0; if (++st.ks == p.S) { st.ks = 0; ++st.kr; } }
    return st;
  };
  auto set_state = [&](const KS& st) { k0 = st.k0; kc = st.kc; ks = st.ks; kr = st.kr; };
  const KS s0{k0, kc, ks, kr};
  KS s1 = adv(s0), s2 = adv(s1);
  // prologue: all of tile 0 (buffer 0), then A0, B1, A1 of tile 1 (buffer 1)
  issue_a(0, 0); issue_b(0, 0); issue_b(1, 0); issue_a(1, 0);
  if (nk > 1) {
    set_state(s1);
    issue_a(0, 1); issue_b(1, 1); issue_a(1, 1);
    wait_vm<2 * NA + NB>();
  } else {
    wait_vm<0>();
  }
  lds_barrier();
  for (int t = 0; t < nk; ++t) {
    const int buf = t & 1, nb = buf ^ 1;
    const bool has1 = t + 1 < nk, has2 = t + 2 < nk;
    // P0: quadrant (0,0); DMA B0(t+1) into nb (its tile t-1 B0 was last read in P3(t-1))
    read_a(0, buf); read_b(0, buf);
    if (has1) { set_state(s1); issue_b(0, nb); }
    mma(0, 0);
    lds_sync();   // WAR: this phase's ds_reads retire before another wave re-DMAs the region
    // P1: quadrant (0,1); DMA A0(t+2) into buf (A0(t) read in P0)
    read_b(1, buf);
    if (has2) { set_state(s2); issue_a(0, buf); }
    mma(0, 1);
    lds_sync();   // WAR: this phase's ds_reads retire before another wave re-DMAs the region
    // P2: quadrant (1,1); DMA B1(t+2) into buf (B1(t) read in P1)
    read_a(1, buf);
    if (has2) issue_b(1, buf);
    mma(1, 1);
    lds_sync();   // WAR: this phase's ds_reads retire before another wave re-DMAs the region
    // P3: quadrant (1,0); DMA A1(t+2) into buf (A1(t) read in P2); retire all of tile t+1
    read_b(0, buf);
    if (has2) issue_a(1, buf);
    mma(1, 0);
    if (has2) wait_vm<2 * NA + NB>(); else wait_vm<0>();
    lds_sync();   // WAR: this phase's ds_reads retire before another wave re-DMAs the region
    s1 = s2;
    s2 = adv(s2);
  }
  igemm_epilogue_fd<MODE, BM, BN, WM, WN, EPI, NTHR, EPD>(p, acc, smem, tid, m0, n0, tile_m, split);
}

// ------------------------------------------------------------------------------------------------
// Waits visible to the compiler (the one-barrier-per-K-tile loops of igemm_dma32_kernel / gemm32_kernel):
// the s_waitcnt builtin rather than inline asm, so hipcc's waitcnt pass sees them and adds no
// conservative lgkmcnt waits in front of the MFMAs.  (Round 4's 8-wave one-barrier "big" FWD/DGRAD
// kernel, igemm_big_kernel, was removed in round 5: neutral for the FWD GEMMs alone and -0.3 % to
// -4.5 % with the DGRADs or the 256x128 tiles in the whole step, profiles/r5_big_fwd_ab.txt.)
template <int N>
__device__ __forceinline__ void wait_vm_b() {   // vmcnt(N) through the builtin (gfx9 simm16 encoding)
  static_assert(N >= 0 && N < 64, "vmcnt");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}
__device__ __forceinline__ void lds_sync_b() {   // lgkmcnt(0) + s_barrier, both visible to the compiler
  __builtin_amdgcn_s_waitcnt(15 | (3 << 14) | (7 << 4));
  __builtin_amdgcn_s_barrier();
}
// ------------------------------------------------------------------------------------------------
// Round-5 critical-path FWD / DGRAD kernel: igemm_dma_kernel's operand staging (LDS-DMA, swizzled
// 128-B rows, block-uniform tap walk) with the one-barrier-per-K-tile main loop of tools/gemm_lab v4
// on v_mfma_f32_32x32x16_bf16 (the loop gemm32_kernel runs for plain GEMMs): two LDS stages, the
// fragments of each 64-deep K-tile double-buffered over its two 32-deep halves,
//   half 0: ds_read frags(t, 1)  || MFMA frags(t, 0)
//           vmcnt(0) [stage t+1 landed] + lgkmcnt(0) + s_barrier [every wave done with stage t]
//   half 1: DMA stage t+2 into stage t's buffer, ds_read frags(t+1, 0)  || MFMA frags(t, 1)
// instead of igemm_dma_kernel's four per-quadrant barriers per K-tile on 16x16x32 (half the MFMA
// instructions for the same wave tile and ds_read bytes; lab: 128x128 4-wave +5-12 %,
// profiles/r4_gemm_lab_mfma32.txt).  4 waves, 2 blocks per CU (the WGRAD side stream keeps its CUs).
//
// Accumulator layout (MFMA runs B x A): lane l holds output pixel (l & 31) of each 32x32 tile and,
// through the B-row channel permutation chan_perm32, the 16 CONSECUTIVE channels 16 * (l >> 5) + r in
// register r -- two 16-B stores per (pixel, 32-channel block), no lane shuffles.  The epilogue
// (igemm_epilogue32) has every igemm_epilogue_fd feature the conv paths use (bias, residual incl. the
// sub-sampled one, ReLU, stride-2 sub-pixel output rows, BatchNorm partial statistics, the fused
// BatchNorm-backward reduction with tensor / bit / recomputed ReLU masks, the dual-BN form); its
// column sums are reduced in registers (a 4-step DPP transpose-reduction over the 16 lanes of a DPP
// row + one ds_swizzle across the row pair, per 32-channel block) instead of an LDS transpose, and
// the per-channel coefficient tables are staged in their own LDS region during the prologue.
__device__ __forceinline__ int chan_perm32(int rho) {   // LDS B row -> channel offset within the tile
  return (rho & ~31) | (((rho >> 2) & 1) << 4) | (((rho >> 3) & 3) << 2) | (rho & 3);
}

// v[0..15] of every lane -> the sum over the 16 lanes of the lane's DPP row of v[lane & 15]
// (butterfly over row_mirror, row_half_mirror, quad xor-2, quad xor-1: each step a lane keeps half of
// its values and adds the partner's copy of that half; 45 VALU for 16 values instead of 64)
__device__ __forceinline__ float row16_transpose_sum(const float (&v)[16], int lane) {
  const bool b3 = lane & 8, b2 = lane & 4, b1 = lane & 2, b0 = lane & 1;
  float w[8], x[4], y[2];
#pragma unroll
  for (int k = 0; k < 8; ++k) w[k] = (b3 ? v[k + 8] : v[k]) + dpp_mov<0x140>(b3 ? v[k] : v[k + 8]);
#pragma unroll
  for (int k = 0; k < 4; ++k) x[k] = (b2 ? w[k + 4] : w[k]) + dpp_mov<0x141>(b2 ? w[k] : w[k + 4]);
#pragma unroll
  for (int k = 0; k < 2; ++k) y[k] = (b1 ? x[k + 2] : x[k]) + dpp_mov<0x4E>(b1 ? x[k] : x[k + 2]);
  return (b0 ? y[1] : y[0]) + dpp_mov<0xB1>(b0 ? y[0] : y[1]);
}

// ctab: [6][BN] coefficient rows (BN-backward: istd, -mean*istd, mask scale, mask shift, istd2,
// -mean2*istd2; otherwise row 0 = bias), filled in the prologue; red: [WM][NS][BN] scratch
template <int MODE, int BM, int BN, int WM, int WN, int EPI, int EPD>
__device__ __forceinline__ void igemm_epilogue32(const IgemmParams& p, f32x16 (&acc)[BN / WN / 32][BM / WM / 32],
                                                 const float* ctab, float* red, int tid, int m0, int n0, int tile_m) {
  constexpr int WTM = BM / WM, WTN = BN / WN;
  constexpr int TM = WTM / 32, TN = WTN / 32;
  constexpr int NTH = 256;
  constexpr int NI = TN * TM * 2;                 // 16-B store items per lane
  constexpr int IPJ = TM * 2;                     // items per 32-channel block
  constexpr bool stats = EPI == EPI_STATS;
  constexpr bool bnr = MODE == MODE_DGRAD && (EPI == EPI_BNR || EPI == EPI_BNR2);
  constexpr bool bnr2 = MODE == MODE_DGRAD && EPI == EPI_BNR2;
  constexpr int NS = bnr2 ? 3 : 2;
  static_assert(EPI != EPI_GELU, "igemm_epilogue32: conv epilogues only");
  const int lane = tid & 63, wid = tid >> 6;
  const int wr = wid / WN, wc = wid % WN;
  const int h = lane >> 5, pr = lane & 31;
  __bf16* out = reinterpret_cast<__bf16*>(p.out);
  const bool has_res = p.resid != nullptr;
  const bool has_mb = bnr && p.bn_mbits != nullptr;
  const bool has_mk = bnr && !has_mb && p.bn_mask != nullptr;
  const bool mfx = bnr && !has_mb && !has_mk && p.bn_msc != nullptr;
  const bool has_bias = MODE == MODE_FWD && p.bias != nullptr;
  size_t orows[TM];
  int rrows[MODE == MODE_DGRAD ? TM : 1];
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int m = m0 + wr * WTM + i * 32 + pr;
    size_t orow = m < p.gm ? m : 0;
    if constexpr (MODE == MODE_DGRAD) {
      rrows[i] = (int)orow;
      if ((p.sub || p.resid_sub) && m < p.gm) {
        const int n = fdiv(m, p.fd_HW);
        const int rem = m - n * p.dH * p.dW;
        const int hh = fdiv(rem, p.fd_W);
        const int ww = rem - hh * p.dW;
        if (p.sub) orow = ((size_t)n * p.H + 2 * hh + p.oph) * p.W + 2 * ww + p.opw;
        else rrows[i] = ((hh | ww) & 1) ? -1 : (n * p.rs_H2 + (hh >> 1)) * p.rs_W2 + (ww >> 1);
      }
    }
    orows[i] = orow;
  }
  // item t: 32-channel block j = t / IPJ (outer: its column sums are reduced when it completes),
  // pixel row group i, 8-channel half c2
  auto item_j = [](int t) { return t / IPJ; };
  auto item_i = [](int t) { return (t / 2) % TM; };
  auto item_c = [](int t) { return t & 1; };
  auto chan = [&](int t) { return wc * WTN + 32 * item_j(t) + 16 * h + 8 * item_c(t); };   // within the tile
  constexpr int D = EPD;
  uint4 rvA[D], mkA[D], xvA[D], xv2A[D];
  unsigned mbA[D];
  auto issue = [&](int t, int b) {
    const int i = item_i(t);
    const int m = m0 + wr * WTM + i * 32 + pr;
    const int n = n0 + chan(t);
    const bool ok = m < p.gm && n < p.gn;
    const size_t o = orows[i] * p.gn + (ok ? n : 0);
    auto ldv = [&](const __bf16* src) { return ok ? *reinterpret_cast<const uint4*>(src + o) : uint4{0, 0, 0, 0}; };
    if (has_res) {
      if constexpr (MODE == MODE_DGRAD) {
        if (p.resid_sub) {
          const bool okr = ok && rrows[i] >= 0;
          const size_t ro = (size_t)(okr ? rrows[i] : 0) * p.gn + (ok ? n : 0);
          rvA[b] = okr ? *reinterpret_cast<const uint4*>(p.resid + ro) : uint4{0, 0, 0, 0};
        } else {
          rvA[b] = ldv(p.resid);
        }
      } else {
        rvA[b] = ldv(p.resid);
      }
    }
    if constexpr (bnr) {
      if (has_mb) mbA[b] = ok ? p.bn_mbits[o >> 3] : 0u;
      if (has_mk) mkA[b] = ldv(p.bn_mask);
      xvA[b] = ldv(p.bn_x);
      if constexpr (bnr2) xv2A[b] = ldv(p.bn_x2);
    }
  };
  if (has_res || bnr) {
#pragma unroll
    for (int d = 0; d < D - 1; ++d)
      if (d < NI) issue(d, d);
  }
  float sm[NS][16];
#pragma unroll
  for (int t = 0; t < NI; ++t) {
    const int b = t % D;
    if ((has_res || bnr) && t + D - 1 < NI) issue(t + D - 1, (t + D - 1) % D);
    const int j = item_j(t), i = item_i(t), c2 = item_c(t);
    if (t % IPJ == 0) {
#pragma unroll
      for (int k = 0; k < NS; ++k)
#pragma unroll
        for (int e = 0; e < 16; ++e) sm[k][e] = 0.f;
    }
    const int m = m0 + wr * WTM + i * 32 + pr;
    const int ct = chan(t);
    const int n = n0 + ct;
    if (m < p.gm && n < p.gn) {
      const size_t o = orows[i] * p.gn + n;
      float x[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) x[e] = acc[j][i][8 * c2 + e];
      if (has_bias) {
        const f32x4 b0 = *reinterpret_cast<const f32x4*>(ctab + ct), b1 = *reinterpret_cast<const f32x4*>(ctab + ct + 4);
#pragma unroll
        for (int e = 0; e < 4; ++e) { x[e] += b0[e]; x[e + 4] += b1[e]; }
      }
      if (has_res) {
        const unsigned rw[4] = {rvA[b].x, rvA[b].y, rvA[b].z, rvA[b].w};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          x[2 * q] += __uint_as_float(rw[q] << 16);
          x[2 * q + 1] += __uint_as_float(rw[q] & 0xffff0000u);
        }
      }
      if (p.relu) {
#pragma unroll
        for (int e = 0; e < 8; ++e) x[e] = fmaxf(x[e], 0.f);
      }
      unsigned ov[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) ov[q] = f2bf2(x[2 * q], x[2 * q + 1]);
      if constexpr (bnr) {
        const unsigned xw[4] = {xvA[b].x, xvA[b].y, xvA[b].z, xvA[b].w};
        if (has_mb) {
          const unsigned bits = mbA[b];
#pragma unroll
          for (int q = 0; q < 4; ++q)
            ov[q] &= (((bits >> (2 * q)) & 1u) ? 0x0000ffffu : 0u) | (((bits >> (2 * q + 1)) & 1u) ? 0xffff0000u : 0u);
        } else if (has_mk) {
          const unsigned yw[4] = {mkA[b].x, mkA[b].y, mkA[b].z, mkA[b].w};
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const unsigned y = yw[q];
            ov[q] &= (((y & 0x8000u) == 0 && (y & 0x7fffu) != 0) ? 0x0000ffffu : 0u) |
                     (((y & 0x80000000u) == 0 && (y & 0x7fff0000u) != 0) ? 0xffff0000u : 0u);
          }
        } else if (mfx) {
          const f32x4 s0 = *reinterpret_cast<const f32x4*>(ctab + 2 * BN + ct), s1 = *reinterpret_cast<const f32x4*>(ctab + 2 * BN + ct + 4);
          const f32x4 h0 = *reinterpret_cast<const f32x4*>(ctab + 3 * BN + ct), h1 = *reinterpret_cast<const f32x4*>(ctab + 3 * BN + ct + 4);
          const float msc[8] = {s0[0], s0[1], s0[2], s0[3], s1[0], s1[1], s1[2], s1[3]};
          const float msh[8] = {h0[0], h0[1], h0[2], h0[3], h1[0], h1[1], h1[2], h1[3]};
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const float z0 = fmaf(__uint_as_float(xw[q] << 16), msc[2 * q], msh[2 * q]);
            const float z1 = fmaf(__uint_as_float(xw[q] & 0xffff0000u), msc[2 * q + 1], msh[2 * q + 1]);
            ov[q] &= (z0 > 0.f ? 0x0000ffffu : 0u) | (z1 > 0.f ? 0xffff0000u : 0u);
          }
        }
        const f32x4 a0 = *reinterpret_cast<const f32x4*>(ctab + ct), a1 = *reinterpret_cast<const f32x4*>(ctab + ct + 4);
        const f32x4 k0 = *reinterpret_cast<const f32x4*>(ctab + BN + ct), k1 = *reinterpret_cast<const f32x4*>(ctab + BN + ct + 4);
        const float ka[8] = {a0[0], a0[1], a0[2], a0[3], a1[0], a1[1], a1[2], a1[3]};
        const float kb[8] = {k0[0], k0[1], k0[2], k0[3], k1[0], k1[1], k1[2], k1[3]};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float g0 = __uint_as_float(ov[q] << 16), g1 = __uint_as_float(ov[q] & 0xffff0000u);
          const int e = 8 * c2 + 2 * q;
          sm[0][e] += g0; sm[0][e + 1] += g1;
          sm[1][e] += g0 * fmaf(__uint_as_float(xw[q] << 16), ka[2 * q], kb[2 * q]);
          sm[1][e + 1] += g1 * fmaf(__uint_as_float(xw[q] & 0xffff0000u), ka[2 * q + 1], kb[2 * q + 1]);
        }
        if constexpr (bnr2) {
          const unsigned xw2[4] = {xv2A[b].x, xv2A[b].y, xv2A[b].z, xv2A[b].w};
          const f32x4 c0 = *reinterpret_cast<const f32x4*>(ctab + 4 * BN + ct), c1 = *reinterpret_cast<const f32x4*>(ctab + 4 * BN + ct + 4);
          const f32x4 d0 = *reinterpret_cast<const f32x4*>(ctab + 5 * BN + ct), d1 = *reinterpret_cast<const f32x4*>(ctab + 5 * BN + ct + 4);
          const float ka2[8] = {c0[0], c0[1], c0[2], c0[3], c1[0], c1[1], c1[2], c1[3]};
          const float kb2[8] = {d0[0], d0[1], d0[2], d0[3], d1[0], d1[1], d1[2], d1[3]};
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const float g0 = __uint_as_float(ov[q] << 16), g1 = __uint_as_float(ov[q] & 0xffff0000u);
            const int e = 8 * c2 + 2 * q;
            sm[2][e] += g0 * fmaf(__uint_as_float(xw2[q] << 16), ka2[2 * q], kb2[2 * q]);
            sm[2][e + 1] += g1 * fmaf(__uint_as_float(xw2[q] & 0xffff0000u), ka2[2 * q + 1], kb2[2 * q + 1]);
          }
        }
      } else if constexpr (stats) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float r0 = __uint_as_float(ov[q] << 16), r1 = __uint_as_float(ov[q] & 0xffff0000u);
          const int e = 8 * c2 + 2 * q;
          sm[0][e] += r0; sm[0][e + 1] += r1;
          sm[1][e] += r0 * r0; sm[1][e + 1] += r1 * r1;
        }
      }
      *reinterpret_cast<uint4*>(out + o) = uint4{ov[0], ov[1], ov[2], ov[3]};
    }
    if constexpr (stats || bnr) {
      if (t % IPJ == IPJ - 1) {   // block j complete: reduce its column sums over the wave's 32 pixels
#pragma unroll
        for (int k = 0; k < NS; ++k) {
          float s = row16_transpose_sum(sm[k], lane);
          s += __int_as_float(__builtin_amdgcn_ds_swizzle(__float_as_int(s), 0x401F));   // lane ^ 16
          if (!(lane & 16)) red[(wr * NS + k) * BN + wc * WTN + 32 * j + 16 * h + (lane & 15)] = s;
        }
      }
    }
  }
  if constexpr (stats || bnr) {
    __syncthreads();
    float* st = p.stats + (size_t)tile_m * 2 * p.gn;
    float* st2 = bnr2 ? p.stats2 + (size_t)tile_m * 2 * p.gn : nullptr;
    for (int c = tid; c < BN; c += NTH) {
      if (n0 + c < p.gn) {
        float t[NS];
#pragma unroll
        for (int k = 0; k < NS; ++k) {
          t[k] = 0.f;
#pragma unroll
          for (int w = 0; w < WM; ++w) t[k] += red[(w * NS + k) * BN + c];
        }
        st[n0 + c] = t[0];
        st[p.gn + n0 + c] = t[1];
        if constexpr (bnr2) {
          st2[n0 + c] = t[0];
          st2[p.gn + n0 + c] = t[2];
        }
      }
    }
  }
}

// XP: the accumulators are transposed through LDS into igemm_dma_kernel's 16x16 D^T / PAIR
// fragment layout and the tile runs igemm_epilogue_fd: a store / load instruction then covers 16
// pixels x 64 B (4 lanes per pixel) instead of 32 pixels x 2 x 16 B, which is what the memory-bound
// short-K DGRAD + BN-backward epilogues (residual, x and mask loads per output) need (per-shape A/B
// profiles/r5_knob_dma32.txt: -14 to -25 % on the 1x1 DGRADs into 1024 / 2048 channels without it).
template <int MODE, int BM, int BN, int WM, int WN, int EPI, int EPD = 2>
__global__ void __launch_bounds__(256, 2) igemm_dma32_kernel(const IgemmParams p) {
  constexpr int NW = 4, NTHR = 256;
  constexpr int WTM = BM / WM, WTN = BN / WN;
  constexpr int TM = WTM / 32, TN = WTN / 32;
  constexpr int A_BYTES = BM * BK * 2, STAGE = (BM + BN) * BK * 2;
  constexpr int NA = BM / 8 / NW, NB = BN / 8 / NW;   // LDS-DMA instructions (8 rows each) per wave
  constexpr bool bnr = MODE == MODE_DGRAD && (EPI == EPI_BNR || EPI == EPI_BNR2);
  constexpr bool bnr2 = MODE == MODE_DGRAD && EPI == EPI_BNR2;
  constexpr int NS = bnr2 ? 3 : 2;
  static_assert(MODE != MODE_WGRAD, "FWD/DGRAD only");
  static_assert(WM * WN == NW && TM >= 1 && TN >= 1 && NA >= 1 && NB >= 1 && NA * 8 * NW == BM && NB * 8 * NW == BN,
                "igemm_dma32 tile");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float* ctab = reinterpret_cast<float*>(smem + 2 * STAGE);   // [6][BN]
  float* red = ctab + 6 * BN;                                 // [WM][NS][BN]
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid / WN, wc = wid % WN;

  const int lin = xcd_remap(blockIdx.x, gridDim.x);
  const int tile_n = lin % p.tiles_n;
  const int tile_m = lin / p.tiles_n;
  const int m0 = tile_m * BM, n0 = tile_n * BN;
  const int nk = p.gk / BK;

  const __amdgpu_buffer_rsrc_t rsA = make_rsrc(p.a, p.a_bytes);
  const __amdgpu_buffer_rsrc_t rsB = make_rsrc(p.b, p.b_bytes);
  const int gch = (lane & 7) ^ (lane >> 3);
  int a_off[NA], a_y[NA], a_x[NA];
  int b_off[NB];
#pragma unroll
  for (int i = 0; i < NA; ++i) {
    const int m = m0 + (wid * NA + i) * 8 + (lane >> 3);
    const bool v = m < p.gm;
    const int mm = v ? m : 0;
    if constexpr (MODE == MODE_FWD) {
      const int n = fdiv(mm, p.fd_PQ);
      const int rem = mm - n * p.P * p.Q;
      const int pp = fdiv(rem, p.fd_Q);
      const int qq = rem - pp * p.Q;
      const int yv = pp * p.stride - p.pad;
      a_y[i] = v ? yv : -(1 << 28);
      a_x[i] = qq * p.stride - p.pad;
      a_off[i] = ((n * p.H + yv) * p.W + a_x[i]) * p.C + gch * 8;
    } else {
      const int n = fdiv(mm, p.fd_HW);
      const int rem = mm - n * p.dH * p.dW;
      const int hh = fdiv(rem, p.fd_W);
      const int ww = rem - hh * p.dW;
      const int yv = hh + p.offy;
      a_y[i] = v ? yv : -(1 << 28);
      a_x[i] = ww + p.offx;
      a_off[i] = ((n * p.P + yv) * p.Q + a_x[i]) * p.K + gch * 8;
    }
  }
#pragma unroll
  for (int i = 0; i < NB; ++i) {
    const int n = n0 + chan_perm32((wid * NB + i) * 8 + (lane >> 3));
    b_off[i] = n < p.gn ? n * p.gk + gch * 8 : -1;
  }
  const int CIN = (MODE == MODE_FWD) ? p.C : p.K;
  int kc = 0, k0 = 0, ks = 0, kr = 0;
  // DMA of the K-tile at (k0, kr, ks, kc) into stage s, then advance; !live: zero-fill (tail)
  auto issue = [&](int s, bool live) {
    int tap;
    if constexpr (MODE == MODE_FWD) tap = (kr * p.W + ks) * p.C + kc;
    else tap = -(kr * p.Q + ks) * p.K + kc;
    char* dst = smem + s * STAGE;
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      bool ok;
      if constexpr (MODE == MODE_FWD)
        ok = (unsigned)(a_y[i] + kr) < (unsigned)p.H && (unsigned)(a_x[i] + ks) < (unsigned)p.W;
      else
        ok = (unsigned)(a_y[i] - kr) < (unsigned)p.P && (unsigned)(a_x[i] - ks) < (unsigned)p.Q;
      const int voff = (ok && live) ? (a_off[i] + tap) * 2 : (int)kOOB;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsA, (__attribute__((address_space(3))) void*)(dst + (wid * NA + i) * 1024),
                                               16, voff, 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      const int voff = (b_off[i] >= 0 && live) ? (b_off[i] + k0) * 2 : (int)kOOB;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rsB, (__attribute__((address_space(3))) void*)(dst + A_BYTES + (wid * NB + i) * 1024), 16, voff, 0, 0, 0);
    }
    k0 += BK;
    kc += BK;
    if (kc >= CIN) {
      kc = 0;
      if (++ks == p.S) { ks = 0; ++kr; }
    }
  };

  // per-channel epilogue coefficients: loaded ahead of the first DMAs, written to LDS once the first
  // stage has landed (the prologue barrier publishes them)
  float cv[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  const bool ld_ct = tid < BN && (bnr || (MODE == MODE_FWD && p.bias != nullptr));
  if (ld_ct) {
    const int c = min(n0 + tid, p.gn - 1);
    if constexpr (bnr) {
      const float is = p.bn_istd[c];
      cv[0] = is;
      cv[1] = -p.bn_mean[c] * is;
      if (!p.bn_mbits && !p.bn_mask && p.bn_msc) { cv[2] = p.bn_msc[c]; cv[3] = p.bn_msh[c]; }
      if constexpr (bnr2) {
        const float is2 = p.bn_istd2[c];
        cv[4] = is2;
        cv[5] = -p.bn_mean2[c] * is2;
      }
    } else {
      cv[0] = p.bias[c];
    }
  }

  f32x16 acc[TN][TM];
#pragma unroll
  for (int j = 0; j < TN; ++j)
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[j][i][r] = 0.f;
  bf16x8 fa0[2][TM], fb0[2][TN], fa1[2][TM], fb1[2][TN];
  auto rd = [&](bf16x8(&fa)[2][TM], bf16x8(&fb)[2][TN], int half, int s) {
    const char* sA = smem + s * STAGE;
    const char* sB = sA + A_BYTES;
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int ch = half * 4 + q * 2 + (lane >> 5);
#pragma unroll
      for (int i = 0; i < TM; ++i) fa[q][i] = *reinterpret_cast<const bf16x8*>(sA + rr_off(wr * WTM + i * 32 + (lane & 31), ch));
#pragma unroll
      for (int j = 0; j < TN; ++j) fb[q][j] = *reinterpret_cast<const bf16x8*>(sB + rr_off(wc * WTN + j * 32 + (lane & 31), ch));
    }
  };
  auto mma = [&](bf16x8(&fa)[2][TM], bf16x8(&fb)[2][TN]) {
#pragma unroll
    for (int q = 0; q < 2; ++q)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int i = 0; i < TM; ++i) acc[j][i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fb[q][j], fa[q][i], acc[j][i], 0, 0, 0);
  };
  constexpr int NMF = 2 * TM * TN, NDS = 2 * (TM + TN), NVM = NA + NB;
  constexpr int DPM = NDS / NMF > 0 ? NDS / NMF : 1, MPD = NMF >= NDS ? NMF / NDS : 1;
  // K-tile t in three forms (compile-time, so each half stays one scheduling region): FULL issues
  // the DMA of tile t+2; NODMA (t = nk-2) only waits for tile t+1; LAST (t = nk-1) has no barrier.
  // No zero-fill DMA of a dead stage is issued or waited for: at 3-4 K-tiles per output tile (the
  // short-K 1x1 DGRADs) two dead-DMA round trips per tile cost more than the loop saves.
  enum { FULL = 0, NODMA = 1, LAST = 2 };
  auto ktile = [&](int t, auto form) {
    constexpr int F = decltype(form)::value;
    const int s = t & 1;
    rd(fa1, fb1, 1, s);
    mma(fa0, fb0);
#pragma unroll
    for (int g = 0; g < NDS; ++g) {
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      if (g % DPM == 0) __builtin_amdgcn_sched_group_barrier(0x8, MPD, 0);
    }
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (F != LAST) {
      wait_vm_b<0>();
      lds_sync_b();   // every wave's reads of stage s retired; stage t+1 landed for every wave
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (F == FULL) issue(s, true);
      rd(fa0, fb0, 0, s ^ 1);
    }
    mma(fa1, fb1);
    if constexpr (F == FULL) {
#pragma unroll
      for (int g = 0; g < NDS; ++g) {
        if (g < NVM) __builtin_amdgcn_sched_group_barrier(0x10, 1, 1);
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 1);
        if (g % DPM == 0) __builtin_amdgcn_sched_group_barrier(0x8, MPD, 1);
      }
    } else if constexpr (F == NODMA) {
#pragma unroll
      for (int g = 0; g < NDS; ++g) {
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 1);
        if (g % DPM == 0) __builtin_amdgcn_sched_group_barrier(0x8, MPD, 1);
      }
    }
    __builtin_amdgcn_sched_barrier(0);
  };
  issue(0, true);
  issue(1, true);   // nk >= 2 (the dispatcher sends >= 3 K-tiles)
  wait_vm_b<NA + NB>();
  if (ld_ct) {
#pragma unroll
    for (int r = 0; r < 6; ++r) ctab[r * BN + tid] = cv[r];
  }
  lds_sync_b();
  rd(fa0, fb0, 0, 0);
  for (int t = 0; t < nk - 2; ++t) ktile(t, std::integral_constant<int, FULL>{});
  ktile(nk - 2, std::integral_constant<int, NODMA>{});
  ktile(nk - 1, std::integral_constant<int, LAST>{});
  (void)NS;
  igemm_epilogue32<MODE, BM, BN, WM, WN, EPI, EPD>(p, acc, ctab, red, tid, m0, n0, tile_m);
}

// ------------------------------------------------------------------------------------------------
// Halo-tiled direct convolution for stride-1 convs with narrow channels: the ResNet layer-1 3x3
// (64 -> 64 channels at 56x56: FWD and DGRAD) and the space-to-depth stem (16 -> 64 channels,
// 4x4 taps at 112x112).  The implicit GEMM above re-reads every input pixel once per filter tap
// (9x / 16x L2->LDS traffic for a 64-wide output tile); here a tile is TR whole output rows of one
// image (BM = 224 pixels) and the block DMAs the (TR+R-1) x (Wo+S-1) input halo into LDS ONCE,
// zero-filled at the borders through the buffer range check.  Every tap's B fragment is read from
// the halo in place: within a filter row r the (s, c) pairs of the KRSC reduction order are
// contiguous in the halo row, so the K32 chunk of reduction index k starts at halo pixel
// (ty + r, tx + s) channel c -- one ds_read_b128 per lane per pixel fragment, no im2col image.
// The 64 output channels' weights (K = R*S*C <= 576) live in REGISTERS for the whole persistent
// kernel (each wave: 32 channels x K), so the only LDS reads are pixel fragments: 7 reads per 14
// MFMAs.  LDS layout: [halo row][16-B channel chunk][column], each (row, chunk) run of HWp >= HWd+15
// slots (HWp % 16 == 0) shifted by skew(row) = (row * Wo) % 16, so the bank quad of (row, col) is
// (linear output pixel + tap offset) % 16: the 16 pixels of a fragment -- row wraps included -- and
// both k-groups of every ds_read_b128 lane group land on 16 distinct quads (an XOR swizzle of a
// pixel-major image left 40 % of the LDS cycles as bank conflicts: profiles/r2_halo_pmc.txt).
// One block per CU walks a contiguous range of tiles (neighbouring tiles share halo rows
// in the XCD's L2); the next tile's halo DMA overlaps this tile's MFMAs and epilogue.  The
// accumulators have igemm_kernel's D^T/PAIR layout, so the shared epilogue (BatchNorm statistics,
// fused BN-backward reduction, residual, ReLU) is reused unchanged.
// DGRAD runs as the forward correlation of dy with the tap-mirrored transposed weight
// (pad' = R-1-pad); FLIP reads wt[c][R-1-r][S-1-s][k] while loading the weight registers.
struct HaloGeom {
  const __bf16* src;      // [N][Hs][Ws][CS]
  const __bf16* wsrc;     // [64][R][S][CS]
  unsigned src_bytes;
  int Hs, Ws, Ho, Wo, padT, padL, TR, HWd, HWp, HR, tiles, tiles_img, lds_bytes, ninstr;
  FastDiv fd_HWp, fd_Wo, fd_timg;
};
constexpr int HALO_BM = 224;


template <int MODE, int EPI, int CS, int RS, bool FLIP, int WO, bool OVL>
__global__ void __launch_bounds__(NT, 1) halo_conv_kernel(const IgemmParams p, const HaloGeom g) {
  constexpr int BM = HALO_BM, BN = 64, WM = 2, WN = 2;
  constexpr int WTM = BM / WM, TM = WTM / 16, TN = BN / WN / 16;
  constexpr int KC = RS * RS * CS / 32;   // K32 chunks
  constexpr int NCH = CS / 8;              // 16-B channel chunks per pixel
  constexpr int TR = BM / WO, HWd = WO + RS - 1, HWp = (HWd + 30) / 16 * 16, HR = TR + RS - 1;
  constexpr int NINSTR = (HR * NCH * HWp * 16 + 1023) / 1024;
  static_assert(TM == 7 && TN == 2 && (RS * CS) % 32 == 0 && BM % WO == 0, "halo tiling");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid / WN, wc = wid % WN;
  constexpr int LDS_BYTES = NINSTR * 1024;
  // OVL (FWD without residual / ReLU / bias): the finished tile goes to LDS as bf16 (ytile, 16-B
  // chunks XOR-swizzled by pixel) and its global stores are spread over the NEXT tile's MFMA steps,
  // so at one wave per SIMD the output traffic hides under the matrix work instead of following it
  constexpr int YT_BYTES = OVL ? BM * BN * 2 : 0;
  constexpr int NYS = BM * BN * 2 / 16 / NT;   // 16-B output chunks per thread per tile (7)
  char* ytile = smem + 2 * LDS_BYTES;
  char* scratch = ytile + YT_BYTES;
  __bf16* yout = reinterpret_cast<__bf16*>(p.out);
  const __amdgpu_buffer_rsrc_t rs = make_rsrc(g.src, g.src_bytes);

  // this wave's 32 output channels x the whole reduction, as MFMA A fragments (PAIR channel order)
  bf16x8 wreg[KC][TN];
#pragma unroll
  for (int kt = 0; kt < KC; ++kt)
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int n = chan_perm<true>(wc * 32 + j * 16 + (lane & 15));
      const int k = kt * 32 + 8 * (lane >> 4);
      const int r = k / (RS * CS), sx = (k / CS) % RS, c = k % CS;
      const int rr = FLIP ? RS - 1 - r : r, ss = FLIP ? RS - 1 - sx : sx;
      wreg[kt][j] = *reinterpret_cast<const bf16x8*>(g.wsrc + ((size_t)(n * RS + rr) * RS + ss) * CS + c);
    }
  // Per lane, fragment and filter row r: the byte address of its K32 chunk 0.  Within a filter row
  // the chunk's offset from there is lane-uniform and compile-time (folded into ds_read_b128's
  // immediate): CS=64: chunk (kt%2)*4 -> +4*HWp slots, tap column s -> +s; CS=16: tap pair s0 -> +s0.
  // The lane's k-group g picks chunk g (CS=64), or pixel +g/2 and chunk g%2 (CS=16).
  const int kg = lane >> 4;
  int base[TM][RS];
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int pp = wr * WTM + i * 16 + (lane & 15);
    const int ty = pp / WO, tx = pp % WO;
#pragma unroll
    for (int r = 0; r < RS; ++r) {
      const int hr = ty + r;
      const int chunk = CS == 64 ? kg : (kg & 1);
      const int col = tx + (CS == 64 ? 0 : (kg >> 1)) + ((hr * WO) & 15);
      base[i][r] = ((hr * NCH + chunk) * HWp + col) * 16;
    }
  }
  // Halo staging: 16-B global loads in PIXEL-major order (8 lanes per 128-B line: full-line,
  // coalesced reads; out-of-image pixels read as zero through the buffer range check), written to
  // the chunk-major LDS image by ds_write_b128 after the MFMAs of the tile before.  (LDS-DMA must
  // write LDS in lane order, so it could only fill the chunk-major image by gathering 16 B from 64
  // different lines per instruction: ~5 us per tile, slower than the MFMAs.)
  // one wave-instruction = PPI consecutive pixels x all NCH chunks = 1 KB of contiguous global
  // memory; lane -> (pixel lane % PPI, chunk lane / PPI), so the 8 lanes of each ds_write_b128 lane
  // group store one chunk of 8 consecutive pixels: 8 consecutive slots, no bank conflict
  constexpr int NPIX = HR * HWd, NSLOT = NPIX * NCH, PPI = 64 / NCH;
  constexpr int NLD = (NSLOT + NT - 1) / NT;
  uint4 stg[NLD];
  auto load_halo = [&](int t) {
    const int n_img = fdiv(t, g.fd_timg);
    const int y0 = (t - n_img * g.tiles_img) * TR - g.padT;
#pragma unroll
    for (int l = 0; l < NLD; ++l) {
      const int pix = (l * NT + wid * 64) / NCH + lane % PPI, c = lane / PPI;
      const int hr = pix / HWd, hc = pix % HWd;
      const int y = y0 + hr, x = hc - g.padL;
      const bool ok = pix < NPIX && (unsigned)y < (unsigned)g.Hs && (unsigned)x < (unsigned)g.Ws;
      stg[l] = bload16(rs, ok ? (unsigned)((((n_img * g.Hs + y) * g.Ws + x) * CS + c * 8) * 2) : kOOB);
    }
  };
  auto store_halo = [&](char* dst) {
#pragma unroll
    for (int l = 0; l < NLD; ++l) {
      const int pix = (l * NT + wid * 64) / NCH + lane % PPI, c = lane / PPI;
      if (NSLOT % NT == 0 || pix < NPIX) {
        const int hr = pix / HWd, hc = pix % HWd;
        *reinterpret_cast<uint4*>(dst + ((hr * NCH + c) * HWp + hc + ((hr * WO) & 15)) * 16) = stg[l];
      }
    }
  };
  const int per = (g.tiles + gridDim.x - 1) / gridDim.x;
  const int t0 = blockIdx.x * per, t1 = min(g.tiles, t0 + per);
  if (t0 < t1) {
    load_halo(t0);
    store_halo(smem);
  }
  // DGRAD OVL (BN-backward reduction with the ReLU mask recomputed from x): per lane the 8 channels
  // wc*32 + fq*8.. of its fragments; their (istd, -mean*istd, mask scale, mask shift) are staged
  // in LDS once, and the tile's x values (7 x 16 B per lane) are loaded right after its MFMAs
  constexpr bool DBNR = OVL && MODE == MODE_DGRAD;
  float* ctab = reinterpret_cast<float*>(scratch) + 4 * BN;   // [4][BN] after the [2][2][BN] sums
  if constexpr (DBNR) {
    if (tid < BN) {
      const float is = p.bn_istd[tid];
      ctab[tid] = is;
      ctab[BN + tid] = -p.bn_mean[tid] * is;
      ctab[2 * BN + tid] = p.bn_msc[tid];
      ctab[3 * BN + tid] = p.bn_msh[tid];
    }
  }
  uint4 xv[DBNR ? TM : 1];
  auto ystore = [&](int tp, int l) {   // chunk l of this thread: ytile -> global (tile tp)
    const int q = l * NT + tid, pix = q >> 3, c = q & 7;
    const uint4 v = *reinterpret_cast<const uint4*>(ytile + pix * 128 + ((c ^ (pix & 7)) << 4));
    *reinterpret_cast<uint4*>(yout + (size_t)tp * BM * BN + (size_t)q * 8) = v;
  };
  for (int t = t0, it = 0; t < t1; ++t, ++it) {
    char* cur = smem + (it & 1) * LDS_BYTES;
    lds_sync();   // the halo of this tile is in LDS; every wave is done reading the other buffer
    const bool more = t + 1 < t1;
    if (more) load_halo(t + 1);   // in flight during this tile's MFMAs
    f32x4 acc[TN][TM];
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int i = 0; i < TM; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};
    // software pipeline one K32 chunk deep: chunk kt+1's fragment reads are issued before chunk
    // kt's MFMAs; the scheduling barrier keeps the compiler from hoisting every chunk's reads to
    // the top of the unrolled loop (126 live fragments -> spills)
    bf16x8 fa[2][TM];
    auto load_frags = [&](int kt, bf16x8 (&f)[TM]) {
      const int r = kt * 32 / (RS * CS);
      int off;   // lane-uniform slot offset inside filter row r
      if constexpr (CS == 64) off = ((kt % 2) * 4) * HWp + (kt / 2) % RS;
      else off = (kt % (RS / 2)) * 2;
#pragma unroll
      for (int i = 0; i < TM; ++i)
        f[i] = *reinterpret_cast<const bf16x8*>(cur + base[i][r] + off * 16);
    };
    // chunk order: with FLIP the taps run mirrored, so the implicit-GEMM DGRAD's accumulation order
    // (its taps ascending) is kept and the two kernels agree bitwise
    constexpr int CH = CS / 32 > 0 ? CS / 32 : 1;
    auto chunk = [&](int u) {
      if constexpr (!FLIP || CS < 32) return u;
      const int kr = u / (RS * CH), ks = (u / CH) % RS, cc = u % CH;
      return ((RS - 1 - kr) * RS + (RS - 1 - ks)) * CH + cc;
    };
    load_frags(chunk(0), fa[0]);
#pragma unroll
    for (int u = 0; u < KC; ++u) {
      if (u + 1 < KC) load_frags(chunk(u + 1), fa[(u + 1) & 1]);
      const int kt = chunk(u);
      if constexpr (OVL)
        if (u < NYS && it > 0) ystore(t - 1, u);   // the previous tile's output, one chunk per step
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int i = 0; i < TM; ++i)
          acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wreg[kt][j], fa[u & 1][i], acc[j][i], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    }
    if constexpr (DBNR) {   // (after the MFMAs: prefetched under them it spills the weight registers)
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int pl = wr * WTM + i * 16 + (lane & 15);
        xv[i] = *reinterpret_cast<const uint4*>(p.bn_x + ((size_t)t * BM + pl) * BN + wc * 32 + (lane >> 4) * 8);
      }
    }
    if constexpr (OVL) {
      lds_sync();   // every wave has read the previous tile out of ytile
      if (more) store_halo(smem + ((it + 1) & 1) * LDS_BYTES);
      // bf16 rounding (the value stored) + per-channel sums of the rounded values, as the shared
      // epilogue does; 8 channels per lane and pixel fragment -> one 16-B LDS store
      const int fr = lane & 15, fq = lane >> 4;
      float sm[2][TN][4];
#pragma unroll
      for (int k = 0; k < 2; ++k)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
          for (int e = 0; e < 4; ++e) sm[k][j][e] = 0.f;
      float ka[DBNR ? 8 : 1], kb[DBNR ? 8 : 1], ms[DBNR ? 8 : 1], mh[DBNR ? 8 : 1];
      if constexpr (DBNR) {   // this lane's 8 channels, once per tile
        const int ch = wc * 32 + fq * 8;
#pragma unroll
        for (int e = 0; e < 8; e += 4) {
          const f32x4 a = *reinterpret_cast<const f32x4*>(ctab + ch + e);
          const f32x4 b = *reinterpret_cast<const f32x4*>(ctab + BN + ch + e);
          const f32x4 c = *reinterpret_cast<const f32x4*>(ctab + 2 * BN + ch + e);
          const f32x4 d = *reinterpret_cast<const f32x4*>(ctab + 3 * BN + ch + e);
#pragma unroll
          for (int k = 0; k < 4; ++k) { ka[e + k] = a[k]; kb[e + k] = b[k]; ms[e + k] = c[k]; mh[e + k] = d[k]; }
        }
      }
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int pl = wr * WTM + i * 16 + fr;
        unsigned ov[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int j = q >> 1, e0 = (q & 1) * 2;
          unsigned u = f2bf2(acc[j][i][e0], acc[j][i][e0 + 1]);
          if constexpr (DBNR) {   // g = round(dgrad) where relu(x*msc+msh) > 0; sums of g, g*xhat
            const int ce = 2 * q;
            const unsigned xw = (&xv[i].x)[q];
            const float xa = __uint_as_float(xw << 16), xb = __uint_as_float(xw & 0xffff0000u);
            const float z0 = fmaf(xa, ms[ce], mh[ce]), z1 = fmaf(xb, ms[ce + 1], mh[ce + 1]);
            u &= (z0 > 0.f ? 0x0000ffffu : 0u) | (z1 > 0.f ? 0xffff0000u : 0u);
            const float r0 = __uint_as_float(u << 16), r1 = __uint_as_float(u & 0xffff0000u);
            sm[0][j][e0] += r0; sm[0][j][e0 + 1] += r1;
            sm[1][j][e0] += r0 * fmaf(xa, ka[ce], kb[ce]);
            sm[1][j][e0 + 1] += r1 * fmaf(xb, ka[ce + 1], kb[ce + 1]);
          } else if constexpr (EPI == EPI_STATS) {
            const float r0 = __uint_as_float(u << 16), r1 = __uint_as_float(u & 0xffff0000u);
            sm[0][j][e0] += r0; sm[0][j][e0 + 1] += r1;
            sm[1][j][e0] += r0 * r0; sm[1][j][e0 + 1] += r1 * r1;
          }
          ov[q] = u;
        }
        const int c = wc * 4 + fq;   // 16-B chunk: channels wc*32 + fq*8 .. +7 (PAIR order)
        *reinterpret_cast<uint4*>(ytile + pl * 128 + ((c ^ (pl & 7)) << 4)) = *reinterpret_cast<const uint4*>(ov);
      }
      if constexpr (EPI == EPI_STATS || DBNR) {
        float* red = reinterpret_cast<float*>(scratch);   // [WM][2][BN]
#pragma unroll
        for (int k = 0; k < 2; ++k)
#pragma unroll
          for (int j = 0; j < TN; ++j) {
            f32x4 v;
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = row16_sum(sm[k][j][e]);
            if (fr == 0) *reinterpret_cast<f32x4*>(red + (wr * 2 + k) * BN + wc * 32 + fq * 8 + j * 4) = v;
          }
        lds_sync();
        if (tid < BN) {
          float* st = p.stats + (size_t)t * 2 * BN;
          st[tid] = red[0 * BN + tid] + red[2 * BN + tid];
          st[BN + tid] = red[1 * BN + tid] + red[3 * BN + tid];
        }
      }
    } else {
      if (more) store_halo(smem + ((it + 1) & 1) * LDS_BYTES);
      igemm_epilogue_fd<MODE, BM, BN, WM, WN, EPI, NT, 2, true>(p, acc, scratch, tid, t * BM, 0, t, 0);
    }
  }
  if constexpr (OVL) {
    if (t0 < t1) {
      lds_sync();
#pragma unroll
      for (int l = 0; l < NYS; ++l) ystore(t1 - 1, l);
    }
  }
  wait_vm<0>();
}

// ------------------------------------------------------------------------------------------------
// Skinny FWD kernel for batch-1 inference (M = output pixels <= a few hundred: ResNet-50 layer 3/4
// and the classifier at batch 1).  Those GEMMs are latency-bound: a block has only a few K-steps
// of tiny MFMA work, so what matters is how many operand loads are in flight, not data reuse.  No
// LDS and no barriers: every lane loads its MFMA fragments straight from global memory into
// registers (16-B buffer loads, hardware zero-fill for padding / tails) in fragment layout, and a
// ring of PF K32-steps of loads stays in flight (the register-staged kernels keep one K-step).
// Block = 4 waves, tile 64 pixels x 64 output channels; wave w owns channels 16w..16w+15 for all 64
// pixels (4 MFMA fragments); D^T = W * X^T so each lane ends with 4 consecutive channels of one
// pixel.  The split index is blockIdx.y-major; splits > 1 write fp32 partials for
// splitk_epilogue_kernel, one split writes bf16 act(acc + bias (+ resid)).
// Requires C % 32 == 0 (a K32 step never straddles a filter tap).
template <int PF>
__global__ void __launch_bounds__(NT, 2) skinny_fwd_kernel(const IgemmParams p) {
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int fr = lane & 15, fq = lane >> 4;
  const int tiles_mn = p.tiles_m * p.tiles_n;
  const int split = blockIdx.x / tiles_mn;
  const int tl = blockIdx.x - split * tiles_mn;
  const int tile_n = tl % p.tiles_n, tile_m = tl / p.tiles_n;
  const int m0 = tile_m * 64, n0 = tile_n * 64 + wid * 16;
  const int kbeg = split * p.ksplit;
  const int kend = min(p.gk, kbeg + p.ksplit);
  const int nsteps = (kend - kbeg) / 32;
  const __amdgpu_buffer_rsrc_t rsA = make_rsrc(p.a, p.a_bytes);
  const __amdgpu_buffer_rsrc_t rsB = make_rsrc(p.b, p.b_bytes);
  // per-fragment pixel geometry (pixel m0 + 16i + fr)
  int a_base[4], a_y[4], a_x[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = m0 + 16 * i + fr;
    const bool v = m < p.gm;
    const int mm = v ? m : 0;
    const int n = fdiv(mm, p.fd_PQ);
    const int rem = mm - n * p.P * p.Q;
    const int pp = fdiv(rem, p.fd_Q);
    const int qq = rem - pp * p.Q;
    a_y[i] = v ? pp * p.stride - p.pad : -(1 << 28);
    a_x[i] = qq * p.stride - p.pad;
    a_base[i] = ((n * p.H + a_y[i]) * p.W + a_x[i]) * p.C + fq * 8;
  }
  const int nrow = n0 + fr;
  const int b_base = nrow < p.gn ? nrow * p.gk + fq * 8 : -1;
  // tap walk of the next K32 step to issue
  int kc = kbeg % p.C, ks = (kbeg / p.C) % p.S, kr = (kbeg / p.C) / p.S, kk = kbeg;
  uint4 ra[PF][4], rb[PF];
  auto issue = [&](int slot) {
    const int tap = (kr * p.W + ks) * p.C + kc;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const bool ok = (unsigned)(a_y[i] + kr) < (unsigned)p.H && (unsigned)(a_x[i] + ks) < (unsigned)p.W;
      ra[slot][i] = bload16(rsA, ok ? (unsigned)(a_base[i] + tap) * 2u : kOOB);
    }
    rb[slot] = bload16(rsB, b_base >= 0 ? (unsigned)(b_base + kk) * 2u : kOOB);
    kk += 32;
    kc += 32;
    if (kc >= p.C) {
      kc = 0;
      if (++ks == p.S) { ks = 0; ++kr; }
    }
  };
  f32x4 acc[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int u = 0; u < PF; ++u)
    if (u < nsteps) issue(u);
  for (int s0 = 0; s0 < nsteps; s0 += PF) {
#pragma unroll
    for (int u = 0; u < PF; ++u) {
      if (s0 + u >= nsteps) break;
      const bf16x8 fb = __builtin_bit_cast(bf16x8, rb[u]);
#pragma unroll
      for (int i = 0; i < 4; ++i)
        acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb, __builtin_bit_cast(bf16x8, ra[u][i]), acc[i], 0, 0, 0);
      if (s0 + u + PF < nsteps) issue(u);
    }
  }
  // epilogue: lane holds channels n0 + 4 fq .. +3 of pixels m0 + 16 i + fr
  const int n = n0 + 4 * fq;
  const bool nok = n < p.gn;
  if (p.nsplit > 1) {
    float* ws = reinterpret_cast<float*>(p.out) + (size_t)split * p.gm * p.gn;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = m0 + 16 * i + fr;
      if (nok && m < p.gm) *reinterpret_cast<f32x4*>(ws + (size_t)m * p.gn + n) = acc[i];
    }
    return;
  }
  if (!nok) return;
  __bf16* out = reinterpret_cast<__bf16*>(p.out);
  float bias[4] = {0.f, 0.f, 0.f, 0.f};
  if (p.bias) {
#pragma unroll
    for (int e = 0; e < 4; ++e) bias[e] = p.bias[n + e];
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = m0 + 16 * i + fr;
    if (m >= p.gm) continue;
    const size_t o = (size_t)m * p.gn + n;
    float v[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = acc[i][e] + bias[e];
    if (p.resid) {
      const uint2 r = *reinterpret_cast<const uint2*>(p.resid + o);
      v[0] += __uint_as_float(r.x << 16); v[1] += __uint_as_float(r.x & 0xffff0000u);
      v[2] += __uint_as_float(r.y << 16); v[3] += __uint_as_float(r.y & 0xffff0000u);
    }
    if (p.relu) {
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = fmaxf(v[e], 0.f);
    }
    *reinterpret_cast<uint2*>(out + o) = uint2{f2bf2(v[0], v[1]), f2bf2(v[2], v[3])};
  }
}

static void launch_skinny(IgemmParams& p, hipStream_t st) {
  p.tiles_m = ceil_div(p.gm, 64);
  p.tiles_n = ceil_div(p.gn, 64);
  TORCH_CHECK(p.C % 32 == 0 && p.ksplit % 32 == 0 && p.gn % 4 == 0, "skinny_fwd: C, ksplit multiples of 32");
  TORCH_CHECK(p.relu < 2, "skinny_fwd: ReLU / plain epilogue only");
  const int grid = p.tiles_m * p.tiles_n * p.nsplit;
  hipLaunchKernelGGL(skinny_fwd_kernel<8>, dim3(grid), dim3(NT), 0, st, p);
  PCMP_LAUNCH_CHECK();
}

// ------------------------------------------------------------------------------------------------
// split-K reduction: dst[i] (+)= sum_s ws[s][i]   (fp32, float4)
static __global__ void splitk_reduce_kernel(const float* __restrict__ ws, float* __restrict__ dst,
                                     int64_t n, int nsplit, int accumulate) {
  const int64_t n4 = n >> 2;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n4;
       i += (int64_t)gridDim.x * blockDim.x) {
    f32x4 s = reinterpret_cast<const f32x4*>(ws)[i];
    int k = 1;
    for (; k + 4 <= nsplit; k += 4) {
      const f32x4 a = reinterpret_cast<const f32x4*>(ws + (size_t)k * n)[i];
      const f32x4 b = reinterpret_cast<const f32x4*>(ws + (size_t)(k + 1) * n)[i];
      const f32x4 c = reinterpret_cast<const f32x4*>(ws + (size_t)(k + 2) * n)[i];
      const f32x4 d = reinterpret_cast<const f32x4*>(ws + (size_t)(k + 3) * n)[i];
      s += (a + b) + (c + d);
    }
    for (; k < nsplit; ++k) s += reinterpret_cast<const f32x4*>(ws + (size_t)k * n)[i];
    if (accumulate) s += reinterpret_cast<f32x4*>(dst)[i];
    reinterpret_cast<f32x4*>(dst)[i] = s;
  }
}

// split-K reduction v2: the split dimension is spread over SL thread lanes of a block as well
// (COLS = 256/SL float4 columns per block), so a reduction of few columns over many splits (WGRAD
// of a 64x576 filter over 256 splits: 36 blocks of 256 threads in v1, each walking all 256 slabs
// serially) runs on SL x more workgroups with SL x shorter dependent chains.  Each lane sums its
// splits l, l+SL, ... in groups of four ((a+b)+(c+d)); the lanes are combined in lane order through
// LDS -- a fixed order for a given split count, so results are run-to-run deterministic.
template <int SL>
__global__ void __launch_bounds__(256) splitk_reduce2_kernel(const float* __restrict__ ws, float* __restrict__ dst,
                                                             int n4, int nsplit, int accumulate) {
  constexpr int COLS = 256 / SL;
  __shared__ f32x4 sh[SL][COLS];
  const int c = threadIdx.x % COLS, l = threadIdx.x / COLS;
  const int col = blockIdx.x * COLS + c;
  const f32x4* w4 = reinterpret_cast<const f32x4*>(ws);
  f32x4 s = {0.f, 0.f, 0.f, 0.f};
  if (col < n4) {
    int k = l;
    for (; k + 3 * SL < nsplit; k += 4 * SL) {
      const f32x4 a = w4[(size_t)k * n4 + col], b = w4[(size_t)(k + SL) * n4 + col];
      const f32x4 cc = w4[(size_t)(k + 2 * SL) * n4 + col], d = w4[(size_t)(k + 3 * SL) * n4 + col];
      s += (a + b) + (cc + d);
    }
    for (; k < nsplit; k += SL) s += w4[(size_t)k * n4 + col];
  }
  if constexpr (SL == 1) {
    if (col < n4) {
      if (accumulate) s += reinterpret_cast<f32x4*>(dst)[col];
      reinterpret_cast<f32x4*>(dst)[col] = s;
    }
    return;
  } else {
    sh[l][c] = s;
    __syncthreads();
    if (l == 0 && col < n4) {
      f32x4 t = sh[0][c];
#pragma unroll
      for (int j = 1; j < SL; ++j) t += sh[j][c];
      if (accumulate) t += reinterpret_cast<f32x4*>(dst)[col];
      reinterpret_cast<f32x4*>(dst)[col] = t;
    }
  }
}

// split-K forward reduction + fused epilogue: out = act(sum_s ws[s] + bias (+ resid)) as bf16
static __global__ void __launch_bounds__(256) splitk_epilogue_kernel(const float* __restrict__ ws, __bf16* __restrict__ out,
                                                              const float* __restrict__ bias,
                                                              const __bf16* __restrict__ resid, int64_t n, int gn,
                                                              int nsplit, int relu, __bf16* __restrict__ aux) {
  // one float4 column per thread over a grid that covers the output (the layout of the BN apply
  // kernels, profiles/r2_ew_apply_ab.txt); the split slabs are read four at a time
  const int64_t n4 = n >> 2;
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= n4) return;
  const f32x4* w4 = reinterpret_cast<const f32x4*>(ws);
  f32x4 s = w4[i];
  int k = 1;
  for (; k + 3 < nsplit; k += 4) {
    const f32x4 a = w4[(size_t)k * n4 + i], b = w4[(size_t)(k + 1) * n4 + i];
    const f32x4 c = w4[(size_t)(k + 2) * n4 + i], d = w4[(size_t)(k + 3) * n4 + i];
    s += (a + b) + (c + d);
  }
  for (; k < nsplit; ++k) s += w4[(size_t)k * n4 + i];
  const int c = (int)((i * 4) % gn);
  u16x4 rv, ov, av;
  if (resid) rv = reinterpret_cast<const u16x4*>(resid)[i];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    float x = s[e] + (bias ? bias[c + e] : 0.f);
    if (resid) x = relu == 3 ? x * dgelu_fast(bf2f(rv[e])) : x + bf2f(rv[e]);
    if (relu == 1) x = fmaxf(x, 0.f);
    else if (relu == 2) { av[e] = f2bf(x); x = gelu_fast(bf2f(av[e])); }
    ov[e] = f2bf(x);
  }
  reinterpret_cast<u16x4*>(out)[i] = ov;
  if (relu == 2) reinterpret_cast<u16x4*>(aux)[i] = av;
}

// weight transpose for DGRAD: wt[c][t][k] = w[k][r(t)][s(t)][c]  (bf16), taps t over a
// (possibly strided) sub-grid r = r0 + rstep*(t / subS), s = s0 + rstep*(t % subS).
static __global__ void wt_transpose_kernel(const unsigned short* __restrict__ w, unsigned short* __restrict__ wt,
                                    int K, int R, int S, int C, int r0, int s0, int rstep, int subS, int T) {
  __shared__ unsigned short tile[64][65];
  const int t = blockIdx.z;
  const int rsrc = (r0 + rstep * (t / subS)) * S + s0 + rstep * (t % subS);
  const int k0 = blockIdx.y * 64, c0 = blockIdx.x * 64;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;  // 256 threads: 4 rows per pass
  for (int r = ty; r < 64; r += 4) {
    const int k = k0 + r, c = c0 + tx;
    tile[r][tx] = (k < K && c < C) ? w[((size_t)k * R * S + rsrc) * C + c] : 0;
  }
  __syncthreads();
  for (int r = ty; r < 64; r += 4) {
    const int c = c0 + r, k = k0 + tx;
    if (c < C && k < K) wt[((size_t)c * T + t) * K + k] = tile[tx][r];
  }
}

// Batched weight transpose of a whole model's conv weights in ONE launch (after each optimizer
// step, instead of one wt_transpose launch per DGRAD): desc[i] = {src_off, dst_off, K, T, C,
// first_block, S, RS, r0, s0, step, subS} (offsets in elements of the flat bf16 shadow /
// transposed-shadow buffers); block b handles one 64x64 (k, c) tile of one tap of entry i = the
// last i with first_block <= b.  Entry tap t (of T) reads source tap
// (r0 + step*(t / subS)) * S + s0 + step*(t % subS) of the [K][RS][C] weight and writes
// dst[c][t][k]: the whole filter (r0 = s0 = 0, step 1, subS = S) or one stride-2 sub-pixel class
// (step 2), whose DGRAD GEMM then reads its taps without a per-call transpose.
static __global__ void wt_transpose_multi_kernel(const unsigned short* __restrict__ src, unsigned short* __restrict__ dst,
                                          const int64_t* __restrict__ desc, int n) {
  __shared__ unsigned short tile[64][65];
  const int b = blockIdx.x;
  int lo = 0, hi = n - 1;   // binary search on first_block (block-uniform)
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (desc[mid * 12 + 5] <= b) lo = mid; else hi = mid - 1;
  }
  const int64_t* d = desc + lo * 12;
  const unsigned short* w = src + d[0];
  unsigned short* wt = dst + d[1];
  const int K = (int)d[2], T = (int)d[3], C = (int)d[4];
  const int S = (int)d[6], RS = (int)d[7], r0 = (int)d[8], s0 = (int)d[9], step = (int)d[10], subS = (int)d[11];
  const int nc = (C + 63) / 64, nk = (K + 63) / 64;
  int local = b - (int)d[5];
  const int t = local / (nc * nk);
  local -= t * nc * nk;
  const int k0 = (local / nc) * 64, c0 = (local % nc) * 64;
  const int ts = (r0 + step * (t / subS)) * S + s0 + step * (t % subS);
  if ((C & 7) == 0 && (K & 7) == 0 && (d[0] & 7) == 0 && (d[1] & 7) == 0) {
    // 16-byte path (every BERT / ResNet weight): each thread moves two 8-element chunks in and two
    // out, so a wave's load / store instruction covers 8 rows x 128 B instead of 1 row x 128 B
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int j = threadIdx.x + 256 * u;
      const int r = j >> 3, cc = (j & 7) * 8;
      const int k = k0 + r, c = c0 + cc;
      uint4 v = {0u, 0u, 0u, 0u};
      if (k < K && c < C) v = *reinterpret_cast<const uint4*>(w + ((size_t)k * RS + ts) * C + c);
      const unsigned short* e = reinterpret_cast<const unsigned short*>(&v);
#pragma unroll
      for (int q = 0; q < 8; ++q) tile[r][cc + q] = e[q];
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int j = threadIdx.x + 256 * u;
      const int r = j >> 3, kc = (j & 7) * 8;   // r: output row (c), kc: first k of the chunk
      const int c = c0 + r, k = k0 + kc;
      if (c < C && k < K) {
        uint4 v;
        unsigned short* e = reinterpret_cast<unsigned short*>(&v);
#pragma unroll
        for (int q = 0; q < 8; ++q) e[q] = tile[kc + q][r];
        *reinterpret_cast<uint4*>(wt + ((size_t)c * T + t) * K + k) = v;
      }
    }
    return;
  }
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  for (int r = ty; r < 64; r += 4) {
    const int k = k0 + r, c = c0 + tx;
    tile[r][tx] = (k < K && c < C) ? w[((size_t)k * RS + ts) * C + c] : 0;
  }
  __syncthreads();
  for (int r = ty; r < 64; r += 4) {
    const int c = c0 + r, k = k0 + tx;
    if (c < C && k < K) wt[((size_t)c * T + t) * K + k] = tile[tx][r];
  }
}

// ------------------------------------------------------------------------------------------------
// host side
template <int MODE, int BM, int BN, int WM, int WN>
static void launch_cfg(IgemmParams& p, hipStream_t st) {
  p.tiles_m = ceil_div(p.gm, BM);
  p.tiles_n = ceil_div(p.gn, BN);
  TORCH_CHECK(MODE == MODE_WGRAD || !p.stats || p.tiles_m <= p.stats_cap, "igemm: partial-stats buffer too small");
  const int grid = p.tiles_m * p.tiles_n * p.nsplit;
  const size_t stage_bytes = (size_t)(BM + BN) * BK * 2;
  const int nk = ceil_div(std::min(p.ksplit, p.gk), BK);
  size_t smem = (nk > 1 ? 2 : 1) * stage_bytes;
  const bool epi_red = (MODE == MODE_FWD && p.stats) || (MODE == MODE_DGRAD && p.bn_x);
  if (epi_red) {  // epilogue column-sum scratch: 4 waves x [16][NS*WTN+4] + [WM][NS][BN] floats
    const int NS = MODE == MODE_DGRAD && p.bn_x2 ? 3 : 2;
    smem = std::max(smem, (size_t)(4 * 16 * (NS * (BN / WN) + 4) + WM * NS * BN) * sizeof(float));
  }
  const int cin = MODE == MODE_FWD ? p.C : p.K;
  const bool unif = MODE != MODE_WGRAD && cin % BK == 0 && p.ksplit % BK == 0;
  int epi = EPI_PLAIN;
  if (MODE == MODE_FWD && p.stats) epi = EPI_STATS;
  if (MODE == MODE_DGRAD && p.bn_x) epi = p.bn_x2 ? EPI_BNR2 : EPI_BNR;
#define PCMP_IGEMM_LAUNCH(U, E)                                                                       \
  do {                                                                                              \
    auto kf_ = &igemm_kernel<MODE, BM, BN, WM, WN, U, E>;                                            \
    static bool attr_ = false;                                                                      \
    if (!attr_) {                                                                                   \
      PCMP_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(kf_),                        \
                                         hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));  \
      attr_ = true;                                                                                 \
    }                                                                                               \
    hipLaunchKernelGGL(kf_, dim3(grid), dim3(NT), smem, st, p);                                     \
  } while (0)
  if constexpr (MODE == MODE_FWD) {
    if (epi == EPI_STATS) {
      if (unif) PCMP_IGEMM_LAUNCH(true, EPI_STATS); else PCMP_IGEMM_LAUNCH(false, EPI_STATS);
    } else if (p.relu >= 2) {
      if (unif) PCMP_IGEMM_LAUNCH(true, EPI_GELU); else PCMP_IGEMM_LAUNCH(false, EPI_GELU);
    } else {
      if (unif) PCMP_IGEMM_LAUNCH(true, EPI_PLAIN); else PCMP_IGEMM_LAUNCH(false, EPI_PLAIN);
    }
  } else if constexpr (MODE == MODE_DGRAD) {
    const bool deep = kn_epi_depth.get() >= 4;
#define PCMP_IGEMM_LAUNCH_D(U, E)                                                                     \
  do {                                                                                              \
    auto kf_ = &igemm_kernel<MODE, BM, BN, WM, WN, U, E, 4>;                                         \
    static bool attr_ = false;                                                                      \
    if (!attr_) {                                                                                   \
      PCMP_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(kf_),                        \
                                         hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));  \
      attr_ = true;                                                                                 \
    }                                                                                               \
    hipLaunchKernelGGL(kf_, dim3(grid), dim3(NT), smem, st, p);                                     \
  } while (0)
    if (epi == EPI_BNR) {
      if (deep) { if (unif) PCMP_IGEMM_LAUNCH_D(true, EPI_BNR); else PCMP_IGEMM_LAUNCH_D(false, EPI_BNR); }
      else if (unif) PCMP_IGEMM_LAUNCH(true, EPI_BNR); else PCMP_IGEMM_LAUNCH(false, EPI_BNR);
    } else if (epi == EPI_BNR2) {
      if (kn_epi_depth_bnr2.get() >= 4) { if (unif) PCMP_IGEMM_LAUNCH_D(true, EPI_BNR2); else PCMP_IGEMM_LAUNCH_D(false, EPI_BNR2); }
      else if (unif) PCMP_IGEMM_LAUNCH(true, EPI_BNR2); else PCMP_IGEMM_LAUNCH(false, EPI_BNR2);
#undef PCMP_IGEMM_LAUNCH_D
    } else if (p.relu >= 2) {
      if (unif) PCMP_IGEMM_LAUNCH(true, EPI_GELU); else PCMP_IGEMM_LAUNCH(false, EPI_GELU);
    } else {
      if (unif) PCMP_IGEMM_LAUNCH(true, EPI_PLAIN); else PCMP_IGEMM_LAUNCH(false, EPI_PLAIN);
    }
  } else {
    bool m32 = false;
    if constexpr ((BM / WM) % 32 == 0 && (BN / WN) % 32 == 0) {
      if (kn_wgrad_m32.get()) {
        auto kf_ = &igemm_kernel<MODE, BM, BN, WM, WN, false, EPI_PLAIN, 2, NT, 0, true>;
        static bool attr_ = false;
        if (!attr_) {
          PCMP_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(kf_),
                                             hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
          attr_ = true;
        }
        hipLaunchKernelGGL(kf_, dim3(grid), dim3(NT), smem, st, p);
        m32 = true;
      }
    }
    if (!m32) PCMP_IGEMM_LAUNCH(false, EPI_PLAIN);
  }
#undef PCMP_IGEMM_LAUNCH
  PCMP_LAUNCH_CHECK();
}

// A/B knobs (torch.ops.pcmp.set_knob; tools/gemm_knob_ab.py)

inline Knob kn_wgrad_wgs("wgrad_wgs", 0);   // > 0: fixed split-K workgroup target (side-stream WGRADs)
inline Knob kn_igemm8("igemm8", 1);
static int igemm8_mode() { return kn_igemm8.get(); }

// minimum 256x256 tile count for the 8-wave kernel (knob igemm8_min_tiles, A/B runs)
inline Knob kn_igemm8_min_tiles("igemm8_min_tiles", 160);
static int igemm8_min_tiles() { return kn_igemm8_min_tiles.get(); }

template <int MODE, int BM, int BN, int WM, int WN, int NTHR, int MINB>
static void launch_dma(IgemmParams& p, hipStream_t st) {
  p.tiles_m = ceil_div(p.gm, BM);
  p.tiles_n = ceil_div(p.gn, BN);
  TORCH_CHECK(!p.stats || p.tiles_m <= p.stats_cap, "igemm_dma: partial-stats buffer too small");
  TORCH_CHECK(p.gk % BK == 0 && (MODE == MODE_FWD ? p.C : p.K) % BK == 0 && p.ksplit % BK == 0,
              "igemm_dma: needs the block-uniform tap walk");
  TORCH_CHECK(p.nsplit == 1 || (!p.stats && !p.bn_x), "igemm_dma: split-K only with the plain epilogue");
  const int grid = p.tiles_m * p.tiles_n * p.nsplit;
  size_t smem = (size_t)2 * (BM + BN) * BK * 2;
  const bool epi_red = (MODE == MODE_FWD && p.stats) || (MODE == MODE_DGRAD && p.bn_x);
  if (epi_red) {
    const int NS = MODE == MODE_DGRAD && p.bn_x2 ? 3 : 2;
    smem = std::max(smem, (size_t)((NTHR / 64) * 16 * (NS * (BN / WN) + 4) + WM * NS * BN) * sizeof(float));
  }
  int epi = EPI_PLAIN;
  if (MODE == MODE_FWD && p.stats) epi = EPI_STATS;
  if (MODE == MODE_DGRAD && p.bn_x) epi = p.bn_x2 ? EPI_BNR2 : EPI_BNR;
#define PCMP_DMA_LAUNCH(E)                                                                              \
  do {                                                                                                \
    constexpr bool can_deep = (E == EPI_BNR || E == EPI_BNR2) && NTHR == 256;                        \
    auto kfn = (can_deep && (E == EPI_BNR2 ? kn_epi_depth_bnr2 : kn_epi_depth).get() >= 4)              \
                   ? &igemm_dma_kernel<MODE, BM, BN, WM, WN, NTHR, MINB, E, 4>                        \
                   : &igemm_dma_kernel<MODE, BM, BN, WM, WN, NTHR, MINB, E, 2>;                       \
    static bool attr_set = false;                                                                     \
    if (!attr_set) {                                                                                  \
      for (auto f : {&igemm_dma_kernel<MODE, BM, BN, WM, WN, NTHR, MINB, E, 2>,                       \
                     &igemm_dma_kernel<MODE, BM, BN, WM, WN, NTHR, MINB, E, 4>})                      \
        PCMP_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(f),                          \
                                           hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));  \
      attr_set = true;                                                                                \
    }                                                                                                 \
    hipLaunchKernelGGL(kfn, dim3(grid), dim3(NTHR), smem, st, p);                                     \
  } while (0)
  if constexpr (MODE == MODE_FWD) {
    if (epi == EPI_STATS) PCMP_DMA_LAUNCH(EPI_STATS); else if (p.relu >= 2) PCMP_DMA_LAUNCH(EPI_GELU); else PCMP_DMA_LAUNCH(EPI_PLAIN);
  } else {
    if (epi == EPI_BNR) PCMP_DMA_LAUNCH(EPI_BNR);
    else if (epi == EPI_BNR2) {
      if constexpr (NTHR == 256) PCMP_DMA_LAUNCH(EPI_BNR2);
      else TORCH_CHECK(false, "igemm8: dual BN-reduce epilogue not instantiated");
    } else if (p.relu >= 2) PCMP_DMA_LAUNCH(EPI_GELU);
    else PCMP_DMA_LAUNCH(EPI_PLAIN);
  }
#undef PCMP_DMA_LAUNCH
  PCMP_LAUNCH_CHECK();
}

// igemm_dma32_kernel in place of igemm_dma_kernel for the 4-wave 128x128 / 128x64 FWD and DGRAD
// GEMMs (use_dma4 cases 1 and 2) with at least dma32_mink K-tiles; not for the GELU epilogues (the
// planner's Linear GEMMs keep their own kernels).  Per-shape A/B on the ResNet-50 B=256 conv shapes
// with their training epilogues (profiles/r5_knob_dma32.txt): every FWD + BN-statistics GEMM gains or
// ties (l2 3x3 85.5 -> 72.4 us, l3 1x1 256->1024 60.4 -> 47.3, l4 3x3 73.3 -> 65.3, l4 1x1 2048->512
// 37.4 -> 32.8), so do the 3x3 DGRAD + BN-reduce GEMMs (l1 157.7 -> 151.0, l2 107.2 -> 102.8, l4 85.5
// -> 81.0); the short-K 1x1 DGRADs into wide outputs lose 4-30 % (l3 1x1 1024->256 125.6 -> 139.8, its
// dual-BN form 153 -> 200) and stay on igemm_dma_kernel: DGRAD takes the new kernel for filters wider
// than 1x1 or >= dma32_dgrad_mink K-tiles.  Knob dma32 = 0 restores igemm_dma_kernel (A/B).
inline Knob kn_dma32("dma32", 1);
inline Knob kn_dma32_modes("dma32_modes", 1);   // bit 0: FWD, bit 1: DGRAD (whole-step A/B: FWD only, profiles/r5_bench_ab_dma32_modes.txt)
inline Knob kn_dma32_mink("dma32_mink", 3);
inline Knob kn_dma32_dgrad_mink("dma32_dgrad_mink", 16);
static bool use_dma32(int mode, const IgemmParams& p) {
  if (!kn_dma32.get() || mode == MODE_WGRAD || p.nsplit != 1 || p.relu >= 2 || p.gn % 8 != 0 ||
      p.gk / BK < kn_dma32_mink.get())
    return false;
  if (!(kn_dma32_modes.get() & (mode == MODE_FWD ? 1 : 2))) return false;
  return mode == MODE_FWD || p.R * p.S > 1 || p.gk / BK >= kn_dma32_dgrad_mink.get();
}

template <int MODE, int BM, int BN, int WM, int WN>
static void launch_dma32(IgemmParams& p, hipStream_t st) {
  p.tiles_m = ceil_div(p.gm, BM);
  p.tiles_n = ceil_div(p.gn, BN);
  TORCH_CHECK(!p.stats || p.tiles_m <= p.stats_cap, "igemm_dma32: partial-stats buffer too small");
  TORCH_CHECK(p.gk % BK == 0 && (MODE == MODE_FWD ? p.C : p.K) % BK == 0 && p.ksplit >= p.gk && p.nsplit == 1,
              "igemm_dma32: needs the block-uniform tap walk and no split-K");
  TORCH_CHECK(p.relu < 2 && p.gn % 8 == 0, "igemm_dma32: conv epilogues with 8-channel groups only");
  TORCH_CHECK(p.gk / BK >= 2, "igemm_dma32: at least two K-tiles");
  const int grid = p.tiles_m * p.tiles_n;
  constexpr size_t smem = (size_t)2 * (BM + BN) * BK * 2 + (size_t)(6 * BN + WM * 3 * BN) * sizeof(float);
  static_assert(2 * smem <= 160 * 1024, "igemm_dma32: two blocks per CU");
  int epi = EPI_PLAIN;
  if (MODE == MODE_FWD && p.stats) epi = EPI_STATS;
  if (MODE == MODE_DGRAD && p.bn_x) epi = p.bn_x2 ? EPI_BNR2 : EPI_BNR;
#define PCMP_DMA32_LAUNCH(E, D)                                                                        \
  do {                                                                                                \
    auto kfn = &igemm_dma32_kernel<MODE, BM, BN, WM, WN, E, D>;                                        \
    static bool attr_set = false;                                                                     \
    if (!attr_set) {                                                                                  \
      PCMP_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(kfn),                          \
                                         hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));    \
      attr_set = true;                                                                                \
    }                                                                                                 \
    hipLaunchKernelGGL(kfn, dim3(grid), dim3(256), smem, st, p);                                      \
  } while (0)
  if constexpr (MODE == MODE_FWD) {
    if (epi == EPI_STATS) PCMP_DMA32_LAUNCH(EPI_STATS, 2); else PCMP_DMA32_LAUNCH(EPI_PLAIN, 2);
  } else {
    if (epi == EPI_BNR) {
      if (kn_epi_depth.get() >= 4) PCMP_DMA32_LAUNCH(EPI_BNR, 4); else PCMP_DMA32_LAUNCH(EPI_BNR, 2);
    } else if (epi == EPI_BNR2) {
      if (kn_epi_depth_bnr2.get() >= 4) PCMP_DMA32_LAUNCH(EPI_BNR2, 4); else PCMP_DMA32_LAUNCH(EPI_BNR2, 2);
    } else {
      PCMP_DMA32_LAUNCH(EPI_PLAIN, 2);
    }
  }
#undef PCMP_DMA32_LAUNCH
  PCMP_LAUNCH_CHECK();
}

// 4-wave LDS-DMA kernel (2 blocks per CU) in place of the register-staged 4-wave kernel for the
// FWD/DGRAD GEMMs with the block-uniform tap walk and >= 3 K-tiles (measured
// profiles/r1_dma4_ab.txt: 3x3 layers 10-16 % faster, e.g. layer4 3x3 DGRAD 97 -> 84 us; GEMMs
// of 2 K-tiles ran up to 9 % slower).  Knob dma4 = 0 disables it (A/B runs); knob dma4_n64 picks
// the narrow-output (gn <= 64) tile: 1 = 128x64 (2x2 waves of 64x32, the default: 6 % faster than
// 256x64 on the layer1 3x3), 2 = 256x64 (4x1 waves of 64x64), 0 = register-staged kernel.
inline Knob kn_dma4("dma4", 1);
inline Knob kn_dma4_n64("dma4_n64", 1);
static int dma4_mode() { return kn_dma4.get(); }
static int dma4_n64() { return kn_dma4_n64.get(); }
// 0: register-staged kernel; 1: 128x128; 2: 128x64; 3: 256x64
// FWD grids with fewer 128x128 tiles than CUs (the B=64 transfer-learning step's layer-3/4 convs:
// 100-196 tiles) take 128x64 tiles: twice the workgroups (dma4_small_n64 = 0: 128x128)
inline Knob kn_dma4_small_n64("dma4_small_n64", 1);   // TL step 2.43 -> 2.38 ms (profiles/r6_tl_small_n64_ab.txt)
static int use_dma4(int mode, const IgemmParams& p) {
  if (!dma4_mode() || mode == MODE_WGRAD || p.nsplit != 1) return 0;
  const int cin = mode == MODE_FWD ? p.C : p.K;
  if (cin % BK != 0 || p.gk % BK != 0 || p.gk / BK < 3 || p.gm <= 64) return 0;
  if (p.gn <= 64) {
    const int v = dma4_n64();
    return v == 1 ? 2 : (v == 2 ? 3 : 0);
  }
  if (mode == MODE_FWD && kn_dma4_small_n64.get() && ceil_div(p.gm, 128) * ceil_div(p.gn, 128) < 256) return 2;
  return 1;
}

// halo-tiled direct conv for the layer-1 3x3 / stem shapes: bit 0 FWD, bit 1 every DGRAD variant,
// bit 2 the overlapped BN-backward DGRAD.  DGRAD is off by default: its BN-backward epilogue loads
// stall the one wave per SIMD (profiles/r2_halo_conv.txt)
inline Knob kn_halo("halo", 1);
inline Knob kn_halo_ovl("halo_ovl", 1);   // output stores overlapped with the next tile's MFMAs

static bool halo_dgrad_ovl(const IgemmParams& p) {
  return kn_halo_ovl.get() && p.bn_x && !p.bn_x2 && !p.resid && !p.relu && !p.bn_mask && !p.bn_mbits && p.bn_msc &&
         p.bn_msh;
}

// Eligibility + geometry of halo_conv_kernel: stride 1, square filter, 64 output channels and
// (C, R) = (64, 3) [layer-1 3x3, FWD and DGRAD] or (16, 4) [space-to-depth stem, FWD]; the output
// width divides 224 (a tile = whole rows) and the grid has at least one tile per CU.
static bool halo_geom(int mode, const IgemmParams& p, HaloGeom& g) {
  const int hk = kn_halo.get();
  if ((mode == MODE_FWD && !(hk & 1)) || (mode == MODE_DGRAD && !(hk & 6)) || mode == MODE_WGRAD || p.nsplit != 1 || p.stride != 1 || p.R != p.S || p.gn != 64 ||
      p.sub || p.relu >= 2)
    return false;
  int CS, pad;
  if (mode == MODE_FWD) {
    CS = p.C; g.Hs = p.H; g.Ws = p.W; g.Ho = p.P; g.Wo = p.Q; pad = p.pad;
    if (p.bias) return false;
  } else {
    CS = p.K; g.Hs = p.P; g.Ws = p.Q; g.Ho = p.H; g.Wo = p.W; pad = p.R - 1 - p.pad;
    if (p.bn_x2 || pad < 0) return false;
    // bit 1 enables every DGRAD variant, bit 2 only the overlapped BN-backward form (mask
    // recomputed from x, no residual)
    if (!(hk & 2) && !((hk & 4) && halo_dgrad_ovl(p))) return false;
  }
  // compiled geometries: layer-1 3x3 at 56 wide, the space-to-depth stem at 112 wide
  if (!((CS == 64 && p.R == 3 && g.Wo == 56) || (CS == 16 && p.R == 4 && g.Wo == 112 && mode == MODE_FWD)))
    return false;
  g.TR = HALO_BM / g.Wo;
  if (g.Ho % g.TR != 0 || g.Ho != g.Hs + 2 * pad - p.R + 1 || g.Wo != g.Ws + 2 * pad - p.S + 1) return false;
  g.tiles_img = g.Ho / g.TR;
  g.tiles = p.N * g.tiles_img;
  if (g.tiles < 256 || (int64_t)g.tiles * HALO_BM != (int64_t)p.gm) return false;
  g.padT = pad; g.padL = pad;
  g.HWd = g.Wo + p.S - 1;
  g.HWp = (g.HWd + 15 + 15) / 16 * 16;    // room for the 0..15-slot row skew, multiple of 16
  g.HR = g.TR + p.R - 1;
  g.ninstr = ceil_div(g.HR * (CS / 8) * g.HWp * 16, 1024);
  g.lds_bytes = g.ninstr * 1024;
  if (2 * g.lds_bytes + HALO_BM * 64 * 2 + 768 * (int)sizeof(float) > 160 * 1024) return false;
  g.src = p.a; g.src_bytes = p.a_bytes; g.wsrc = p.b;
  g.fd_HWp = make_fastdiv(g.HWp);
  g.fd_Wo = make_fastdiv(g.Wo);
  g.fd_timg = make_fastdiv(g.tiles_img);
  return true;
}
static bool use_halo(int mode, const IgemmParams& p) {
  HaloGeom g;
  return halo_geom(mode, p, g);
}

template <int MODE>
static void launch_halo(IgemmParams& p, hipStream_t st) {
  HaloGeom g;
  TORCH_CHECK(halo_geom(MODE, p, g), "halo_conv: shape not eligible");
  p.tiles_m = g.tiles;
  p.tiles_n = 1;
  TORCH_CHECK(!p.stats || p.tiles_m <= p.stats_cap, "halo_conv: partial-stats buffer too small");
  const int grid = std::min(g.tiles, 256);
  size_t smem = (size_t)2 * g.lds_bytes + 768 * sizeof(float);
  const int CS = MODE == MODE_FWD ? p.C : p.K;
#define PCMP_HALO_LAUNCH(E, C_, R_, FL, WO_, OV)                                                       \
  do {                                                                                                 \
    auto kfn = &halo_conv_kernel<MODE, E, C_, R_, FL, WO_, OV>;                                        \
    static bool attr_set = false;                                                                      \
    if (!attr_set) {                                                                                   \
      PCMP_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(kfn),                           \
                                         hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));     \
      attr_set = true;                                                                                 \
    }                                                                                                  \
    hipLaunchKernelGGL(kfn, dim3(grid), dim3(NT), smem, st, p, g);                                     \
  } while (0)
  if constexpr (MODE == MODE_FWD) {
    const bool ovl = !p.resid && !p.relu && !p.bias && kn_halo_ovl.get();
    if (ovl) smem += (size_t)HALO_BM * 64 * 2;
    if (CS == 64) {
      if (ovl) {
        if (p.stats) PCMP_HALO_LAUNCH(EPI_STATS, 64, 3, false, 56, true); else PCMP_HALO_LAUNCH(EPI_PLAIN, 64, 3, false, 56, true);
      } else {
        if (p.stats) PCMP_HALO_LAUNCH(EPI_STATS, 64, 3, false, 56, false); else PCMP_HALO_LAUNCH(EPI_PLAIN, 64, 3, false, 56, false);
      }
    } else {
      if (ovl) {
        if (p.stats) PCMP_HALO_LAUNCH(EPI_STATS, 16, 4, false, 112, true); else PCMP_HALO_LAUNCH(EPI_PLAIN, 16, 4, false, 112, true);
      } else {
        if (p.stats) PCMP_HALO_LAUNCH(EPI_STATS, 16, 4, false, 112, false); else PCMP_HALO_LAUNCH(EPI_PLAIN, 16, 4, false, 112, false);
      }
    }
  } else if constexpr (MODE == MODE_DGRAD) {
    if (halo_dgrad_ovl(p)) {
      smem += (size_t)HALO_BM * 64 * 2;
      PCMP_HALO_LAUNCH(EPI_BNR, 64, 3, true, 56, true);
    } else if (p.bn_x) {
      PCMP_HALO_LAUNCH(EPI_BNR, 64, 3, true, 56, false);
    } else {
      PCMP_HALO_LAUNCH(EPI_PLAIN, 64, 3, true, 56, false);
    }
  }
#undef PCMP_HALO_LAUNCH
  PCMP_LAUNCH_CHECK();
}

// 8-wave LDS-DMA kernel eligibility: FWD/DGRAD with the block-uniform tap walk (source channels a
// multiple of BK), no split-K, enough K-tiles for the phase pipeline, and a grid that still covers
// most CUs with BM = 256 tiles: >= 160 tiles (ResNet-50 layer3 at B=256 has 196 and runs 20-28 %
// faster than on the 4-wave kernel's 784 tiles; layer4's 98 tiles run 25-35 % slower, measured
// profiles/r1_igemm8_mintiles_ab.txt), and >= 8 K-tiles: with one block per CU a short main loop
// cannot hide the load / epilogue latency that two 4-wave blocks per CU overlap (1x1 convs over
// 256 input channels ran 6-12 % faster on the 4-wave kernel, profiles/r1_igemm8_ab_v2.txt).
// PCMP_IGEMM8=0 disables it (A/B runs).
static int use_igemm8(int mode, const IgemmParams& p) {
  if (!igemm8_mode() || mode == MODE_WGRAD || p.nsplit != 1) return 0;
  const int cin = mode == MODE_FWD ? p.C : p.K;
  if (cin % BK != 0 || p.gk % BK != 0 || p.gk / BK < 8 || p.gn < 256) return 0;
  // (measured: the BN=128 variant does not beat the 4-wave 128x128 kernel; the dual BN-reduce
  //  epilogue of a 128x64 wave tile spills)
  if (mode == MODE_DGRAD && p.bn_x2) return 0;
  if (ceil_div(p.gm, BM8) * ceil_div(p.gn, 256) < igemm8_min_tiles()) return 0;
  return 256;
}

// WGRAD tiles with 64x64 wave tiles where one GEMM side is narrow: RSC <= 64 (gn) -> 256x64 with
// the 4 waves along M; cout <= 64 (gm) -> 64x256 with the waves along N, only for the Cin=8 stem
// (measured profiles/r1_wgrad_wide_ab.txt: stem -7 %, 1x1 64->256 -5 %, but the layer1 3x3 and
// 1x1 256->64 WGRADs ran 5-16 % slower on 64x256).  Knob wg64 = 0 disables them (A/B runs).
inline Knob kn_wg64("wg64", 1);
static int wgrad_wide(const IgemmParams& p) {
  if (!kn_wg64.get()) return 0;
  if (p.gm > 32 && p.gm <= 64 && p.gn >= 256 && (p.C == 8 || p.C == 16)) return 1;   // 64 x 256 (stem)
  if (p.gn > 32 && p.gn <= 64 && p.gm >= 256) return 2;   // 256 x 64
  return 0;
}

static void wgrad_tile(const IgemmParams& p, int& BM, int& BN) {
  if (p.fold_x || p.act_sc) {   // launch_fold's choice
    if (!p.act_sc && wgrad_wide(p) == 1) { BM = 64; BN = 256; return; }
    BM = p.gm <= 64 ? 64 : 128;
    BN = p.gn <= 64 ? 64 : 128;
    return;
  }
  const int w = wgrad_wide(p);
  if (w == 1) { BM = 64; BN = 256; return; }
  if (w == 2) { BM = 256; BN = 64; return; }
  BM = p.gm <= 32 ? 32 : (p.gm <= 64 ? 64 : 128);
  BN = p.gn <= 64 ? 64 : 128;
}

// FWD/DGRAD grids of fewer 128x128 tiles than CUs (BERT-base's M=4096 token GEMMs with N=768:
// 192 tiles) run 64x128 tiles instead: twice the workgroups, every CU busy.  Knob bm64_smallgrid =
// 0 disables it (A/B runs).  FWD convs with BN statistics keep the LDS-DMA tiles (bm64_smallgrid = 1):
// the ResNet-50 transfer-learning step at B=64 (layer-3/4 convs: 100-196 tiles) ran 2.41 -> 2.38
// ms/step without the 64x128 register-staged form (profiles/r6_tl_bm64_ab.txt, r6_tl_bm64_ab2.txt); 2 = every GEMM.
inline Knob kn_bm64_smallgrid("bm64_smallgrid", 1);
static bool use_bm64_smallgrid(int mode, const IgemmParams& p) {
  if (!(mode != MODE_WGRAD && p.nsplit == 1 && p.gm > 64 && p.gn > 64)) return false;
  const int k = kn_bm64_smallgrid.get();
  if (k == 0 || (k == 1 && mode == MODE_FWD && p.stats)) return false;   // (conv_fwd sets p.stats before igemm_bm)
  return ceil_div(p.gm, 128) * ceil_div(p.gn, 128) < 256;
}

// BM of the kernel dispatch<> will pick (per-tile partial statistics are allocated per BM row tile)
static int igemm_bm(int mode, const IgemmParams& p) {
  if (p.fold_x || p.act_sc) return 128;
  if (use_halo(mode, p)) return HALO_BM;
  if (use_igemm8(mode, p)) return BM8;
  if (use_bm64_smallgrid(mode, p)) return 64;
  if (use_dma4(mode, p) == 3) return 256;
  return p.gm <= 32 ? 32 : (p.gm <= 64 ? 64 : 128);
}

// BatchNorm fold launches (IgemmParams::fold_x / act_sc): register-staged kernel only -- the LDS-DMA
// kernels move operands straight into LDS with no register pass in which the operand could be formed.
template <int MODE, int BM, int BN, int WM, int WN, int FOLD>
static void launch_fold_cfg(IgemmParams& p, hipStream_t st) {
  p.tiles_m = ceil_div(p.gm, BM);
  p.tiles_n = ceil_div(p.gn, BN);
  TORCH_CHECK(MODE == MODE_WGRAD || !p.stats || p.tiles_m <= p.stats_cap, "igemm fold: partial-stats buffer too small");
  const int grid = p.tiles_m * p.tiles_n * p.nsplit;
  const int nk = ceil_div(std::min(p.ksplit, p.gk), BK);
  size_t smem = (size_t)(nk > 1 ? 2 : 1) * (BM + BN) * BK * 2;
  const bool epi_red = (MODE == MODE_FWD && p.stats) || (MODE == MODE_DGRAD && p.bn_x);
  if (epi_red) {
    const int NS = MODE == MODE_DGRAD && p.bn_x2 ? 3 : 2;
    smem = std::max(smem, (size_t)(4 * 16 * (NS * (BN / WN) + 4) + WM * NS * BN) * sizeof(float));
  }
  if (MODE != MODE_WGRAD) {   // the coefficient copy sits after every buffer the kernel uses
    p.fold_lds = (int)((smem + 15) / 16 * 16);
    smem = (size_t)p.fold_lds + (MODE == MODE_FWD ? (size_t)2 * p.C : (size_t)3 * p.K) * sizeof(float);
  }
#define PCMP_FOLD_LAUNCH(U, E, D)                                                                     \
  do {                                                                                              \
    auto kf_ = &igemm_kernel<MODE, BM, BN, WM, WN, U, E, D, NT, FOLD>;                               \
    static bool attr_ = false;                                                                      \
    if (!attr_) {                                                                                   \
      PCMP_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(kf_),                        \
                                         hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));  \
      attr_ = true;                                                                                 \
    }                                                                                               \
    hipLaunchKernelGGL(kf_, dim3(grid), dim3(NT), smem, st, p);                                     \
  } while (0)
  if constexpr (MODE == MODE_DGRAD) {
    TORCH_CHECK(p.bn_x, "igemm fold: DGRAD only with the fused BN-backward-reduce epilogue");
    if (p.bn_x2) {
      if (kn_epi_depth_bnr2.get() >= 4) PCMP_FOLD_LAUNCH(true, EPI_BNR2, 4); else PCMP_FOLD_LAUNCH(true, EPI_BNR2, 2);
    } else {
      if (kn_epi_depth.get() >= 4) PCMP_FOLD_LAUNCH(true, EPI_BNR, 4); else PCMP_FOLD_LAUNCH(true, EPI_BNR, 2);
    }
  } else if constexpr (MODE == MODE_FWD) {
    if (p.stats) PCMP_FOLD_LAUNCH(true, EPI_STATS, 2); else PCMP_FOLD_LAUNCH(true, EPI_PLAIN, 2);
  } else {
    bool m32 = false;
    if constexpr ((BM / WM) % 32 == 0 && (BN / WN) % 32 == 0) {
      if (kn_wgrad_m32.get()) {
        auto kf_ = &igemm_kernel<MODE, BM, BN, WM, WN, false, EPI_PLAIN, 2, NT, FOLD, true>;
        static bool attr_ = false;
        if (!attr_) {
          PCMP_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(kf_),
                                             hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
          attr_ = true;
        }
        hipLaunchKernelGGL(kf_, dim3(grid), dim3(NT), smem, st, p);
        m32 = true;
      }
    }
    if (!m32) PCMP_FOLD_LAUNCH(false, EPI_PLAIN, 2);
  }
#undef PCMP_FOLD_LAUNCH
  PCMP_LAUNCH_CHECK();
}

template <int MODE>
static void launch_fold(IgemmParams& p, hipStream_t st) {
  if constexpr (MODE == MODE_DGRAD) {
    TORCH_CHECK(p.fold_x && !p.act_sc, "igemm fold: DGRAD folds only the BatchNorm-backward dz");
    TORCH_CHECK(p.R == 1 && p.S == 1 && p.stride == 1 && p.K % BK == 0 && p.nsplit == 1 && p.ksplit % BK == 0,
                "igemm fold: DGRAD of a 1x1 stride-1 conv with K % 64 == 0, no split");
    if (p.gn <= 64) launch_fold_cfg<MODE, 128, 64, 2, 2, 1>(p, st);
    else launch_fold_cfg<MODE, 128, 128, 2, 2, 1>(p, st);
  } else if constexpr (MODE == MODE_FWD) {
    TORCH_CHECK(p.act_sc && p.act_sh && !p.fold_x, "igemm fold: FWD folds only the BatchNorm-forward activation");
    TORCH_CHECK(p.R == 1 && p.S == 1 && p.stride == 1 && p.C % BK == 0 && p.nsplit == 1 && p.ksplit % BK == 0,
                "igemm fold: FWD of a 1x1 stride-1 conv with C % 64 == 0, no split");
    if (p.gn <= 64) launch_fold_cfg<MODE, 128, 64, 2, 2, 1>(p, st);
    else launch_fold_cfg<MODE, 128, 128, 2, 2, 1>(p, st);
  } else {
    TORCH_CHECK(p.K % 8 == 0 && p.C % 8 == 0, "igemm fold: WGRAD needs K % 8 == 0 and C % 8 == 0");
    if (p.act_sc) {   // B-operand fold (optionally with the A-operand dz fold): 128-row tiles
      TORCH_CHECK(p.gm > 64, "igemm fold: WGRAD activation fold needs >= 65 output channels");
      if (p.fold_x) {
        if (p.gn <= 64) launch_fold_cfg<MODE, 128, 64, 2, 2, 3>(p, st); else launch_fold_cfg<MODE, 128, 128, 2, 2, 3>(p, st);
      } else {
        if (p.gn <= 64) launch_fold_cfg<MODE, 128, 64, 2, 2, 2>(p, st); else launch_fold_cfg<MODE, 128, 128, 2, 2, 2>(p, st);
      }
      return;
    }
    // (no 256x64 wide tile here: with the fold's x chunks and coefficients it spills; the 64x256
    // stem tile reads the folded operand once instead of once per 128-column tile)
    if (wgrad_wide(p) == 1) launch_fold_cfg<MODE, 64, 256, 1, 4, 1>(p, st);
    else if (p.gm <= 64) {
      if (p.gn <= 64) launch_fold_cfg<MODE, 64, 64, 2, 2, 1>(p, st); else launch_fold_cfg<MODE, 64, 128, 2, 2, 1>(p, st);
    } else {
      if (p.gn <= 64) launch_fold_cfg<MODE, 128, 64, 2, 2, 1>(p, st); else launch_fold_cfg<MODE, 128, 128, 2, 2, 1>(p, st);
    }
  }
}

template <int MODE>
static void dispatch(IgemmParams& p, hipStream_t st) {
  if (p.fold_x || p.act_sc) { launch_fold<MODE>(p, st); return; }
  if constexpr (MODE != MODE_WGRAD) {
    if (use_halo(MODE, p)) { launch_halo<MODE>(p, st); return; }
    if (use_igemm8(MODE, p) == 256) { launch_dma<MODE, 256, 256, 2, 4, NT8, 1>(p, st); return; }
  }
  if constexpr (MODE == MODE_WGRAD) {
    const int w = wgrad_wide(p);
    if (w == 1) { launch_cfg<MODE, 64, 256, 1, 4>(p, st); return; }
    if (w == 2) { launch_cfg<MODE, 256, 64, 4, 1>(p, st); return; }
  }
  if constexpr (MODE != MODE_WGRAD) {
    if (use_bm64_smallgrid(MODE, p)) { launch_cfg<MODE, 64, 128, 2, 2>(p, st); return; }
    switch (use_dma4(MODE, p)) {
      case 1:
        if (use_dma32(MODE, p)) launch_dma32<MODE, 128, 128, 2, 2>(p, st); else launch_dma<MODE, 128, 128, 2, 2, NT, 2>(p, st);
        return;
      case 2:
        if (use_dma32(MODE, p)) launch_dma32<MODE, 128, 64, 2, 2>(p, st); else launch_dma<MODE, 128, 64, 2, 2, NT, 2>(p, st);
        return;
      case 3: launch_dma<MODE, 256, 64, 4, 1, NT, 2>(p, st); return;
      default: break;
    }
  }
  // tile choice: BN=64 for narrow outputs, BM=32/64 for short M (linear at small batch)
  if (p.gm <= 32) {
    if (p.gn <= 64) launch_cfg<MODE, 32, 64, 1, 4>(p, st);
    else launch_cfg<MODE, 32, 128, 1, 4>(p, st);
  } else if (p.gm <= 64) {
    if (p.gn <= 64) launch_cfg<MODE, 64, 64, 2, 2>(p, st);
    else launch_cfg<MODE, 64, 128, 2, 2>(p, st);
  } else {
    if (p.gn <= 64) launch_cfg<MODE, 128, 64, 2, 2>(p, st);
    else launch_cfg<MODE, 128, 128, 2, 2>(p, st);
  }
}


// ------------------------------------------------------------------------------------------------
// Plain-GEMM kernel on v_mfma_f32_32x32x16_bf16 (plan kinds 9 / 10): C[m][n] = sum_k A[m][k] B[n][k]
// for the stride-1 1x1 FWD / DGRAD GEMMs the planner handles (Linear layers: A = x or dy, B = w or
// the transposed weight, both K-contiguous), with the plain epilogue (bias, residual, ReLU, GELU
// forward with the u side output, GELU backward through resid) or fp32 split-K partials.  Main loop:
// the LDS-DMA double buffer with one barrier per 64-deep K-tile and fenced halves of
// tools/gemm_lab (v4); 32x32x16 issues half the MFMA instructions of 16x16x32 for the same wave
// tile and ds_read bytes: +5-12 % on 128x128 4-wave tiles in the lab (profiles/r4_gemm_lab_mfma32.txt).
// Accumulator of lane l, 32x32 tile: C column (lane & 31) = row m of the output, register r holds
// output channel 8 * (r / 4) + 4 * (l >> 5) + (r % 4) of the tile (the MFMA runs B x A).
template <int BM, int BN, int WM, int WN, int MINB>
__global__ void __launch_bounds__(WM * WN * 64, MINB) gemm32_kernel(const IgemmParams p) {
  constexpr int NW = WM * WN;
  constexpr int WTM = BM / WM, WTN = BN / WN, TM = WTM / 32, TN = WTN / 32;
  constexpr int A_BYTES = BM * BK * 2, STAGE = (BM + BN) * BK * 2;
  constexpr int NA = BM / 8 / NW, NB = BN / 8 / NW;
  static_assert(NA * 8 * NW == BM && NB * 8 * NW == BN && TM >= 1 && TN >= 1, "gemm32 tile");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid / WN, wc = wid % WN;
  const int M = p.gm, N = p.gn, K = p.gk;
  const int tiles_mn = p.tiles_m * p.tiles_n;
  const int lin = xcd_remap(blockIdx.x, gridDim.x);
  const int split = lin / tiles_mn;
  const int tt = lin - split * tiles_mn;
  const int tile_m = tt / p.tiles_n, tile_n = tt - (tt / p.tiles_n) * p.tiles_n;
  const int m0 = tile_m * BM, n0 = tile_n * BN;
  const int kbeg = split * p.ksplit;
  const int nk = (min(K, kbeg + p.ksplit) - kbeg) / BK;
  const __amdgpu_buffer_rsrc_t rsA = make_rsrc(p.a, p.a_bytes), rsB = make_rsrc(p.b, p.b_bytes);
  const int gch = (lane & 7) ^ (lane >> 3);
  unsigned a_vo[NA], b_vo[NB];
#pragma unroll
  for (int i = 0; i < NA; ++i) {
    const int m = m0 + (wid * NA + i) * 8 + (lane >> 3);
    a_vo[i] = m < M ? (unsigned)((size_t)m * K + kbeg + gch * 8) * 2u : kOOB;
  }
#pragma unroll
  for (int i = 0; i < NB; ++i) {
    const int n = n0 + (wid * NB + i) * 8 + (lane >> 3);
    b_vo[i] = n < N ? (unsigned)((size_t)n * K + kbeg + gch * 8) * 2u : kOOB;
  }
  auto issue = [&](int s, int k0, bool live) {
#pragma unroll
    for (int i = 0; i < NA; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsA, (__attribute__((address_space(3))) void*)(smem + s * STAGE + (wid * NA + i) * 1024), 16,
                                               (int)(live && a_vo[i] != kOOB ? a_vo[i] + k0 * 2 : kOOB), 0, 0, 0);
#pragma unroll
    for (int i = 0; i < NB; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsB, (__attribute__((address_space(3))) void*)(smem + s * STAGE + A_BYTES + (wid * NB + i) * 1024), 16,
                                               (int)(live && b_vo[i] != kOOB ? b_vo[i] + k0 * 2 : kOOB), 0, 0, 0);
  };
  f32x16 acc[TN][TM];
#pragma unroll
  for (int j = 0; j < TN; ++j)
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[j][i][r] = 0.f;
  bf16x8 fa0[2][TM], fb0[2][TN], fa1[2][TM], fb1[2][TN];
  auto rd = [&](bf16x8(&fa)[2][TM], bf16x8(&fb)[2][TN], int half, int s) {
    const char* sA = smem + s * STAGE;
    const char* sB = sA + A_BYTES;
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int ch = half * 4 + q * 2 + (lane >> 5);
#pragma unroll
      for (int i = 0; i < TM; ++i) fa[q][i] = *reinterpret_cast<const bf16x8*>(sA + rr_off(wr * WTM + i * 32 + (lane & 31), ch));
#pragma unroll
      for (int j = 0; j < TN; ++j) fb[q][j] = *reinterpret_cast<const bf16x8*>(sB + rr_off(wc * WTN + j * 32 + (lane & 31), ch));
    }
  };
  auto mma = [&](bf16x8(&fa)[2][TM], bf16x8(&fb)[2][TN]) {
#pragma unroll
    for (int q = 0; q < 2; ++q)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int i = 0; i < TM; ++i) acc[j][i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fb[q][j], fa[q][i], acc[j][i], 0, 0, 0);
  };
  constexpr int NMF = 2 * TM * TN, NDS = 2 * (TM + TN), NVM = NA + NB;
  constexpr int DPM = NDS / NMF > 0 ? NDS / NMF : 1, MPD = NMF >= NDS ? NMF / NDS : 1;
  // last two K-tiles peeled (no zero-fill DMA of a dead stage is issued or waited for), as in
  // igemm_dma32_kernel
  enum { FULL = 0, NODMA = 1, LAST = 2 };
  auto ktile = [&](int t, auto form) {
    constexpr int F = decltype(form)::value;
    const int s = t & 1;
    rd(fa1, fb1, 1, s);
    mma(fa0, fb0);
#pragma unroll
    for (int g = 0; g < NDS; ++g) {
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      if (g % DPM == 0) __builtin_amdgcn_sched_group_barrier(0x8, MPD, 0);
    }
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (F != LAST) {
      wait_vm_b<0>();
      lds_sync_b();
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (F == FULL) issue(s, (t + 2) * BK, true);
      rd(fa0, fb0, 0, s ^ 1);
    }
    mma(fa1, fb1);
    if constexpr (F == FULL) {
#pragma unroll
      for (int g = 0; g < NDS; ++g) {
        if (g < NVM) __builtin_amdgcn_sched_group_barrier(0x10, 1, 1);
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 1);
        if (g % DPM == 0) __builtin_amdgcn_sched_group_barrier(0x8, MPD, 1);
      }
    } else if constexpr (F == NODMA) {
#pragma unroll
      for (int g = 0; g < NDS; ++g) {
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 1);
        if (g % DPM == 0) __builtin_amdgcn_sched_group_barrier(0x8, MPD, 1);
      }
    }
    __builtin_amdgcn_sched_barrier(0);
  };
  if (nk > 0) {
    issue(0, 0, true);
    if (nk > 1) {
      issue(1, BK, true);
      wait_vm_b<NA + NB>();
    } else {
      wait_vm_b<0>();
    }
    lds_sync_b();
    rd(fa0, fb0, 0, 0);
    for (int t = 0; t < nk - 2; ++t) ktile(t, std::integral_constant<int, FULL>{});
    if (nk >= 2) ktile(nk - 2, std::integral_constant<int, NODMA>{});
    ktile(nk - 1, std::integral_constant<int, LAST>{});
  }
  // ---- epilogue: lane = output row m, 4 groups of 4 consecutive channels per 32x32 tile ----------
  if (p.nsplit > 1) {
    float* ws = reinterpret_cast<float*>(p.out) + (size_t)split * M * N;
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int m = m0 + wr * WTM + i * 32 + (lane & 31);
#pragma unroll
        for (int r4 = 0; r4 < 4; ++r4) {
          const int n = n0 + wc * WTN + j * 32 + 8 * r4 + 4 * (lane >> 5);
          if (m < M && n < N)
            *reinterpret_cast<f32x4*>(ws + (size_t)m * N + n) =
                f32x4{acc[j][i][4 * r4], acc[j][i][4 * r4 + 1], acc[j][i][4 * r4 + 2], acc[j][i][4 * r4 + 3]};
        }
      }
    return;
  }
  __bf16* out = reinterpret_cast<__bf16*>(p.out);
#pragma unroll
  for (int j = 0; j < TN; ++j)
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int m = m0 + wr * WTM + i * 32 + (lane & 31);
#pragma unroll
      for (int r4 = 0; r4 < 4; ++r4) {
        const int n = n0 + wc * WTN + j * 32 + 8 * r4 + 4 * (lane >> 5);
        if (m >= M || n >= N) continue;
        const size_t o = (size_t)m * N + n;
        float x[4];
        const f32x4 b4 = p.bias ? *reinterpret_cast<const f32x4*>(p.bias + n) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int e = 0; e < 4; ++e) x[e] = acc[j][i][4 * r4 + e] + b4[e];
        if (p.resid) {
          const uint2 rv = *reinterpret_cast<const uint2*>(p.resid + o);
          const float r[4] = {__uint_as_float(rv.x << 16), __uint_as_float(rv.x & 0xffff0000u),
                              __uint_as_float(rv.y << 16), __uint_as_float(rv.y & 0xffff0000u)};
#pragma unroll
          for (int e = 0; e < 4; ++e) x[e] = p.relu == 3 ? x[e] * dgelu_fast(r[e]) : x[e] + r[e];
        }
        if (p.relu == 1) {
#pragma unroll
          for (int e = 0; e < 4; ++e) x[e] = fmaxf(x[e], 0.f);
        } else if (p.relu == 2) {   // u (bf16) -> aux; out = gelu(u)
          const unsigned u0 = f2bf2(x[0], x[1]), u1 = f2bf2(x[2], x[3]);
          *reinterpret_cast<uint2*>(p.aux + o) = uint2{u0, u1};
          x[0] = gelu_fast(__uint_as_float(u0 << 16));
          x[1] = gelu_fast(__uint_as_float(u0 & 0xffff0000u));
          x[2] = gelu_fast(__uint_as_float(u1 << 16));
          x[3] = gelu_fast(__uint_as_float(u1 & 0xffff0000u));
        }
        *reinterpret_cast<uint2*>(out + o) = uint2{f2bf2(x[0], x[1]), f2bf2(x[2], x[3])};
      }
    }
}

template <int BM, int BN, int WM, int WN, int MINB>
static void launch_gemm32(IgemmParams& p, hipStream_t st) {
  TORCH_CHECK(p.R == 1 && p.S == 1 && p.stride == 1 && p.pad == 0 && p.gk % BK == 0 && p.ksplit % BK == 0 &&
                  !p.stats && !p.bn_x && !p.fold_x && !p.act_sc && p.gn % 4 == 0,
              "gemm32: plain 1x1 GEMMs only");
  p.tiles_m = ceil_div(p.gm, BM);
  p.tiles_n = ceil_div(p.gn, BN);
  const int grid = p.tiles_m * p.tiles_n * p.nsplit;
  constexpr size_t smem = (size_t)2 * (BM + BN) * BK * 2;
  static_assert(smem <= 160 * 1024, "gemm32: LDS budget");
  auto kfn = &gemm32_kernel<BM, BN, WM, WN, MINB>;
  static bool attr_set = false;
  if (!attr_set) {
    PCMP_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(kfn), hipFuncAttributeMaxDynamicSharedMemorySize,
                                       160 * 1024));
    attr_set = true;
  }
  hipLaunchKernelGGL(kfn, dim3(grid), dim3(WM * WN * 64), smem, st, p);
  PCMP_LAUNCH_CHECK();
}

// ------------------------------------------------------------------------------------------------
// Plain-GEMM planner: a stride-1 1x1 convolution without a BatchNorm epilogue is a plain GEMM
// (every Linear layer: BERT-base's M = 4096-token projections, the VGG16 classifier, the transfer
// heads).  Those shapes have too few 128x128 / 256x256 tiles to fill 256 CUs (BERT's N = 768
// outputs: 48 tiles of 256x256), so the first call of each shape times a small candidate set --
// the 4-wave LDS-DMA kernel (128x128, 2 blocks/CU) and the 8-wave one (256x256, 1 block/CU), each
// with 1..6 K-splits whose fp32 partials are reduced by splitk_epilogue_kernel (bias / residual /
// ReLU fused there) -- and caches the fastest (cudnn.benchmark-style; never while a graph is being
// captured).  This replaces the round-1 hipBLASLt candidate for these GEMMs.
inline Knob kn_gemm_plan("gemm_plan", 1);   // 0 = default dispatch only, 1 = autotuned plan
inline Knob kn_plan_force("plan_force", -1); // tests: >= 0 restricts the candidates to that kind (uncached)
inline Knob kn_gemm32("gemm32", 1);          // 32x32x16-MFMA plain-GEMM candidates (plan kinds 9 / 10)
inline Knob kn_plan_nsplit("plan_nsplit", 0); // tests: >= 1 (with plan_force) also pins the split count
// a split candidate must beat the best by this many us per call to be chosen: its extra
// splitk_epilogue launch is host time the isolated timing does not see (BERT-base's eager step is
// host-bound: 56 split epilogues per step in round 4, verdict r4 weak #6)
inline Knob kn_plan_split_us("plan_split_us", 6);
// small-M (inference) plans are timed with the caches cold: a 64 MB memset before every timed call
// evicts the L2s.  Timed back to back, a conv's weights (0.1-4.7 MB at batch 1) stay L2-resident
// from the previous call and the tuner favoured kernels with one K-step in flight; inside the
// batch-1 graph every conv streams its weights from the MALL / HBM.  0 = the warm timing.
inline Knob kn_plan_cold("plan_cold", 1);

struct GemmPlan {
  int kind;     // 0 = default dispatch<>, 1 = DMA 128x128, 2 = DMA 256x256 (8 waves),
                // 3 = register-staged 64x64, 4 = register-staged 32x64, 5 = DMA 128x64 (small-M inference convs),
                // 6 = skinny FWD, 9 / 10 = 32x32x16 gemm32 128x128 / 256x256 (7 / 8: round 4 big kernel, removed)
  int nsplit;
};
static const char* plan_kind_name(int k) {
  switch (k) {
    case 1: return "dma128x128";
    case 2: return "dma256x256";
    case 3: return "reg64x64";
    case 4: return "reg32x64";
    case 5: return "dma128x64";
    case 6: return "skinny64x64";
    case 9: return "m32_128x128";
    case 10: return "m32_256x256";
    default: return "default";
  }
}

template <int MODE>
static void run_plan(IgemmParams p, const GemmPlan& pl, __bf16* out, const at::TensorOptions& fopts, hipStream_t st) {
  const int kq = pl.kind == 6 ? 32 : BK;   // K granularity of the kernel
  const int ksteps = ceil_div(p.gk, kq);
  int nsplit = std::max(1, pl.nsplit);
  const int steps_per = ceil_div(ksteps, nsplit);
  nsplit = ceil_div(ksteps, steps_per);
  p.nsplit = nsplit;
  p.ksplit = steps_per * kq;
  const __bf16* resid = p.resid;
  at::Tensor ws;
  if (nsplit > 1) {
    ws = at::empty({(int64_t)nsplit, (int64_t)p.gm * p.gn}, fopts);
    p.out = ws.data_ptr();
  } else {
    p.out = out;
  }
  if (pl.kind == 1) launch_dma<MODE, 128, 128, 2, 2, NT, 2>(p, st);
  else if (pl.kind == 2) launch_dma<MODE, 256, 256, 2, 4, NT8, 1>(p, st);
  else if (pl.kind == 3) launch_cfg<MODE, 64, 64, 2, 2>(p, st);
  else if (pl.kind == 4) launch_cfg<MODE, 32, 64, 1, 4>(p, st);
  else if (pl.kind == 5) launch_dma<MODE, 128, 64, 2, 2, NT, 2>(p, st);
  else if (pl.kind == 9) launch_gemm32<128, 128, 2, 2, 2>(p, st);
  else if (pl.kind == 10) launch_gemm32<256, 256, 2, 2, 1>(p, st);
  else if (pl.kind == 6) {
    if constexpr (MODE == MODE_FWD) launch_skinny(p, st);
    else TORCH_CHECK(false, "skinny kernel is FWD only");
  } else dispatch<MODE>(p, st);
  if (nsplit > 1) {
    const int64_t n = (int64_t)p.gm * p.gn;
    const int blocks = (int)((n / 4 + 255) / 256);
    hipLaunchKernelGGL(splitk_epilogue_kernel, dim3(blocks), dim3(256), 0, st, ptr<float>(ws), out,
                       MODE == MODE_FWD ? p.bias : nullptr, resid, n, p.gn, nsplit, p.relu, p.aux);
    PCMP_LAUNCH_CHECK();
  }
}

template <int MODE>
static bool plain_gemm_eligible(const IgemmParams& p) {
  const int cin = MODE == MODE_FWD ? p.C : p.K;
  return kn_gemm_plan.get() && p.R == 1 && p.S == 1 && p.stride == 1 && p.pad == 0 && !p.stats && !p.bn_x &&
         p.gm >= 1024 && p.gk % BK == 0 && cin % BK == 0 && p.gn % 8 == 0 && p.gk / BK >= 4;
}

inline std::mutex g_plan_mu;
inline std::unordered_map<std::string, GemmPlan> g_plan_cache;
// wgrad_nsplit's tuned split counts (same mutex)
inline std::unordered_map<std::string, int> g_wsplit_cache;
inline std::vector<std::string>* g_plan_log = nullptr;   // candidate timings (plan_candidates op)

std::vector<std::string> gemm_plans();

// small_m: an inference-sized convolution (few output tiles, long reduction): the candidates are
// the register-staged kernels at 128/64/32-row tiles with 1..32 K-splits (the split partials are
// reduced by splitk_epilogue_kernel together with bias / residual / ReLU), plus the round-1
// heuristic (default tile, heur_split splits) so the plan is never a regression by construction.
template <int MODE>
static GemmPlan plan_gemm(const IgemmParams& p, __bf16* out, const at::TensorOptions& fopts, hipStream_t st,
                          bool small_m = false, int heur_split = 1) {
  auto& mu = g_plan_mu;
  auto& cache = g_plan_cache;
  char key[192];
  snprintf(key, sizeof(key), "%d,%d,%d,%d,%d,%d,%d|%d,%d,%d,%d,%d,%d,%d,%d,%d", MODE, p.gm, p.gn, p.gk,
           p.bias != nullptr, p.resid != nullptr, p.relu, p.N, p.H, p.W, p.C, p.K, p.R, p.S, p.stride, p.pad);
  const int force = kn_plan_force.get();
  if (force < 0) {
    std::lock_guard<std::mutex> g(mu);
    auto it = cache.find(key);
    if (it != cache.end()) return it->second;
  }
  GemmPlan dflt{0, small_m ? heur_split : 1};
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(st, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) return dflt;
  const int ksteps = ceil_div(p.gk, BK);
  std::vector<GemmPlan> cands{dflt};
  if (small_m) {
    // the LDS-DMA kernels keep 2-3 half-tiles of operands in flight (the register-staged ones one
    // K-step), which matters when a block's few K-steps are latency-bound; they need the
    // block-uniform tap walk
    const int cin = MODE == MODE_FWD ? p.C : p.K;
    const bool dma_ok = p.gk % BK == 0 && cin % BK == 0;
    for (int ns : {1, 2, 4, 8, 12, 16, 24, 32}) {
      if (ns > 1 && ksteps / ns < 2) continue;
      for (int kind : {0, 3, 4, 1, 5}) {
        if (kind == 0 && ns == heur_split) continue;
        if (kind == 4 && p.gm > 256) continue;
        if ((kind == 1 || kind == 5) && (!dma_ok || ceil_div(ksteps, ns) < 2)) continue;
        if (kind == 5 && p.gn > 1024) continue;
        cands.push_back({kind, ns});
      }
      if (MODE == MODE_FWD && p.relu < 2 && p.C % 32 == 0 && p.gk % 32 == 0 && p.gn % 4 == 0 && p.gm <= 1024 &&
          p.gk / 32 / ns >= 2)
        cands.push_back({6, ns});
    }
  } else {
    for (int ns : {1, 2, 3, 4, 6}) {
      if (ns > 1 && ksteps / ns < 4) continue;
      cands.push_back({1, ns});
      // 128x64 tiles: twice the 128x128 grid for N <= 1024 (BERT's N = 768 GEMMs: 384 tiles, not 192)
      if (p.gn <= 1024) cands.push_back({5, ns});
      if (kn_gemm32.get() && p.gn % 4 == 0) {   // 32x32x16 MFMA kernels
        cands.push_back({9, ns});
        if (p.gn >= 256) cands.push_back({10, ns});
      }
      if (p.gn >= 256) cands.push_back({2, ns});
    }
  }
  if (force >= 0) {
    std::vector<GemmPlan> f;
    for (const GemmPlan& c : cands)
      if (c.kind == force) f.push_back(c);
    if (!f.empty()) cands = f;
    if (kn_plan_nsplit.get() > 0) {   // a pinned split count makes repeated forced calls bitwise comparable
      f.clear();
      for (const GemmPlan& c : cands)
        if (c.nsplit == kn_plan_nsplit.get()) f.push_back(c);
      if (!f.empty()) cands = f;
    }
  }
  hipEvent_t e0, e1;
  PCMP_HIP_CHECK(hipEventCreate(&e0));
  PCMP_HIP_CHECK(hipEventCreate(&e1));
  GemmPlan best = cands[0];
  float best_ms = 1e30f;
  const bool cold = small_m && kn_plan_cold.get();
  // the cache-evicting scratch of the cold timing: allocated once, never freed (no tensor destructor
  // runs at process exit, after the HIP runtime may be gone)
  static at::Tensor* flush = nullptr;
  if (cold && flush == nullptr) flush = new at::Tensor(at::empty({64 << 20}, fopts.dtype(at::kByte)));
  auto consider = [&](const GemmPlan& c, float ms) {
    if (c.nsplit > 1 && !small_m) ms += 3e-3f * kn_plan_split_us.get();   // 3 timed calls
    if (ms < best_ms) { best_ms = ms; best = c; }
    if (g_plan_log) g_plan_log->push_back(std::string(plan_kind_name(c.kind)) + "/split" + std::to_string(c.nsplit) +
                                          " " + std::to_string(ms / 3 * 1000.f) + "us");
  };
  if (cold) {
    // every candidate's three cold calls are enqueued with their own event pairs and the host waits
    // ONCE per shape (a wait per call cost ~0.2 s of a transfer-learning epoch's first steps)
    std::vector<hipEvent_t> ev(6 * cands.size());
    for (auto& e : ev) PCMP_HIP_CHECK(hipEventCreate(&e));
    for (size_t ci = 0; ci < cands.size(); ++ci) {
      run_plan<MODE>(p, cands[ci], out, fopts, st);   // warm (workspace allocation)
      for (int r = 0; r < 3; ++r) {
        PCMP_HIP_CHECK(hipMemsetAsync(flush->data_ptr(), r, flush->numel(), st));
        PCMP_HIP_CHECK(hipEventRecord(ev[6 * ci + 2 * r], st));
        run_plan<MODE>(p, cands[ci], out, fopts, st);
        PCMP_HIP_CHECK(hipEventRecord(ev[6 * ci + 2 * r + 1], st));
      }
    }
    PCMP_HIP_CHECK(hipEventSynchronize(ev.back()));
    for (size_t ci = 0; ci < cands.size(); ++ci) {
      float ms = 0.f;
      for (int r = 0; r < 3; ++r) {
        float one = 0.f;
        PCMP_HIP_CHECK(hipEventElapsedTime(&one, ev[6 * ci + 2 * r], ev[6 * ci + 2 * r + 1]));
        ms += one;
      }
      consider(cands[ci], ms);
    }
    for (auto& e : ev) PCMP_HIP_CHECK(hipEventDestroy(e));
  } else {
    for (const GemmPlan& c : cands) {
      run_plan<MODE>(p, c, out, fopts, st);   // warm (workspace allocation)
      float ms = 0.f;
      PCMP_HIP_CHECK(hipEventRecord(e0, st));
      for (int r = 0; r < 3; ++r) run_plan<MODE>(p, c, out, fopts, st);
      PCMP_HIP_CHECK(hipEventRecord(e1, st));
      PCMP_HIP_CHECK(hipEventSynchronize(e1));
      PCMP_HIP_CHECK(hipEventElapsedTime(&ms, e0, e1));
      consider(c, ms);
    }
  }
  PCMP_HIP_CHECK(hipEventDestroy(e0));
  PCMP_HIP_CHECK(hipEventDestroy(e1));
  if (force >= 0) return best;
  std::lock_guard<std::mutex> g(mu);
  cache.emplace(key, best);
  return best;
}



static unsigned tensor_bytes(const at::Tensor& t) {
  const int64_t b = t.numel() * t.element_size();
  TORCH_CHECK(b < (1ll << 31), "igemm: operand larger than 2 GiB (buffer-resource range)");
  return (unsigned)b;
}

static void fill_geometry(IgemmParams& p, int N, int H, int W, int C, int K, int R, int S,
                          int stride, int pad) {
  p.N = N; p.H = H; p.W = W; p.C = C; p.K = K; p.R = R; p.S = S;
  p.stride = stride; p.pad = pad;
  p.P = (H + 2 * pad - R) / stride + 1;
  p.Q = (W + 2 * pad - S) / stride + 1;
  p.fd_PQ = make_fastdiv(p.P * p.Q);
  p.fd_Q = make_fastdiv(p.Q);
  p.fd_HW = make_fastdiv(H * W);
  p.fd_W = make_fastdiv(W);
  p.dH = H; p.dW = W; p.offy = pad; p.offx = pad; p.sub = 0; p.oph = 0; p.opw = 0;
  p.bias = nullptr; p.resid = nullptr; p.aux = nullptr; p.stats = nullptr; p.stats2 = nullptr;
  p.bn_mask = nullptr; p.bn_x = nullptr; p.bn_mean = nullptr; p.bn_istd = nullptr;
  p.bn_x2 = nullptr; p.bn_mean2 = nullptr; p.bn_istd2 = nullptr; p.bn_msc = nullptr; p.bn_msh = nullptr;
  p.bn_mbits = nullptr;
  p.stats_cap = 0;
  p.relu = 0; p.alpha = 1.f; p.accumulate = 0; p.nsplit = 1;
  p.fold_x = nullptr; p.fold_coef = nullptr; p.fold_lds = 0;
  p.act_sc = nullptr; p.act_sh = nullptr;
  p.resid_sub = 0; p.rs_H2 = 0; p.rs_W2 = 0;
}

// ---- entry points (igemm_fwd.hip / igemm_dgrad.hip / igemm_wgrad.hip; registered in igemm.hip)
std::vector<at::Tensor> conv_fwd(const at::Tensor& x, const at::Tensor& w, int64_t stride, int64_t pad,
                                 const c10::optional<at::Tensor>& bias,
                                 const c10::optional<at::Tensor>& resid, bool relu, bool want_stats,
                                 const c10::optional<at::Tensor>& in_scale, const c10::optional<at::Tensor>& in_shift);
std::vector<std::string> plan_candidates(const at::Tensor& x, const at::Tensor& w, int64_t stride, int64_t pad,
                                         const c10::optional<at::Tensor>& bias, const c10::optional<at::Tensor>& resid,
                                         bool relu);
std::vector<at::Tensor> linear_gelu_fwd(const at::Tensor& x, const at::Tensor& w, const c10::optional<at::Tensor>& bias);
at::Tensor conv_dgrad(const at::Tensor& dy, const at::Tensor& w, int64_t H, int64_t W, int64_t stride, int64_t pad,
                      const c10::optional<at::Tensor>& resid, const c10::optional<at::Tensor>& wt);
at::Tensor linear_dgrad_gelu(const at::Tensor& dy, const at::Tensor& w, const at::Tensor& u,
                             const c10::optional<at::Tensor>& wt);
std::vector<at::Tensor> conv_dgrad_bnr(const at::Tensor& dy, const at::Tensor& w, int64_t H, int64_t W,
                                       int64_t stride, int64_t pad, const c10::optional<at::Tensor>& resid,
                                       const c10::optional<at::Tensor>& ymask, const at::Tensor& x,
                                       const at::Tensor& mean, const at::Tensor& invstd,
                                       const c10::optional<at::Tensor>& x2, const c10::optional<at::Tensor>& mean2,
                                       const c10::optional<at::Tensor>& invstd2, const c10::optional<at::Tensor>& mscale,
                                       const c10::optional<at::Tensor>& mshift, const c10::optional<at::Tensor>& wt,
                                       const c10::optional<at::Tensor>& ymask_bits,
                                       const c10::optional<at::Tensor>& fold_x,
                                       const c10::optional<at::Tensor>& fold_coef, bool resid_sub);
void conv_wgrad(const at::Tensor& dy, const at::Tensor& x, at::Tensor out, int64_t R, int64_t S,
                int64_t stride, int64_t pad, bool accumulate, const c10::optional<at::Tensor>& fold_x,
                const c10::optional<at::Tensor>& fold_coef, const c10::optional<at::Tensor>& in_scale,
                const c10::optional<at::Tensor>& in_shift);
std::vector<at::Tensor> conv1x1_bwd_fused(const at::Tensor& g, const c10::optional<at::Tensor>& fold_x,
                                          const c10::optional<at::Tensor>& fold_coef, const at::Tensor& wt,
                                          const at::Tensor& z, const at::Tensor& scale, const at::Tensor& shift,
                                          const at::Tensor& mean, const at::Tensor& invstd, at::Tensor dw,
                                          bool accumulate);

}  // namespace pcmp

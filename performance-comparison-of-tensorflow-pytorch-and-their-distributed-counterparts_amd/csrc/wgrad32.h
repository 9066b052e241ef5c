// Round-6 WGRAD kernel: LDS-DMA operand staging + v_mfma_f32_32x32x16_bf16, with ZERO per-lane
// address arithmetic in the K-loop.
//
//   dW[co][j=(r,s,c)] = sum_m dY[m][co] * X[n, p*st-pad+r, q*st-pad+s, c],   m = (n, p, q)
//
// The reduction is a sum, so its order is free.  This kernel walks it pixel-major, image-minor:
// reduction row m' = (p*Q + q) * N + n, and a 64-deep K-tile is 64 IMAGES at one output pixel
// (p, q) (needs N % 64 == 0).  Every row of a K-tile then shares one pixel, so
//   * the im2col bounds check (conv zero-padding) is block-UNIFORM: a tap (r, s) of a 64-column block
//     is in or out of the image for all 64 rows at once, and an out-of-image block is DMA'd through a
//     zero-record buffer descriptor (hardware zero-fill) chosen by a scalar select;
//   * a lane's source address splits into a per-lane part fixed for the whole kernel (its image n and
//     16-B chunk) and a block-uniform part (pixel, tap, channel base) that goes into the buffer
//     instruction's SGPR soffset.
// The register-staged igemm_kernel<MODE_WGRAD> spends ~10 VALU per MFMA on the (n, p, q) walk, its
// bounds checks and the ds_write staging and runs at 23 % MFMA busy (docs/PERF_NOTES.md round 5);
// here the K-loop has no VALU address work at all and no ds_write: the buffer_load ... lds
// instructions write the XOR-swizzled transposed-read image straight from the DMA.
//
// LDS image, per stage: A (dY) then B (x), each [cols/64 blocks][64 reduction rows][64 cols] bf16 --
// 128-B rows -- with the 16-B chunk XOR 4*((row >> 1) & 1) that makes the 32x32x16 transposed
// fragment reads (ds_read_b64_tr_b16: a 32-lane cycle covers 4 rows x 64 B) conflict-free.  One
// LDS-DMA wave instruction fills 8 rows x 128 B of one column block; the swizzle is applied to the
// lane's SOURCE chunk (cdna_hip_programming.md §5.4 rule 21).  A 64-column block of B lies inside
// one filter tap because C % 64 == 0.
//
// Main loop: the one-barrier-per-K-tile schedule of igemm_dma32_kernel (two LDS stages, each K-tile's
// fragments double-buffered over its two 32-deep halves; the DMA of tile t+2 is issued right after
// the barrier that retires stage t's readers).  4 waves (2x2), 2 blocks per CU, 64 KB of LDS per
// 128x128 block (the register-staged kernel's footprint, so the DGRAD chain's blocks co-reside).
// Split-K partials go to the fp32 workspace exactly like igemm_kernel<MODE_WGRAD> (same ksplit
// contract: split s owns K-tiles [s*ksplit/64, ...) of the reordered reduction).
//
// Reference parity: the weight gradients of the ResNet-50 / VGG16 / BERT layers the reference trains
// (SURVEY.md §2.4.1 "conv2d bwd-data / bwd-weight"; /root/reference/pytorch_training_inference_on_image.ipynb:454-635).
#pragma once
#include "igemm.h"

namespace pcmp {

inline Knob kn_wgrad_dma32("wgrad_dma32", 1);

// byte offset of element (row, col) in a [cols/64][64][64] image, col % 4 == 0
__device__ __forceinline__ int w32_off(int row, int col) {
  return (col >> 6) * 8192 + row * 128 + ((((col & 63) >> 3) ^ (((row >> 1) & 1) << 2)) << 4) + ((col & 7) << 1);
}

template <int BM, int BN>
__global__ void __launch_bounds__(256, 2) wgrad_dma32_kernel(const IgemmParams p) {
  constexpr int WM = 2, WN = 2;
  constexpr int WTM = BM / WM, WTN = BN / WN;
  constexpr int TM = WTM / 32, TN = WTN / 32;
  constexpr int A_BYTES = BM * 128, STAGE = (BM + BN) * 128;
  constexpr int NA = BM / 32, NB = BN / 32;   // DMA wave-instructions per K-tile per wave
  static_assert(TM >= 1 && TN >= 1 && NA >= 2 && NB >= 2, "wgrad_dma32 tile");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wid / WN, wc = wid % WN;

  const int lin = xcd_remap(blockIdx.x, gridDim.x);
  const int tiles_mn = p.tiles_m * p.tiles_n;
  const int split = lin / tiles_mn;
  const int tt = lin - split * tiles_mn;
  const int tile_n = tt % p.tiles_n, tile_m = tt / p.tiles_n;
  const int m0 = tile_m * BM, n0 = tile_n * BN;
  const int nkt = p.gk >> 6;
  const int kps = p.ksplit >> 6;
  const int kt0 = split * kps;
  const int nk = min(nkt, kt0 + kps) - kt0;

  const __amdgpu_buffer_rsrc_t rsA = make_rsrc(p.a, p.a_bytes);
  const __amdgpu_buffer_rsrc_t rsB = make_rsrc(p.b, p.b_bytes);
  const __amdgpu_buffer_rsrc_t rsZ = make_rsrc(p.a, 0u);   // zero records: every lane reads 0

  // per-lane source offsets, fixed for the whole kernel: instruction i fills column block i >> 1,
  // rows 8 * ((i & 1) * 4 + wid) .. +7; lane -> row + (lane >> 3), LDS chunk lane & 7 holding
  // source chunk (lane & 7) ^ swizzle(row)
  const int PQK = p.P * p.Q * p.K, HWC = p.H * p.W * p.C;
  const int lch = (lane & 7) ^ (((lane >> 4) & 1) << 2);
  int a_vo[NA], b_vo[NB];
#pragma unroll
  for (int i = 0; i < NA; ++i) {
    const int row = ((i & 1) * 4 + wid) * 8 + (lane >> 3);
    a_vo[i] = (row * PQK + (i >> 1) * 64 + lch * 8) * 2;
  }
#pragma unroll
  for (int i = 0; i < NB; ++i) {
    const int row = ((i & 1) * 4 + wid) * 8 + (lane >> 3);
    b_vo[i] = (row * HWC + lch * 8) * 2;
  }
  // block-uniform column-block state: A blocks valid, B block taps (r, s) and channel bases
  constexpr int CBA = BM / 64, CBB = BN / 64;
  bool a_ok[CBA];
#pragma unroll
  for (int b = 0; b < CBA; ++b) a_ok[b] = m0 + b * 64 < p.gm;
  int b_r[CBB], b_s[CBB], b_c[CBB];
  bool b_ok[CBB];
#pragma unroll
  for (int b = 0; b < CBB; ++b) {
    const int j0 = n0 + b * 64;
    b_ok[b] = j0 < p.gn;
    const int jj = b_ok[b] ? j0 : 0;
    const int rs = jj / p.C;
    b_c[b] = jj - rs * p.C;
    b_s[b] = rs % p.S;
    b_r[b] = rs / p.S;
  }
  // K-tile walk (uniform): image group g, output pixel (pp, qq)
  const int NG = p.N >> 6;
  int g = kt0 % NG;
  const int pq0 = kt0 / NG;
  int pp = pq0 / p.Q, qq = pq0 - (pq0 / p.Q) * p.Q;
  auto issue = [&](int s) {
    char* dst = smem + s * STAGE;
    const unsigned a_so = (unsigned)(g * 64 * PQK + (pp * p.Q + qq) * p.K + m0) * 2u;
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      const int b = i >> 1;
      // (builtin arguments as plain locals: an array element or a ?: passed directly makes clang drop the kernel's
      //  host stub without a diagnostic)
      const int vo = a_vo[i], so = a_ok[b] ? (int)a_so : 0;
      const __amdgpu_buffer_rsrc_t rs = a_ok[b] ? rsA : rsZ;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs,
                                               (__attribute__((address_space(3))) void*)(dst + b * 8192 + ((i & 1) * 4 + wid) * 1024),
                                               16, vo, so, 0, 0);
    }
    const int gb = g * 64 * HWC;
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      const int b = i >> 1;
      const int y = pp * p.stride + b_r[b] - p.pad, x = qq * p.stride + b_s[b] - p.pad;
      const bool ok = b_ok[b] && (unsigned)y < (unsigned)p.H && (unsigned)x < (unsigned)p.W;
      const int so = ok ? (gb + (y * p.W + x) * p.C + b_c[b]) * 2 : 0;
      const int vo = b_vo[i];
      const __amdgpu_buffer_rsrc_t rs = ok ? rsB : rsZ;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs,
                                               (__attribute__((address_space(3))) void*)(dst + A_BYTES + b * 8192 + ((i & 1) * 4 + wid) * 1024),
                                               16, vo, so, 0, 0);
    }
    if (++g == NG) {
      g = 0;
      if (++qq == p.Q) { qq = 0; ++pp; }
    }
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  typedef short s16x4 __attribute__((ext_vector_type(4)));
  typedef __attribute__((address_space(3))) s16x4 lds_s16x4_t;
  // fragment byte offsets within a stage: lane group g4 = lane >> 4 reads columns 16 * (g4 & 1) + pc
  // .. +3 of a 32-column slice at reduction rows 8 * (g4 >> 1) + q4 (+4): the MFMA's lane l then
  // holds column l & 31 and reduction rows 8 * (l >> 5) .. +7 (igemm_kernel's M32 fragment map)
  const int g4 = lane >> 4, q4 = (lane >> 2) & 3, pc = (lane & 3) * 4;
  const int frow = 8 * (g4 >> 1) + q4;
  int fa_off[TM], fb_off[TN];
#pragma unroll
  for (int i = 0; i < TM; ++i) fa_off[i] = w32_off(frow, wr * WTM + i * 32 + 16 * (g4 & 1) + pc);
#pragma unroll
  for (int j = 0; j < TN; ++j) fb_off[j] = A_BYTES + w32_off(frow, wc * WTN + j * 32 + 16 * (g4 & 1) + pc);
  bf16x8 fa0[2][TM], fb0[2][TN], fa1[2][TM], fb1[2][TN];
  // rows rowb and rowb + 4 share the swizzle (bit 1 of the row), +16 rows = +2048 B: immediates
  auto rd = [&](bf16x8(&fa)[2][TM], bf16x8(&fb)[2][TN], int half, int s) {
    const char* base = smem + s * STAGE;
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int ro = (half * 2 + k) * 16 * 128;
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t*)(base + fa_off[i] + ro));
        s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t*)(base + fa_off[i] + ro + 512));
        fa[k][i] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t*)(base + fb_off[j] + ro));
        s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t*)(base + fb_off[j] + ro + 512));
        fb[k][j] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
      }
    }
  };
  auto mma = [&](bf16x8(&fa)[2][TM], bf16x8(&fb)[2][TN]) {
#pragma unroll
    for (int k = 0; k < 2; ++k)
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[k][i], fb[k][j], acc[i][j], 0, 0, 0);
  };
  constexpr int NMF = 2 * TM * TN, NDS = 4 * (TM + TN), NVM = NA + NB;
  constexpr int DPM = NDS / NMF > 0 ? NDS / NMF : 1, MPD = NMF >= NDS ? NMF / NDS : 1;
  enum { FULL = 0, NODMA = 1, LAST = 2 };
  // K-tile in stage S (compile-time: immediate LDS offsets); FULL issues the DMA of tile t+2
  auto ktile = [&](auto stage, auto form) {
    constexpr int S = decltype(stage)::value;
    constexpr int F = decltype(form)::value;
    rd(fa1, fb1, 1, S);
    mma(fa0, fb0);
#pragma unroll
    for (int q = 0; q < NDS; ++q) {
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      if (q % DPM == 0) __builtin_amdgcn_sched_group_barrier(0x8, MPD, 0);
    }
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (F != LAST) {
      wait_vm_b<0>();
      lds_sync_b();   // every wave's reads of stage S retired; the next tile's stage landed
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (F == FULL) issue(S);
      rd(fa0, fb0, 0, S ^ 1);
    }
    mma(fa1, fb1);
    if constexpr (F == FULL) {
#pragma unroll
      for (int q = 0; q < NDS; ++q) {
        if (q < NVM) __builtin_amdgcn_sched_group_barrier(0x10, 1, 1);
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 1);
        if (q % DPM == 0) __builtin_amdgcn_sched_group_barrier(0x8, MPD, 1);
      }
    } else if constexpr (F == NODMA) {
#pragma unroll
      for (int q = 0; q < NDS; ++q) {
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 1);
        if (q % DPM == 0) __builtin_amdgcn_sched_group_barrier(0x8, MPD, 1);
      }
    }
    __builtin_amdgcn_sched_barrier(0);
  };
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  using FF = std::integral_constant<int, FULL>;
  using FN = std::integral_constant<int, NODMA>;
  using FL = std::integral_constant<int, LAST>;
  if (nk > 0) {
    issue(0);
    if (nk > 1) {
      issue(1);
      wait_vm_b<NA + NB>();
    } else {
      wait_vm_b<0>();
    }
    lds_sync_b();
    rd(fa0, fb0, 0, 0);
    int t = 0;
    for (; t + 3 < nk; t += 2) {   // tiles t, t+1 both issue a DMA (t + 1 < nk - 2)
      ktile(I0{}, FF{});
      ktile(I1{}, FF{});
    }
    const int rem = nk - t;   // 1, 2 or 3 tiles left, tile t in stage 0
    if (rem == 3) {
      ktile(I0{}, FF{});
      ktile(I1{}, FN{});
      ktile(I0{}, FL{});
    } else if (rem == 2) {
      ktile(I0{}, FN{});
      ktile(I1{}, FL{});
    } else {
      ktile(I0{}, FL{});
    }
  }

  // epilogue: fp32 partial / result tile; 32x32 accumulator: column (lane & 31), register r ->
  // row 8 * (r / 4) + 4 * (lane >> 5) + r % 4
  float* out = reinterpret_cast<float*>(p.out) + (size_t)split * p.gm * p.gn;
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int col = n0 + wc * WTN + j * 32 + (lane & 31);
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = m0 + wr * WTM + i * 32 + 8 * (r >> 2) + 4 * (lane >> 5) + (r & 3);
        if (row < p.gm && col < p.gn) {
          float v = acc[i][j][r] * p.alpha;
          float* d = out + (size_t)row * p.gn + col;
          if (p.accumulate) v += *d;
          *d = v;
        }
      }
    }
}

// eligible shapes: no BatchNorm fold (those operands are formed in registers), a batch of whole
// 64-image groups, 64-multiple channel counts (a 64-column block is one tap / one 128-B row run)
static bool use_wgrad_dma32(const IgemmParams& p) {
  if (!kn_wgrad_dma32.get() || p.fold_x || p.act_sc) return false;
  if (p.N % 64 || p.C % 64 || p.K % 64 || p.gk % 64) return false;
  // 32-bit offsets: per-lane parts and the block-uniform parts stay below 2^31 bytes
  return (int64_t)p.N * p.P * p.Q * p.K * 2 < (1ll << 31) && (int64_t)p.N * p.H * p.W * p.C * 2 < (1ll << 31);
}
static void wgrad_dma32_tile(const IgemmParams& p, int& BM, int& BN) {
  BM = p.gm <= 64 ? 64 : 128;
  BN = p.gn <= 64 ? 64 : 128;
}

template <int BM, int BN>
static void launch_wgrad_dma32_cfg(IgemmParams& p, hipStream_t st) {
  p.tiles_m = ceil_div(p.gm, BM);
  p.tiles_n = ceil_div(p.gn, BN);
  TORCH_CHECK(p.ksplit % 64 == 0 && p.gk % 64 == 0 && p.N % 64 == 0 && p.C % 64 == 0, "wgrad_dma32: geometry");
  TORCH_CHECK((int64_t)p.nsplit * (p.ksplit / 64) >= p.gk / 64, "wgrad_dma32: splits do not cover the reduction");
  const int grid = p.tiles_m * p.tiles_n * p.nsplit;
  const size_t smem = (size_t)2 * (BM + BN) * 128;
  auto kf = &wgrad_dma32_kernel<BM, BN>;
  static bool attr = false;
  if (!attr) {
    PCMP_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(kf), hipFuncAttributeMaxDynamicSharedMemorySize,
                                       160 * 1024));
    attr = true;
  }
  hipLaunchKernelGGL(kf, dim3(grid), dim3(256), smem, st, p);
  PCMP_LAUNCH_CHECK();
}

static void launch_wgrad_dma32(IgemmParams& p, hipStream_t st) {
  int BM, BN;
  wgrad_dma32_tile(p, BM, BN);
  if (BM == 64) {
    if (BN == 64) launch_wgrad_dma32_cfg<64, 64>(p, st); else launch_wgrad_dma32_cfg<64, 128>(p, st);
  } else {
    if (BN == 64) launch_wgrad_dma32_cfg<128, 64>(p, st); else launch_wgrad_dma32_cfg<128, 128>(p, st);
  }
}

}  // namespace pcmp

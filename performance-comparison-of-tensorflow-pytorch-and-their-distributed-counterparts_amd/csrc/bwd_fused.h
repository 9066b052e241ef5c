// Round-6 fused backward of a 1x1 stride-1 conv: DGRAD + its BatchNorm-backward reduction AND the
// WGRAD in ONE streaming pass over the shared operands.
//
// The ResNet layer-1 conv3 (64 -> 256 channels at 56x56, B = 256) backward reads, per pixel,
//   * the BatchNorm-backward input of its output BN: g and x (256 channels each, folded into
//     dz = k1*g + k2*x + k3 -- or a materialised dz),
//   * its input z2 (the pre-BN output of conv2, 64 channels; the conv consumed relu(bn2(z2)))
// twice: once in the DGRAD (dz x W -> g2, masked by relu(bn2(z2)) > 0, + bn2's backward partial sums)
// and once more in the WGRAD (dz^T x relu(bn2(z2)) -> dW) on the side stream -- 2 x 1.15 KB per pixel,
// 1.85 GB per call, three calls per step, all while layer 1 is HBM-bound (the DGRAD alone streams at
// ~5 TB/s isolated and half that beside the WGRAD: profiles/r6b_prof_bench.txt).  Here each workgroup
// walks a fixed set of 32-pixel tiles (the bnr_stream_kernel pipeline: the next tile's g / x / z2 DMA'd
// into the other LDS stage while the current one computes) and per tile
//   1. folds dz in place (bn_bwd_apply's rounding) and forms y2 = relu(bn2(z2)) (bn_apply's rounding);
//   2. DGRAD: [32 px x 64] = dz [32 x 256] . Wt^T on v_mfma_f32_32x32x16_bf16 (Wt resident in LDS), then
//      the BN-reduce epilogue in the BatchNorm-apply layout (per-thread column sums in registers);
//   3. WGRAD: dW [256 x 64] += dz^T [256 x 32] . y2 [32 x 64] from the same LDS tiles (transposed
//      fragment reads), accumulated in registers across all of the workgroup's tiles (64 per lane);
// and writes its dW partial once at the end (one fp32 row per workgroup; splitk_reduce2 sums them in
// a fixed order: run-to-run deterministic).  1.03 GB per call instead of 1.85 + 0.82.
//
// dz image layout [32 px][256 co] (512-B rows): 16-B chunk c of row r sits at c ^ S(r),
// S(r) = ((r & 3) << 2) | ((r >> 2) & 3), which keeps both reads conflict-free: the DGRAD's row reads
// (16 lanes = 16 rows at one chunk: S is a permutation of 0..15) and the WGRAD's transposed reads
// (ds_read_b64_tr_b16: a 32-lane cycle = 4 consecutive rows x one 64-B group: S(r) differs by 4s).
//
// Reference parity: BatchNorm2d / conv backward of torchvision's Bottleneck conv3 (SURVEY.md §2.4.1;
// /root/reference/pytorch_training_inference_on_image.ipynb:454-626).
#pragma once
#include "bnr_stream.h"

namespace pcmp {

inline Knob kn_bwd_fused("bwd_fused", 1);
inline Knob kn_bwd_fused_wgs("bwd_fused_wgs", 256);

__device__ __forceinline__ int bwf_swz(int r) { return ((r & 3) << 2) | ((r >> 2) & 3); }
// byte offset of element (row, col) in a [rows][256] bf16 image with the S swizzle, col % 4 == 0
__device__ __forceinline__ int bwf_off(int row, int col) {
  return row * 512 + (((col >> 3) ^ bwf_swz(row)) << 4) + ((col & 7) << 1);
}

struct BwdFusedParams {
  const __bf16* g;        // [M][KC] masked BN-input gradient (FOLD) or dz
  const __bf16* fx;       // [M][KC] BN input x (FOLD)
  const float* fcoef;     // [3][KC] (FOLD)
  const __bf16* wt;       // [CC][KC] transposed weight
  const __bf16* z;        // [M][CC] pre-BN input of the conv
  const float* sc;        // [CC] the input BN's scale (act fold + ReLU mask)
  const float* sh;        // [CC]
  const float* mean;      // [CC] the input BN's batch mean / invstd (backward reduction)
  const float* istd;
  __bf16* gout;           // [M][CC] masked input gradient
  float* part;            // [groups][2][CC]
  float* dw;              // [groups][KC * CC] WGRAD partials
  int M;
  unsigned g_bytes, z_bytes, wt_bytes;
};

template <int KC, int CC, bool FOLD>
__global__ void __launch_bounds__(256, 1) bwd_fused_kernel(const BwdFusedParams p, int groups) {
  static_assert(KC == 256 && CC == 64, "bwd_fused: the layer-1 conv3 geometry");
  constexpr int BM = 32, NTHR = 256;
  constexpr int G_IMG = BM * KC * 2;                 // 16 KB
  constexpr int Z_IMG = BM * CC * 2;                 // 4 KB
  constexpr int STAGE = G_IMG * (FOLD ? 2 : 1) + Z_IMG;
  constexpr int W_BYTES = CC * KC * 2;               // 32 KB
  constexpr int CS = CC + 8;
  constexpr int NGI = G_IMG / 1024 / 4;              // 4 DMA instructions per wave per image
  constexpr int NWI = W_BYTES / 1024 / 4;            // 8
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* sW = smem;
  char* sS = smem + W_BYTES;
  char* sY = sS + 2 * STAGE;                         // y2 [32][64] bf16, tr_off<64, M32> swizzle
  float* sC = reinterpret_cast<float*>(sY + Z_IMG);  // [32][CS]
  float* sK = sC + BM * CS;                          // fold coefficients [3][KC]

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int grp = xcd_remap(blockIdx.x, gridDim.x);
  const int npt = p.M / BM;
  const int nmine = grp < npt ? (npt - 1 - grp) / groups + 1 : 0;

  const __amdgpu_buffer_rsrc_t rsG = make_rsrc(p.g, p.g_bytes);
  const __amdgpu_buffer_rsrc_t rsX = make_rsrc(FOLD ? p.fx : p.g, p.g_bytes);
  const __amdgpu_buffer_rsrc_t rsZ = make_rsrc(p.z, p.z_bytes);
  const __amdgpu_buffer_rsrc_t rsW = make_rsrc(p.wt, p.wt_bytes);
  const __amdgpu_buffer_rsrc_t rs0 = make_rsrc(p.g, 0u);

  // per-lane DMA source offsets: image instruction u covers rows 2u, 2u+1 (512-B rows); LDS chunk
  // (lane & 31) of row r holds source chunk (lane & 31) ^ S(r); z image: rows 8u.. (128-B rows, plain)
  int g_vo[NGI];
#pragma unroll
  for (int i = 0; i < NGI; ++i) {
    const int u = wid * NGI + i;
    const int row = 2 * u + (lane >> 5);
    g_vo[i] = (row * KC + (((lane & 31) ^ bwf_swz(row)) << 3)) * 2;
  }
  const int z_vo = ((wid * 8 + (lane >> 3)) * CC + (lane & 7) * 8) * 2;
  auto issue = [&](int s, int pt, bool live) {
    char* dst = sS + s * STAGE;
    const __amdgpu_buffer_rsrc_t rg = live ? rsG : rs0, rx = live ? rsX : rs0, rz = live ? rsZ : rs0;
    const int sg = live ? pt * BM * KC * 2 : 0, sz = live ? pt * BM * CC * 2 : 0;
#pragma unroll
    for (int i = 0; i < NGI; ++i) {
      const int vo = g_vo[i];
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rg, (__attribute__((address_space(3))) void*)(dst + (wid * NGI + i) * 1024),
                                               16, vo, sg, 0, 0);
    }
    if constexpr (FOLD) {
#pragma unroll
      for (int i = 0; i < NGI; ++i) {
        const int vo = g_vo[i];
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            rx, (__attribute__((address_space(3))) void*)(dst + G_IMG + (wid * NGI + i) * 1024), 16, vo, sg, 0, 0);
      }
    }
    {
      const int vo = z_vo;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rz, (__attribute__((address_space(3))) void*)(dst + G_IMG * (FOLD ? 2 : 1) + wid * 1024), 16, vo, sz, 0, 0);
    }
  };
  // resident Wt [64][256] (same swizzle), fold coefficients
  {
#pragma unroll
    for (int i = 0; i < NWI; ++i) {
      const int u = wid * NWI + i;
      const int row = 2 * u + (lane >> 5);
      const int vo = (row * KC + (((lane & 31) ^ bwf_swz(row)) << 3)) * 2;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsW, (__attribute__((address_space(3))) void*)(sW + u * 1024), 16, vo, 0,
                                               0, 0);
    }
  }
  if constexpr (FOLD) {
    for (int i = tid; i < 3 * KC; i += NTHR) sK[i] = p.fcoef[i];
  }
  // per-thread channel group (act pass and epilogue): row tid / 8, channels 8 * (tid & 7) .. +7
  const int er = tid >> 3, ec = (tid & 7) * 8;
  float a_sc[8], a_sh[8], ka[8], kb[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    a_sc[e] = p.sc[ec + e];
    a_sh[e] = p.sh[ec + e];
    ka[e] = p.istd[ec + e];
    kb[e] = -p.mean[ec + e] * ka[e];
  }
  float sm0[8], sm1[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) { sm0[e] = 0.f; sm1[e] = 0.f; }
  f32x16 acc2[2][2];   // dW rows 64 * wid + 32 i, columns 32 j
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc2[i][j][r] = 0.f;

  typedef short s16x4 __attribute__((ext_vector_type(4)));
  typedef __attribute__((address_space(3))) s16x4 lds_s16x4_t;
  const int g4 = lane >> 4, q4 = (lane >> 2) & 3, pc = (lane & 3) * 4;
  // WGRAD transposed-read offsets (k = pixel rows rowb, rowb + 4 of k-step kq)
  int ta_off[2][2][2], tb_off[2][2][2];   // [kq][i or j][lo / hi]
#pragma unroll
  for (int kq = 0; kq < 2; ++kq) {
    const int rowb = kq * 16 + 8 * (g4 >> 1) + q4;
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int colA = 64 * wid + 32 * t + 16 * (g4 & 1) + pc;
      const int colB = 32 * t + 16 * (g4 & 1) + pc;
      ta_off[kq][t][0] = bwf_off(rowb, colA);
      ta_off[kq][t][1] = bwf_off(rowb + 4, colA);
      tb_off[kq][t][0] = tr_off<CC, true>(rowb, colB);
      tb_off[kq][t][1] = tr_off<CC, true>(rowb + 4, colB);
    }
  }

  const int pt0 = grp;
  issue(0, pt0, nmine > 0);
  wait_vm_b<0>();
  lds_sync_b();

  auto tile = [&](auto sel, int j) {
    constexpr int S = decltype(sel)::value;
    const int pt = pt0 + j * groups;
    if (j > 0) {
      wait_vm_b<1>();   // stage S landed: issued after its DMA was tile j-1's one store
      lds_sync_b();
    }
    char* sG = sS + S * STAGE;
    char* sZ = sG + G_IMG * (FOLD ? 2 : 1);
    // 1. dz = k1*g + k2*x + k3 in place; y2 = relu(sc * z + sh) into sY
    if constexpr (FOLD) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int q = tid + NTHR * i, row = q >> 5;
        const int kc = (((q & 31) ^ bwf_swz(row)) << 3);
        char* gp = sG + q * 16;
        const uint4 gv = *reinterpret_cast<const uint4*>(gp);
        const uint4 xv = *reinterpret_cast<const uint4*>(gp + G_IMG);
        float k1[8], k2[8], k3[8];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const f32x4 a = *reinterpret_cast<const f32x4*>(sK + kc + 4 * h);
          const f32x4 b = *reinterpret_cast<const f32x4*>(sK + KC + kc + 4 * h);
          const f32x4 c = *reinterpret_cast<const f32x4*>(sK + 2 * KC + kc + 4 * h);
#pragma unroll
          for (int e = 0; e < 4; ++e) { k1[4 * h + e] = a[e]; k2[4 * h + e] = b[e]; k3[4 * h + e] = c[e]; }
        }
        *reinterpret_cast<uint4*>(gp) = fold_dz(gv, xv, k1, k2, k3, true);
      }
    }
    const uint4 zv = *reinterpret_cast<const uint4*>(sZ + tid * 16);   // row er, channels ec..ec+7
    *reinterpret_cast<uint4*>(sY + tr_off<CC, true>(er, ec)) = fold_act(zv, a_sc, a_sh, true);
    lds_sync_b();
    // next tile's operands (after the in-place fold: see bnr_stream_kernel)
    __builtin_amdgcn_sched_barrier(0);
    issue(S ^ 1, pt + groups, j + 1 < nmine);
    __builtin_amdgcn_sched_barrier(0);
    // 2. DGRAD (waves 0, 1: output channels 32 * wid ..): D[px][c] -> sC
    if (wid < 2) {
      f32x16 acc;
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[r] = 0.f;
      const int ra = lane & 31, rb = wid * 32 + (lane & 31);
#pragma unroll
      for (int ks = 0; ks < KC / 16; ++ks) {
        const int ch = ks * 2 + (lane >> 5);
        const bf16x8 fa = *reinterpret_cast<const bf16x8*>(sG + ra * 512 + ((ch ^ bwf_swz(ra)) << 4));
        const bf16x8 fb = *reinterpret_cast<const bf16x8*>(sW + rb * 512 + ((ch ^ bwf_swz(rb)) << 4));
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa, fb, acc, 0, 0, 0);
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) sC[(8 * (r >> 2) + 4 * (lane >> 5) + (r & 3)) * CS + wid * 32 + (lane & 31)] = acc[r];
    }
    // 3. WGRAD: dW[64 wid + 32 i][32 t] += dz^T . y2 over this tile's 32 pixels
#pragma unroll
    for (int kq = 0; kq < 2; ++kq) {
      bf16x8 fa[2], fb[2];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t*)(sG + ta_off[kq][t][0]));
        s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t*)(sG + ta_off[kq][t][1]));
        fa[t] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
        s16x4 lb = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t*)(sY + tb_off[kq][t][0]));
        s16x4 hb = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4_t*)(sY + tb_off[kq][t][1]));
        fb[t] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lb, hb, 0, 1, 2, 3, 4, 5, 6, 7));
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int t = 0; t < 2; ++t) acc2[i][t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i], fb[t], acc2[i][t], 0, 0, 0);
    }
    lds_sync_b();
    // 4. BN-reduce epilogue: g2 = mask * bf16(D), mask = relu(sc * z + sh) > 0; sums g2, g2 * xhat
    {
      const f32x4 a0 = *reinterpret_cast<const f32x4*>(sC + er * CS + ec);
      const f32x4 a1 = *reinterpret_cast<const f32x4*>(sC + er * CS + ec + 4);
      const float av[8] = {a0[0], a0[1], a0[2], a0[3], a1[0], a1[1], a1[2], a1[3]};
      const unsigned zw[4] = {zv.x, zv.y, zv.z, zv.w};
      unsigned ov[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        unsigned u = f2bf2(av[2 * q], av[2 * q + 1]);
        const float za = __uint_as_float(zw[q] << 16), zb = __uint_as_float(zw[q] & 0xffff0000u);
        u &= (fmaf(za, a_sc[2 * q], a_sh[2 * q]) > 0.f ? 0x0000ffffu : 0u) |
             (fmaf(zb, a_sc[2 * q + 1], a_sh[2 * q + 1]) > 0.f ? 0xffff0000u : 0u);
        const float g0 = __uint_as_float(u << 16), g1 = __uint_as_float(u & 0xffff0000u);
        sm0[2 * q] += g0;
        sm0[2 * q + 1] += g1;
        sm1[2 * q] += g0 * fmaf(za, ka[2 * q], kb[2 * q]);
        sm1[2 * q + 1] += g1 * fmaf(zb, ka[2 * q + 1], kb[2 * q + 1]);
        ov[q] = u;
      }
      *reinterpret_cast<uint4*>(p.gout + (size_t)(pt * BM + er) * CC + ec) = uint4{ov[0], ov[1], ov[2], ov[3]};
    }
  };
  int j = 0;
  for (; j + 1 < nmine; j += 2) {
    tile(std::integral_constant<int, 0>{}, j);
    tile(std::integral_constant<int, 1>{}, j + 1);
  }
  if (j < nmine) tile(std::integral_constant<int, 0>{}, j);

  // WGRAD partial of this workgroup: row grp of dw [groups][KC][CC]
  float* dwp = p.dw + (size_t)grp * KC * CC;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = 64 * wid + 32 * i + 8 * (r >> 2) + 4 * (lane >> 5) + (r & 3);
        dwp[row * CC + 32 * t + (lane & 31)] = acc2[i][t][r];
      }
  // BN partial sums: [32 rows of threads][2][64] through LDS, one row of part
  __syncthreads();
  float* red = reinterpret_cast<float*>(sS);
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    red[(er * 2 + 0) * CC + ec + e] = sm0[e];
    red[(er * 2 + 1) * CC + ec + e] = sm1[e];
  }
  __syncthreads();
  if (tid < 2 * CC) {
    const int q = tid / CC, c = tid % CC;
    float t = 0.f;
    for (int r = 0; r < BM; ++r) t += red[(r * 2 + q) * CC + c];
    p.part[(size_t)grp * 2 * CC + q * CC + c] = t;
  }
}

}  // namespace pcmp

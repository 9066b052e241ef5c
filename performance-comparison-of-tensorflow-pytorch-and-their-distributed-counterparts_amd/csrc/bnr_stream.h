// Round-6 streaming DGRAD + BatchNorm-backward-reduce kernel for the memory-bound short-K 1x1 DGRADs
// of ResNet layers 1-2 (K = 64 / 128 / 256 reduction channels).
//
//   g[m][c] = mask(m, c) * bf16( sum_k dz[m][k] * Wt[c][k]  +  resid[m][c] )
//   part[grp][0][c] += g,  part[grp][1][c] += g * (x[m][c] - mean[c]) * istd[c]   (+ x2 / part2: dual BN)
//
// These GEMMs are epilogue streams: per output element they read the residual gradient and the BN
// input x (and x2), write g, and do ~25 VALU of BN-reduce math, against a 64-256-deep reduction.  The
// round-1..5 kernel (igemm_kernel<MODE_DGRAD, ..., EPI_BNR>) runs ONE tile per workgroup: operand
// loads -> LDS -> MFMA -> an epilogue with a 3-step register load ring, so every tile pays its operand
// latency serially and the streams ran at 2.2-3.5 TB/s (r4 PMC: 63 % of cycles waiting, VALU 32 %
// busy -- latency-bound, profiles/r4_dgrad_pmc.txt).  Here a workgroup walks a fixed set of 32-pixel
// tiles and always has the NEXT tile's operands in flight while it computes the current one:
//   * the next tile's dz operand (or g and x of the BatchNorm-backward fold) by LDS-DMA into the other
//     of two LDS stages (buffer_load ... lds, no VGPRs);
//   * the next tile's epilogue operands (resid / x / x2 16-B chunks and the ReLU-mask bits) by buffer
//     loads into a second register set;
//   * the transposed weight Wt[c-tile][K] stays resident in LDS for the whole kernel.
// The MFMA result (v_mfma_f32_32x32x16_bf16, one 32x32 tile per wave) goes to an fp32 LDS tile, and the
// epilogue runs in the BatchNorm-apply layout: each thread owns ONE fixed 8-channel group, so its
// per-channel coefficients and its column sums live in registers across all of its tiles (one
// cross-thread reduction per workgroup at the end, not per tile), and every load / store is a
// coalesced 16-B row chunk.  The partial-statistics buffer gets one row per workgroup group (T <= 512
// rows: the one-launch BN finalize) instead of one per 128-pixel tile.
//
// vmcnt bookkeeping: every load and store of a tile is issued unconditionally (absent operands read
// through a zero-record buffer descriptor, which returns 0), so the counts are compile-time constants
// and the top-of-tile wait retires exactly the stage the tile reads.  Summation order is fixed per
// workgroup (static tile assignment): results are run-to-run deterministic.
//
// Reference parity: the BatchNorm2d / conv backward of torchvision's Bottleneck (SURVEY.md §2.4.1;
// /root/reference/pytorch_training_inference_on_image.ipynb:454-626).
#pragma once
#include "igemm.h"

namespace pcmp {

inline Knob kn_bnr_stream("bnr_stream", 1);
// workgroups: 256 (one per CU, ~2x the tiles per workgroup of 512) streams layers 1-3 at 3.5-5.5 TB/s
// (profiles/r6_bnr_stream_micro_v2.txt)
inline Knob kn_bnr_stream_wgs("bnr_stream_wgs", 256);

template <int BN, int GK, bool FOLD, bool DUAL>
__global__ void __launch_bounds__(256, 2) bnr_stream_kernel(const IgemmParams p, int groups) {
  constexpr int BM = 32, NTHR = 256;
  constexpr int KB = GK / 64;                       // 64-deep reduction blocks
  constexpr int A_IMG = BM * GK * 2;                // one [KB][BM][128 B] operand image
  constexpr int STAGE = A_IMG * (FOLD ? 2 : 1);
  constexpr int W_BYTES = BN * GK * 2;
  constexpr int CS = BN + 8;                        // fp32 result tile row stride (floats)
  constexpr int C_BYTES = BM * CS * 4;
  constexpr int CPR = BN / 8;                       // 16-B chunks per tile row
  constexpr int NCH = BM * BN / 8 / NTHR;           // epilogue chunks per thread (1 or 2)
  constexpr int RPP = NTHR / CPR;                   // rows per pass
  constexpr int NS = DUAL ? 3 : 2;
  constexpr int NWT = BN / 32;                      // 32x32 MFMA tiles (waves that run the GEMM)
  constexpr int NAI = A_IMG / 1024 / 4;             // A-image DMA instructions per wave
  constexpr int NWI = W_BYTES / 1024 / 4;           // Wt-image DMA instructions per wave
  constexpr int NEL = NCH * (DUAL ? 4 : 3);         // epilogue-operand loads per tile per thread
  static_assert(NCH >= 1 && NAI >= 1 && NWI >= 1 && NWT <= 4, "bnr_stream tile");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* sW = smem;
  char* sS = smem + W_BYTES;                        // two stages
  float* sC = reinterpret_cast<float*>(smem + W_BYTES + 2 * STAGE);
  float* sK = sC + BM * CS;                         // fold coefficients [3][GK]

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int ntn = p.gn / BN;
  const int lin = xcd_remap(blockIdx.x, gridDim.x);
  const int grp = lin / ntn, n0 = (lin - grp * ntn) * BN;
  const int npt = p.gm / BM;                        // pixel tiles
  const int nmine = grp < npt ? (npt - 1 - grp) / groups + 1 : 0;

  const __amdgpu_buffer_rsrc_t rsA = make_rsrc(p.a, p.a_bytes);
  const __amdgpu_buffer_rsrc_t rsF = make_rsrc(FOLD ? p.fold_x : p.a, p.a_bytes);
  const __amdgpu_buffer_rsrc_t rsW = make_rsrc(p.b, p.b_bytes);
  const unsigned ebytes = (unsigned)((size_t)p.gm * p.gn * 2);
  const bool has_res = p.resid != nullptr;
  const unsigned rbytes = !has_res ? 0u : (p.resid_sub ? (unsigned)((size_t)p.N * p.rs_H2 * p.rs_W2 * p.gn * 2) : ebytes);
  const __amdgpu_buffer_rsrc_t rsR = make_rsrc(has_res ? (const void*)p.resid : (const void*)p.a, rbytes);
  const __amdgpu_buffer_rsrc_t rsX = make_rsrc(p.bn_x, ebytes);
  const __amdgpu_buffer_rsrc_t rsX2 = make_rsrc(DUAL ? p.bn_x2 : p.bn_x, DUAL ? ebytes : 0u);
  const bool has_mb = p.bn_mbits != nullptr;
  const __amdgpu_buffer_rsrc_t rsM = make_rsrc(has_mb ? (const void*)p.bn_mbits : (const void*)p.a,
                                               has_mb ? (unsigned)((size_t)p.gm * p.gn / 8) : 0u);

  // ---- A-operand DMA: image u-th instruction of wave w covers k-block u/4, rows (u%4)*8..+7 -------
  const int lch = (lane & 7) ^ ((lane >> 3) & 7);   // source chunk of LDS chunk (lane & 7), row & 7 = lane >> 3
  int a_vo[NAI];
#pragma unroll
  for (int i = 0; i < NAI; ++i) {
    const int u = wid * NAI + i;
    const int row = (u & 3) * 8 + (lane >> 3);
    a_vo[i] = (row * GK + (u >> 2) * 64 + lch * 8) * 2;
  }
  const __amdgpu_buffer_rsrc_t rsZ = make_rsrc(p.a, 0u);   // zero records
  auto issue_a = [&](int s, int pt, bool live) {
    char* dst = sS + s * STAGE;
    const int so = live ? pt * BM * GK * 2 : 0;
    const __amdgpu_buffer_rsrc_t ra = live ? rsA : rsZ, rf = live ? rsF : rsZ;
#pragma unroll
    for (int i = 0; i < NAI; ++i) {
      const int vo = a_vo[i];
      __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, (__attribute__((address_space(3))) void*)(dst + (wid * NAI + i) * 1024),
                                               16, vo, so, 0, 0);
    }
    if constexpr (FOLD) {
#pragma unroll
      for (int i = 0; i < NAI; ++i) {
        const int vo = a_vo[i];
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            rf, (__attribute__((address_space(3))) void*)(dst + A_IMG + (wid * NAI + i) * 1024), 16, vo, so, 0, 0);
      }
    }
  };

  // ---- epilogue operands: thread t owns channels n0 + c8*8 .. +7 of rows t / CPR + k * RPP ---------
  const int c8 = tid % CPR, r0 = tid / CPR;
  uint4 eR[2][NCH], eX[2][NCH], eX2[2][DUAL ? NCH : 1];
  unsigned eM[2][NCH];   // the dword holding the chunk's mask byte (a byte load's widening would wait for it)
  auto issue_e = [&](auto sel, int pt, bool live) {
    constexpr int E = decltype(sel)::value;
    if (!live) pt = 0;
    unsigned o[NCH], ro[NCH];   // every offset first, then the loads (no address math behind a load)
#pragma unroll
    for (int k = 0; k < NCH; ++k) {
      const int m = pt * BM + r0 + k * RPP;
      o[k] = (unsigned)m * (unsigned)p.gn + (unsigned)(n0 + c8 * 8);
      ro[k] = o[k] * 2u;
      if (p.resid_sub) {   // compact [N][H/2][W/2][C] residual, added at even pixels only
        const unsigned n = fdiv((unsigned)m, p.fd_HW);
        const unsigned rem = (unsigned)m - n * (unsigned)(p.H * p.W);
        const unsigned hh = fdiv(rem, p.fd_W);
        const unsigned ww = rem - hh * (unsigned)p.W;
        ro[k] = ((hh | ww) & 1u) ? kOOB
                                 : (((n * (unsigned)p.rs_H2 + (hh >> 1)) * (unsigned)p.rs_W2 + (ww >> 1)) * (unsigned)p.gn +
                                    (unsigned)(n0 + c8 * 8)) * 2u;
      }
    }
#pragma unroll
    for (int k = 0; k < NCH; ++k) {
      if (!live) { o[k] = kOOB / 2u; ro[k] = kOOB; }
    }
#pragma unroll
    for (int k = 0; k < NCH; ++k) {
      eR[E][k] = bload16(rsR, ro[k]);
      eX[E][k] = bload16(rsX, o[k] * 2u);
      if constexpr (DUAL) eX2[E][k] = bload16(rsX2, o[k] * 2u);
      eM[E][k] = __builtin_amdgcn_raw_buffer_load_b32(rsM, (int)((o[k] >> 3) & ~3u), 0, 0);   // (OOB: 2^27 is past the bits)
    }
  };

  // ---- per-thread channel constants and column sums ------------------------------------------------
  float ka[8], kb[8], ka2[DUAL ? 8 : 1], kb2[DUAL ? 8 : 1], msc[8], msh[8];
  const bool mfx = !has_mb;   // mask recomputed from x: relu(x * msc + msh) > 0
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const int c = n0 + c8 * 8 + e;
    const float is = p.bn_istd[c];
    ka[e] = is;
    kb[e] = -p.bn_mean[c] * is;
    msc[e] = mfx ? p.bn_msc[c] : 0.f;
    msh[e] = mfx ? p.bn_msh[c] : 0.f;
    if constexpr (DUAL) {
      const float is2 = p.bn_istd2[c];
      ka2[e] = is2;
      kb2[e] = -p.bn_mean2[c] * is2;
    }
  }
  float sm[NS][8];
#pragma unroll
  for (int q = 0; q < NS; ++q)
#pragma unroll
    for (int e = 0; e < 8; ++e) sm[q][e] = 0.f;

  // ---- prologue: resident Wt tile, fold coefficients, tile 0's operands -----------------------------
  {
    int w_vo[NWI];
#pragma unroll
    for (int i = 0; i < NWI; ++i) {
      const int u = wid * NWI + i;                      // k-block u / (BN/8), rows ((u % (BN/8)) * 8)..
      const int row = (u % (BN / 8)) * 8 + (lane >> 3);
      w_vo[i] = ((n0 + row) * GK + (u / (BN / 8)) * 64 + lch * 8) * 2;
    }
#pragma unroll
    for (int i = 0; i < NWI; ++i) {
      const int vo = w_vo[i];
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsW, (__attribute__((address_space(3))) void*)(sW + (wid * NWI + i) * 1024),
                                               16, vo, 0, 0, 0);
    }
  }
  if constexpr (FOLD) {
    for (int i = tid; i < 3 * GK; i += NTHR) sK[i] = p.fold_coef[(i / GK) * p.K + (i % GK)];
  }
  const int pt0 = grp;
  issue_a(0, pt0, nmine > 0);
  issue_e(std::integral_constant<int, 0>{}, pt0, nmine > 0);
  wait_vm_b<0>();
  lds_sync_b();

  // ---- one tile: stage S / register set S hold tile j; tile j+1 is issued into S^1 ------------------
  auto tile = [&](auto sel, int j) {
    constexpr int S = decltype(sel)::value;
    const int pt = pt0 + j * groups;
    if (j > 0) {
      // stage S landed: issued after its DMA were tile j's epilogue-operand loads and tile j-1's stores
      wait_vm_b<NEL + NCH>();
      lds_sync_b();
    }
    char* sA = sS + S * STAGE;
    if constexpr (FOLD) {   // dz = k1*g + k2*x + k3 in place (bn_bwd_apply's rounding)
#pragma unroll
      for (int i = 0; i < KB; ++i) {
        const int row = tid >> 3;
        const int kc = i * 64 + (((tid & 7) ^ (row & 7)) << 3);
        char* gp = sA + i * (BM * 128) + tid * 16;
        const uint4 g = *reinterpret_cast<const uint4*>(gp);
        const uint4 x = *reinterpret_cast<const uint4*>(gp + A_IMG);
        float k1[8], k2[8], k3[8];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const f32x4 a = *reinterpret_cast<const f32x4*>(sK + kc + 4 * h);
          const f32x4 b = *reinterpret_cast<const f32x4*>(sK + GK + kc + 4 * h);
          const f32x4 c = *reinterpret_cast<const f32x4*>(sK + 2 * GK + kc + 4 * h);
#pragma unroll
          for (int e = 0; e < 4; ++e) { k1[4 * h + e] = a[e]; k2[4 * h + e] = b[e]; k3[4 * h + e] = c[e]; }
        }
        *reinterpret_cast<uint4*>(gp) = fold_dz(g, x, k1, k2, k3, true);
      }
      lds_sync_b();
    }
    // the next tile's operands, issued unconditionally (after the last tile through zero-record
    // descriptors: no traffic) so the vmcnt counts are the same on every path; after the in-place
    // fold, whose LDS writes the compiler would otherwise order behind the DMA (a vmcnt(0) wait)
    __builtin_amdgcn_sched_barrier(0);
    const bool more = j + 1 < nmine;
    issue_a(S ^ 1, pt + groups, more);
    __builtin_amdgcn_sched_barrier(0);   // the count above needs the DMAs ahead of the loads
    issue_e(std::integral_constant<int, S ^ 1>{}, pt + groups, more);
    __builtin_amdgcn_sched_barrier(0);
    // GEMM: wave w < NWT computes pixels 0..31 x channels 32w..32w+31 of the tile
    if (wid < NWT) {
      f32x16 acc;
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[r] = 0.f;
#pragma unroll
      for (int ks = 0; ks < GK / 16; ++ks) {
        const int ch = ks * 2 + (lane >> 5);             // 8-element k chunk
        const int kb = ch >> 3, cc = ch & 7;
        const bf16x8 fa = *reinterpret_cast<const bf16x8*>(sA + kb * (BM * 128) + rr_off(lane & 31, cc));
        const bf16x8 fb = *reinterpret_cast<const bf16x8*>(sW + kb * (BN * 128) + rr_off(wid * 32 + (lane & 31), cc));
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa, fb, acc, 0, 0, 0);
      }
      // D[px][ch]: lane holds channel (lane & 31), pixel rows 8*(r/4) + 4*(lane/32) + r%4
#pragma unroll
      for (int r = 0; r < 16; ++r)
        sC[(8 * (r >> 2) + 4 * (lane >> 5) + (r & 3)) * CS + wid * 32 + (lane & 31)] = acc[r];
    }
    lds_sync_b();
    // epilogue (BatchNorm-apply layout)
    __bf16* out = reinterpret_cast<__bf16*>(p.out);
    const int mshift = ((n0 + c8 * 8) >> 3 & 3) * 8;   // byte of the chunk's mask in its dword (gn % 32 == 0)
#pragma unroll
    for (int k = 0; k < NCH; ++k) {
      const int row = r0 + k * RPP;
      const f32x4 a0 = *reinterpret_cast<const f32x4*>(sC + row * CS + c8 * 8);
      const f32x4 a1 = *reinterpret_cast<const f32x4*>(sC + row * CS + c8 * 8 + 4);
      const float av[8] = {a0[0], a0[1], a0[2], a0[3], a1[0], a1[1], a1[2], a1[3]};
      const unsigned rw[4] = {eR[S][k].x, eR[S][k].y, eR[S][k].z, eR[S][k].w};
      const unsigned xw[4] = {eX[S][k].x, eX[S][k].y, eX[S][k].z, eX[S][k].w};
      unsigned ov[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float x0 = av[2 * q] + __uint_as_float(rw[q] << 16);
        const float x1 = av[2 * q + 1] + __uint_as_float(rw[q] & 0xffff0000u);
        unsigned u = f2bf2(x0, x1);
        const float xa = __uint_as_float(xw[q] << 16), xb = __uint_as_float(xw[q] & 0xffff0000u);
        // both masks, then a select (a runtime branch here splits the chunk into 8 basic blocks)
        const float z0 = fmaf(xa, msc[2 * q], msh[2 * q]);
        const float z1 = fmaf(xb, msc[2 * q + 1], msh[2 * q + 1]);
        const unsigned kz = (z0 > 0.f ? 0x0000ffffu : 0u) | (z1 > 0.f ? 0xffff0000u : 0u);
        const unsigned bits = eM[S][k] >> (mshift + 2 * q);
        const unsigned kbits = ((bits & 1u) ? 0x0000ffffu : 0u) | ((bits & 2u) ? 0xffff0000u : 0u);
        u &= mfx ? kz : kbits;
        const float g0 = __uint_as_float(u << 16), g1 = __uint_as_float(u & 0xffff0000u);
        sm[0][2 * q] += g0;
        sm[0][2 * q + 1] += g1;
        sm[1][2 * q] += g0 * fmaf(xa, ka[2 * q], kb[2 * q]);
        sm[1][2 * q + 1] += g1 * fmaf(xb, ka[2 * q + 1], kb[2 * q + 1]);
        if constexpr (DUAL) {
          const unsigned x2w = q == 0 ? eX2[S][k].x : q == 1 ? eX2[S][k].y : q == 2 ? eX2[S][k].z : eX2[S][k].w;
          sm[2][2 * q] += g0 * fmaf(__uint_as_float(x2w << 16), ka2[2 * q], kb2[2 * q]);
          sm[2][2 * q + 1] += g1 * fmaf(__uint_as_float(x2w & 0xffff0000u), ka2[2 * q + 1], kb2[2 * q + 1]);
        }
        ov[q] = u;
      }
      const size_t o = (size_t)(pt * BM + row) * p.gn + n0 + c8 * 8;
      *reinterpret_cast<uint4*>(out + o) = uint4{ov[0], ov[1], ov[2], ov[3]};
    }
  };
  // (the back edge always runs both stages: a path that skipped stage 1 would leave its register set's
  //  loads pending at the loop head, and the compiler would wait for them there)
  int j = 0;
  for (; j + 1 < nmine; j += 2) {
    tile(std::integral_constant<int, 0>{}, j);
    tile(std::integral_constant<int, 1>{}, j + 1);
  }
  if (j < nmine) tile(std::integral_constant<int, 0>{}, j);

  // ---- column sums: [RPP rows][NS][BN] through LDS, then one row of the partial buffers --------------
  __syncthreads();
  float* red = reinterpret_cast<float*>(sS);   // stages and result tile are dead (launch sizes LDS for it)
#pragma unroll
  for (int q = 0; q < NS; ++q) {
    *reinterpret_cast<f32x4*>(red + (r0 * NS + q) * BN + c8 * 8) = f32x4{sm[q][0], sm[q][1], sm[q][2], sm[q][3]};
    *reinterpret_cast<f32x4*>(red + (r0 * NS + q) * BN + c8 * 8 + 4) = f32x4{sm[q][4], sm[q][5], sm[q][6], sm[q][7]};
  }
  __syncthreads();
  for (int i = tid; i < NS * BN; i += NTHR) {
    const int q = i / BN, c = i - q * BN;
    float t = 0.f;
    for (int r = 0; r < RPP; ++r) t += red[(r * NS + q) * BN + c];
    float* st = p.stats + (size_t)grp * 2 * p.gn;
    if (q == 0) {
      st[n0 + c] = t;
      if constexpr (DUAL) p.stats2[(size_t)grp * 2 * p.gn + n0 + c] = t;
    } else if (q == 1) {
      st[p.gn + n0 + c] = t;
    } else {
      p.stats2[(size_t)grp * 2 * p.gn + p.gn + n0 + c] = t;
    }
  }
}

// eligible: 1x1 stride-1 DGRAD with the BN-reduce epilogue, a 64-multiple channel count, K of 64 / 128
// / 256, the ReLU mask as bits or recomputed from x (not a mask tensor), 32-bit byte offsets, and
// more output than (folded) input channels
static bool use_bnr_stream(const IgemmParams& p) {
  if (!kn_bnr_stream.get() || !p.bn_x || p.R != 1 || p.S != 1 || p.stride != 1 || p.pad != 0) return false;
  if (!(p.gk == 64 || p.gk == 128 || p.gk == 256) || p.gn % 64 || p.gm % 32) return false;
  if (!p.bn_mbits && !(p.bn_msc && !p.bn_mask)) return false;
  if (p.relu) return false;
  // the stream pays off where the epilogue's bytes dominate (resid / x / g per output channel): with
  // a dz operand at least as wide as the output (the layer-1 conv3 DGRAD: 2 x 256 folded input
  // channels -> 64) the one-tile kernel is as fast or faster (profiles/r6_bnr_stream_micro.txt)
  if ((p.fold_x ? 2 : 1) * p.gk >= p.gn) return false;
  return (int64_t)p.gm * p.gn * 2 < (1ll << 31) && (int64_t)p.gm * p.gk * 2 < (1ll << 31);
}

static int bnr_stream_bn(const IgemmParams& p) { return p.gn == 64 ? 64 : 128; }

// workgroup groups (= partial-statistics rows) of a bnr_stream launch
static int bnr_stream_groups(const IgemmParams& p) {
  const int ntn = p.gn / bnr_stream_bn(p);
  const int npt = p.gm / 32;
  return std::max(1, std::min(npt, std::max(1, kn_bnr_stream_wgs.get() / ntn)));
}

template <int BN, int GK, bool FOLD, bool DUAL>
static void launch_bnr_stream_cfg(IgemmParams& p, hipStream_t st) {
  constexpr int BM = 32;
  const int ntn = p.gn / BN;
  const int groups = bnr_stream_groups(p);
  TORCH_CHECK(p.stats && p.stats_cap >= groups && (!DUAL || p.stats2), "bnr_stream: partial-stats buffers");
  constexpr size_t stage = (size_t)BM * GK * 2 * (FOLD ? 2 : 1);
  constexpr size_t red = (size_t)(256 / (BN / 8)) * (DUAL ? 3 : 2) * BN * 4;
  constexpr size_t body = 2 * stage + (size_t)BM * (BN + 8) * 4 + (FOLD ? 3 * GK * 4 : 0);
  constexpr size_t smem = (size_t)BN * GK * 2 + std::max(body, red);
  static_assert(smem <= 160 * 1024, "bnr_stream: LDS");
  auto kf = &bnr_stream_kernel<BN, GK, FOLD, DUAL>;
  static bool attr = false;
  if (!attr) {
    PCMP_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(kf), hipFuncAttributeMaxDynamicSharedMemorySize,
                                       160 * 1024));
    attr = true;
  }
  hipLaunchKernelGGL(kf, dim3(groups * ntn), dim3(256), smem, st, p, groups);
  PCMP_LAUNCH_CHECK();
}

static void launch_bnr_stream(IgemmParams& p, hipStream_t st) {
  const bool fold = p.fold_x != nullptr, dual = p.bn_x2 != nullptr;
  const int BN = bnr_stream_bn(p);
#define PCMP_BNRS(B, G)                                                                      \
  do {                                                                                      \
    if (fold) {                                                                             \
      if (dual) launch_bnr_stream_cfg<B, G, true, true>(p, st);                             \
      else launch_bnr_stream_cfg<B, G, true, false>(p, st);                                 \
    } else {                                                                                \
      if (dual) launch_bnr_stream_cfg<B, G, false, true>(p, st);                            \
      else launch_bnr_stream_cfg<B, G, false, false>(p, st);                                \
    }                                                                                       \
  } while (0)
  if (BN == 64) {
    if (p.gk == 64) PCMP_BNRS(64, 64); else if (p.gk == 128) PCMP_BNRS(64, 128); else PCMP_BNRS(64, 256);
  } else {
    if (p.gk == 64) PCMP_BNRS(128, 64); else if (p.gk == 128) PCMP_BNRS(128, 128); else PCMP_BNRS(128, 256);
  }
#undef PCMP_BNRS
}

}  // namespace pcmp

namespace pcmp {

// ------------------------------------------------------------------------------------------------
// The same streaming structure for the expanding 1x1 FWD convs with BatchNorm statistics (the conv3
// of every bottleneck of layers 1-3 and the stride-1 layer-1 downsample: K = 64 / 128 / 256 input
// channels -> 4x as many outputs):
//   y[m][n] = bf16( sum_k a[m][k] * W[n][k] ),  a = x  or  relu(scale[k] * z[m][k] + shift[k])
//   part[grp][0][n] += y,  part[grp][1][n] += y * y
// The one-tile kernels (igemm_kernel<MODE_FWD, ..., EPI_STATS> / igemm_dma32_kernel) write one
// partial-statistics row per 128-pixel tile and pay each tile's operand latency serially; here the
// next tile's operand is DMA'd while the current tile's output streams out, Wt stays in LDS, the
// BatchNorm-forward fold (the previous BN's relu(scale * z + shift), in-place on the LDS operand) is
// applied once per operand element, and each thread's per-channel sums stay in registers for all of
// its tiles (one statistics row per workgroup group).
inline Knob kn_fwd_stream("fwd_stream", 1);
inline Knob kn_fwd_stream_wgs("fwd_stream_wgs", 512);   // 512 > 256 (profiles/r6_fwd_stream_micro.txt)

template <int BN, int GK, bool FOLD>
__global__ void __launch_bounds__(256, 2) fwd_stream_kernel(const IgemmParams p, int groups) {
  constexpr int BM = 32, NTHR = 256;
  constexpr int KB = GK / 64;
  constexpr int A_IMG = BM * GK * 2;
  constexpr int STAGE = A_IMG;
  constexpr int W_BYTES = BN * GK * 2;
  constexpr int CS = BN + 8;
  constexpr int CPR = BN / 8;
  constexpr int NCH = BM * BN / 8 / NTHR;           // 2 (BN 128) or 4 (BN 256)
  constexpr int RPP = NTHR / CPR;
  constexpr int NWT = BN / 32;                      // 32x32 output tiles
  constexpr int TPW = NWT > 4 ? NWT / 4 : 1;        // tiles per GEMM wave
  constexpr int NAI = A_IMG / 1024 / 4;
  constexpr int NWI = W_BYTES / 1024 / 4;
  static_assert(NCH >= 1 && NAI >= 1 && NWI >= 1 && (NWT <= 4 || NWT % 4 == 0), "fwd_stream tile");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* sW = smem;
  char* sS = smem + W_BYTES;
  float* sC = reinterpret_cast<float*>(smem + W_BYTES + 2 * STAGE);
  float* sK = sC + BM * CS;                         // act-fold coefficients [2][GK]

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int ntn = p.gn / BN;
  const int lin = xcd_remap(blockIdx.x, gridDim.x);
  const int grp = lin / ntn, n0 = (lin - grp * ntn) * BN;
  const int npt = p.gm / BM;
  const int nmine = grp < npt ? (npt - 1 - grp) / groups + 1 : 0;

  const __amdgpu_buffer_rsrc_t rsA = make_rsrc(p.a, p.a_bytes);
  const __amdgpu_buffer_rsrc_t rsW = make_rsrc(p.b, p.b_bytes);
  const __amdgpu_buffer_rsrc_t rsZ = make_rsrc(p.a, 0u);
  const int lch = (lane & 7) ^ ((lane >> 3) & 7);
  int a_vo[NAI];
#pragma unroll
  for (int i = 0; i < NAI; ++i) {
    const int u = wid * NAI + i;
    const int row = (u & 3) * 8 + (lane >> 3);
    a_vo[i] = (row * GK + (u >> 2) * 64 + lch * 8) * 2;
  }
  auto issue_a = [&](int s, int pt, bool live) {
    char* dst = sS + s * STAGE;
    const int so = live ? pt * BM * GK * 2 : 0;
    const __amdgpu_buffer_rsrc_t ra = live ? rsA : rsZ;
#pragma unroll
    for (int i = 0; i < NAI; ++i) {
      const int vo = a_vo[i];
      __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, (__attribute__((address_space(3))) void*)(dst + (wid * NAI + i) * 1024),
                                               16, vo, so, 0, 0);
    }
  };
  {
    int w_vo[NWI];
#pragma unroll
    for (int i = 0; i < NWI; ++i) {
      const int u = wid * NWI + i;
      const int row = (u % (BN / 8)) * 8 + (lane >> 3);
      w_vo[i] = ((n0 + row) * GK + (u / (BN / 8)) * 64 + lch * 8) * 2;
    }
#pragma unroll
    for (int i = 0; i < NWI; ++i) {
      const int vo = w_vo[i];
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsW, (__attribute__((address_space(3))) void*)(sW + (wid * NWI + i) * 1024),
                                               16, vo, 0, 0, 0);
    }
  }
  if constexpr (FOLD) {
    for (int i = tid; i < 2 * GK; i += NTHR) sK[i] = i < GK ? p.act_sc[i] : p.act_sh[i - GK];
  }
  const int c8 = tid % CPR, r0 = tid / CPR;
  float sm[2][8];
#pragma unroll
  for (int q = 0; q < 2; ++q)
#pragma unroll
    for (int e = 0; e < 8; ++e) sm[q][e] = 0.f;
  const int pt0 = grp;
  issue_a(0, pt0, nmine > 0);
  wait_vm_b<0>();
  lds_sync_b();

  auto tile = [&](auto sel, int j) {
    constexpr int S = decltype(sel)::value;
    const int pt = pt0 + j * groups;
    if (j > 0) {
      wait_vm_b<NCH>();   // stage S landed: issued after its DMA were tile j-1's stores
      lds_sync_b();
    }
    char* sA = sS + S * STAGE;
    if constexpr (FOLD) {   // a = relu(scale * z + shift), bf16-rounded as bn_apply rounds it
#pragma unroll
      for (int i = 0; i < KB; ++i) {
        const int row = tid >> 3;
        const int kc = i * 64 + (((tid & 7) ^ (row & 7)) << 3);
        char* zp = sA + i * (BM * 128) + tid * 16;
        float a[8], b[8];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const f32x4 u = *reinterpret_cast<const f32x4*>(sK + kc + 4 * h);
          const f32x4 v = *reinterpret_cast<const f32x4*>(sK + GK + kc + 4 * h);
#pragma unroll
          for (int e = 0; e < 4; ++e) { a[4 * h + e] = u[e]; b[4 * h + e] = v[e]; }
        }
        *reinterpret_cast<uint4*>(zp) = fold_act(*reinterpret_cast<const uint4*>(zp), a, b, true);
      }
      lds_sync_b();
    }
    // next tile's operand (after the in-place fold: see bnr_stream_kernel)
    __builtin_amdgcn_sched_barrier(0);
    issue_a(S ^ 1, pt + groups, j + 1 < nmine);
    __builtin_amdgcn_sched_barrier(0);
    if (wid < NWT) {
#pragma unroll
      for (int tt = 0; tt < TPW; ++tt) {
        const int ct = wid + 4 * tt;   // channel tile
        f32x16 acc;
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[r] = 0.f;
#pragma unroll
        for (int ks = 0; ks < GK / 16; ++ks) {
          const int ch = ks * 2 + (lane >> 5);
          const int kb = ch >> 3, cc = ch & 7;
          const bf16x8 fa = *reinterpret_cast<const bf16x8*>(sA + kb * (BM * 128) + rr_off(lane & 31, cc));
          const bf16x8 fb = *reinterpret_cast<const bf16x8*>(sW + kb * (BN * 128) + rr_off(ct * 32 + (lane & 31), cc));
          acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa, fb, acc, 0, 0, 0);
        }
#pragma unroll
        for (int r = 0; r < 16; ++r)
          sC[(8 * (r >> 2) + 4 * (lane >> 5) + (r & 3)) * CS + ct * 32 + (lane & 31)] = acc[r];
      }
    }
    lds_sync_b();
    __bf16* out = reinterpret_cast<__bf16*>(p.out);
#pragma unroll
    for (int k = 0; k < NCH; ++k) {
      const int row = r0 + k * RPP;
      const f32x4 a0 = *reinterpret_cast<const f32x4*>(sC + row * CS + c8 * 8);
      const f32x4 a1 = *reinterpret_cast<const f32x4*>(sC + row * CS + c8 * 8 + 4);
      const float av[8] = {a0[0], a0[1], a0[2], a0[3], a1[0], a1[1], a1[2], a1[3]};
      unsigned ov[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const unsigned u = f2bf2(av[2 * q], av[2 * q + 1]);
        const float y0 = __uint_as_float(u << 16), y1 = __uint_as_float(u & 0xffff0000u);
        sm[0][2 * q] += y0;
        sm[0][2 * q + 1] += y1;
        sm[1][2 * q] += y0 * y0;
        sm[1][2 * q + 1] += y1 * y1;
        ov[q] = u;
      }
      const size_t o = (size_t)(pt * BM + row) * p.gn + n0 + c8 * 8;
      *reinterpret_cast<uint4*>(out + o) = uint4{ov[0], ov[1], ov[2], ov[3]};
    }
  };
  // (the back edge always runs both stages: a path that skipped stage 1 would leave its register set's
  //  loads pending at the loop head, and the compiler would wait for them there)
  int j = 0;
  for (; j + 1 < nmine; j += 2) {
    tile(std::integral_constant<int, 0>{}, j);
    tile(std::integral_constant<int, 1>{}, j + 1);
  }
  if (j < nmine) tile(std::integral_constant<int, 0>{}, j);

  __syncthreads();
  float* red = reinterpret_cast<float*>(sS);   // stages / result tile dead (launch sizes LDS for it)
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    *reinterpret_cast<f32x4*>(red + (r0 * 2 + q) * BN + c8 * 8) = f32x4{sm[q][0], sm[q][1], sm[q][2], sm[q][3]};
    *reinterpret_cast<f32x4*>(red + (r0 * 2 + q) * BN + c8 * 8 + 4) = f32x4{sm[q][4], sm[q][5], sm[q][6], sm[q][7]};
  }
  __syncthreads();
  for (int i = tid; i < 2 * BN; i += NTHR) {
    const int q = i / BN, c = i - q * BN;
    float t = 0.f;
    for (int r = 0; r < RPP; ++r) t += red[(r * 2 + q) * BN + c];
    p.stats[(size_t)grp * 2 * p.gn + q * p.gn + n0 + c] = t;
  }
}

// eligible (called for a training FWD, i.e. with statistics): a 1x1 stride-1 conv expanding K = 64 /
// 128 / 256 channels into more outputs (a 128-multiple), no bias / residual / activation
static bool use_fwd_stream(const IgemmParams& p) {
  if (!kn_fwd_stream.get() || p.bias || p.resid || p.relu) return false;
  if (p.R != 1 || p.S != 1 || p.stride != 1 || p.pad != 0) return false;
  // (K = 256, the layer-3 conv3, measured 48 -> 54 us on the stream: the one-tile kernel keeps it)
  if (!(p.gk == 64 || p.gk == 128) || p.gk >= p.gn || p.gn % 128 || p.gm % 32) return false;
  return (int64_t)p.gm * p.gn * 2 < (1ll << 31);
}
static int fwd_stream_bn(const IgemmParams& p) { return (p.gk == 64 && p.gn % 256 == 0) ? 256 : 128; }
static int fwd_stream_groups(const IgemmParams& p) {
  const int ntn = p.gn / fwd_stream_bn(p);
  return std::max(1, std::min(p.gm / 32, std::max(1, kn_fwd_stream_wgs.get() / ntn)));
}

template <int BN, int GK, bool FOLD>
static void launch_fwd_stream_cfg(IgemmParams& p, hipStream_t st) {
  constexpr int BM = 32;
  const int ntn = p.gn / BN;
  const int groups = fwd_stream_groups(p);
  TORCH_CHECK(p.stats && p.stats_cap >= groups, "fwd_stream: partial-stats buffer");
  constexpr size_t body = (size_t)2 * BM * GK * 2 + (size_t)BM * (BN + 8) * 4 + (FOLD ? 2 * GK * 4 : 0);
  constexpr size_t red = (size_t)(256 / (BN / 8)) * 2 * BN * 4;
  constexpr size_t smem = (size_t)BN * GK * 2 + std::max(body, red);
  static_assert(smem <= 160 * 1024, "fwd_stream: LDS");
  auto kf = &fwd_stream_kernel<BN, GK, FOLD>;
  static bool attr = false;
  if (!attr) {
    PCMP_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(kf), hipFuncAttributeMaxDynamicSharedMemorySize,
                                       160 * 1024));
    attr = true;
  }
  hipLaunchKernelGGL(kf, dim3(groups * ntn), dim3(256), smem, st, p, groups);
  PCMP_LAUNCH_CHECK();
}

static void launch_fwd_stream(IgemmParams& p, hipStream_t st) {
  const bool fold = p.act_sc != nullptr;
  if (fwd_stream_bn(p) == 256) {
    if (fold) launch_fwd_stream_cfg<256, 64, true>(p, st); else launch_fwd_stream_cfg<256, 64, false>(p, st);
  } else if (p.gk == 64) {
    if (fold) launch_fwd_stream_cfg<128, 64, true>(p, st); else launch_fwd_stream_cfg<128, 64, false>(p, st);
  } else {
    if (fold) launch_fwd_stream_cfg<128, 128, true>(p, st); else launch_fwd_stream_cfg<128, 128, false>(p, st);
  }
}

}  // namespace pcmp

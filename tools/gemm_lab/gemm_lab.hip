// GEMM main-loop lab (standalone, no torch): C[M,N] = A[M,K] . B[N,K]^T, bf16 in, fp32 accumulate.
// Variants of the LDS-DMA MFMA main loop are timed on uniform random [-1,1) operands
// (cdna_hip_programming.md §5.4 rule 25), interleaved over rounds in one process (rule 24), and
// checked against a plain fp32 reference kernel.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/gemm_lab/gemm_lab.hip -o tools/gemm_lab/gemm_lab
// Run:   tools/gemm_lab/gemm_lab [rounds]
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                           \
  do {                                                                                  \
    hipError_t e_ = (x);                                                                \
    if (e_ != hipSuccess) {                                                             \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                          \
    }                                                                                   \
  } while (0)

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
constexpr int BK = 64;
constexpr unsigned kOOB = 0x80000000u;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
}
// [rows][64] bf16 image, 128-B rows, 16-B chunk c of row r at position c ^ (r & 7)
__device__ __forceinline__ int rr_off(int row, int chunk) { return row * 128 + ((chunk ^ (row & 7)) << 4); }
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  if (nwg <= 8) return bid;
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  const int base = (xcd < r) ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + (bid >> 3);
}
// s_waitcnt through the builtin (gfx9 simm16: vmcnt[3:0] + vmcnt_hi[15:14], expcnt[6:4],
// lgkmcnt[11:8]), not inline asm: the compiler's waitcnt pass sees a builtin wait and does not add
// its own conservative lgkmcnt waits behind it (an asm wait is opaque to it)
template <int N>
__device__ __forceinline__ void wait_vm() {
  static_assert(N >= 0 && N < 64, "vmcnt");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | (7 << 4) | (15 << 8));
}
__device__ __forceinline__ void wait_lgkm0() { __builtin_amdgcn_s_waitcnt(15 | (3 << 14) | (7 << 4)); }
__device__ __forceinline__ void lds_sync() {
  wait_lgkm0();
  __builtin_amdgcn_s_barrier();
}
__device__ __forceinline__ unsigned short f2bf(float f) {
  unsigned u = __builtin_bit_cast(unsigned, f);
  return (unsigned short)((u + 0x7FFFu + ((u >> 16) & 1u)) >> 16);
}
__device__ __forceinline__ float bf2f(__bf16 v) { return (float)v; }

// V1: one block per CU, WM x WN waves, 2 LDS stages, fragments double-buffered over the two
// 32-deep halves of each 64-deep K-tile, ONE barrier per K-tile; the DMA of tile t+2 is issued
// right after the barrier that retires the reads of tile t.
template <int BM, int BN, int WM, int WN, bool INPLACE_B = false>
__global__ void __launch_bounds__(WM * WN * 64, 1) gemm_v1(const __bf16* __restrict__ A, const __bf16* __restrict__ B,
                                                         __bf16* __restrict__ C, int M, int N, int K, unsigned a_bytes,
                                                         unsigned b_bytes) {
  constexpr int NW = WM * WN;
  constexpr int WTM = BM / WM, WTN = BN / WN, TM = WTM / 16, TN = WTN / 16;
  constexpr int A_BYTES = BM * BK * 2, STAGE = (BM + BN) * BK * 2;
  constexpr int NA = BM / 8 / NW, NB = BN / 8 / NW;
  static_assert(NA * 8 * NW == BM && NB * 8 * NW == BN, "loader");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid / WN, wc = wid % WN;
  const int tiles_n = (N + BN - 1) / BN;
  const int lin = xcd_remap(blockIdx.x, gridDim.x);
  const int tile_m = lin / tiles_n, tile_n = lin % tiles_n;
  const int m0 = tile_m * BM, n0 = tile_n * BN;
  const int nk = K / BK;
  const __amdgpu_buffer_rsrc_t rsA = make_rsrc(A, a_bytes), rsB = make_rsrc(B, b_bytes);
  const int gch = (lane & 7) ^ (lane >> 3);
  unsigned a_vo[NA], b_vo[NB];
  int a_l[NA], b_l[NB];
#pragma unroll
  for (int i = 0; i < NA; ++i) {
    const int r0 = wid * 8 * NA + i * 8;
    a_l[i] = r0 * 128;
    const int m = m0 + r0 + (lane >> 3);
    a_vo[i] = m < M ? (unsigned)(m * K + gch * 8) * 2u : kOOB;
  }
#pragma unroll
  for (int i = 0; i < NB; ++i) {
    const int r0 = wid * 8 * NB + i * 8;
    b_l[i] = A_BYTES + r0 * 128;
    const int n = n0 + r0 + (lane >> 3);
    b_vo[i] = n < N ? (unsigned)(n * K + gch * 8) * 2u : kOOB;
  }
  auto issue = [&](int s, int k0) {
#pragma unroll
    for (int i = 0; i < NA; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsA, (__attribute__((address_space(3))) void*)(smem + s * STAGE + a_l[i]), 16,
                                               (int)(a_vo[i] + k0 * 2), 0, 0, 0);
#pragma unroll
    for (int i = 0; i < NB; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsB, (__attribute__((address_space(3))) void*)(smem + s * STAGE + b_l[i]), 16,
                                               (int)(b_vo[i] + k0 * 2), 0, 0, 0);
  };
  f32x4 acc[TN][TM];
#pragma unroll
  for (int j = 0; j < TN; ++j)
#pragma unroll
    for (int i = 0; i < TM; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 fa0[TM], fb0[TN], fa1[TM], fb1[TN];
  auto rd = [&](bf16x8(&fa)[TM], bf16x8(&fb)[TN], int kk, int s) {
    const char* sA = smem + s * STAGE;
    const char* sB = sA + A_BYTES;
#pragma unroll
    for (int i = 0; i < TM; ++i)
      fa[i] = *reinterpret_cast<const bf16x8*>(sA + rr_off(wr * WTM + i * 16 + (lane & 15), kk * 4 + (lane >> 4)));
#pragma unroll
    for (int j = 0; j < TN; ++j)
      fb[j] = *reinterpret_cast<const bf16x8*>(sB + rr_off(wc * WTN + j * 16 + (lane & 15), kk * 4 + (lane >> 4)));
  };
  auto mma = [&](bf16x8(&fa)[TM], bf16x8(&fb)[TN]) {
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int i = 0; i < TM; ++i) acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[j], fa[i], acc[j][i], 0, 0, 0);
  };

  issue(0, 0);
  if (nk > 1) {
    issue(1, BK);
    wait_vm<NA + NB>();
  } else {
    wait_vm<0>();
  }
  lds_sync();
  if constexpr (!INPLACE_B) {
    rd(fa0, fb0, 0, 0);
    for (int t = 0; t < nk; ++t) {
      const int s = t & 1;
      rd(fa1, fb1, 1, s);
      mma(fa0, fb0);
      if (t + 1 < nk) wait_vm<0>();
      lds_sync();   // every wave's reads of stage s retired; stage t+1 landed for every wave
      if (t + 2 < nk) issue(s, (t + 2) * BK);
      if (t + 1 < nk) rd(fa0, fb0, 0, s ^ 1);
      mma(fa1, fb1);
    }
  } else {
    // B fragments reloaded in place column by column (96 fragment VGPRs instead of 128)
    auto rd_a = [&](bf16x8(&fa)[TM], int kk, int s) {
      const char* sA = smem + s * STAGE;
#pragma unroll
      for (int i = 0; i < TM; ++i)
        fa[i] = *reinterpret_cast<const bf16x8*>(sA + rr_off(wr * WTM + i * 16 + (lane & 15), kk * 4 + (lane >> 4)));
    };
    auto rd_b1 = [&](int j, int kk, int s) {
      return *reinterpret_cast<const bf16x8*>(smem + s * STAGE + A_BYTES +
                                             rr_off(wc * WTN + j * 16 + (lane & 15), kk * 4 + (lane >> 4)));
    };
    rd_a(fa0, 0, 0);
#pragma unroll
    for (int j = 0; j < TN; ++j) fb0[j] = rd_b1(j, 0, 0);
    for (int t = 0; t < nk; ++t) {
      const int s = t & 1;
      rd_a(fa1, 1, s);
#pragma unroll
      for (int j = 0; j < TN; ++j) {
#pragma unroll
        for (int i = 0; i < TM; ++i) acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb0[j], fa0[i], acc[j][i], 0, 0, 0);
        fb0[j] = rd_b1(j, 1, s);
      }
      if (t + 1 < nk) wait_vm<0>();
      lds_sync();
      if (t + 2 < nk) issue(s, (t + 2) * BK);
      const bool nx = t + 1 < nk;
      if (nx) rd_a(fa0, 0, s ^ 1);
#pragma unroll
      for (int j = 0; j < TN; ++j) {
#pragma unroll
        for (int i = 0; i < TM; ++i) acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb0[j], fa1[i], acc[j][i], 0, 0, 0);
        if (nx) fb0[j] = rd_b1(j, 0, s ^ 1);
      }
    }
  }
  // epilogue: lane holds C[m][n..n+3] of each fragment
#pragma unroll
  for (int j = 0; j < TN; ++j)
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int m = m0 + wr * WTM + i * 16 + (lane & 15);
      const int n = n0 + wc * WTN + j * 16 + (lane >> 4) * 4;
      if (m < M && n < N) {
        const f32x4 v = acc[j][i];
        uint2 w;
        w.x = f2bf(v[0]) | ((unsigned)f2bf(v[1]) << 16);
        w.y = f2bf(v[2]) | ((unsigned)f2bf(v[3]) << 16);
        *reinterpret_cast<uint2*>(C + (size_t)m * N + n) = w;
      }
    }
}


// V3: V1's loop made branch-free (DMA / fragment reads of the last iterations point out of range or
// at dead stages) so each half is one scheduling region, and sched_group_barrier interleaves the
// LDS-DMA issues and ds_reads between the MFMAs: half 0 = 16 x {1 DS_READ, 4 MFMA}, half 1 =
// 16 x {1 VMEM, 1 DS_READ, 4 MFMA} (the DMA issue cost no longer stalls one wave per SIMD).
template <int BM, int BN, int WM, int WN, int SG>
__global__ void __launch_bounds__(WM * WN * 64, 1) gemm_v3(const __bf16* __restrict__ A, const __bf16* __restrict__ B,
                                                         __bf16* __restrict__ C, int M, int N, int K, unsigned a_bytes,
                                                         unsigned b_bytes) {
  constexpr int NW = WM * WN;
  constexpr int WTM = BM / WM, WTN = BN / WN, TM = WTM / 16, TN = WTN / 16;
  constexpr int A_BYTES = BM * BK * 2, STAGE = (BM + BN) * BK * 2;
  constexpr int NA = BM / 8 / NW, NB = BN / 8 / NW;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid / WN, wc = wid % WN;
  const int tiles_n = (N + BN - 1) / BN;
  const int lin = xcd_remap(blockIdx.x, gridDim.x);
  const int tile_m = lin / tiles_n, tile_n = lin % tiles_n;
  const int m0 = tile_m * BM, n0 = tile_n * BN;
  const int nk = K / BK;
  const __amdgpu_buffer_rsrc_t rsA = make_rsrc(A, a_bytes), rsB = make_rsrc(B, b_bytes);
  const int gch = (lane & 7) ^ (lane >> 3);
  unsigned a_vo[NA], b_vo[NB];
#pragma unroll
  for (int i = 0; i < NA; ++i) {
    const int m = m0 + (wid * NA + i) * 8 + (lane >> 3);
    a_vo[i] = m < M ? (unsigned)(m * K + gch * 8) * 2u : kOOB;
  }
#pragma unroll
  for (int i = 0; i < NB; ++i) {
    const int n = n0 + (wid * NB + i) * 8 + (lane >> 3);
    b_vo[i] = n < N ? (unsigned)(n * K + gch * 8) * 2u : kOOB;
  }
  auto issue = [&](int s, int k0, bool live) {
#pragma unroll
    for (int i = 0; i < NA; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsA, (__attribute__((address_space(3))) void*)(smem + s * STAGE + (wid * NA + i) * 1024), 16,
                                               (int)(live ? a_vo[i] + k0 * 2 : kOOB), 0, 0, 0);
#pragma unroll
    for (int i = 0; i < NB; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsB, (__attribute__((address_space(3))) void*)(smem + s * STAGE + A_BYTES + (wid * NB + i) * 1024), 16,
                                               (int)(live ? b_vo[i] + k0 * 2 : kOOB), 0, 0, 0);
  };
  f32x4 acc[TN][TM];
#pragma unroll
  for (int j = 0; j < TN; ++j)
#pragma unroll
    for (int i = 0; i < TM; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 fa0[TM], fb0[TN], fa1[TM], fb1[TN];
  auto rd = [&](bf16x8(&fa)[TM], bf16x8(&fb)[TN], int kk, int s) {
    const char* sA = smem + s * STAGE;
    const char* sB = sA + A_BYTES;
#pragma unroll
    for (int i = 0; i < TM; ++i)
      fa[i] = *reinterpret_cast<const bf16x8*>(sA + rr_off(wr * WTM + i * 16 + (lane & 15), kk * 4 + (lane >> 4)));
#pragma unroll
    for (int j = 0; j < TN; ++j)
      fb[j] = *reinterpret_cast<const bf16x8*>(sB + rr_off(wc * WTN + j * 16 + (lane & 15), kk * 4 + (lane >> 4)));
  };
  auto mma = [&](bf16x8(&fa)[TM], bf16x8(&fb)[TN]) {
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int i = 0; i < TM; ++i) acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[j], fa[i], acc[j][i], 0, 0, 0);
  };
  constexpr int NMF = TM * TN, NDS = TM + TN, NVM = NA + NB;
  issue(0, 0, true);
  issue(1, BK, nk > 1);
  wait_vm<NA + NB>();
  lds_sync();
  rd(fa0, fb0, 0, 0);
  for (int t = 0; t < nk; ++t) {
    const int s = t & 1;
    rd(fa1, fb1, 1, s);
    mma(fa0, fb0);
    if constexpr (SG) {
#pragma unroll
      for (int g = 0; g < NDS; ++g) {
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x8, NMF / NDS, 0);
      }
    }
    if constexpr (SG >= 2) __builtin_amdgcn_sched_barrier(0);
    wait_vm<0>();
    lds_sync();
    if constexpr (SG >= 2) __builtin_amdgcn_sched_barrier(0);
    issue(s, (t + 2) * BK, t + 2 < nk);
    rd(fa0, fb0, 0, s ^ 1);
    mma(fa1, fb1);
    if constexpr (SG) {
#pragma unroll
      for (int g = 0; g < NDS; ++g) {
        if (g < NVM) __builtin_amdgcn_sched_group_barrier(0x10, 1, 1);
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 1);
        __builtin_amdgcn_sched_group_barrier(0x8, NMF / NDS, 1);
      }
    }
    if constexpr (SG >= 2) __builtin_amdgcn_sched_barrier(0);
  }
  wait_vm<0>();
#pragma unroll
  for (int j = 0; j < TN; ++j)
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int m = m0 + wr * WTM + i * 16 + (lane & 15);
      const int n = n0 + wc * WTN + j * 16 + (lane >> 4) * 4;
      if (m < M && n < N) {
        const f32x4 v = acc[j][i];
        uint2 w;
        w.x = f2bf(v[0]) | ((unsigned)f2bf(v[1]) << 16);
        w.y = f2bf(v[2]) | ((unsigned)f2bf(v[3]) << 16);
        *reinterpret_cast<uint2*>(C + (size_t)m * N + n) = w;
      }
    }
}

// V4: V3 (fenced halves, one barrier per K-tile) on v_mfma_f32_32x32x16_bf16: 32x32 output tiles,
// K = 16 per instruction (lane: row / column lane & 31, k-group (lane >> 5) * 8), half as many MFMA
// instructions as 16x16x32 for the same wave tile and the same ds_read bytes.
typedef float f32x16 __attribute__((ext_vector_type(16)));
template <int BM, int BN, int WM, int WN>
__global__ void __launch_bounds__(WM * WN * 64, 1) gemm_v4(const __bf16* __restrict__ A, const __bf16* __restrict__ B,
                                                         __bf16* __restrict__ C, int M, int N, int K, unsigned a_bytes,
                                                         unsigned b_bytes) {
  constexpr int NW = WM * WN;
  constexpr int WTM = BM / WM, WTN = BN / WN, TM = WTM / 32, TN = WTN / 32;
  constexpr int A_BYTES = BM * BK * 2, STAGE = (BM + BN) * BK * 2;
  constexpr int NA = BM / 8 / NW, NB = BN / 8 / NW;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid / WN, wc = wid % WN;
  const int tiles_n = (N + BN - 1) / BN;
  const int lin = xcd_remap(blockIdx.x, gridDim.x);
  const int tile_m = lin / tiles_n, tile_n = lin % tiles_n;
  const int m0 = tile_m * BM, n0 = tile_n * BN;
  const int nk = K / BK;
  const __amdgpu_buffer_rsrc_t rsA = make_rsrc(A, a_bytes), rsB = make_rsrc(B, b_bytes);
  const int gch = (lane & 7) ^ (lane >> 3);
  unsigned a_vo[NA], b_vo[NB];
#pragma unroll
  for (int i = 0; i < NA; ++i) {
    const int m = m0 + (wid * NA + i) * 8 + (lane >> 3);
    a_vo[i] = m < M ? (unsigned)(m * K + gch * 8) * 2u : kOOB;
  }
#pragma unroll
  for (int i = 0; i < NB; ++i) {
    const int n = n0 + (wid * NB + i) * 8 + (lane >> 3);
    b_vo[i] = n < N ? (unsigned)(n * K + gch * 8) * 2u : kOOB;
  }
  auto issue = [&](int s, int k0, bool live) {
#pragma unroll
    for (int i = 0; i < NA; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsA, (__attribute__((address_space(3))) void*)(smem + s * STAGE + (wid * NA + i) * 1024), 16,
                                               (int)(live ? a_vo[i] + k0 * 2 : kOOB), 0, 0, 0);
#pragma unroll
    for (int i = 0; i < NB; ++i)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsB, (__attribute__((address_space(3))) void*)(smem + s * STAGE + A_BYTES + (wid * NB + i) * 1024), 16,
                                               (int)(live ? b_vo[i] + k0 * 2 : kOOB), 0, 0, 0);
  };
  f32x16 acc[TN][TM];
#pragma unroll
  for (int j = 0; j < TN; ++j)
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[j][i][r] = 0.f;
  // a half = 32 of the tile's 64 K = two 16-deep MFMA steps; fragments of both steps read together
  bf16x8 fa0[2][TM], fb0[2][TN], fa1[2][TM], fb1[2][TN];
  auto rd = [&](bf16x8(&fa)[2][TM], bf16x8(&fb)[2][TN], int half, int s) {
    const char* sA = smem + s * STAGE;
    const char* sB = sA + A_BYTES;
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int ch = half * 4 + q * 2 + (lane >> 5);   // 16-B chunk (8 k) of this lane's k-group
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
  issue(0, 0, true);
  issue(1, BK, nk > 1);
  wait_vm<NA + NB>();
  lds_sync();
  rd(fa0, fb0, 0, 0);
  for (int t = 0; t < nk; ++t) {
    const int s = t & 1;
    rd(fa1, fb1, 1, s);
    mma(fa0, fb0);
#pragma unroll
    for (int g = 0; g < NDS; ++g) {
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      if (g % (NDS / NMF > 0 ? NDS / NMF : 1) == 0) __builtin_amdgcn_sched_group_barrier(0x8, NMF >= NDS ? NMF / NDS : 1, 0);
    }
    __builtin_amdgcn_sched_barrier(0);
    wait_vm<0>();
    lds_sync();
    __builtin_amdgcn_sched_barrier(0);
    issue(s, (t + 2) * BK, t + 2 < nk);
    rd(fa0, fb0, 0, s ^ 1);
    mma(fa1, fb1);
#pragma unroll
    for (int g = 0; g < NDS; ++g) {
      if (g < NVM) __builtin_amdgcn_sched_group_barrier(0x10, 1, 1);
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 1);
      if (g % (NDS / NMF > 0 ? NDS / NMF : 1) == 0) __builtin_amdgcn_sched_group_barrier(0x8, NMF >= NDS ? NMF / NDS : 1, 1);
    }
    __builtin_amdgcn_sched_barrier(0);
  }
  wait_vm<0>();
  // 32x32 accumulator: register r of lane l holds C[row][col], col = l & 31,
  // row = 8 * (r / 4) + 4 * (l >> 5) + (r % 4); here the MFMA ran B (rows = n) x A (cols = m)
#pragma unroll
  for (int j = 0; j < TN; ++j)
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int m = m0 + wr * WTM + i * 32 + (lane & 31);
#pragma unroll
      for (int r4 = 0; r4 < 4; ++r4) {
        const int n = n0 + wc * WTN + j * 32 + 8 * r4 + 4 * (lane >> 5);
        if (m < M && n < N) {
          uint2 w;
          w.x = f2bf(acc[j][i][4 * r4]) | ((unsigned)f2bf(acc[j][i][4 * r4 + 1]) << 16);
          w.y = f2bf(acc[j][i][4 * r4 + 2]) | ((unsigned)f2bf(acc[j][i][4 * r4 + 3]) << 16);
          *reinterpret_cast<uint2*>(C + (size_t)m * N + n) = w;
        }
      }
    }
}

__global__ void ref_gemm(const __bf16* A, const __bf16* B, float* C, int M, int N, int K) {
  const int n = blockIdx.x * blockDim.x + threadIdx.x, m = blockIdx.y;
  if (n >= N) return;
  float s = 0.f;
  for (int k = 0; k < K; ++k) s += bf2f(A[(size_t)m * K + k]) * bf2f(B[(size_t)n * K + k]);
  C[(size_t)m * N + n] = s;
}

__global__ void fill_rand(__bf16* p, size_t n, unsigned seed) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    unsigned x = (unsigned)i * 2654435761u ^ seed;
    x ^= x >> 13; x *= 0x5bd1e995u; x ^= x >> 15;
    p[i] = (__bf16)((x & 0xFFFFFF) / 8388608.0f - 1.0f);
  }
}

struct Variant {
  const char* name;
  void (*launch)(const __bf16*, const __bf16*, __bf16*, int, int, int, hipStream_t);
  int bm, bn;
};

template <int BM, int BN, int WM, int WN, bool IB = false>
void launch_v1(const __bf16* A, const __bf16* B, __bf16* C, int M, int N, int K, hipStream_t st) {
  static bool attr = false;
  constexpr size_t smem = 2 * (BM + BN) * BK * 2;
  auto kfn = &gemm_v1<BM, BN, WM, WN, IB>;
  if (!attr) {
    CK(hipFuncSetAttribute(reinterpret_cast<const void*>(kfn), hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    attr = true;
  }
  const int grid = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  hipLaunchKernelGGL(kfn, dim3(grid), dim3(WM * WN * 64), smem, st, A, B, C, M, N, K,
                     (unsigned)((size_t)M * K * 2), (unsigned)((size_t)N * K * 2));
}


template <int BM, int BN, int WM, int WN, int SG>
void launch_v3(const __bf16* A, const __bf16* B, __bf16* C, int M, int N, int K, hipStream_t st) {
  static bool attr = false;
  constexpr size_t smem = 2 * (BM + BN) * BK * 2;
  auto kfn = &gemm_v3<BM, BN, WM, WN, SG>;
  if (!attr) {
    CK(hipFuncSetAttribute(reinterpret_cast<const void*>(kfn), hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    attr = true;
  }
  const int grid = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  hipLaunchKernelGGL(kfn, dim3(grid), dim3(WM * WN * 64), smem, st, A, B, C, M, N, K,
                     (unsigned)((size_t)M * K * 2), (unsigned)((size_t)N * K * 2));
}

template <int BM, int BN, int WM, int WN>
void launch_v4(const __bf16* A, const __bf16* B, __bf16* C, int M, int N, int K, hipStream_t st) {
  static bool attr = false;
  constexpr size_t smem = 2 * (BM + BN) * BK * 2;
  auto kfn = &gemm_v4<BM, BN, WM, WN>;
  if (!attr) {
    CK(hipFuncSetAttribute(reinterpret_cast<const void*>(kfn), hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    attr = true;
  }
  const int grid = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  hipLaunchKernelGGL(kfn, dim3(grid), dim3(WM * WN * 64), smem, st, A, B, C, M, N, K,
                     (unsigned)((size_t)M * K * 2), (unsigned)((size_t)N * K * 2));
}

int main(int argc, char** argv) {
  const int rounds = argc > 1 ? atoi(argv[1]) : 3;
  std::vector<Variant> vars = {
      {"v3f_256x256_w8", launch_v3<256, 256, 2, 4, 2>, 256, 256},
      {"v4_256x256_w8", launch_v4<256, 256, 2, 4>, 256, 256},
      {"v3f_256x256_w4", launch_v3<256, 256, 2, 2, 2>, 256, 256},
      {"v4_256x256_w4", launch_v4<256, 256, 2, 2>, 256, 256},
      {"v3f_128x128_w4", launch_v3<128, 128, 2, 2, 2>, 128, 128},
      {"v4_128x128_w4", launch_v4<128, 128, 2, 2>, 128, 128},
  };
  struct Shape { int M, N, K; };
  std::vector<Shape> shapes = {{4096, 4096, 4096}, {8192, 8192, 8192}, {50176, 256, 2304}, {12544, 512, 4608},
                               {200704, 128, 1152}, {4096, 3072, 768}, {4096, 768, 3072}};
  hipStream_t st;
  CK(hipStreamCreate(&st));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (const Shape& sh : shapes) {
    const int M = sh.M, N = sh.N, K = sh.K;
    __bf16 *A, *B, *C;
    float* R;
    CK(hipMalloc(&A, (size_t)M * K * 2));
    CK(hipMalloc(&B, (size_t)N * K * 2));
    CK(hipMalloc(&C, (size_t)M * N * 2));
    CK(hipMalloc(&R, (size_t)M * N * 4));
    hipLaunchKernelGGL(fill_rand, dim3(2048), dim3(256), 0, st, A, (size_t)M * K, 1u);
    hipLaunchKernelGGL(fill_rand, dim3(2048), dim3(256), 0, st, B, (size_t)N * K, 7u);
    hipLaunchKernelGGL(ref_gemm, dim3((N + 255) / 256, M), dim3(256), 0, st, A, B, R, M, N, K);
    std::vector<float> ref((size_t)M * N);
    std::vector<unsigned short> out((size_t)M * N);
    CK(hipMemcpy(ref.data(), R, ref.size() * 4, hipMemcpyDeviceToHost));
    const double fl = 2.0 * M * N * K;
    std::vector<double> best(vars.size(), 1e30);
    std::vector<double> err(vars.size(), 0);
    for (size_t v = 0; v < vars.size(); ++v) {
      if (K % BK) continue;
      CK(hipMemset(C, 0xFF, (size_t)M * N * 2));
      vars[v].launch(A, B, C, M, N, K, st);
      CK(hipStreamSynchronize(st));
      CK(hipMemcpy(out.data(), C, out.size() * 2, hipMemcpyDeviceToHost));
      double mx = 0, rm = 0;
      for (size_t i = 0; i < out.size(); ++i) {
        unsigned u = (unsigned)out[i] << 16;
        float f;
        std::memcpy(&f, &u, 4);
        mx = std::max(mx, (double)std::fabs(f - ref[i]));
        rm = std::max(rm, (double)std::fabs(ref[i]));
        if (!(f == f)) mx = 1e30;
      }
      err[v] = mx / rm;
    }
    for (int r = 0; r < rounds; ++r)
      for (size_t v = 0; v < vars.size(); ++v) {
        const int it = 10;
        vars[v].launch(A, B, C, M, N, K, st);
        CK(hipEventRecord(e0, st));
        for (int i = 0; i < it; ++i) vars[v].launch(A, B, C, M, N, K, st);
        CK(hipEventRecord(e1, st));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        best[v] = std::min(best[v], ms * 1e3 / it);
      }
    for (size_t v = 0; v < vars.size(); ++v)
      printf("%6d x %5d x %5d  %-16s %8.1f us %6.0f TF  relerr %.2e\n", M, N, K, vars[v].name, best[v],
             fl / best[v] / 1e6, err[v]);
    fflush(stdout);
    CK(hipFree(A)); CK(hipFree(B)); CK(hipFree(C)); CK(hipFree(R));
  }
  return 0;
}

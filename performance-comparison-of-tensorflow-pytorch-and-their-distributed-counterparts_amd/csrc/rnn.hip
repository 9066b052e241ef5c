// BiLSTM text-classifier kernels: embedding gather / scatter-add, masked mean pooling and a
// persistent bidirectional LSTM recurrence (forward and backward-through-time).
//
// North-star text path (BASELINE.json config 5): token ids [B,128] (vocab 30522,
// id 0 = padding, mask = id > 0 exactly as pytorch_on_language_distr.py:84-103 builds it),
// embedding -> BiLSTM layers -> masked mean pool -> Linear -> CE.
//
// Recurrence design (MI355X): the input projection x_t W_ih^T for all t and both directions is
// ONE MFMA GEMM outside the recurrence (igemm linear).  The recurrence h_{t-1} W_hh^T runs in ONE
// persistent launch per layer: each workgroup owns J=16 hidden units of one direction and keeps
// its 4J x H slice of W_hh resident in LDS for all 128 timesteps; per step it reads h_{t-1} of
// its direction (16 KB), does the 32x64x256 product on MFMA, applies the fused gate
// nonlinearities + cell update and publishes its h_t slice.  Workgroups of a direction meet once
// per step at an agent-scope counter barrier (cdna_hip_programming.md §6 Guideline 16: producer
// vmcnt(0) -> barrier -> release fence -> vmcnt(0) -> relaxed atomic; consumer relaxed poll ->
// acquire fence -> vmcnt(0) -> barrier).  2*H/J = 32 workgroups are trivially co-resident on
// 256 CUs; every spin is bounded and a timeout sets an error word instead of hanging.
//
// Masking = packed-sequence semantics: at a padded step (mask 0) the state is carried unchanged
// (h_t = h_{t-1}, c_t = c_{t-1}); the reverse direction therefore starts at the last real token.
// Backward: the same layout in reverse time computes dgates and dh_rec = dgates W_hh
// (workgroup j owns columns j of dh_rec and the W_hh[:, j] slice); weight gradients are then
// plain MFMA GEMMs over all timesteps (igemm wgrad), outside the recurrence.
#include "common.h"
#include "embed.h"
#include "f32.h"

namespace pcmp {

// ------------------------------------------------------------------------------- embedding
// out[r][:] = W[ids[r]][:]   (W bf16 [V][E], E % 8 == 0)
__global__ void embedding_fwd_kernel(const int64_t* __restrict__ ids, const __bf16* __restrict__ W,
                                     __bf16* __restrict__ out, int64_t rows, int E) {
  const int EV = E / 8;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < rows * EV;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / EV;
    const int v = i % EV;
    const int64_t id = ids[r];
    reinterpret_cast<uint4*>(out)[i] = reinterpret_cast<const uint4*>(W + id * E)[v];
  }
}

// dW[ids[r]][:] += dy[r][:]  (fp32 atomics; rows with id == padding_idx skipped)
__global__ void embedding_bwd_kernel(const int64_t* __restrict__ ids, const __bf16* __restrict__ dy,
                                     float* __restrict__ dW, int64_t rows, int E, int64_t padding_idx) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < rows * E;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / E;
    const int e = i % E;
    const int64_t id = ids[r];
    if (id == padding_idx) continue;
    atomicAdd(dW + id * E + e, bf2f(reinterpret_cast<const unsigned short*>(dy)[i]));
  }
}

Knob kn_emb_atomic("emb_atomic", 0);

// ------------------------------------------------------------------------------- masked mean
// x [B][S][D] bf16, mask [B][S] (int64 ids > 0 or bool/uint8) -> y [B][D] bf16 = mean over valid t
__global__ void masked_mean_fwd_kernel(const __bf16* __restrict__ x, const int64_t* __restrict__ ids, int B, int S,
                                       int D, __bf16* __restrict__ y) {
  const int b = blockIdx.x;
  __shared__ float cnt_sh;
  if (threadIdx.x == 0) {
    int c = 0;
    for (int t = 0; t < S; ++t) c += ids[(size_t)b * S + t] > 0;
    cnt_sh = (float)max(c, 1);
  }
  __syncthreads();
  const float inv = 1.f / cnt_sh;
  for (int d = threadIdx.x; d < D; d += blockDim.x) {
    float s = 0.f;
    for (int t = 0; t < S; ++t)
      if (ids[(size_t)b * S + t] > 0) s += bf2f(reinterpret_cast<const unsigned short*>(x)[((size_t)b * S + t) * D + d]);
    reinterpret_cast<unsigned short*>(y)[(size_t)b * D + d] = f2bf(s * inv);
  }
}

__global__ void masked_mean_bwd_kernel(const __bf16* __restrict__ dy, const int64_t* __restrict__ ids, int B, int S,
                                       int D, __bf16* __restrict__ dx) {
  const int b = blockIdx.x;
  __shared__ float cnt_sh;
  if (threadIdx.x == 0) {
    int c = 0;
    for (int t = 0; t < S; ++t) c += ids[(size_t)b * S + t] > 0;
    cnt_sh = (float)max(c, 1);
  }
  __syncthreads();
  const float inv = 1.f / cnt_sh;
  for (int i = threadIdx.x; i < S * D; i += blockDim.x) {
    const int t = i / D, d = i % D;
    const float g = ids[(size_t)b * S + t] > 0 ? bf2f(reinterpret_cast<const unsigned short*>(dy)[(size_t)b * D + d]) * inv : 0.f;
    reinterpret_cast<unsigned short*>(dx)[((size_t)b * S + t) * D + d] = f2bf(g);
  }
}

// ------------------------------------------------------------------------------- LSTM
constexpr int LJ = 16;         // hidden units per workgroup
constexpr int LB = 32;         // batch rows handled per launch (B must be <= 32; host tiles larger B)
constexpr int LT = 256;        // threads
constexpr unsigned kSpinLimit = 1u << 26;

typedef __attribute__((address_space(1))) unsigned gu32;
#define RLX_AGENT __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT

// v_exp_f32 + v_rcp_f32 (1 ulp): a full-precision IEEE division is ~10 dependent instructions, and
// the cell update (3 sigmoids + 2 tanh per unit) sits on the recurrence's per-step critical path
__device__ __forceinline__ float sigm(float x) { return __builtin_amdgcn_rcpf(1.f + __expf(-x)); }
__device__ __forceinline__ float tanh_f(float x) {
  const float e = __expf(-2.f * fabsf(x));
  const float r = (1.f - e) * __builtin_amdgcn_rcpf(1.f + e);
  return copysignf(r, x);
}

// Per-step exchange (cdna_hip_programming.md §6 Guideline 16, recipe R1 with sc1 loads): the
// handed-off tile (h_t / dgates_t) is stored WRITE-THROUGH (16-B buffer stores with aux = sc1) by
// one wave, every wave drains (s_waitcnt vmcnt(0)), the workgroup barrier, then ONE lane adds to the
// direction's arrival counter (relaxed, agent scope); consumers poll that counter relaxed and read
// the tile with sc1 buffer loads ONLY -- so neither a release (L2 write-back of every dirty line,
// including the bulk activations this kernel streams out) nor an acquire (L1 invalidate) is needed
// per step.  Every other load of the kernel reads bytes no workgroup writes in this launch.
typedef unsigned u32x4v __attribute__((ext_vector_type(4)));
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rnn_rsrc(const void* base, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ void st16_sc1(__amdgpu_buffer_rsrc_t r, unsigned off, uint4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(u32x4v{v.x, v.y, v.z, v.w}, r, (int)off, 0, 16);   // aux 16 = sc1
}
__device__ __forceinline__ uint4 ld16_sc1(__amdgpu_buffer_rsrc_t r, unsigned off) {
  const u32x4v v = __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 16);                // aux 16 = sc1
  return uint4{v[0], v[1], v[2], v[3]};
}

// grid barrier among the workgroups of one direction: arrive + wait for `target` arrivals
__device__ __forceinline__ bool dir_barrier(unsigned* counter, unsigned target, unsigned* err, bool drain = true) {
  if (drain) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every wave that stored payload drains
  __syncthreads();
  bool ok = true;
  if (threadIdx.x == 0) {
    __hip_atomic_fetch_add((gu32*)counter, 1u, RLX_AGENT);
    unsigned spins = 0;
    while (__hip_atomic_load((gu32*)counter, RLX_AGENT) < target) {
      __builtin_amdgcn_s_sleep(1);
      if (++spins > kSpinLimit) {
        __hip_atomic_store((gu32*)err, 1u, RLX_AGENT);
        ok = false;
        break;
      }
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");   // compiler ordering only: tile loads are sc1
  __syncthreads();
  return ok;
}

struct LstmFwdParams {
  const __bf16* gx;      // [B][S][2][4H] bf16 input projections (+ both biases), dir-major gates i,f,g,o
  const __bf16* whh;     // [2][4H][H] bf16
  const int64_t* ids;    // [B][S] token ids (mask = id > 0)
  __bf16* hout;          // [B][S][2H] bf16 layer output (dir 0 = cols 0..H-1)
  float* gates;          // [B][S][2][4H] fp32 saved activations (i,f,g,o after nonlinearity)
  float* cst;            // [B][S][2][H] fp32 cell state c_t
  __bf16* hbuf;          // [2][2][LB][H] bf16 ping-pong h exchange buffer
  unsigned* counters;    // [2] per-direction arrival counters (zeroed by host)
  unsigned* err;
  int B, S, H;
  unsigned long long* prof;   // knob lstm_prof: per-phase shader-clock totals of workgroup 0 (else null)
};

// grid = 2 * (H / LJ) workgroups; wg -> (dir = wg / (H/LJ), unit block ub = wg % (H/LJ))
__global__ void __launch_bounds__(LT) lstm_fwd_persistent(const LstmFwdParams p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int H = p.H, nub = H / LJ;
  const int dir = blockIdx.x / nub, ub = blockIdx.x % nub, j0 = ub * LJ;
  // LDS: W slice [4*LJ rows][H] bf16 (row r = gate*LJ + jj), h tile [LB][H] bf16, pre-acts [LB][4LJ] f32
  __bf16* sW = reinterpret_cast<__bf16*>(smem);
  __bf16* sH = sW + 4 * LJ * H;
  float* sG = reinterpret_cast<float*>(sH + LB * H);
  __bf16* sHo = reinterpret_cast<__bf16*>(sG + LB * 4 * LJ);   // [LB][LJ] this workgroup's h_t slice
  const __amdgpu_buffer_rsrc_t rsH = rnn_rsrc(p.hbuf, (unsigned)(4 * LB * H * 2));
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  for (int i = tid; i < 4 * LJ * H / 8; i += LT) {
    const int r = i / (H / 8), c8 = i % (H / 8);
    const int gate = r / LJ, jj = r % LJ;
    reinterpret_cast<uint4*>(sW)[i] =
        reinterpret_cast<const uint4*>(p.whh + ((size_t)dir * 4 * H + gate * H + j0 + jj) * H)[c8];
  }
  // cell state for (b, jj) pairs owned by this thread: 2 pairs per thread (LB*LJ = 512)
  float creg[2] = {0.f, 0.f};
  float hreg[2] = {0.f, 0.f};
  __syncthreads();
  unsigned* cnt = p.counters + dir;
  const int nwg_dir = nub;
  // input projections and masks of the NEXT step are loaded during the current one (they do not
  // depend on the recurrence), so only the h exchange sits on the per-step critical path
  float gxn[2][4];
  bool vn[2];
  auto fetch = [&](int stp) {
    const int tt = dir == 0 ? stp : p.S - 1 - stp;
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int q = tid + LT * k;
      const int b = q / LJ, j = j0 + q % LJ;
      vn[k] = false;
#pragma unroll
      for (int g = 0; g < 4; ++g) gxn[k][g] = 0.f;
      if (b < p.B) {
        vn[k] = p.ids[(size_t)b * p.S + tt] > 0;
        const size_t gb = (((size_t)b * p.S + tt) * 2 + dir) * 4 * H;
#pragma unroll
        for (int g = 0; g < 4; ++g) gxn[k][g] = bf2f(reinterpret_cast<const unsigned short*>(p.gx)[gb + g * H + j]);
      }
    }
  };
  fetch(0);
  for (int step = 0; step < p.S; ++step) {
    const int t = dir == 0 ? step : p.S - 1 - step;
    const int cur = step & 1;
    // ---- load h_{t-1} [LB][H] of this direction into LDS (zeros at step 0)
    if (step == 0) {
      for (int i = tid; i < LB * H / 8; i += LT) reinterpret_cast<uint4*>(sH)[i] = uint4{0, 0, 0, 0};
    } else {
      const unsigned src = (unsigned)(((cur ^ 1) * 2 + dir) * LB * H) * 2u;
      for (int i = tid; i < LB * H / 8; i += LT) reinterpret_cast<uint4*>(sH)[i] = ld16_sc1(rsH, src + i * 16u);
    }
    __syncthreads();
    // ---- pre-activations [LB=32][4LJ=64] = h @ Wslice^T : wave w -> m-tile (w&1), n-tiles 2*(w>>1)+{0,1}
    {
      const int mt = wid & 1;
      f32x4 acc0 = {0, 0, 0, 0}, acc1 = {0, 0, 0, 0};
      for (int k0 = 0; k0 < H; k0 += 32) {
        const int kk = k0 + 8 * (lane >> 4);
        const bf16x8 a = *reinterpret_cast<const bf16x8*>(sH + (mt * 16 + (lane & 15)) * H + kk);
        const int n0 = (2 * (wid >> 1)) * 16 + (lane & 15);
        const bf16x8 b0 = *reinterpret_cast<const bf16x8*>(sW + n0 * H + kk);
        const bf16x8 b1 = *reinterpret_cast<const bf16x8*>(sW + (n0 + 16) * H + kk);
        acc0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b0, acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b1, acc1, 0, 0, 0);
      }
      const int col = (2 * (wid >> 1)) * 16 + (lane & 15);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int row = mt * 16 + (lane >> 4) * 4 + e;
        sG[row * 4 * LJ + col] = acc0[e];
        sG[row * 4 * LJ + col + 16] = acc1[e];
      }
    }
    __syncthreads();
    // ---- cell update for (b, jj): pair q = tid + LT*k
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int q = tid + LT * k;
      const int b = q / LJ, jj = q % LJ, j = j0 + jj;
      float hn = 0.f;
      if (b < p.B) {
        const bool valid = vn[k];
        const size_t gbase = (((size_t)b * p.S + t) * 2 + dir) * 4 * H;
        float pre[4];
#pragma unroll
        for (int g = 0; g < 4; ++g) pre[g] = sG[b * 4 * LJ + g * LJ + jj] + gxn[k][g];
        const float ig = sigm(pre[0]), fg = sigm(pre[1]), gg = tanh_f(pre[2]), og = sigm(pre[3]);
        float cn, hv;
        if (valid) {
          cn = fg * creg[k] + ig * gg;
          hv = og * tanh_f(cn);
        } else {
          cn = creg[k];
          hv = hreg[k];
        }
        creg[k] = cn;
        hreg[k] = hv;
        hn = hv;
        p.gates[gbase + 0 * H + j] = ig;
        p.gates[gbase + 1 * H + j] = fg;
        p.gates[gbase + 2 * H + j] = gg;
        p.gates[gbase + 3 * H + j] = og;
        p.cst[(((size_t)b * p.S + t) * 2 + dir) * H + j] = cn;
        reinterpret_cast<unsigned short*>(p.hout)[((size_t)b * p.S + t) * 2 * H + dir * H + j] = f2bf(hv);
      }
      reinterpret_cast<unsigned short*>(sHo)[b * LJ + jj] = f2bf(hn);
    }
    if (step + 1 < p.S) {
      __syncthreads();
      if (wid == 0) {   // publish h_t[:, j0:j0+LJ]: 32 rows x 32 B = 64 lanes x 16 B, write-through
        const int b = lane >> 1, half = lane & 1;
        const uint4 v = *reinterpret_cast<const uint4*>(sHo + b * LJ + half * 8);
        st16_sc1(rsH, (unsigned)((cur * 2 + dir) * LB * H + b * H + j0 + half * 8) * 2u, v);
      }
      fetch(step + 1);
      // only wave 0 stored payload; the other waves' loads / bulk stores stay in flight
      if (!dir_barrier(cnt, (unsigned)(step + 1) * nwg_dir, p.err, wid == 0)) return;
    }
  }
}

struct LstmBwdParams {
  const float* gates;    // [B][S][2][4H] activations i,f,g,o
  const float* cst;      // [B][S][2][H]
  const __bf16* whh;     // [2][4H][H] bf16
  const int64_t* ids;
  const __bf16* dhout;   // [B][S][2H] bf16 gradient w.r.t. layer output
  __bf16* dgates;        // [B][S][2][4H] bf16 gradient w.r.t. gate pre-activations
  __bf16* dgbuf;         // [2][2][LB][4H] bf16 ping-pong dgates exchange (v3: fp32 partials [2][2][nub][H][LB])
  unsigned* counters;
  unsigned* err;
  int B, S, H;
  unsigned long long* prof;
};

// wg owns hidden units j0..j0+LJ of its direction: cell backward for those units and
// columns j0..j0+LJ of dh_rec = dgates_{t} @ W_hh  (needs W_hh[:, j0:j0+LJ], all 4H rows)
__global__ void __launch_bounds__(LT) lstm_bwd_persistent(const LstmBwdParams p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int H = p.H, nub = H / LJ;
  const int dir = blockIdx.x / nub, ub = blockIdx.x % nub, j0 = ub * LJ;
  const int G4 = 4 * H;
  // LDS: Wt slice [LJ cols][4H] bf16 (transposed: row jj holds W_hh[:, j0+jj]), dgates tile [LB][4H] bf16,
  //      dh_rec [LB][LJ] f32
  __bf16* sWt = reinterpret_cast<__bf16*>(smem);
  __bf16* sD = sWt + LJ * G4;
  float* sR = reinterpret_cast<float*>(sD + LB * G4);
  __bf16* sDo = reinterpret_cast<__bf16*>(sR + LB * LJ);   // [LB][4][LJ] this workgroup's dgates_t slice
  const __amdgpu_buffer_rsrc_t rsD = rnn_rsrc(p.dgbuf, (unsigned)(4 * LB * G4 * 2));
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  for (int i = tid; i < LJ * G4; i += LT) {
    const int jj = i / G4, r = i % G4;
    reinterpret_cast<unsigned short*>(sWt)[i] =
        reinterpret_cast<const unsigned short*>(p.whh)[((size_t)dir * G4 + r) * H + j0 + jj];
  }
  float dcreg[2] = {0.f, 0.f};
  float dhcarry[2] = {0.f, 0.f};  // dh flowing to the previous step (recurrent part)
  __syncthreads();
  unsigned* cnt = p.counters + dir;
  // per-step inputs that do not depend on the recurrence (mask, output gradient, saved gates and
  // cell states) are loaded one step ahead
  float fin[2][7];   // dh_out, i, f, g, o, c, c_prev
  bool vin[2];
  auto fetch = [&](int stp) {
    const int tt = dir == 0 ? p.S - 1 - stp : stp;
    const int tp = dir == 0 ? tt - 1 : tt + 1;
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int q = tid + LT * k;
      const int b = q / LJ, j = j0 + q % LJ;
      vin[k] = false;
#pragma unroll
      for (int u = 0; u < 7; ++u) fin[k][u] = 0.f;
      if (b < p.B) {
        vin[k] = p.ids[(size_t)b * p.S + tt] > 0;
        const size_t gb = (((size_t)b * p.S + tt) * 2 + dir) * 4 * H;
        fin[k][0] = bf2f(reinterpret_cast<const unsigned short*>(p.dhout)[((size_t)b * p.S + tt) * 2 * H + dir * H + j]);
        fin[k][1] = p.gates[gb + j];
        fin[k][2] = p.gates[gb + H + j];
        fin[k][3] = p.gates[gb + 2 * H + j];
        fin[k][4] = p.gates[gb + 3 * H + j];
        fin[k][5] = p.cst[(((size_t)b * p.S + tt) * 2 + dir) * H + j];
        fin[k][6] = (tp >= 0 && tp < p.S) ? p.cst[(((size_t)b * p.S + tp) * 2 + dir) * H + j] : 0.f;
      }
    }
  };
  fetch(0);
  for (int step = 0; step < p.S; ++step) {
    const int t = dir == 0 ? p.S - 1 - step : step;      // reverse of the forward order
    const int cur = step & 1;
    const unsigned dst = (unsigned)((cur * 2 + dir) * LB * G4) * 2u;   // byte offset of dgates_t in dgbuf
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int q = tid + LT * k;
      const int b = q / LJ, jj = q % LJ, j = j0 + jj;
      float dgi = 0.f, dgf = 0.f, dgg = 0.f, dgo = 0.f;
      if (b < p.B) {
        const bool valid = vin[k];
        const size_t gbase = (((size_t)b * p.S + t) * 2 + dir) * 4 * H;
        const float dh = fin[k][0] + dhcarry[k];
        if (valid) {
          const float ig = fin[k][1], fg = fin[k][2], gg = fin[k][3], og = fin[k][4];
          const float c = fin[k][5];
          const float cprev = fin[k][6];
          const float tc = tanh_f(c);
          const float dc = dcreg[k] + dh * og * (1.f - tc * tc);
          dgo = dh * tc * og * (1.f - og);
          dgi = dc * gg * ig * (1.f - ig);
          dgg = dc * ig * (1.f - gg * gg);
          dgf = dc * cprev * fg * (1.f - fg);
          dcreg[k] = dc * fg;
          dhcarry[k] = 0.f;  // replaced by dgates @ W_hh below
        } else {
          // carried state: dh and dc pass through unchanged
          dhcarry[k] = dh;
        }
        __bf16* dg = p.dgates + gbase;
        reinterpret_cast<unsigned short*>(dg)[j] = f2bf(dgi);
        reinterpret_cast<unsigned short*>(dg)[H + j] = f2bf(dgf);
        reinterpret_cast<unsigned short*>(dg)[2 * H + j] = f2bf(dgg);
        reinterpret_cast<unsigned short*>(dg)[3 * H + j] = f2bf(dgo);
      }
      unsigned short* d16 = reinterpret_cast<unsigned short*>(sDo) + b * 4 * LJ + jj;
      d16[0] = f2bf(dgi);
      d16[LJ] = f2bf(dgf);
      d16[2 * LJ] = f2bf(dgg);
      d16[3 * LJ] = f2bf(dgo);
    }
    if (step + 1 == p.S) break;
    __syncthreads();
    {   // publish dgates_t[:, g*H + j0 .. +LJ] for the 4 gates: LB x 4 x 2 chunks of 16 B, write-through
      const int b = tid >> 3, g = (tid >> 1) & 3, half = tid & 1;
      const uint4 v = *reinterpret_cast<const uint4*>(sDo + (b * 4 + g) * LJ + half * 8);
      st16_sc1(rsD, dst + (unsigned)(b * G4 + g * H + j0 + half * 8) * 2u, v);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every wave stored payload: drain before the arrival
    fetch(step + 1);
    if (!dir_barrier(cnt, (unsigned)(step + 1) * nub, p.err, false)) return;
    // ---- gather dgates_t of all units of this direction [LB][4H] into LDS (sc1 loads)
    for (int i = tid; i < LB * G4 / 8; i += LT) reinterpret_cast<uint4*>(sD)[i] = ld16_sc1(rsD, dst + i * 16u);
    __syncthreads();
    // ---- dh_rec[b][jj] = sum_r dgates[b][r] * W[r][j0+jj] : M=32 (2 tiles), N=16 (1 tile), K=4H
    //      waves 0,1 -> m-tile 0,1 with K split in two halves (waves 2,3 take the upper K half)
    {
      const int mt = wid & 1, kh = wid >> 1;
      f32x4 acc = {0, 0, 0, 0};
      const int kbeg = kh * (G4 / 2), kend = kbeg + G4 / 2;
      for (int k0 = kbeg; k0 < kend; k0 += 32) {
        const int kk = k0 + 8 * (lane >> 4);
        const bf16x8 a = *reinterpret_cast<const bf16x8*>(sD + (mt * 16 + (lane & 15)) * G4 + kk);
        const bf16x8 b = *reinterpret_cast<const bf16x8*>(sWt + (lane & 15) * G4 + kk);
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc, 0, 0, 0);
      }
      if (kh == 0) {
#pragma unroll
        for (int e = 0; e < 4; ++e) sR[(mt * 16 + (lane >> 4) * 4 + e) * LJ + (lane & 15)] = acc[e];
      }
      __syncthreads();
      if (kh == 1) {
#pragma unroll
        for (int e = 0; e < 4; ++e) sR[(mt * 16 + (lane >> 4) * 4 + e) * LJ + (lane & 15)] += acc[e];
      }
      __syncthreads();
    }
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int q = tid + LT * k;
      const int b = q / LJ, jj = q % LJ;
      if (b < p.B) dhcarry[k] += sR[b * LJ + jj];
    }
    __syncthreads();
  }
}

// ------------------------------------------------------------------------- LSTM, role-split waves
// Round-6 form of the two persistent recurrences (knob lstm_v2, default on): 512-thread workgroups
// whose waves take fixed roles, so the per-step critical path -- the h_t / dgates_t hand-off between
// the workgroups of a direction -- never waits for bulk memory traffic.  (On gfx9-family hardware
// stores count in vmcnt like loads: in the round-1 kernels every wave streamed the step's bulk
// inputs and outputs, so the drain before the arrival and the wait for the exchange tile also
// waited for those.)
//   * compute waves 0-3: wave 0 publishes this workgroup's slice (sc1 stores, drain, one agent
//     atomic add) and polls the direction's arrival counter; after a workgroup barrier all four
//     gather the whole exchange tile (sc1 loads to registers, up to 16 in flight per lane: one wave
//     alone reads a fresh 64 KB slot in ~4.9 us, MI355X_MICROARCH.md handoff-payload) into LDS
//     (forward); in the backward each compute wave loads its own MFMA A fragments of the 64 KB
//     dgates tile straight into registers and runs its part of the recurrent product;
//   * IO waves 4-7: after the cell update they store the step's outputs from LDS staging (small: 4 KB
//     of dgates / 11 KB of activations per step); beside the MFMA product (after the gather) they
//     issue the loads of a later step's per-unit inputs into registers, committed to LDS while the
//     compute waves gather.
//     Their loads are still in flight while they join the forward's MFMA product (one 16x16 output
//     tile per wave) and both cell updates (one (b, unit) pair per thread);
//   * every barrier is an LDS-only one (lds_barrier), so no wave's outstanding loads hold it.
// LDS rows of the MFMA operands are XOR-swizzled by row (conflict-free 16-row fragment reads).  The
// arithmetic (MFMA tile mapping and K order, cell math) is the round-1 kernels': results are bitwise
// equal (tests/test_text_kernels_gpu.py::test_lstm_v2_bitwise).
constexpr int LT2 = 512;   // threads: 4 compute + 4 IO waves
constexpr int LC = 256;    // compute threads (waves 0-3); IO threads are tid - LC
static_assert(LB * LJ == LT2, "lstm v2: one (b, unit) pair per thread in the cell updates");

// IO-wave loads are raw buffer loads whose masked lanes read out of bounds (zeros): no branches
// around them, so the compiler has no conditional block to unpack the data in right after the load
// (which forced a wait on it) and the loads stay in flight until their commit
constexpr unsigned kIoOOB = 0x80000000u;
__device__ __forceinline__ uint4 io_ld16(__amdgpu_buffer_rsrc_t r, unsigned off) {
  const u32x4v v = __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 0);
  return uint4{v[0], v[1], v[2], v[3]};
}
__device__ __forceinline__ long long io_ld8(__amdgpu_buffer_rsrc_t r, unsigned off) {
  typedef unsigned u32x2v __attribute__((ext_vector_type(2)));
  const u32x2v v = __builtin_amdgcn_raw_buffer_load_b64(r, (int)off, 0, 0);
  return (long long)(((unsigned long long)v[1] << 32) | v[0]);
}

// Workgroup barrier for LDS hand-offs only: waits for this wave's LDS operations, not for its
// global ones (__syncthreads() = workgroup release fence + s_barrier waits vmcnt(0) too, so an IO
// wave with its loads in flight would hold every barrier of the step until they land).  Global data
// never passes between the waves of a workgroup through memory here: the exchange tile is loaded
// (sc1, to registers) after this barrier has ordered it behind the polling wave's match.
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// chunk c of row r at 16-B slot c ^ (r & m): the 16 lanes of an MFMA fragment read 16 rows at the
// same column, which unswizzled (row pitch a multiple of 256 B) all hit the same LDS banks
__host__ __device__ constexpr int swz_mask(int nchunks) {
  return ((nchunks & -nchunks) < 16 ? (nchunks & -nchunks) : 16) - 1;
}
__device__ __forceinline__ int swz(int row, int chunk, int nchunks) {
  return row * nchunks + (chunk ^ (row & swz_mask(nchunks)));
}

// wave 0, lane 0 polls the arrival counter (sc1 loads); the wave's other lanes wait in lockstep
__device__ __forceinline__ bool exch_wait(unsigned* counter, unsigned target, unsigned* err) {
  bool ok = true;
  if ((threadIdx.x & 63) == 0) {
    unsigned spins = 0;
    while (__hip_atomic_load((gu32*)counter, RLX_AGENT) < target) {
      __builtin_amdgcn_s_sleep(1);
      if (++spins > kSpinLimit) {
        __hip_atomic_store((gu32*)err, 1u, RLX_AGENT);
        ok = false;
        break;
      }
    }
  }
  const bool r = __shfl(ok ? 1 : 0, 0) != 0;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");   // compiler ordering only: tile loads are sc1
  return r;
}

// exchange-tile gather by the 256 compute threads: [rows][nchunks] 16-B chunks (byte offset src),
// sc1 loads to registers, MAXN in flight per lane, written to swizzled LDS
template <int MAXN>
__device__ __forceinline__ void gather_tile_sc1(__amdgpu_buffer_rsrc_t rs, unsigned src, uint4* lds, int rows,
                                                int nchunks, int ctid) {
  const int n = rows * nchunks / LC;   // a whole number of passes (checked on the host)
  for (int e0 = 0; e0 < n; e0 += MAXN) {
    uint4 v[MAXN];
#pragma unroll
    for (int e = 0; e < MAXN; ++e)
      if (e0 + e < n) v[e] = ld16_sc1(rs, src + (unsigned)(((e0 + e) * LC + ctid) * 16));
#pragma unroll
    for (int e = 0; e < MAXN; ++e)
      if (e0 + e < n) {
        const int i = (e0 + e) * LC + ctid;
        lds[swz(i / nchunks, i % nchunks, nchunks)] = v[e];
      }
  }
}

// phase clocks (knob lstm_prof): workgroup 0, thread 0, shader clocks per phase over the launch
struct PhaseClock {
  bool on;
  unsigned long long pc[8] = {0, 0, 0, 0, 0, 0, 0, 0}, tp = 0;
  __device__ void mark(int ph) {
    if (on) {
      const unsigned long long now = __builtin_amdgcn_s_memtime();
      if (ph >= 0) pc[ph] += now - tp;
      tp = now;
    }
  }
  __device__ void flush(unsigned long long* out, int n) {
    if (on)
      for (int i = 0; i < n; ++i) out[i] = pc[i];
  }
};

__global__ void __launch_bounds__(LT2) lstm_fwd_persistent2(const LstmFwdParams p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int H = p.H, nub = H / LJ, G4 = 4 * H, NCH = H / 8;
  const int dir = blockIdx.x / nub, ub = blockIdx.x % nub, j0 = ub * LJ;
  __bf16* sW = reinterpret_cast<__bf16*>(smem);               // [4LJ][H]   W_hh rows (swizzled)
  __bf16* sH = sW + 4 * LJ * H;                                // [LB][H]    h_{t-1} (swizzled)
  float* sG = reinterpret_cast<float*>(sH + LB * H);           // [LB][4LJ]  recurrent pre-activations
  float* sGx = sG + LB * 4 * LJ;                               // [2][LB][4LJ] input projections (ping-pong)
  float* sA = sGx + 2 * LB * 4 * LJ;                           // [LB][4LJ]  activations i,f,g,o (staging)
  float* sC = sA + LB * 4 * LJ;                                // [LB][LJ]   c_t (staging)
  __bf16* sHo = reinterpret_cast<__bf16*>(sC + LB * LJ);      // [LB][LJ]   h_t (exchange + output)
  int* sV = reinterpret_cast<int*>(sHo + LB * LJ);            // [2][LB] token valid flags; [2*LB] abort
  const __amdgpu_buffer_rsrc_t rsH = rnn_rsrc(p.hbuf, (unsigned)(4 * LB * H * 2));
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, it = tid - LC;
  const bool io = tid >= LC;
  for (int i = tid; i < 4 * LJ * H / 8; i += LT2) {
    const int r = i / NCH, c8 = i % NCH;
    const int gate = r / LJ, jj = r % LJ;
    reinterpret_cast<uint4*>(sW)[swz(r, c8, NCH)] =
        reinterpret_cast<const uint4*>(p.whh + ((size_t)dir * G4 + gate * H + j0 + jj) * H)[c8];
  }
  for (int i = tid; i < LB * H / 8; i += LT2) reinterpret_cast<uint4*>(sH)[i] = uint4{0, 0, 0, 0};
  if (tid == 0) sV[2 * LB] = 0;
  unsigned* cnt = p.counters + dir;
  // IO threads: the step's gx slice [b][gate][16 units] = 2 x 16 B per (b, gate): 256 items, + 32 ids
  const __amdgpu_buffer_rsrc_t rsGx = rnn_rsrc(p.gx, (unsigned)((size_t)p.B * p.S * 2 * G4 * 2));
  const __amdgpu_buffer_rsrc_t rsId = rnn_rsrc(p.ids, (unsigned)((size_t)p.B * p.S * 8));
  uint4 fv = uint4{0, 0, 0, 0};
  long long fid = 0;   // the raw token id: compared at commit
  auto io_fetch = [&](int stp) {
    const int tt = dir == 0 ? stp : p.S - 1 - stp;
    const int b = it >> 3, g = (it >> 1) & 3, half = it & 1;
    fv = io_ld16(rsGx, b < p.B ? (unsigned)(((((unsigned)b * p.S + tt) * 2 + dir) * G4 + g * H + j0 + half * 8) * 2)
                               : kIoOOB);
    fid = io_ld8(rsId, (it < LB && it < p.B) ? (unsigned)((it * p.S + tt) * 8) : kIoOOB);
  };
  auto io_commit = [&](int slot) {
    const int b = it >> 3, g = (it >> 1) & 3, half = it & 1;
    const unsigned short* u = reinterpret_cast<const unsigned short*>(&fv);
    float* d = sGx + slot * LB * 4 * LJ + b * 4 * LJ + g * LJ + half * 8;
#pragma unroll
    for (int e = 0; e < 8; ++e) d[e] = bf2f(u[e]);
    if (it < LB) sV[slot * LB + it] = fid > 0 ? 1 : 0;
  };
  // IO threads: this step's outputs: activations 4 x 64 B per b, c_t 64 B per b, h_t 32 B per b
  auto io_store = [&](int t) {
    constexpr int NA = LB * 16, NC = LB * 4, NH = LB * 2;
    for (int i = it; i < NA + NC + NH; i += LT2 - LC) {
      if (i < NA) {
        const int b = i >> 4, g = (i >> 2) & 3, q = i & 3;
        if (b < p.B)
          *reinterpret_cast<float4*>(p.gates + (((size_t)b * p.S + t) * 2 + dir) * G4 + g * H + j0 + q * 4) =
              *reinterpret_cast<const float4*>(sA + b * 4 * LJ + g * LJ + q * 4);
      } else if (i < NA + NC) {
        const int b = (i - NA) >> 2, q = (i - NA) & 3;
        if (b < p.B)
          *reinterpret_cast<float4*>(p.cst + (((size_t)b * p.S + t) * 2 + dir) * H + j0 + q * 4) =
              *reinterpret_cast<const float4*>(sC + b * LJ + q * 4);
      } else {
        const int b = (i - NA - NC) >> 1, half = (i - NA - NC) & 1;
        if (b < p.B)
          *reinterpret_cast<uint4*>(p.hout + ((size_t)b * p.S + t) * 2 * H + dir * H + j0 + half * 8) =
              *reinterpret_cast<const uint4*>(sHo + b * LJ + half * 8);
      }
    }
  };
  if (io) {
    io_fetch(0);
    io_commit(0);
    if (p.S > 1) io_fetch(1);
  }
  float creg = 0.f, hreg = 0.f;   // the thread's (b, unit) pair
  PhaseClock clk{p.prof != nullptr && blockIdx.x == 0 && tid == 0};   // poll, gather, MFMA, cell, publish
  lds_barrier();
  for (int step = 0; step < p.S; ++step) {
    const int t = dir == 0 ? step : p.S - 1 - step;
    const int cur = step & 1;
    clk.mark(-1);
    // ---- A: wave 0 waits for every workgroup's h_{t-1} slice
    if (wid == 0 && step > 0) {
      if (!exch_wait(cnt, (unsigned)step * nub, p.err) && lane == 0) sV[2 * LB] = 1;
      clk.mark(0);
    }
    lds_barrier();
    if (sV[2 * LB]) return;
    // ---- gather h_{t-1} (compute waves); the IO waves commit this step's inputs (loaded last step)
    if (!io) {
      if (step > 0)
        gather_tile_sc1<4>(rsH, (unsigned)(((cur ^ 1) * 2 + dir) * LB * H) * 2u, reinterpret_cast<uint4*>(sH), LB,
                           NCH, tid);
      clk.mark(1);
    } else if (step > 0) {
      io_commit(cur);   // this step's inputs, loaded during the previous step's MFMA phase
    }
    lds_barrier();
    if (io && step > 0 && step + 1 < p.S) io_fetch(step + 1);   // beside the MFMA phase, committed next step
    // ---- B: pre-activations [LB][4LJ] = h @ Wslice^T: all 8 waves, one 16x16 tile each (m-tile
    //      w & 1, n-tile w >> 1), round-1 K order
    {
      const int mt = wid & 1, nt = wid >> 1;
      f32x4 acc = {0, 0, 0, 0};
      const bf16x8* sH8 = reinterpret_cast<const bf16x8*>(sH);
      const bf16x8* sW8 = reinterpret_cast<const bf16x8*>(sW);
      const int ar = mt * 16 + (lane & 15), n0 = nt * 16 + (lane & 15);
      for (int k0 = 0; k0 < H; k0 += 128) {   // fragments of 4 K-steps read ahead of their MFMAs
        bf16x8 a[4], b0[4];
#pragma unroll
        for (int u = 0; u < 4; ++u)
          if (k0 + 32 * u < H) {
            const int kc = ((k0 + 32 * u) >> 3) + (lane >> 4);
            a[u] = sH8[swz(ar, kc, NCH)];
            b0[u] = sW8[swz(n0, kc, NCH)];
          }
#pragma unroll
        for (int u = 0; u < 4; ++u)
          if (k0 + 32 * u < H) acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[u], b0[u], acc, 0, 0, 0);
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) sG[(mt * 16 + (lane >> 4) * 4 + e) * 4 * LJ + n0] = acc[e];
      clk.mark(2);
    }
    lds_barrier();
    // ---- C: cell update, one (b, jj) pair per thread (LB * LJ = 512), outputs to LDS staging
    {
      const int b = tid / LJ, jj = tid % LJ;
      float hn = 0.f;
      if (b < p.B) {
        const bool valid = sV[cur * LB + b] != 0;
        const float* gx = sGx + cur * LB * 4 * LJ + b * 4 * LJ;
        float pre[4];
#pragma unroll
        for (int g = 0; g < 4; ++g) pre[g] = sG[b * 4 * LJ + g * LJ + jj] + gx[g * LJ + jj];
        const float ig = sigm(pre[0]), fg = sigm(pre[1]), gg = tanh_f(pre[2]), og = sigm(pre[3]);
        float cn, hv;
        if (valid) {
          cn = fg * creg + ig * gg;
          hv = og * tanh_f(cn);
        } else {
          cn = creg;
          hv = hreg;
        }
        creg = cn;
        hreg = hv;
        hn = hv;
        float* a = sA + b * 4 * LJ + jj;
        a[0] = ig;
        a[LJ] = fg;
        a[2 * LJ] = gg;
        a[3 * LJ] = og;
        sC[b * LJ + jj] = cn;
      }
      reinterpret_cast<unsigned short*>(sHo)[b * LJ + jj] = f2bf(hn);
      clk.mark(3);
    }
    lds_barrier();
    // ---- D: wave 0 publishes h_t and arrives; the IO waves store the step's outputs
    if (wid == 0 && step + 1 < p.S) {
      const int b = lane >> 1, half = lane & 1;
      const uint4 v = *reinterpret_cast<const uint4*>(sHo + b * LJ + half * 8);
      st16_sc1(rsH, (unsigned)((cur * 2 + dir) * LB * H + b * H + j0 + half * 8) * 2u, v);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // only the publish store is outstanding
      if (lane == 0) __hip_atomic_fetch_add((gu32*)cnt, 1u, RLX_AGENT);
      clk.mark(4);
    } else if (io) {
      io_store(t);
    }
  }
  clk.flush(p.prof, 5);
}

__global__ void __launch_bounds__(LT2) lstm_bwd_persistent2(const LstmBwdParams p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int H = p.H, nub = H / LJ, G4 = 4 * H, NCD = G4 / 8;
  const int dir = blockIdx.x / nub, ub = blockIdx.x % nub, j0 = ub * LJ;
  __bf16* sWt = reinterpret_cast<__bf16*>(smem);               // [LJ][4H] W_hh columns (swizzled)
  float* sR = reinterpret_cast<float*>(sWt + LJ * G4);          // [LB][LJ] dh_rec
  __bf16* sDo = reinterpret_cast<__bf16*>(sR + LB * LJ);       // [LB][4][LJ] this slice's dgates_t
  float* sF = reinterpret_cast<float*>(sDo + LB * 4 * LJ);      // [2][7][LB][LJ] per-step inputs
  int* sV = reinterpret_cast<int*>(sF + 2 * 7 * LB * LJ);       // [2][LB] valid flags; [2*LB] abort
  const __amdgpu_buffer_rsrc_t rsD = rnn_rsrc(p.dgbuf, (unsigned)(4 * LB * G4 * 2));
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, it = tid - LC;
  const bool io = tid >= LC;
  for (int i = tid; i < LJ * G4; i += LT2) {
    const int jj = i / G4, r = i % G4;
    reinterpret_cast<unsigned short*>(sWt)[swz(jj, r >> 3, NCD) * 8 + (r & 7)] =
        reinterpret_cast<const unsigned short*>(p.whh)[((size_t)dir * G4 + r) * H + j0 + jj];
  }
  if (tid == 0) sV[2 * LB] = 0;
  unsigned* cnt = p.counters + dir;
  // IO threads: per-step inputs as 16-B items, each load instruction from ONE source (uniform buffer
  // resource, out-of-bounds zeros for masked lanes): gates 512 items (2 per thread: b, gate, quarter),
  // c_t 128 (threads 0-127) or c_prev 128 (threads 128-255), dh_out 64 (threads 0-63), ids 32
  const __amdgpu_buffer_rsrc_t rsG = rnn_rsrc(p.gates, (unsigned)((size_t)p.B * p.S * 2 * G4 * 4));
  const __amdgpu_buffer_rsrc_t rsC = rnn_rsrc(p.cst, (unsigned)((size_t)p.B * p.S * 2 * H * 4));
  const __amdgpu_buffer_rsrc_t rsDh = rnn_rsrc(p.dhout, (unsigned)((size_t)p.B * p.S * 2 * H * 2));
  const __amdgpu_buffer_rsrc_t rsId = rnn_rsrc(p.ids, (unsigned)((size_t)p.B * p.S * 8));
  uint4 fv[4];
  long long fid = 0;
  auto io_fetch = [&](int stp) {
    const int tt = dir == 0 ? p.S - 1 - stp : stp;
    const int tp = dir == 0 ? tt - 1 : tt + 1;
#pragma unroll
    for (int k = 0; k < 2; ++k) {   // gates
      const int i = it + 256 * k, b = i >> 4, g = (i >> 2) & 3, q = i & 3;
      fv[k] = io_ld16(rsG, b < p.B ? (unsigned)(((((unsigned)b * p.S + tt) * 2 + dir) * G4 + g * H + j0 + q * 4) * 4)
                                   : kIoOOB);
    }
    {   // c_t (threads 0-127) / c_prev (threads 128-255)
      const int i = it & 127, b = i >> 2, q = i & 3, ts = it < 128 ? tt : tp;
      const bool ok = b < p.B && ts >= 0 && ts < p.S;
      fv[2] = io_ld16(rsC, ok ? (unsigned)(((((unsigned)b * p.S + ts) * 2 + dir) * H + j0 + q * 4) * 4) : kIoOOB);
    }
    {   // dh_out (threads 0-63)
      const int b = it >> 1, half = it & 1;
      fv[3] = io_ld16(rsDh, (it < 64 && b < p.B)
                                ? (unsigned)((((unsigned)b * p.S + tt) * 2 * H + dir * H + j0 + half * 8) * 2) : kIoOOB);
    }
    fid = io_ld8(rsId, (it < LB && it < p.B) ? (unsigned)((it * p.S + tt) * 8) : kIoOOB);
  };
  auto io_commit = [&](int slot) {   // F rows: 0 dh_out, 1-4 gates i,f,g,o, 5 c_t, 6 c_prev
    float* F = sF + slot * 7 * LB * LJ;
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int i = it + 256 * k, b = i >> 4, g = (i >> 2) & 3, q = i & 3;
      *reinterpret_cast<uint4*>(F + (1 + g) * LB * LJ + b * LJ + q * 4) = fv[k];
    }
    {
      const int i = it & 127, b = i >> 2, q = i & 3;
      *reinterpret_cast<uint4*>(F + (it < 128 ? 5 : 6) * LB * LJ + b * LJ + q * 4) = fv[2];
    }
    if (it < 64) {
      const int b = it >> 1, half = it & 1;
      const unsigned short* u = reinterpret_cast<const unsigned short*>(&fv[3]);
#pragma unroll
      for (int e = 0; e < 8; ++e) F[b * LJ + half * 8 + e] = bf2f(u[e]);
    }
    if (it < LB) sV[slot * LB + it] = fid > 0 ? 1 : 0;
  };
  // IO threads: this step's dgates [b][gate][16 units] bf16 = 2 x 16 B per (b, gate)
  auto io_store = [&](int t) {
    const int b = it >> 3, g = (it >> 1) & 3, half = it & 1;
    if (b < p.B)
      *reinterpret_cast<uint4*>(p.dgates + (((size_t)b * p.S + t) * 2 + dir) * G4 + g * H + j0 + half * 8) =
          *reinterpret_cast<const uint4*>(sDo + (b * 4 + g) * LJ + half * 8);
  };
  if (io) {
    io_fetch(0);
    io_commit(0);
    if (p.S > 1) io_fetch(1);
  }
  float dcreg = 0.f, dhcarry = 0.f;   // the thread's (b, unit) pair
  PhaseClock clk{p.prof != nullptr && blockIdx.x == 0 && tid == 0};   // cell, publish, poll, gather, MFMA
  lds_barrier();
  for (int step = 0; step < p.S; ++step) {
    const int t = dir == 0 ? p.S - 1 - step : step;
    const int cur = step & 1;
    const unsigned dst = (unsigned)((cur * 2 + dir) * LB * G4) * 2u;
    clk.mark(-1);
    // ---- C: cell backward (round-1 math), one (b, jj) pair per thread, dgates slice to LDS
    {
      const float* F = sF + cur * 7 * LB * LJ;
      const int b = tid / LJ, jj = tid % LJ;
      float dgi = 0.f, dgf = 0.f, dgg = 0.f, dgo = 0.f;
      if (b < p.B) {
        const int o = b * LJ + jj;
        const float dh = F[o] + dhcarry;
        if (sV[cur * LB + b]) {
          const float ig = F[LB * LJ + o], fg = F[2 * LB * LJ + o], gg = F[3 * LB * LJ + o], og = F[4 * LB * LJ + o];
          const float c = F[5 * LB * LJ + o];
          const float cprev = F[6 * LB * LJ + o];
          const float tc = tanh_f(c);
          const float dc = dcreg + dh * og * (1.f - tc * tc);
          dgo = dh * tc * og * (1.f - og);
          dgi = dc * gg * ig * (1.f - ig);
          dgg = dc * ig * (1.f - gg * gg);
          dgf = dc * cprev * fg * (1.f - fg);
          dcreg = dc * fg;
          dhcarry = 0.f;
        } else {
          dhcarry = dh;
        }
      }
      unsigned short* d16 = reinterpret_cast<unsigned short*>(sDo) + b * 4 * LJ + jj;
      d16[0] = f2bf(dgi);
      d16[LJ] = f2bf(dgf);
      d16[2 * LJ] = f2bf(dgg);
      d16[3 * LJ] = f2bf(dgo);
      clk.mark(0);
    }
    lds_barrier();
    // ---- D: wave 0 publishes dgates_t and arrives; the IO waves store it and load the next step
    if (wid == 0) {
      if (step + 1 < p.S) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int i = lane + 64 * e, b = i >> 3, g = (i >> 1) & 3, half = i & 1;
          const uint4 v = *reinterpret_cast<const uint4*>(sDo + (b * 4 + g) * LJ + half * 8);
          st16_sc1(rsD, dst + (unsigned)(b * G4 + g * H + j0 + half * 8) * 2u, v);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // only the publish stores are outstanding
        if (lane == 0) __hip_atomic_fetch_add((gu32*)cnt, 1u, RLX_AGENT);
        clk.mark(1);
      }
    } else if (io) {
      io_store(t);
    }
    if (step + 1 == p.S) break;
    // ---- A: wave 0 waits for every workgroup's dgates_t slice
    if (wid == 0) {
      if (!exch_wait(cnt, (unsigned)(step + 1) * nub, p.err) && lane == 0) sV[2 * LB] = 1;
      clk.mark(2);
    }
    lds_barrier();
    if (sV[2 * LB]) return;
    if (io) {
      io_commit(cur ^ 1);   // the next step's inputs, loaded beside the previous MFMA phase
      if (step + 2 < p.S) io_fetch(step + 2);   // beside this MFMA phase, committed next step
    }
    // ---- B: dh_rec[b][jj] = sum_r dgates[b][r] W[r][j0+jj] (round-1 split: waves 2,3 the upper K half).
    //      Each compute wave loads its own A fragments (rows mt*16 + lane%16, its K half) straight from
    //      the exchange buffer into registers, all in flight at once: no LDS copy of the 64 KB tile and
    //      no barrier between the gather and the MFMAs.
    f32x4 acc = {0, 0, 0, 0};
    const int mt = wid & 1, kh = (wid >> 1) & 1;
    if (!io) {
      const int kbeg = kh * (G4 / 2), nks = G4 / 2 / 32;
      const bf16x8* sW8 = reinterpret_cast<const bf16x8*>(sWt);
      const int ar = mt * 16 + (lane & 15), br = lane & 15;
      const unsigned abase = dst + (unsigned)(ar * G4 + kbeg + 8 * (lane >> 4)) * 2u;
      for (int c0 = 0; c0 < nks; c0 += 16) {
        uint4 av[16];
#pragma unroll
        for (int u = 0; u < 16; ++u)
          if (c0 + u < nks) av[u] = ld16_sc1(rsD, abase + (unsigned)((c0 + u) * 64));
#pragma unroll
        for (int u = 0; u < 16; ++u)
          if (c0 + u < nks) {
            const int kc = ((kbeg + 32 * (c0 + u)) >> 3) + (lane >> 4);
            acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, av[u]), sW8[swz(br, kc, NCD)],
                                                          acc, 0, 0, 0);
          }
      }
      clk.mark(3);
      if (kh == 0) {
#pragma unroll
        for (int e = 0; e < 4; ++e) sR[(mt * 16 + (lane >> 4) * 4 + e) * LJ + (lane & 15)] = acc[e];
      }
    }
    lds_barrier();
    if (!io) {
      if (kh == 1) {
#pragma unroll
        for (int e = 0; e < 4; ++e) sR[(mt * 16 + (lane >> 4) * 4 + e) * LJ + (lane & 15)] += acc[e];
      }
    }
    lds_barrier();
    {
      const int b = tid / LJ, jj = tid % LJ;
      if (b < p.B) dhcarry += sR[b * LJ + jj];
      clk.mark(4);
    }
  }
  clk.flush(p.prof, 5);
}

// Backward, partial-sum exchange (knob lstm_v2 = 2): instead of handing the 64 KB dgates_t tile of
// the direction to every workgroup (each then multiplies it by its own 16 columns of W_hh), each
// workgroup multiplies ITS dgates slice [LB][4*LJ] by its 4*LJ rows of W_hh -- a partial dh_rec over
// all H units -- and publishes that (fp32 [H][LB], 32 KB); each workgroup then sums, for its LJ units,
// the nub partials in source order (32 KB gathered as 4-B sc1 loads).  The partial product needs no
// exchange, so the hand-off carries a product instead of an operand and the MFMA leaves the
// critical path's gather.  Same math in another summation order: equal to the other forms to fp32
// reassociation (tests/test_text_kernels_gpu.py::test_lstm_bwd_partial_exchange).  dgbuf holds the
// fp32 partials here: [2 slots][2 dirs][nub sources][H][LB].
__global__ void __launch_bounds__(LT2) lstm_bwd_persistent3(const LstmBwdParams p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int H = p.H, nub = H / LJ, G4 = 4 * H, NCD = G4 / 8;
  const int dir = blockIdx.x / nub, ub = blockIdx.x % nub, j0 = ub * LJ;
  __bf16* sWr = reinterpret_cast<__bf16*>(smem);               // [H][4LJ] this slice's W_hh rows, j-major (swizzled)
  float* sR = reinterpret_cast<float*>(sWr + H * 4 * LJ);       // [LB][LJ] dh_rec
  __bf16* sDo = reinterpret_cast<__bf16*>(sR + LB * LJ);       // [LB][4][LJ] this slice's dgates_t
  float* sF = reinterpret_cast<float*>(sDo + LB * 4 * LJ);      // [2][7][LB][LJ] per-step inputs
  int* sV = reinterpret_cast<int*>(sF + 2 * 7 * LB * LJ);       // [2][LB] valid flags; [2*LB] abort
  const __amdgpu_buffer_rsrc_t rsP = rnn_rsrc(p.dgbuf, (unsigned)((size_t)4 * nub * H * LB * 4));
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6, it = tid - LC;
  const bool io = tid >= LC;
  // sWr[j][r] = W_hh[dir][gate*H + j0 + jj][j], r = gate*LJ + jj: 8 chunks of 16 B per j row
  for (int i = tid; i < H * 4 * LJ; i += LT2) {
    const int r = i / H, j = i % H, gate = r / LJ, jj = r % LJ;
    reinterpret_cast<unsigned short*>(sWr)[swz(j, r >> 3, 8) * 8 + (r & 7)] =
        reinterpret_cast<const unsigned short*>(p.whh)[((size_t)dir * G4 + gate * H + j0 + jj) * H + j];
  }
  if (tid == 0) sV[2 * LB] = 0;
  unsigned* cnt = p.counters + dir;
  // IO threads: per-step inputs as 16-B items, each load instruction from ONE source (uniform buffer
  // resource, out-of-bounds zeros for masked lanes): gates 512 items (2 per thread: b, gate, quarter),
  // c_t 128 (threads 0-127) or c_prev 128 (threads 128-255), dh_out 64 (threads 0-63), ids 32
  const __amdgpu_buffer_rsrc_t rsG = rnn_rsrc(p.gates, (unsigned)((size_t)p.B * p.S * 2 * G4 * 4));
  const __amdgpu_buffer_rsrc_t rsC = rnn_rsrc(p.cst, (unsigned)((size_t)p.B * p.S * 2 * H * 4));
  const __amdgpu_buffer_rsrc_t rsDh = rnn_rsrc(p.dhout, (unsigned)((size_t)p.B * p.S * 2 * H * 2));
  const __amdgpu_buffer_rsrc_t rsId = rnn_rsrc(p.ids, (unsigned)((size_t)p.B * p.S * 8));
  uint4 fv[4];
  long long fid = 0;
  auto io_fetch = [&](int stp) {
    const int tt = dir == 0 ? p.S - 1 - stp : stp;
    const int tp = dir == 0 ? tt - 1 : tt + 1;
#pragma unroll
    for (int k = 0; k < 2; ++k) {   // gates
      const int i = it + 256 * k, b = i >> 4, g = (i >> 2) & 3, q = i & 3;
      fv[k] = io_ld16(rsG, b < p.B ? (unsigned)(((((unsigned)b * p.S + tt) * 2 + dir) * G4 + g * H + j0 + q * 4) * 4)
                                   : kIoOOB);
    }
    {   // c_t (threads 0-127) / c_prev (threads 128-255)
      const int i = it & 127, b = i >> 2, q = i & 3, ts = it < 128 ? tt : tp;
      const bool ok = b < p.B && ts >= 0 && ts < p.S;
      fv[2] = io_ld16(rsC, ok ? (unsigned)(((((unsigned)b * p.S + ts) * 2 + dir) * H + j0 + q * 4) * 4) : kIoOOB);
    }
    {   // dh_out (threads 0-63)
      const int b = it >> 1, half = it & 1;
      fv[3] = io_ld16(rsDh, (it < 64 && b < p.B)
                                ? (unsigned)((((unsigned)b * p.S + tt) * 2 * H + dir * H + j0 + half * 8) * 2) : kIoOOB);
    }
    fid = io_ld8(rsId, (it < LB && it < p.B) ? (unsigned)((it * p.S + tt) * 8) : kIoOOB);
  };
  auto io_commit = [&](int slot) {   // F rows: 0 dh_out, 1-4 gates i,f,g,o, 5 c_t, 6 c_prev
    float* F = sF + slot * 7 * LB * LJ;
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int i = it + 256 * k, b = i >> 4, g = (i >> 2) & 3, q = i & 3;
      *reinterpret_cast<uint4*>(F + (1 + g) * LB * LJ + b * LJ + q * 4) = fv[k];
    }
    {
      const int i = it & 127, b = i >> 2, q = i & 3;
      *reinterpret_cast<uint4*>(F + (it < 128 ? 5 : 6) * LB * LJ + b * LJ + q * 4) = fv[2];
    }
    if (it < 64) {
      const int b = it >> 1, half = it & 1;
      const unsigned short* u = reinterpret_cast<const unsigned short*>(&fv[3]);
#pragma unroll
      for (int e = 0; e < 8; ++e) F[b * LJ + half * 8 + e] = bf2f(u[e]);
    }
    if (it < LB) sV[slot * LB + it] = fid > 0 ? 1 : 0;
  };
  // IO threads: this step's dgates [b][gate][16 units] bf16 = 2 x 16 B per (b, gate)
  auto io_store = [&](int t) {
    const int b = it >> 3, g = (it >> 1) & 3, half = it & 1;
    if (b < p.B)
      *reinterpret_cast<uint4*>(p.dgates + (((size_t)b * p.S + t) * 2 + dir) * G4 + g * H + j0 + half * 8) =
          *reinterpret_cast<const uint4*>(sDo + (b * 4 + g) * LJ + half * 8);
  };
  if (io) {
    io_fetch(0);
    io_commit(0);
    if (p.S > 1) io_fetch(1);
  }
  float dcreg = 0.f, dhcarry = 0.f;   // the thread's (b, unit) pair
  PhaseClock clk{p.prof != nullptr && blockIdx.x == 0 && tid == 0};   // cell, MFMA+publish, poll, gather, carry
  lds_barrier();
  for (int step = 0; step < p.S; ++step) {
    const int t = dir == 0 ? p.S - 1 - step : step;
    const int cur = step & 1;
    clk.mark(-1);
    // ---- C: cell backward (round-1 math), one (b, jj) pair per thread, dgates slice to LDS
    {
      const float* F = sF + cur * 7 * LB * LJ;
      const int b = tid / LJ, jj = tid % LJ;
      float dgi = 0.f, dgf = 0.f, dgg = 0.f, dgo = 0.f;
      if (b < p.B) {
        const int o = b * LJ + jj;
        const float dh = F[o] + dhcarry;
        if (sV[cur * LB + b]) {
          const float ig = F[LB * LJ + o], fg = F[2 * LB * LJ + o], gg = F[3 * LB * LJ + o], og = F[4 * LB * LJ + o];
          const float c = F[5 * LB * LJ + o];
          const float cprev = F[6 * LB * LJ + o];
          const float tc = tanh_f(c);
          const float dc = dcreg + dh * og * (1.f - tc * tc);
          dgo = dh * tc * og * (1.f - og);
          dgi = dc * gg * ig * (1.f - ig);
          dgg = dc * ig * (1.f - gg * gg);
          dgf = dc * cprev * fg * (1.f - fg);
          dcreg = dc * fg;
          dhcarry = 0.f;
        } else {
          dhcarry = dh;
        }
      }
      unsigned short* d16 = reinterpret_cast<unsigned short*>(sDo) + b * 4 * LJ + jj;
      d16[0] = f2bf(dgi);
      d16[LJ] = f2bf(dgf);
      d16[2 * LJ] = f2bf(dgg);
      d16[3 * LJ] = f2bf(dgo);
      clk.mark(0);
    }
    lds_barrier();
    // ---- D: the IO waves store dgates_t; then every wave multiplies the slice by this workgroup's
    //      W_hh rows (partial dh_rec for all H units: [LB] x [4LJ] x [H]) and publishes it (sc1)
    if (io) io_store(t);
    if (step + 1 < p.S) {   // all 8 waves: 2 m-tiles x H/16 n-tiles
      const int mt = wid & 1;
      const bf16x8* sD8 = reinterpret_cast<const bf16x8*>(sDo);
      const bf16x8* sW8 = reinterpret_cast<const bf16x8*>(sWr);
      bf16x8 a[2];
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) a[ks] = sD8[(mt * 16 + (lane & 15)) * 8 + ks * 4 + (lane >> 4)];
      const unsigned pbase = (unsigned)(((cur * 2 + dir) * nub + ub) * H * LB) * 4u;
      for (int nt = wid >> 1; nt < H / 16; nt += LT2 / 128) {
        const int j = nt * 16 + (lane & 15);
        f32x4 acc = {0, 0, 0, 0};
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
          acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[ks], sW8[swz(j, ks * 4 + (lane >> 4), 8)], acc, 0, 0, 0);
        const int b0 = mt * 16 + (lane >> 4) * 4;   // 4 consecutive b of column j: one 16-B store
        st16_sc1(rsP, pbase + (unsigned)(j * LB + b0) * 4u, __builtin_bit_cast(uint4, acc));
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every wave drains its partial stores
      clk.mark(1);
    }
    if (step + 1 == p.S) break;
    lds_barrier();   // every wave's partial stores drained
    if (tid == 0) __hip_atomic_fetch_add((gu32*)cnt, 1u, RLX_AGENT);
    // ---- A: wave 0 waits for every workgroup's partial
    if (wid == 0) {
      if (!exch_wait(cnt, (unsigned)(step + 1) * nub, p.err) && lane == 0) sV[2 * LB] = 1;
      clk.mark(2);
    }
    lds_barrier();
    if (sV[2 * LB]) return;
    if (io) {
      io_commit(cur ^ 1);   // the next step's inputs, loaded beside the previous MFMA phase
      if (step + 2 < p.S) io_fetch(step + 2);   // beside this MFMA phase, committed next step
    }
    // ---- B: dh_rec[b][jj] = sum over the nub sources (in source order) of their partials: the compute
    //      threads take 2 (b, jj) pairs each (b fastest: a wave reads 256 contiguous bytes per source),
    //      16 sources' loads in flight per pair, branch-free (sources past nub read out of bounds: 0)
    if (!io) {
      const unsigned sbase = (unsigned)((cur * 2 + dir) * nub * H * LB) * 4u, sstride = (unsigned)(H * LB) * 4u;
      unsigned o[2];
      float acc[2] = {0.f, 0.f};
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        const int q = tid + LC * k;
        o[k] = sbase + (unsigned)((j0 + q / LB) * LB + (q & (LB - 1))) * 4u;
      }
      for (int u0 = 0; u0 < nub; u0 += 16) {
        float v[2][16];
#pragma unroll
        for (int u = 0; u < 16; ++u)
#pragma unroll
          for (int k = 0; k < 2; ++k)
            v[k][u] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(
                rsP, (int)(u0 + u < nub ? o[k] + (unsigned)(u0 + u) * sstride : kIoOOB), 0, 16));   // aux 16 = sc1
#pragma unroll
        for (int u = 0; u < 16; ++u)
#pragma unroll
          for (int k = 0; k < 2; ++k) acc[k] += v[k][u];
      }
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        const int q = tid + LC * k;
        sR[(q & (LB - 1)) * LJ + q / LB] = acc[k];
      }
      clk.mark(3);
    }
    lds_barrier();
    {
      const int b = tid / LJ, jj = tid % LJ;
      if (b < p.B) dhcarry += sR[b * LJ + jj];
      clk.mark(4);
    }
  }
  clk.flush(p.prof, 5);
}


inline Knob kn_lstm_v2("lstm_v2", 2);   // 0: round-1 kernels, 1: role-split v2, 2 (default): v2 forward + partial-exchange backward
inline Knob kn_lstm_prof("lstm_prof", 0);   // phase clocks of the v2 recurrences into sync[4:20] (tools/lstm_micro.py)

// ------------------------------------------------------------------------------- host
static int ew_grid(int64_t n) { return (int)std::max<int64_t>(1, std::min<int64_t>(4096, (n + 255) / 256)); }

at::Tensor embedding_fwd(const at::Tensor& ids, const at::Tensor& W) {
  if (W.scalar_type() == at::kFloat) return f32::embedding_fwd(ids, W);
  PCMP_CHECK_CUDA(ids); PCMP_CHECK_BF16(W); PCMP_CHECK_CONTIG(W);
  TORCH_CHECK(ids.scalar_type() == at::kLong, "ids int64");
  const int E = W.size(1);
  TORCH_CHECK(E % 8 == 0, "embedding dim % 8");
  auto idc = ids.contiguous();
  auto sizes = idc.sizes().vec();
  sizes.push_back(E);
  auto out = at::empty(sizes, W.options());
  const int64_t rows = idc.numel();
  hipLaunchKernelGGL(embedding_fwd_kernel, dim3(ew_grid(rows * E / 8)), dim3(256), 0, cur_stream(), idc.data_ptr<int64_t>(),
                     ptr<__bf16>(W), ptr<__bf16>(out), rows, E);
  PCMP_LAUNCH_CHECK();
  return out;
}

void embedding_bwd(const at::Tensor& ids, const at::Tensor& dy, at::Tensor dW, int64_t padding_idx, bool accumulate) {
  if (dy.scalar_type() == at::kFloat) return f32::embedding_bwd(ids, dy, dW, padding_idx, accumulate);
  PCMP_CHECK_BF16(dy); PCMP_CHECK_F32(dW);
  auto idc = ids.contiguous();
  auto dyc = dy.contiguous();
  const int E = dW.size(-1);
  if (!accumulate) dW.zero_();
  const int64_t rows = idc.numel();
  if (rows == 0) return;
  if (kn_emb_atomic.get()) {
    hipLaunchKernelGGL(embedding_bwd_kernel, dim3(ew_grid(rows * E)), dim3(256), 0, cur_stream(), idc.data_ptr<int64_t>(),
                       ptr<__bf16>(dyc), ptr<float>(dW), rows, E, padding_idx);
  } else {
    embedding_bwd_det<__bf16>(idc, ptr<__bf16>(dyc), ptr<float>(dW), dW.size(0), E, padding_idx, cur_stream());
  }
  PCMP_LAUNCH_CHECK();
}

at::Tensor masked_mean_fwd(const at::Tensor& x, const at::Tensor& ids) {
  if (x.scalar_type() == at::kFloat) return f32::masked_mean_fwd(x, ids);
  PCMP_CHECK_BF16(x); PCMP_CHECK_CONTIG(x);
  const int B = x.size(0), S = x.size(1), D = x.size(2);
  auto y = at::empty({B, D}, x.options());
  auto idc = ids.contiguous();
  hipLaunchKernelGGL(masked_mean_fwd_kernel, dim3(B), dim3(256), 0, cur_stream(), ptr<__bf16>(x), idc.data_ptr<int64_t>(),
                     B, S, D, ptr<__bf16>(y));
  PCMP_LAUNCH_CHECK();
  return y;
}

at::Tensor masked_mean_bwd(const at::Tensor& dy, const at::Tensor& ids, int64_t S) {
  if (dy.scalar_type() == at::kFloat) return f32::masked_mean_bwd(dy, ids, S);
  PCMP_CHECK_BF16(dy);
  const int B = dy.size(0), D = dy.size(1);
  auto dx = at::empty({B, S, D}, dy.options());
  auto idc = ids.contiguous();
  auto dyc = dy.contiguous();
  hipLaunchKernelGGL(masked_mean_bwd_kernel, dim3(B), dim3(256), 0, cur_stream(), ptr<__bf16>(dyc),
                     idc.data_ptr<int64_t>(), B, (int)S, D, ptr<__bf16>(dx));
  PCMP_LAUNCH_CHECK();
  return dx;
}

static void check_lstm_shapes(int B, int H) {
  TORCH_CHECK(B <= LB, "lstm: per-launch batch must be <= 32 (host splits larger batches)");
  TORCH_CHECK(H % LJ == 0 && H % 32 == 0 && H <= 512, "lstm: hidden size must be a multiple of 32, <= 512");
}

// gx [B][S][2][4H] bf16 (input projection incl. biases), whh [2][4H][H] bf16, ids [B][S]
// -> [hout bf16 [B][S][2H], gates f32 [B][S][2][4H], c f32 [B][S][2][H]]
std::vector<at::Tensor> lstm_seq_fwd(const at::Tensor& gx, const at::Tensor& whh, const at::Tensor& ids) {
  if (gx.scalar_type() == at::kFloat) return f32::lstm_seq_fwd(gx, whh, ids);
  PCMP_CHECK_BF16(gx); PCMP_CHECK_CONTIG(gx); PCMP_CHECK_BF16(whh); PCMP_CHECK_CONTIG(whh);
  const int B = gx.size(0), S = gx.size(1), H = whh.size(2);
  check_lstm_shapes(B, H);
  TORCH_CHECK(gx.size(2) == 2 && gx.size(3) == 4 * H, "lstm_seq_fwd: gx shape");
  auto idc = ids.contiguous();
  auto hout = at::empty({B, S, 2 * H}, whh.options());
  auto f32 = gx.options().dtype(at::kFloat);
  auto gates = at::empty({B, S, 2, 4 * H}, f32);
  auto cst = at::empty({B, S, 2, H}, f32);
  auto hbuf = at::empty({2, 2, LB, H}, whh.options());
  const bool prof = kn_lstm_prof.get() != 0;
  auto sync = at::zeros({prof ? 4 + 16 : 4}, gx.options().dtype(at::kInt));
  LstmFwdParams p{ptr<__bf16>(gx), ptr<__bf16>(whh), idc.data_ptr<int64_t>(), ptr<__bf16>(hout), ptr<float>(gates),
                  ptr<float>(cst), ptr<__bf16>(hbuf), reinterpret_cast<unsigned*>(sync.data_ptr()),
                  reinterpret_cast<unsigned*>(sync.data_ptr()) + 2, B, S, H,
                  prof ? reinterpret_cast<unsigned long long*>(reinterpret_cast<int*>(sync.data_ptr()) + 4) : nullptr};
  const size_t smem2 = (size_t)4 * LJ * H * 2 + (size_t)LB * H * 2 + (size_t)4 * LB * 4 * LJ * 4 +
                       (size_t)LB * LJ * 4 + (size_t)LB * LJ * 2 + (2 * LB + 1) * 4;
  // v2: the exchange tile [LB][H] is gathered in whole 256-thread passes of 16-B chunks; the IO
  // buffer resources take 32-bit byte offsets
  if (kn_lstm_v2.get() && smem2 <= 160 * 1024 && (LB * H / 8) % LC == 0 && gates.numel() * 4 < (1ll << 31)) {
    static bool attr = false;
    if (!attr) {
      PCMP_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(&lstm_fwd_persistent2),
                                         hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
      attr = true;
    }
    hipLaunchKernelGGL(lstm_fwd_persistent2, dim3(2 * (H / LJ)), dim3(LT2), smem2, cur_stream(), p);
    PCMP_LAUNCH_CHECK();
    return {hout, gates, cst, sync};
  }
  const size_t smem = (size_t)4 * LJ * H * 2 + (size_t)LB * H * 2 + (size_t)LB * 4 * LJ * 4 + (size_t)LB * LJ * 2;
  TORCH_CHECK(smem <= 160 * 1024, "lstm_seq_fwd: LDS budget exceeded");
  hipLaunchKernelGGL(lstm_fwd_persistent, dim3(2 * (H / LJ)), dim3(LT), smem, cur_stream(), p);
  PCMP_LAUNCH_CHECK();
  return {hout, gates, cst, sync};
}

// -> dgates bf16 [B][S][2][4H]  (and the sync/error words)
std::vector<at::Tensor> lstm_seq_bwd(const at::Tensor& dhout, const at::Tensor& gates, const at::Tensor& cst,
                                     const at::Tensor& whh, const at::Tensor& ids) {
  if (whh.scalar_type() == at::kFloat) return f32::lstm_seq_bwd(dhout, gates, cst, whh, ids);
  PCMP_CHECK_BF16(dhout); PCMP_CHECK_F32(gates); PCMP_CHECK_F32(cst);
  const int B = gates.size(0), S = gates.size(1), H = whh.size(2);
  check_lstm_shapes(B, H);
  auto idc = ids.contiguous();
  auto dh = dhout.contiguous();
  auto dgates = at::empty({B, S, 2, 4 * H}, whh.options());
  auto dgbuf = at::empty({2, 2, LB, 4 * H}, whh.options());
  const bool prof = kn_lstm_prof.get() != 0;
  auto sync = at::zeros({prof ? 4 + 16 : 4}, gates.options().dtype(at::kInt));
  LstmBwdParams p{ptr<float>(gates), ptr<float>(cst), ptr<__bf16>(whh), idc.data_ptr<int64_t>(), ptr<__bf16>(dh),
                  ptr<__bf16>(dgates), ptr<__bf16>(dgbuf), reinterpret_cast<unsigned*>(sync.data_ptr()),
                  reinterpret_cast<unsigned*>(sync.data_ptr()) + 2, B, S, H,
                  prof ? reinterpret_cast<unsigned long long*>(reinterpret_cast<int*>(sync.data_ptr()) + 4) : nullptr};
  const size_t smem2 = (size_t)LJ * 4 * H * 2 + (size_t)LB * LJ * 4 + (size_t)LB * 4 * LJ * 2 +
                       (size_t)2 * 7 * LB * LJ * 4 + (2 * LB + 1) * 4;
  if (kn_lstm_v2.get() == 2 && smem2 <= 160 * 1024 && gates.numel() * 4 < (1ll << 31)) {
    static bool attr3 = false;
    if (!attr3) {
      PCMP_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(&lstm_bwd_persistent3),
                                         hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
      attr3 = true;
    }
    auto pbuf = at::empty({2, 2, H / LJ, H, LB}, gates.options());   // fp32 partial-sum exchange
    p.dgbuf = reinterpret_cast<__bf16*>(pbuf.data_ptr<float>());
    hipLaunchKernelGGL(lstm_bwd_persistent3, dim3(2 * (H / LJ)), dim3(LT2), smem2, cur_stream(), p);
    PCMP_LAUNCH_CHECK();
    return {dgates, sync};
  }
  if (kn_lstm_v2.get() && smem2 <= 160 * 1024 && (LB * 4 * H / 8) % LC == 0 && gates.numel() * 4 < (1ll << 31)) {
    static bool attr = false;
    if (!attr) {
      PCMP_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(&lstm_bwd_persistent2),
                                         hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
      attr = true;
    }
    hipLaunchKernelGGL(lstm_bwd_persistent2, dim3(2 * (H / LJ)), dim3(LT2), smem2, cur_stream(), p);
    PCMP_LAUNCH_CHECK();
    return {dgates, sync};
  }
  const size_t smem = (size_t)LJ * 4 * H * 2 + (size_t)LB * 4 * H * 2 + (size_t)LB * LJ * 4 + (size_t)LB * 4 * LJ * 2;
  TORCH_CHECK(smem <= 160 * 1024, "lstm_seq_bwd: LDS budget exceeded");
  hipLaunchKernelGGL(lstm_bwd_persistent, dim3(2 * (H / LJ)), dim3(LT), smem, cur_stream(), p);
  PCMP_LAUNCH_CHECK();
  return {dgates, sync};
}

}  // namespace pcmp

TORCH_LIBRARY_FRAGMENT(pcmp, m) {
  m.def("embedding_fwd(Tensor ids, Tensor W) -> Tensor", &pcmp::embedding_fwd);
  m.def("embedding_bwd(Tensor ids, Tensor dy, Tensor(a!) dW, int padding_idx, bool accumulate) -> ()",
        &pcmp::embedding_bwd);
  m.def("masked_mean_fwd(Tensor x, Tensor ids) -> Tensor", &pcmp::masked_mean_fwd);
  m.def("masked_mean_bwd(Tensor dy, Tensor ids, int S) -> Tensor", &pcmp::masked_mean_bwd);
  m.def("lstm_seq_fwd(Tensor gx, Tensor whh, Tensor ids) -> Tensor[]", &pcmp::lstm_seq_fwd);
  m.def("lstm_seq_bwd(Tensor dhout, Tensor gates, Tensor cst, Tensor whh, Tensor ids) -> Tensor[]", &pcmp::lstm_seq_bwd);
}

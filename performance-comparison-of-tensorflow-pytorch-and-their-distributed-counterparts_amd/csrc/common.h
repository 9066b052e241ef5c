// Shared device/host helpers for every CDNA4 (gfx950) kernel in this framework.
//
// Conventions used across csrc/:
//   * activations are NHWC (channels-last) bf16, weights KRSC ([Cout][kh][kw][Cin]) bf16 for
//     compute with an fp32 master copy owned by the optimizer;
//   * per-channel statistics / gradients are fp32;
//   * every launch goes on the current PyTorch HIP stream so ops compose with torch's own
//     kernels, RCCL and hipGraph capture (no host syncs, no allocation inside launches other
//     than through the torch caching allocator).
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>
#include <atomic>
#include <cstdint>

namespace pcmp {

// Runtime tuning knob (kernel-variant switches for in-process A/B measurements, cdna_hip_programming
// §5.4 rule 24): a named integer, registered at static-initialisation time, read with one relaxed
// atomic load per launch, set from Python with torch.ops.pcmp.set_knob(name, value).  The default
// is the measured-best variant; nothing in a training step changes a knob.
struct Knob {
  const char* name;
  std::atomic<int> value;
  Knob(const char* n, int dflt);
  int get() const { return value.load(std::memory_order_relaxed); }
};

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef unsigned short u16x8 __attribute__((ext_vector_type(8)));
typedef unsigned short u16x4 __attribute__((ext_vector_type(4)));

constexpr int kWave = 64;

__device__ __forceinline__ float bf2f(unsigned short u) {
  return __uint_as_float(((unsigned)u) << 16);
}
// round-to-nearest-even f32 -> bf16: the gfx950 hardware conversion (v_cvt_pk_bf16_f32, NaN-safe)
__device__ __forceinline__ unsigned short f2bf(float f) {
  return __builtin_bit_cast(unsigned short, (__bf16)f);
}
// two floats -> packed bf16 pair (one v_cvt_pk_bf16_f32): low half = a, high half = b
typedef float f32x2_t __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ unsigned f2bf2(float a, float b) {
  return __builtin_bit_cast(unsigned, __builtin_convertvector((f32x2_t){a, b}, bf16x2_t));
}

// erf-GELU and its derivative (BERT's hidden activation); shared by the GELU kernels and the
// GEMM epilogues that fuse it (igemm.hip act 2 / 3)
__device__ __forceinline__ float gelu_erf(float x) { return 0.5f * x * (1.f + erff(x * 0.70710678118654752f)); }
__device__ __forceinline__ float dgelu_erf(float x) {
  const float cdf = 0.5f * (1.f + erff(x * 0.70710678118654752f));
  const float pdf = 0.3989422804014327f * __expf(-0.5f * x * x);
  return cdf + x * pdf;
}

// bf16-epilogue GELU: erf by Abramowitz-Stegun 7.1.26 (|error| <= 1.5e-7, far below the bf16
// rounding of the stored value), branch-free: one reciprocal, one exp2, five FMAs -- the library
// erff is ~45 instructions over two divergent branches.  The exp(-x^2/2) term is shared with the
// derivative.  fp32 kernels (text_f32.hip) keep erff.
__device__ __forceinline__ float erf_as_core(float a, float e) {   // a = |z|, e = exp(-z^2)
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, a, 1.f));
  float y = fmaf(1.061405429f, t, -1.453152027f);
  y = fmaf(y, t, 1.421413741f);
  y = fmaf(y, t, -0.284496736f);
  y = fmaf(y, t, 0.254829592f);
  return 1.f - y * t * e;
}
__device__ __forceinline__ float gelu_fast(float x) {
  const float z = x * 0.70710678118654752f;
  const float e = __expf(-z * z);
  const float er = copysignf(erf_as_core(fabsf(z), e), x);
  return 0.5f * x * (1.f + er);
}
__device__ __forceinline__ float dgelu_fast(float x) {
  const float z = x * 0.70710678118654752f;
  const float e = __expf(-z * z);   // = exp(-x^2 / 2)
  const float er = copysignf(erf_as_core(fabsf(z), e), x);
  return 0.5f * (1.f + er) + x * 0.3989422804014327f * e;
}

__device__ __forceinline__ float warp_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float warp_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Block-wide sum for blockDim.x a multiple of 64 (<= 1024). `sh` needs >= 16 floats.
__device__ __forceinline__ float block_sum(float v, float* sh) {
  v = warp_sum(v);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  __syncthreads();
  if (lane == 0) sh[wid] = v;
  __syncthreads();
  float r = 0.f;
  for (int i = 0; i < nw; ++i) r += sh[i];
  return r;
}

// Counter-based hash RNG (stateless): used for dropout so backward regenerates the mask
// from (seed, offset, index) instead of storing it.  32-bit "lowbias32" finaliser rounds: the high
// index word (eager dropout's per-call counter, offset = counter << 32) is mixed with the folded
// 64-bit seed by one round, and that per-call key is XORed into the low word before a second round.
// (Round 4 folded both words into ONE round: every call's mask was then an XOR relabelling of the
// same bijective sequence, and two calls whose keys differed by less than numel drew index
// permutations of one mask; tests/test_transformer_gpu.py checks consecutive calls are uncorrelated.)
// Two 32-bit multiplies per round where splitmix64 needed three 64-bit ones (~40 VALU ops).
// ops/ref.py hash_uniform is the bit-exact torch port.
__device__ __forceinline__ uint32_t lowbias32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7FEB352Du;
  x ^= x >> 15;
  x *= 0x846CA68Bu;
  x ^= x >> 16;
  return x;
}
__device__ __forceinline__ uint32_t hash_u32(uint64_t seed, uint64_t idx) {
  const uint32_t key = (uint32_t)seed ^ ((uint32_t)(seed >> 32) * 0x9E3779B9u);
  return lowbias32((uint32_t)idx ^ lowbias32((uint32_t)(idx >> 32) ^ key));
}
__device__ __forceinline__ float uniform01(uint64_t seed, uint64_t idx) {
  return (hash_u32(seed, idx) >> 8) * (1.0f / 16777216.0f);
}

// Dropout seed with an optional device-side salt: a captured hipGraph replays its kernels with the
// arguments of the capture, so a training step replayed from a graph reads a per-replay counter
// (incremented by the step itself) to draw a new mask every step; eager launches pass no salt.
__device__ __forceinline__ uint64_t dropout_seed(uint64_t seed, const int64_t* salt) {
  return salt ? seed + (uint64_t)salt[0] * 0x9E3779B97F4A7C15ull : seed;
}
inline const int64_t* salt_ptr(const c10::optional<at::Tensor>& t) {
  if (!t.has_value() || !t->defined()) return nullptr;
  TORCH_CHECK(t->is_cuda() && t->scalar_type() == at::kLong && t->numel() >= 1, "dropout salt: int64 GPU tensor");
  return t->data_ptr<int64_t>();
}

inline hipStream_t cur_stream() { return c10::hip::getCurrentHIPStream().stream(); }

inline int ceil_div(int64_t a, int64_t b) { return (int)((a + b - 1) / b); }

#define PCMP_CHECK_CUDA(x) TORCH_CHECK((x).is_cuda(), #x " must be a GPU tensor")
#define PCMP_CHECK_CONTIG(x) TORCH_CHECK((x).is_contiguous(), #x " must be contiguous")
#define PCMP_CHECK_BF16(x) TORCH_CHECK((x).scalar_type() == at::kBFloat16, #x " must be bf16")
#define PCMP_CHECK_F32(x) TORCH_CHECK((x).scalar_type() == at::kFloat, #x " must be fp32")
#define PCMP_LAUNCH_CHECK() C10_HIP_KERNEL_LAUNCH_CHECK()
#define PCMP_HIP_CHECK(expr)                                                                  \
  do {                                                                                        \
    const hipError_t e_ = (expr);                                                             \
    TORCH_CHECK(e_ == hipSuccess, #expr " failed: ", hipGetErrorString(e_));                  \
  } while (0)
// Launches whose dynamic LDS may exceed 64 KB need the per-kernel opt-in (once per call site).
#define PCMP_ALLOW_BIG_LDS(kfn)                                                                             \
  do {                                                                                                    \
    static const bool pcmp_lds_ = [] {                                                                    \
      PCMP_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(&kfn),                             \
                                         hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));        \
      return true;                                                                                        \
    }();                                                                                                  \
    (void)pcmp_lds_;                                                                                      \
  } while (0)

template <typename T>
inline T* ptr(const at::Tensor& t) { return reinterpret_cast<T*>(t.data_ptr()); }
template <typename T>
inline T* optr(const c10::optional<at::Tensor>& t) {
  return (t.has_value() && t->defined()) ? reinterpret_cast<T*>(t->data_ptr()) : nullptr;
}

// Deterministic column reduction of fp32 partials: out[l] (+)= sum_t part[t][l]  (L % 4 == 0).
// Defined in elementwise.hip; shared by the bias-gradient and LayerNorm-backward reductions.
void launch_col_reduce(const float* part, int T, int L, float* out, bool accumulate, hipStream_t st,
                       float* out2 = nullptr, int L1 = -1);

}  // namespace pcmp

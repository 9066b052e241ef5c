// Embedding backward shared by the bf16 (rnn.hip) and fp32 (text_f32.hip) paths.
// dW[ids[r]][:] += dy[r][:] for every row r whose id is not padding_idx.
#pragma once
#include "common.h"

namespace pcmp {

extern Knob kn_emb_atomic;   // 1: the round-4 fp32-atomic kernels (order of the adds not fixed)

// Deterministic form (default; knob emb_atomic = 1 restores the atomics): the rows sorted by id with
// a STABLE sort (equal ids keep their row order); block i handles the segment that starts at sorted
// position i (every other block returns at once) and adds its rows in that fixed order -- one writer
// per vocabulary row, the same bits on every run (SURVEY §5.2 deterministic mode).
template <typename T>
__global__ void __launch_bounds__(256) embedding_bwd_seg_kernel(const int64_t* __restrict__ sid,
                                                                const int64_t* __restrict__ perm,
                                                                const T* __restrict__ dy, float* __restrict__ dW,
                                                                int64_t rows, int E, int64_t padding_idx) {
  const int64_t i = blockIdx.x;
  const int64_t id = sid[i];
  if (id == padding_idx || (i > 0 && sid[i - 1] == id)) return;
  int64_t end = i + 1;
  while (end < rows && sid[end] == id) ++end;
  for (int e = threadIdx.x; e < E; e += blockDim.x) {
    float s = 0.f;
    for (int64_t r = i; r < end; ++r) {
      const T v = dy[perm[r] * E + e];
      if constexpr (sizeof(T) == 2) s += bf2f(__builtin_bit_cast(unsigned short, v));
      else s += v;
    }
    dW[id * E + e] += s;
  }
}

// Packed-key form of the same reduction (rows <= 16384 and ids < 2^(32 - pbits)): the stable sort is
// ONE workgroup's bitonic sort of 32-bit keys (id << pbits | row) in LDS -- the row in the low bits
// makes equal ids keep their row order -- instead of the library's 64-bit key/value radix sort
// (40 us per call at 4,096 tokens; round-5 ADVICE: the deterministic backward cost BERT 0.9 % and the
// BiLSTM 2.1 % of a step against the atomic form, profiles/r6_emb_atomic_ab.txt).
constexpr int kEmbSortMax = 16384;
static __global__ void __launch_bounds__(1024) embedding_sort_kernel(const int64_t* __restrict__ ids, int rows, int pbits,
                                                               unsigned* __restrict__ keys) {
  __shared__ unsigned k[kEmbSortMax];
  int n2 = 1;
  while (n2 < rows) n2 <<= 1;
  for (int i = threadIdx.x; i < n2; i += blockDim.x)
    k[i] = i < rows ? (unsigned)(ids[i] << pbits) | (unsigned)i : 0xffffffffu;
  __syncthreads();
  for (int size = 2; size <= n2; size <<= 1)
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int t = threadIdx.x; t < n2 / 2; t += blockDim.x) {
        const int i = 2 * t - (t & (stride - 1)), j = i + stride;   // pair (i, j), i's bit `stride` clear
        const bool up = (i & size) == 0;
        const unsigned a = k[i], b = k[j];
        if ((a > b) == up) { k[i] = b; k[j] = a; }
      }
      __syncthreads();
    }
  for (int i = threadIdx.x; i < rows; i += blockDim.x) keys[i] = k[i];
}

template <typename T>
__global__ void __launch_bounds__(256) embedding_bwd_key_kernel(const unsigned* __restrict__ keys, int pbits,
                                                                const T* __restrict__ dy, float* __restrict__ dW,
                                                                int rows, int E, int64_t padding_idx) {
  const int i = blockIdx.x;
  const unsigned id = keys[i] >> pbits, pmask = (1u << pbits) - 1u;
  if ((int64_t)id == padding_idx || (i > 0 && (keys[i - 1] >> pbits) == id)) return;
  int end = i + 1;
  while (end < rows && (keys[end] >> pbits) == id) ++end;
  for (int e = threadIdx.x; e < E; e += blockDim.x) {
    float s = 0.f;
    for (int r = i; r < end; ++r) {
      const T v = dy[(int64_t)(keys[r] & pmask) * E + e];
      if constexpr (sizeof(T) == 2) s += bf2f(__builtin_bit_cast(unsigned short, v));
      else s += v;
    }
    dW[(int64_t)id * E + e] += s;
  }
}

// deterministic embedding backward (both precisions): packed-key sort when it fits, else the
// library stable sort + embedding_bwd_seg_kernel
template <typename T>
inline void embedding_bwd_det(const at::Tensor& idc, const T* dy, float* dW, int64_t V, int E, int64_t padding_idx,
                              hipStream_t st) {
  const int64_t rows = idc.numel();
  int pbits = 1;
  while ((1ll << pbits) < rows) ++pbits;
  if (rows <= kEmbSortMax && V <= (1ll << (32 - pbits)) - 1) {
    auto keys = at::empty({rows}, idc.options().dtype(at::kInt));
    hipLaunchKernelGGL(embedding_sort_kernel, dim3(1), dim3(1024), 0, st, idc.data_ptr<int64_t>(), (int)rows, pbits,
                       reinterpret_cast<unsigned*>(keys.data_ptr<int>()));
    hipLaunchKernelGGL(embedding_bwd_key_kernel<T>, dim3((unsigned)rows), dim3(256), 0, st,
                       reinterpret_cast<const unsigned*>(keys.data_ptr<int>()), pbits, dy, dW, (int)rows, E, padding_idx);
    return;
  }
  auto sorted = at::sort(idc.reshape({-1}), /*stable=*/true, /*dim=*/0, /*descending=*/false);
  const at::Tensor sid = std::get<0>(sorted).contiguous(), perm = std::get<1>(sorted).contiguous();
  hipLaunchKernelGGL(embedding_bwd_seg_kernel<T>, dim3(rows), dim3(256), 0, st, sid.data_ptr<int64_t>(),
                     perm.data_ptr<int64_t>(), dy, dW, rows, E, padding_idx);
}

}  // namespace pcmp

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

}  // namespace pcmp

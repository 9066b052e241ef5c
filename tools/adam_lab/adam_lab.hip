// Standalone bandwidth lab for the fused AdamW step over a flat 110 M-parameter buffer (BERT-base):
// variants of the update kernel, timed with hip events.  Build: hipcc --offload-arch=gfx950 -O3
// adam_lab.hip -o adam_lab ; run: ./adam_lab
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cmath>
#include <vector>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned short u16x4 __attribute__((ext_vector_type(4)));
#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

__device__ __forceinline__ unsigned short f2bf(float f) {
  unsigned u = __float_as_uint(f);
  u += 0x7fffu + ((u >> 16) & 1u);
  return (unsigned short)(u >> 16);
}

struct Args {
  float* w; const float* g; float* m1; float* m2; unsigned short* sh; long n;
  float lr, b1, b2, eps, wd, step_size, bc2s;
};

// V0: the shipped form (IEEE sqrt / div, one vec4 per thread per iteration)
__global__ void adam_v0(Args a) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < a.n / 4; i += (long)gridDim.x * blockDim.x) {
    f32x4 wv = reinterpret_cast<f32x4*>(a.w)[i];
    const f32x4 gv = reinterpret_cast<const f32x4*>(a.g)[i];
    f32x4 m = reinterpret_cast<f32x4*>(a.m1)[i];
    f32x4 v = reinterpret_cast<f32x4*>(a.m2)[i];
    u16x4 s;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      wv[e] *= (1.f - a.lr * a.wd);
      m[e] = a.b1 * m[e] + (1.f - a.b1) * gv[e];
      v[e] = a.b2 * v[e] + (1.f - a.b2) * gv[e] * gv[e];
      const float denom = sqrtf(v[e]) / a.bc2s + a.eps;
      wv[e] -= a.step_size * m[e] / denom;
      s[e] = f2bf(wv[e]);
    }
    reinterpret_cast<f32x4*>(a.w)[i] = wv;
    reinterpret_cast<f32x4*>(a.m1)[i] = m;
    reinterpret_cast<f32x4*>(a.m2)[i] = v;
    reinterpret_cast<u16x4*>(a.sh)[i] = s;
  }
}

// V1: same math, two vec4 per thread per iteration (loads of both issued first)
__global__ void adam_v1(Args a) {
  const long nv = a.n / 4, st = (long)gridDim.x * blockDim.x;
  long i = blockIdx.x * (long)blockDim.x + threadIdx.x;
  for (; i < nv; i += 2 * st) {
    const long j = i + st < nv ? i + st : i;
    f32x4 wv[2] = {reinterpret_cast<f32x4*>(a.w)[i], reinterpret_cast<f32x4*>(a.w)[j]};
    const f32x4 gv[2] = {reinterpret_cast<const f32x4*>(a.g)[i], reinterpret_cast<const f32x4*>(a.g)[j]};
    f32x4 m[2] = {reinterpret_cast<f32x4*>(a.m1)[i], reinterpret_cast<f32x4*>(a.m1)[j]};
    f32x4 v[2] = {reinterpret_cast<f32x4*>(a.m2)[i], reinterpret_cast<f32x4*>(a.m2)[j]};
    u16x4 s[2];
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        wv[u][e] *= (1.f - a.lr * a.wd);
        m[u][e] = a.b1 * m[u][e] + (1.f - a.b1) * gv[u][e];
        v[u][e] = a.b2 * v[u][e] + (1.f - a.b2) * gv[u][e] * gv[u][e];
        const float denom = sqrtf(v[u][e]) / a.bc2s + a.eps;
        wv[u][e] -= a.step_size * m[u][e] / denom;
        s[u][e] = f2bf(wv[u][e]);
      }
    reinterpret_cast<f32x4*>(a.w)[i] = wv[0];
    reinterpret_cast<f32x4*>(a.m1)[i] = m[0];
    reinterpret_cast<f32x4*>(a.m2)[i] = v[0];
    reinterpret_cast<u16x4*>(a.sh)[i] = s[0];
    if (j != i) {
      reinterpret_cast<f32x4*>(a.w)[j] = wv[1];
      reinterpret_cast<f32x4*>(a.m1)[j] = m[1];
      reinterpret_cast<f32x4*>(a.m2)[j] = v[1];
      reinterpret_cast<u16x4*>(a.sh)[j] = s[1];
    }
  }
}

// V2: V0 with fast reciprocal forms (v_sqrt / v_rcp, ~1 ulp) instead of IEEE sqrt + two divisions
__global__ void adam_v2(Args a) {
  const float ibc2s = 1.f / a.bc2s;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < a.n / 4; i += (long)gridDim.x * blockDim.x) {
    f32x4 wv = reinterpret_cast<f32x4*>(a.w)[i];
    const f32x4 gv = reinterpret_cast<const f32x4*>(a.g)[i];
    f32x4 m = reinterpret_cast<f32x4*>(a.m1)[i];
    f32x4 v = reinterpret_cast<f32x4*>(a.m2)[i];
    u16x4 s;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      wv[e] *= (1.f - a.lr * a.wd);
      m[e] = a.b1 * m[e] + (1.f - a.b1) * gv[e];
      v[e] = a.b2 * v[e] + (1.f - a.b2) * gv[e] * gv[e];
      const float denom = __builtin_amdgcn_sqrtf(v[e]) * ibc2s + a.eps;
      wv[e] -= a.step_size * m[e] * __builtin_amdgcn_rcpf(denom);
      s[e] = f2bf(wv[e]);
    }
    reinterpret_cast<f32x4*>(a.w)[i] = wv;
    reinterpret_cast<f32x4*>(a.m1)[i] = m;
    reinterpret_cast<f32x4*>(a.m2)[i] = v;
    reinterpret_cast<u16x4*>(a.sh)[i] = s;
  }
}

// V3: V0 with nontemporal loads / stores (streamed once per step)
__global__ void adam_v3(Args a) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < a.n / 4; i += (long)gridDim.x * blockDim.x) {
    f32x4 wv = __builtin_nontemporal_load(reinterpret_cast<f32x4*>(a.w) + i);
    const f32x4 gv = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(a.g) + i);
    f32x4 m = __builtin_nontemporal_load(reinterpret_cast<f32x4*>(a.m1) + i);
    f32x4 v = __builtin_nontemporal_load(reinterpret_cast<f32x4*>(a.m2) + i);
    u16x4 s;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      wv[e] *= (1.f - a.lr * a.wd);
      m[e] = a.b1 * m[e] + (1.f - a.b1) * gv[e];
      v[e] = a.b2 * v[e] + (1.f - a.b2) * gv[e] * gv[e];
      const float denom = sqrtf(v[e]) / a.bc2s + a.eps;
      wv[e] -= a.step_size * m[e] / denom;
      s[e] = f2bf(wv[e]);
    }
    __builtin_nontemporal_store(wv, reinterpret_cast<f32x4*>(a.w) + i);
    __builtin_nontemporal_store(m, reinterpret_cast<f32x4*>(a.m1) + i);
    __builtin_nontemporal_store(v, reinterpret_cast<f32x4*>(a.m2) + i);
    __builtin_nontemporal_store(s, reinterpret_cast<u16x4*>(a.sh) + i);
  }
}

// copy reference: w -> m1 (read 4 B + write 4 B per element)
__global__ void copy_ref(Args a) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < a.n / 4; i += (long)gridDim.x * blockDim.x)
    reinterpret_cast<f32x4*>(a.m1)[i] = reinterpret_cast<const f32x4*>(a.w)[i];
}

int main() {
  const long n = 109482240;   // BERT-base + classifier, rounded to a multiple of 4
  Args a{};
  CK(hipMalloc(&a.w, n * 4)); CK(hipMalloc((void**)&a.g, n * 4)); CK(hipMalloc(&a.m1, n * 4));
  CK(hipMalloc(&a.m2, n * 4)); CK(hipMalloc(&a.sh, n * 2));
  CK(hipMemset(a.w, 0, n * 4)); CK(hipMemset((void*)a.g, 0, n * 4)); CK(hipMemset(a.m1, 0, n * 4));
  CK(hipMemset(a.m2, 0, n * 4));
  a.n = n; a.lr = 2e-5f; a.b1 = 0.9f; a.b2 = 0.999f; a.eps = 1e-8f; a.wd = 0.01f; a.step_size = 2e-5f; a.bc2s = 0.1f;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  struct V { const char* name; void (*k)(Args); int grid; double bytes; };
  const double adam_b = 30.0 * n, copy_b = 8.0 * n;
  std::vector<V> vs = {
      {"copy_ref g2048", copy_ref, 2048, copy_b},   {"copy_ref g8192", copy_ref, 8192, copy_b},
      {"v0 g2048", adam_v0, 2048, adam_b},           {"v0 g4096", adam_v0, 4096, adam_b},
      {"v0 g8192", adam_v0, 8192, adam_b},           {"v0 g1024", adam_v0, 1024, adam_b},
      {"v1 g2048", adam_v1, 2048, adam_b},           {"v1 g1024", adam_v1, 1024, adam_b},
      {"v2 g2048", adam_v2, 2048, adam_b},           {"v2 g8192", adam_v2, 8192, adam_b},
      {"v3 g2048", adam_v3, 2048, adam_b},           {"v3 g8192", adam_v3, 8192, adam_b},
  };
  for (int round = 0; round < 2; ++round)
    for (auto& v : vs) {
      hipLaunchKernelGGL(v.k, dim3(v.grid), dim3(256), 0, 0, a);
      CK(hipEventRecord(e0));
      for (int r = 0; r < 10; ++r) hipLaunchKernelGGL(v.k, dim3(v.grid), dim3(256), 0, 0, a);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      const double us = ms * 100.0;
      if (round) printf("%-16s %8.1f us  %5.2f TB/s\n", v.name, us, v.bytes / us / 1e6);
    }
  return 0;
}

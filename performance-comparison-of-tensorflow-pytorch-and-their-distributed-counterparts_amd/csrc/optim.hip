// Fused flat-buffer optimizers and global gradient-norm clipping.
//
// Every trainable parameter of a model lives in ONE fp32 master buffer (and its bf16 compute
// shadow in one bf16 buffer); gradients live in ONE fp32 buffer whose slices are the DDP
// all-reduce buckets.  An optimizer step is therefore a single streaming kernel over the whole
// model (ResNet-50: 25.6 M params in one launch), not a per-tensor loop:
//   sgd_flat   : torch.optim.SGD semantics (momentum, dampening, weight decay, nesterov)
//                -- Keras SGD(lr=0.001) of resnet.py:24 and the north-star SGD
//   adam_flat  : torch.optim.Adam (L2 weight decay) / AdamW (decoupled decay)
//                -- Adam(lr=3e-3) of another_neural_net.py:114,258 and HF AdamW(lr=2e-5,
//                eps=1e-8) of pytorch_on_language_distr.py:167-170
//   grad_norm  : global L2 norm over the flat gradient (clip_grad_norm_, :271-273); the clip
//                coefficient is computed ON DEVICE and consumed by the optimizer kernel through a
//                pointer, so clipping needs no host synchronisation and is graph-capturable.
// Learning rate and step count are also read through device pointers (LR schedules update a
// device scalar; hipGraph replays stay valid).  The kernels write the refreshed bf16 shadow in
// the same pass ("cast fused into the update").
#include "common.h"

namespace pcmp {

struct OptScalars {
  const float* lr;         // device scalar
  const float* gscale;     // device scalar multiplier on grads (clip coef * 1/world), may be null
  const float* step;       // device scalar (Adam bias correction), may be null
};

__device__ __forceinline__ float read_or(const float* p, float d) { return p ? *p : d; }

__global__ void sgd_flat_kernel(float* __restrict__ w, const float* __restrict__ g, float* __restrict__ mom,
                                __bf16* __restrict__ shadow, const uint8_t* __restrict__ mask, int64_t n,
                                OptScalars sc, float momentum, float dampening, float wd, int nesterov,
                                int first_step) {
  const float lr = *sc.lr, gs = read_or(sc.gscale, 1.f);
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n / 4;
       i += (int64_t)gridDim.x * blockDim.x) {
    f32x4 wv = reinterpret_cast<f32x4*>(w)[i];
    f32x4 gv = reinterpret_cast<const f32x4*>(g)[i] * gs;
    f32x4 m = momentum != 0.f ? reinterpret_cast<f32x4*>(mom)[i] : f32x4{0, 0, 0, 0};
    u16x4 sh;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const bool on = !mask || mask[i * 4 + e];
      float d = gv[e] + wd * wv[e];
      if (momentum != 0.f) {
        m[e] = first_step ? d : momentum * m[e] + (1.f - dampening) * d;
        d = nesterov ? d + momentum * m[e] : m[e];
      }
      if (on) wv[e] -= lr * d;
      sh[e] = f2bf(wv[e]);
    }
    reinterpret_cast<f32x4*>(w)[i] = wv;
    if (momentum != 0.f) reinterpret_cast<f32x4*>(mom)[i] = m;
    if (shadow) reinterpret_cast<u16x4*>(shadow)[i] = sh;
  }
}

__global__ void adam_flat_kernel(float* __restrict__ w, const float* __restrict__ g, float* __restrict__ m1,
                                 float* __restrict__ m2, __bf16* __restrict__ shadow, const uint8_t* __restrict__ mask,
                                 int64_t n, OptScalars sc, float beta1, float beta2, float eps, float wd,
                                 int decoupled) {
  const float lr = *sc.lr, gs = read_or(sc.gscale, 1.f);
  const float t = read_or(sc.step, 1.f);
  const float bc1 = 1.f - powf(beta1, t), bc2 = 1.f - powf(beta2, t);
  const float step_size = lr / bc1;
  const float bc2s = sqrtf(bc2);
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n / 4;
       i += (int64_t)gridDim.x * blockDim.x) {
    // every operand is streamed exactly once per step: nontemporal loads / stores (5.1 -> 5.5 TB/s
    // over a 110 M-parameter buffer, profiles/r4_adam_lab.txt)
    f32x4 wv = __builtin_nontemporal_load(reinterpret_cast<f32x4*>(w) + i);
    const f32x4 gv0 = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(g) + i) * gs;
    f32x4 a = __builtin_nontemporal_load(reinterpret_cast<f32x4*>(m1) + i);
    f32x4 b = __builtin_nontemporal_load(reinterpret_cast<f32x4*>(m2) + i);
    u16x4 sh;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const bool on = !mask || mask[i * 4 + e];
      float gv = gv0[e];
      if (on) {
        if (decoupled) wv[e] *= (1.f - lr * wd);
        else gv += wd * wv[e];
        a[e] = beta1 * a[e] + (1.f - beta1) * gv;
        b[e] = beta2 * b[e] + (1.f - beta2) * gv * gv;
        const float denom = sqrtf(b[e]) / bc2s + eps;
        wv[e] -= step_size * a[e] / denom;
      }
      sh[e] = f2bf(wv[e]);
    }
    __builtin_nontemporal_store(wv, reinterpret_cast<f32x4*>(w) + i);
    __builtin_nontemporal_store(a, reinterpret_cast<f32x4*>(m1) + i);
    __builtin_nontemporal_store(b, reinterpret_cast<f32x4*>(m2) + i);
    if (shadow) __builtin_nontemporal_store(sh, reinterpret_cast<u16x4*>(shadow) + i);
  }
}

// partial sums of squares -> part[blockIdx]
__global__ void sumsq_kernel(const float* __restrict__ g, int64_t n, float* __restrict__ part) {
  __shared__ float sh[16];
  float s = 0.f;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n / 4;
       i += (int64_t)gridDim.x * blockDim.x) {
    const f32x4 v = reinterpret_cast<const f32x4*>(g)[i];
    s += v[0] * v[0] + v[1] * v[1] + v[2] * v[2] + v[3] * v[3];
  }
  s = block_sum(s, sh);
  if (threadIdx.x == 0) part[blockIdx.x] = s;
}

// norm = sqrt(sum part) * pre_scale ; coef = min(1, max_norm / (norm + 1e-6)) * post_scale
__global__ void clip_coef_kernel(const float* __restrict__ part, int np, float pre_scale, float max_norm,
                                 float post_scale, float* __restrict__ norm_out, float* __restrict__ coef_out) {
  __shared__ float sh[16];
  float s = 0.f;
  for (int i = threadIdx.x; i < np; i += blockDim.x) s += part[i];
  s = block_sum(s, sh);
  if (threadIdx.x == 0) {
    const float norm = sqrtf(s) * pre_scale;
    *norm_out = norm;
    float c = max_norm > 0.f ? max_norm / (norm + 1e-6f) : 1.f;
    c = fminf(c, 1.f);
    *coef_out = c * post_scale;
  }
}

__global__ void cast_f32_bf16_kernel(const float* __restrict__ x, __bf16* __restrict__ y, int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    reinterpret_cast<unsigned short*>(y)[i] = f2bf(x[i]);
}

static int flat_grid(int64_t n) { return (int)std::max<int64_t>(1, std::min<int64_t>(2048, (n / 4 + 255) / 256)); }

void sgd_flat(at::Tensor w, const at::Tensor& g, at::Tensor mom, const c10::optional<at::Tensor>& shadow,
              const c10::optional<at::Tensor>& mask, const at::Tensor& lr, const c10::optional<at::Tensor>& gscale,
              double momentum, double dampening, double wd, bool nesterov, bool first_step) {
  PCMP_CHECK_F32(w); PCMP_CHECK_F32(g);
  const int64_t n = w.numel();
  TORCH_CHECK(n % 4 == 0 && g.numel() == n, "sgd_flat: sizes");
  OptScalars sc{ptr<float>(lr), optr<float>(gscale), nullptr};
  hipLaunchKernelGGL(sgd_flat_kernel, dim3(flat_grid(n)), dim3(256), 0, cur_stream(), ptr<float>(w), ptr<float>(g),
                     momentum != 0 ? ptr<float>(mom) : nullptr, optr<__bf16>(shadow), optr<uint8_t>(mask), n, sc,
                     (float)momentum, (float)dampening, (float)wd, (int)nesterov, (int)first_step);
  PCMP_LAUNCH_CHECK();
}

void adam_flat(at::Tensor w, const at::Tensor& g, at::Tensor m1, at::Tensor m2, const c10::optional<at::Tensor>& shadow,
               const c10::optional<at::Tensor>& mask, const at::Tensor& lr, const c10::optional<at::Tensor>& gscale,
               const at::Tensor& step, double beta1, double beta2, double eps, double wd, bool decoupled) {
  PCMP_CHECK_F32(w); PCMP_CHECK_F32(g);
  const int64_t n = w.numel();
  TORCH_CHECK(n % 4 == 0 && g.numel() == n, "adam_flat: sizes");
  OptScalars sc{ptr<float>(lr), optr<float>(gscale), ptr<float>(step)};
  hipLaunchKernelGGL(adam_flat_kernel, dim3(flat_grid(n)), dim3(256), 0, cur_stream(), ptr<float>(w), ptr<float>(g),
                     ptr<float>(m1), ptr<float>(m2), optr<__bf16>(shadow), optr<uint8_t>(mask), n, sc,
                     (float)beta1, (float)beta2, (float)eps, (float)wd, (int)decoupled);
  PCMP_LAUNCH_CHECK();
}

// returns [norm, coef] device scalars (f32)
std::vector<at::Tensor> grad_clip_coef(const at::Tensor& g, double pre_scale, double max_norm, double post_scale) {
  PCMP_CHECK_F32(g);
  const int64_t n = g.numel();
  TORCH_CHECK(n % 4 == 0, "grad_clip_coef: numel % 4");
  const int nb = flat_grid(n);
  auto part = at::empty({nb}, g.options());
  hipLaunchKernelGGL(sumsq_kernel, dim3(nb), dim3(256), 0, cur_stream(), ptr<float>(g), n, ptr<float>(part));
  PCMP_LAUNCH_CHECK();
  auto out = at::empty({2}, g.options());
  hipLaunchKernelGGL(clip_coef_kernel, dim3(1), dim3(256), 0, cur_stream(), ptr<float>(part), nb, (float)pre_scale,
                     (float)max_norm, (float)post_scale, ptr<float>(out), ptr<float>(out) + 1);
  PCMP_LAUNCH_CHECK();
  return {out[0], out[1]};
}

// Two-phase global-norm clip for the per-bucket optimizer (parallel/ddp.py): each gradient bucket's
// block partial sums of squares go to part[offset, offset + flat_grid(n)) as soon as that bucket's
// all-reduce completes; clip_coef_parts then reduces every bucket's partials in one launch.
void grad_sumsq_parts(const at::Tensor& g, at::Tensor part, int64_t offset) {
  PCMP_CHECK_F32(g); PCMP_CHECK_F32(part);
  const int64_t n = g.numel();
  TORCH_CHECK(n % 4 == 0, "grad_sumsq_parts: numel % 4");
  const int nb = flat_grid(n);
  TORCH_CHECK(offset >= 0 && offset + nb <= part.numel(), "grad_sumsq_parts: partial buffer too small");
  hipLaunchKernelGGL(sumsq_kernel, dim3(nb), dim3(256), 0, cur_stream(), ptr<float>(g), n, ptr<float>(part) + offset);
  PCMP_LAUNCH_CHECK();
}

std::vector<at::Tensor> clip_coef_parts(const at::Tensor& part, double pre_scale, double max_norm, double post_scale) {
  PCMP_CHECK_F32(part);
  auto out = at::empty({2}, part.options());
  hipLaunchKernelGGL(clip_coef_kernel, dim3(1), dim3(256), 0, cur_stream(), ptr<float>(part), (int)part.numel(),
                     (float)pre_scale, (float)max_norm, (float)post_scale, ptr<float>(out), ptr<float>(out) + 1);
  PCMP_LAUNCH_CHECK();
  return {out[0], out[1]};
}

void cast_to_bf16(const at::Tensor& x, at::Tensor y) {
  PCMP_CHECK_F32(x); PCMP_CHECK_BF16(y);
  TORCH_CHECK(x.numel() == y.numel() && x.is_contiguous() && y.is_contiguous(), "cast_to_bf16: shapes");
  const int64_t n = x.numel();
  hipLaunchKernelGGL(cast_f32_bf16_kernel, dim3((int)std::min<int64_t>(4096, (n + 255) / 256)), dim3(256), 0,
                     cur_stream(), ptr<float>(x), ptr<__bf16>(y), n);
  PCMP_LAUNCH_CHECK();
}

}  // namespace pcmp

TORCH_LIBRARY_FRAGMENT(pcmp, m) {
  m.def("sgd_flat(Tensor(a!) w, Tensor g, Tensor(b!) mom, Tensor(c!)? shadow, Tensor? mask, Tensor lr, Tensor? gscale, "
        "float momentum, float dampening, float wd, bool nesterov, bool first_step) -> ()",
        &pcmp::sgd_flat);
  m.def("adam_flat(Tensor(a!) w, Tensor g, Tensor(b!) m1, Tensor(c!) m2, Tensor(d!)? shadow, Tensor? mask, Tensor lr, "
        "Tensor? gscale, Tensor step, float beta1, float beta2, float eps, float wd, bool decoupled) -> ()",
        &pcmp::adam_flat);
  m.def("grad_clip_coef(Tensor g, float pre_scale, float max_norm, float post_scale) -> Tensor[]",
        &pcmp::grad_clip_coef);
  m.def("grad_sumsq_parts(Tensor g, Tensor(a!) part, int offset) -> ()", &pcmp::grad_sumsq_parts);
  m.def("clip_coef_parts(Tensor part, float pre_scale, float max_norm, float post_scale) -> Tensor[]",
        &pcmp::clip_coef_parts);
  m.def("cast_to_bf16(Tensor x, Tensor(a!) y) -> ()", &pcmp::cast_to_bf16);
}

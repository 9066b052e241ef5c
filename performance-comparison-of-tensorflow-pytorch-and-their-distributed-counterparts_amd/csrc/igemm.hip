// Implicit-GEMM convolution / linear kernels on CDNA4 MFMA (v_mfma_f32_16x16x32_bf16).
//
// One kernel template covers the three GEMMs of a convolution (and of a Linear layer, which is
// a 1x1 conv over [M,1,1,Cin]):
//   FWD   : Y[m=(n,p,q)][co]      = sum_{k=(r,s,ci)}  X[n,p*st-pad+r,q*st-pad+s,ci] * W[co][r][s][ci]
//   DGRAD : dX[m=(n,h,w)][ci]     = sum_{k=(r,s,co)} dY[n,(h+pad-r)/st,(w+pad-s)/st,co] * Wt[ci][r][s][co]
//   WGRAD : dW[co][j=(r,s,ci)]    = sum_{m=(n,p,q)}  dY[m][co] * X[n,p*st-pad+r,q*st-pad+s,ci]   (split-K)
// Layouts: activations NHWC bf16, weights KRSC bf16, accumulation fp32.
//
// Reference parity: these replace the cuDNN/MKL-DNN convolutions and Linear layers executed by
// torchvision ResNet-50 / VGG16 and the HF BERT / transfer heads in the reference
// (another_neural_net.py:95-112,244-255;
// pytorch_training_inference_on_image.ipynb:454-635).
//
// Structure (cdna_hip_programming.md §5): 256 threads = 4 waves (2x2), block tile BMxBN, BK=64,
// register-staged double-buffered LDS (global loads for tile t+1 are issued before the MFMAs of
// tile t and written to the other LDS buffer after them: one barrier per K-step), XOR-swizzled
// LDS images (ds_read_b128 row reads for FWD/DGRAD; ds_read_b64_tr_b16 transposed reads for
// WGRAD whose operands are both reduction-index-major), XCD-aware bijective block remap, and an
// LDS-staged epilogue that writes 16-byte coalesced rows and emits per-column BatchNorm partial
// statistics of the stored (bf16-rounded) output.
#include "igemm.h"

namespace pcmp {

// "mode,gm,gn,gk,bias,resid,relu -> kind/nsplit" for every planned shape (reports, tests)
std::vector<std::string> gemm_plans() {
  std::lock_guard<std::mutex> g(g_plan_mu);
  std::vector<std::string> r;
  for (auto& kv : g_plan_cache)
    r.push_back(kv.first + " -> " + plan_kind_name(kv.second.kind) + "/split" + std::to_string(kv.second.nsplit));
  return r;
}

// src/dst: flat bf16 buffers; desc: int64 [n][12] on device (see wt_transpose_multi_kernel)
void wt_transpose_multi(const at::Tensor& src, at::Tensor dst, const at::Tensor& desc, int64_t blocks) {
  PCMP_CHECK_CUDA(src); PCMP_CHECK_BF16(src); PCMP_CHECK_BF16(dst); PCMP_CHECK_CONTIG(src); PCMP_CHECK_CONTIG(dst);
  TORCH_CHECK(desc.is_cuda() && desc.scalar_type() == at::kLong && desc.is_contiguous() && desc.dim() == 2 &&
              desc.size(1) == 12, "wt_transpose_multi: desc must be int64 [n,12] on the device");
  const int n = desc.size(0);
  if (n == 0 || blocks <= 0) return;
  hipLaunchKernelGGL(wt_transpose_multi_kernel, dim3((unsigned)blocks), dim3(256), 0, cur_stream(),
                     ptr<unsigned short>(src), ptr<unsigned short>(dst), desc.data_ptr<int64_t>(), n);
  PCMP_LAUNCH_CHECK();
}

// Autotune tables as portable strings -- "G;<plan key>;<kind>;<nsplit>" (plan_gemm) and
// "W;<shape key>;<nsplit>" (wgrad_nsplit) -- so a data-parallel job can make every rank run rank 0's
// kernel choices (pcmp.parallel.ddp.sync_autotune): each rank times its candidates on its own GPU,
// and timing noise would otherwise let ranks pick different kernels (different speed, different
// summation order), the slowest rank gating every step.
std::vector<std::string> autotune_table() {
  std::lock_guard<std::mutex> g(g_plan_mu);
  std::vector<std::string> r;
  for (auto& kv : g_plan_cache)
    r.push_back("G;" + kv.first + ";" + std::to_string(kv.second.kind) + ";" + std::to_string(kv.second.nsplit));
  for (auto& kv : g_wsplit_cache) r.push_back("W;" + kv.first + ";" + std::to_string(kv.second));
  std::sort(r.begin(), r.end());
  return r;
}

// insert or overwrite entries of autotune_table()'s form; returns how many were applied
int64_t autotune_load(std::vector<std::string> entries) {
  std::lock_guard<std::mutex> g(g_plan_mu);
  int64_t n = 0;
  for (const std::string& e : entries) {
    std::vector<std::string> f;
    size_t b = 0;
    for (size_t i = 0; i <= e.size(); ++i)
      if (i == e.size() || e[i] == ';') { f.push_back(e.substr(b, i - b)); b = i + 1; }
    if (f.size() == 4 && f[0] == "G") {
      g_plan_cache[f[1]] = GemmPlan{std::stoi(f[2]), std::stoi(f[3])};
      ++n;
    } else if (f.size() == 3 && f[0] == "W") {
      g_wsplit_cache[f[1]] = std::stoi(f[2]);
      ++n;
    } else {
      TORCH_CHECK(false, "autotune_load: malformed entry '", e, "'");
    }
  }
  return n;
}

// forget every autotuned GEMM plan (A/B tools: a variant's predictor re-plans under its own knobs)
int64_t autotune_clear() {
  std::lock_guard<std::mutex> g(g_plan_mu);
  const int64_t n = (int64_t)g_plan_cache.size();
  g_plan_cache.clear();
  return n;
}

// optional compiled-in kernel variants of this build (none since round 4: the measured-losing
// epilogue variants sk_fixup / epi_coal / bn_group were removed, docs/PERF_NOTES.md)
std::vector<std::string> build_features() { return {}; }

}  // namespace pcmp

TORCH_LIBRARY_FRAGMENT(pcmp, m) {
  m.def("build_features() -> str[]", &pcmp::build_features);
  m.def("gemm_plans() -> str[]", &pcmp::gemm_plans);
  m.def("autotune_table() -> str[]", &pcmp::autotune_table);
  m.def("autotune_load(str[] entries) -> int", &pcmp::autotune_load);
  m.def("autotune_clear() -> int", &pcmp::autotune_clear);
  m.def("plan_candidates(Tensor x, Tensor w, int stride, int pad, Tensor? bias, Tensor? resid, bool relu) -> str[]",
        &pcmp::plan_candidates);
  m.def("wt_transpose_multi(Tensor src, Tensor(a!) dst, Tensor desc, int blocks) -> ()", &pcmp::wt_transpose_multi);
  m.def("conv_fwd(Tensor x, Tensor w, int stride, int pad, Tensor? bias, Tensor? resid, bool relu, bool want_stats, "
        "Tensor? in_scale=None, Tensor? in_shift=None) -> Tensor[]",
        &pcmp::conv_fwd);
  m.def("conv_dgrad(Tensor dy, Tensor w, int H, int W, int stride, int pad, Tensor? resid, Tensor? wt=None) -> Tensor",
        &pcmp::conv_dgrad);
  m.def("conv_dgrad_bnr(Tensor dy, Tensor w, int H, int W, int stride, int pad, Tensor? resid, Tensor? ymask, "
        "Tensor x, Tensor mean, Tensor invstd, Tensor? x2, Tensor? mean2, Tensor? invstd2, Tensor? mscale, "
        "Tensor? mshift, Tensor? wt=None, Tensor? ymask_bits=None, Tensor? fold_x=None, Tensor? fold_coef=None, "
        "bool resid_sub=False) -> Tensor[]",
        &pcmp::conv_dgrad_bnr);
  m.def("conv_wgrad(Tensor dy, Tensor x, Tensor(a!) out, int R, int S, int stride, int pad, bool accumulate, "
        "Tensor? fold_x=None, Tensor? fold_coef=None, Tensor? in_scale=None, Tensor? in_shift=None) -> ()",
        &pcmp::conv_wgrad);
  m.def("conv1x1_bwd_fused(Tensor g, Tensor? fold_x, Tensor? fold_coef, Tensor wt, Tensor z, Tensor scale, "
        "Tensor shift, Tensor mean, Tensor invstd, Tensor(a!) dw, bool accumulate) -> Tensor[]",
        &pcmp::conv1x1_bwd_fused);
  m.def("linear_gelu_fwd(Tensor x, Tensor w, Tensor? bias) -> Tensor[]", &pcmp::linear_gelu_fwd);
  m.def("linear_dgrad_gelu(Tensor dy, Tensor w, Tensor u, Tensor? wt=None) -> Tensor", &pcmp::linear_dgrad_gelu);
}

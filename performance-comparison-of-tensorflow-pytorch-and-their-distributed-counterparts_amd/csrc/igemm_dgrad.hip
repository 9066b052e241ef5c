// Implicit-GEMM convolution / Linear: data-gradient (DGRAD) entry points.
// Kernels, launchers, dispatch and the GEMM planner live in igemm.h; this translation unit holds the
// DGRAD entry points (split from igemm.hip in round 4 so the three modes compile in parallel).
#include "igemm.h"
#include "bnr_stream.h"
#include "bwd_fused.h"

namespace pcmp {

static at::Tensor transpose_taps(const at::Tensor& w, int r0, int s0, int rstep, int subR, int subS,
                                 hipStream_t st) {
  const int K = w.size(0), R = w.size(1), S = w.size(2), C = w.size(3);
  auto wt = at::empty({C, subR, subS, K}, w.options());
  dim3 grid(ceil_div(C, 64), ceil_div(K, 64), subR * subS);
  hipLaunchKernelGGL(wt_transpose_kernel, grid, dim3(256), 0, st, ptr<unsigned short>(w), ptr<unsigned short>(wt), K,
                     R, S, C, r0, s0, rstep, subS, subR * subS);
  PCMP_LAUNCH_CHECK();
  return wt;
}

// dy: [N,P,Q,K], w: [K,R,S,C] -> dx [N,H,W,C] (H, W given) = dgrad + resid (resid optional).
// Stride 2 runs as up to 4 sub-pixel (parity-class) GEMMs, each over only the taps that reach
// that class of output pixels (no MFMA work on structural zeros); their epilogues accumulate in
// place into the residual buffer, which is CONSUMED (its memory becomes dx).
struct BnrArgs {  // fused BatchNorm-backward reduction in the dgrad epilogue (see IgemmParams)
  const __bf16* fold_x = nullptr;     // BatchNorm-backward fold of dy (IgemmParams::fold_x)
  const float* fold_coef = nullptr;
  const uint8_t* mbits = nullptr;
  const __bf16* mask = nullptr;
  const __bf16* x = nullptr;
  const float* mean = nullptr;
  const float* istd = nullptr;
  const __bf16* x2 = nullptr;
  const float* mean2 = nullptr;
  const float* istd2 = nullptr;
  const float* msc = nullptr;
  const float* msh = nullptr;
};

static std::vector<at::Tensor> dgrad_impl(const at::Tensor& dy, const at::Tensor& w, int64_t H, int64_t W,
                                          int64_t stride, int64_t pad, const c10::optional<at::Tensor>& resid,
                                          const BnrArgs* bn, const c10::optional<at::Tensor>& wt_given,
                                          const at::Tensor* dgelu_u = nullptr, bool resid_sub = false) {
  PCMP_CHECK_CUDA(dy); PCMP_CHECK_BF16(dy); PCMP_CHECK_BF16(w);
  PCMP_CHECK_CONTIG(dy); PCMP_CHECK_CONTIG(w);
  const int N = dy.size(0), K = w.size(0), R = w.size(1), S = w.size(2), C = w.size(3);
  IgemmParams p;
  fill_geometry(p, N, H, W, C, K, R, S, stride, pad);
  TORCH_CHECK(dy.size(1) == p.P && dy.size(2) == p.Q && dy.size(3) == K, "conv_dgrad: dy shape");
  const bool has_res = resid.has_value() && resid->defined();
  if (has_res) {
    PCMP_CHECK_BF16(*resid); PCMP_CHECK_CONTIG(*resid);
    if (resid_sub) {
      TORCH_CHECK(stride == 1, "conv_dgrad: a sub-sampled residual needs a stride-1 DGRAD");
      p.resid_sub = 1; p.rs_H2 = (int)(H + 1) / 2; p.rs_W2 = (int)(W + 1) / 2;
      TORCH_CHECK(resid->numel() == (int64_t)N * p.rs_H2 * p.rs_W2 * C, "conv_dgrad: sub-sampled residual shape");
    } else {
      TORCH_CHECK(resid->numel() == (int64_t)N * H * W * C, "conv_dgrad: residual shape");
    }
  } else {
    TORCH_CHECK(!resid_sub, "conv_dgrad: resid_sub without a residual");
  }
  auto set_bn = [&](IgemmParams& q) {
    if (!bn) return;
    q.bn_mask = bn->mask; q.bn_x = bn->x; q.bn_mean = bn->mean; q.bn_istd = bn->istd;
    q.bn_x2 = bn->x2; q.bn_mean2 = bn->mean2; q.bn_istd2 = bn->istd2;
    q.bn_msc = bn->msc; q.bn_msh = bn->msh;
    q.bn_mbits = bn->mbits;
    q.fold_x = bn->fold_x; q.fold_coef = bn->fold_coef;
  };
  auto fopts = dy.options().dtype(at::kFloat);
  const bool two = bn && bn->x2;
  auto st = cur_stream();
  // a pre-transposed weight [C][R][S][K] (batched refresh, pcmp.utils.flat) replaces the per-call
  // transpose wherever the GEMM uses every tap: stride 1, and 1x1 stride 2 (one parity class)
  // A 1-D wt (stride 2 only) is the class-blocked layout of utils/flat.py: the sub-pixel classes
  // (oph, opw) = (0,0), (0,1), (1,0), (1,1) one after another, each [C][subR][subS][K] -- every
  // class GEMM reads its taps from there instead of transposing them per call.
  at::Tensor wt_full, wt_cls;
  if (wt_given.has_value() && wt_given->defined()) {
    PCMP_CHECK_BF16(*wt_given); PCMP_CHECK_CONTIG(*wt_given);
    TORCH_CHECK(wt_given->numel() == w.numel(), "conv_dgrad: transposed weight numel");
    if (wt_given->dim() == 1) {
      TORCH_CHECK(stride == 2, "conv_dgrad: class-blocked transposed weight needs stride 2");
      wt_cls = *wt_given;
    } else {
      TORCH_CHECK(wt_given->size(0) == C && wt_given->size(-1) == K, "conv_dgrad: transposed weight must be [C,R,S,K]");
      wt_full = *wt_given;
    }
  }
  TORCH_CHECK(!bn || !bn->fold_x || (stride == 1 && R == 1 && S == 1 && K % BK == 0),
              "conv_dgrad_bnr: the BatchNorm-backward fold needs a 1x1 stride-1 conv with K % 64 == 0");
  if (stride == 2) {
    struct Cls { int oph, opw, r0, s0, subR, subS, dH, dW; };
    std::vector<Cls> cls;
    bool uncovered = false;   // a parity class no tap reaches (1x1/2): its dx is resid or zero
    for (int oph = 0; oph < 2; ++oph)
      for (int opw = 0; opw < 2; ++opw) {
        const int r0 = (oph + pad) & 1, s0 = (opw + pad) & 1;
        const int subR = r0 < R ? (R - r0 + 1) / 2 : 0, subS = s0 < S ? (S - s0 + 1) / 2 : 0;
        const int dH = (H - oph + 1) / 2, dW = (W - opw + 1) / 2;
        if (dH <= 0 || dW <= 0) continue;
        if (subR == 0 || subS == 0) {
          // no tap reaches this pixel class: its dx is resid (or 0) -- a fused BN reduction would miss it
          TORCH_CHECK(!bn, "conv_dgrad_bnr: stride-2 filter leaves pixel classes uncovered");
          uncovered = true;
          continue;
        }
        cls.push_back({oph, opw, r0, s0, subR, subS, dH, dW});
      }
    // the classes partition dx: without a residual and with every class covered, each pixel is
    // written exactly once -> no zero fill and no read-back of the accumulation buffer
    const bool accum = has_res || uncovered;
    at::Tensor dx = has_res ? *resid : (uncovered ? at::zeros({N, H, W, C}, dy.options())
                                                  : at::empty({N, H, W, C}, dy.options()));
    auto class_params = [&](const Cls& c, const at::Tensor& wt) {
      IgemmParams q = p;
      q.R = c.subR; q.S = c.subS;
      q.sub = 1; q.oph = c.oph; q.opw = c.opw;
      q.dH = c.dH; q.dW = c.dW;
      q.fd_HW = make_fastdiv(c.dH * c.dW);
      q.fd_W = make_fastdiv(c.dW);
      q.offy = (c.oph + pad - c.r0) / 2;
      q.offx = (c.opw + pad - c.s0) / 2;
      q.gm = N * c.dH * c.dW; q.gn = C; q.gk = c.subR * c.subS * K;
      q.a = ptr<__bf16>(dy); q.out = dx.data_ptr();
      q.a_bytes = tensor_bytes(dy);
      if (wt.defined()) { q.b = ptr<__bf16>(wt); q.b_bytes = tensor_bytes(wt); }
      q.resid = accum ? ptr<__bf16>(dx) : nullptr;   // in-place accumulate
      q.ksplit = q.gk;
      set_bn(q);                   // (the kernel choice, hence the partial-row count, depends on it)
      return q;
    };
    at::Tensor part, part2;
    if (bn) {
      int T = 0;
      for (auto& c : cls) {
        const IgemmParams q = class_params(c, at::Tensor());
        T += ceil_div(q.gm, igemm_bm(MODE_DGRAD, q));
      }
      part = at::empty({T, 2, C}, fopts);
      if (two) part2 = at::empty({T, 2, C}, fopts);
    }
    // element offset of each class block in a class-blocked wt (every class counted, as utils/flat.py does)
    int64_t cls_off[2][2] = {{0, 0}, {0, 0}}, cls_total = 0;
    for (int oph = 0; oph < 2; ++oph)
      for (int opw = 0; opw < 2; ++opw) {
        const int r0 = (oph + pad) & 1, s0 = (opw + pad) & 1;
        const int subR = r0 < R ? (R - r0 + 1) / 2 : 0, subS = s0 < S ? (S - s0 + 1) / 2 : 0;
        cls_off[oph][opw] = cls_total;
        cls_total += (int64_t)C * subR * subS * K;
      }
    TORCH_CHECK(!wt_cls.defined() || cls_total == wt_cls.numel(), "conv_dgrad: class-blocked weight size");
    int toff = 0;
    for (auto& c : cls) {
      const bool whole = c.subR == R && c.subS == S && wt_full.defined();
      at::Tensor wt = wt_cls.defined()
                          ? wt_cls.narrow(0, cls_off[c.oph][c.opw], (int64_t)C * c.subR * c.subS * K)
                                .view({C, c.subR, c.subS, K})
                          : (whole ? wt_full : transpose_taps(w, c.r0, c.s0, 2, c.subR, c.subS, st));
      IgemmParams q = class_params(c, wt);
      if (bn) {
        q.stats = ptr<float>(part) + (size_t)toff * 2 * C;
        if (two) q.stats2 = ptr<float>(part2) + (size_t)toff * 2 * C;
        q.stats_cap = (int)part.size(0) - toff;
        toff += ceil_div(q.gm, igemm_bm(MODE_DGRAD, q));
      }
      dispatch<MODE_DGRAD>(q, st);
    }
    if (!bn) return {dx};
    if (two) return {dx, part, part2};
    return {dx, part};
  }
  at::Tensor wt = wt_full.defined() ? wt_full : transpose_taps(w, 0, 0, 1, R, S, st);
  auto dx = at::empty({N, H, W, C}, dy.options());
  p.gm = N * H * W; p.gn = C; p.gk = R * S * K;
  p.a = ptr<__bf16>(dy); p.b = ptr<__bf16>(wt); p.out = dx.data_ptr();
  p.a_bytes = tensor_bytes(dy); p.b_bytes = tensor_bytes(wt);
  if (has_res) p.resid = ptr<__bf16>(*resid);
  if (dgelu_u) {   // dx = dgrad * gelu'(u): the GELU backward of the layer that produced dy's input
    TORCH_CHECK(!has_res && !bn && stride == 1 && R == 1 && S == 1, "linear_dgrad_gelu: plain 1x1 GEMM only");
    PCMP_CHECK_BF16(*dgelu_u); PCMP_CHECK_CONTIG(*dgelu_u);
    TORCH_CHECK(dgelu_u->numel() == (int64_t)N * H * W * C, "linear_dgrad_gelu: u shape");
    p.resid = ptr<__bf16>(*dgelu_u);
    p.relu = 3;
  }
  p.ksplit = p.gk;
  if (!bn && plain_gemm_eligible<MODE_DGRAD>(p)) {
    const GemmPlan pl = plan_gemm<MODE_DGRAD>(p, ptr<__bf16>(dx), fopts, st);
    run_plan<MODE_DGRAD>(p, pl, ptr<__bf16>(dx), fopts, st);
    return {dx};
  }
  at::Tensor part, part2;
  if (bn) {
    set_bn(p);   // before igemm_bm: the kernel choice depends on the epilogue variant
    if (use_bnr_stream(p)) {   // memory-bound short-K 1x1: the streaming kernel (bnr_stream.h)
      const int T = bnr_stream_groups(p);
      part = at::empty({T, 2, C}, fopts);
      p.stats_cap = T;
      p.stats = ptr<float>(part);
      if (two) { part2 = at::empty({T, 2, C}, fopts); p.stats2 = ptr<float>(part2); }
      launch_bnr_stream(p, st);
      if (two) return {dx, part, part2};
      return {dx, part};
    }
    const int T = ceil_div(p.gm, igemm_bm(MODE_DGRAD, p));
    part = at::empty({T, 2, C}, fopts);
    p.stats_cap = T;
    p.stats = ptr<float>(part);
    if (two) { part2 = at::empty({T, 2, C}, fopts); p.stats2 = ptr<float>(part2); }
  }
  dispatch<MODE_DGRAD>(p, st);
  if (!bn) return {dx};
  if (two) return {dx, part, part2};
  return {dx, part};
}

// dy: [N,P,Q,K], w: [K,R,S,C] -> dx [N,H,W,C] (H, W given) = dgrad + resid (resid optional).
// Stride 2 runs as up to 4 sub-pixel (parity-class) GEMMs, each over only the taps that reach
// that class of output pixels (no MFMA work on structural zeros); their epilogues accumulate in
// place into the residual buffer, which is CONSUMED (its memory becomes dx).
at::Tensor conv_dgrad(const at::Tensor& dy, const at::Tensor& w, int64_t H, int64_t W, int64_t stride,
                      int64_t pad, const c10::optional<at::Tensor>& resid, const c10::optional<at::Tensor>& wt) {
  if (dy.scalar_type() == at::kFloat) return f32::conv_dgrad(dy, w, H, W, stride, pad, resid);
  return dgrad_impl(dy, w, H, W, stride, pad, resid, nullptr, wt)[0];
}

// Linear input gradient through a GELU: dy [M, N], w [N, C] -> du = (dy W) * gelu'(u), u [M, C] the
// pre-activation saved by linear_gelu_fwd (the GELU backward fused into the DGRAD epilogue).
at::Tensor linear_dgrad_gelu(const at::Tensor& dy, const at::Tensor& w, const at::Tensor& u,
                             const c10::optional<at::Tensor>& wt) {
  if (dy.scalar_type() == at::kFloat) return f32::linear_dgrad_gelu(dy, w, u);
  TORCH_CHECK(dy.dim() == 2 && w.dim() == 2 && u.dim() == 2 && dy.size(1) == w.size(0) && u.size(1) == w.size(1) &&
              u.size(0) == dy.size(0), "linear_dgrad_gelu: dy [M, N], w [N, C], u [M, C]");
  const int64_t M = dy.size(0), N = w.size(0), C = w.size(1);
  const at::Tensor u4 = u.view({M, 1, 1, C});
  auto dx = dgrad_impl(dy.view({M, 1, 1, N}), w.view({N, 1, 1, C}), 1, 1, 1, 0, c10::nullopt, nullptr, wt, &u4)[0];
  return dx.view({M, C});
}

// conv_dgrad with the BatchNorm-backward reduction of the layer(s) whose output gradient this is
// fused into the epilogue: returns [g, part(, part2)] with g = (dgrad + resid) * (ymask > 0) (bf16)
// and part = per-tile [T][2][C] partial (sum g, sum g * (x - mean) * invstd) for bn_bwd_finalize.
std::vector<at::Tensor> conv_dgrad_bnr(const at::Tensor& dy, const at::Tensor& w, int64_t H, int64_t W,
                                       int64_t stride, int64_t pad, const c10::optional<at::Tensor>& resid,
                                       const c10::optional<at::Tensor>& ymask, const at::Tensor& x,
                                       const at::Tensor& mean, const at::Tensor& invstd,
                                       const c10::optional<at::Tensor>& x2, const c10::optional<at::Tensor>& mean2,
                                       const c10::optional<at::Tensor>& invstd2,
                                       const c10::optional<at::Tensor>& mscale,
                                       const c10::optional<at::Tensor>& mshift,
                                       const c10::optional<at::Tensor>& wt,
                                       const c10::optional<at::Tensor>& ymask_bits,
                                       const c10::optional<at::Tensor>& fold_x,
                                       const c10::optional<at::Tensor>& fold_coef, bool resid_sub) {
  const bool fold = fold_x.has_value() && fold_x->defined();
  TORCH_CHECK(!resid_sub || dy.scalar_type() != at::kFloat, "conv_dgrad_bnr: the sub-sampled residual is bf16 only");
  TORCH_CHECK(!fold || dy.scalar_type() != at::kFloat, "conv_dgrad_bnr: the BatchNorm-backward fold is bf16 only");
  if (dy.scalar_type() == at::kFloat)
    return f32::conv_dgrad_bnr(dy, w, H, W, stride, pad, resid, ymask, x, mean, invstd, x2, mean2, invstd2, mscale,
                               mshift, ymask_bits);
  const int64_t n = (int64_t)dy.size(0) * H * W * w.size(3);
  auto chk = [&](const at::Tensor& t, const char* nm) {
    PCMP_CHECK_BF16(t); PCMP_CHECK_CONTIG(t);
    TORCH_CHECK(t.numel() == n, "conv_dgrad_bnr: ", nm, " shape");
  };
  BnrArgs a;
  chk(x, "x");
  PCMP_CHECK_F32(mean); PCMP_CHECK_F32(invstd);
  a.x = ptr<__bf16>(x); a.mean = ptr<float>(mean); a.istd = ptr<float>(invstd);
  if (ymask.has_value() && ymask->defined()) { chk(*ymask, "ymask"); a.mask = ptr<__bf16>(*ymask); }
  if (ymask_bits.has_value() && ymask_bits->defined()) {
    TORCH_CHECK(ymask_bits->scalar_type() == at::kByte && ymask_bits->is_contiguous() && ymask_bits->numel() * 8 == n,
                "conv_dgrad_bnr: ymask_bits must be contiguous uint8 with one byte per 8 elements");
    a.mbits = ymask_bits->data_ptr<uint8_t>();
  }
  if (x2.has_value() && x2->defined()) {
    chk(*x2, "x2");
    TORCH_CHECK(mean2.has_value() && invstd2.has_value(), "conv_dgrad_bnr: mean2/invstd2 required with x2");
    a.x2 = ptr<__bf16>(*x2); a.mean2 = ptr<float>(*mean2); a.istd2 = ptr<float>(*invstd2);
  }
  if (!a.mask && !a.mbits && mscale.has_value() && mscale->defined()) {
    TORCH_CHECK(mshift.has_value() && mshift->defined(), "conv_dgrad_bnr: mshift required with mscale");
    PCMP_CHECK_F32(*mscale); PCMP_CHECK_F32(*mshift);
    a.msc = ptr<float>(*mscale); a.msh = ptr<float>(*mshift);
  }
  if (fold) {
    PCMP_CHECK_BF16(*fold_x); PCMP_CHECK_CONTIG(*fold_x);
    TORCH_CHECK(fold_x->numel() == dy.numel(), "conv_dgrad_bnr: fold_x must have dy's shape");
    TORCH_CHECK(fold_coef.has_value() && fold_coef->defined(), "conv_dgrad_bnr: fold_coef required with fold_x");
    PCMP_CHECK_F32(*fold_coef); PCMP_CHECK_CONTIG(*fold_coef);
    TORCH_CHECK(fold_coef->numel() == 3 * dy.size(-1), "conv_dgrad_bnr: fold_coef must be [3, K]");
    a.fold_x = ptr<__bf16>(*fold_x); a.fold_coef = ptr<float>(*fold_coef);
  }
  return dgrad_impl(dy, w, H, W, stride, pad, resid, &a, wt, nullptr, resid_sub);
}

// Fused backward of a 1x1 stride-1 conv whose input is relu(BN(z)) (bwd_fused.h): returns [g_in, part]
// (conv_dgrad_bnr's outputs for that BN, mask recomputed from z) and writes dW into `dw` (fp32
// [K,1,1,C], accumulate optional).  g: [N,H,W,K] masked BN-input gradient with fold_x / fold_coef (the
// BatchNorm-backward fold of the conv's output BN), or dz itself; wt: [C,1,1,K] transposed weight.
std::vector<at::Tensor> conv1x1_bwd_fused(const at::Tensor& g, const c10::optional<at::Tensor>& fold_x,
                                          const c10::optional<at::Tensor>& fold_coef, const at::Tensor& wt,
                                          const at::Tensor& z, const at::Tensor& scale, const at::Tensor& shift,
                                          const at::Tensor& mean, const at::Tensor& invstd, at::Tensor dw,
                                          bool accumulate) {
  PCMP_CHECK_CUDA(g); PCMP_CHECK_BF16(g); PCMP_CHECK_CONTIG(g);
  PCMP_CHECK_BF16(wt); PCMP_CHECK_CONTIG(wt); PCMP_CHECK_BF16(z); PCMP_CHECK_CONTIG(z);
  PCMP_CHECK_F32(dw); PCMP_CHECK_CONTIG(dw);
  for (const at::Tensor* t : {&scale, &shift, &mean, &invstd}) { PCMP_CHECK_F32(*t); PCMP_CHECK_CONTIG(*t); }
  const int64_t KC = g.size(-1), CC = z.size(-1);
  const int64_t M = g.numel() / KC;
  TORCH_CHECK(KC == 256 && CC == 64, "conv1x1_bwd_fused: the 64 -> 256 channel geometry only");
  TORCH_CHECK(z.numel() == M * CC && wt.numel() == KC * CC && dw.numel() == KC * CC && M % 32 == 0,
              "conv1x1_bwd_fused: shapes");
  const bool fold = fold_x.has_value() && fold_x->defined();
  if (fold) {
    PCMP_CHECK_BF16(*fold_x); PCMP_CHECK_CONTIG(*fold_x);
    TORCH_CHECK(fold_x->numel() == g.numel() && fold_coef.has_value() && fold_coef->numel() == 3 * KC,
                "conv1x1_bwd_fused: fold_x / fold_coef");
  }
  BwdFusedParams p;
  p.g = ptr<__bf16>(g);
  p.fx = fold ? ptr<__bf16>(*fold_x) : nullptr;
  p.fcoef = fold ? ptr<float>(*fold_coef) : nullptr;
  p.wt = ptr<__bf16>(wt); p.z = ptr<__bf16>(z);
  p.sc = ptr<float>(scale); p.sh = ptr<float>(shift); p.mean = ptr<float>(mean); p.istd = ptr<float>(invstd);
  p.M = (int)M;
  p.g_bytes = tensor_bytes(g); p.z_bytes = tensor_bytes(z); p.wt_bytes = tensor_bytes(wt);
  const int groups = std::max(1, std::min((int)(M / 32), kn_bwd_fused_wgs.get()));
  auto gout = at::empty_like(z);
  auto part = at::empty({groups, 2, CC}, g.options().dtype(at::kFloat));
  auto ws = at::empty({groups, KC * CC}, g.options().dtype(at::kFloat));
  p.gout = ptr<__bf16>(gout); p.part = ptr<float>(part); p.dw = ptr<float>(ws);
  constexpr size_t smem = (size_t)64 * 256 * 2 + 2 * ((size_t)32 * 256 * 2 * 2 + 32 * 64 * 2) + 32 * 64 * 2 +
                          (size_t)32 * 72 * 4 + 3 * 256 * 4;
  static_assert(smem <= 160 * 1024, "bwd_fused: LDS");
  auto st = cur_stream();
  auto launch = [&](auto kf) {
    static bool attr = false;
    if (!attr) {
      PCMP_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(kf), hipFuncAttributeMaxDynamicSharedMemorySize,
                                         160 * 1024));
      attr = true;
    }
    hipLaunchKernelGGL(kf, dim3(groups), dim3(256), smem, st, p, groups);
    PCMP_LAUNCH_CHECK();
  };
  if (fold) launch(&bwd_fused_kernel<256, 64, true>); else launch(&bwd_fused_kernel<256, 64, false>);
  // dW = sum of the workgroup partials, in a fixed order (deterministic)
  const int n4 = (int)(KC * CC / 4);
  const int SL = groups <= 8 ? 1 : (groups <= 32 ? 4 : 16);
  const dim3 grid(ceil_div(n4, 256 / SL));
  if (SL == 1) hipLaunchKernelGGL(splitk_reduce2_kernel<1>, grid, dim3(256), 0, st, ptr<float>(ws), ptr<float>(dw), n4, groups, (int)accumulate);
  else if (SL == 4) hipLaunchKernelGGL(splitk_reduce2_kernel<4>, grid, dim3(256), 0, st, ptr<float>(ws), ptr<float>(dw), n4, groups, (int)accumulate);
  else hipLaunchKernelGGL(splitk_reduce2_kernel<16>, grid, dim3(256), 0, st, ptr<float>(ws), ptr<float>(dw), n4, groups, (int)accumulate);
  PCMP_LAUNCH_CHECK();
  return {gout, part};
}

}  // namespace pcmp

// fp32 compute path (the reference's precision: another_neural_net.py:95-115, nb :655-702 run fp32
// everywhere): entry points called by the op wrappers of igemm.hip / bn.hip /
// elementwise.hip when their activations are fp32 (``--dtype fp32``).  Kernels in f32.hip.
#pragma once
#include "common.h"

#include <vector>

namespace pcmp {
namespace f32 {

// in_scale / in_shift (optional, per input channel): the conv reads relu(x * in_scale + in_shift)
// (a BatchNorm + ReLU left unmaterialised by the producer; zero padding stays zero).
std::vector<at::Tensor> conv_fwd(const at::Tensor& x, const at::Tensor& w, int64_t stride, int64_t pad,
                                 const c10::optional<at::Tensor>& bias, const c10::optional<at::Tensor>& resid,
                                 bool relu, bool want_stats, const at::Tensor* in_scale = nullptr,
                                 const at::Tensor* in_shift = nullptr);
at::Tensor conv_dgrad(const at::Tensor& dy, const at::Tensor& w, int64_t H, int64_t W, int64_t stride, int64_t pad,
                      const c10::optional<at::Tensor>& resid);
std::vector<at::Tensor> conv_dgrad_bnr(const at::Tensor& dy, const at::Tensor& w, int64_t H, int64_t W,
                                       int64_t stride, int64_t pad, const c10::optional<at::Tensor>& resid,
                                       const c10::optional<at::Tensor>& ymask, const at::Tensor& x,
                                       const at::Tensor& mean, const at::Tensor& invstd,
                                       const c10::optional<at::Tensor>& x2, const c10::optional<at::Tensor>& mean2,
                                       const c10::optional<at::Tensor>& invstd2, const c10::optional<at::Tensor>& mscale,
                                       const c10::optional<at::Tensor>& mshift,
                                       const c10::optional<at::Tensor>& ymask_bits);
void conv_wgrad(const at::Tensor& dy, const at::Tensor& x, at::Tensor out, int64_t R, int64_t S, int64_t stride,
                int64_t pad, bool accumulate, const at::Tensor* in_scale = nullptr,
                const at::Tensor* in_shift = nullptr);

at::Tensor bn_partials(const at::Tensor& x);
at::Tensor bn_apply(const at::Tensor& x, const at::Tensor& scale, const at::Tensor& shift,
                    const c10::optional<at::Tensor>& x2, const c10::optional<at::Tensor>& scale2,
                    const c10::optional<at::Tensor>& shift2, bool relu, const c10::optional<at::Tensor>& mbits);
std::vector<at::Tensor> bn_bwd_reduce(const at::Tensor& dy, const c10::optional<at::Tensor>& ymask,
                                      const at::Tensor& x, const at::Tensor& mean, const at::Tensor& invstd,
                                      const c10::optional<at::Tensor>& x2, const c10::optional<at::Tensor>& mean2,
                                      const c10::optional<at::Tensor>& invstd2);
std::vector<at::Tensor> bn_bwd_apply(const at::Tensor& dy, const c10::optional<at::Tensor>& ymask,
                                     const at::Tensor& x, const at::Tensor& coef,
                                     const c10::optional<at::Tensor>& x2, const c10::optional<at::Tensor>& coef2,
                                     bool want_g);

std::vector<at::Tensor> maxpool_fwd(const at::Tensor& x, int64_t k, int64_t s, int64_t pad, bool want_idx,
                                    const c10::optional<at::Tensor>& scale, const c10::optional<at::Tensor>& shift);
at::Tensor maxpool_bwd(const at::Tensor& dy, const at::Tensor& idx, int64_t H, int64_t W, int64_t k, int64_t s,
                       int64_t pad);
std::vector<at::Tensor> maxpool_bwd_bnr(const at::Tensor& dy, const at::Tensor& idx, const at::Tensor& cx,
                                        const at::Tensor& mean, const at::Tensor& invstd, const at::Tensor& scale,
                                        const at::Tensor& shift, int64_t k, int64_t s, int64_t pad);
at::Tensor gap_fwd(const at::Tensor& x);
at::Tensor gap_bwd(const at::Tensor& dy, int64_t H, int64_t W);
at::Tensor dropout(const at::Tensor& x, double p, int64_t seed, int64_t offset, const c10::optional<at::Tensor>& salt);
at::Tensor relu_bwd(const at::Tensor& dy, const at::Tensor& y);
void colsum(const at::Tensor& x, at::Tensor out, bool accumulate);

// text encoders (text_f32.hip): LayerNorm, attention, GELU / tanh, embedding, pooling, BiLSTM
at::Tensor act_fwd(const at::Tensor& x, int mode);                               // 0 GELU, 1 tanh
at::Tensor act_bwd(const at::Tensor& dy, const at::Tensor& xy, int mode);
at::Tensor add(const at::Tensor& a, const at::Tensor& b);
std::vector<at::Tensor> layernorm_fwd(const at::Tensor& x, const c10::optional<at::Tensor>& r, const at::Tensor& g,
                                      const at::Tensor& b, double eps, double p, int64_t seed, int64_t offset,
                                      const c10::optional<at::Tensor>& salt);
std::vector<at::Tensor> embed_layernorm_fwd(const at::Tensor& x, const at::Tensor& pos, const at::Tensor& tt,
                                            const at::Tensor& g, const at::Tensor& b, double eps);
std::vector<at::Tensor> layernorm_bwd_fused(const at::Tensor& dy, const at::Tensor& xs, const at::Tensor& mean,
                                            const at::Tensor& rstd, const at::Tensor& g,
                                            const c10::optional<at::Tensor>& dg, const c10::optional<at::Tensor>& db,
                                            const c10::optional<at::Tensor>& dbias, int64_t accmask, double p,
                                            int64_t seed, int64_t offset, const c10::optional<at::Tensor>& salt);
at::Tensor layernorm_bwd(const at::Tensor& dy, const at::Tensor& xs, const at::Tensor& mean, const at::Tensor& rstd,
                         const at::Tensor& g, const c10::optional<at::Tensor>& dg, const c10::optional<at::Tensor>& db,
                         bool accumulate);
std::vector<at::Tensor> attention_fwd(const at::Tensor& qkv, const c10::optional<at::Tensor>& ids, int64_t B,
                                      int64_t S, int64_t H, double p_drop, int64_t seed, int64_t offset,
                                      const c10::optional<at::Tensor>& salt);
at::Tensor attention_bwd(const at::Tensor& dctx, const at::Tensor& qkv, const at::Tensor& ctx, const at::Tensor& lse,
                         const c10::optional<at::Tensor>& ids, int64_t B, int64_t S, int64_t H, double p_drop,
                         int64_t seed, int64_t offset, const c10::optional<at::Tensor>& salt);
at::Tensor embedding_fwd(const at::Tensor& ids, const at::Tensor& W);
void embedding_bwd(const at::Tensor& ids, const at::Tensor& dy, at::Tensor dW, int64_t padding_idx, bool accumulate);
at::Tensor masked_mean_fwd(const at::Tensor& x, const at::Tensor& ids);
at::Tensor masked_mean_bwd(const at::Tensor& dy, const at::Tensor& ids, int64_t S);
std::vector<at::Tensor> lstm_seq_fwd(const at::Tensor& gx, const at::Tensor& whh, const at::Tensor& ids);
std::vector<at::Tensor> lstm_seq_bwd(const at::Tensor& dhout, const at::Tensor& gates, const at::Tensor& cst,
                                     const at::Tensor& whh, const at::Tensor& ids);
std::vector<at::Tensor> linear_gelu_fwd(const at::Tensor& x, const at::Tensor& w, const c10::optional<at::Tensor>& bias);
at::Tensor linear_dgrad_gelu(const at::Tensor& dy, const at::Tensor& w, const at::Tensor& u);

}  // namespace f32
}  // namespace pcmp

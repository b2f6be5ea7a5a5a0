// Thin PyTorch bindings for the cloudtik_amd CDNA4 op library.
// Every function validates shapes/dtypes on the host (a mis-shaped launch of a hand-written
// kernel can fault the GPU), fetches the current HIP stream and calls the extern "C"
// launcher.  No allocation happens inside the launchers; workspaces come from the caller.
#include <torch/extension.h>
#include <map>
#include <mutex>
#include <ATen/hip/HIPContext.h>
#include <hip/hip_runtime.h>

extern "C" {
int ct_layernorm_fwd(const void*, const void*, const void*, const void*, const void*, void*, void*,
                     float*, float*, int, int, float, int, float, uint64_t, uint64_t, hipStream_t);
int ct_layernorm_bwd_grid(int M, int N);
int ct_layernorm_bwd(const void*, const void*, const void*, const float*, const float*,
                     const void*, void*, void*, float*, void*, void*, void*, int, int, int, int,
                     int, float, uint64_t, uint64_t, hipStream_t);
int ct_layernorm_bwd2(const void*, const void*, const void*, const float*, const float*,
                      const void*, void*, void*, float*, void*, void*, void*, int, int, int, int,
                      int, float, uint64_t, uint64_t, int, const void*, hipStream_t);
int ct_colsum(const float*, void*, int, int, int, int, hipStream_t);
int ct_bias_act_fwd(const void*, const void*, void*, long, int, int, hipStream_t);
int ct_bias_act_bwd_grid(long M);
int ct_bias_act_bwd(const void*, const void*, const void*, void*, float*, void*, long, int, int,
                    int, int, hipStream_t);
int ct_dropout(const void*, void*, long, float, uint64_t, uint64_t, hipStream_t);
int ct_embed3_fwd(const int64_t*, const int64_t*, const void*, const void*, const void*, void*, int,
                  int, int, hipStream_t);
int ct_embed3_bwd(const int64_t*, const int64_t*, const void*, float*, float*, float*, int, int, int, int, hipStream_t);
int ct_cast(const void*, int, void*, int, long, float, int, hipStream_t);
int ct_splitk_reduce(const float*, int, long, void*, int, hipStream_t);
int ct_splitk_reduce_clear(float*, int, long, void*, int, hipStream_t);
int ct_splitk_reduce2(const float*, int, long, void*, const float*, int, long, void*, int, hipStream_t);
int ct_lamb(const void*, int, float*, float*, float*, void*, int, const int*, const long*,
            const int*, int, const int*, int, const float*, const float*, float, float, float, int,
            int, float*, float*, int, hipStream_t);
int ct_adam(const void*, int, float*, float*, float*, void*, int, const int*, const long*,
            const int*, int, const float*, const float*, float, float, float, int, hipStream_t);
int ct_sgd(const void*, int, float*, float*, void*, int, const int*, const long*, const int*, int,
           const float*, const float*, float, float, int, int, hipStream_t);
int ct_sumsq(const void*, int, long, float*, float*, hipStream_t);
int ct_clip_coef(const float*, float*, float, float, hipStream_t);
int ct_xent_fwd(const void*, void*, int, int, const int64_t*, float*, float*, const float*, int, int,
                float, hipStream_t);
int ct_bn_fwd_train(const void*, const void*, const void*, const void*, float*, float*, void*, float*,
                    float*, int, int, float, float, int, void*, hipStream_t);
int ct_bn_apply(const void*, const void*, const float*, const float*, void*, int, int, int, hipStream_t);
int ct_bn_fwd_train_given(const void*, const void*, const void*, const void*, float*, float*, void*, const float*, int,
                          int, float*, int, int, float, float, int, void*, hipStream_t);
int ct_bn_fwd_train_pool_given(const void*, const void*, const void*, float*, float*, void*, void*, const float*, int, int,
                               float*, int, int, int, int, int, int, float, float, hipStream_t);
int ct_bn_fwd_train_pool(const void*, const void*, const void*, float*, float*, void*, void*, float*, float*, int, int,
                         int, int, int, int, float, float, hipStream_t);
int ct_maxpool3s2_bwd(const void*, const void*, void*, int, int, int, int, int, int, hipStream_t);
int ct_bn_fwd_train_given2(const void*, const void*, const void*, float*, float*, const float*, int, int, float*,
                           const void*, const void*, const void*, float*, float*, const float*, int, int, float*,
                           void*, void*, int, int, float, float, hipStream_t);
int ct_maxpool3s2_bwd_bn(const void*, const void*, const void*, const float*, void*, float*, int, int, int, int, int,
                         int, hipStream_t);
long ct_maxpool3s2_bwd_bn_rows(int, int);
int ct_bn_bwd_given_pair(const void*, const void*, const void*, const float*, const float*, long, int, const void*,
                         const void*, const float*, void*, void*, void*, void*, void*, void*, int, float*, float*,
                         float*, int, int, hipStream_t);
int ct_bn_bwd_given(const void*, const void*, const void*, const float*, void*, void*, void*, int, const float*, long,
                    int, float*, int, int, hipStream_t);
int ct_bn_bwd(const void*, const void*, const void*, const void*, const float*, void*, void*, void*, void*, int,
              float*, float*, int, int, int, hipStream_t);
int ct_attn_fwd(const void*, const long*, const void*, const long*, const void*, const long*, void*,
                const long*, const float*, long, float*, int, int, int, int, float, float, uint64_t,
                uint64_t, int, hipStream_t);
int ct_attn_fwd_relbias(const void*, const long*, const void*, const long*, const void*, const long*, void*,
                        const long*, const float*, long, const float*, long, int, int, float*, int, int, int, int,
                        float, int, hipStream_t);
int ct_attn_bwd(const void*, const long*, const void*, const long*, const void*, const long*,
                const void*, const long*, const void*, const long*, void*, const long*, void*,
                const long*, void*, const long*, const float*, long, const float*, float*, float*,
                int, int, int, int, float, float, uint64_t, uint64_t, int, hipStream_t);
}

#define CHECK_CUDA(x) TORCH_CHECK((x).is_cuda(), #x " must be a GPU tensor")
#define CHECK_CONTIG(x) TORCH_CHECK((x).is_contiguous(), #x " must be contiguous")
#define CHECK_BF16(x) TORCH_CHECK((x).scalar_type() == at::kBFloat16, #x " must be bf16")
#define CHECK_F32(x) TORCH_CHECK((x).scalar_type() == at::kFloat, #x " must be fp32")
#define CHECK_IN(x) do { CHECK_CUDA(x); CHECK_CONTIG(x); } while (0)

static inline hipStream_t cur_stream() { return at::hip::getCurrentHIPStream().stream(); }
static inline const void* optr(const c10::optional<at::Tensor>& t) {
  return (t.has_value() && t->defined()) ? t->data_ptr() : nullptr;
}
static inline void* optr_mut(const c10::optional<at::Tensor>& t) {
  return (t.has_value() && t->defined()) ? t->data_ptr() : nullptr;
}
static inline int dt_code(const at::Tensor& t) {
  if (t.scalar_type() == at::kFloat) return 0;
  if (t.scalar_type() == at::kBFloat16) return 1;
  TORCH_CHECK(false, "only fp32 / bf16 supported");
  return -1;
}

// ---------------------------------------------------------------- layernorm
// returns (y, s, mean, rstd); s is undefined when no bias/residual/dropout was applied
std::vector<at::Tensor> layernorm_fwd(at::Tensor x, c10::optional<at::Tensor> bias,
                                      c10::optional<at::Tensor> res, at::Tensor gamma,
                                      c10::optional<at::Tensor> beta, double eps, bool rms,
                                      double p_drop, int64_t seed, int64_t offset, bool keep_sum) {
  CHECK_IN(x); CHECK_BF16(x); CHECK_IN(gamma); CHECK_BF16(gamma);
  const int N = x.size(-1);
  const int M = x.numel() / N;
  TORCH_CHECK(gamma.numel() == N, "gamma size");
  if (bias.has_value() && bias->defined()) { CHECK_IN(*bias); CHECK_BF16(*bias); TORCH_CHECK(bias->numel() == N); }
  if (res.has_value() && res->defined()) { CHECK_IN(*res); CHECK_BF16(*res); TORCH_CHECK(res->numel() == x.numel()); }
  if (beta.has_value() && beta->defined()) { CHECK_IN(*beta); CHECK_BF16(*beta); TORCH_CHECK(beta->numel() == N); }
  auto y = at::empty_like(x);
  // keep_sum = false: the caller's backward runs from y (layernorm_bwd_into from_y), so the
  // normalised input sum s is not written
  const bool need_s = keep_sum && (optr(bias) || optr(res) || p_drop > 0.0);
  at::Tensor s = need_s ? at::empty_like(x) : at::Tensor();
  auto fo = x.options().dtype(at::kFloat);
  auto mean = at::empty({M}, fo);
  auto rstd = at::empty({M}, fo);
  int rc = ct_layernorm_fwd(x.data_ptr(), optr(bias), optr(res), gamma.data_ptr(), optr(beta),
                            y.data_ptr(), need_s ? s.data_ptr() : nullptr, mean.data_ptr<float>(),
                            rstd.data_ptr<float>(), M, N, (float)eps, rms ? 1 : 0, (float)p_drop,
                            (uint64_t)seed, (uint64_t)offset, cur_stream());
  TORCH_CHECK(rc == 0, "layernorm_fwd: unsupported shape N=", N);
  return {y, s, mean, rstd};
}

// returns (ds, dx, dgamma, dbeta, dbias)
std::vector<at::Tensor> layernorm_bwd(at::Tensor dy, at::Tensor s, at::Tensor gamma, at::Tensor mean,
                                      at::Tensor rstd, c10::optional<at::Tensor> dextra, bool rms,
                                      bool has_beta, bool has_bias, bool need_dx, double p_drop,
                                      int64_t seed, int64_t offset) {
  CHECK_IN(dy); CHECK_BF16(dy); CHECK_IN(s); CHECK_BF16(s); CHECK_IN(gamma);
  const int N = s.size(-1);
  const int M = s.numel() / N;
  TORCH_CHECK(dy.numel() == s.numel());
  auto ds = at::empty_like(s);
  at::Tensor dx = need_dx ? at::empty_like(s) : at::Tensor();
  auto dgamma = at::empty_like(gamma);
  at::Tensor dbeta = has_beta ? at::empty_like(gamma) : at::Tensor();
  at::Tensor dbias = has_bias ? at::empty_like(gamma) : at::Tensor();
  const int grid = ct_layernorm_bwd_grid(M, N);
  auto part = at::empty({3 * (long)grid * N}, s.options().dtype(at::kFloat));
  int rc = ct_layernorm_bwd(dy.data_ptr(), s.data_ptr(), gamma.data_ptr(), mean.data_ptr<float>(),
                            rstd.data_ptr<float>(), optr(dextra), ds.data_ptr(),
                            need_dx ? dx.data_ptr() : nullptr, part.data_ptr<float>(),
                            dgamma.data_ptr(), has_beta ? dbeta.data_ptr() : nullptr,
                            has_bias ? dbias.data_ptr() : nullptr, M, N, rms ? 1 : 0,
                            gamma.scalar_type() == at::kFloat ? 1 : 0, 0, (float)p_drop,
                            (uint64_t)seed, (uint64_t)offset, cur_stream());
  TORCH_CHECK(rc == 0, "layernorm_bwd: unsupported shape N=", N);
  return {ds, dx, dgamma, dbeta, dbias};
}

// Same as layernorm_bwd but parameter grads are ACCUMULATED into caller-provided tensors
// (views of the flat gradient buffer) and the activation grads may go to given outputs.
// returns (ds, dx); dx is undefined when need_dx is false.
std::vector<at::Tensor> layernorm_bwd_into(at::Tensor dy, at::Tensor s, at::Tensor gamma,
                                           at::Tensor mean, at::Tensor rstd, bool rms,
                                           at::Tensor dgamma, c10::optional<at::Tensor> dbeta,
                                           c10::optional<at::Tensor> dbias, bool need_dx,
                                           double p_drop, int64_t seed, int64_t offset,
                                           c10::optional<at::Tensor> beta_y) {
  CHECK_IN(dy); CHECK_BF16(dy); CHECK_IN(s); CHECK_BF16(s); CHECK_IN(gamma); CHECK_IN(dgamma);
  const int N = s.size(-1);
  const int M = s.numel() / N;
  TORCH_CHECK(dy.numel() == s.numel() && dgamma.numel() == N);
  if (dbeta.has_value() && dbeta->defined()) { CHECK_IN(*dbeta); TORCH_CHECK(dbeta->numel() == N && dbeta->scalar_type() == dgamma.scalar_type()); }
  if (dbias.has_value() && dbias->defined()) { CHECK_IN(*dbias); TORCH_CHECK(dbias->numel() == N && dbias->scalar_type() == dgamma.scalar_type()); }
  auto ds = at::empty_like(s);
  at::Tensor dx = need_dx ? at::empty_like(s) : at::Tensor();
  const int grid = ct_layernorm_bwd_grid(M, N);
  auto part = at::empty({3 * (long)grid * N}, s.options().dtype(at::kFloat));
  // beta_y given: s is the forward's OUTPUT y (its keep_sum = false form), xhat = (y - beta) / gamma
  const bool from_y = beta_y.has_value() && beta_y->defined();
  if (from_y) { CHECK_IN(*beta_y); CHECK_BF16(*beta_y); CHECK_BF16(gamma); TORCH_CHECK(beta_y->numel() == N && !rms); }
  int rc = ct_layernorm_bwd2(dy.data_ptr(), s.data_ptr(), gamma.data_ptr(), mean.data_ptr<float>(),
                             rstd.data_ptr<float>(), nullptr, ds.data_ptr(),
                             need_dx ? dx.data_ptr() : nullptr, part.data_ptr<float>(),
                             dgamma.data_ptr(), optr_mut(dbeta), optr_mut(dbias), M, N, rms ? 1 : 0,
                             dgamma.scalar_type() == at::kFloat ? 1 : 0, 1, (float)p_drop,
                             (uint64_t)seed, (uint64_t)offset, from_y ? 1 : 0, optr(beta_y), cur_stream());
  TORCH_CHECK(rc == 0, "layernorm_bwd_into: unsupported shape N=", N);
  return {ds, dx};
}

// ---------------------------------------------------------------- bias + activation
at::Tensor bias_act_fwd(at::Tensor z, c10::optional<at::Tensor> bias, int64_t act) {
  CHECK_IN(z); CHECK_BF16(z);
  const int N = z.size(-1);
  auto y = at::empty_like(z);
  int rc = ct_bias_act_fwd(z.data_ptr(), optr(bias), y.data_ptr(), z.numel() / N, N, (int)act, cur_stream());
  TORCH_CHECK(rc == 0, "bias_act_fwd: N % 8 != 0");
  return y;
}

std::vector<at::Tensor> bias_act_bwd(at::Tensor dy, at::Tensor z, c10::optional<at::Tensor> bias,
                                     int64_t act, bool need_dbias) {
  CHECK_IN(dy); CHECK_IN(z); CHECK_BF16(z); CHECK_BF16(dy);
  const int N = z.size(-1);
  const long M = z.numel() / N;
  auto dz = at::empty_like(z);
  at::Tensor dbias, part;
  if (need_dbias) {
    dbias = at::empty({N}, z.options());
    part = at::empty({(long)ct_bias_act_bwd_grid(M) * N}, z.options().dtype(at::kFloat));
  }
  int rc = ct_bias_act_bwd(dy.data_ptr(), z.data_ptr(), optr(bias), dz.data_ptr(),
                           need_dbias ? part.data_ptr<float>() : nullptr,
                           need_dbias ? dbias.data_ptr() : nullptr, M, N, (int)act, 0, 0, cur_stream());
  TORCH_CHECK(rc == 0, "bias_act_bwd: N % 8 != 0");
  return {dz, dbias};
}

// dz = dy * act'(z + bias) (skipped when want_dz is false: pure bias-gradient reduction);
// d(bias) accumulated into `dbias` (a view of the flat gradient buffer).
at::Tensor bias_act_bwd_into(at::Tensor dy, at::Tensor z, c10::optional<at::Tensor> bias, int64_t act,
                             at::Tensor dbias, bool want_dz) {
  CHECK_IN(dy); CHECK_IN(z); CHECK_BF16(z); CHECK_BF16(dy); CHECK_IN(dbias);
  const int N = z.size(-1);
  const long M = z.numel() / N;
  TORCH_CHECK(dbias.numel() == N && dy.numel() == z.numel());
  at::Tensor dz = want_dz ? at::empty_like(z) : at::Tensor();
  auto part = at::empty({(long)ct_bias_act_bwd_grid(M) * N}, z.options().dtype(at::kFloat));
  int rc = ct_bias_act_bwd(dy.data_ptr(), z.data_ptr(), optr(bias), want_dz ? dz.data_ptr() : nullptr,
                           part.data_ptr<float>(), dbias.data_ptr(), M, N, (int)act,
                           dbias.scalar_type() == at::kFloat ? 1 : 0, 1, cur_stream());
  TORCH_CHECK(rc == 0, "bias_act_bwd_into: N % 8 != 0");
  return dz;
}

at::Tensor dropout_fwd(at::Tensor x, double p, int64_t seed, int64_t offset) {
  CHECK_IN(x); CHECK_BF16(x);
  auto y = at::empty_like(x);
  int rc = ct_dropout(x.data_ptr(), y.data_ptr(), x.numel(), (float)p, (uint64_t)seed, (uint64_t)offset, cur_stream());
  TORCH_CHECK(rc == 0, "dropout: numel % 8 != 0");
  return y;
}

// ---------------------------------------------------------------- embeddings
at::Tensor embed3_fwd(at::Tensor ids, c10::optional<at::Tensor> tt, at::Tensor W,
                      c10::optional<at::Tensor> P, c10::optional<at::Tensor> T) {
  CHECK_IN(ids); CHECK_IN(W); CHECK_BF16(W);
  TORCH_CHECK(ids.scalar_type() == at::kLong, "ids must be int64");
  TORCH_CHECK(ids.dim() == 2, "ids must be [B, S]");
  const int S = ids.size(1), N = W.size(1), ntok = ids.numel();
  if (P.has_value() && P->defined()) TORCH_CHECK(P->size(0) >= S && P->size(1) == N);
  if (tt.has_value() && tt->defined()) TORCH_CHECK(tt->numel() == ntok && tt->scalar_type() == at::kLong);
  auto out = at::empty({ids.size(0), S, N}, W.options());
  int rc = ct_embed3_fwd(ids.data_ptr<int64_t>(),
                         (tt.has_value() && tt->defined()) ? tt->data_ptr<int64_t>() : nullptr,
                         W.data_ptr(), optr(P), optr(T), out.data_ptr(), ntok, S, N, cur_stream());
  TORCH_CHECK(rc == 0, "embed3_fwd: N % 8 != 0");
  return out;
}

void embed3_bwd(at::Tensor ids, c10::optional<at::Tensor> tt, at::Tensor g,
                c10::optional<at::Tensor> dW, c10::optional<at::Tensor> dP,
                c10::optional<at::Tensor> dT) {
  CHECK_IN(ids); CHECK_IN(g); CHECK_BF16(g);
  const int S = ids.size(1), N = g.size(-1), ntok = ids.numel();
  TORCH_CHECK(ids.dim() == 2 && g.numel() == (int64_t)ntok * N, "embed3_bwd: g must be [ids.numel(), N]");
  if (tt.has_value() && tt->defined()) TORCH_CHECK(tt->numel() == ntok, "embed3_bwd: token types shape");
  if (dP.has_value() && dP->defined()) TORCH_CHECK(dP->size(0) >= S, "embed3_bwd: position table too short");
  for (auto* t : {&dW, &dP, &dT}) if (t->has_value() && (*t)->defined()) { CHECK_F32(**t); CHECK_IN(**t); TORCH_CHECK((*t)->size(1) == N); }
  ct_embed3_bwd(ids.data_ptr<int64_t>(), (tt.has_value() && tt->defined()) ? tt->data_ptr<int64_t>() : nullptr,
                g.data_ptr(), (float*)optr_mut(dW), (float*)optr_mut(dP), (float*)optr_mut(dT), ntok, S,
                N, (dT.has_value() && dT->defined()) ? (int)dT->size(0) : 0, cur_stream());
}

void cast_into(at::Tensor x, at::Tensor y, double scale, bool accumulate) {
  CHECK_IN(x); CHECK_IN(y);
  TORCH_CHECK(x.numel() == y.numel());
  ct_cast(x.data_ptr(), dt_code(x), y.data_ptr(), dt_code(y), x.numel(), (float)scale, accumulate ? 1 : 0, cur_stream());
}

void splitk_reduce(at::Tensor partials, at::Tensor g, bool accumulate) {
  CHECK_IN(partials); CHECK_IN(g); CHECK_F32(partials); CHECK_BF16(g);
  TORCH_CHECK(partials.dim() >= 2 && partials[0].numel() == g.numel(), "splitk_reduce: shape mismatch");
  TORCH_CHECK(g.numel() % 8 == 0, "splitk_reduce: numel must be a multiple of 8");
  TORCH_CHECK(ct_splitk_reduce(partials.data_ptr<float>(), (int)partials.size(0), g.numel(), g.data_ptr(),
                               accumulate ? 1 : 0, cur_stream()) == 0);
}

// the same, and the partials are zeroed once read (persistent accumulation buffers)
// two (partials, g) reductions in one launch (see ct_splitk_reduce2)
void splitk_reduce2(at::Tensor p1, at::Tensor g1, at::Tensor p2, at::Tensor g2, bool accumulate) {
  for (auto* t : {&p1, &p2}) { CHECK_IN(*t); TORCH_CHECK(t->scalar_type() == at::kFloat && t->dim() >= 2); }
  for (auto* t : {&g1, &g2}) { CHECK_IN(*t); CHECK_BF16(*t); TORCH_CHECK(t->numel() % 8 == 0, "splitk_reduce2: numel % 8"); }
  TORCH_CHECK(p1[0].numel() == g1.numel() && p2[0].numel() == g2.numel(), "splitk_reduce2: shape mismatch");
  TORCH_CHECK(ct_splitk_reduce2(p1.data_ptr<float>(), (int)p1.size(0), g1.numel(), g1.data_ptr(),
                                p2.data_ptr<float>(), (int)p2.size(0), g2.numel(), g2.data_ptr(),
                                accumulate ? 1 : 0, cur_stream()) == 0);
}

void splitk_reduce_clear(at::Tensor partials, at::Tensor g, bool accumulate) {
  CHECK_IN(partials); CHECK_F32(partials); CHECK_IN(g); CHECK_BF16(g);
  TORCH_CHECK(partials.dim() >= 2 && partials[0].numel() == g.numel(), "splitk_reduce_clear: shape mismatch");
  TORCH_CHECK(g.numel() % 8 == 0, "splitk_reduce_clear: numel must be a multiple of 8");
  TORCH_CHECK(ct_splitk_reduce_clear(partials.data_ptr<float>(), (int)partials.size(0), g.numel(), g.data_ptr(),
                                     accumulate ? 1 : 0, cur_stream()) == 0, "splitk_reduce_clear failed");
}

// ---------------------------------------------------------------- optimizers
void lamb_step(at::Tensor g, at::Tensor m, at::Tensor v, at::Tensor w, c10::optional<at::Tensor> w_model,
               at::Tensor seg_tensor, at::Tensor seg_start, at::Tensor seg_len, at::Tensor tensor_first_seg,
               at::Tensor tensor_wd, at::Tensor dyn, double beta1, double beta2, double eps,
               bool bias_corr, bool trust_all, at::Tensor seg_part, at::Tensor tensor_part, int64_t stage) {
  for (auto* t : {&g, &m, &v, &w, &seg_tensor, &seg_start, &seg_len, &tensor_first_seg, &tensor_wd, &dyn, &seg_part, &tensor_part}) CHECK_IN(*t);
  CHECK_F32(m); CHECK_F32(v); CHECK_F32(w);
  TORCH_CHECK(g.numel() >= w.numel() && m.numel() == w.numel() && v.numel() == w.numel());
  const int nseg = seg_len.numel(), T = tensor_wd.numel();
  TORCH_CHECK(seg_part.numel() >= 2 * nseg && tensor_part.numel() >= 2 * T && tensor_first_seg.numel() == T + 1);
  int pdt = 0;
  if (w_model.has_value() && w_model->defined()) { CHECK_IN(*w_model); pdt = dt_code(*w_model); TORCH_CHECK(w_model->numel() >= w.numel()); }
  ct_lamb(g.data_ptr(), dt_code(g), m.data_ptr<float>(), v.data_ptr<float>(), w.data_ptr<float>(),
          optr_mut(w_model), pdt, seg_tensor.data_ptr<int>(), seg_start.data_ptr<int64_t>(),
          seg_len.data_ptr<int>(), nseg, tensor_first_seg.data_ptr<int>(), T,
          tensor_wd.data_ptr<float>(), dyn.data_ptr<float>(), (float)beta1, (float)beta2, (float)eps,
          bias_corr ? 1 : 0, trust_all ? 1 : 0, seg_part.data_ptr<float>(), tensor_part.data_ptr<float>(),
          (int)stage, cur_stream());
}

void adam_step(at::Tensor g, at::Tensor m, at::Tensor v, at::Tensor w, c10::optional<at::Tensor> w_model,
               at::Tensor seg_tensor, at::Tensor seg_start, at::Tensor seg_len, at::Tensor tensor_wd,
               at::Tensor dyn, double beta1, double beta2, double eps, bool adamw) {
  for (auto* t : {&g, &m, &v, &w, &seg_tensor, &seg_start, &seg_len, &tensor_wd, &dyn}) CHECK_IN(*t);
  CHECK_F32(m); CHECK_F32(v); CHECK_F32(w);
  TORCH_CHECK(g.numel() >= w.numel() && m.numel() == w.numel() && v.numel() == w.numel());
  int pdt = 0;
  if (w_model.has_value() && w_model->defined()) { CHECK_IN(*w_model); pdt = dt_code(*w_model); }
  ct_adam(g.data_ptr(), dt_code(g), m.data_ptr<float>(), v.data_ptr<float>(), w.data_ptr<float>(),
          optr_mut(w_model), pdt, seg_tensor.data_ptr<int>(), seg_start.data_ptr<int64_t>(),
          seg_len.data_ptr<int>(), seg_len.numel(), tensor_wd.data_ptr<float>(), dyn.data_ptr<float>(),
          (float)beta1, (float)beta2, (float)eps, adamw ? 1 : 0, cur_stream());
}

void sgd_step(at::Tensor g, c10::optional<at::Tensor> buf, at::Tensor w, c10::optional<at::Tensor> w_model,
              at::Tensor seg_tensor, at::Tensor seg_start, at::Tensor seg_len, at::Tensor tensor_wd,
              at::Tensor dyn, double momentum, double dampening, bool nesterov, bool first) {
  for (auto* t : {&g, &w, &seg_tensor, &seg_start, &seg_len, &tensor_wd, &dyn}) CHECK_IN(*t);
  CHECK_F32(w);
  TORCH_CHECK(g.numel() >= w.numel());
  if (momentum != 0.0) TORCH_CHECK(buf.has_value() && buf->defined() && buf->numel() == w.numel(), "momentum buffer");
  int pdt = 0;
  if (w_model.has_value() && w_model->defined()) { CHECK_IN(*w_model); pdt = dt_code(*w_model); }
  ct_sgd(g.data_ptr(), dt_code(g), (float*)optr_mut(buf), w.data_ptr<float>(), optr_mut(w_model), pdt,
         seg_tensor.data_ptr<int>(), seg_start.data_ptr<int64_t>(), seg_len.data_ptr<int>(), seg_len.numel(),
         tensor_wd.data_ptr<float>(), dyn.data_ptr<float>(), (float)momentum, (float)dampening,
         nesterov ? 1 : 0, first ? 1 : 0, cur_stream());
}

void sumsq_into(at::Tensor x, at::Tensor out) {
  CHECK_IN(x); CHECK_IN(out); CHECK_F32(out);
  TORCH_CHECK(x.numel() % 4 == 0, "sumsq: numel % 4");
  auto part = at::empty({2048}, out.options());
  ct_sumsq(x.data_ptr(), dt_code(x), x.numel(), out.data_ptr<float>(), part.data_ptr<float>(), cur_stream());
}

void clip_coef(at::Tensor sumsq, at::Tensor dyn, double base_scale, double max_norm) {
  ct_clip_coef(sumsq.data_ptr<float>(), dyn.data_ptr<float>(), (float)base_scale, (float)max_norm, cur_stream());
}

// ---------------------------------------------------------------- cross entropy
// logits [R, ld] bf16 (ld % 8 == 0); gradient written into `dlogits` (may be logits itself)
std::vector<at::Tensor> xent_fwd(at::Tensor logits, at::Tensor dlogits, int64_t V, at::Tensor labels,
                                 c10::optional<at::Tensor> scale, int64_t ignore_index,
                                 double label_smoothing) {
  CHECK_IN(logits); CHECK_BF16(logits); CHECK_IN(dlogits); CHECK_BF16(dlogits); CHECK_IN(labels);
  TORCH_CHECK(logits.dim() == 2 && dlogits.sizes() == logits.sizes());
  TORCH_CHECK(labels.scalar_type() == at::kLong && labels.numel() == logits.size(0));
  const int R = logits.size(0), ld = logits.size(1);
  TORCH_CHECK(V <= ld && ld % 8 == 0, "xent: ld must be a multiple of 8 and >= V");
  auto fo = logits.options().dtype(at::kFloat);
  auto loss = at::empty({R}, fo), lse = at::empty({R}, fo);
  const float* sp = nullptr;
  if (scale.has_value() && scale->defined()) { CHECK_F32(*scale); sp = scale->data_ptr<float>(); }
  ct_xent_fwd(logits.data_ptr(), dlogits.data_ptr(), ld, (int)V, labels.data_ptr<int64_t>(),
              loss.data_ptr<float>(), lse.data_ptr<float>(), sp, R, (int)ignore_index,
              (float)label_smoothing, cur_stream());
  return {loss, lse};
}

// ---------------------------------------------------------------- attention (head_dim 64)
// q, k, v, o: 4-D [B, S, H, 64] views with unit stride on the last dim (e.g. slices of a
// packed [B, S, 3, H, 64] QKV projection output); key_bias: fp32 [B, Sk] additive.
static void bshd_strides(const at::Tensor& t, long* st, const char* name) {
  TORCH_CHECK(t.dim() == 4 && t.size(3) == 64 && t.stride(3) == 1, name, " must be [B,S,H,64] with unit last stride");
  CHECK_CUDA(t); CHECK_BF16(t);
  st[0] = t.stride(0); st[1] = t.stride(1); st[2] = t.stride(2);
}

at::Tensor attn_fwd(at::Tensor q, at::Tensor k, at::Tensor v, at::Tensor o,
                    c10::optional<at::Tensor> key_bias, double scale, double p, int64_t seed,
                    int64_t offset, bool causal) {
  long qs[3], ks[3], vs[3], os[3];
  bshd_strides(q, qs, "q"); bshd_strides(k, ks, "k"); bshd_strides(v, vs, "v"); bshd_strides(o, os, "o");
  const int B = q.size(0), Sq = q.size(1), H = q.size(2), Sk = k.size(1);
  TORCH_CHECK(k.size(0) == B && v.size(0) == B && k.size(2) == H && v.size(2) == H && v.size(1) == Sk);
  TORCH_CHECK(o.size(0) == B && o.size(1) == Sq && o.size(2) == H);
  const float* kb = nullptr; long kb_sb = 0;
  if (key_bias.has_value() && key_bias->defined()) {
    CHECK_F32(*key_bias); CHECK_CUDA(*key_bias);
    TORCH_CHECK(key_bias->dim() == 2 && key_bias->size(0) == B && key_bias->size(1) == Sk && key_bias->stride(1) == 1);
    kb = key_bias->data_ptr<float>(); kb_sb = key_bias->stride(0);
  }
  auto lse = at::empty({(long)B * H, Sq}, q.options().dtype(at::kFloat));
  int rc = ct_attn_fwd(q.data_ptr(), qs, k.data_ptr(), ks, v.data_ptr(), vs, o.data_ptr(), os, kb, kb_sb,
                       lse.data_ptr<float>(), B, H, Sq, Sk, (float)scale, (float)p, (uint64_t)seed,
                       (uint64_t)offset, causal ? 1 : 0, cur_stream());
  TORCH_CHECK(rc == 0, "attn_fwd failed rc=", rc);
  return lse;
}

// inference forward with a T5-style relative-position bias vector relb [H, L]
at::Tensor attn_fwd_relbias(at::Tensor q, at::Tensor k, at::Tensor v, at::Tensor o,
                            c10::optional<at::Tensor> key_bias, at::Tensor relb, int64_t rel_base, double scale,
                            bool causal) {
  long qs[3], ks[3], vs[3], os[3];
  bshd_strides(q, qs, "q"); bshd_strides(k, ks, "k"); bshd_strides(v, vs, "v"); bshd_strides(o, os, "o");
  const int B = q.size(0), Sq = q.size(1), H = q.size(2), Sk = k.size(1);
  TORCH_CHECK(k.size(0) == B && v.size(0) == B && k.size(2) == H && v.size(2) == H && v.size(1) == Sk);
  TORCH_CHECK(o.size(0) == B && o.size(1) == Sq && o.size(2) == H);
  CHECK_F32(relb); CHECK_CUDA(relb);
  TORCH_CHECK(relb.dim() == 2 && relb.size(0) == H && (relb.stride(1) == 1 || relb.size(1) == 1),
              "relb must be [H, L] fp32");
  const long L = relb.size(1);
  TORCH_CHECK(rel_base >= Sq - 1 && rel_base + Sk <= L, "relb does not cover every (key - query) offset");
  const float* kb = nullptr; long kb_sb = 0;
  if (key_bias.has_value() && key_bias->defined()) {
    CHECK_F32(*key_bias); CHECK_CUDA(*key_bias);
    TORCH_CHECK(key_bias->dim() == 2 && key_bias->size(0) == B && key_bias->size(1) == Sk && key_bias->stride(1) == 1);
    kb = key_bias->data_ptr<float>(); kb_sb = key_bias->stride(0);
  }
  auto lse = at::empty({(long)B * H, Sq}, q.options().dtype(at::kFloat));
  int rc = ct_attn_fwd_relbias(q.data_ptr(), qs, k.data_ptr(), ks, v.data_ptr(), vs, o.data_ptr(), os, kb, kb_sb,
                               relb.data_ptr<float>(), relb.stride(0), (int)L, (int)rel_base, lse.data_ptr<float>(),
                               B, H, Sq, Sk, (float)scale, causal ? 1 : 0, cur_stream());
  TORCH_CHECK(rc == 0, "attn_fwd_relbias failed rc=", rc);
  return lse;
}

void attn_bwd(at::Tensor q, at::Tensor k, at::Tensor v, at::Tensor o, at::Tensor dO, at::Tensor dq,
              at::Tensor dk, at::Tensor dv, c10::optional<at::Tensor> key_bias, at::Tensor lse,
              double scale, double p, int64_t seed, int64_t offset, bool causal) {
  long qs[3], ks[3], vs[3], os[3], dos[3], dqs[3], dks[3], dvs[3];
  bshd_strides(q, qs, "q"); bshd_strides(k, ks, "k"); bshd_strides(v, vs, "v"); bshd_strides(o, os, "o");
  bshd_strides(dO, dos, "dO"); bshd_strides(dq, dqs, "dq"); bshd_strides(dk, dks, "dk"); bshd_strides(dv, dvs, "dv");
  const int B = q.size(0), Sq = q.size(1), H = q.size(2), Sk = k.size(1);
  TORCH_CHECK(dO.sizes() == o.sizes() && dq.sizes() == q.sizes() && dk.sizes() == k.sizes() && dv.sizes() == v.sizes());
  TORCH_CHECK(lse.numel() == (long)B * H * Sq);
  const float* kb = nullptr; long kb_sb = 0;
  if (key_bias.has_value() && key_bias->defined()) { kb = key_bias->data_ptr<float>(); kb_sb = key_bias->stride(0); }
  auto fo = q.options().dtype(at::kFloat);
  auto delta = at::empty({(long)B * H * Sq}, fo);
  at::Tensor dq_acc;
  if (Sk > 128) dq_acc = at::empty({(long)B * H * Sq * 64}, fo);
  int rc = ct_attn_bwd(q.data_ptr(), qs, k.data_ptr(), ks, v.data_ptr(), vs, o.data_ptr(), os, dO.data_ptr(), dos,
                       dq.data_ptr(), dqs, dk.data_ptr(), dks, dv.data_ptr(), dvs, kb, kb_sb,
                       lse.data_ptr<float>(), delta.data_ptr<float>(), Sk > 128 ? dq_acc.data_ptr<float>() : nullptr,
                       B, H, Sq, Sk, (float)scale, (float)p, (uint64_t)seed, (uint64_t)offset,
                       causal ? 1 : 0, cur_stream());
  TORCH_CHECK(rc == 0, "attn_bwd failed rc=", rc);
}

// ---------------------------------------------------------------- batchnorm (NHWC)
static void check_nhwc(const at::Tensor& x, const char* name) {
  CHECK_CUDA(x); CHECK_BF16(x);
  TORCH_CHECK(x.dim() == 4 ? x.is_contiguous(at::MemoryFormat::ChannelsLast) : x.is_contiguous(),
              name, " must be channels_last (4-D) or contiguous [M, C]");
}
static int64_t nhwc_rows(const at::Tensor& x) { return x.numel() / x.size(1); }

// optional ReLU bitmask output of the training forwards: uint8, one byte per 8 channels
static void* mask_ptr(const c10::optional<at::Tensor>& mask, const at::Tensor& x) {
  if (!mask.has_value() || !mask->defined()) return nullptr;
  TORCH_CHECK(mask->is_cuda() && mask->scalar_type() == at::kByte && mask->is_contiguous() &&
              mask->numel() * 8 == x.numel(), "ReLU mask: uint8 [numel / 8]");
  return mask->data_ptr();
}

// returns (y, stat) with stat = float[4C]: save_mean, save_invstd, a, b (y = x * a + b ...);
// mask_out (optional, uint8 [numel / 8]) receives the ReLU bitmask (bit j of byte v: y > 0)
std::vector<at::Tensor> bn_fwd_train(at::Tensor x, c10::optional<at::Tensor> res, at::Tensor gamma,
                                     at::Tensor beta, at::Tensor run_mean, at::Tensor run_var,
                                     double eps, double momentum, bool relu,
                                     c10::optional<at::Tensor> mask_out) {
  check_nhwc(x, "x");
  const int C = x.size(1);
  const long M = nhwc_rows(x);
  TORCH_CHECK(C <= 2048, "bn_fwd_train: C <= 2048");
  if (res.has_value() && res->defined()) { check_nhwc(*res, "residual"); TORCH_CHECK(res->sizes() == x.sizes()); }
  TORCH_CHECK(gamma.numel() == C && beta.numel() == C && run_mean.numel() == C && run_var.numel() == C);
  CHECK_F32(run_mean); CHECK_F32(run_var);
  auto y = at::empty_like(x);
  auto stat = at::empty({4 * (long)C}, x.options().dtype(at::kFloat));
  auto part = at::empty({2 * 2048 * (long)C}, x.options().dtype(at::kFloat));
  int rc = ct_bn_fwd_train(x.data_ptr(), optr(res), gamma.data_ptr(), beta.data_ptr(),
                           run_mean.data_ptr<float>(), run_var.data_ptr<float>(), y.data_ptr(),
                           part.data_ptr<float>(), stat.data_ptr<float>(), (int)M, C, (float)eps,
                           (float)momentum, relu ? 1 : 0, mask_ptr(mask_out, x), cur_stream());
  TORCH_CHECK(rc == 0, "bn_fwd_train: unsupported C=", C);
  return {y, stat};
}

// bn_fwd_train with the statistics already reduced per tile by x's producer (conv epilogue):
// part = means [tiles][C] then M2 [tiles][C], tiles = ceil(M / rows_per_tile)
std::vector<at::Tensor> bn_fwd_train_given(at::Tensor x, c10::optional<at::Tensor> res, at::Tensor gamma,
                                           at::Tensor beta, at::Tensor run_mean, at::Tensor run_var, at::Tensor part,
                                           int64_t rows_per_tile, double eps, double momentum, bool relu,
                                           c10::optional<at::Tensor> mask_out) {
  check_nhwc(x, "x");
  const int C = x.size(1);
  const long M = nhwc_rows(x);
  if (res.has_value() && res->defined()) { check_nhwc(*res, "residual"); TORCH_CHECK(res->sizes() == x.sizes()); }
  TORCH_CHECK(gamma.numel() == C && beta.numel() == C && run_mean.numel() == C && run_var.numel() == C);
  CHECK_F32(run_mean); CHECK_F32(run_var); CHECK_IN(part); CHECK_F32(part);
  const long tiles = (M + rows_per_tile - 1) / rows_per_tile;
  // the tail holds the first-level merge (ct_bn_fwd_train_given) when there are many tiles
  TORCH_CHECK(part.numel() >= 2 * (tiles + (tiles > 128 ? (tiles + 63) / 64 : 0)) * C,
              "bn_fwd_train_given: part buffer");
  auto y = at::empty_like(x);
  auto stat = at::empty({4 * (long)C}, x.options().dtype(at::kFloat));
  int rc = ct_bn_fwd_train_given(x.data_ptr(), optr(res), gamma.data_ptr(), beta.data_ptr(),
                                 run_mean.data_ptr<float>(), run_var.data_ptr<float>(), y.data_ptr(),
                                 part.data_ptr<float>(), (int)tiles, (int)rows_per_tile, stat.data_ptr<float>(),
                                 (int)M, C, (float)eps, (float)momentum, relu ? 1 : 0, mask_ptr(mask_out, x),
                                 cur_stream());
  TORCH_CHECK(rc == 0, "bn_fwd_train_given: unsupported C=", C);
  return {y, stat};
}

// y = relu(bn(x) + bn2(x2)) with both BatchNorms' statistics from their producers' partials (the
// ResNet downsample block: bn3(conv3) + down_bn(down)): returns (y, mask bytes, stat, stat2)
std::vector<at::Tensor> bn_fwd_train_given2(at::Tensor x, at::Tensor gamma, at::Tensor beta, at::Tensor run_mean,
                                            at::Tensor run_var, at::Tensor part, int64_t rows_per_tile,
                                            at::Tensor x2, at::Tensor gamma2, at::Tensor beta2,
                                            at::Tensor run_mean2, at::Tensor run_var2, at::Tensor part2,
                                            int64_t rows_per_tile2, double eps, double momentum) {
  check_nhwc(x, "x");
  check_nhwc(x2, "x2");
  TORCH_CHECK(x2.sizes() == x.sizes() && x2.strides() == x.strides(), "bn_fwd_train_given2: x2 layout");
  const int C = x.size(1);
  const long M = nhwc_rows(x);
  for (const at::Tensor* t : {&gamma, &beta, &run_mean, &run_var, &gamma2, &beta2, &run_mean2, &run_var2})
    TORCH_CHECK(t->numel() == C, "bn_fwd_train_given2: per-channel tensors");
  CHECK_F32(run_mean); CHECK_F32(run_var); CHECK_F32(run_mean2); CHECK_F32(run_var2);
  CHECK_IN(part); CHECK_F32(part); CHECK_IN(part2); CHECK_F32(part2);
  const long tiles = (M + rows_per_tile - 1) / rows_per_tile, tiles2 = (M + rows_per_tile2 - 1) / rows_per_tile2;
  TORCH_CHECK(part.numel() >= 2 * (tiles + (tiles > 128 ? (tiles + 63) / 64 : 0)) * C &&
              part2.numel() >= 2 * (tiles2 + (tiles2 > 128 ? (tiles2 + 63) / 64 : 0)) * C,
              "bn_fwd_train_given2: part buffers");
  auto y = at::empty_like(x);
  auto mask = at::empty({x.numel() / 8}, x.options().dtype(at::kByte));
  auto stat = at::empty({4 * (long)C}, x.options().dtype(at::kFloat));
  auto stat2 = at::empty({4 * (long)C}, x.options().dtype(at::kFloat));
  int rc = ct_bn_fwd_train_given2(x.data_ptr(), gamma.data_ptr(), beta.data_ptr(), run_mean.data_ptr<float>(),
                                  run_var.data_ptr<float>(), part.data_ptr<float>(), (int)tiles, (int)rows_per_tile,
                                  stat.data_ptr<float>(), x2.data_ptr(), gamma2.data_ptr(), beta2.data_ptr(),
                                  run_mean2.data_ptr<float>(), run_var2.data_ptr<float>(), part2.data_ptr<float>(),
                                  (int)tiles2, (int)rows_per_tile2, stat2.data_ptr<float>(), y.data_ptr(),
                                  mask.data_ptr(), (int)M, C, (float)eps, (float)momentum, cur_stream());
  TORCH_CHECK(rc == 0, "bn_fwd_train_given2: unsupported C=", C);
  return {y, mask, stat, stat2};
}

// backward of bn_fwd_train_given2 with the masked gradient and bn's partials from the consuming
// conv's epilogue: [dx, dx2, dgamma, dbeta, dgamma2, dbeta2] (accumulated into the *_acc targets,
// all four or none, when given)
std::vector<at::Tensor> bn_bwd_given_pair(at::Tensor dym, at::Tensor x, at::Tensor gamma, at::Tensor stat,
                                          at::Tensor part, int64_t tiles, int64_t rows, at::Tensor x2,
                                          at::Tensor gamma2, at::Tensor stat2,
                                          c10::optional<at::Tensor> dgamma_acc, c10::optional<at::Tensor> dbeta_acc,
                                          c10::optional<at::Tensor> dgamma2_acc,
                                          c10::optional<at::Tensor> dbeta2_acc) {
  check_nhwc(x, "x");
  check_nhwc(x2, "x2");
  check_nhwc(dym, "dym");
  const int C = x.size(1);
  const long M = nhwc_rows(x);
  TORCH_CHECK(dym.sizes() == x.sizes() && dym.strides() == x.strides() && x2.sizes() == x.sizes() &&
              x2.strides() == x.strides(), "bn_bwd_given_pair: layouts");
  TORCH_CHECK(C <= 2048 && stat.numel() == 4 * (long)C && stat2.numel() == 4 * (long)C, "bn_bwd_given_pair: stat");
  CHECK_F32(stat); CHECK_F32(stat2); CHECK_F32(part);
  TORCH_CHECK(tiles > 0 && tiles <= rows && part.numel() >= 2 * rows * C, "bn_bwd_given_pair: part buffer");
  TORCH_CHECK(gamma2.scalar_type() == gamma.scalar_type(), "bn_bwd_given_pair: parameter dtypes");
  const bool acc = dgamma_acc.has_value() && dgamma_acc->defined();
  for (const auto* t : {&dbeta_acc, &dgamma2_acc, &dbeta2_acc})
    TORCH_CHECK((t->has_value() && (*t)->defined()) == acc, "bn_bwd_given_pair: accumulate targets: all or none");
  if (acc) {
    for (const auto* t : {&dgamma_acc, &dbeta_acc, &dgamma2_acc, &dbeta2_acc})
      TORCH_CHECK((*t)->is_contiguous() && (*t)->numel() == C && (*t)->scalar_type() == gamma.scalar_type(),
                  "bn_bwd_given_pair: bad accumulate target");
  }
  auto dx = at::empty_like(x), dx2 = at::empty_like(x2);
  auto dg = acc ? *dgamma_acc : at::empty_like(gamma), db = acc ? *dbeta_acc : at::empty_like(gamma);
  auto dg2 = acc ? *dgamma2_acc : at::empty_like(gamma2), db2 = acc ? *dbeta2_acc : at::empty_like(gamma2);
  const long G = (tiles + 63) / 64;
  auto work = at::empty({2 * G * C + 3 * (long)C}, x.options().dtype(at::kFloat));
  auto part2 = at::empty({2 * 2048 * (long)C}, x.options().dtype(at::kFloat));
  auto coef2 = at::empty({3 * (long)C}, x.options().dtype(at::kFloat));
  int rc = ct_bn_bwd_given_pair(dym.data_ptr(), x.data_ptr(), gamma.data_ptr(), stat.data_ptr<float>(),
                                part.data_ptr<float>(), rows * C, (int)tiles, x2.data_ptr(), gamma2.data_ptr(),
                                stat2.data_ptr<float>(), dx.data_ptr(), dx2.data_ptr(), dg.data_ptr(), db.data_ptr(),
                                dg2.data_ptr(), db2.data_ptr(),
                                (gamma.scalar_type() == at::kFloat ? 1 : 0) | (acc ? 2 : 0), work.data_ptr<float>(),
                                part2.data_ptr<float>(), coef2.data_ptr<float>(), (int)M, C, cur_stream());
  TORCH_CHECK(rc == 0, "bn_bwd_given_pair: unsupported C=", C);
  return {dx, dx2, dg, db, dg2, db2};
}

// ResNet stem: returns (y_pool [N, C, OH, OW] channels_last, argmax bytes [N, OH, OW, C] uint8, stat)
std::vector<at::Tensor> bn_fwd_train_pool(at::Tensor x, at::Tensor gamma, at::Tensor beta, at::Tensor run_mean,
                                          at::Tensor run_var, double eps, double momentum) {
  check_nhwc(x, "x");
  TORCH_CHECK(x.dim() == 4, "bn_fwd_train_pool: 4-D NHWC input");
  const int N = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3);
  const int OH = (H - 1) / 2 + 1, OW = (W - 1) / 2 + 1;
  TORCH_CHECK(C % 8 == 0 && C <= 2048, "bn_fwd_train_pool: C % 8 == 0, C <= 2048");
  TORCH_CHECK(gamma.numel() == C && beta.numel() == C && run_mean.numel() == C && run_var.numel() == C);
  CHECK_F32(run_mean); CHECK_F32(run_var);
  auto y = at::empty({N, C, OH, OW}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  auto arg = at::empty({N, OH, OW, C}, x.options().dtype(at::kByte));
  auto stat = at::empty({4 * (long)C}, x.options().dtype(at::kFloat));
  auto part = at::empty({2 * 2048 * (long)C}, x.options().dtype(at::kFloat));
  int rc = ct_bn_fwd_train_pool(x.data_ptr(), gamma.data_ptr(), beta.data_ptr(), run_mean.data_ptr<float>(),
                                run_var.data_ptr<float>(), y.data_ptr(), arg.data_ptr(), part.data_ptr<float>(),
                                stat.data_ptr<float>(), N, H, W, C, OH, OW, (float)eps, (float)momentum, cur_stream());
  TORCH_CHECK(rc == 0, "bn_fwd_train_pool: unsupported shape");
  return {y, arg, stat};
}

// bn_fwd_train_pool with the statistics from the conv epilogue's per-tile partials (part, rows
// per tile: conv_fwd(..., partials=True)); returns (y_pool, argmax bytes, stat)
std::vector<at::Tensor> bn_fwd_train_pool_given(at::Tensor x, at::Tensor gamma, at::Tensor beta,
                                                at::Tensor run_mean, at::Tensor run_var, at::Tensor part,
                                                int64_t rows_per_tile, double eps, double momentum) {
  check_nhwc(x, "x");
  TORCH_CHECK(x.dim() == 4, "bn_fwd_train_pool_given: 4-D NHWC input");
  const int N = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3);
  const int OH = (H - 1) / 2 + 1, OW = (W - 1) / 2 + 1;
  const long M = (long)N * H * W;
  TORCH_CHECK(C % 8 == 0 && C <= 2048, "bn_fwd_train_pool_given: C % 8 == 0, C <= 2048");
  TORCH_CHECK(gamma.numel() == C && beta.numel() == C && run_mean.numel() == C && run_var.numel() == C);
  CHECK_F32(run_mean); CHECK_F32(run_var); CHECK_IN(part); CHECK_F32(part);
  TORCH_CHECK(rows_per_tile > 0, "bn_fwd_train_pool_given: rows per tile");
  const long tiles = (M + rows_per_tile - 1) / rows_per_tile;
  TORCH_CHECK(part.numel() >= 2 * (tiles + (tiles > 128 ? (tiles + 63) / 64 : 0)) * C,
              "bn_fwd_train_pool_given: part buffer");
  auto y = at::empty({N, C, OH, OW}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  auto arg = at::empty({N, OH, OW, C}, x.options().dtype(at::kByte));
  auto stat = at::empty({4 * (long)C}, x.options().dtype(at::kFloat));
  int rc = ct_bn_fwd_train_pool_given(x.data_ptr(), gamma.data_ptr(), beta.data_ptr(), run_mean.data_ptr<float>(),
                                      run_var.data_ptr<float>(), y.data_ptr(), arg.data_ptr(), part.data_ptr<float>(),
                                      (int)tiles, (int)rows_per_tile, stat.data_ptr<float>(), N, H, W, C, OH, OW,
                                      (float)eps, (float)momentum, cur_stream());
  TORCH_CHECK(rc == 0, "bn_fwd_train_pool_given: unsupported shape");
  return {y, arg, stat};
}

// gradient of maxpool3x3/s2/p1 from the byte argmax: dx [N, C, H, W] channels_last
at::Tensor maxpool3s2_bwd(at::Tensor dy, at::Tensor arg, int64_t H, int64_t W) {
  at::Tensor dyc = dy.contiguous(at::MemoryFormat::ChannelsLast);
  check_nhwc(dyc, "dy");
  const int N = dyc.size(0), C = dyc.size(1), OH = dyc.size(2), OW = dyc.size(3);
  TORCH_CHECK(arg.scalar_type() == at::kByte && arg.is_contiguous() && arg.numel() == dyc.numel(),
              "maxpool3s2_bwd: argmax bytes");
  TORCH_CHECK(OH == (H - 1) / 2 + 1 && OW == (W - 1) / 2 + 1 && C % 8 == 0, "maxpool3s2_bwd: shape");
  auto dx = at::empty({N, C, (long)H, (long)W}, dyc.options().memory_format(at::MemoryFormat::ChannelsLast));
  int rc = ct_maxpool3s2_bwd(dyc.data_ptr(), arg.data_ptr(), dx.data_ptr(), N, (int)H, (int)W, C, OH, OW,
                             cur_stream());
  TORCH_CHECK(rc == 0, "maxpool3s2_bwd: unsupported shape");
  return dx;
}

// stem backward: the max-pool gradient gather + the BatchNorm's ReLU mask and backward sums in one
// pass; returns the masked gradient (at x's shape) and fills part (float[2 * rows * C]: p1 rows
// then p2 rows, rows = maxpool3s2_bwd_bn_rows(N, H) tiles) for bn_bwd_given
at::Tensor maxpool3s2_bwd_bn(at::Tensor dy, at::Tensor arg, at::Tensor x, at::Tensor stat, at::Tensor part) {
  at::Tensor dyc = dy.contiguous(at::MemoryFormat::ChannelsLast);
  check_nhwc(dyc, "dy");
  check_nhwc(x, "x");
  CHECK_F32(stat);
  CHECK_F32(part);
  const int N = dyc.size(0), C = dyc.size(1), OH = dyc.size(2), OW = dyc.size(3);
  const int H = x.size(2), W = x.size(3);
  TORCH_CHECK(x.size(0) == N && x.size(1) == C && stat.numel() == 4 * (long)C, "maxpool3s2_bwd_bn: shapes");
  TORCH_CHECK(arg.scalar_type() == at::kByte && arg.is_contiguous() && arg.numel() == dyc.numel(),
              "maxpool3s2_bwd_bn: argmax bytes");
  TORCH_CHECK(part.is_contiguous() && part.numel() >= 2L * ct_maxpool3s2_bwd_bn_rows(N, H) * C,
              "maxpool3s2_bwd_bn: part buffer");
  auto dxm = at::empty_like(x);
  int rc = ct_maxpool3s2_bwd_bn(dyc.data_ptr(), arg.data_ptr(), x.data_ptr(), stat.data_ptr<float>(), dxm.data_ptr(),
                                part.data_ptr<float>(), N, H, W, C, OH, OW, cur_stream());
  TORCH_CHECK(rc == 0, "maxpool3s2_bwd_bn: unsupported shape");
  return dxm;
}

at::Tensor bn_apply(at::Tensor x, c10::optional<at::Tensor> res, at::Tensor a, at::Tensor b, bool relu) {
  check_nhwc(x, "x");
  const int C = x.size(1);
  CHECK_F32(a); CHECK_F32(b); TORCH_CHECK(a.numel() == C && b.numel() == C);
  auto y = at::empty_like(x);
  int rc = ct_bn_apply(x.data_ptr(), optr(res), a.data_ptr<float>(), b.data_ptr<float>(), y.data_ptr(),
                       (int)nhwc_rows(x), C, relu ? 1 : 0, cur_stream());
  TORCH_CHECK(rc == 0, "bn_apply: unsupported C");
  return y;
}

// returns (dx, dres, dgamma, dbeta).  relu_mode: 0 no ReLU, 1 mask from y (forward had a
// residual), 2 mask recomputed from x and the forward's (a, b) -- y may be undefined then,
// 3 y is the forward's ReLU bitmask (uint8 [numel / 8]).
std::vector<at::Tensor> bn_bwd(at::Tensor dy, c10::optional<at::Tensor> y, at::Tensor x, at::Tensor gamma,
                               at::Tensor stat, int64_t relu_mode, bool need_dres,
                               c10::optional<at::Tensor> dgamma_acc, c10::optional<at::Tensor> dbeta_acc) {
  check_nhwc(x, "x");
  at::Tensor dyc = dy.dim() == 4 ? dy.contiguous(at::MemoryFormat::ChannelsLast) : dy.contiguous();
  check_nhwc(dyc, "dy");
  const int C = x.size(1);
  const long M = nhwc_rows(x);
  TORCH_CHECK(C <= 2048 && stat.numel() == 4 * (long)C, "bn_bwd: stat must be float[4C], C <= 2048");
  CHECK_F32(stat);
  TORCH_CHECK(relu_mode >= 0 && relu_mode <= 3, "bn_bwd: relu_mode 0/1/2/3");
  if (relu_mode == 1) {
    TORCH_CHECK(y.has_value() && y->defined(), "bn_bwd: relu_mode 1 needs y");
    check_nhwc(*y, "y");
    TORCH_CHECK(y->sizes() == x.sizes(), "bn_bwd: y shape");
  }
  if (relu_mode == 3) {
    TORCH_CHECK(y.has_value() && y->defined(), "bn_bwd: relu_mode 3 needs the mask");
    mask_ptr(y, x);
  }
  TORCH_CHECK(dyc.sizes() == x.sizes(), "bn_bwd: dy shape");
  auto dx = at::empty_like(x);
  at::Tensor dres = need_dres ? at::empty_like(x) : at::Tensor();
  // optional accumulate targets (flat gradient buffer views): both or neither
  const bool acc = dgamma_acc.has_value() && dgamma_acc->defined();
  if (acc) {
    TORCH_CHECK(dbeta_acc.has_value() && dbeta_acc->defined(), "bn_bwd: dgamma_acc needs dbeta_acc");
    TORCH_CHECK(dgamma_acc->is_contiguous() && dbeta_acc->is_contiguous() && dgamma_acc->numel() == C &&
                dbeta_acc->numel() == C && dgamma_acc->scalar_type() == gamma.scalar_type() &&
                dbeta_acc->scalar_type() == gamma.scalar_type(), "bn_bwd: bad accumulate targets");
  }
  auto dgamma = acc ? *dgamma_acc : at::empty_like(gamma), dbeta = acc ? *dbeta_acc : at::empty_like(gamma);
  auto coef = at::empty({3 * (long)C}, x.options().dtype(at::kFloat));
  auto part = at::empty({2 * 2048 * (long)C}, x.options().dtype(at::kFloat));
  int rc = ct_bn_bwd(dyc.data_ptr(), (relu_mode == 1 || relu_mode == 3) ? y->data_ptr() : nullptr, x.data_ptr(),
                     gamma.data_ptr(),
                     stat.data_ptr<float>(), dx.data_ptr(), need_dres ? dres.data_ptr() : nullptr,
                     dgamma.data_ptr(), dbeta.data_ptr(),
                     (gamma.scalar_type() == at::kFloat ? 1 : 0) | (acc ? 2 : 0), part.data_ptr<float>(),
                     coef.data_ptr<float>(), (int)M, C, (int)relu_mode, cur_stream());
  TORCH_CHECK(rc == 0, "bn_bwd: unsupported C=", C);
  return {dx, dres, dgamma, dbeta};
}

// BatchNorm (+ ReLU) backward from the reduction done by the conv that produced dy
// (conv_igemm_bn): dym = the masked gradient, part = float[2 * rows * C] per-tile sums (first
// `tiles` rows of each half).  Returns (dx, dgamma, dbeta).
std::vector<at::Tensor> bn_bwd_given(at::Tensor dym, at::Tensor x, at::Tensor gamma, at::Tensor stat, at::Tensor part,
                                     int64_t tiles, int64_t rows, c10::optional<at::Tensor> dgamma_acc,
                                     c10::optional<at::Tensor> dbeta_acc) {
  check_nhwc(x, "x");
  check_nhwc(dym, "dym");
  const int C = x.size(1);
  const long M = nhwc_rows(x);
  TORCH_CHECK(dym.sizes() == x.sizes() && dym.strides() == x.strides(), "bn_bwd_given: dym / x layout");
  TORCH_CHECK(C <= 2048 && stat.numel() == 4 * (long)C, "bn_bwd_given: stat must be float[4C], C <= 2048");
  CHECK_F32(stat);
  CHECK_F32(part);
  TORCH_CHECK(tiles > 0 && tiles <= rows && part.numel() >= 2 * rows * C, "bn_bwd_given: part buffer");
  const bool acc = dgamma_acc.has_value() && dgamma_acc->defined();
  if (acc) {
    TORCH_CHECK(dbeta_acc.has_value() && dbeta_acc->defined(), "bn_bwd_given: dgamma_acc needs dbeta_acc");
    TORCH_CHECK(dgamma_acc->is_contiguous() && dbeta_acc->is_contiguous() && dgamma_acc->numel() == C &&
                dbeta_acc->numel() == C && dgamma_acc->scalar_type() == gamma.scalar_type() &&
                dbeta_acc->scalar_type() == gamma.scalar_type(), "bn_bwd_given: bad accumulate targets");
  }
  auto dx = at::empty_like(x);
  auto dgamma = acc ? *dgamma_acc : at::empty_like(gamma), dbeta = acc ? *dbeta_acc : at::empty_like(gamma);
  const long G = (tiles + 63) / 64;
  auto work = at::empty({2 * G * C + 3 * (long)C}, x.options().dtype(at::kFloat));
  int rc = ct_bn_bwd_given(dym.data_ptr(), x.data_ptr(), gamma.data_ptr(), stat.data_ptr<float>(), dx.data_ptr(),
                           dgamma.data_ptr(), dbeta.data_ptr(),
                           (gamma.scalar_type() == at::kFloat ? 1 : 0) | (acc ? 2 : 0), part.data_ptr<float>(),
                           rows * C, (int)tiles, work.data_ptr<float>(), (int)M, C, cur_stream());
  TORCH_CHECK(rc == 0, "bn_bwd_given: unsupported C=", C);
  return {dx, dgamma, dbeta};
}

// The BatchNorm backward's per-channel results WITHOUT the apply pass: (dgamma, dbeta, coef) from
// the producer's per-tile sums, coef = float[3C] = (ca, c1, c0) with dx = ca dym + c1 x + c0.  For
// a BatchNorm whose input gradient only feeds a weight gradient (the ResNet stem: dW = ca G1 +
// c1 G2 + c0 G0 over the conv's im2col columns, ops/functional.py _StemBlockFn).
std::vector<at::Tensor> bn_bwd_coefs_given(int64_t M, at::Tensor gamma, at::Tensor stat, at::Tensor part,
                                           int64_t tiles, int64_t rows, c10::optional<at::Tensor> dgamma_acc,
                                           c10::optional<at::Tensor> dbeta_acc) {
  const int C = (int)gamma.numel();
  TORCH_CHECK(gamma.is_cuda() && C % 8 == 0 && C <= 2048 && stat.numel() == 4 * (long)C, "bn_bwd_coefs_given: stat");
  CHECK_F32(stat);
  CHECK_F32(part);
  TORCH_CHECK(M > 0 && tiles > 0 && tiles <= rows && part.numel() >= 2 * rows * C, "bn_bwd_coefs_given: part buffer");
  const bool acc = dgamma_acc.has_value() && dgamma_acc->defined();
  if (acc) {
    TORCH_CHECK(dbeta_acc.has_value() && dbeta_acc->defined() && dgamma_acc->is_contiguous() &&
                dbeta_acc->is_contiguous() && dgamma_acc->numel() == C && dbeta_acc->numel() == C &&
                dgamma_acc->scalar_type() == gamma.scalar_type() && dbeta_acc->scalar_type() == gamma.scalar_type(),
                "bn_bwd_coefs_given: bad accumulate targets");
  }
  auto dgamma = acc ? *dgamma_acc : at::empty_like(gamma), dbeta = acc ? *dbeta_acc : at::empty_like(gamma);
  const long G = (tiles + 63) / 64;
  auto work = at::empty({2 * G * C + 3 * (long)C}, gamma.options().dtype(at::kFloat));
  int rc = ct_bn_bwd_given(nullptr, nullptr, gamma.data_ptr(), stat.data_ptr<float>(), nullptr, dgamma.data_ptr(),
                           dbeta.data_ptr(), (gamma.scalar_type() == at::kFloat ? 1 : 0) | (acc ? 2 : 0),
                           part.data_ptr<float>(), rows * C, (int)tiles, work.data_ptr<float>(), (int)M, C, cur_stream());
  TORCH_CHECK(rc == 0, "bn_bwd_coefs_given: unsupported C=", C);
  return {dgamma, dbeta, work.narrow(0, 2 * G * C, 3 * (long)C)};
}

void register_ext(pybind11::module& m);   // bindings_ext.cpp
void register_graph(pybind11::module& m); // bindings_graph.cpp
void register_deform(pybind11::module& m); // bindings_deform.cpp
void register_p2p(pybind11::module& m);    // bindings_p2p.cpp
void register_lt(pybind11::module& m);     // bindings_lt.cpp
void register_conv(pybind11::module& m);   // bindings_conv.cpp

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.doc() = "cloudtik_amd CDNA4 (gfx950) op library";
  register_ext(m);
  register_graph(m);
  register_deform(m);
  register_p2p(m);
  register_lt(m);
  register_conv(m);
  m.def("maxpool3s2_bwd_bn", &maxpool3s2_bwd_bn);
  m.def("bn_fwd_train_given2", &bn_fwd_train_given2);
  m.def("bn_bwd_given_pair", &bn_bwd_given_pair);
  m.def("maxpool3s2_bwd_bn_rows", [](int64_t N, int64_t H) { return (int64_t)ct_maxpool3s2_bwd_bn_rows((int)N, (int)H); });
  m.def("layernorm_fwd", &layernorm_fwd, pybind11::arg("x"), pybind11::arg("bias"), pybind11::arg("res"),
        pybind11::arg("gamma"), pybind11::arg("beta"), pybind11::arg("eps"), pybind11::arg("rms"),
        pybind11::arg("p_drop"), pybind11::arg("seed"), pybind11::arg("offset"), pybind11::arg("keep_sum") = true);
  m.def("layernorm_bwd", &layernorm_bwd);
  m.def("bias_act_fwd", &bias_act_fwd);
  m.def("bias_act_bwd", &bias_act_bwd);
  m.def("bias_act_bwd_into", &bias_act_bwd_into);
  m.def("layernorm_bwd_into", &layernorm_bwd_into, pybind11::arg("dy"), pybind11::arg("s"), pybind11::arg("gamma"),
        pybind11::arg("mean"), pybind11::arg("rstd"), pybind11::arg("rms"), pybind11::arg("dgamma"),
        pybind11::arg("dbeta"), pybind11::arg("dbias"), pybind11::arg("need_dx"), pybind11::arg("p_drop"),
        pybind11::arg("seed"), pybind11::arg("offset"), pybind11::arg("beta_y") = pybind11::none());
  m.def("dropout_fwd", &dropout_fwd);
  m.def("embed3_fwd", &embed3_fwd);
  m.def("embed3_bwd", &embed3_bwd);
  m.def("cast_into", &cast_into);
  m.def("splitk_reduce", &splitk_reduce);
  m.def("splitk_reduce_clear", &splitk_reduce_clear);
  m.def("splitk_reduce2", &splitk_reduce2);
  m.def("lamb_step", &lamb_step);
  m.def("adam_step", &adam_step);
  m.def("sgd_step", &sgd_step);
  m.def("sumsq_into", &sumsq_into);
  m.def("clip_coef", &clip_coef);
  m.def("xent_fwd", &xent_fwd);
  m.def("bn_fwd_train", &bn_fwd_train, pybind11::arg("x"), pybind11::arg("res"), pybind11::arg("gamma"),
        pybind11::arg("beta"), pybind11::arg("run_mean"), pybind11::arg("run_var"), pybind11::arg("eps"),
        pybind11::arg("momentum"), pybind11::arg("relu"), pybind11::arg("mask_out") = pybind11::none());
  m.def("bn_apply", &bn_apply);
  m.def("bn_fwd_train_given", &bn_fwd_train_given, pybind11::arg("x"), pybind11::arg("res"), pybind11::arg("gamma"),
        pybind11::arg("beta"), pybind11::arg("run_mean"), pybind11::arg("run_var"), pybind11::arg("part"),
        pybind11::arg("rows_per_tile"), pybind11::arg("eps"), pybind11::arg("momentum"), pybind11::arg("relu"),
        pybind11::arg("mask_out") = pybind11::none());
  m.def("bn_fwd_train_pool", &bn_fwd_train_pool);
  m.def("bn_fwd_train_pool_given", &bn_fwd_train_pool_given);
  m.def("maxpool3s2_bwd", &maxpool3s2_bwd);
  m.def("bn_bwd", &bn_bwd);
  m.def("bn_bwd_given", &bn_bwd_given);
  m.def("bn_bwd_coefs_given", &bn_bwd_coefs_given);
  m.def("attn_fwd_relbias", &attn_fwd_relbias);
  m.def("attn_fwd", &attn_fwd);
  m.def("attn_bwd", &attn_bwd);
}

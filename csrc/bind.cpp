// Python bindings for the gfx950 kernel library (one in-tree extension: distributed_llms_example_amd/_C).
// Host-side validation lives here: every shape / dtype / stride / alignment a kernel assumes is checked
// BEFORE launch (a kernel that faults can reset every GPU on the node), then the C-ABI launchers in
// csrc/*.hip run on the current torch HIP stream.
#include <algorithm>
#include <climits>
#include <cstdlib>

#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>
#include <c10/hip/HIPStream.h>

#include "attn_f32_params.h"
#include "attn_params.h"
#include "gemm_params.h"
#include "route.h"

extern "C" {
int dllm_norm_fwd(const void*, const void*, const void*, const void*, void*, void*, float*, float*, int, int, float,
                  float, uint32_t, int, int, hipStream_t);
int dllm_norm_bwd_grid(int);
int dllm_norm_bwd(const void*, const void*, const void*, const void*, const float*, const float*, void*, void*,
                  float*, float*, float*, float*, void*, void*, float*, float*, int, int, float, uint32_t, int, int, int,
                  hipStream_t);
int dllm_act_fwd(const void*, void*, long, int, int, int, float, uint32_t, int, hipStream_t);
int dllm_act_bwd(const void*, const void*, void*, long, int, int, int, float, uint32_t, int, hipStream_t);
int dllm_dropout(const void*, void*, long, float, uint32_t, int, hipStream_t);
int dllm_ce_fwd(const void*, const int64_t*, const float*, float*, float*, long, int, float, long, int, hipStream_t);
int dllm_ce_bwd(const float*, const void*, const int64_t*, const float*, const float*, void*, long, int, float, long,
                int, hipStream_t);
int dllm_sq_norm(const void*, long, float*, float*, int, hipStream_t);
int dllm_adamw(void*, float*, const void*, float*, float*, const uint8_t*, const float*, long, float, float, float,
               float, float, float, float, int, int, const float*, hipStream_t);
int dllm_set_seed_step_norm(const uint32_t*);
int dllm_set_seed_step_act(const uint32_t*);
int dllm_set_seed_step_attn(const uint32_t*);
int dllm_set_seed_step_gemm_fused(const uint32_t*);
int dllm_attn_fwd(AttnParams*, hipStream_t);
int dllm_attn_bwd(AttnParams*, hipStream_t);
int dllm_attn_params_size();
int dllm_attn_dropout_mask(AttnParams*, hipStream_t);
int dllm_attn_f32_fwd(AttnF32Params*, hipStream_t);
int dllm_attn_f32_bwd(AttnF32Params*, hipStream_t);
int dllm_set_seed_step_attn_f32(const uint32_t*);
int dllm_wgrad_reduce(const GemmWgradParams*, hipStream_t);
int dllm_gemm_fused(const GemmFusedParams*, int, int, hipStream_t);
int dllm_gemm_w4(const GemmW4Params*, int, int, int, hipStream_t);
int dllm_set_seed_step_gemm_w4(const uint32_t*);
int dllm_colsum_rows();
int dllm_ce_chunk_fwd(const void*, long, const int64_t*, const float*, float*, float*, float*, long, int, int, int, float,
                      long, int, int, int, hipStream_t);
int dllm_ce_chunk_bwd(const float*, void*, long, const int64_t*, const float*, const float*, long, int, int, int, float,
                      long, int, hipStream_t);
int dllm_embed_bwd(const int64_t*, const int64_t*, const void*, long, long, int, float*, void*, long, long, int,
                   hipStream_t);
int dllm_colsum_acc(const void*, long, long, int, float*, void*, int, hipStream_t);
int dllm_colsum_partials_acc(const float*, void*, int, int, int, hipStream_t);
int dllm_ce_merge(const float*, int, long, const float*, const int64_t*, float*, float*, long, int, float, long,
                  hipStream_t);
int dllm_kv_reorder(void*, const int64_t*, int, int, int, int, int, int, hipStream_t);
int dllm_beam_topk(const void*, long, int, const float*, const int64_t*, long, int, int, int, int, int, int, int, int,
                   float*, int64_t*, hipStream_t);
}

namespace {

using at::Tensor;
using c10::optional;

hipStream_t stream() { return c10::hip::getCurrentHIPStream().stream(); }

void check_rc(int rc, const char* what) {
  TORCH_CHECK(rc == 0, "dllm kernel launch failed (", what, "): rc=", rc,
              rc > 0 ? std::string(" ") + hipGetErrorString((hipError_t)rc) : std::string(""));
}

void check_gpu(const Tensor& t, const char* n) {
  TORCH_CHECK(t.is_cuda(), n, " must be a GPU tensor");
}

bool is_bf16(const Tensor& t) {
  TORCH_CHECK(t.scalar_type() == at::kBFloat16 || t.scalar_type() == at::kFloat, "unsupported dtype ",
              t.scalar_type());
  return t.scalar_type() == at::kBFloat16;
}

void check_aligned(const Tensor& t, int bytes, const char* n) {
  TORCH_CHECK(reinterpret_cast<uintptr_t>(t.data_ptr()) % bytes == 0, n, " must be ", bytes, "-byte aligned");
}

const void* opt_ptr(const optional<Tensor>& t) { return t.has_value() && t->defined() ? t->data_ptr() : nullptr; }

// ------------------------------------------------------------------------------------------- norms
std::vector<Tensor> norm_fwd(const Tensor& x, const optional<Tensor>& resid, const Tensor& w,
                             const optional<Tensor>& b, double eps, double p, int64_t seed, int64_t kind,
                             bool want_s) {
  check_gpu(x, "x");
  TORCH_CHECK(x.dim() == 2 && x.is_contiguous(), "x must be contiguous [N, d]");
  const int N = x.size(0), d = x.size(1);
  TORCH_CHECK(d % 4 == 0 && d <= 2048, "norm: d must be a multiple of 4 and <= 2048, got ", d);
  TORCH_CHECK(w.numel() == d && w.is_contiguous() && w.scalar_type() == x.scalar_type(), "norm weight mismatch");
  if (resid.has_value() && resid->defined())
    TORCH_CHECK(resid->sizes() == x.sizes() && resid->is_contiguous() && resid->scalar_type() == x.scalar_type(),
                "resid mismatch");
  if (b.has_value() && b->defined())
    TORCH_CHECK(b->numel() == d && b->is_contiguous() && b->scalar_type() == x.scalar_type(), "norm bias mismatch");
  const bool need_s = want_s && ((resid.has_value() && resid->defined()) || p > 0.0);
  auto out = at::empty_like(x);
  Tensor s = need_s ? at::empty_like(x) : Tensor();
  auto f32 = x.options().dtype(at::kFloat);
  auto rstd = at::empty({N}, f32);
  auto mean = kind == 1 ? at::empty({N}, f32) : Tensor();
  if (N > 0)
    check_rc(dllm_norm_fwd(x.data_ptr(), opt_ptr(resid), w.data_ptr(), opt_ptr(b), out.data_ptr(),
                           need_s ? s.data_ptr() : nullptr, kind == 1 ? mean.data_ptr<float>() : nullptr,
                           rstd.data_ptr<float>(), N, d, (float)eps, (float)p, (uint32_t)seed, (int)kind, is_bf16(x),
                           stream()),
             "norm_fwd");
  return {out, s, mean, rstd};
}

std::vector<Tensor> norm_bwd(const optional<Tensor>& dout_o, const optional<Tensor>& ds, const Tensor& s,
                             const Tensor& w, const optional<Tensor>& b, const optional<Tensor>& mean,
                             const Tensor& rstd, double p, int64_t seed, int64_t kind, bool want_stream,
                             const optional<Tensor>& dw_acc, const optional<Tensor>& db_acc, bool want_colsum,
                             bool partials_only) {
  check_gpu(s, "s");
  TORCH_CHECK(s.dim() == 2 && s.is_contiguous(), "s must be contiguous [N, d]");
  const int N = s.size(0), d = s.size(1);
  Tensor dout = dout_o.has_value() && dout_o->defined() ? dout_o->contiguous() : at::zeros_like(s);
  TORCH_CHECK(dout.sizes() == s.sizes() && dout.scalar_type() == s.scalar_type(), "dout mismatch");
  Tensor dse;
  if (ds.has_value() && ds->defined()) {
    dse = ds->contiguous();
    TORCH_CHECK(dse.sizes() == s.sizes() && dse.scalar_type() == s.scalar_type(), "ds mismatch");
  }
  TORCH_CHECK(rstd.numel() == N, "rstd mismatch");
  if (kind == 1) TORCH_CHECK(mean.has_value() && mean->numel() == N, "mean required for LayerNorm");
  auto dx = at::empty_like(s);
  Tensor dstream = want_stream ? at::empty_like(s) : Tensor();
  const int G = dllm_norm_bwd_grid(N > 0 ? N : 1);
  auto f32 = s.options().dtype(at::kFloat);
  auto dw_part = at::empty({G, d}, f32);
  const bool has_b = b.has_value() && b->defined();
  // dw_acc / db_acc: accumulate the parameter gradients in place (param dtype, contiguous, d elements)
  // partials_only: no reduction at all — dw / db come back as the fp32 per-block partials [G, d] (deferred windows)
  const bool acc = !partials_only && dw_acc.has_value() && dw_acc->defined();
  if (acc) {
    // the flat gradient buffer: param dtype or fp32 (FlatParams grad_dtype)
    TORCH_CHECK(dw_acc->numel() == d && dw_acc->is_contiguous() &&
                    (dw_acc->scalar_type() == s.scalar_type() || dw_acc->scalar_type() == at::kFloat),
                "dw_acc mismatch");
    TORCH_CHECK(!has_b || (db_acc.has_value() && db_acc->defined() && db_acc->numel() == d &&
                           db_acc->is_contiguous() && db_acc->scalar_type() == dw_acc->scalar_type()),
                "db_acc mismatch");
  }
  Tensor dw = (acc || partials_only) ? Tensor() : at::zeros({d}, f32);
  Tensor db_part = has_b ? at::empty({G, d}, f32) : Tensor();
  Tensor db = (has_b && !acc && !partials_only) ? at::zeros({d}, f32) : Tensor();
  // column sums of dx (the upstream linear layer's bias gradient), fp32 [d]
  Tensor dxs_part = want_colsum ? at::empty({G, d}, f32) : Tensor();
  // the dx column sums stay per-block partials: the consuming bias gradient reduces them (ops/gemm.py, one kernel)
  if (N > 0)
    check_rc(dllm_norm_bwd(dout.data_ptr(), dse.defined() ? dse.data_ptr() : nullptr, s.data_ptr(), w.data_ptr(),
                           kind == 1 ? mean->data_ptr<float>() : nullptr, rstd.data_ptr<float>(), dx.data_ptr(),
                           want_stream ? dstream.data_ptr() : nullptr, dw_part.data_ptr<float>(),
                           has_b ? db_part.data_ptr<float>() : nullptr, dw.defined() ? dw.data_ptr<float>() : nullptr,
                           db.defined() ? db.data_ptr<float>() : nullptr, acc ? dw_acc->data_ptr() : nullptr,
                           (acc && has_b) ? db_acc->data_ptr() : nullptr,
                           want_colsum ? dxs_part.data_ptr<float>() : nullptr,
                           nullptr, N, d, (float)p, (uint32_t)seed, (int)kind,
                           is_bf16(s), acc && dw_acc->scalar_type() == at::kFloat, stream()),
             "norm_bwd");
  if (partials_only) return {dx, dstream, dw_part, db_part, dxs_part};
  return {dx, dstream, dw, db, dxs_part};
}

// ------------------------------------------------------------------------------------------- activations
Tensor act_fwd(const Tensor& x, int64_t act, bool gated, double p, int64_t seed) {
  check_gpu(x, "x");
  TORCH_CHECK(x.dim() == 2 && x.is_contiguous(), "act: x must be contiguous [N, F]");
  const long N = x.size(0);
  const int F = gated ? x.size(1) / 2 : x.size(1);
  TORCH_CHECK(F % 4 == 0 && (!gated || x.size(1) == 2 * F), "act: F must be a multiple of 4");
  auto y = at::empty({N, F}, x.options());
  if (N > 0) check_rc(dllm_act_fwd(x.data_ptr(), y.data_ptr(), N, F, (int)act, gated, (float)p, (uint32_t)seed,
                                   is_bf16(x), stream()), "act_fwd");
  return y;
}

Tensor act_bwd(const Tensor& dy_, const Tensor& x, int64_t act, bool gated, double p, int64_t seed) {
  check_gpu(x, "x");
  Tensor dy = dy_.contiguous();
  const long N = x.size(0);
  const int F = gated ? x.size(1) / 2 : x.size(1);
  TORCH_CHECK(dy.dim() == 2 && dy.size(0) == N && dy.size(1) == F && dy.scalar_type() == x.scalar_type(),
              "act_bwd: dy shape mismatch");
  auto dx = at::empty_like(x);
  if (N > 0) check_rc(dllm_act_bwd(dy.data_ptr(), x.data_ptr(), dx.data_ptr(), N, F, (int)act, gated, (float)p,
                                   (uint32_t)seed, is_bf16(x), stream()), "act_bwd");
  return dx;
}

Tensor dropout_fwd(const Tensor& x, double p, int64_t seed) {
  check_gpu(x, "x");
  TORCH_CHECK(x.is_contiguous() && x.numel() % 4 == 0, "dropout: contiguous, numel % 4 == 0");
  auto y = at::empty_like(x);
  if (x.numel() > 0)
    check_rc(dllm_dropout(x.data_ptr(), y.data_ptr(), x.numel(), (float)p, (uint32_t)seed, is_bf16(x), stream()),
             "dropout");
  return y;
}

// ------------------------------------------------------------------------------------------- cross entropy
std::vector<Tensor> ce_fwd(const Tensor& logits, const Tensor& labels, const optional<Tensor>& bias, double eps,
                           int64_t ignore) {
  check_gpu(logits, "logits");
  TORCH_CHECK(logits.dim() == 2 && logits.is_contiguous(), "ce: logits must be contiguous [N, V]");
  TORCH_CHECK(labels.scalar_type() == at::kLong && labels.numel() == logits.size(0) && labels.is_contiguous(),
              "ce: labels must be int64 [N]");
  const long N = logits.size(0);
  const int V = logits.size(1);
  Tensor bf;
  if (bias.has_value() && bias->defined()) {
    bf = bias->to(at::kFloat).contiguous();
    TORCH_CHECK(bf.numel() == V, "ce: bias must have V entries");
  }
  auto f32 = logits.options().dtype(at::kFloat);
  auto loss = at::empty({N}, f32), lse = at::empty({N}, f32);
  if (N > 0)
    check_rc(dllm_ce_fwd(logits.data_ptr(), labels.data_ptr<int64_t>(), bf.defined() ? bf.data_ptr<float>() : nullptr,
                         loss.data_ptr<float>(), lse.data_ptr<float>(), N, V, (float)eps, ignore, is_bf16(logits),
                         stream()),
             "ce_fwd");
  return {loss, lse};
}

Tensor ce_bwd(const Tensor& scale, Tensor logits, const Tensor& labels, const Tensor& lse,
              const optional<Tensor>& bias, double eps, int64_t ignore, bool inplace) {
  check_gpu(logits, "logits");
  TORCH_CHECK(scale.scalar_type() == at::kFloat && scale.numel() >= 1 && scale.is_cuda(), "ce: scale");
  const long N = logits.size(0);
  const int V = logits.size(1);
  Tensor bf;
  if (bias.has_value() && bias->defined()) bf = bias->to(at::kFloat).contiguous();
  Tensor out = inplace ? logits : at::empty_like(logits);
  if (N > 0)
    check_rc(dllm_ce_bwd(scale.data_ptr<float>(), logits.data_ptr(), labels.data_ptr<int64_t>(),
                         lse.data_ptr<float>(), bf.defined() ? bf.data_ptr<float>() : nullptr, out.data_ptr(), N, V,
                         (float)eps, ignore, is_bf16(logits), stream()),
             "ce_bwd");
  return out;
}

// vocab-chunked LM head + CE (ops/lm_head.py): logits chunk [N, Vc] bf16 (row stride ld) holding vocab ids c0..c0+Vc-1
void ce_chunk_fwd(const Tensor& logits, const Tensor& labels, const optional<Tensor>& bias, Tensor& state, Tensor& loss,
                  Tensor& lse, int64_t c0, int64_t V, double eps, int64_t ignore, bool first, bool last, int64_t skip) {
  check_gpu(logits, "logits");
  TORCH_CHECK(logits.dim() == 2 && logits.scalar_type() == at::kBFloat16 && logits.stride(1) == 1 &&
                  logits.stride(0) % 4 == 0 && logits.size(1) % 4 == 0 && reinterpret_cast<uintptr_t>(logits.data_ptr()) % 8 == 0,
              "ce_chunk: logits must be bf16 [N, Vc] with Vc % 4 == 0 and 8-B aligned rows");
  const int64_t N = logits.size(0), Vc = logits.size(1);
  TORCH_CHECK(labels.scalar_type() == at::kLong && labels.numel() == N && labels.is_contiguous(), "ce_chunk: labels");
  TORCH_CHECK(state.scalar_type() == at::kFloat && state.numel() == 4 * N && state.is_contiguous(), "ce_chunk: state");
  TORCH_CHECK(loss.numel() == N && lse.numel() == N && loss.scalar_type() == at::kFloat && lse.scalar_type() == at::kFloat,
              "ce_chunk: loss / lse");
  TORCH_CHECK(c0 >= 0 && c0 + Vc <= V, "ce_chunk: chunk outside the vocabulary");
  const float* bp = nullptr;
  if (bias.has_value() && bias->defined()) {
    TORCH_CHECK(bias->scalar_type() == at::kFloat && bias->numel() == V && bias->is_contiguous(), "ce_chunk: bias fp32 [V]");
    bp = bias->data_ptr<float>();
  }
  if (N == 0) return;
  check_rc(dllm_ce_chunk_fwd(logits.data_ptr(), logits.stride(0), labels.data_ptr<int64_t>(), bp, state.data_ptr<float>(),
                             loss.data_ptr<float>(), lse.data_ptr<float>(), N, (int)Vc, (int)c0, (int)V, (float)eps,
                             ignore, first, last, (int)skip, stream()),
           "ce_chunk_fwd");
}

void ce_chunk_bwd(const Tensor& scale, Tensor& logits, const Tensor& labels, const Tensor& lse,
                  const optional<Tensor>& bias, int64_t c0, int64_t V, double eps, int64_t ignore, int64_t skip) {
  check_gpu(logits, "logits");
  TORCH_CHECK(logits.dim() == 2 && logits.scalar_type() == at::kBFloat16 && logits.stride(1) == 1 &&
                  logits.stride(0) % 4 == 0 && logits.size(1) % 4 == 0, "ce_chunk_bwd: logits");
  const int64_t N = logits.size(0), Vc = logits.size(1);
  TORCH_CHECK(scale.scalar_type() == at::kFloat && scale.is_cuda() && labels.numel() == N && lse.numel() == N,
              "ce_chunk_bwd: args");
  const float* bp = (bias.has_value() && bias->defined()) ? bias->data_ptr<float>() : nullptr;
  if (N == 0) return;
  check_rc(dllm_ce_chunk_bwd(scale.data_ptr<float>(), logits.data_ptr(), logits.stride(0), labels.data_ptr<int64_t>(),
                             lse.data_ptr<float>(), bp, N, (int)Vc, (int)c0, (int)V, (float)eps, ignore, (int)skip,
                             stream()),
           "ce_chunk_bwd");
}

// ------------------------------------------------------------------------------------------- optimizer
Tensor sq_norm(const Tensor& g) {
  check_gpu(g, "g");
  TORCH_CHECK(g.is_contiguous() && g.numel() % 4 == 0, "sq_norm: contiguous, numel % 4 == 0");
  check_aligned(g, 16, "g");
  auto f32 = g.options().dtype(at::kFloat);
  auto part = at::empty({1024}, f32);
  auto out = at::empty({}, f32);
  check_rc(dllm_sq_norm(g.data_ptr(), g.numel(), part.data_ptr<float>(), out.data_ptr<float>(), is_bf16(g),
                        stream()),
           "sq_norm");
  return out;
}

void adamw_step(Tensor param, const optional<Tensor>& master, const Tensor& grad, Tensor m, Tensor v,
                const optional<Tensor>& wd_mask, const Tensor& coef, double lr, double b1, double b2, double eps,
                double wd, double bc1, double bc2, const optional<Tensor>& hyper) {
  check_gpu(param, "param");
  const long n = param.numel();
  TORCH_CHECK(n % 4 == 0 && param.is_contiguous() && grad.numel() == n && m.numel() == n && v.numel() == n,
              "adamw: flat buffers must match, numel % 4 == 0");
  TORCH_CHECK(grad.scalar_type() == param.scalar_type() || grad.scalar_type() == at::kFloat,
              "adamw: grad dtype must be the param dtype or fp32");
  check_aligned(grad, 16, "adamw grad");
  TORCH_CHECK(m.scalar_type() == at::kFloat && v.scalar_type() == at::kFloat, "adamw: moments fp32");
  if (master.has_value() && master->defined())
    TORCH_CHECK(master->numel() == n && master->scalar_type() == at::kFloat, "adamw: master fp32 [n]");
  if (wd_mask.has_value() && wd_mask->defined())
    TORCH_CHECK(wd_mask->numel() == n && wd_mask->scalar_type() == at::kByte, "adamw: wd_mask u8 [n]");
  TORCH_CHECK(coef.scalar_type() == at::kFloat && coef.is_cuda(), "adamw: coef fp32 device scalar");
  const bool has_hyper = hyper.has_value() && hyper->defined();
  if (has_hyper)
    TORCH_CHECK(hyper->is_cuda() && hyper->scalar_type() == at::kFloat && hyper->numel() >= 3 && hyper->is_contiguous(),
                "adamw: hyper must be a contiguous fp32 device tensor [lr, lr / bc1, 1 / sqrt(bc2)]");
  for (auto* t : {&param, &m, &v}) check_aligned(*t, 16, "adamw buffer");
  check_rc(dllm_adamw(param.data_ptr(),
                      master.has_value() && master->defined() ? master->data_ptr<float>() : nullptr, grad.data_ptr(),
                      m.data_ptr<float>(), v.data_ptr<float>(),
                      wd_mask.has_value() && wd_mask->defined() ? wd_mask->data_ptr<uint8_t>() : nullptr,
                      coef.data_ptr<float>(), n, (float)lr, (float)b1, (float)b2, (float)eps, (float)wd, (float)bc1,
                      (float)bc2, is_bf16(param), grad.scalar_type() == at::kFloat,
                      has_hyper ? hyper->data_ptr<float>() : nullptr, stream()),
           "adamw");
}

// ------------------------------------------------------------------------------------------- attention
void check_bshd(const Tensor& t, const char* n, int64_t B, int64_t S, int64_t H) {
  check_gpu(t, n);
  TORCH_CHECK(t.scalar_type() == at::kBFloat16, n, ": attention kernels take bf16");
  TORCH_CHECK(t.dim() == 4 && t.size(0) == B && t.size(1) == S && t.size(2) == H && t.size(3) == 64, n,
              ": expected [B, S, H, 64], got ", t.sizes());
  TORCH_CHECK(t.stride(3) == 1, n, ": head dim must be contiguous");
  TORCH_CHECK(t.stride(0) % 8 == 0 && t.stride(1) % 8 == 0 && t.stride(2) % 8 == 0, n,
              ": strides must be multiples of 8 elements (16-B vector loads)");
  check_aligned(t, 16, n);
}

void fill_qkv(AttnParams& P, const Tensor& q, const Tensor& k, const Tensor& v, const optional<Tensor>& kpm,
              const optional<Tensor>& lut, double scale, bool causal, double p, int64_t seed) {
  const int64_t B = q.size(0), Sq = q.size(1), H = q.size(2), Sk = k.size(1);
  check_bshd(q, "q", B, Sq, H);
  check_bshd(k, "k", B, Sk, H);
  check_bshd(v, "v", B, Sk, H);
  TORCH_CHECK(Sq > 0 && Sk > 0, "empty attention");
  TORCH_CHECK(Sk <= 16384 && Sq <= 16384, "attention: sequence length > 16384 unsupported");
  TORCH_CHECK(B * H * Sq * Sk < (int64_t)1 << 40, "attention too large");
  P.q = reinterpret_cast<const uint16_t*>(q.data_ptr());
  P.k = reinterpret_cast<const uint16_t*>(k.data_ptr());
  P.v = reinterpret_cast<const uint16_t*>(v.data_ptr());
  P.q_sb = q.stride(0); P.q_ss = q.stride(1); P.q_sh = q.stride(2);
  P.k_sb = k.stride(0); P.k_ss = k.stride(1); P.k_sh = k.stride(2);
  P.v_sb = v.stride(0); P.v_ss = v.stride(1); P.v_sh = v.stride(2);
  P.B = B; P.H = H; P.Sq = Sq; P.Sk = Sk;
  P.scale = (float)scale;
  P.causal = causal ? 1 : 0;
  P.causal_off = Sk - Sq;
  P.p_drop = (float)p;
  P.seed = (uint32_t)seed;
  P.kpm = nullptr;
  P.lut = nullptr;
  if (kpm.has_value() && kpm->defined()) {
    TORCH_CHECK(kpm->scalar_type() == at::kByte && kpm->is_contiguous() && kpm->dim() == 2 && kpm->size(0) == B &&
                    kpm->size(1) == Sk && kpm->is_cuda(),
                "key_padding_mask must be uint8 [B, Sk] contiguous on GPU");
    P.kpm = kpm->data_ptr<uint8_t>();
  }
  if (lut.has_value() && lut->defined()) {
    TORCH_CHECK(lut->scalar_type() == at::kFloat && lut->is_contiguous() && lut->dim() == 2 && lut->size(0) == H &&
                    lut->size(1) == Sq + Sk - 1 && lut->is_cuda(),
                "bias_lut must be fp32 [H, Sq + Sk - 1] contiguous on GPU");
    P.lut = lut->data_ptr<float>();
  }
  P.sat_lo = INT_MIN / 2;  // saturated-bias ranges off unless the caller declares them (set_sat)
  P.sat_hi = INT_MAX / 2;
}

// sat_lo / sat_hi: LUT index ranges [0, sat_lo] and [sat_hi, L) of constant bias whose gradient is consumed per
// bucket only (ops/attention.py relative_bias_lut); negative = off
void set_sat(AttnParams& P, int64_t sat_lo, int64_t sat_hi) {
  if (P.lut == nullptr || sat_lo < 0 || sat_hi < 0) return;
  const int64_t L = (int64_t)P.Sq + P.Sk - 1;
  TORCH_CHECK(sat_lo < L && sat_hi > sat_lo && sat_hi <= L, "attention: bad saturated-bias bounds");
  P.sat_lo = (int)sat_lo;
  P.sat_hi = (int)sat_hi;
}

int64_t dmask_numel(const AttnParams& P) {
  const int64_t sq_pad = (P.Sq + 127) / 128 * 128, nkt = (P.Sk + 63) / 64;
  return (int64_t)P.B * P.H * nkt * 2 * sq_pad;
}

std::vector<Tensor> attn_fwd(const Tensor& q, const Tensor& k, const Tensor& v, const optional<Tensor>& kpm,
                             const optional<Tensor>& lut, double scale, bool causal, double p, int64_t seed,
                             const optional<Tensor>& dmask_in, int64_t sat_lo, int64_t sat_hi) {
  AttnParams P{};
  fill_qkv(P, q, k, v, kpm, lut, scale, causal, p, seed);
  set_sat(P, sat_lo, sat_hi);
  auto o = at::empty({P.B, P.Sq, P.H, 64}, q.options());
  auto lse = at::empty({P.B, P.H, P.Sq}, q.options().dtype(at::kFloat));
  P.o_out = reinterpret_cast<uint16_t*>(o.data_ptr());
  P.o_sb = o.stride(0); P.o_ss = o.stride(1); P.o_sh = o.stride(2);
  P.lse = lse.data_ptr<float>();
  // dropout keep bits: [B*H][ceil(Sk/64)][2][ceil(Sq/128)*128] uint32, written here, read by attn_bwd
  Tensor dmask;
  if (p > 0.0) {
    if (dmask_in.has_value() && dmask_in->defined()) {  // planes from attn_dropout_mask (same seed and shapes)
      TORCH_CHECK(dmask_in->scalar_type() == at::kInt && dmask_in->is_contiguous() && dmask_in->is_cuda() &&
                      dmask_in->numel() == dmask_numel(P),
                  "attn_fwd: dmask_in must come from attn_dropout_mask for the same shapes");
      dmask = *dmask_in;
      P.dmask_ready = 1;
    } else {
      dmask = at::empty({dmask_numel(P)}, q.options().dtype(at::kInt));
    }
    P.dmask = reinterpret_cast<uint32_t*>(dmask.data_ptr());
  }
  check_rc(dllm_attn_fwd(&P, stream()), "attn_fwd");
  return {o, lse, dmask};
}

// ------------------------------------------------------------------------------------------- fp32 attention
// csrc/attn_f32.hip: the same op at the reference's precision (fp32 in, fp32 out, f32 MFMA).
void check_bshd_f32(const Tensor& t, const char* n, int64_t B, int64_t S, int64_t H) {
  check_gpu(t, n);
  TORCH_CHECK(t.scalar_type() == at::kFloat, n, ": fp32 attention kernels take fp32");
  TORCH_CHECK(t.dim() == 4 && t.size(0) == B && t.size(1) == S && t.size(2) == H && t.size(3) == 64, n,
              ": expected [B, S, H, 64], got ", t.sizes());
  TORCH_CHECK(t.stride(3) == 1, n, ": head dim must be contiguous");
  TORCH_CHECK(t.stride(0) % 4 == 0 && t.stride(1) % 4 == 0 && t.stride(2) % 4 == 0, n,
              ": strides must be multiples of 4 elements (16-B vector loads)");
  check_aligned(t, 16, n);
}

void fill_f32(AttnF32Params& P, const Tensor& q, const Tensor& k, const Tensor& v, const optional<Tensor>& kpm,
              const optional<Tensor>& lut, double scale, bool causal, double p, int64_t seed) {
  const int64_t B = q.size(0), Sq = q.size(1), H = q.size(2), Sk = k.size(1);
  check_bshd_f32(q, "q", B, Sq, H);
  check_bshd_f32(k, "k", B, Sk, H);
  check_bshd_f32(v, "v", B, Sk, H);
  TORCH_CHECK(Sq > 0 && Sk > 0, "empty attention");
  TORCH_CHECK(B * H <= 65535, "attention: B * H > 65535 unsupported (grid y)");
  TORCH_CHECK(B * H * Sq < (int64_t)1 << 31 && (Sq + Sk) < (1 << 30), "attention too large");
  TORCH_CHECK(p >= 0.0 && p < 1.0, "dropout p must be in [0, 1)");
  P.q = q.data_ptr<float>();
  P.k = k.data_ptr<float>();
  P.v = v.data_ptr<float>();
  P.q_sb = q.stride(0); P.q_ss = q.stride(1); P.q_sh = q.stride(2);
  P.k_sb = k.stride(0); P.k_ss = k.stride(1); P.k_sh = k.stride(2);
  P.v_sb = v.stride(0); P.v_ss = v.stride(1); P.v_sh = v.stride(2);
  P.B = B; P.H = H; P.Sq = Sq; P.Sk = Sk;
  P.scale = (float)scale;
  P.causal = causal ? 1 : 0;
  P.causal_off = Sk - Sq;
  P.p_drop = (float)p;
  P.seed = (uint32_t)seed;
  P.thr = p > 0.0 ? (uint32_t)std::min(65535.0, p * 65536.0) : 0u;  // ops/rng.py threshold16
  if (kpm.has_value() && kpm->defined()) {
    TORCH_CHECK(kpm->scalar_type() == at::kByte && kpm->is_contiguous() && kpm->dim() == 2 && kpm->size(0) == B &&
                    kpm->size(1) == Sk && kpm->is_cuda(),
                "key_padding_mask must be uint8 [B, Sk] contiguous on GPU");
    P.kpm = kpm->data_ptr<uint8_t>();
  }
  if (lut.has_value() && lut->defined()) {
    TORCH_CHECK(lut->scalar_type() == at::kFloat && lut->is_contiguous() && lut->dim() == 2 && lut->size(0) == H &&
                    lut->size(1) == Sq + Sk - 1 && lut->is_cuda(),
                "bias_lut must be fp32 [H, Sq + Sk - 1] contiguous on GPU");
    P.lut = lut->data_ptr<float>();
  }
}

std::vector<Tensor> attn_f32_fwd(const Tensor& q, const Tensor& k, const Tensor& v, const optional<Tensor>& kpm,
                                 const optional<Tensor>& lut, double scale, bool causal, double p, int64_t seed) {
  AttnF32Params P{};
  fill_f32(P, q, k, v, kpm, lut, scale, causal, p, seed);
  auto o = at::empty({P.B, P.Sq, P.H, 64}, q.options());
  auto lse = at::empty({P.B, P.H, P.Sq}, q.options());
  P.o_out = o.data_ptr<float>();
  P.o_sb = o.stride(0); P.o_ss = o.stride(1); P.o_sh = o.stride(2);
  P.lse = lse.data_ptr<float>();
  check_rc(dllm_attn_f32_fwd(&P, stream()), "attn_f32_fwd");
  return {o, lse};
}

std::vector<Tensor> attn_f32_bwd(const Tensor& dout, const Tensor& q, const Tensor& k, const Tensor& v,
                                 const Tensor& o, const Tensor& lse, const optional<Tensor>& kpm,
                                 const optional<Tensor>& lut, double scale, bool causal, double p, int64_t seed,
                                 bool need_dlut, const optional<Tensor>& dq_out, const optional<Tensor>& dk_out,
                                 const optional<Tensor>& dv_out) {
  AttnF32Params P{};
  fill_f32(P, q, k, v, kpm, lut, scale, causal, p, seed);
  check_bshd_f32(o, "o", P.B, P.Sq, P.H);
  check_bshd_f32(dout, "dout", P.B, P.Sq, P.H);
  TORCH_CHECK(lse.scalar_type() == at::kFloat && lse.numel() == (int64_t)P.B * P.H * P.Sq && lse.is_contiguous() &&
                  lse.is_cuda(),
              "lse mismatch");
  auto pick = [&](const optional<Tensor>& t, int64_t S, const char* n) {
    if (t.has_value() && t->defined()) {
      check_bshd_f32(*t, n, P.B, S, P.H);
      return *t;
    }
    return at::empty({P.B, S, P.H, 64}, q.options());
  };
  Tensor dq = pick(dq_out, P.Sq, "dq_out");
  Tensor dk = pick(dk_out, P.Sk, "dk_out");
  Tensor dv = pick(dv_out, P.Sk, "dv_out");
  auto delta = at::empty({P.B, P.H, P.Sq}, q.options());
  Tensor dlut;
  if (need_dlut && P.lut) {
    dlut = at::zeros({P.H, P.Sq + P.Sk - 1}, q.options());
    P.dlut = dlut.data_ptr<float>();
  }
  P.o = o.data_ptr<float>();
  P.o_sb = o.stride(0); P.o_ss = o.stride(1); P.o_sh = o.stride(2);
  P.dout = dout.data_ptr<float>();
  P.do_sb = dout.stride(0); P.do_ss = dout.stride(1); P.do_sh = dout.stride(2);
  P.lse = lse.data_ptr<float>();
  P.delta = delta.data_ptr<float>();
  P.dq = dq.data_ptr<float>();
  P.dq_sb = dq.stride(0); P.dq_ss = dq.stride(1); P.dq_sh = dq.stride(2);
  P.dk = dk.data_ptr<float>();
  P.dk_sb = dk.stride(0); P.dk_ss = dk.stride(1); P.dk_sh = dk.stride(2);
  P.dv = dv.data_ptr<float>();
  P.dv_sb = dv.stride(0); P.dv_ss = dv.stride(1); P.dv_sh = dv.stride(2);
  check_rc(dllm_attn_f32_bwd(&P, stream()), "attn_f32_bwd");
  return {dq, dk, dv, dlut};
}

// dropout keep-bit planes of an attention call (generated ahead, e.g. on a side stream)
Tensor attn_dropout_mask(int64_t B, int64_t H, int64_t Sq, int64_t Sk, double p, int64_t seed, const Tensor& like) {
  TORCH_CHECK(p > 0.0 && B > 0 && H > 0 && Sq > 0 && Sk > 0 && like.is_cuda(), "attn_dropout_mask: bad arguments");
  AttnParams P{};
  P.B = B; P.H = H; P.Sq = Sq; P.Sk = Sk;
  P.p_drop = (float)p;
  P.seed = (uint32_t)seed;
  auto dmask = at::empty({dmask_numel(P)}, like.options().dtype(at::kInt));
  P.dmask = reinterpret_cast<uint32_t*>(dmask.data_ptr());
  check_rc(dllm_attn_dropout_mask(&P, stream()), "attn_dropout_mask");
  return dmask;
}

std::vector<Tensor> attn_bwd(const Tensor& dout, const Tensor& q, const Tensor& k, const Tensor& v, const Tensor& o,
                             const Tensor& lse, const optional<Tensor>& kpm, const optional<Tensor>& lut,
                             double scale, bool causal, double p, int64_t seed, bool need_dlut,
                             const optional<Tensor>& dq_out, const optional<Tensor>& dk_out,
                             const optional<Tensor>& dv_out, const optional<Tensor>& dmask, int64_t sat_lo,
                             int64_t sat_hi, const optional<Tensor>& csq, const optional<Tensor>& csk,
                             const optional<Tensor>& csv) {
  AttnParams P{};
  fill_qkv(P, q, k, v, kpm, lut, scale, causal, p, seed);
  set_sat(P, sat_lo, sat_hi);
  if (p > 0.0) {
    TORCH_CHECK(dmask.has_value() && dmask->defined() && dmask->scalar_type() == at::kInt && dmask->is_contiguous() &&
                    dmask->numel() == dmask_numel(P) && dmask->is_cuda(),
                "attn_bwd: dropout needs the bit planes attn_fwd returned");
    P.dmask = reinterpret_cast<uint32_t*>(dmask->data_ptr());
  }
  check_bshd(o, "o", P.B, P.Sq, P.H);
  check_bshd(dout, "dout", P.B, P.Sq, P.H);
  TORCH_CHECK(lse.scalar_type() == at::kFloat && lse.numel() == (int64_t)P.B * P.H * P.Sq && lse.is_contiguous(),
              "lse mismatch");
  auto f32 = q.options().dtype(at::kFloat);
  // outputs may be caller-provided strided views (e.g. slices of one packed d(qkv) buffer)
  auto pick = [&](const optional<Tensor>& t, int64_t S, const char* n) {
    if (t.has_value() && t->defined()) {
      check_bshd(*t, n, P.B, S, P.H);
      return *t;
    }
    return at::empty({P.B, S, P.H, 64}, q.options());
  };
  Tensor dq = pick(dq_out, P.Sq, "dq_out");
  Tensor dk = pick(dk_out, P.Sk, "dk_out");
  Tensor dv = pick(dv_out, P.Sk, "dv_out");
  auto delta = at::empty({P.B, P.H, P.Sq}, f32);
  // per-row terms the dQ kernel hands to the dK/dV kernel ([B*H][sq_pad/64][4][64])
  Tensor rowrec = at::empty({(int64_t)P.B * P.H * ((P.Sq + 127) / 128 * 128) * 4}, f32);
  P.rowrec = rowrec.data_ptr<float>();
  Tensor dlut;
  if (P.lut != nullptr) dlut = at::zeros({P.H, P.Sq + P.Sk - 1}, f32);
  P.o = reinterpret_cast<const uint16_t*>(o.data_ptr());
  P.o_sb = o.stride(0); P.o_ss = o.stride(1); P.o_sh = o.stride(2);
  P.dout = reinterpret_cast<const uint16_t*>(dout.data_ptr());
  P.do_sb = dout.stride(0); P.do_ss = dout.stride(1); P.do_sh = dout.stride(2);
  P.lse = lse.data_ptr<float>();
  P.delta = delta.data_ptr<float>();
  P.dq = reinterpret_cast<uint16_t*>(dq.data_ptr());
  P.dq_sb = dq.stride(0); P.dq_ss = dq.stride(1); P.dq_sh = dq.stride(2);
  P.dk = reinterpret_cast<uint16_t*>(dk.data_ptr());
  P.dk_sb = dk.stride(0); P.dk_ss = dk.stride(1); P.dk_sh = dk.stride(2);
  P.dv = reinterpret_cast<uint16_t*>(dv.data_ptr());
  P.dv_sb = dv.stride(0); P.dv_ss = dv.stride(1); P.dv_sh = dv.stride(2);
  P.dlut = dlut.defined() ? dlut.data_ptr<float>() : nullptr;
  // optional per-block column sums ([B * ceil(S / 128)][H * 64] fp32 views, unit column stride; dK / dV share a row
  // stride): the bias gradients of the q / k / v projections, summed over blocks by the caller
  auto cs = [&](const optional<Tensor>& t, int64_t S, const char* n, long* ld) -> float* {
    if (!t.has_value() || !t->defined()) return nullptr;
    TORCH_CHECK(t->is_cuda() && t->scalar_type() == at::kFloat && t->dim() == 2 && t->size(0) == P.B * ((S + 127) / 128) &&
                    t->size(1) == (int64_t)P.H * 64 && t->stride(1) == 1 && t->stride(0) >= t->size(1),
                n, ": expected fp32 [B * ceil(S / 128), H * 64] with unit column stride");
    *ld = t->stride(0);
    return t->data_ptr<float>();
  };
  long ldk = 0, ldv = 0;
  P.csq = cs(csq, P.Sq, "csq", &P.csq_ld);
  P.csk = cs(csk, P.Sk, "csk", &ldk);
  P.csv = cs(csv, P.Sk, "csv", &ldv);
  TORCH_CHECK((P.csk == nullptr) == (P.csv == nullptr) && ldk == ldv, "csk / csv: both or neither, one row stride");
  P.cskv_ld = ldk;
  check_rc(dllm_attn_bwd(&P, stream()), "attn_bwd");
  return {dq, dk, dv, need_dlut ? dlut : Tensor()};
}

}  // namespace

// ------------------------------------------------------------------------------------------- GEMM
// c[M][N] (+)= a^T b with a = [K][M], b = [K][N] (token-major), bf16; returns the split count used.
bool gemm_wgrad_supported(const Tensor& a, const Tensor& b, const Tensor& c) {
  auto ok2 = [](const Tensor& t) {
    return t.is_cuda() && t.dim() == 2 && t.scalar_type() == at::kBFloat16 && t.stride(1) == 1 && t.stride(0) % 8 == 0 &&
           reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0;
  };
  const bool c_ok = c.is_cuda() && c.dim() == 2 && c.stride(1) == 1 && c.stride(0) % 8 == 0 &&
                    (c.scalar_type() == at::kBFloat16 || c.scalar_type() == at::kFloat) &&
                    reinterpret_cast<uintptr_t>(c.data_ptr()) % 16 == 0;
  if (!ok2(a) || !ok2(b) || !c_ok) return false;
  const int64_t K = a.size(0), M = a.size(1), N = b.size(1);
  return b.size(0) == K && c.size(0) == M && c.size(1) == N && K % 64 == 0 && K > 0 && M % 8 == 0 && M >= 8 &&
         N % 256 == 0 &&
         K < (1LL << 31) && M * N < (1LL << 31);
}

// K split count of the weight-gradient GEMM.  One 128-KB-LDS workgroup per CU, all workgroups equally long, so the
// kernel runs ceil(T s / CUs) rounds of 1/s of a tile's K each: minimise that (the tail of the last round) plus the
// split-K reduce pass (s fp32 slabs of the output; relative cost ~ 1.7 T s / K at ~1.1 PF/s and ~5 TB/s), fewest
// splits on ties, at least 4 k-stages of 64 per split.  378 tiles (t5 LM head): 2 (3 full rounds instead of 1.48);
// 216 (t5 cross-attention K/V of 12 layers): 13 (11 rounds, 99 % full, instead of one at 84 %);
// 9 / 36 (768 x 768 / 768 x 3072 at 512K tokens): 28 / 7, one round; 27 (QKV): 28, three rounds.
int wgrad_splits(int T, int K) {
  static const int cus = [] {
    const int n = at::cuda::getCurrentDeviceProperties()->multiProcessorCount;
    return n > 0 ? n : 256;
  }();
  const int smax = std::max(1, std::min(K / 256, 64));
  int best = 1;
  double bestc = 1e30;
  for (int s = 1; s <= smax; ++s) {
    const double rounds = (double)((T * s + cus - 1) / cus);
    const double c = rounds / s + (s > 1 ? 1.7 * T * s / K : 0.0);
    if (c < bestc * (1.0 - 1e-6)) {
      bestc = c;
      best = s;
    }
  }
  return best;
}

constexpr int64_t kWgradW4 = 12;  // the only gemm_wgrad variant: csrc/gemm_w4.hip's weight-gradient mode

int64_t gemm_wgrad(const Tensor& a, const Tensor& b, Tensor& c, bool beta, int64_t variant, int64_t splits_req) {
  TORCH_CHECK(gemm_wgrad_supported(a, b, c),
              "gemm_wgrad: need bf16 GPU [K,M] x [K,N] -> bf16/fp32 [M,N], unit inner stride, 16-B aligned rows, K % 64 == 0, "
              "M % 8 == 0, N a multiple of 256");
  TORCH_CHECK(a.device() == b.device() && a.device() == c.device(), "gemm_wgrad: device mismatch");
  TORCH_CHECK(variant < 0 || variant == kWgradW4, "gemm_wgrad: variant must be -1 (the w4 weight-gradient mode)");
  const int K = a.size(0), M = a.size(1), N = b.size(1);
  GemmWgradParams P{};
  P.A = reinterpret_cast<const uint16_t*>(a.data_ptr());
  P.B = reinterpret_cast<const uint16_t*>(b.data_ptr());
  P.C = c.data_ptr();
  P.c_f32 = c.scalar_type() == at::kFloat ? 1 : 0;
  P.lda = a.stride(0);
  P.ldb = b.stride(0);
  P.ldc = c.stride(0);
  P.M = M;
  P.N = N;
  P.K = K;
  P.tn = N / 256;
  P.ntiles = ((M + 255) / 256) * (N / 256);  // ragged last M tile (vocab-sized LM-head gradients)
  P.beta = beta ? 1 : 0;
  int splits = splits_req > 0 ? (int)splits_req : wgrad_splits(P.ntiles, K);
  splits = std::max(1, std::min(splits, K / 256));
  int kchunk = ((K + splits - 1) / splits + 63) / 64 * 64;
  // the w4 kernel addresses a split's k-rows through one 32-bit buffer-descriptor range: more splits when a wide
  // operand (e.g. the decoder's stacked cross-attention K/V gradient, 24576 columns) would overflow it
  const long ld = std::max(P.lda, P.ldb), wd = std::max(M, N);
  while (kchunk > 64 && ((long)(kchunk - 1) * ld + wd) * 2 >= 0xFFFFFFFFL) {
    ++splits;
    kchunk = ((K + splits - 1) / splits + 63) / 64 * 64;
  }
  TORCH_CHECK(((long)(kchunk - 1) * ld + wd) * 2 < 0xFFFFFFFFL, "gemm_wgrad: operand rows too long for 64-row splits");
  splits = (K + kchunk - 1) / kchunk;
  P.kchunk = kchunk;
  P.splits = splits;
  Tensor ws;
  if (splits > 1) {
    ws = at::empty({(int64_t)splits * M * N}, a.options().dtype(at::kFloat));
    P.ws = ws.data_ptr<float>();
  }
  {
    // csrc/gemm_w4.hip weight-gradient mode: one wave per SIMD, both operands k-major, fp32 split slabs
    GemmW4Params Q{};
    Q.A = P.A;
    Q.B = P.B;
    Q.lda = P.lda;
    Q.ldb = P.ldb;
    Q.ldc = P.ldc;
    Q.M = M;
    Q.N = N;
    Q.K = K;
    Q.tm = (M + 255) / 256;
    Q.tn = N / 256;
    Q.grp = 8;
    Q.ws = P.ws;
    Q.Cw = P.C;
    Q.splits = splits;
    Q.kchunk = kchunk;
    Q.c_f32 = P.c_f32;
    Q.beta = P.beta;
    check_rc(dllm_gemm_w4(&Q, 1, 0, 10, stream()), "gemm_wgrad (w4)");
    if (splits > 1) check_rc(dllm_wgrad_reduce(&P, stream()), "gemm_wgrad (w4) split-K reduce");
  }
  return splits;
}

// c[M][N] (+)= sum_i a_i^T b_i over the deferred micro-batches of a gradient-accumulation window (ops/gemm.py
// WgradDefer): equal-shaped token-major segments a_i = [rows][M], b_i = [rows][N] (up to W4_MAX_SEGS), read in place
// by the w4 weight-gradient mode — each segment cut into seg_chunks splits, split-K slabs as gemm_wgrad.  Returns the
// split count.
int64_t gemm_wgrad_segs(const std::vector<Tensor>& as, const std::vector<Tensor>& bs, Tensor& c, bool beta) {
  const int nseg = (int)as.size();
  TORCH_CHECK(nseg >= 1 && nseg <= W4_MAX_SEGS && (int)bs.size() == nseg, "gemm_wgrad_segs: 1..", W4_MAX_SEGS,
              " (a, b) segment pairs");
  for (int i = 0; i < nseg; ++i) {
    TORCH_CHECK(gemm_wgrad_supported(as[i], bs[i], c), "gemm_wgrad_segs: segment ", i, " unsupported");
    TORCH_CHECK(as[i].sizes() == as[0].sizes() && bs[i].sizes() == bs[0].sizes() &&
                    as[i].stride(0) == as[0].stride(0) && bs[i].stride(0) == bs[0].stride(0) &&
                    as[i].device() == c.device() && bs[i].device() == c.device(),
                "gemm_wgrad_segs: segments must share shapes, leading dimensions and device");
  }
  const int rows = as[0].size(0), M = as[0].size(1), N = bs[0].size(1);
  GemmW4Params Q{};
  Q.lda = as[0].stride(0);
  Q.ldb = bs[0].stride(0);
  Q.ldc = c.stride(0);
  Q.M = M;
  Q.N = N;
  Q.K = rows * nseg;
  Q.tm = (M + 255) / 256;
  Q.tn = N / 256;
  Q.grp = 8;
  for (int i = 0; i < nseg; ++i) {
    Q.segA[i] = reinterpret_cast<const uint16_t*>(as[i].data_ptr());
    Q.segB[i] = reinterpret_cast<const uint16_t*>(bs[i].data_ptr());
  }
  // the split count gemm_wgrad would pick for the window's whole K, spread over the segments
  const int want = wgrad_splits(Q.tm * Q.tn, Q.K);
  int chunks = std::max(1, std::min((want + nseg / 2) / nseg, rows / 64));
  int kchunk = ((rows + chunks - 1) / chunks + 63) / 64 * 64;
  const long ld = std::max(Q.lda, Q.ldb), wd = std::max(M, N);
  while (kchunk > 64 && ((long)(kchunk - 1) * ld + wd) * 2 >= 0xFFFFFFFFL) kchunk -= 64;
  TORCH_CHECK(((long)(kchunk - 1) * ld + wd) * 2 < 0xFFFFFFFFL, "gemm_wgrad_segs: leading dimension too large");
  chunks = (rows + kchunk - 1) / kchunk;
  Q.nseg = nseg;
  Q.seg_rows = rows;
  Q.seg_chunks = chunks;
  Q.kchunk = kchunk;
  Q.splits = nseg * chunks;
  Q.c_f32 = c.scalar_type() == at::kFloat ? 1 : 0;
  Q.beta = beta ? 1 : 0;
  Q.Cw = c.data_ptr();
  Tensor ws;
  if (Q.splits > 1) {
    ws = at::empty({(int64_t)Q.splits * M * N}, as[0].options().dtype(at::kFloat));
    Q.ws = ws.data_ptr<float>();
  }
  check_rc(dllm_gemm_w4(&Q, 1, 0, 10, stream()), "gemm_wgrad_segs (w4)");
  if (Q.splits > 1) {
    GemmWgradParams P{};
    P.ws = Q.ws;
    P.C = c.data_ptr();
    P.ldc = Q.ldc;
    P.M = M;
    P.N = N;
    P.splits = Q.splits;
    P.beta = Q.beta;
    P.c_f32 = Q.c_f32;
    check_rc(dllm_wgrad_reduce(&P, stream()), "gemm_wgrad_segs split-K reduce");
  }
  return Q.splits;
}

// c[M][N] = epi(a[M][K] . b) with b = [N][K] (nn.Linear weight, b_kmajor = false) or [K][N] (b_kmajor = true).
// epi (csrc/gemm_fused.hip): 0 none, 1 relu, 2 gelu-erf, 3 d-relu, 4 d-gelu-erf, 5 gelu-tanh, 6 d-gelu-tanh.
// Forward activations apply dropout(p, seed) on the output element index m * N + n (ops/rng.py); the GELU
// forwards also write G = dropout'(act'(u)) to aux_out; the backward epilogues read aux (saved activation for
// d-relu, whose dropout backward they apply; G for d-gelu, which they multiply in).
int64_t gemm_fused_variant(int64_t K) {
  // ping-pong kernel (16x16x32 MFMA, BK = 64, two wave rows one barrier apart), persistent for store-only epilogues:
  // fastest on every T5 / BART shape measured (profiles/r1_gemm_*_bench*.jsonl, r1_gemm_experiments.md);
  // K % 64 != 0: BK = 32 x 4 stages
  return K % 64 == 0 ? 9 : 1;
}

bool gemm_fused_supported(const Tensor& a, const Tensor& b, bool b_kmajor) {
  auto ok2 = [](const Tensor& t) {
    return t.is_cuda() && t.dim() == 2 && t.scalar_type() == at::kBFloat16 && t.stride(1) == 1 && t.stride(0) % 8 == 0 &&
           reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0;
  };
  if (!ok2(a) || !ok2(b)) return false;
  const int64_t M = a.size(0), K = a.size(1);
  const int64_t N = b_kmajor ? b.size(1) : b.size(0);
  const int64_t Kb = b_kmajor ? b.size(0) : b.size(1);
  return Kb == K && M % 256 == 0 && N % 256 == 0 && K % 64 == 0 && K > 0 && M > 0 && M * N < (1LL << 32) &&
         K < (1LL << 31);
}

Tensor gemm_fused(const Tensor& a, const Tensor& b, bool b_kmajor, int64_t epi, const optional<Tensor>& bias,
                  const optional<Tensor>& aux, const optional<Tensor>& aux_out, double p, int64_t seed,
                  int64_t variant, const optional<Tensor>& mask, const optional<Tensor>& colsum) {
  TORCH_CHECK(gemm_fused_supported(a, b, b_kmajor),
              "gemm_fused: need bf16 GPU a [M,K], b [N,K] (or [K,N] k-major), unit inner stride, 16-B aligned rows, "
              "M and N multiples of 256, K % 64 == 0, M*N < 2^32");
  TORCH_CHECK(a.device() == b.device(), "gemm_fused: device mismatch");
  TORCH_CHECK(epi >= 0 && epi <= 7, "gemm_fused: bad epilogue ", epi);
  TORCH_CHECK(p >= 0.0 && p < 1.0, "gemm_fused: dropout p must be in [0, 1)");
  const int64_t M = a.size(0), K = a.size(1), N = b_kmajor ? b.size(1) : b.size(0);
  auto out = at::empty({M, N}, a.options());
  GemmFusedParams P{};
  P.A = reinterpret_cast<const uint16_t*>(a.data_ptr());
  P.B = reinterpret_cast<const uint16_t*>(b.data_ptr());
  P.C = reinterpret_cast<uint16_t*>(out.data_ptr());
  P.lda = a.stride(0);
  P.ldb = b.stride(0);
  P.ldc = out.stride(0);
  P.M = (int)M;
  P.N = (int)N;
  P.K = (int)K;
  P.tm = (int)(M / 256);
  P.tn = (int)(N / 256);
  P.epi = (int)epi;
  if (bias.has_value() && bias->defined()) {
    TORCH_CHECK(bias->is_cuda() && bias->scalar_type() == at::kBFloat16 && bias->is_contiguous() && bias->numel() == N &&
                    reinterpret_cast<uintptr_t>(bias->data_ptr()) % 8 == 0,
                "gemm_fused: bias must be a contiguous 8-B aligned bf16 [N] GPU tensor");
    TORCH_CHECK(epi <= 2 || epi == 5, "gemm_fused: bias only on forward epilogues");
    P.bias = reinterpret_cast<const uint16_t*>(bias->data_ptr());
  }
  const bool needs_aux = epi == 3 || epi == 4 || epi == 6;
  const bool needs_aux_out = epi == 2 || epi == 5;
  auto check_mn = [&](const Tensor& t, const char* n) {
    TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kBFloat16 && t.dim() == 2 && t.size(0) == M && t.size(1) == N &&
                    t.stride(1) == 1 && t.stride(0) % 4 == 0 && reinterpret_cast<uintptr_t>(t.data_ptr()) % 8 == 0,
                "gemm_fused: ", n, " must be a bf16 [M, N] GPU tensor with unit inner stride, 8-B aligned rows");
  };
  if (needs_aux) {
    TORCH_CHECK(aux.has_value() && aux->defined(), "gemm_fused: epilogue ", epi, " needs aux");
    check_mn(*aux, "aux");
    P.aux = reinterpret_cast<const uint16_t*>(aux->data_ptr());
    P.ldaux = aux->stride(0);
  }
  if (needs_aux_out) {
    TORCH_CHECK(aux_out.has_value() && aux_out->defined(), "gemm_fused: epilogue ", epi, " needs aux_out");
    check_mn(*aux_out, "aux_out");
    P.aux_out = reinterpret_cast<uint16_t*>(aux_out->data_ptr());
    P.ldaux = aux_out->stride(0);
  }
  P.p = (float)p;
  P.scale = p > 0.0 ? (float)(1.0 / (1.0 - p)) : 1.f;
  P.seed = (uint32_t)seed;
  {  // 16-bit keep threshold, identical to common.h drop_threshold
    const double t = p * 65536.0;
    P.thr = t >= 65535.0 ? 0xFFFFu : (uint32_t)t;
  }
  {  // tile-order group size of the ping-pong kernel (read per call so microbenchmarks can A/B it in one process)
    P.grp = std::max(0, dllm::route_int("gemm_grp", 4));  // 4: +1-3 % over row-major (profiles/r1_gemm_experiments.md)
  }
  const int v = variant >= 0 ? (int)variant : (int)gemm_fused_variant(K);
  TORCH_CHECK(v == 1 || v == 8 || v == 9, "gemm_fused: variant must be 1, 8 or 9, got ", v);
  // ReLU derivative bit mask (ping-pong kernel only): epi 1 writes it when given, epi 7 (d-relu) reads it instead of aux
  const bool has_mask = mask.has_value() && mask->defined();
  TORCH_CHECK(epi != 7 || has_mask, "gemm_fused: epilogue 7 needs the ReLU mask");
  if (has_mask) {
    TORCH_CHECK(epi == 1 || epi == 7, "gemm_fused: a mask goes with epilogue 1 (write) or 7 (read)");
    TORCH_CHECK(v == 8 || v == 9, "gemm_fused: the ReLU mask needs the ping-pong kernel (variant 8 / 9)");
    TORCH_CHECK(mask->is_cuda() && mask->device() == a.device() && mask->scalar_type() == at::kInt &&
                    mask->is_contiguous() && mask->numel() == M * N / 32 &&
                    reinterpret_cast<uintptr_t>(mask->data_ptr()) % 16 == 0,
                "gemm_fused: mask must be a contiguous 16-B aligned int32 GPU tensor of M*N/32 words");
    P.mask = reinterpret_cast<uint32_t*>(mask->data_ptr());
  }
  if (colsum.has_value() && colsum->defined()) {  // per-128-row column sums of the output (GELU backward: bias grad)
    TORCH_CHECK(epi == 4 || epi == 6, "gemm_fused: colsum goes with the GELU backward epilogues (4 / 6)");
    TORCH_CHECK(v == 8 || v == 9, "gemm_fused: colsum needs the ping-pong kernel (variant 8 / 9)");
    TORCH_CHECK(colsum->is_cuda() && colsum->device() == a.device() && colsum->scalar_type() == at::kFloat &&
                    colsum->is_contiguous() && colsum->dim() == 2 && colsum->size(0) == M / 128 && colsum->size(1) == N,
                "gemm_fused: colsum must be a contiguous fp32 [M / 128, N] GPU tensor");
    P.colsum = colsum->data_ptr<float>();
  }
  check_rc(dllm_gemm_fused(&P, b_kmajor ? 1 : 0, v, stream()), "gemm_fused");
  return out;
}

// ---- one-wave-per-SIMD projection GEMM (csrc/gemm_w4.hip): out (+)= a . b (+ bias), b = [N][K] (nn.Linear weight)
// or [K][N] (b_kmajor, the input-gradient GEMM).  Ragged M / N; K % 64 == 0; N % 8 == 0.
// One beam-search step (csrc/beam.hip): logits [B * nb, V] (bf16 / fp32, unit inner stride), beam scores [B * nb]
// fp32, generated prefix seqs [B * nb, L] int64 -> (top scores [B, k_out] fp32, flat indices [B, k_out] int64).
std::vector<Tensor> beam_topk(const Tensor& logits, const Tensor& beam_scores, const Tensor& seqs, int64_t cur,
                              int64_t ngram, int64_t ban_tok, int64_t force_tok, int64_t nb, int64_t k_out) {
  TORCH_CHECK(logits.is_cuda() && logits.dim() == 2 && logits.stride(1) == 1 &&
                  (logits.scalar_type() == at::kBFloat16 || logits.scalar_type() == at::kFloat),
              "beam_topk: logits must be a 2-D bf16 / fp32 GPU tensor with unit inner stride");
  TORCH_CHECK(beam_scores.is_cuda() && beam_scores.scalar_type() == at::kFloat && beam_scores.is_contiguous() &&
                  beam_scores.numel() == logits.size(0),
              "beam_topk: beam_scores must be a contiguous fp32 [rows] GPU tensor");
  TORCH_CHECK(seqs.is_cuda() && seqs.scalar_type() == at::kLong && seqs.dim() == 2 && seqs.stride(1) == 1 &&
                  seqs.size(0) == logits.size(0) && cur <= seqs.size(1),
              "beam_topk: seqs must be an int64 [rows, L >= cur] GPU tensor with unit inner stride");
  TORCH_CHECK(nb > 0 && logits.size(0) % nb == 0, "beam_topk: rows must be a multiple of nb");
  const int64_t B = logits.size(0) / nb, V = logits.size(1);
  TORCH_CHECK(force_tok < V && ban_tok < V, "beam_topk: token id out of range");
  auto top_s = at::empty({B, k_out}, beam_scores.options());
  auto top_i = at::empty({B, k_out}, seqs.options());
  if (B > 0)
    check_rc(dllm_beam_topk(logits.data_ptr(), logits.stride(0), logits.scalar_type() == at::kBFloat16,
                            beam_scores.data_ptr<float>(), seqs.data_ptr<int64_t>(), seqs.stride(0), (int)cur,
                            (int)ngram, (int)ban_tok, (int)force_tok, (int)B, (int)nb, (int)V, (int)k_out,
                            top_s.data_ptr<float>(), top_i.data_ptr<int64_t>(), stream()),
             "beam_topk");
  return {top_s, top_i};
}

// In-place beam reorder of a [layers * 2, rows, max_len, hd] bf16 cache's live prefix (csrc/beam.hip kv_reorder).
void kv_reorder(Tensor& cache, const Tensor& src, int64_t nb, int64_t n) {
  TORCH_CHECK(cache.is_cuda() && cache.scalar_type() == at::kBFloat16 && cache.is_contiguous() && cache.dim() == 4,
              "kv_reorder: cache must be a contiguous bf16 [layers*2, rows, max_len, hd] GPU tensor");
  TORCH_CHECK(src.is_cuda() && src.scalar_type() == at::kLong && src.is_contiguous() && src.numel() == cache.size(1),
              "kv_reorder: src must be an int64 [rows] GPU tensor");
  if (n <= 0) return;
  check_rc(dllm_kv_reorder(cache.data_ptr(), src.data_ptr<int64_t>(), (int)cache.size(0), (int)cache.size(1), (int)nb,
                           (int)cache.size(2), (int)cache.size(3), (int)n, stream()),
           "kv_reorder");
}

// ---- LM head + cross-entropy on the w4 GEMM's CE epilogues (csrc/gemm_w4.hip W4_EPI_CEF / W4_EPI_CEB)
void check_lmhead_operands(const Tensor& h, const Tensor& w, const Tensor& labels, const optional<Tensor>& cbias,
                           int64_t V) {
  auto ok2 = [](const Tensor& t) {
    return t.is_cuda() && t.dim() == 2 && t.scalar_type() == at::kBFloat16 && t.stride(1) == 1 && t.stride(0) % 8 == 0 &&
           t.stride(0) >= t.size(1) && reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0 &&
           256 * t.stride(0) * 2 < (1LL << 31);
  };
  TORCH_CHECK(ok2(h) && ok2(w), "lmhead: h [N, d] and w [n, d] must be bf16 GPU, unit inner stride, 16-B aligned rows");
  TORCH_CHECK(h.size(1) == w.size(1) && h.size(1) % 64 == 0 && h.size(0) > 0 && w.size(0) > 0,
              "lmhead: d must match and be a multiple of 64");
  TORCH_CHECK(h.device() == w.device(), "lmhead: device mismatch");
  TORCH_CHECK(labels.is_cuda() && labels.scalar_type() == at::kLong && labels.is_contiguous() &&
                  labels.numel() == h.size(0),
              "lmhead: labels must be a contiguous int64 [N] GPU tensor");
  if (cbias.has_value() && cbias->defined())
    TORCH_CHECK(cbias->is_cuda() && cbias->scalar_type() == at::kFloat && cbias->is_contiguous() &&
                    cbias->numel() == V,
                "lmhead: bias must be a contiguous fp32 [V] GPU tensor");
}

void fill_w4_tiles(GemmW4Params& P, int64_t M, int64_t N, int64_t K) {
  TORCH_CHECK((M + 255) / 256 * ((N + 255) / 256) < INT_MAX && M < INT_MAX && N < INT_MAX, "gemm_w4: too large");
  P.M = (int)M; P.N = (int)N; P.K = (int)K;
  P.tm = (int)((M + 255) / 256);
  P.tn = (int)((N + 255) / 256);
  P.grp = 0;
}

// forward: loss_rows [N], lse [N] over the whole vocabulary w [V, d]; the logits are never written
std::vector<Tensor> lmhead_ce_fwd(const Tensor& h, const Tensor& w, const Tensor& labels,
                                  const optional<Tensor>& cbias, double eps, int64_t ignore) {
  const int64_t V = w.size(0);
  check_lmhead_operands(h, w, labels, cbias, V);
  const int64_t N = h.size(0), K = h.size(1);
  const int64_t np = (V + 127) / 128;
  auto f32 = h.options().dtype(at::kFloat);
  auto part = at::empty({N, np, 4}, f32);
  auto xlab = at::zeros({N}, f32);
  auto loss = at::empty({N}, f32);
  auto lse = at::empty({N}, f32);
  GemmW4Params P{};
  P.A = reinterpret_cast<const uint16_t*>(h.data_ptr());
  P.B = reinterpret_cast<const uint16_t*>(w.data_ptr());
  P.lda = h.stride(0); P.ldb = w.stride(0); P.ldc = 0;
  fill_w4_tiles(P, N, V, K);
  P.labels = labels.data_ptr<int64_t>();
  P.cbias = (cbias.has_value() && cbias->defined()) ? cbias->data_ptr<float>() : nullptr;
  P.part = part.data_ptr<float>();
  P.xlab = xlab.data_ptr<float>();
  P.pstride = (int)np;
  P.c0 = 0; P.V = (int)V; P.skip = 0; P.eps = (float)eps; P.ignore = ignore;
  check_rc(dllm_gemm_w4(&P, 0, 1, 8, stream()), "lmhead_ce_fwd (gemm_w4 CEF)");
  check_rc(dllm_ce_merge(P.part, (int)np, np, P.xlab, P.labels, loss.data_ptr<float>(), lse.data_ptr<float>(), N,
                         (int)V, (float)eps, ignore, stream()),
           "lmhead_ce_fwd (merge)");
  return {loss, lse};
}

// backward of one vocabulary slice: out = dlogits of columns [c0, c0 + w_slice.size(0)) (bf16 [N, n], n % 8 == 0)
void lmhead_ce_bwd_slice(const Tensor& h, const Tensor& w_slice, const Tensor& labels, const Tensor& lse,
                         const Tensor& gscale, const optional<Tensor>& cbias, Tensor& out, int64_t c0, int64_t V,
                         double eps, int64_t ignore, int64_t skip) {
  check_lmhead_operands(h, w_slice, labels, cbias, V);
  const int64_t N = h.size(0), K = h.size(1), n = w_slice.size(0);
  TORCH_CHECK(n % 8 == 0 && c0 >= 0 && c0 + n <= V && skip >= 0 && skip < n, "lmhead_ce_bwd_slice: bad slice");
  TORCH_CHECK(out.is_cuda() && out.device() == h.device() && out.scalar_type() == at::kBFloat16 && out.dim() == 2 &&
                  out.size(0) == N && out.size(1) == n && out.stride(1) == 1 && out.stride(0) % 8 == 0 &&
                  reinterpret_cast<uintptr_t>(out.data_ptr()) % 16 == 0 && 256 * out.stride(0) * 2 < (1LL << 31),
              "lmhead_ce_bwd_slice: out must be a bf16 [N, n] GPU tensor, 16-B aligned rows");
  TORCH_CHECK(lse.is_cuda() && lse.scalar_type() == at::kFloat && lse.is_contiguous() && lse.numel() == N,
              "lmhead_ce_bwd_slice: lse must be fp32 [N]");
  TORCH_CHECK(gscale.is_cuda() && gscale.scalar_type() == at::kFloat && gscale.numel() >= 1,
              "lmhead_ce_bwd_slice: gscale must be a fp32 GPU scalar");
  GemmW4Params P{};
  P.A = reinterpret_cast<const uint16_t*>(h.data_ptr());
  P.B = reinterpret_cast<const uint16_t*>(w_slice.data_ptr());
  P.C = reinterpret_cast<uint16_t*>(out.data_ptr());
  P.lda = h.stride(0); P.ldb = w_slice.stride(0); P.ldc = out.stride(0);
  fill_w4_tiles(P, N, n, K);
  P.labels = labels.data_ptr<int64_t>();
  P.cbias = (cbias.has_value() && cbias->defined()) ? cbias->data_ptr<float>() : nullptr;
  P.lse = lse.data_ptr<float>();
  P.gscale = gscale.data_ptr<float>();
  P.c0 = (int)c0; P.V = (int)V; P.skip = (int)skip; P.eps = (float)eps; P.ignore = ignore;
  check_rc(dllm_gemm_w4(&P, 0, 1, 9, stream()), "lmhead_ce_bwd_slice (gemm_w4 CEB)");
}

bool gemm_w4_supported(const Tensor& a, const Tensor& b, bool b_kmajor) {
  auto ok2 = [](const Tensor& t) {
    return t.is_cuda() && t.dim() == 2 && t.scalar_type() == at::kBFloat16 && t.stride(1) == 1 && t.stride(0) % 8 == 0 &&
           t.stride(0) >= t.size(1) && reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0;
  };
  if (!ok2(a) || !ok2(b)) return false;
  const int64_t M = a.size(0), K = a.size(1);
  const int64_t N = b_kmajor ? b.size(1) : b.size(0);
  const int64_t Kb = b_kmajor ? b.size(0) : b.size(1);
  // buffer-descriptor offsets are 32-bit with 0x80000000 as the out-of-range marker: every per-tile byte range < 2^31
  const bool ranges = 256 * a.stride(0) * 2 < (1LL << 31) &&
                      (b_kmajor ? K * b.stride(0) * 2 < (1LL << 31) : 256 * b.stride(0) * 2 < (1LL << 31));
  return Kb == K && K > 0 && K % 64 == 0 && M > 0 && N > 0 && N % 8 == 0 && ranges && (M + 255) / 256 * ((N + 255) / 256) < INT_MAX;
}

// epi 0: plain; 1: ReLU + dropout(p, seed) writing the keep-and-positive bit mask (NT); 7: input gradient through
// that mask (NN).  mask: int32 tensor of >= ceil(M/256) * ceil(N/256) * 2048 words (gemm_w4_mask_words).
Tensor gemm_w4(const Tensor& a, const Tensor& b, bool b_kmajor, const optional<Tensor>& bias, const optional<Tensor>& out,
               bool accumulate, int64_t grp, bool persist, int64_t epi, double p, int64_t seed,
               const optional<Tensor>& mask, bool mask_pp, const optional<Tensor>& aux,
               const optional<Tensor>& aux_out, const optional<Tensor>& colsum) {
  TORCH_CHECK(gemm_w4_supported(a, b, b_kmajor),
              "gemm_w4: need bf16 GPU a [M,K], b [N,K] (or [K,N] k-major), unit inner stride, 16-B aligned rows, K % 64 == 0, "
              "N % 8 == 0");
  TORCH_CHECK(a.device() == b.device(), "gemm_w4: device mismatch");
  const int64_t M = a.size(0), K = a.size(1), N = b_kmajor ? b.size(1) : b.size(0);
  Tensor c;
  if (out.has_value() && out->defined()) {
    c = *out;
    TORCH_CHECK(c.is_cuda() && c.device() == a.device() && c.scalar_type() == at::kBFloat16 && c.dim() == 2 &&
                    c.size(0) == M && c.size(1) == N && c.stride(1) == 1 && c.stride(0) % 8 == 0 &&
                    reinterpret_cast<uintptr_t>(c.data_ptr()) % 16 == 0 && 256 * c.stride(0) * 2 < (1LL << 31),
                "gemm_w4: out must be a bf16 [M, N] GPU tensor with unit inner stride, 16-B aligned rows and a 256-row "
                "byte range < 2^31");
  } else {
    TORCH_CHECK(!accumulate, "gemm_w4: accumulate needs out");
    c = at::empty({M, N}, a.options());
  }
  GemmW4Params P{};
  P.A = reinterpret_cast<const uint16_t*>(a.data_ptr());
  P.B = reinterpret_cast<const uint16_t*>(b.data_ptr());
  P.C = reinterpret_cast<uint16_t*>(c.data_ptr());
  if (bias.has_value() && bias->defined()) {
    TORCH_CHECK(bias->is_cuda() && bias->device() == a.device() && bias->scalar_type() == at::kBFloat16 &&
                    bias->is_contiguous() && bias->numel() == N && reinterpret_cast<uintptr_t>(bias->data_ptr()) % 8 == 0,
                "gemm_w4: bias must be a contiguous 8-B aligned bf16 [N] GPU tensor");
    P.bias = reinterpret_cast<const uint16_t*>(bias->data_ptr());
  }
  P.lda = a.stride(0);
  P.ldb = b.stride(0);
  P.ldc = c.stride(0);
  P.M = (int)M;
  P.N = (int)N;
  P.K = (int)K;
  P.tm = (int)((M + 255) / 256);
  P.tn = (int)((N + 255) / 256);
  P.grp = grp >= 0 ? (int)grp : 8;  // tile-group sweep: profiles/r3_gemm_w4_grp_sweep.txt
  P.accumulate = accumulate ? 1 : 0;
  if (epi == 11 || epi == 12) {
    // GELU FFN (csrc/gemm_w4.hip W4_EPI_GELU / W4_EPI_DGELU): bf16 [M, N] derivative out (forward) / in (backward),
    // and the backward's fp32 [M / 128, N] dU column partials
    const optional<Tensor>& x = epi == 11 ? aux_out : aux;
    TORCH_CHECK(x.has_value() && x->defined() && x->is_cuda() && x->device() == a.device() &&
                    x->scalar_type() == at::kBFloat16 && x->dim() == 2 && x->size(0) == M && x->size(1) == N &&
                    x->stride(1) == 1 && x->stride(0) % 8 == 0 && reinterpret_cast<uintptr_t>(x->data_ptr()) % 16 == 0 &&
                    256 * x->stride(0) * 2 < (1LL << 31),
                "gemm_w4: GELU epilogues need a bf16 [M, N] aux tensor with 16-B aligned rows");
    TORCH_CHECK(M * N < (1LL << 32), "gemm_w4: dropout element index must fit 32 bits");
    TORCH_CHECK(p >= 0.0 && p < 1.0, "gemm_w4: dropout p in [0, 1)");
    P.ldaux = x->stride(0);
    if (epi == 11) {
      P.aux_out = reinterpret_cast<uint16_t*>(x->data_ptr());
    } else {
      P.aux = reinterpret_cast<const uint16_t*>(x->data_ptr());
      TORCH_CHECK(colsum.has_value() && colsum->defined() && colsum->is_cuda() &&
                      colsum->scalar_type() == at::kFloat && colsum->is_contiguous() && M % 128 == 0 &&
                      colsum->numel() == (M / 128) * N && reinterpret_cast<uintptr_t>(colsum->data_ptr()) % 16 == 0,
                  "gemm_w4: GELU backward needs an fp32 contiguous [M / 128, N] colsum tensor (M % 128 == 0)");
      P.colsum = colsum->data_ptr<float>();
    }
    P.p = (float)p;
    P.scale = p > 0.0 ? (float)(1.0 / (1.0 - p)) : 1.f;
    P.seed = (uint32_t)seed;
    const double t = p * 65536.0;  // csrc/common.h drop_threshold
    P.thr = t >= 65535.0 ? 0xFFFFu : (uint32_t)t;
  } else if (epi != 0) {
    TORCH_CHECK(mask.has_value() && mask->defined() && mask->is_cuda() && mask->device() == a.device() &&
                    mask->scalar_type() == at::kInt && mask->is_contiguous() &&
                    mask->numel() >= (int64_t)P.tm * P.tn * 2048 && reinterpret_cast<uintptr_t>(mask->data_ptr()) % 16 == 0,
                "gemm_w4: epilogue mask must be a contiguous int32 GPU tensor of >= ceil(M/256)*ceil(N/256)*2048 words");
    TORCH_CHECK(M * N < (1LL << 32), "gemm_w4: dropout element index must fit 32 bits");
    TORCH_CHECK(p >= 0.0 && p < 1.0, "gemm_w4: dropout p in [0, 1)");
    P.mask = reinterpret_cast<uint32_t*>(mask->data_ptr());
    P.mask_pp = mask_pp ? 1 : 0;
    P.p = (float)p;
    P.scale = p > 0.0 ? (float)(1.0 / (1.0 - p)) : 1.f;
    P.seed = (uint32_t)seed;
    const double t = p * 65536.0;  // csrc/common.h drop_threshold
    P.thr = t >= 65535.0 ? 0xFFFFu : (uint32_t)t;
  }
  check_rc(dllm_gemm_w4(&P, b_kmajor ? 1 : 0, persist ? 1 : 0, (int)epi, stream()), "gemm_w4");
  return c;
}

int64_t gemm_w4_mask_words(int64_t M, int64_t N) { return ((M + 255) / 256) * ((N + 255) / 256) * 2048; }

// Gated-GELU FFN (FLAN-T5 / T5 v1.1 "gated-gelu", tanh GELU) on the ping-pong kernel, csrc/gemm_fused.hip epi 8 / 9.
// forward: x [M, d] . [wi_0; wi_1]^T ([2F, d], the stacked wi weight) -> h = dropout(gelu(x wi_0^T) * (x wi_1^T)) [M, F]
//          plus G1 = s gelu'(gate) up and G2 = s gelu(gate) ([M, F] each, s = keep / (1 - p)) for the backward;
// backward: dH = dy [M, d] . wo [d, F] (k-major) -> [dH G1 | dH G2] = d(stacked wi output) [M, 2F].
// M % 256 == 0, F % 256 == 0, d % 64 == 0 (the fused FFN's shape rule, ops/ffn.py).
static GemmFusedParams geglu_params(const Tensor& a, const Tensor& b, bool b_kmajor, int epi) {
  TORCH_CHECK(gemm_fused_supported(a, b, b_kmajor), "gemm_geglu: unsupported operands (bf16 GPU, M / N % 256, K % 64)");
  TORCH_CHECK(a.device() == b.device(), "gemm_geglu: device mismatch");
  const int64_t M = a.size(0), K = a.size(1), N = b_kmajor ? b.size(1) : b.size(0);
  GemmFusedParams P{};
  P.A = reinterpret_cast<const uint16_t*>(a.data_ptr());
  P.B = reinterpret_cast<const uint16_t*>(b.data_ptr());
  P.lda = a.stride(0);
  P.ldb = b.stride(0);
  P.M = (int)M;
  P.N = (int)N;
  P.K = (int)K;
  P.tm = (int)(M / 256);
  P.tn = (int)(N / 256);
  P.epi = epi;
  P.scale = 1.f;
  P.grp = std::max(0, dllm::route_int("gemm_grp", 4));
  return P;
}

std::vector<Tensor> gemm_geglu(const Tensor& x, const Tensor& wi, double p, int64_t seed) {
  TORCH_CHECK(p >= 0.0 && p < 1.0, "gemm_geglu: dropout p must be in [0, 1)");
  GemmFusedParams P = geglu_params(x, wi, false, 8);
  const int64_t M = P.M, F = P.N / 2;
  TORCH_CHECK(F % 256 == 0, "gemm_geglu: d_ff must be a multiple of 256");
  auto h = at::empty({M, F}, x.options());
  auto g1 = at::empty({M, F}, x.options());
  auto g2 = at::empty({M, F}, x.options());
  P.C = reinterpret_cast<uint16_t*>(h.data_ptr());
  P.ldc = F;
  P.aux_out = reinterpret_cast<uint16_t*>(g1.data_ptr());
  P.aux_out2 = reinterpret_cast<uint16_t*>(g2.data_ptr());
  P.ldaux = F;
  P.p = (float)p;
  P.scale = p > 0.0 ? (float)(1.0 / (1.0 - p)) : 1.f;
  P.seed = (uint32_t)seed;
  const double t = p * 65536.0;
  P.thr = t >= 65535.0 ? 0xFFFFu : (uint32_t)t;
  check_rc(dllm_gemm_fused(&P, 0, 9, stream()), "gemm_geglu");
  return {h, g1, g2};
}

Tensor gemm_dgeglu(const Tensor& dy, const Tensor& wo, const Tensor& g1, const Tensor& g2) {
  GemmFusedParams P = geglu_params(dy, wo, true, 9);
  const int64_t M = P.M, F = P.N;
  for (const Tensor* t : {&g1, &g2})
    TORCH_CHECK(t->is_cuda() && t->device() == dy.device() && t->scalar_type() == at::kBFloat16 && t->is_contiguous() &&
                    t->dim() == 2 && t->size(0) == M && t->size(1) == F,
                "gemm_dgeglu: G1 / G2 must be contiguous bf16 [M, F] GPU tensors");
  auto du = at::empty({M, 2 * F}, dy.options());
  P.C = reinterpret_cast<uint16_t*>(du.data_ptr());
  P.ldc = 2 * F;
  P.aux = reinterpret_cast<const uint16_t*>(g1.data_ptr());
  P.aux2 = reinterpret_cast<const uint16_t*>(g2.data_ptr());
  P.ldaux = F;
  check_rc(dllm_gemm_fused(&P, 1, 9, stream()), "gemm_dgeglu");
  return du;
}

// out (+)= column sums of x ([T, N] bf16, unit inner stride): bias gradients accumulated in place
void colsum_partials_acc(const Tensor& part, Tensor& out) {
  TORCH_CHECK(part.is_cuda() && part.scalar_type() == at::kFloat && part.dim() == 2 && part.is_contiguous() &&
                  out.is_cuda() && out.is_contiguous() && out.numel() == part.size(1) &&
                  (out.scalar_type() == at::kFloat || out.scalar_type() == at::kBFloat16),
              "colsum_partials_acc: part fp32 [G, d] contiguous, out fp32/bf16 [d] contiguous");
  TORCH_CHECK(part.size(0) < INT_MAX && part.size(1) < INT_MAX, "colsum_partials_acc: too large");
  check_rc(dllm_colsum_partials_acc(part.data_ptr<float>(), out.data_ptr(), out.scalar_type() == at::kBFloat16 ? 1 : 0,
                                    (int)part.size(0), (int)part.size(1), stream()),
           "colsum_partials_acc");
}

void colsum_acc(const Tensor& x, Tensor& out) {
  check_gpu(x, "x");
  TORCH_CHECK(x.dim() == 2 && x.scalar_type() == at::kBFloat16 && x.stride(1) == 1 && x.stride(0) % 2 == 0 &&
                  reinterpret_cast<uintptr_t>(x.data_ptr()) % 4 == 0,
              "colsum_acc: x must be bf16 [T, N] with unit inner stride and 4-B aligned rows");
  const int64_t T = x.size(0), N = x.size(1);
  TORCH_CHECK(N % 2 == 0 && N < (1LL << 31), "colsum_acc: N must be even");
  TORCH_CHECK(out.is_cuda() && out.is_contiguous() && out.numel() == N &&
                  (out.scalar_type() == at::kBFloat16 || out.scalar_type() == at::kFloat),
              "colsum_acc: out must be a contiguous bf16/fp32 [N] GPU tensor");
  if (T == 0) return;
  const int R = (int)std::min<int64_t>(T, dllm_colsum_rows());
  auto part = at::empty({(int64_t)R * N}, x.options().dtype(at::kFloat));
  check_rc(dllm_colsum_acc(x.data_ptr(), x.stride(0), T, (int)N, part.data_ptr<float>(), out.data_ptr(),
                           out.scalar_type() == at::kBFloat16, stream()),
           "colsum_acc");
}

// out[ids[t]] += dy[t] for every token (sorted ids + their positions), deterministic (csrc/embed.hip)
void embed_bwd(const Tensor& ids_sorted, const Tensor& perm, const Tensor& dy, Tensor& out, int64_t padding_idx) {
  check_gpu(dy, "dy");
  TORCH_CHECK(ids_sorted.scalar_type() == at::kLong && perm.scalar_type() == at::kLong && ids_sorted.dim() == 1 &&
                  perm.sizes() == ids_sorted.sizes() && ids_sorted.is_contiguous() && perm.is_contiguous(),
              "embed_bwd: ids / perm must be contiguous int64 [T]");
  TORCH_CHECK(dy.dim() == 2 && dy.scalar_type() == at::kBFloat16 && dy.stride(1) == 1 && dy.stride(0) % 8 == 0 &&
                  reinterpret_cast<uintptr_t>(dy.data_ptr()) % 16 == 0 && dy.size(0) == ids_sorted.size(0),
              "embed_bwd: dy must be bf16 [T, d] with 16-B aligned rows");
  const int64_t T = dy.size(0), d = dy.size(1);
  TORCH_CHECK(d % 8 == 0 && d <= 2048, "embed_bwd: d must be a multiple of 8 and <= 2048");
  TORCH_CHECK(out.is_cuda() && out.dim() == 2 && out.size(1) == d && out.is_contiguous() &&
                  (out.scalar_type() == at::kBFloat16 || out.scalar_type() == at::kFloat),
              "embed_bwd: out must be a contiguous bf16/fp32 [V, d] GPU tensor");
  if (T == 0) return;
  auto ws = at::empty({(T + 63) / 64 * d}, dy.options().dtype(at::kFloat));
  check_rc(dllm_embed_bwd(ids_sorted.data_ptr<int64_t>(), perm.data_ptr<int64_t>(), dy.data_ptr(), dy.stride(0), T,
                          (int)d, ws.data_ptr<float>(), out.data_ptr(), out.size(0), padding_idx,
                          out.scalar_type() == at::kFloat, stream()),
           "embed_bwd");
}

// Device step counter for graph-replayable dropout (csrc/common.h DLLM_SEED_STEP_TU): every dropout kernel mixes
// *step into its site seed; None turns it off (site seeds used as given).  The tensor must outlive its use.
void set_seed_step(const optional<Tensor>& step) {
  const uint32_t* p = nullptr;
  if (step.has_value() && step->defined()) {
    TORCH_CHECK(step->is_cuda() && step->scalar_type() == at::kInt && step->numel() == 1,
                "set_seed_step: a 1-element int32 GPU tensor");
    p = reinterpret_cast<const uint32_t*>(step->data_ptr());
  }
  check_rc(dllm_set_seed_step_norm(p), "set_seed_step(norm)");
  check_rc(dllm_set_seed_step_act(p), "set_seed_step(act)");
  check_rc(dllm_set_seed_step_attn(p), "set_seed_step(attn)");
  check_rc(dllm_set_seed_step_attn_f32(p), "set_seed_step(attn_f32)");
  check_rc(dllm_set_seed_step_gemm_fused(p), "set_seed_step(gemm_fused)");
  check_rc(dllm_set_seed_step_gemm_w4(p), "set_seed_step(gemm_w4)");
}

namespace dllm {
void bind_reducer(pybind11::module& m);  // csrc/reducer.cpp
}

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.doc() = "gfx950 (MI355X) kernel library for distributed_llms_example_amd";
  m.def("norm_fwd", &norm_fwd);
  m.def("norm_bwd", &norm_bwd, py::arg("dout"), py::arg("ds"), py::arg("s"), py::arg("w"), py::arg("b"),
        py::arg("mean"), py::arg("rstd"), py::arg("p"), py::arg("seed"), py::arg("kind"), py::arg("want_stream"),
        py::arg("dw_acc") = py::none(), py::arg("db_acc") = py::none(), py::arg("want_colsum") = false,
        py::arg("partials_only") = false);
  m.def("act_fwd", &act_fwd);
  m.def("act_bwd", &act_bwd);
  m.def("dropout_fwd", &dropout_fwd);
  m.def("ce_fwd", &ce_fwd);
  m.def("ce_bwd", &ce_bwd);
  m.def("sq_norm", &sq_norm);
  m.def("embed_bwd", &embed_bwd);
  m.def("ce_chunk_fwd", &ce_chunk_fwd);
  m.def("ce_chunk_bwd", &ce_chunk_bwd);
  m.def("adamw_step", &adamw_step, py::arg("param"), py::arg("master"), py::arg("grad"), py::arg("m"), py::arg("v"),
        py::arg("wd_mask"), py::arg("coef"), py::arg("lr"), py::arg("b1"), py::arg("b2"), py::arg("eps"), py::arg("wd"),
        py::arg("bc1"), py::arg("bc2"), py::arg("hyper") = py::none());
  m.def("set_seed_step", &set_seed_step, "device step counter mixed into every dropout site seed (None: off)");
  m.def("attn_fwd", &attn_fwd, py::arg("q"), py::arg("k"), py::arg("v"), py::arg("kpm"), py::arg("lut"),
        py::arg("scale"), py::arg("causal"), py::arg("p"), py::arg("seed"), py::arg("dmask_in") = py::none(),
        py::arg("sat_lo") = -1, py::arg("sat_hi") = -1);
  m.def("attn_dropout_mask", &attn_dropout_mask);
  m.def("attn_bwd", &attn_bwd, py::arg("dout"), py::arg("q"), py::arg("k"), py::arg("v"), py::arg("o"),
        py::arg("lse"), py::arg("kpm"), py::arg("lut"), py::arg("scale"), py::arg("causal"), py::arg("p"),
        py::arg("seed"), py::arg("need_dlut"), py::arg("dq_out") = py::none(), py::arg("dk_out") = py::none(),
        py::arg("dv_out") = py::none(), py::arg("dmask") = py::none(), py::arg("sat_lo") = -1,
        py::arg("sat_hi") = -1, py::arg("csq") = py::none(), py::arg("csk") = py::none(),
        py::arg("csv") = py::none());
  m.def("attn_params_size", []() { return dllm_attn_params_size(); });
  m.def("attn_f32_fwd", &attn_f32_fwd, py::arg("q"), py::arg("k"), py::arg("v"), py::arg("kpm"), py::arg("lut"),
        py::arg("scale"), py::arg("causal"), py::arg("p"), py::arg("seed"));
  m.def("attn_f32_bwd", &attn_f32_bwd, py::arg("dout"), py::arg("q"), py::arg("k"), py::arg("v"), py::arg("o"),
        py::arg("lse"), py::arg("kpm"), py::arg("lut"), py::arg("scale"), py::arg("causal"), py::arg("p"),
        py::arg("seed"), py::arg("need_dlut"), py::arg("dq_out") = py::none(), py::arg("dk_out") = py::none(),
        py::arg("dv_out") = py::none());
  m.def("gemm_wgrad_segs", &gemm_wgrad_segs, "c (+)= sum_i a_i^T b_i (deferred micro-batch segments, w4)",
        py::arg("a"), py::arg("b"), py::arg("c"), py::arg("beta") = true);
  m.def("gemm_wgrad", &gemm_wgrad, "c (+)= a^T b (token-major bf16 operands)", py::arg("a"), py::arg("b"), py::arg("c"),
        py::arg("beta") = true, py::arg("variant") = 0, py::arg("splits") = 0);
  m.def("gemm_wgrad_supported", &gemm_wgrad_supported);
  m.def("gemm_fused", &gemm_fused, "epi(a . b) with a fused bias / activation / dropout (or their backward) epilogue",
        py::arg("a"), py::arg("b"), py::arg("b_kmajor"), py::arg("epi"), py::arg("bias") = py::none(),
        py::arg("aux") = py::none(), py::arg("aux_out") = py::none(), py::arg("p") = 0.0, py::arg("seed") = 0,
        py::arg("variant") = -1, py::arg("mask") = py::none(), py::arg("colsum") = py::none());
  m.def("gemm_fused_supported", &gemm_fused_supported);
  m.def("gemm_geglu", &gemm_geglu, "gated-GELU FFN input GEMM: (h, G1, G2) from x and the stacked [wi_0; wi_1]");
  m.def("gemm_dgeglu", &gemm_dgeglu, "gated-GELU FFN backward GEMM: d(stacked wi output) from dy, wo, G1, G2");
  m.def("gemm_fused_variant", &gemm_fused_variant, "default kernel variant for reduction length K");
  m.def("gemm_w4", &gemm_w4, "out (+)= a . b (+ bias) on the one-wave-per-SIMD GEMM (csrc/gemm_w4.hip)", py::arg("a"),
        py::arg("b"), py::arg("b_kmajor"), py::arg("bias") = py::none(), py::arg("out") = py::none(),
        py::arg("accumulate") = false, py::arg("grp") = -1, py::arg("persist") = true, py::arg("epi") = 0,
        py::arg("p") = 0.0, py::arg("seed") = 0, py::arg("mask") = py::none(), py::arg("mask_pp") = false,
        py::arg("aux") = py::none(), py::arg("aux_out") = py::none(), py::arg("colsum") = py::none());
  m.def("gemm_w4_mask_words", &gemm_w4_mask_words);
  m.def("lmhead_ce_fwd", &lmhead_ce_fwd, "LM-head GEMM + CE forward (gemm_w4 CE epilogue + row merge): (loss_rows, lse)");
  m.def("lmhead_ce_bwd_slice", &lmhead_ce_bwd_slice, "dlogits of one vocabulary slice from the GEMM's CE epilogue");
  m.def("gemm_w4_supported", &gemm_w4_supported);
  m.def("beam_topk", &beam_topk);
  m.def("kv_reorder", &kv_reorder);
  m.def("colsum_partials_acc", &colsum_partials_acc, "out += part.sum(0) for fp32 partial column sums [G, d]");
  m.def("colsum_acc", &colsum_acc, "out += x.sum(0) for a token-major bf16 x (bias gradients)");
  dllm::bind_reducer(m);
  m.attr("arch") = "gfx950";
}

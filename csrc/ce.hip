// Fused (label-smoothed) cross-entropy on LM-head logits, for gfx950.
// fwd: one 256-thread block per row: online max/sum-exp over V (fp32 math on bf16 logits, optional
//      additive fp32 bias = BART final_logits_bias), writes loss_row and lse.
//      loss = lse - (1-eps)*x_y - eps*mean_v(x_v);  ignored rows (label == ignore_index) -> 0.
// bwd: dx_v = g * (exp(x_v - lse) - eps/V - (1-eps)*[v==y]) with g = *scale (device scalar, no host
//      sync), written as bf16 — optionally in place over the logits (the only consumer).
#include "common.h"

using namespace dllm;

namespace {

template <typename T, bool VEC>
__global__ __launch_bounds__(256) void ce_fwd_kernel(const T* __restrict__ logits, const int64_t* __restrict__ labels,
                                                     const float* __restrict__ bias, float* __restrict__ loss_out,
                                                     float* __restrict__ lse_out, int V, float eps, long ignore) {
  __shared__ float red[4];
  const long row = blockIdx.x;
  const T* x = logits + row * (long)V;
  float m = -INFINITY, s = 0.f, sx = 0.f;
  if (VEC) {
    for (int c = threadIdx.x * 4; c < V; c += 256 * 4) {
      f32x4 v = Elem<T>::load4(x + c);
      if (bias != nullptr) v += *reinterpret_cast<const f32x4*>(bias + c);
      const float lm = fmaxf(fmaxf(v.x, v.y), fmaxf(v.z, v.w));
      const float nm = fmaxf(m, lm);
      s = s * __expf(m - nm) + __expf(v.x - nm) + __expf(v.y - nm) + __expf(v.z - nm) + __expf(v.w - nm);
      m = nm;
      sx += v.x + v.y + v.z + v.w;
    }
  } else {
    for (int c = threadIdx.x; c < V; c += 256) {
      float v = Elem<T>::load(x + c);
      if (bias != nullptr) v += bias[c];
      const float nm = fmaxf(m, v);
      s = s * __expf(m - nm) + __expf(v - nm);
      m = nm;
      sx += v;
    }
  }
  const float M = block_max<256>(m, red);
  const float scaled = (m == -INFINITY) ? 0.f : s * __expf(m - M);
  const float S = block_sum<256>(scaled, red);
  const float SX = block_sum<256>(sx, red);
  if (threadIdx.x == 0) {
    const float lse = M + __logf(S);
    const long y = labels[row];
    float loss = 0.f;
    if (y != ignore && y >= 0 && y < V) {
      float xy = Elem<T>::load(x + y);
      if (bias != nullptr) xy += bias[y];
      loss = lse - (1.f - eps) * xy - eps * SX / (float)V;
    }
    loss_out[row] = loss;
    lse_out[row] = lse;
  }
}

template <typename T, bool VEC>
__global__ __launch_bounds__(256) void ce_bwd_kernel(const float* __restrict__ scale, const T* __restrict__ logits,
                                                     const int64_t* __restrict__ labels,
                                                     const float* __restrict__ lse_in, const float* __restrict__ bias,
                                                     T* __restrict__ dlogits, int V, float eps, long ignore) {
  const long row = blockIdx.x;
  const T* x = logits + row * (long)V;
  T* dx = dlogits + row * (long)V;
  const long y = labels[row];
  const bool valid = (y != ignore && y >= 0 && y < V);
  const float g = valid ? scale[0] : 0.f;
  const float lse = lse_in[row];
  const float off = eps / (float)V;
  const float hit = 1.f - eps;
  if (VEC) {
    for (int c = threadIdx.x * 4; c < V; c += 256 * 4) {
      f32x4 v = Elem<T>::load4(x + c);
      if (bias != nullptr) v += *reinterpret_cast<const f32x4*>(bias + c);
      f32x4 r;
#pragma unroll
      for (int k = 0; k < 4; ++k) r[k] = g * (__expf(v[k] - lse) - off - ((c + k) == y ? hit : 0.f));
      Elem<T>::store4(dx + c, r);
    }
  } else {
    for (int c = threadIdx.x; c < V; c += 256) {
      float v = Elem<T>::load(x + c);
      if (bias != nullptr) v += bias[c];
      Elem<T>::store(dx + c, g * (__expf(v - lse) - off - (c == y ? hit : 0.f)));
    }
  }
}

}  // namespace

extern "C" int dllm_ce_fwd(const void* logits, const int64_t* labels, const float* bias, float* loss, float* lse,
                           long N, int V, float eps, long ignore, int is_bf16, hipStream_t st) {
  const bool vec = (V % 4) == 0;
  dim3 g(N), b(256);
#define L(T, VE) hipLaunchKernelGGL((ce_fwd_kernel<T, VE>), g, b, 0, st, (const T*)logits, labels, bias, loss, lse, V, eps, ignore)
  if (is_bf16) { if (vec) L(uint16_t, true); else L(uint16_t, false); }
  else { if (vec) L(float, true); else L(float, false); }
#undef L
  DLLM_CHECK_LAUNCH();
  return 0;
}

extern "C" int dllm_ce_bwd(const float* scale, const void* logits, const int64_t* labels, const float* lse,
                           const float* bias, void* dlogits, long N, int V, float eps, long ignore, int is_bf16,
                           hipStream_t st) {
  const bool vec = (V % 4) == 0;
  dim3 g(N), b(256);
#define L(T, VE) hipLaunchKernelGGL((ce_bwd_kernel<T, VE>), g, b, 0, st, scale, (const T*)logits, labels, lse, bias, (T*)dlogits, V, eps, ignore)
  if (is_bf16) { if (vec) L(uint16_t, true); else L(uint16_t, false); }
  else { if (vec) L(float, true); else L(float, false); }
#undef L
  DLLM_CHECK_LAUNCH();
  return 0;
}

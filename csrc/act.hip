// FFN activation (+ gate) (+ dropout) forward/backward and standalone dropout, for gfx950.
// act: 0 relu (T5 v1.0), 1 gelu-erf (BART), 2 gelu_new/tanh (flan-T5 gated), 3 silu.
// gated: x is [N, 2F] = [wi_0 x | wi_1 x] (one fused GEMM); y = act(x[:, :F]) * x[:, F:].
// Dropout keep-decision on OUTPUT element index (row*F + col), regenerated in backward.
#include "common.h"

using namespace dllm;

DLLM_SEED_STEP_TU(act)

namespace {

constexpr float kSqrt2OverPi = 0.7978845608028654f;
constexpr float kInvSqrt2 = 0.7071067811865476f;
constexpr float kInvSqrt2Pi = 0.3989422804014327f;

template <int ACT>
DLLM_DEVICE float act_f(float x) {
  if (ACT == 0) return x > 0.f ? x : 0.f;
  if (ACT == 1) return 0.5f * x * (1.f + erff(x * kInvSqrt2));
  if (ACT == 2) return 0.5f * x * (1.f + tanhf(kSqrt2OverPi * (x + 0.044715f * x * x * x)));
  return x / (1.f + __expf(-x));
}

template <int ACT>
DLLM_DEVICE float act_df(float x) {
  if (ACT == 0) return x > 0.f ? 1.f : 0.f;
  if (ACT == 1) return 0.5f * (1.f + erff(x * kInvSqrt2)) + x * kInvSqrt2Pi * __expf(-0.5f * x * x);
  if (ACT == 2) {
    const float u = kSqrt2OverPi * (x + 0.044715f * x * x * x);
    const float t = tanhf(u);
    return 0.5f * (1.f + t) + 0.5f * x * (1.f - t * t) * kSqrt2OverPi * (1.f + 3.f * 0.044715f * x * x);
  }
  const float s = 1.f / (1.f + __expf(-x));
  return s * (1.f + x * (1.f - s));
}

// dropout of the activation output: the row-Weyl decisions of (token row, output column) that the fused FFN GEMM
// epilogues draw (common.h rw_*, csrc/gemm_w4.hip / gemm_fused.hip; ops/rng.py rowwise_keep_mask)
DLLM_DEVICE void drop4(f32x4& v, uint32_t seed, uint32_t thr, long row, int col, float dscale) {
  rw_dropout4(v, mix32(seed, (uint32_t)row), rw_t2(thr), (uint32_t)col, dscale);
}

// one thread = 4 consecutive output elements of one row; F % 4 == 0
template <typename T, int ACT, bool GATED>
__global__ __launch_bounds__(256) void act_fwd_kernel(const T* __restrict__ x, T* __restrict__ y, long total4, int F,
                                                      float p, uint32_t seed, uint32_t thr) {
  if (p > 0.f) seed = eff_seed(seed);
  const float dscale = p > 0.f ? 1.f / (1.f - p) : 1.f;
  const int F4 = F / 4;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < total4; i += (long)gridDim.x * 256) {
    const long row = i / F4;
    const int col = (int)(i - row * F4) * 4;
    const long oidx = row * F + col;
    f32x4 a, r;
    if (GATED) {
      a = Elem<T>::load4(x + row * 2 * F + col);
      f32x4 g = Elem<T>::load4(x + row * 2 * F + F + col);
#pragma unroll
      for (int k = 0; k < 4; ++k) r[k] = act_f<ACT>(a[k]) * g[k];
    } else {
      a = Elem<T>::load4(x + oidx);
#pragma unroll
      for (int k = 0; k < 4; ++k) r[k] = act_f<ACT>(a[k]);
    }
    if (p > 0.f) drop4(r, seed, thr, row, col, dscale);
    Elem<T>::store4(y + oidx, r);
  }
}

template <typename T, int ACT, bool GATED>
__global__ __launch_bounds__(256) void act_bwd_kernel(const T* __restrict__ dy, const T* __restrict__ x,
                                                      T* __restrict__ dx, long total4, int F, float p, uint32_t seed,
                                                      uint32_t thr) {
  if (p > 0.f) seed = eff_seed(seed);
  const float dscale = p > 0.f ? 1.f / (1.f - p) : 1.f;
  const int F4 = F / 4;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < total4; i += (long)gridDim.x * 256) {
    const long row = i / F4;
    const int col = (int)(i - row * F4) * 4;
    const long oidx = row * F + col;
    f32x4 g = Elem<T>::load4(dy + oidx);
    if (p > 0.f) drop4(g, seed, thr, row, col, dscale);
    if (GATED) {
      f32x4 a = Elem<T>::load4(x + row * 2 * F + col);
      f32x4 b = Elem<T>::load4(x + row * 2 * F + F + col);
      f32x4 da, db;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        da[k] = g[k] * b[k] * act_df<ACT>(a[k]);
        db[k] = g[k] * act_f<ACT>(a[k]);
      }
      Elem<T>::store4(dx + row * 2 * F + col, da);
      Elem<T>::store4(dx + row * 2 * F + F + col, db);
    } else {
      f32x4 a = Elem<T>::load4(x + oidx);
#pragma unroll
      for (int k = 0; k < 4; ++k) g[k] *= act_df<ACT>(a[k]);
      Elem<T>::store4(dx + oidx, g);
    }
  }
}

template <typename T>
__global__ __launch_bounds__(256) void dropout_kernel(const T* __restrict__ x, T* __restrict__ y, long total4, float p,
                                                      uint32_t seed, uint32_t thr) {
  seed = eff_seed(seed);
  const float dscale = 1.f / (1.f - p);
  for (long i = blockIdx.x * 256L + threadIdx.x; i < total4; i += (long)gridDim.x * 256) {
    f32x4 v = Elem<T>::load4(x + i * 4);
    dropout4(v, seed, thr, (uint32_t)(i * 4), dscale);
    Elem<T>::store4(y + i * 4, v);
  }
}

inline int grid_for(long total4) {
  long g = (total4 + 255) / 256;
  return (int)(g < 8192 ? (g > 0 ? g : 1) : 8192);
}

template <typename T>
int act_dispatch(bool fwd, const void* a, const void* b, void* out, long N, int F, int act, bool gated, float p,
                 uint32_t seed, hipStream_t st) {
  const long total4 = N * (long)F / 4;
  const int g = grid_for(total4);
  const uint32_t thr = drop_threshold(p);
#define CASE(A, G)                                                                                                 \
  if (act == A && gated == G) {                                                                                    \
    if (fwd)                                                                                                       \
      hipLaunchKernelGGL((act_fwd_kernel<T, A, G>), dim3(g), dim3(256), 0, st, (const T*)a, (T*)out, total4, F, p, \
                         seed, thr);                                                                               \
    else                                                                                                           \
      hipLaunchKernelGGL((act_bwd_kernel<T, A, G>), dim3(g), dim3(256), 0, st, (const T*)a, (const T*)b, (T*)out,  \
                         total4, F, p, seed, thr);                                                                 \
    DLLM_CHECK_LAUNCH();                                                                                           \
    return 0;                                                                                                      \
  }
  CASE(0, false) CASE(1, false) CASE(2, false) CASE(3, false)
  CASE(0, true) CASE(1, true) CASE(2, true) CASE(3, true)
#undef CASE
  return -1;
}

}  // namespace

// fwd: a = x [N, F or 2F], out = y [N, F].   bwd: a = dy [N, F], b = x, out = dx.
extern "C" int dllm_act_fwd(const void* x, void* y, long N, int F, int act, int gated, float p, uint32_t seed,
                            int is_bf16, hipStream_t st) {
  if (F % 4) return -2;
  return is_bf16 ? act_dispatch<uint16_t>(true, x, nullptr, y, N, F, act, gated, p, seed, st)
                 : act_dispatch<float>(true, x, nullptr, y, N, F, act, gated, p, seed, st);
}

extern "C" int dllm_act_bwd(const void* dy, const void* x, void* dx, long N, int F, int act, int gated, float p,
                            uint32_t seed, int is_bf16, hipStream_t st) {
  if (F % 4) return -2;
  return is_bf16 ? act_dispatch<uint16_t>(false, dy, x, dx, N, F, act, gated, p, seed, st)
                 : act_dispatch<float>(false, dy, x, dx, N, F, act, gated, p, seed, st);
}

extern "C" int dllm_dropout(const void* x, void* y, long numel, float p, uint32_t seed, int is_bf16, hipStream_t st) {
  if (numel % 4) return -2;
  const long total4 = numel / 4;
  const uint32_t thr = drop_threshold(p);
  if (is_bf16)
    hipLaunchKernelGGL(dropout_kernel<uint16_t>, dim3(grid_for(total4)), dim3(256), 0, st, (const uint16_t*)x,
                       (uint16_t*)y, total4, p, seed, thr);
  else
    hipLaunchKernelGGL(dropout_kernel<float>, dim3(grid_for(total4)), dim3(256), 0, st, (const float*)x, (float*)y,
                       total4, p, seed, thr);
  DLLM_CHECK_LAUNCH();
  return 0;
}

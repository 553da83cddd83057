// GELU activations with their derivatives for GEMM epilogues (csrc/gemm_fused.hip, csrc/gemm_w4.hip).
#pragma once
#include "common.h"

namespace dllm_gelu {

constexpr float kInvSqrt2 = 0.7071067811865476f;
constexpr float kInvSqrt2Pi = 0.3989422804014327f;
constexpr float kSqrt2OverPi = 0.7978845608028654f;

// GELU and its derivative from ONE exp and ONE reciprocal: erf by Abramowitz-Stegun 7.1.26 (|error| <= 1.5e-7, far
// below bf16 output rounding), whose exp(-x^2) at x = u / sqrt(2) is exactly the exp(-u^2 / 2) of the Gaussian density
// in the derivative.  libm erff + expf cost ~40 VALU instructions per element, a large share of the GEMM itself.
DLLM_DEVICE void gelu_pair(float u, float& g, float& dg) {
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f * kInvSqrt2, fabsf(u), 1.f));
  const float poly =
      fmaf(fmaf(fmaf(fmaf(1.061405429f, t, -1.453152027f), t, 1.421413741f), t, -0.284496736f), t, 0.254829592f) * t;
  const float e = __builtin_amdgcn_exp2f(u * u * (-0.5f * 1.4426950408889634f));  // exp(-u^2 / 2)
  const float cdf = fmaf(0.5f, copysignf(fmaf(-poly, e, 1.f), u), 0.5f);         // Phi(u) = (1 + erf(u / sqrt 2)) / 2
  g = u * cdf;
  dg = fmaf(u * kInvSqrt2Pi, e, cdf);
}
// tanh approximation (gelu_new): tanh(z) = 1 - 2 / (exp(2z) + 1), saturating correctly at both ends
DLLM_DEVICE void gelu_tanh_pair(float u, float& g, float& dg) {
  const float u2 = u * u;
  const float z = kSqrt2OverPi * fmaf(0.044715f * u2, u, u);
  const float th = 1.f - 2.f * __builtin_amdgcn_rcpf(__builtin_amdgcn_exp2f(z * (2.f * 1.4426950408889634f)) + 1.f);
  g = 0.5f * u * (1.f + th);
  dg = fmaf(0.5f * u * fmaf(-th, th, 1.f), kSqrt2OverPi * fmaf(3.f * 0.044715f, u2, 1.f), 0.5f * (1.f + th));
}

}  // namespace dllm_gelu

// Split-K slab reduction of the weight-gradient GEMM (gfx950 / MI355X).
//
// The weight gradient dW[out][in] = dY^T X reduces over tokens (10^4..10^5 rows) into a small output, so
// csrc/gemm_w4.hip's weight-gradient mode splits K over workgroups to fill the 256 CUs; each split stores an fp32
// [M][N] slab and this bandwidth-bound pass sums the slabs and accumulates into the gradient (the flat gradient
// buffer of parallel/flat.py: bf16, or fp32 for fp32 gradient accumulation), so no AccumulateGrad kernel runs.
//
// (Round 6: the twelve csrc/gemm.hip weight-gradient kernel variants that the w4 mode replaced as the default in
// round 5 — profiles/r5_wgrad_w4_ab.txt — were deleted; this pass is what remains of the file.)
#include "common.h"

#include <algorithm>

#include "gemm_params.h"

using namespace dllm;

namespace {

// C[m][n] = sum_s ws[s][m][n] (+ C[m][n]), 8 columns per thread (N % 8 == 0); C bf16 or fp32 (TC)
template <typename TC>
__global__ __launch_bounds__(256) void splitk_reduce_kernel(const float* __restrict__ ws, TC* __restrict__ C,
                                                            long ldc, int M, int N, int splits, int beta) {
  const long n8 = (long)M * N / 8;
  const long slab = (long)M * N;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += (long)gridDim.x * blockDim.x) {
    const long e = i * 8;
    const int m = (int)(e / N), n = (int)(e % N);
    f32x4 a = *reinterpret_cast<const f32x4*>(ws + e);
    f32x4 b = *reinterpret_cast<const f32x4*>(ws + e + 4);
    for (int s = 1; s < splits; ++s) {
      a += *reinterpret_cast<const f32x4*>(ws + s * slab + e);
      b += *reinterpret_cast<const f32x4*>(ws + s * slab + e + 4);
    }
    TC* cp = C + (long)m * ldc + n;
    if constexpr (sizeof(TC) == 4) {
      if (beta) {
        a += *reinterpret_cast<const f32x4*>(cp);
        b += *reinterpret_cast<const f32x4*>(cp + 4);
      }
      *reinterpret_cast<f32x4*>(cp) = a;
      *reinterpret_cast<f32x4*>(cp + 4) = b;
    } else {
      if (beta) {
        const u16x8 c = *reinterpret_cast<const u16x8*>(cp);
        a.x += bf2f(c[0]); a.y += bf2f(c[1]); a.z += bf2f(c[2]); a.w += bf2f(c[3]);
        b.x += bf2f(c[4]); b.y += bf2f(c[5]); b.z += bf2f(c[6]); b.w += bf2f(c[7]);
      }
      const u16x8 o = {f2bf(a.x), f2bf(a.y), f2bf(a.z), f2bf(a.w), f2bf(b.x), f2bf(b.y), f2bf(b.z), f2bf(b.w)};
      *reinterpret_cast<u16x8*>(cp) = o;
    }
  }
}

}  // namespace

// C (+)= sum of p.splits fp32 slabs p.ws (the w4 weight-gradient kernel's, csrc/gemm_w4.hip)
extern "C" int dllm_wgrad_reduce(const GemmWgradParams* pp, hipStream_t st) {
  const GemmWgradParams& p = *pp;
  if (p.splits < 2 || p.ws == nullptr || p.N % 8 || p.M <= 0) return -4;
  const long n8 = (long)p.M * p.N / 8;
  const int blocks = (int)std::min<long>((n8 + 255) / 256, 2048);
  if (p.c_f32)
    hipLaunchKernelGGL(splitk_reduce_kernel<float>, dim3(blocks), dim3(256), 0, st, p.ws, (float*)p.C, p.ldc, p.M, p.N,
                       p.splits, p.beta);
  else
    hipLaunchKernelGGL(splitk_reduce_kernel<uint16_t>, dim3(blocks), dim3(256), 0, st, p.ws, (uint16_t*)p.C, p.ldc,
                       p.M, p.N, p.splits, p.beta);
  DLLM_CHECK_LAUNCH();
  return 0;
}

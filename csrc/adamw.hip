// Fused AdamW over the flat parameter space + global gradient L2 norm, for gfx950.
// sq_norm: grid-stride sum of squares (fp32) -> per-block partials -> one final block -> *out.
// adamw:   one pass over (param bf16|fp32, master fp32?, grad, m, v, wd_mask u8?) reading the clip
//          coefficient from device memory (no host sync); decoupled weight decay as torch.optim.AdamW:
//          w *= 1 - lr*wd; m = b1 m + (1-b1) g; v = b2 v + (1-b2) g^2;
//          w -= lr/bc1 * m / (sqrt(v)/sqrt(bc2) + eps).
#include "common.h"

using namespace dllm;

namespace {

template <typename T>
__global__ __launch_bounds__(256) void sq_norm_partial(const T* __restrict__ g, long n4, float* __restrict__ part) {
  __shared__ float red[4];
  float acc = 0.f;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n4; i += (long)gridDim.x * 256) {
    f32x4 v = Elem<T>::load4(g + i * 4);
    acc += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
  }
  acc = block_sum<256>(acc, red);
  if (threadIdx.x == 0) part[blockIdx.x] = acc;
}

__global__ __launch_bounds__(256) void sum_partials(const float* __restrict__ part, int n, float* __restrict__ out) {
  __shared__ float red[4];
  float acc = 0.f;
  for (int i = threadIdx.x; i < n; i += 256) acc += part[i];
  acc = block_sum<256>(acc, red);
  if (threadIdx.x == 0) out[0] = acc;
}

template <typename TP, typename TG, bool MASTER>
__global__ __launch_bounds__(256) void adamw_kernel(TP* __restrict__ param, float* __restrict__ master,
                                                    const TG* __restrict__ grad, float* __restrict__ m,
                                                    float* __restrict__ v, const uint8_t* __restrict__ wd_mask,
                                                    const float* __restrict__ coef_p, long n4, float lr, float b1,
                                                    float b2, float eps, float wd, float step_size,
                                                    float inv_sqrt_bc2) {
  const float coef = coef_p[0];
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n4; i += (long)gridDim.x * 256) {
    const long o = i * 4;
    f32x4 g = Elem<TG>::load4(grad + o) * coef;
    f32x4 w = MASTER ? *reinterpret_cast<const f32x4*>(master + o) : Elem<TP>::load4(param + o);
    f32x4 mm = *reinterpret_cast<const f32x4*>(m + o);
    f32x4 vv = *reinterpret_cast<const f32x4*>(v + o);
    float dec = lr * wd;
    f32x4 decv = f32x4{dec, dec, dec, dec};
    if (wd_mask != nullptr) {
      const uchar4 mk = *reinterpret_cast<const uchar4*>(wd_mask + o);
      decv = f32x4{mk.x ? dec : 0.f, mk.y ? dec : 0.f, mk.z ? dec : 0.f, mk.w ? dec : 0.f};
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      w[k] *= 1.f - decv[k];
      mm[k] = mm[k] + (1.f - b1) * (g[k] - mm[k]);
      vv[k] = b2 * vv[k] + (1.f - b2) * g[k] * g[k];
      const float denom = sqrtf(vv[k]) * inv_sqrt_bc2 + eps;
      w[k] -= step_size * mm[k] / denom;
    }
    *reinterpret_cast<f32x4*>(m + o) = mm;
    *reinterpret_cast<f32x4*>(v + o) = vv;
    if (MASTER) *reinterpret_cast<f32x4*>(master + o) = w;
    Elem<TP>::store4(param + o, w);
  }
}

inline int grid_for(long n4, int cap) {
  long g = (n4 + 255) / 256;
  return (int)(g < cap ? (g > 0 ? g : 1) : cap);
}

}  // namespace

// `part` must hold at least 1024 floats.
extern "C" int dllm_sq_norm(const void* g, long n, float* part, float* out, int is_bf16, hipStream_t st) {
  if (n % 4) return -2;
  const long n4 = n / 4;
  const int G = grid_for(n4, 1024);
  if (is_bf16)
    hipLaunchKernelGGL(sq_norm_partial<uint16_t>, dim3(G), dim3(256), 0, st, (const uint16_t*)g, n4, part);
  else
    hipLaunchKernelGGL(sq_norm_partial<float>, dim3(G), dim3(256), 0, st, (const float*)g, n4, part);
  hipLaunchKernelGGL(sum_partials, dim3(1), dim3(256), 0, st, part, G, out);
  DLLM_CHECK_LAUNCH();
  return 0;
}

extern "C" int dllm_adamw(void* param, float* master, const void* grad, float* m, float* v, const uint8_t* wd_mask,
                          const float* coef, long n, float lr, float b1, float b2, float eps, float wd, float bc1,
                          float bc2, int is_bf16, int grad_f32, hipStream_t st) {
  if (n % 4) return -2;
  const long n4 = n / 4;
  const int G = grid_for(n4, 4096);
  const float step_size = lr / bc1;
  const float inv_sqrt_bc2 = 1.f / sqrtf(bc2);
  if (is_bf16 && grad_f32) {  // bf16 params, fp32 gradients (accumulated across micro-batches in fp32)
    if (master)
      hipLaunchKernelGGL((adamw_kernel<uint16_t, float, true>), dim3(G), dim3(256), 0, st, (uint16_t*)param, master,
                         (const float*)grad, m, v, wd_mask, coef, n4, lr, b1, b2, eps, wd, step_size, inv_sqrt_bc2);
    else
      hipLaunchKernelGGL((adamw_kernel<uint16_t, float, false>), dim3(G), dim3(256), 0, st, (uint16_t*)param, master,
                         (const float*)grad, m, v, wd_mask, coef, n4, lr, b1, b2, eps, wd, step_size, inv_sqrt_bc2);
  } else if (is_bf16) {
    if (master)
      hipLaunchKernelGGL((adamw_kernel<uint16_t, uint16_t, true>), dim3(G), dim3(256), 0, st, (uint16_t*)param,
                         master, (const uint16_t*)grad, m, v, wd_mask, coef, n4, lr, b1, b2, eps, wd, step_size,
                         inv_sqrt_bc2);
    else
      hipLaunchKernelGGL((adamw_kernel<uint16_t, uint16_t, false>), dim3(G), dim3(256), 0, st, (uint16_t*)param,
                         master, (const uint16_t*)grad, m, v, wd_mask, coef, n4, lr, b1, b2, eps, wd, step_size,
                         inv_sqrt_bc2);
  } else {
    if (master)
      hipLaunchKernelGGL((adamw_kernel<float, float, true>), dim3(G), dim3(256), 0, st, (float*)param, master,
                         (const float*)grad, m, v, wd_mask, coef, n4, lr, b1, b2, eps, wd, step_size, inv_sqrt_bc2);
    else
      hipLaunchKernelGGL((adamw_kernel<float, float, false>), dim3(G), dim3(256), 0, st, (float*)param, master,
                         (const float*)grad, m, v, wd_mask, coef, n4, lr, b1, b2, eps, wd, step_size, inv_sqrt_bc2);
  }
  DLLM_CHECK_LAUNCH();
  return 0;
}

// Fused AdamW over the flat parameter space + global gradient L2 norm, for gfx950.
// sq_norm: grid-stride sum of squares (fp32) -> per-block partials -> one final block -> *out.
// adamw:   one pass over (param bf16|fp32, master fp32?, grad, m, v, wd_mask u8?) reading the clip
//          coefficient from device memory (no host sync); decoupled weight decay as torch.optim.AdamW:
//          w *= 1 - lr*wd; m = b1 m + (1-b1) g; v = b2 v + (1-b2) g^2;
//          w -= lr/bc1 * m / (sqrt(v)/sqrt(bc2) + eps).
#include "common.h"
#include <stdlib.h>
#include <type_traits>

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
                                                    float inv_sqrt_bc2, const float* __restrict__ hyper) {
  const float coef = coef_p[0];
  if (hyper != nullptr) {  // graph-replayed steps: lr / bias corrections computed on the device (ops/optim.py)
    lr = hyper[0];
    step_size = hyper[1];
    inv_sqrt_bc2 = hyper[2];
  }
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

// Bandwidth version (n % 8 == 0, the flat buffers are 64-element aligned): 8 elements per thread and iteration, every
// load of both halves issued before any math (two 16-B loads in flight per stream).  It moves 31 B per parameter with
// fp32 gradients and master weights (17 read, 14 written) at ~4.9 TB/s, i.e. HBM-bound; nontemporal access
// (non-temporal loads / stores) measured 1.8x slower (tools/adamw_bench.py, profiles/r2_adamw_bench.jsonl).
template <bool NT, typename T>
DLLM_DEVICE f32x4 ld4_nt(T* p) {
  if constexpr (!NT) {
    return Elem<std::remove_const_t<T>>::load4(p);
  } else if constexpr (sizeof(T) == 4) {
    return __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(p));
  } else {
    typedef __attribute__((ext_vector_type(2))) unsigned int u32x2v;
    const u32x2v r = __builtin_nontemporal_load(reinterpret_cast<const u32x2v*>(p));
    return f32x4{__uint_as_float(r.x << 16), __uint_as_float(r.x & 0xFFFF0000u), __uint_as_float(r.y << 16),
                 __uint_as_float(r.y & 0xFFFF0000u)};
  }
}
template <bool NT, typename T>
DLLM_DEVICE void st4_nt(T* p, f32x4 v) {
  if constexpr (!NT) {
    Elem<T>::store4(p, v);
  } else if constexpr (sizeof(T) == 4) {
    __builtin_nontemporal_store(v, reinterpret_cast<f32x4*>(p));
  } else {
    typedef __attribute__((ext_vector_type(2))) unsigned int u32x2v;
    const u32x2v r = {pack_bf16x2(v.x, v.y), pack_bf16x2(v.z, v.w)};
    __builtin_nontemporal_store(r, reinterpret_cast<u32x2v*>(p));
  }
}

template <typename TP, typename TG, bool MASTER, bool NT>
__global__ __launch_bounds__(256) void adamw8_kernel(TP* __restrict__ param, float* __restrict__ master,
                                                     const TG* __restrict__ grad, float* __restrict__ m,
                                                     float* __restrict__ v, const uint8_t* __restrict__ wd_mask,
                                                     const float* __restrict__ coef_p, long n8, float lr, float b1,
                                                     float b2, float eps, float wd, float step_size,
                                                     float inv_sqrt_bc2, const float* __restrict__ hyper) {
  const float coef = coef_p[0];
  if (hyper != nullptr) {  // graph-replayed steps: lr / bias corrections computed on the device (ops/optim.py)
    lr = hyper[0];
    step_size = hyper[1];
    inv_sqrt_bc2 = hyper[2];
  }
  const float dec = lr * wd;
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n8; i += (long)gridDim.x * 256) {
    const long o = i * 8;
    f32x4 g[2], w[2], mm[2], vv[2];
    uint2 mk = {0x01010101u, 0x01010101u};
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      g[h] = ld4_nt<NT>(grad + o + 4 * h);
      w[h] = MASTER ? ld4_nt<NT>(master + o + 4 * h) : ld4_nt<NT>(param + o + 4 * h);
      mm[h] = ld4_nt<NT>(m + o + 4 * h);
      vv[h] = ld4_nt<NT>(v + o + 4 * h);
    }
    if (wd_mask != nullptr) mk = *reinterpret_cast<const uint2*>(wd_mask + o);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const uint32_t mw = h == 0 ? mk.x : mk.y;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float gk = g[h][k] * coef;
        const float d = ((mw >> (8 * k)) & 0xFFu) ? dec : 0.f;
        float wk = w[h][k] * (1.f - d);
        const float mk2 = mm[h][k] + (1.f - b1) * (gk - mm[h][k]);
        const float vk = b2 * vv[h][k] + (1.f - b2) * gk * gk;
        wk -= step_size * mk2 / (sqrtf(vk) * inv_sqrt_bc2 + eps);
        w[h][k] = wk;
        mm[h][k] = mk2;
        vv[h][k] = vk;
      }
    }
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      st4_nt<NT>(m + o + 4 * h, mm[h]);
      st4_nt<NT>(v + o + 4 * h, vv[h]);
      if (MASTER) st4_nt<NT>(master + o + 4 * h, w[h]);
      st4_nt<NT>(param + o + 4 * h, w[h]);
    }
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
                          float bc2, int is_bf16, int grad_f32, const float* hyper, hipStream_t st) {
  if (n % 4) return -2;
  const long n4 = n / 4;
  const int G = grid_for(n4, 4096);
  const float step_size = lr / bc1;
  const float inv_sqrt_bc2 = 1.f / sqrtf(bc2);
  if (n % 8 == 0) {
    const long n8 = n / 8;
    const int G8 = grid_for(n8, 1024);  // tools/adamw_bench.py: ~4.9 TB/s moved (non-temporal stores: 2.8, slower)
#define A8(TP, TG, MS)                                                                                                  \
  hipLaunchKernelGGL((adamw8_kernel<TP, TG, MS, false>), dim3(G8), dim3(256), 0, st, (TP*)param, master,               \
                     (const TG*)grad, m, v, wd_mask, coef, n8, lr, b1, b2, eps, wd, step_size, inv_sqrt_bc2, hyper)
    if (is_bf16 && grad_f32) { if (master) A8(uint16_t, float, true); else A8(uint16_t, float, false); }
    else if (is_bf16) { if (master) A8(uint16_t, uint16_t, true); else A8(uint16_t, uint16_t, false); }
    else { if (master) A8(float, float, true); else A8(float, float, false); }
#undef A8
    DLLM_CHECK_LAUNCH();
    return 0;
  }
  if (is_bf16 && grad_f32) {  // bf16 params, fp32 gradients (accumulated across micro-batches in fp32)
    if (master)
      hipLaunchKernelGGL((adamw_kernel<uint16_t, float, true>), dim3(G), dim3(256), 0, st, (uint16_t*)param, master,
                         (const float*)grad, m, v, wd_mask, coef, n4, lr, b1, b2, eps, wd, step_size, inv_sqrt_bc2, hyper);
    else
      hipLaunchKernelGGL((adamw_kernel<uint16_t, float, false>), dim3(G), dim3(256), 0, st, (uint16_t*)param, master,
                         (const float*)grad, m, v, wd_mask, coef, n4, lr, b1, b2, eps, wd, step_size, inv_sqrt_bc2, hyper);
  } else if (is_bf16) {
    if (master)
      hipLaunchKernelGGL((adamw_kernel<uint16_t, uint16_t, true>), dim3(G), dim3(256), 0, st, (uint16_t*)param,
                         master, (const uint16_t*)grad, m, v, wd_mask, coef, n4, lr, b1, b2, eps, wd, step_size,
                         inv_sqrt_bc2, hyper);
    else
      hipLaunchKernelGGL((adamw_kernel<uint16_t, uint16_t, false>), dim3(G), dim3(256), 0, st, (uint16_t*)param,
                         master, (const uint16_t*)grad, m, v, wd_mask, coef, n4, lr, b1, b2, eps, wd, step_size,
                         inv_sqrt_bc2, hyper);
  } else {
    if (master)
      hipLaunchKernelGGL((adamw_kernel<float, float, true>), dim3(G), dim3(256), 0, st, (float*)param, master,
                         (const float*)grad, m, v, wd_mask, coef, n4, lr, b1, b2, eps, wd, step_size, inv_sqrt_bc2, hyper);
    else
      hipLaunchKernelGGL((adamw_kernel<float, float, false>), dim3(G), dim3(256), 0, st, (float*)param, master,
                         (const float*)grad, m, v, wd_mask, coef, n4, lr, b1, b2, eps, wd, step_size, inv_sqrt_bc2, hyper);
  }
  DLLM_CHECK_LAUNCH();
  return 0;
}

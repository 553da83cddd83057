// Fused (label-smoothed) cross-entropy on LM-head logits, for gfx950.
// fwd: one 256-thread block per row: online max/sum-exp over V (fp32 math on bf16 logits, optional
//      additive fp32 bias = BART final_logits_bias), writes loss_row and lse.
//      loss = lse - (1-eps)*x_y - eps*mean_v(x_v);  ignored rows (label == ignore_index) -> 0.
// bwd: dx_v = g * (exp(x_v - lse) - eps/V - (1-eps)*[v==y]) with g = *scale (device scalar, no host
//      sync), written as bf16 — optionally in place over the logits (the only consumer).
#include "common.h"

using namespace dllm;

namespace {

// Rows of any length V: row r starts at logits + r * V, 16-B aligned only when V is a multiple of 16 / sizeof(T)
// (BART's V = 50265 is odd).  Each row is walked as a scalar head up to the first 16-B boundary, 16-B vectors (8 bf16
// or 4 fp32 per thread and step: one global_load_dwordx4), and a scalar tail — every row at the vector rate whatever
// its alignment (an odd V with element-wise loads ran at 1.5-2.3 TB/s on bart-large 1024/1024, r5 profile).
template <typename T>
DLLM_DEVICE int row_head(const T* p, int V) {
  const int mis = (int)(reinterpret_cast<uintptr_t>(p) & 15);
  return min(V, ((16 - mis) & 15) / (int)sizeof(T));
}

template <typename T>
struct Vec16 {
  static constexpr int N = 16 / (int)sizeof(T);
  DLLM_DEVICE static void load(const T* p, float (&v)[16 / sizeof(T)]) {
    if constexpr (sizeof(T) == 2) {
      const u16x8 u = *reinterpret_cast<const u16x8*>(p);
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] = bf2f(u[k]);
    } else {
      const f32x4 u = *reinterpret_cast<const f32x4*>(p);
#pragma unroll
      for (int k = 0; k < 4; ++k) v[k] = u[k];
    }
  }
  DLLM_DEVICE static void store(T* p, const float (&v)[16 / sizeof(T)]) {
    if constexpr (sizeof(T) == 2) {
      u16x8 u;
#pragma unroll
      for (int k = 0; k < 8; ++k) u[k] = f2bf(v[k]);
      *reinterpret_cast<u16x8*>(p) = u;
    } else {
      *reinterpret_cast<f32x4*>(p) = f32x4{v[0], v[1], v[2], v[3]};
    }
  }
};

template <typename T>
__global__ __launch_bounds__(256) void ce_fwd_kernel(const T* __restrict__ logits, const int64_t* __restrict__ labels,
                                                     const float* __restrict__ bias, float* __restrict__ loss_out,
                                                     float* __restrict__ lse_out, int V, float eps, long ignore) {
  __shared__ float red[4];
  constexpr int E = Vec16<T>::N;
  const long row = blockIdx.x;
  const T* x = logits + row * (long)V;
  float m = -INFINITY, s = 0.f, sx = 0.f;
  auto add1 = [&](float v) {
    const float nm = fmaxf(m, v);
    if (nm != -INFINITY) {
      s = (m == -INFINITY ? 0.f : s * __expf(m - nm)) + __expf(v - nm);
      m = nm;
    }
    sx += v;
  };
  const int head = row_head(x, V);
  const int nvec = (V - head) / E;
  const int body_end = head + nvec * E;
  if ((int)threadIdx.x < head) add1(Elem<T>::load(x + threadIdx.x) + (bias != nullptr ? bias[threadIdx.x] : 0.f));
  for (int c = head + (int)threadIdx.x * E; c < body_end; c += 256 * E) {
    float v[E];
    Vec16<T>::load(x + c, v);
    if (bias != nullptr) {
#pragma unroll
      for (int k = 0; k < E; ++k) v[k] += bias[c + k];
    }
    float lm = v[0];
#pragma unroll
    for (int k = 1; k < E; ++k) lm = fmaxf(lm, v[k]);
    const float nm = fmaxf(m, lm);
    if (nm != -INFINITY) {
      float e = 0.f;
#pragma unroll
      for (int k = 0; k < E; ++k) e += __expf(v[k] - nm);
      s = (m == -INFINITY ? 0.f : s * __expf(m - nm)) + e;
      m = nm;
    }
#pragma unroll
    for (int k = 0; k < E; ++k) sx += v[k];
  }
  for (int c = body_end + (int)threadIdx.x; c < V; c += 256)
    add1(Elem<T>::load(x + c) + (bias != nullptr ? bias[c] : 0.f));
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

template <typename T>
__global__ __launch_bounds__(256) void ce_bwd_kernel(const float* __restrict__ scale, const T* __restrict__ logits,
                                                     const int64_t* __restrict__ labels,
                                                     const float* __restrict__ lse_in, const float* __restrict__ bias,
                                                     T* __restrict__ dlogits, int V, float eps, long ignore) {
  constexpr int E = Vec16<T>::N;
  const long row = blockIdx.x;
  const T* x = logits + row * (long)V;
  T* dx = dlogits + row * (long)V;
  const long y = labels[row];
  const bool valid = (y != ignore && y >= 0 && y < V);
  const float g = valid ? scale[0] : 0.f;
  const float lse = lse_in[row];
  const float off = eps / (float)V;
  const float hit = 1.f - eps;
  auto one = [&](int c) {
    const float v = Elem<T>::load(x + c) + (bias != nullptr ? bias[c] : 0.f);
    Elem<T>::store(dx + c, g * (__expf(v - lse) - off - (c == y ? hit : 0.f)));
  };
  // vector body only when input and output rows share their 16-B phase (in place, or equally aligned buffers)
  if (((reinterpret_cast<uintptr_t>(x) ^ reinterpret_cast<uintptr_t>(dx)) & 15) != 0) {
    for (int c = threadIdx.x; c < V; c += 256) one(c);
    return;
  }
  const int head = row_head(x, V);
  const int body_end = head + ((V - head) / E) * E;
  if ((int)threadIdx.x < head) one(threadIdx.x);
  for (int c = head + (int)threadIdx.x * E; c < body_end; c += 256 * E) {
    float v[E];
    Vec16<T>::load(x + c, v);
#pragma unroll
    for (int k = 0; k < E; ++k) {
      const float b = bias != nullptr ? bias[c + k] : 0.f;
      v[k] = g * (__expf(v[k] + b - lse) - off - ((c + k) == y ? hit : 0.f));
    }
    Vec16<T>::store(dx + c, v);
  }
  for (int c = body_end + (int)threadIdx.x; c < V; c += 256) one(c);
}

// bias[c0 + c .. + 3]: one 16-B load when that address is 16-B aligned, else four scalar loads (the ragged vocab tail
// chunk starts at c0 = V - Vc, odd for BART's V = 50265)
DLLM_DEVICE f32x4 bias4(const float* __restrict__ bias, int i) {
  if ((i & 3) == 0) return *reinterpret_cast<const f32x4*>(bias + i);
  return f32x4{bias[i], bias[i + 1], bias[i + 2], bias[i + 3]};
}

// ---- vocab-chunked LM head + CE (ops/lm_head.py): the logits exist one [N, Vc] chunk at a time
// Per row running state st[row] = {max, sum exp(x - max), sum x, x_label} merged over chunks; the last chunk writes
// loss_row and lse.  Chunk columns are global vocab ids c0 .. c0 + Vc - 1; eps / V uses the full vocab size.
__global__ __launch_bounds__(256) void ce_chunk_fwd_kernel(const uint16_t* __restrict__ logits, long ld,
                                                           const int64_t* __restrict__ labels,
                                                           const float* __restrict__ bias, f32x4* __restrict__ st,
                                                           float* __restrict__ loss_out, float* __restrict__ lse_out,
                                                           int Vc, int c0, int V, float eps, long ignore, int first,
                                                           int last, int skip) {
  __shared__ float red[4];
  const long row = blockIdx.x;
  const uint16_t* x = logits + row * ld;
  float m = -INFINITY, s = 0.f, sx = 0.f;
  for (int c = threadIdx.x * 4; c < Vc; c += 256 * 4) {  // Vc % 4 == 0
    f32x4 v = Elem<uint16_t>::load4(x + c);
    if (bias != nullptr) v += bias4(bias, c0 + c);
    if (c < skip) {  // leading columns already covered by the previous chunk (ragged vocab tail)
#pragma unroll
      for (int k = 0; k < 4; ++k) v[k] = c + k < skip ? -INFINITY : v[k];
    }
    const float lm = fmaxf(fmaxf(v.x, v.y), fmaxf(v.z, v.w));
    const float nm = fmaxf(m, lm);
    if (nm != -INFINITY) {
      s = s * __expf(m - nm) + __expf(v.x - nm) + __expf(v.y - nm) + __expf(v.z - nm) + __expf(v.w - nm);
      m = nm;
    }
    if (c < skip) {
#pragma unroll
      for (int k = 0; k < 4; ++k) sx += c + k < skip ? 0.f : v[k];
    } else {
      sx += (v.x + v.y) + (v.z + v.w);
    }
  }
  const float M = block_max<256>(m, red);
  const float scaled = (m == -INFINITY) ? 0.f : s * __expf(m - M);
  const float S = block_sum<256>(scaled, red);
  const float SX = block_sum<256>(sx, red);
  if (threadIdx.x == 0) {
    const long y = labels[row];
    f32x4 cur = first ? f32x4{-INFINITY, 0.f, 0.f, 0.f} : st[row];
    const float nm = fmaxf(cur.x, M);
    cur.y = (cur.x == -INFINITY ? 0.f : cur.y * __expf(cur.x - nm)) + (M == -INFINITY ? 0.f : S * __expf(M - nm));
    cur.x = nm;
    cur.z += SX;
    if (y >= c0 + skip && y < c0 + Vc) cur.w = Elem<uint16_t>::load(x + (y - c0)) + (bias != nullptr ? bias[y] : 0.f);
    st[row] = cur;
    if (last) {
      const float lse = cur.x + __logf(cur.y);
      const bool valid = y != ignore && y >= 0 && y < V;
      loss_out[row] = valid ? lse - (1.f - eps) * cur.w - eps * cur.z / (float)V : 0.f;
      lse_out[row] = lse;
    }
  }
}

// dlogits of one chunk, in place: g * (exp(x - lse) - eps / V - (1 - eps) [c0 + col == y])
__global__ __launch_bounds__(256) void ce_chunk_bwd_kernel(const float* __restrict__ scale, uint16_t* __restrict__ x_io,
                                                           long ld, const int64_t* __restrict__ labels,
                                                           const float* __restrict__ lse_in,
                                                           const float* __restrict__ bias, int Vc, int c0, int V,
                                                           float eps, long ignore, int skip) {
  const long row = blockIdx.x;
  uint16_t* x = x_io + row * ld;
  const long y = labels[row];
  const bool valid = (y != ignore && y >= 0 && y < V);
  const float g = valid ? scale[0] : 0.f;
  const float lse = lse_in[row];
  const float off = eps / (float)V;
  const float hit = 1.f - eps;
  const long yl = y - c0;
  for (int c = threadIdx.x * 4; c < Vc; c += 256 * 4) {
    f32x4 v = Elem<uint16_t>::load4(x + c);
    if (bias != nullptr) v += bias4(bias, c0 + c);
    f32x4 r;
#pragma unroll
    for (int k = 0; k < 4; ++k)
      r[k] = c + k < skip ? 0.f : g * (__expf(v[k] - lse) - off - ((c + k) == yl ? hit : 0.f));
    Elem<uint16_t>::store4(x + c, r);
  }
}

// LM-head CE forward, fused path (ops/lm_head.py): merge the per-(row, 128-column) online-softmax partials the
// W4_EPI_CEF GEMM epilogue wrote (csrc/gemm_w4.hip) into the row's lse and loss.  One wave per row.
__global__ __launch_bounds__(256) void ce_merge_kernel(const f32x4* __restrict__ part, int np, long pstride,
                                                       const float* __restrict__ xlab, const int64_t* __restrict__ labels,
                                                       float* __restrict__ loss_out, float* __restrict__ lse_out, long N,
                                                       int V, float eps, long ignore) {
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= N) return;
  const f32x4* pr = part + row * pstride;
  float m = -INFINITY, s = 0.f, sx = 0.f;
  for (int c = lane; c < np; c += 64) {
    const f32x4 v = pr[c];
    const float nm = fmaxf(m, v.x);
    if (nm != -INFINITY) {
      s = (m == -INFINITY ? 0.f : s * __expf(m - nm)) + (v.x == -INFINITY ? 0.f : v.y * __expf(v.x - nm));
      m = nm;
    }
    sx += v.z;
  }
  const float M = wave_max(m);
  const float S = wave_sum(m == -INFINITY ? 0.f : s * __expf(m - M));
  const float SX = wave_sum(sx);
  if (lane == 0) {
    const long y = labels[row];
    const bool valid = y != ignore && y >= 0 && y < V;
    const float lse = M + __logf(S);
    loss_out[row] = valid ? lse - (1.f - eps) * xlab[row] - eps * SX / (float)V : 0.f;
    lse_out[row] = lse;
  }
}

}  // namespace

extern "C" int dllm_ce_chunk_fwd(const void* logits, long ld, const int64_t* labels, const float* bias, float* state,
                                 float* loss, float* lse, long N, int Vc, int c0, int V, float eps, long ignore,
                                 int first, int last, int skip, hipStream_t st) {
  if (Vc % 4 || ld % 4 || N <= 0 || skip < 0 || skip >= Vc) return -2;
  hipLaunchKernelGGL(ce_chunk_fwd_kernel, dim3(N), dim3(256), 0, st, (const uint16_t*)logits, ld, labels, bias,
                     (f32x4*)state, loss, lse, Vc, c0, V, eps, ignore, first, last, skip);
  DLLM_CHECK_LAUNCH();
  return 0;
}

extern "C" int dllm_ce_chunk_bwd(const float* scale, void* logits, long ld, const int64_t* labels, const float* lse,
                                 const float* bias, long N, int Vc, int c0, int V, float eps, long ignore, int skip,
                                 hipStream_t st) {
  if (Vc % 4 || ld % 4 || N <= 0 || skip < 0 || skip >= Vc) return -2;
  hipLaunchKernelGGL(ce_chunk_bwd_kernel, dim3(N), dim3(256), 0, st, scale, (uint16_t*)logits, ld, labels, lse, bias,
                     Vc, c0, V, eps, ignore, skip);
  DLLM_CHECK_LAUNCH();
  return 0;
}

extern "C" int dllm_ce_fwd(const void* logits, const int64_t* labels, const float* bias, float* loss, float* lse,
                           long N, int V, float eps, long ignore, int is_bf16, hipStream_t st) {
  dim3 g(N), b(256);
  if (is_bf16)
    hipLaunchKernelGGL((ce_fwd_kernel<uint16_t>), g, b, 0, st, (const uint16_t*)logits, labels, bias, loss, lse, V, eps,
                       ignore);
  else
    hipLaunchKernelGGL((ce_fwd_kernel<float>), g, b, 0, st, (const float*)logits, labels, bias, loss, lse, V, eps, ignore);
  DLLM_CHECK_LAUNCH();
  return 0;
}

extern "C" int dllm_ce_bwd(const float* scale, const void* logits, const int64_t* labels, const float* lse,
                           const float* bias, void* dlogits, long N, int V, float eps, long ignore, int is_bf16,
                           hipStream_t st) {
  dim3 g(N), b(256);
  if (is_bf16)
    hipLaunchKernelGGL((ce_bwd_kernel<uint16_t>), g, b, 0, st, scale, (const uint16_t*)logits, labels, lse, bias,
                       (uint16_t*)dlogits, V, eps, ignore);
  else
    hipLaunchKernelGGL((ce_bwd_kernel<float>), g, b, 0, st, scale, (const float*)logits, labels, lse, bias,
                       (float*)dlogits, V, eps, ignore);
  DLLM_CHECK_LAUNCH();
  return 0;
}

extern "C" int dllm_ce_merge(const float* part, int np, long pstride, const float* xlab, const int64_t* labels,
                             float* loss, float* lse, long N, int V, float eps, long ignore, hipStream_t st) {
  if (N <= 0 || np <= 0 || pstride < np) return -2;
  hipLaunchKernelGGL(ce_merge_kernel, dim3((unsigned)((N + 3) / 4)), dim3(256), 0, st, (const f32x4*)part, np, pstride,
                     xlab, labels, loss, lse, N, V, eps, ignore);
  DLLM_CHECK_LAUNCH();
  return 0;
}

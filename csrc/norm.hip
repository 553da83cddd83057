// Fused (residual + dropout +) RMSNorm / LayerNorm, forward and backward, for gfx950.
//
// One wave64 owns one row; the row stays in registers (up to MAXV*256 columns, 4 elements / lane /
// chunk, 8-byte bf16 vector loads) so the residual stream is read once and written once.
// fwd:  s = (resid) + dropout(x)          [stored if resid or dropout]
//       out = norm(s) * w (+ b)            [RMS: T5 (fp32 variance, weight only); LN: BART]
// bwd:  ds = norm_bwd(dout) + ds_extra     [ds_extra = gradient of the stream from later layers]
//       dx = dropout_bwd(ds);  dstream = ds (optional);  dw/db via per-block column partials.
// Dropout keep-decision for element row*d + col: common.h dropout4 / ops/rng.py keep_mask.
#include "common.h"

#include <cstdlib>

using namespace dllm;

DLLM_SEED_STEP_TU(norm)

namespace {

template <typename T, int KIND, int MAXV>
__global__ __launch_bounds__(256) void norm_fwd_kernel(const T* __restrict__ x, const T* __restrict__ resid,
                                                       const T* __restrict__ w, const T* __restrict__ b,
                                                       T* __restrict__ out, T* __restrict__ s_out,
                                                       float* __restrict__ mean_out, float* __restrict__ rstd_out,
                                                       int N, int d, float eps, float p, uint32_t seed,
                                                       uint32_t thr) {
  if (p > 0.f) seed = eff_seed(seed);
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= N) return;
  const size_t base = (size_t)row * d;
  const bool drop = p > 0.f;
  const float dscale = drop ? 1.f / (1.f - p) : 1.f;
  f32x4 v[MAXV];
  float sum = 0.f;
#pragma unroll
  for (int c = 0; c < MAXV; ++c) {
    const int col = (c * 64 + lane) * 4;
    v[c] = f32x4{0.f, 0.f, 0.f, 0.f};
    if (col < d) {
      f32x4 xv = Elem<T>::load4(x + base + col);
      if (drop) dropout4(xv, seed, thr, (uint32_t)(base + col), dscale);
      if (resid != nullptr) {
        f32x4 rv = Elem<T>::load4(resid + base + col);
        xv += rv;
      }
      if (s_out != nullptr) {
        Elem<T>::store4(s_out + base + col, xv);
#pragma unroll
        for (int k = 0; k < 4; ++k) xv[k] = Elem<T>::round(xv[k]);
      }
      v[c] = xv;
      sum += xv.x + xv.y + xv.z + xv.w;
    }
  }
  float mean = 0.f;
  if (KIND == 1) mean = wave_sum(sum) / (float)d;
  float sq = 0.f;
#pragma unroll
  for (int c = 0; c < MAXV; ++c) {
    const int col = (c * 64 + lane) * 4;
    if (col < d) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float t = v[c][k] - mean;
        sq += t * t;
      }
    }
  }
  const float rstd = rsqrtf(wave_sum(sq) / (float)d + eps);
#pragma unroll
  for (int c = 0; c < MAXV; ++c) {
    const int col = (c * 64 + lane) * 4;
    if (col < d) {
      f32x4 wv = Elem<T>::load4(w + col);
      f32x4 o = (v[c] - mean) * rstd * wv;
      if (KIND == 1 && b != nullptr) o += Elem<T>::load4(b + col);
      Elem<T>::store4(out + base + col, o);
    }
  }
  if (lane == 0) {
    rstd_out[row] = rstd;
    if (KIND == 1) mean_out[row] = mean;
  }
}

// Latency-bound at one row per wave (3 TB/s measured on the t5-base shapes): each wave now takes two rows per
// iteration (d <= 1024) with every load of both rows (s, dout, ds_extra) issued before the first reduction, the weight row
// hoisted out of the loop, and out-of-range columns / the missing second row read a clamped address and are
// zeroed instead of branched around, so the body stays straight-line.
template <typename T, int KIND, int MAXV, bool EX>
__global__ __launch_bounds__(256) void norm_bwd_kernel(const T* __restrict__ dout, const T* __restrict__ ds_extra,
                                                       const T* __restrict__ s, const T* __restrict__ w,
                                                       const float* __restrict__ mean_in,
                                                       const float* __restrict__ rstd_in, T* __restrict__ dx,
                                                       T* __restrict__ dstream, float* __restrict__ dw_part,
                                                       float* __restrict__ db_part, float* __restrict__ dxs_part,
                                                       int N, int d, float p, uint32_t seed, uint32_t thr) {
  if (p > 0.f) seed = eff_seed(seed);
  extern __shared__ __attribute__((aligned(16))) float red[];  // [4][d]
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const bool drop = p > 0.f;
  const float dscale = drop ? 1.f / (1.f - p) : 1.f;
  // adx: column sums of the stored dx (dxs_part != nullptr) — the bias gradient of the linear layer whose output fed
  // this norm's x (BART post-LN: out_proj / fc2), so that layer's backward needs no separate column-sum pass over dx
  f32x4 adw[MAXV], adb[MAXV], adx[MAXV], wgt[MAXV];
  int cof[MAXV];
  float cm[MAXV];  // 1 for a column chunk inside the row, else 0
#pragma unroll
  for (int c = 0; c < MAXV; ++c) {
    const int col = (c * 64 + lane) * 4;
    cm[c] = col < d ? 1.f : 0.f;
    cof[c] = col < d ? col : 0;
    wgt[c] = Elem<T>::load4(w + cof[c]) * cm[c];
    adw[c] = adb[c] = adx[c] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  constexpr int R = MAXV <= 4 ? 2 : 1;  // rows per iteration (registers: d = 2048 stays at one row)
  const int stride = gridDim.x * 4;
  for (int row = blockIdx.x * 4 + wv; row < N; row += R * stride) {
    const bool two = R == 2 && row + stride < N;
    const int rr[2] = {row, two ? row + stride : row};
    f32x4 sv[R][MAXV], dy[R][MAXV], ex[R][MAXV];
#pragma unroll
    for (int u = 0; u < R; ++u) {
      const size_t base = (size_t)rr[u] * d;
#pragma unroll
      for (int c = 0; c < MAXV; ++c) {
        sv[u][c] = Elem<T>::load4(s + base + cof[c]);
        dy[u][c] = Elem<T>::load4(dout + base + cof[c]);
        if (EX) ex[u][c] = Elem<T>::load4(ds_extra + base + cof[c]);
      }
    }
    float rs[R], s1[R], s2[R];
    f32x4 xh[R][MAXV], g[R][MAXV];
#pragma unroll
    for (int u = 0; u < R; ++u) {
      rs[u] = rstd_in[rr[u]];
      const float mean = KIND == 1 ? mean_in[rr[u]] : 0.f;
      const float live = (u == 0 || two) ? 1.f : 0.f;  // the duplicated row of an odd tail adds nothing
      float a1 = 0.f, a2 = 0.f;
#pragma unroll
      for (int c = 0; c < MAXV; ++c) {
        xh[u][c] = (sv[u][c] - mean) * rs[u];
        const f32x4 dyv = dy[u][c] * (cm[c] * live);
        g[u][c] = dyv * wgt[c];
        adw[c] += dyv * xh[u][c];
        adb[c] += dyv;
        a1 += g[u][c].x + g[u][c].y + g[u][c].z + g[u][c].w;
        const f32x4 gx = g[u][c] * xh[u][c];
        a2 += gx.x + gx.y + gx.z + gx.w;
      }
      s1[u] = a1;
      s2[u] = a2;
    }
#pragma unroll
    for (int u = 0; u < R; ++u) {
      s2[u] = wave_sum(s2[u]) / (float)d;
      s1[u] = KIND == 1 ? wave_sum(s1[u]) / (float)d : 0.f;
    }
#pragma unroll
    for (int u = 0; u < R; ++u) {
      if (u == 1 && !two) break;
      const size_t base = (size_t)rr[u] * d;
#pragma unroll
      for (int c = 0; c < MAXV; ++c) {
        const int col = (c * 64 + lane) * 4;
        if (col < d) {
          f32x4 dsv = (g[u][c] - s1[u] - xh[u][c] * s2[u]) * rs[u];
          if (EX) dsv += ex[u][c];
          if (dstream != nullptr) Elem<T>::store4(dstream + base + col, dsv);
          if (drop) dropout4(dsv, seed, thr, (uint32_t)(base + col), dscale);
          Elem<T>::store4(dx + base + col, dsv);
          if (dxs_part != nullptr) adx[c] += dsv;
        }
      }
    }
  }
  // block-reduce the column partials of the 4 waves, one pass each for dw, db (if any), dx column sums (if asked)
  for (int pass = 0; pass < 3; ++pass) {
    if ((pass == 1 && db_part == nullptr) || (pass == 2 && dxs_part == nullptr)) continue;
    __syncthreads();
#pragma unroll
    for (int c = 0; c < MAXV; ++c) {
      const int col = (c * 64 + lane) * 4;
      if (col < d) *reinterpret_cast<f32x4*>(red + wv * d + col) = pass == 0 ? adw[c] : (pass == 1 ? adb[c] : adx[c]);
    }
    __syncthreads();
    float* dst = (pass == 0 ? dw_part : (pass == 1 ? db_part : dxs_part)) + (size_t)blockIdx.x * d;
    for (int col = threadIdx.x; col < d; col += 256) dst[col] = red[col] + red[d + col] + red[2 * d + col] + red[3 * d + col];
  }
}

// out[col] += sum over a chunk of partial rows; grid (ceil(d/64), row-chunks), 4 waves split the chunk,
// lane = column (256-B coalesced rows), LDS combine, one fp32 atomic per column per block (out pre-zeroed).
constexpr int kColChunks = 16;
__global__ __launch_bounds__(256) void col_sum_kernel(const float* __restrict__ part, float* __restrict__ out, int G,
                                                      int d) {
  __shared__ float red[4][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int col = blockIdx.x * 64 + lane;
  const int per = (G + gridDim.y - 1) / gridDim.y;
  const int g0 = blockIdx.y * per;
  const int g1 = g0 + per < G ? g0 + per : G;
  float acc = 0.f;
  if (col < d)
    for (int g = g0 + w; g < g1; g += 4) acc += part[(size_t)g * d + col];
  red[w][lane] = acc;
  __syncthreads();
  if (w == 0 && col < d) atomicAdd(out + col, red[0][lane] + red[1][lane] + red[2][lane] + red[3][lane]);
}

// out[col] (+)= sum over ALL partial rows, stored in the parameter dtype: accumulates a norm weight/bias
// gradient straight into its slice of the flat gradient buffer (no zero-fill, atomics, cast, or add kernel)
template <typename T>
__global__ __launch_bounds__(1024) void col_sum_acc_kernel(const float* __restrict__ part, T* __restrict__ out, int G,
                                                           int d) {
  // 16 waves x 64 columns; each wave sums rows w, w+16, ... with 8 independent loads in flight
  __shared__ float red[16][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int col = blockIdx.x * 64 + lane;
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (col < d) {
    int g = w;
    for (; g + 16 * 7 < G; g += 16 * 8) {
#pragma unroll
      for (int u = 0; u < 8; ++u) acc[u] += part[(size_t)(g + 16 * u) * d + col];
    }
    for (; g < G; g += 16) acc[0] += part[(size_t)g * d + col];
  }
  red[w][lane] = ((acc[0] + acc[1]) + (acc[2] + acc[3])) + ((acc[4] + acc[5]) + (acc[6] + acc[7]));
  __syncthreads();
  if (w == 0 && col < d) {
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) s += red[i][lane];
    Elem<T>::store(out + col, Elem<T>::load(out + col) + s);
  }
}

template <typename T, int KIND>
int launch_fwd(const void* x, const void* resid, const void* w, const void* b, void* out, void* s_out, float* mean,
               float* rstd, int N, int d, float eps, float p, uint32_t seed, hipStream_t st) {
  const int chunks = (d + 255) / 256;
  dim3 grid((N + 3) / 4), block(256);
  const uint32_t thr = drop_threshold(p);
#define L(MV)                                                                                                     \
  hipLaunchKernelGGL((norm_fwd_kernel<T, KIND, MV>), grid, block, 0, st, (const T*)x, (const T*)resid,           \
                     (const T*)w, (const T*)b, (T*)out, (T*)s_out, mean, rstd, N, d, eps, p, seed, thr)
  if (chunks <= 1) L(1);
  else if (chunks <= 2) L(2);
  else if (chunks <= 3) L(3);
  else if (chunks <= 4) L(4);
  else if (chunks <= 8) L(8);
  else return -1;
#undef L
  DLLM_CHECK_LAUNCH();
  return 0;
}

template <typename T, int KIND>
int launch_bwd(const void* dout, const void* ds_extra, const void* s, const void* w, const float* mean,
               const float* rstd, void* dx, void* dstream, float* dw_part, float* db_part, float* dw, float* db,
               void* dw_acc, void* db_acc, float* dxs_part, float* dxs, int N, int d, float p, uint32_t seed, int G,
               int acc_f32, hipStream_t st) {
  const int chunks = (d + 255) / 256;
  dim3 grid(G), block(256);
  const size_t lds = (size_t)4 * d * sizeof(float);
  const uint32_t thr = drop_threshold(p);
#define L(MV)                                                                                                     \
  do {                                                                                                            \
    if (ds_extra != nullptr)                                                                                      \
      hipLaunchKernelGGL((norm_bwd_kernel<T, KIND, MV, true>), grid, block, lds, st, (const T*)dout,              \
                         (const T*)ds_extra, (const T*)s, (const T*)w, mean, rstd, (T*)dx, (T*)dstream, dw_part,  \
                         db_part, dxs_part, N, d, p, seed, thr);                                                  \
    else                                                                                                          \
      hipLaunchKernelGGL((norm_bwd_kernel<T, KIND, MV, false>), grid, block, lds, st, (const T*)dout,             \
                         (const T*)ds_extra, (const T*)s, (const T*)w, mean, rstd, (T*)dx, (T*)dstream, dw_part,  \
                         db_part, dxs_part, N, d, p, seed, thr);                                                  \
  } while (0)
  if (chunks <= 1) L(1);
  else if (chunks <= 2) L(2);
  else if (chunks <= 3) L(3);
  else if (chunks <= 4) L(4);
  else if (chunks <= 8) L(8);
  else return -1;
#undef L
  DLLM_CHECK_LAUNCH();
  if (dxs_part != nullptr && dxs != nullptr)  // dx column sums -> dxs (fp32, pre-zeroed); else the caller reduces
    hipLaunchKernelGGL(col_sum_acc_kernel<float>, dim3((d + 63) / 64), dim3(1024), 0, st, dxs_part, dxs, G, d);
  if (dw_acc != nullptr && acc_f32) {  // fp32 flat gradient buffer
    hipLaunchKernelGGL(col_sum_acc_kernel<float>, dim3((d + 63) / 64), dim3(1024), 0, st, dw_part, (float*)dw_acc, G,
                       d);
    if (db_part != nullptr)
      hipLaunchKernelGGL(col_sum_acc_kernel<float>, dim3((d + 63) / 64), dim3(1024), 0, st, db_part, (float*)db_acc,
                         G, d);
  } else if (dw_acc != nullptr) {
    hipLaunchKernelGGL(col_sum_acc_kernel<T>, dim3((d + 63) / 64), dim3(1024), 0, st, dw_part, (T*)dw_acc, G, d);
    if (db_part != nullptr)
      hipLaunchKernelGGL(col_sum_acc_kernel<T>, dim3((d + 63) / 64), dim3(1024), 0, st, db_part, (T*)db_acc, G, d);
  } else if (dw != nullptr) {
    const dim3 cg((d + 63) / 64, kColChunks);
    hipLaunchKernelGGL(col_sum_kernel, cg, dim3(256), 0, st, dw_part, dw, G, d);
    if (db_part != nullptr) hipLaunchKernelGGL(col_sum_kernel, cg, dim3(256), 0, st, db_part, db, G, d);
  }  // neither: the caller keeps the per-block partials (a deferred gradient-accumulation window, ops/gemm.py)
  DLLM_CHECK_LAUNCH();
  return 0;
}

}  // namespace

extern "C" int dllm_norm_fwd(const void* x, const void* resid, const void* w, const void* b, void* out, void* s_out,
                             float* mean, float* rstd, int N, int d, float eps, float p, uint32_t seed, int kind,
                             int is_bf16, hipStream_t st) {
  if (d % 4 != 0) return -2;
  if (is_bf16) {
    return kind ? launch_fwd<uint16_t, 1>(x, resid, w, b, out, s_out, mean, rstd, N, d, eps, p, seed, st)
                : launch_fwd<uint16_t, 0>(x, resid, w, b, out, s_out, mean, rstd, N, d, eps, p, seed, st);
  }
  return kind ? launch_fwd<float, 1>(x, resid, w, b, out, s_out, mean, rstd, N, d, eps, p, seed, st)
              : launch_fwd<float, 0>(x, resid, w, b, out, s_out, mean, rstd, N, d, eps, p, seed, st);
}

// Number of partial rows the caller must allocate for dw_part/db_part: the workgroup cap, 512 = 2 per CU (each wave
// then walks N / 2048 rows, two at a time; other caps measured no better, profiles/r4_norm_bandwidth.txt)
static int norm_bwd_cap() { return 512; }

// out[col] (+)= sum of the G rows of part [G][d] (fp32 partial column sums handed to a bias gradient, ops/gemm.py)
extern "C" int dllm_colsum_partials_acc(const float* part, void* out, int out_is_bf16, int G, int d, hipStream_t st) {
  if (G <= 0 || d <= 0) return -4;
  if (out_is_bf16)
    hipLaunchKernelGGL(col_sum_acc_kernel<uint16_t>, dim3((d + 63) / 64), dim3(1024), 0, st, part, (uint16_t*)out, G, d);
  else
    hipLaunchKernelGGL(col_sum_acc_kernel<float>, dim3((d + 63) / 64), dim3(1024), 0, st, part, (float*)out, G, d);
  DLLM_CHECK_LAUNCH();
  return 0;
}

extern "C" int dllm_norm_bwd_grid(int N) {
  const int g = (N + 3) / 4, cap = norm_bwd_cap();
  return g < cap ? g : cap;
}

extern "C" int dllm_norm_bwd(const void* dout, const void* ds_extra, const void* s, const void* w, const float* mean,
                             const float* rstd, void* dx, void* dstream, float* dw_part, float* db_part, float* dw,
                             float* db, void* dw_acc, void* db_acc, float* dxs_part, float* dxs, int N, int d, float p,
                             uint32_t seed, int kind, int is_bf16, int acc_f32, hipStream_t st) {
  if (d % 4 != 0) return -2;
  const int G = dllm_norm_bwd_grid(N);
#define A dout, ds_extra, s, w, mean, rstd, dx, dstream, dw_part, db_part, dw, db, dw_acc, db_acc, dxs_part, dxs, N, d, p, \
          seed, G, acc_f32, st
  if (is_bf16) return kind ? launch_bwd<uint16_t, 1>(A) : launch_bwd<uint16_t, 0>(A);
  return kind ? launch_bwd<float, 1>(A) : launch_bwd<float, 0>(A);
#undef A
}

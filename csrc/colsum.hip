// Column sums of a token-major bf16 matrix, accumulated into a parameter gradient: the bias gradient of a
// linear layer (db = sum over tokens of dY).  torch's generic reduction needs ~31 us per BART-large bias
// (profiles/r1_bart_large_b32_prof18_summary.txt, plus a separate add into the flat gradient buffer);
// here: pass 1 = grid (N/512 column blocks, R row chunks), each lane sums 8 adjacent columns over its
// rows (16-B loads, 1-KB coalesced rows per wave, 2 independent accumulator sets), fp32 partials [R][N];
// pass 2 = 16 waves per 64 columns sum the R partials (independent loads, fixed order) and add into the gradient.
#include "common.h"

using namespace dllm;

namespace {

constexpr int kRowChunks = 256;  // most row chunks (the caller's scratch is kRowChunks x N floats)

// pass 1: a lane sums 8 adjacent columns (one 16-B load per row) over the rows of its chunk, 2 independent
// accumulator sets; a wave covers 512 columns of one row per load (1 KB coalesced), the block's 4 waves interleave
// rows.  VEC = false: 2 columns per lane (rows only 4-B aligned / N not a multiple of 8).
template <bool VEC>
__global__ __launch_bounds__(256) void colsum_partial_kernel(const uint16_t* __restrict__ x, long ld, long T, int N,
                                                             float* __restrict__ part) {
  constexpr int CPL = VEC ? 8 : 2;       // columns per lane
  constexpr int CPB = 64 * CPL;          // columns per block
  __shared__ float red[4][CPB];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c = blockIdx.x * CPB + CPL * lane;
  const long per = (T + gridDim.y - 1) / gridDim.y;
  const long r0 = (long)blockIdx.y * per;
  const long r1 = r0 + per < T ? r0 + per : T;
  float a0[CPL], a1[CPL];
#pragma unroll
  for (int k = 0; k < CPL; ++k) a0[k] = a1[k] = 0.f;
  if (c < N) {
    long r = r0 + w;
    for (; r + 4 < r1; r += 8) {
      if constexpr (VEC) {
        const u16x8 v0 = *reinterpret_cast<const u16x8*>(x + r * ld + c);
        const u16x8 v1 = *reinterpret_cast<const u16x8*>(x + (r + 4) * ld + c);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          a0[k] += bf2f(v0[k]);
          a1[k] += bf2f(v1[k]);
        }
      } else {
        const uint32_t v0 = *reinterpret_cast<const uint32_t*>(x + r * ld + c);
        const uint32_t v1 = *reinterpret_cast<const uint32_t*>(x + (r + 4) * ld + c);
        a0[0] += bf2f((uint16_t)(v0 & 0xFFFFu));
        a0[1] += bf2f((uint16_t)(v0 >> 16));
        a1[0] += bf2f((uint16_t)(v1 & 0xFFFFu));
        a1[1] += bf2f((uint16_t)(v1 >> 16));
      }
    }
    for (; r < r1; r += 4) {
      if constexpr (VEC) {
        const u16x8 v0 = *reinterpret_cast<const u16x8*>(x + r * ld + c);
#pragma unroll
        for (int k = 0; k < 8; ++k) a0[k] += bf2f(v0[k]);
      } else {
        const uint32_t v0 = *reinterpret_cast<const uint32_t*>(x + r * ld + c);
        a0[0] += bf2f((uint16_t)(v0 & 0xFFFFu));
        a0[1] += bf2f((uint16_t)(v0 >> 16));
      }
    }
  }
#pragma unroll
  for (int k = 0; k < CPL; ++k) red[w][CPL * lane + k] = a0[k] + a1[k];
  __syncthreads();
  for (int i = threadIdx.x; i < CPB; i += 256) {
    const int col = blockIdx.x * CPB + i;
    if (col < N) part[(long)blockIdx.y * N + col] = (red[0][i] + red[1][i]) + (red[2][i] + red[3][i]);
  }
}

// pass 2: 64 columns per 1024-thread block; wave w sums partial rows w, w + 16, ... (independent loads, 8 in flight)
// and the 16 wave sums are added in a fixed order (deterministic)
template <typename T>
__global__ __launch_bounds__(1024) void colsum_finish_kernel(const float* __restrict__ part, int R, int N,
                                                            T* __restrict__ out) {
  __shared__ float red[16][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int col = blockIdx.x * 64 + lane;
  float acc = 0.f;
  if (col < N) {
    int g = w;
    for (; g + 7 * 16 < R; g += 8 * 16) {
      float v[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] = part[(long)(g + 16 * k) * N + col];
#pragma unroll
      for (int k = 0; k < 8; ++k) acc += v[k];
    }
    for (; g < R; g += 16) acc += part[(long)g * N + col];
  }
  red[w][lane] = acc;
  __syncthreads();
  if (w == 0 && col < N) {
    float t = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) t += red[k][lane];
    Elem<T>::store(out + col, Elem<T>::load(out + col) + t);
  }
}

}  // namespace

extern "C" int dllm_colsum_rows() { return kRowChunks; }

// out[n] += sum_t x[t][n]; x bf16 [T][ld] (N <= ld, N even, rows 4-B aligned), part fp32 [R][N] scratch
extern "C" int dllm_colsum_acc(const void* x, long ld, long T, int N, float* part, void* out, int out_is_bf16,
                               hipStream_t st) {
  if (N <= 0 || T <= 0 || (N & 1) || (ld & 1)) return -2;
  const bool vec = (N % 8) == 0 && (ld % 8) == 0 && ((uintptr_t)x % 16) == 0;
  // ~1024 blocks in flight for the HBM stream (N = 1024 has only 2 column blocks of 512), chunks of >= 32 rows
  const int cblk = vec ? (N + 511) / 512 : (N + 127) / 128;
  long R = 1024 / cblk;
  R = R < 16 ? 16 : (R > kRowChunks ? kRowChunks : R);
  R = R < (T + 31) / 32 ? R : (T + 31) / 32;
  R = R < 1 ? 1 : R;
  if (vec)
    hipLaunchKernelGGL(colsum_partial_kernel<true>, dim3(cblk, (int)R), dim3(256), 0, st, (const uint16_t*)x, ld,
                       T, N, part);
  else
    hipLaunchKernelGGL(colsum_partial_kernel<false>, dim3(cblk, (int)R), dim3(256), 0, st, (const uint16_t*)x,
                       ld, T, N, part);
  DLLM_CHECK_LAUNCH();
  if (out_is_bf16)
    hipLaunchKernelGGL(colsum_finish_kernel<uint16_t>, dim3((N + 63) / 64), dim3(1024), 0, st, part, (int)R, N,
                       (uint16_t*)out);
  else
    hipLaunchKernelGGL(colsum_finish_kernel<float>, dim3((N + 63) / 64), dim3(1024), 0, st, part, (int)R, N, (float*)out);
  DLLM_CHECK_LAUNCH();
  return 0;
}

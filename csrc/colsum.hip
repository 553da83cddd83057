// Column sums of a token-major bf16 matrix, accumulated into a parameter gradient: the bias gradient of a
// linear layer (db = sum over tokens of dY).  torch's generic reduction needs ~31 us per BART-large bias
// (profiles/r1_bart_large_b32_prof18_summary.txt, plus a separate add into the flat gradient buffer);
// here: pass 1 = grid (N/128 column blocks, R row chunks), each lane sums 2 adjacent columns over its
// rows with 4 independent accumulators (bf16x2 loads, 256-B coalesced rows), fp32 partials [R][N];
// pass 2 = one block per 64 columns sums the R partials and adds into the bf16/fp32 gradient in place.
#include "common.h"

using namespace dllm;

namespace {

constexpr int kRowChunks = 64;

__global__ __launch_bounds__(256) void colsum_partial_kernel(const uint16_t* __restrict__ x, long ld, long T, int N,
                                                             float* __restrict__ part) {
  __shared__ float red[4][128];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c = blockIdx.x * 128 + 2 * lane;
  const long per = (T + gridDim.y - 1) / gridDim.y;
  const long r0 = (long)blockIdx.y * per;
  const long r1 = r0 + per < T ? r0 + per : T;
  float a0[4] = {0.f, 0.f, 0.f, 0.f}, a1[4] = {0.f, 0.f, 0.f, 0.f};
  if (c < N) {
    long r = r0 + w;
    for (; r + 12 < r1; r += 16) {
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const uint32_t v = *reinterpret_cast<const uint32_t*>(x + (r + 4 * u) * ld + c);
        a0[u] += bf2f((uint16_t)(v & 0xFFFFu));
        a1[u] += bf2f((uint16_t)(v >> 16));
      }
    }
    for (; r < r1; r += 4) {
      const uint32_t v = *reinterpret_cast<const uint32_t*>(x + r * ld + c);
      a0[0] += bf2f((uint16_t)(v & 0xFFFFu));
      a1[0] += bf2f((uint16_t)(v >> 16));
    }
  }
  red[w][2 * lane] = (a0[0] + a0[1]) + (a0[2] + a0[3]);
  red[w][2 * lane + 1] = (a1[0] + a1[1]) + (a1[2] + a1[3]);
  __syncthreads();
  for (int i = threadIdx.x; i < 128; i += 256) {
    const int col = blockIdx.x * 128 + i;
    if (col < N) part[(long)blockIdx.y * N + col] = red[0][i] + red[1][i] + red[2][i] + red[3][i];
  }
}

template <typename T>
__global__ __launch_bounds__(256) void colsum_finish_kernel(const float* __restrict__ part, int R, int N,
                                                           T* __restrict__ out) {
  __shared__ float red[4][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int col = blockIdx.x * 64 + lane;
  float acc = 0.f;
  if (col < N)
    for (int g = w; g < R; g += 4) acc += part[(long)g * N + col];
  red[w][lane] = acc;
  __syncthreads();
  if (w == 0 && col < N)
    Elem<T>::store(out + col, Elem<T>::load(out + col) + red[0][lane] + red[1][lane] + red[2][lane] + red[3][lane]);
}

}  // namespace

extern "C" int dllm_colsum_rows() { return kRowChunks; }

// out[n] += sum_t x[t][n]; x bf16 [T][ld] (N <= ld, N even, rows 4-B aligned), part fp32 [R][N] scratch
extern "C" int dllm_colsum_acc(const void* x, long ld, long T, int N, float* part, void* out, int out_is_bf16,
                               hipStream_t st) {
  if (N <= 0 || T <= 0 || (N & 1) || (ld & 1)) return -2;
  const int R = (int)(T < kRowChunks ? T : kRowChunks);
  hipLaunchKernelGGL(colsum_partial_kernel, dim3((N + 127) / 128, R), dim3(256), 0, st, (const uint16_t*)x, ld, T, N,
                     part);
  DLLM_CHECK_LAUNCH();
  if (out_is_bf16)
    hipLaunchKernelGGL(colsum_finish_kernel<uint16_t>, dim3((N + 63) / 64), dim3(256), 0, st, part, R, N,
                       (uint16_t*)out);
  else
    hipLaunchKernelGGL(colsum_finish_kernel<float>, dim3((N + 63) / 64), dim3(256), 0, st, part, R, N, (float*)out);
  DLLM_CHECK_LAUNCH();
  return 0;
}

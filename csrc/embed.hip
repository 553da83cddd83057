// Embedding backward for gfx950: deterministic sorted segment-sum straight into the flat gradient buffer.
//
// dW[id] += sum over tokens t with ids[t] == id of dY[t]  (torch nn.Embedding backward, which the reference
// reaches through AutoModelForSeq2SeqLM's shared / positional embeddings).  ATen's version scatters with
// atomics or a sort + per-segment reduce into a fresh [V, d] tensor that AccumulateGrad then adds into the
// gradient; here the token ids are sorted once (torch.sort, rocPRIM radix sort) and the rows of each id are
// summed in sorted order, so the result is bitwise reproducible run to run, and added in place to the
// parameter's slice of the flat gradient buffer (bf16 or fp32).
//
// Sorted positions are cut into fixed 64-row windows, one workgroup each, threads over 8-column chunks
// (16-B loads of each dY row):
//   pass 1 (embed_cont_kernel): a window whose first id continues a run from the window before writes the sum of
//           that continuation into a per-window fp32 slot;
//   pass 2 (embed_bwd_kernel): every run that STARTS in a window is summed by that window's workgroup, which
//           then adds the slots of the following windows while the run continues into them (in order), and
//           accumulates the total into dW[id].  A run of any length (padding tokens: tens of thousands of
//           rows of one id) is therefore split over ceil(len / 64) workgroups and combined in a fixed order.
#include "common.h"

using namespace dllm;

namespace {

constexpr int WIN = 64;

DLLM_DEVICE void add_row(float (&acc)[8], const uint16_t* row) {
  const u16x8 v = *reinterpret_cast<const u16x8*>(row);
#pragma unroll
  for (int j = 0; j < 8; ++j) acc[j] += bf2f(v[j]);
}

__global__ __launch_bounds__(256) void embed_cont_kernel(const int64_t* __restrict__ ids, const int64_t* __restrict__ perm,
                                                         const uint16_t* __restrict__ dy, long ld, long T, int d,
                                                         float* __restrict__ ws) {
  const long start = (long)blockIdx.x * WIN;
  if (start == 0 || start >= T) return;
  const int64_t id = ids[start];
  if (ids[start - 1] != id) return;  // the window's first run starts here: pass 2 owns it
  const int c = threadIdx.x;
  if (c * 8 >= d) return;
  const long end = min(start + WIN, T);
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  for (long i = start; i < end && ids[i] == id; ++i) add_row(acc, dy + perm[i] * ld + c * 8);
  float* o = ws + (long)blockIdx.x * d + c * 8;
  *reinterpret_cast<f32x4*>(o) = f32x4{acc[0], acc[1], acc[2], acc[3]};
  *reinterpret_cast<f32x4*>(o + 4) = f32x4{acc[4], acc[5], acc[6], acc[7]};
}

template <typename TO>
__global__ __launch_bounds__(256) void embed_bwd_kernel(const int64_t* __restrict__ ids, const int64_t* __restrict__ perm,
                                                        const uint16_t* __restrict__ dy, long ld, long T, int d,
                                                        const float* __restrict__ ws, TO* __restrict__ out, long V,
                                                        long padding_idx) {
  const long start = (long)blockIdx.x * WIN;
  const long wend = min(start + WIN, T);
  const int c = threadIdx.x;
  const bool active = c * 8 < d;
  long i = start;
  if (start > 0 && ids[start] == ids[start - 1]) {  // skip the continuation run (pass 1 summed it)
    const int64_t id = ids[start];
    while (i < wend && ids[i] == id) ++i;
  }
  while (i < wend) {
    const int64_t id = ids[i];
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (; i < wend && ids[i] == id; ++i)
      if (active) add_row(acc, dy + perm[i] * ld + c * 8);
    if (i == wend) {  // the run may continue into the next windows: their pass-1 slots, in order
      for (long w2 = blockIdx.x + 1; w2 * WIN < T && ids[w2 * WIN] == id; ++w2) {
        if (active) {
          const float* s = ws + w2 * d + c * 8;
          const f32x4 a = *reinterpret_cast<const f32x4*>(s), b = *reinterpret_cast<const f32x4*>(s + 4);
          acc[0] += a.x; acc[1] += a.y; acc[2] += a.z; acc[3] += a.w;
          acc[4] += b.x; acc[5] += b.y; acc[6] += b.z; acc[7] += b.w;
        }
      }
    }
    if (!active || id == padding_idx || id < 0 || id >= V) continue;
    TO* o = out + id * (long)d + c * 8;
#pragma unroll
    for (int j = 0; j < 8; ++j) Elem<TO>::store(o + j, Elem<TO>::load(o + j) + acc[j]);
  }
}

}  // namespace

// ids: sorted token ids [T] (int64), perm: their positions in dy ([T, d] bf16, row stride ld); out: [V, d] bf16 / fp32
// (accumulated into); ws: fp32 [ceil(T / 64) * d].  d % 8 == 0, d <= 2048.
extern "C" int dllm_embed_bwd(const int64_t* ids, const int64_t* perm, const void* dy, long ld, long T, int d,
                              float* ws, void* out, long V, long padding_idx, int out_f32, hipStream_t st) {
  if (d % 8 || d > 2048 || T <= 0) return -2;
  const long nwin = (T + WIN - 1) / WIN;
  if (nwin > 0x7fffffffL) return -4;
  const int threads = ((d / 8 + 63) / 64) * 64;
  hipLaunchKernelGGL(embed_cont_kernel, dim3((unsigned)nwin), dim3(threads), 0, st, ids, perm, (const uint16_t*)dy, ld,
                     T, d, ws);
  if (out_f32)
    hipLaunchKernelGGL(embed_bwd_kernel<float>, dim3((unsigned)nwin), dim3(threads), 0, st, ids, perm,
                       (const uint16_t*)dy, ld, T, d, (const float*)ws, (float*)out, V, padding_idx);
  else
    hipLaunchKernelGGL(embed_bwd_kernel<uint16_t>, dim3((unsigned)nwin), dim3(threads), 0, st, ids, perm,
                       (const uint16_t*)dy, ld, T, d, (const float*)ws, (uint16_t*)out, V, padding_idx);
  DLLM_CHECK_LAUNCH();
  return 0;
}

// One beam-search step on the LM-head logits, for gfx950 (models/generation.py _beam_search_device).
//
// The reference's generate() (ref/train-accelerator.py:245-249: num_beams=2, max_length=128) runs, per decode step,
// transformers' beam search: fp32 log_softmax over the vocabulary, the logits processors (min_length bans eos,
// no_repeat_ngram bans the completions of earlier n-grams, forced BOS / EOS), + the running beam score, and the top
// 2*num_beams candidates over num_beams x V.  As torch ops that is ~8 launches and five passes over [rows, V] fp32.
// Here one workgroup per batch entry reads each of its beams' logits ONCE:
//
//   * online max / sum-exp (the log_softmax normaliser, over every token: processors act after it);
//   * the n-gram bans of the row, computed in the kernel from the generated prefix (one thread per earlier window),
//     as an LDS bitmap over the vocabulary (plus the min_length eos ban): a banned token never enters the top-K;
//   * a per-thread sorted top-K of the raw logits (K = 2 * num_beams rounded up to a template size), merged across
//     the block by K rounds of a (value, index) argmax;
//   * candidates beam_score + (x - max) - log(sum) of every beam, and the final top-K over num_beams x K of them —
//     the overall top-K is contained in the union of the per-beam top-K lists.
//
// A forced token (BOS at step 1, EOS at the last step) replaces the row by that single candidate with log-prob 0,
// as transformers' ForcedBOS/EOS processors do after the bans.  Ties resolve to the lower flat index.
#include "common.h"

using namespace dllm;

namespace {

struct BeamParams {
  const void* logits;  // [B * nb, V] rows with leading dimension ld (bf16 or fp32)
  long ld;
  const float* beam_scores;  // [B * nb]
  const int64_t* seqs;       // [B * nb, lds] generated prefix (positions 0 .. cur-1)
  long lds;
  int cur, ngram, ban_tok, force_tok, nb, V, k_out;
  float* top_s;     // [B, k_out]
  int64_t* top_i;   // [B, k_out] flat index beam * V + token
};

template <typename T>
DLLM_DEVICE float ld1(const T* p, long i);
template <>
DLLM_DEVICE float ld1<float>(const float* p, long i) { return p[i]; }
template <>
DLLM_DEVICE float ld1<uint16_t>(const uint16_t* p, long i) { return bf2f(p[i]); }

// (value, index) order: larger value first, then smaller index
DLLM_DEVICE bool better(float a, int ia, float b, int ib) { return a > b || (a == b && ia < ib); }

template <int K>
DLLM_DEVICE void insert(float (&tv)[K], int (&ti)[K], float v, int i) {
  if (!better(v, i, tv[K - 1], ti[K - 1])) return;
  tv[K - 1] = v;
  ti[K - 1] = i;
#pragma unroll
  for (int k = K - 1; k > 0; --k) {
    if (better(tv[k], ti[k], tv[k - 1], ti[k - 1])) {
      const float t = tv[k];
      tv[k] = tv[k - 1];
      tv[k - 1] = t;
      const int u = ti[k];
      ti[k] = ti[k - 1];
      ti[k - 1] = u;
    }
  }
}

template <typename T, int K>
__global__ __launch_bounds__(256) void beam_topk_kernel(BeamParams P) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  __shared__ float red_v[4];
  __shared__ int red_i[4];
  __shared__ float cand_s[8 * 16];
  __shared__ int cand_i[8 * 16];
  uint32_t* bits = reinterpret_cast<uint32_t*>(smem);  // [ceil(V / 32)] ban bitmap of the current row
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int b = blockIdx.x, V = P.V, nwords = (V + 31) >> 5;
  const bool bans = P.ngram > 0 || P.ban_tok >= 0;

  for (int j = 0; j < P.nb; ++j) {
    const long row = (long)b * P.nb + j;
    const float bs = P.beam_scores[row];
    if (bans) {  // ---- ban bitmap of this row
      for (int i = tid; i < nwords; i += 256) bits[i] = 0u;
      __syncthreads();
      if (tid == 0 && P.ban_tok >= 0 && P.ban_tok < V) atomicOr(&bits[P.ban_tok >> 5], 1u << (P.ban_tok & 31));
      const int n = P.ngram;
      if (n > 0 && P.cur >= n) {
        const int64_t* s = P.seqs + row * P.lds;
        for (int i = tid; i <= P.cur - n; i += 256) {  // window i: tokens i .. i+n-1; prefix = last n-1 generated
          bool match = true;
          for (int q = 0; q < n - 1; ++q) match = match && s[i + q] == s[P.cur - n + 1 + q];
          const int64_t tok = s[i + n - 1];
          if (match && tok >= 0 && tok < V) atomicOr(&bits[tok >> 5], 1u << (tok & 31));
        }
      }
      __syncthreads();
    }
    if (P.force_tok >= 0) {  // forced token: the single candidate, log-prob 0 (after the bans, as transformers)
      if (tid < K) {
        cand_s[j * K + tid] = tid == 0 ? bs : -INFINITY;
        cand_i[j * K + tid] = j * V + (tid == 0 ? P.force_tok : V - 1);
      }
      __syncthreads();
      continue;
    }
    // ---- one pass: normaliser + per-thread top-K of the unbanned logits
    const T* x = reinterpret_cast<const T*>(P.logits) + row * P.ld;
    float m = -INFINITY, s = 0.f;
    float tv[K];
    int ti[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
      tv[k] = -INFINITY;
      ti[k] = 0x7FFFFFFF;
    }
    auto visit = [&](float v, int c) {
      if (v > m) {
        s = s * expf(m - v) + 1.f;
        m = v;
      } else if (v != -INFINITY) {
        s += expf(v - m);
      }
      if (!bans || !((bits[c >> 5] >> (c & 31)) & 1u)) insert<K>(tv, ti, v, c);
    };
    // 16-B loads (8 bf16 / 4 fp32 per lane) when the row is 16-B aligned; scalar otherwise and for the tail
    constexpr int VW = sizeof(T) == 2 ? 8 : 4;
    const bool vec = (reinterpret_cast<uintptr_t>(x) & 15) == 0;
    const int vend = vec ? V / VW * VW : 0;
    for (int c0 = tid * VW; c0 < vend; c0 += 256 * VW) {
      const u32x4 raw = *reinterpret_cast<const u32x4*>(x + c0);
      if constexpr (sizeof(T) == 2) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          visit(bf2f((uint16_t)(raw[e] & 0xFFFFu)), c0 + 2 * e);
          visit(bf2f((uint16_t)(raw[e] >> 16)), c0 + 2 * e + 1);
        }
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) visit(__uint_as_float(raw[e]), c0 + e);
      }
    }
    for (int c = vend + tid; c < V; c += 256) visit(ld1<T>(x, c), c);
    // block max / sum-exp
    float M = m;
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) M = fmaxf(M, __shfl_xor(M, o, 64));
    __syncthreads();
    if (lane == 0) red_v[w] = M;
    __syncthreads();
    M = fmaxf(fmaxf(red_v[0], red_v[1]), fmaxf(red_v[2], red_v[3]));
    float S = m == -INFINITY ? 0.f : s * expf(m - M);
    S = wave_sum(S);
    __syncthreads();
    if (lane == 0) red_v[w] = S;
    __syncthreads();
    S = red_v[0] + red_v[1] + red_v[2] + red_v[3];
    const float logS = logf(S);
    // block top-K: K rounds of a block-wide (value, index) argmax over the threads' list heads
    for (int k = 0; k < K; ++k) {
      float v = tv[0];
      int i = ti[0];
#pragma unroll
      for (int o = 32; o >= 1; o >>= 1) {
        const float v2 = __shfl_xor(v, o, 64);
        const int i2 = __shfl_xor(i, o, 64);
        if (better(v2, i2, v, i)) {
          v = v2;
          i = i2;
        }
      }
      __syncthreads();
      if (lane == 0) {
        red_v[w] = v;
        red_i[w] = i;
      }
      __syncthreads();
      float bv = red_v[0];
      int bi = red_i[0];
#pragma unroll
      for (int q = 1; q < 4; ++q)
        if (better(red_v[q], red_i[q], bv, bi)) {
          bv = red_v[q];
          bi = red_i[q];
        }
      if (tid == 0) {
        const bool fin = bv != -INFINITY;
        cand_s[j * K + k] = fin ? bs + ((bv - M) - logS) : -INFINITY;
        cand_i[j * K + k] = j * V + (fin ? bi : V - 1);
      }
      if (ti[0] == bi && tv[0] == bv && bv != -INFINITY) {  // the owner pops its head
#pragma unroll
        for (int q = 0; q < K - 1; ++q) {
          tv[q] = tv[q + 1];
          ti[q] = ti[q + 1];
        }
        tv[K - 1] = -INFINITY;
        ti[K - 1] = 0x7FFFFFFF;
      }
    }
    __syncthreads();
  }
  // ---- final top-k_out over the nb x K candidates (<= 128): one thread, selection
  if (tid == 0) {
    const int n = P.nb * K;
    for (int k = 0; k < P.k_out; ++k) {
      int best = -1;
      for (int q = 0; q < n; ++q) {
        if (cand_i[q] < 0) continue;
        if (best < 0 || better(cand_s[q], cand_i[q], cand_s[best], cand_i[best])) best = q;
      }
      P.top_s[(long)b * P.k_out + k] = cand_s[best];
      P.top_i[(long)b * P.k_out + k] = cand_i[best];
      cand_i[best] = -1;
    }
  }
}

template <typename T>
int launch(const BeamParams& p, int B, hipStream_t st) {
  const size_t lds = (size_t)((p.V + 31) / 32) * 4;
  const int need = p.k_out;  // per-beam list length: the overall top-k_out needs at most k_out from one beam
  if (need <= 2) hipLaunchKernelGGL((beam_topk_kernel<T, 2>), dim3(B), dim3(256), lds, st, p);
  else if (need <= 4) hipLaunchKernelGGL((beam_topk_kernel<T, 4>), dim3(B), dim3(256), lds, st, p);
  else if (need <= 8) hipLaunchKernelGGL((beam_topk_kernel<T, 8>), dim3(B), dim3(256), lds, st, p);
  else hipLaunchKernelGGL((beam_topk_kernel<T, 16>), dim3(B), dim3(256), lds, st, p);
  DLLM_CHECK_LAUNCH();
  return 0;
}

}  // namespace

// returns -4 on unsupported arguments (k_out > 16, nb > 8, V too large for the LDS bitmap)
extern "C" int dllm_beam_topk(const void* logits, long ld, int is_bf16, const float* beam_scores, const int64_t* seqs,
                              long lds, int cur, int ngram, int ban_tok, int force_tok, int B, int nb, int V, int k_out,
                              float* top_s, int64_t* top_i, hipStream_t st) {
  if (B <= 0 || nb <= 0 || nb > 8 || k_out <= 0 || k_out > 16 || V <= 0 || (V + 31) / 32 * 4 > 64 * 1024) return -4;
  const int K = k_out <= 2 ? 2 : k_out <= 4 ? 4 : k_out <= 8 ? 8 : 16;
  if (nb * K > 8 * 16) return -4;
  BeamParams p{logits, ld, beam_scores, seqs, lds, cur, ngram, ban_tok, force_tok, nb, V, k_out, top_s, top_i};
  return is_bf16 ? launch<uint16_t>(p, B, st) : launch<float>(p, B, st);
}

// ---- beam reorder of every decoder layer's self-attention cache, in place (models/generation.py KVStore)
// cache [LK = layers * 2][rows][max_len][hd] bf16, rows = batch * nb; row r takes the live prefix (positions < n) of
// row src[r], which always lies in r's own group of nb rows (its batch entry).  One workgroup per (lk, group): a group
// whose hypotheses all kept their own row is skipped (no bytes move); otherwise per position the group's source rows
// are read into registers first and only the rows that change are written — an in-place permutation inside the group,
// no second buffer, no copy of unchanged rows (vs a gather of every row into a temporary and a copy back).
namespace {
__global__ __launch_bounds__(256) void kv_reorder_kernel(uint16_t* __restrict__ cache, const int64_t* __restrict__ src,
                                                         int rows, int nb, int max_len, int hd, int n) {
  const int lk = blockIdx.y, g = blockIdx.x;
  const int r0 = g * nb;
  bool moved = false;
  for (int j = 0; j < nb; ++j) moved |= src[r0 + j] != r0 + j;
  if (!moved) return;  // uniform: every thread read the same indices
  const int cpr = hd / 8;  // 16-B chunks per row
  const long rowlen = (long)max_len * hd;
  uint16_t* base = cache + ((long)lk * rows + r0) * rowlen;
  const int per = cpr * nb;  // chunks of one position of the group
  for (int p = 0; p < n; ++p) {
    // each thread moves up to 2 chunks of this position (nb * hd / 8 <= 512, host-checked)
    u32x4 v[2];
    int dst_row[2], chunk[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int t = threadIdx.x + 256 * u;
      dst_row[u] = -1;
      if (t < per) {
        const int j = t / cpr, c = t % cpr;
        const int s = (int)src[r0 + j] - r0;
        chunk[u] = c;
        if (s != j) {
          dst_row[u] = j;
          v[u] = *reinterpret_cast<const u32x4*>(base + s * rowlen + (long)p * hd + 8 * c);
        }
      }
    }
    __syncthreads();  // every source chunk of this position is in registers before any row of the group changes
#pragma unroll
    for (int u = 0; u < 2; ++u)
      if (dst_row[u] >= 0)
        *reinterpret_cast<u32x4*>(base + dst_row[u] * rowlen + (long)p * hd + 8 * chunk[u]) = v[u];
    __syncthreads();
  }
}
}  // namespace

extern "C" int dllm_kv_reorder(void* cache, const int64_t* src, int lk, int rows, int nb, int max_len, int hd, int n,
                               hipStream_t st) {
  if (lk <= 0 || rows <= 0 || nb <= 0 || rows % nb || hd % 8 || (long)nb * hd / 8 > 512 || n <= 0 || n > max_len)
    return -4;
  hipLaunchKernelGGL(kv_reorder_kernel, dim3(rows / nb, lk), dim3(256), 0, st, (uint16_t*)cache, src, rows, nb, max_len,
                     hd, n);
  DLLM_CHECK_LAUNCH();
  return 0;
}

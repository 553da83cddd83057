// Parameter block shared by csrc/gemm.hip and the host binding (csrc/bind.cpp).
#pragma once
#include <stdint.h>

struct GemmWgradParams {
  const uint16_t* A;  // [K][lda]
  const uint16_t* B;  // [K][ldb]
  void* C;            // [M][ldc], bf16 or fp32 (c_f32): the flat gradient buffer's view
  float* ws;          // [splits][M][N] fp32 (splits > 1)
  long lda, ldb, ldc;
  int M, N, K;
  int tn;      // N / 256
  int ntiles;  // (M / 256) * (N / 256)
  int kchunk;  // k rows per split (multiple of BK)
  int splits;
  int beta;  // 1: C += A^T B, 0: C = A^T B
  int c_f32;  // C is fp32 (fp32 gradient accumulation across micro-batches), else bf16
};

#define W4_MAX_SEGS 32

// csrc/gemm_w4.hip: C[M][N] (+)= A[M][K] . B (+ bias), B = [N][K] (b_kmajor = 0) or [K][N] (b_kmajor = 1).
// Ragged M and N (loads past the edge return 0 through the buffer descriptor's range check, stores are masked);
// K % 64 == 0.
struct GemmW4Params {
  const uint16_t* A;
  const uint16_t* B;
  uint16_t* C;
  const uint16_t* bias;  // [N] or null
  long lda, ldb, ldc;
  int M, N, K;
  int tm, tn;      // ceil(M / 256), ceil(N / 256)
  int grp;         // tile order: groups of grp 256-row blocks, column-major inside a group; 0 = row-major
  int accumulate;  // 1: C += A . B (bf16 read-modify-write), 0: C = A . B
  // epilogue (csrc/gemm_w4.hip W4_EPI_*): ReLU + dropout forward writing the keep-and-positive bit mask, or the input
  // gradient through that mask.  mask: 8 words per thread per 256x256 tile (tile-major, thread-minor), bit 4 j + r of
  // word i <-> accumulator acc[i][j][r]
  uint32_t* mask;
  float p, scale;  // dropout probability, 1 / (1 - p)
  uint32_t seed, thr;
  int mask_pp;  // DRELU_M: the mask was written by csrc/gemm_fused.hip's ping-pong ReLU forward (its thread layout)
  // LM-head cross-entropy epilogues (NT: A = decoder hidden [M][K], B = a vocabulary slice of the tied embedding
  // [N][K] = vocab columns [c0, c0 + N)):
  //   W4_EPI_CEF  no C stores; per row and 128-column half tile the online-softmax partial {max, sum exp, sum x} ->
  //               part[row * pstride + (n / 128)] (f32x4) and the label's logit -> xlab[row]
  //   W4_EPI_CEB  C = dlogits = g * (exp(x - lse[row]) - eps / V - (1 - eps) [c0 + n == label])  (bf16)
  // x = the fp32 accumulator (+ cbias[c0 + n]); columns n < skip (re-covered by a previous slice) and rows whose label
  // is ignore / out of range contribute nothing
  const int64_t* labels;
  const float* cbias;   // [V] fp32 or null (BART final_logits_bias)
  const float* lse;     // CEB: [M]
  const float* gscale;  // CEB: device scalar g / count
  float* part;          // CEF
  float* xlab;          // CEF
  int c0, V, skip, pstride;
  float eps;
  long ignore;
  // weight-gradient epilogue (W4_EPI_WG): A = [K][M] k-major too; K split in `splits` chunks of `kchunk` rows; fp32
  // slabs ws[splits][M][N] (splits > 1), else Cw (fp32 if c_f32, else bf16; += when beta) with row stride ldc
  float* ws;
  void* Cw;
  int splits, kchunk, c_f32, beta;
  // ... over the deferred micro-batches of a gradient-accumulation window (nseg > 0, ops/gemm.py WgradDefer): split ks
  // reads segment ks / seg_chunks (A = segA[], B = segB[], seg_rows k-rows each, leading dimensions lda / ldb), k-rows
  // [(ks % seg_chunks) kchunk, + kchunk); A / B / K unused.  No concatenated copy of the window's operands.
  // GELU epilogues: forward (NT + bias) writes C = s gelu(u) and aux_out = s gelu'(u) (s = dropout keep / (1 - p));
  // backward (NN) C = dU = (A . B) * aux and per-128-row column sums of dU -> colsum [M / 128][N] (fc1 bias gradient)
  uint16_t* aux_out;
  const uint16_t* aux;
  long ldaux;
  float* colsum;
  const uint16_t* segA[W4_MAX_SEGS];
  const uint16_t* segB[W4_MAX_SEGS];
  int nseg, seg_rows, seg_chunks;
};

// csrc/gemm_fused.hip: C[M][N] = epi(A[M][K] . B), B = [N][K] (b_kmajor = 0) or [K][N] (b_kmajor = 1)
struct GemmFusedParams {
  const uint16_t* A;
  const uint16_t* B;
  uint16_t* C;
  const uint16_t* bias;  // [N] or null (added before the activation)
  const uint16_t* aux;   // backward epilogues: saved activation (ReLU) / pre-activation (GELU), [M][ldaux]
  uint16_t* aux_out;     // GELU forward: pre-activation output, [M][ldaux]
  const uint16_t* aux2;  // gated backward (epi 9): second saved factor, [M][ldaux]
  uint16_t* aux_out2;    // gated forward (epi 8): second saved factor, [M][ldaux]
  long lda, ldb, ldc, ldaux;
  int M, N, K;
  int tm, tn;  // M / 256, N / 256
  int epi;     // 0 none, 1 relu, 2 gelu(erf), 3 d-relu, 4 d-gelu(erf), 5 gelu(tanh), 6 d-gelu(tanh),
               // 7 d-relu from bits, 8 gated gelu(tanh) (N = 2F, output [M][F]), 9 its backward (N = F, output [M][2F])
  float p;     // dropout probability on the activation output (forward element index m * N + n)
  float scale; // 1 / (1 - p), or 1
  uint32_t seed, thr;
  int grp;     // tile order (gemm_pp_kernel): groups of grp 256-row blocks, column-major inside a group; 0 = row-major
  uint32_t* mask;  // ReLU derivative bits (ping-pong kernel): written by epi 1 when non-null, read by epi 7; M*N/32 words
  float* colsum;   // optional (ping-pong kernel, epi 4 / 6): [M / 128][N] per-128-row column sums of the output C
};

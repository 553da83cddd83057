// Parameter block shared by csrc/gemm.hip and the host binding (csrc/bind.cpp).
#pragma once
#include <stdint.h>

struct GemmWgradParams {
  const uint16_t* A;  // [K][lda]
  const uint16_t* B;  // [K][ldb]
  uint16_t* C;        // [M][ldc]
  float* ws;          // [splits][M][N] fp32 (splits > 1)
  long lda, ldb, ldc;
  int M, N, K;
  int tn;      // N / 256
  int ntiles;  // (M / 256) * (N / 256)
  int kchunk;  // k rows per split (multiple of BK)
  int splits;
  int beta;  // 1: C += A^T B, 0: C = A^T B
};

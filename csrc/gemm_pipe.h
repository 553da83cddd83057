// One-wave-per-SIMD GEMM main loop for gfx950 (MI355X / CDNA4), shared by csrc/gemm_fused.hip (projection
// GEMMs with fused epilogues) and csrc/gemm.hip (weight gradients).
//
// Why: the 8-wave (2 per SIMD) 256x256 kernels synchronise the whole CU at every k-stage barrier and read 12 LDS
// fragments per 32 MFMAs; rocprofv3 PMC on the t5-base wi GEMM showed the MFMA pipe busy only 38 % of the kernel
// (hipBLASLt: 58 %) with 22 % of wave cycles parked on barriers / waitcnt (profiles/r1_gemm_pmc.txt).
// This loop runs 4 waves per 256x256 tile, each wave owning a 128x128 block (8x8 v_mfma_f32_16x16x32_bf16 tiles,
// 256 accumulator registers: one wave per SIMD, the whole 512-entry register file), so:
// * 16 LDS fragment reads feed 64 MFMAs (half the LDS traffic per MFMA);
// * the next k-step's fragments are read into a second register set while this k-step's MFMAs run — the LDS
//   latency never reaches the MFMA pipe;
// * operands stream global -> LDS by LDS-DMA (global_load_lds_dwordx4, pre-swizzled source addresses, no VGPR
//   staging) into a 4-deep ring of 32-deep k-stages (4 x 32 KB), issued 3 stages ahead: one barrier per stage,
//   a counted vmcnt keeps the next stage in flight across it, ~2 stages (2 x 1024 MFMA cycles) of DMA latency
//   hidden;
// * hazards: stage s is read (prefetch) in iteration s-1, after barrier B_{s-1}, which every wave passes only
//   after its own vmcnt for stage s; iteration it refills the buffer of stage it-1, whose reads every wave
//   consumed (lgkmcnt) before reaching B_it.
//
// Operand images per stage (BK = 32):
//   row image  [256][32] (64-B rows; the operand is K-contiguous, e.g. activations [tokens][in] or an nn.Linear
//              weight [out][in]): 16-B chunk c of row r at chunk c ^ SW32[(r >> 2) & 3], SW32 = {0, 2, 3, 1} —
//              each 16-lane group of a 16x16x32 fragment read (16 rows x one chunk) hits 16 distinct bank slots;
//   k-major    [32][256] (512-B rows; the operand is M/N-contiguous, e.g. dY [tokens][out] in a weight gradient or
//              a weight [out][in] read as [K][N] in the input gradient): fragments by hardware-transposed reads
//              (ds_read_b64_tr_b16); chunk c of k-row r at c ^ ((r & 3) << 2 ^ ((r >> 3) & 1) << 1).
#pragma once
#include "common.h"

namespace dllm {
namespace pipe4 {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8v;
typedef __attribute__((ext_vector_type(4))) short s16x4;

constexpr int BK = 32;            // k per stage
constexpr int NBUF = 4;           // LDS ring depth
constexpr int AHEAD = 3;          // stages issued ahead
constexpr int IMG = 256 * BK;     // elements of one operand image (16 KB)
constexpr int STAGE = 2 * IMG;    // A image | B image
constexpr int LDS_BYTES = NBUF * STAGE * 2;  // 128 KB
constexpr int PW = 4;             // 1-KB DMA instructions per wave per operand per stage (16 KB / 4 waves)
constexpr int LPS = 2 * PW;       // per wave per stage

DLLM_DEVICE int sw32(int r) { return (0x1320 >> (4 * ((r >> 2) & 3))) & 3; }  // {0, 2, 3, 1}
DLLM_DEVICE int swkm(int r) { return ((r & 3) << 2) ^ (((r >> 3) & 1) << 1); }

// 16x16x32 fragment from a row image: lane l holds row cb + (l & 15), k = 8 (l >> 4) + 0..7
DLLM_DEVICE bf16x8v frag_row(const uint16_t* T, int cb, int lane) {
  const int r = cb + (lane & 15);
  const int c = lane >> 4;
  const u16x8 v = *reinterpret_cast<const u16x8*>(T + r * BK + ((c ^ sw32(r)) << 3));
  return __builtin_bit_cast(bf16x8v, v);
}

DLLM_DEVICE u16x4 ld_tr(const uint16_t* T, int r, int col) {
  const int off = (r << 8) + (((col >> 3) ^ swkm(r)) << 3) + (col & 7);
  s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(T + off));
  return __builtin_bit_cast(u16x4, v);
}

// 16x16x32 fragment from a k-major image: lane l holds column cb + (l & 15), k = 8 (l >> 4) + 0..7.  Within each
// 16-lane group, lane 4q+p addresses k-row q (+4 for the high half), columns 4p..4p+3.
DLLM_DEVICE bf16x8v frag_km(const uint16_t* T, int cb, int lane) {
  const int i = lane & 15;
  const int r = 8 * (lane >> 4) + (i >> 2);
  const int col = cb + 4 * (i & 3);
  const u16x4 lo = ld_tr(T, r, col);
  const u16x4 hi = ld_tr(T, r + 4, col);
  const u16x8 v = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
  return __builtin_bit_cast(bf16x8v, v);
}

// Per-lane DMA source offsets (elements, relative to the operand's tile origin at k = 0) of this wave's PW
// instructions for one operand.  Row image: instruction q covers rows 16q..16q+15, lane -> (row l/4, chunk l%4).
// k-major: instruction q covers k-rows 2q, 2q+1, lane -> (k-row l/32, chunk l%32).
template <bool KM>
DLLM_DEVICE void dma_offsets(long (&off)[PW], long ld, int w, int lane) {
#pragma unroll
  for (int i = 0; i < PW; ++i) {
    const int q = w * PW + i;
    if (KM) {
      const int kr = 2 * q + (lane >> 5);
      off[i] = (long)kr * ld + (((lane & 31) ^ swkm(kr)) << 3);
    } else {
      const int r = 16 * q + (lane >> 2);
      off[i] = (long)r * ld + (((lane & 3) ^ sw32(r)) << 3);
    }
  }
}

// acc[i][j] (i: 16-row tile of the wave's 128 rows, j: 16-column tile of its 128 columns) +=
//   sum over nk stages of A_tile . B_tile, with the MFMA roles swapped so that lane l holds
//   C[row 16 i + (l & 15)][cols 16 j + 4 (l >> 4) + 0..3] of the wave block.
// Ag / Bg: operand tile origins at the first k (row image: &X[row0][k0], k-major: &X[k0][col0]); lda / ldb their
// leading dimensions.  All 256 threads of the workgroup must call this (barriers inside).
template <bool AKM, bool BKM>
DLLM_DEVICE void mainloop(f32x4 (&acc)[8][8], const uint16_t* Ag, long lda, const uint16_t* Bg, long ldb, int nk,
                          uint16_t* lds) {
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  const int wm = w >> 1, wn = w & 1;
  long aoff[PW], boff[PW];
  dma_offsets<AKM>(aoff, lda, w, lane);
  dma_offsets<BKM>(boff, ldb, w, lane);
  const long astep = AKM ? (long)BK * lda : BK;  // element advance of one stage
  const long bstep = BKM ? (long)BK * ldb : BK;
  const uint32_t lds0 = lds_addr(lds);
  auto issue = [&](int s) {
    const uint32_t Al = lds0 + (uint32_t)((s % NBUF) * STAGE) * 2u;
    const uint32_t Bl = Al + IMG * 2u;
    const uint16_t* a = Ag + s * astep;
    const uint16_t* b = Bg + s * bstep;
#pragma unroll
    for (int i = 0; i < PW; ++i) {
      const uint32_t q = __builtin_amdgcn_readfirstlane(w * PW + i);
      glds16(a + aoff[i], __builtin_amdgcn_readfirstlane(Al + q * 1024u));
      glds16(b + boff[i], __builtin_amdgcn_readfirstlane(Bl + q * 1024u));
    }
  };
  auto read = [&](int s, bf16x8v (&a)[8], bf16x8v (&b)[8]) {
    const uint16_t* As = lds + (s % NBUF) * STAGE;
    const uint16_t* Bs = As + IMG;
#pragma unroll
    for (int i = 0; i < 8; ++i) a[i] = AKM ? frag_km(As, wm * 128 + 16 * i, lane) : frag_row(As, wm * 128 + 16 * i, lane);
#pragma unroll
    for (int j = 0; j < 8; ++j) b[j] = BKM ? frag_km(Bs, wn * 128 + 16 * j, lane) : frag_row(Bs, wn * 128 + 16 * j, lane);
  };
  auto mma = [&](const bf16x8v (&a)[8], const bf16x8v (&b)[8]) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[j], a[i], acc[i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };
  // stage s + 1 landed (this wave's DMA) and visible to every wave; stage s + 2 may stay in flight
  auto sync_next = [&](int s) {
    if (s + 2 < nk) wait_vm<LPS>();
    else wait_vm<0>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };

#pragma unroll
  for (int s = 0; s < AHEAD; ++s)
    if (s < nk) issue(s);
  // stage 0 landed: stages 1 and 2 may stay in flight
  if (nk > 2) wait_vm<2 * LPS>();
  else if (nk > 1) wait_vm<LPS>();
  else wait_vm<0>();
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");

  bf16x8v a0[8], b0[8], a1[8], b1[8];
  read(0, a0, b0);
  // two stages per trip so the fragment register sets alternate without moves; odd tail after the loop
  int it = 0;
  for (; it + 1 < nk; it += 2) {
    sync_next(it);
    if (it + AHEAD < nk) issue(it + AHEAD);
    read(it + 1, a1, b1);
    mma(a0, b0);
    if (it + 2 < nk) {
      sync_next(it + 1);
      if (it + 1 + AHEAD < nk) issue(it + 1 + AHEAD);
      read(it + 2, a0, b0);
    }
    mma(a1, b1);
  }
  if (it < nk) mma(a0, b0);
}

}  // namespace pipe4
}  // namespace dllm

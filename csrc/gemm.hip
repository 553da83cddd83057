// Weight-gradient GEMM for gfx950 (MI355X / CDNA4):  C[M][N] (+)= A^T B,  A = [K][M], B = [K][N].
//
// In a linear layer's backward dW[out][in] = dY^T X with dY = [tokens][out] and X = [tokens][in]: both
// operands are token-major, so the reduction dim (tokens, K = 10^4..10^5) is the SLOW index of both — the
// layout library GEMMs handle worst (hipBLASLt reaches 450-900 TF/s on these shapes vs ~1.3-1.5 PF/s for
// the forward projections, profiles/r1_t5base_b64_prof10_summary.txt).  This kernel is built for it:
//
// * 256x256 output tile per 512-thread workgroup (8 waves as 2(M) x 4(N), 128x64 per wave = 4x2
//   v_mfma_f32_32x32x16_bf16 accumulators), BK = 64 k-rows per stage;
// * operand tiles go global -> LDS by LDS-DMA (global_load_lds_dwordx4, no VGPR staging) into [BK][256]
//   images with 512-B rows; the MFMA fragments (k = 8 consecutive rows of one column per lane) come out
//   with hardware-transposed reads (ds_read_b64_tr_b16), so neither operand is ever transposed in memory.
//   16-B chunk c of row r lives at chunk c ^ 4(r&3): the DMA's lane-linear image is fed from pre-swizzled
//   source addresses, and every transposed read (4 rows x 64 B per half-wave) hits 64 distinct banks;
// * NBUF-deep LDS ring, one barrier per k-stage, counted vmcnt so the next stages' DMA stays in flight;
// * output is small (out x in) while K is huge, so K is split over workgroups to fill all 256 CUs:
//   each split writes an fp32 slab, a bandwidth-bound pass sums the slabs and accumulates into the bf16
//   gradient (beta = 1: the flat gradient buffer of parallel/flat.py, no AccumulateGrad kernel).
//   Split ids are the slow index of the XCD-remapped block id so one XCD works one K range (L2 reuse).
#include "common.h"

using namespace dllm;

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8v;
typedef __attribute__((ext_vector_type(4))) short s16x4;

#include "gemm_params.h"

namespace {

constexpr int BM = 256, BN = 256, NT = 512;

DLLM_DEVICE int xcd_remap(int bid, int nblk) {
  const int q = nblk / 8, r = nblk % 8, x = bid % 8;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + bid / 8;
}

DLLM_DEVICE int crow(int reg, int hh) { return (reg & 3) + 8 * (reg >> 2) + 4 * hh; }

// bit 3 of the k-row also enters the swizzle so the two 16-lane groups of a 16x16x32 fragment read (k-rows
// kk..kk+3 and kk+8..kk+11 of the same 16 columns, one ds_read_b64_tr_b16) land on distinct banks
DLLM_DEVICE int gsw(int r) { return ((r & 3) << 2) ^ (((r >> 3) & 1) << 1); }

// element offset of (row r, col) in a swizzled [rows][256] bf16 image
DLLM_DEVICE int loff(int r, int col) { return (r << 8) + (((col >> 3) ^ gsw(r)) << 3) + (col & 7); }

// ds_read_b64_tr_b16: the calling lane's 16-lane group reads rows r0..r0+3 x columns c0..c0+15; group
// lane i receives column c0 + i (row q in element q).  Lane 4q+p supplies the address of row q, cols 4p..
DLLM_DEVICE u16x4 ld_tr(const uint16_t* T, int r0, int c0, int i) {
  const int r = r0 + (i >> 2);
  const int col = c0 + 4 * (i & 3);
  s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(T + loff(r, col)));
  return __builtin_bit_cast(u16x4, v);
}

// 32x32x16 operand for columns [cb, cb+32) and k rows [kk, kk+16): lane l holds column cb + (l & 31),
// k = kk + 8 (l >> 5) + j — the same fragment shape for A (column = m) and B (column = n).
DLLM_DEVICE bf16x8v frag(const uint16_t* T, int kk, int cb, int lane) {
  const int g = lane >> 4;
  const int r0 = kk + 8 * (g >> 1);
  const int c0 = cb + 16 * (g & 1);
  const u16x4 lo = ld_tr(T, r0, c0, lane & 15);
  const u16x4 hi = ld_tr(T, r0 + 4, c0, lane & 15);
  const u16x8 v = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
  return __builtin_bit_cast(bf16x8v, v);
}

// 16x16x32 operand for columns [cb, cb+16) and k rows [kk, kk+32): lane l holds column cb + (l & 15),
// k = kk + 8 (l >> 4) + j
DLLM_DEVICE bf16x8v frag16(const uint16_t* T, int kk, int cb, int lane) {
  const int r0 = kk + 8 * (lane >> 4);
  const u16x4 lo = ld_tr(T, r0, cb, lane & 15);
  const u16x4 hi = ld_tr(T, r0 + 4, cb, lane & 15);
  const u16x8 v = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
  return __builtin_bit_cast(bf16x8v, v);
}

// NI = 32x32 MFMA tiles per wave along N: NI = 2 -> 8 waves of 128x64 (2 waves per SIMD), NI = 4 -> 4 waves of
// 128x128 (one wave per SIMD, 256 fp32 accumulators in AGPRs, next k-step's fragments prefetched in VGPRs)
// MF = 16: v_mfma_f32_16x16x32_bf16 with the NI = 2 geometry (8 waves of 128x64, 8x4 tiles of 16x16 per wave):
// same cycles per FLOP as 32x32x16, higher sustained clock on random data (MI355X_MICROARCH.md "DVFS give-back" 7)
// PRE (16x16, BK = 64): both 32-deep k-steps' fragments are read before the first MFMA of a stage.  Not used:
// with both operands on transposed reads it needs > 256 VGPRs and spills (2x slower, r1_gemm_wgrad_bench_v4).
// PP = 2 (16x16, BK = 64, NBUF = 2): the barrier of stage s + 1 sits between the two 32-deep halves of stage s, so the
// first fragments of stage s + 1 are read while the second half of stage s is on the matrix cores (the default
// structure reads them after the barrier with every wave of the CU stalled on them).  Legal because the barrier only
// needs stage s + 1 landed (its DMA is the one in flight) and every wave's reads of stage s done (lgkmcnt(0) before it:
// the second half's fragments are in registers) before stage s + 2 refills stage s's slot.
// PP = 1 (16x16, BK = 32, NBUF = 4): the two wave groups (wm = 0 / 1: one wave of each on every SIMD) run one stage apart —
// group 1 passes one extra barrier first — so on each SIMD one wave is in its MFMA block while the other is at the start
// of its stage (barrier, LDS reads, waits) instead of both stalling there together (cdna_hip_programming.md, the 256^2
// template's staggered wave groups).  Every global barrier g: each wave first waits for its own DMA of stage g (stage g + 1
// may stay in flight), then issues stage g + 2 into the buffer of stage g - 2, which group 0 finished before barrier
// g - 1 and group 1 before barrier g; group 0 computes stage g, group 1 stage g - 1; barriers 0 .. nk for both.
template <int BK, int NBUF, bool PRIO, int NI, int MF = 32, bool PRE = false, int PP = 0>
__global__ __launch_bounds__((256 / (32 * NI)) * 2 * 64, 1) void gemm_wgrad_kernel(GemmWgradParams P) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  uint16_t* lds = reinterpret_cast<uint16_t*>(smem);  // [NBUF][A tile | B tile], each [BK][256]
  constexpr int WAVES_N = 256 / (32 * NI), NW = 2 * WAVES_N;
  constexpr int TILE = BK * 256;
  constexpr int PW = (BK / 2) / NW;  // DMA instructions per wave per operand per stage (1 KB = 2 rows each)
  constexpr int LPS = 2 * PW;        // per wave per stage (A + B)
  static_assert(NBUF >= 2 && NBUF <= 4 && PW >= 1, "ring depth / DMA split");

  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63, hh = lane >> 5;
  const int wm = w / WAVES_N, wn = w % WAVES_N;
  const int logical = xcd_remap(blockIdx.x, gridDim.x);
  const int s = logical / P.ntiles, t = logical % P.ntiles;
  const int m0 = (t / P.tn) * BM, n0 = (t % P.tn) * BN;  // rows m >= P.M of the last M tile: computed, not stored
  const int kbeg = s * P.kchunk;
  const int nk = min(P.kchunk, P.K - kbeg) / BK;

  // this lane's DMA source: row 2*rp + hh of the stage, chunk (lane & 31) of the swizzled image
  const uint16_t* Ag = P.A + m0 + (long)kbeg * P.lda;
  const uint16_t* Bg = P.B + n0 + (long)kbeg * P.ldb;
  int srow[PW], scol[PW];
#pragma unroll
  for (int i = 0; i < PW; ++i) {
    const int r = 2 * (w * PW + i) + hh;
    srow[i] = r;
    scol[i] = ((lane & 31) ^ gsw(r)) << 3;
  }
  // ragged last M tile (LM-head weight gradient, M = vocab): A columns past M re-read column M - 8 (finite values
  // whose output rows are never stored; M % 8 == 0 keeps every 16-B chunk inside the row)
  int acol[PW];
#pragma unroll
  for (int i = 0; i < PW; ++i) acol[i] = min(m0 + scol[i], P.M - 8) - m0;
  const uint32_t lds0 = lds_addr(lds);
  auto issue = [&](int buf, int kt) {
    const long k0 = (long)kt * BK;
    const uint32_t Al = lds0 + (uint32_t)(buf * 2 * TILE) * 2u;
    const uint32_t Bl = Al + TILE * 2u;
#pragma unroll
    for (int i = 0; i < PW; ++i) {
      const uint32_t rp = __builtin_amdgcn_readfirstlane(w * PW + i);
      glds16(Ag + (k0 + srow[i]) * P.lda + acol[i], __builtin_amdgcn_readfirstlane(Al + rp * 1024u));
      glds16(Bg + (k0 + srow[i]) * P.ldb + scol[i], __builtin_amdgcn_readfirstlane(Bl + rp * 1024u));
    }
  };

#pragma unroll
  for (int p = 0; p < (PP == 1 ? 2 : NBUF - 1); ++p)
    if (p < nk) issue(p, p);

  auto stage_sync = [&](int it) {
    // stage `it` must have landed; stages it+1 .. it+NBUF-2 (if issued) may stay in flight
    const int ahead = min(NBUF - 2, nk - 1 - it);
    if (NBUF >= 4 && ahead >= 2) wait_vm<(NBUF >= 4 ? 2 * LPS : 0)>();
    else if (NBUF >= 3 && ahead >= 1) wait_vm<(NBUF >= 3 ? LPS : 0)>();
    else wait_vm<0>();
    // every wave's reads of the buffer about to be refilled are complete before anyone passes
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (it + NBUF - 1 < nk) issue((it + NBUF - 1) % NBUF, it + NBUF - 1);
  };

  if constexpr (MF == 16) {
    static_assert(NI == 2, "16x16x32 path uses the 8-wave 128x64 geometry");
    f32x4 acc[8][4];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    auto stage_compute = [&](int it) __attribute__((always_inline)) {
      const uint16_t* As = lds + (it % NBUF) * 2 * TILE;
      const uint16_t* Bs = As + TILE;
      auto load_k = [&](int kk, bf16x8v (&a)[8], bf16x8v (&b)[4]) {
#pragma unroll
        for (int i = 0; i < 8; ++i) a[i] = frag16(As, kk, wm * 128 + 16 * i, lane);
#pragma unroll
        for (int j = 0; j < 4; ++j) b[j] = frag16(Bs, kk, wn * 64 + 16 * j, lane);
      };
      auto mfma_block = [&](const bf16x8v (&a)[8], const bf16x8v (&b)[4]) {
        if (PRIO) __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)  // swapped roles: lane holds row m = lane & 15, 4 consecutive columns n
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[j], a[i], acc[i][j], 0, 0, 0);
        if (PRIO) __builtin_amdgcn_s_setprio(0);
      };
      if constexpr (PRE && BK == 64) {
        bf16x8v a0[8], b0[4], a1[8], b1[4];
        load_k(0, a0, b0);
        load_k(32, a1, b1);
        mfma_block(a0, b0);
        mfma_block(a1, b1);
      } else {
#pragma unroll
        for (int ks = 0; ks < BK / 32; ++ks) {
          bf16x8v a[8], b[4];
          load_k(32 * ks, a, b);
          mfma_block(a, b);
        }
      }
    };
    if constexpr (PP == 2) {
      static_assert(BK == 64 && NBUF == 2, "cross-stage pipeline: two 32-deep halves per stage, 2-slot ring");
      // fragments: A i = 0..3 and all of B of a stage's first half cross the barrier (32 VGPRs, what the register file
      // holds beside the second half's 48); A i = 4..7 are read under the first 16 MFMAs
      auto load_a = [&](int it, int kk, int i0, bf16x8v (&a)[8]) __attribute__((always_inline)) {
        const uint16_t* As = lds + (it % NBUF) * 2 * TILE;
#pragma unroll
        for (int i = i0; i < i0 + 4; ++i) a[i] = frag16(As, kk, wm * 128 + 16 * i, lane);
      };
      auto load_b = [&](int it, int kk, bf16x8v (&b)[4]) __attribute__((always_inline)) {
        const uint16_t* Bs = lds + (it % NBUF) * 2 * TILE + TILE;
#pragma unroll
        for (int j = 0; j < 4; ++j) b[j] = frag16(Bs, kk, wn * 64 + 16 * j, lane);
      };
      auto mfma_rows = [&](const bf16x8v (&a)[8], const bf16x8v (&b)[4], int i0, int i1) __attribute__((always_inline)) {
        if (PRIO) __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = i0; i < i1; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[j], a[i], acc[i][j], 0, 0, 0);
        if (PRIO) __builtin_amdgcn_s_setprio(0);
      };
      wait_vm<0>();  // stage 0 landed
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      if (nk > 1) issue(1, 1);
      bf16x8v fa[8], fb[4], ga[8], gb[4];
      load_a(0, 0, 0, fa);
      load_b(0, 0, fb);
      for (int it = 0; it < nk; ++it) {
        load_a(it, 0, 4, fa);          // rest of the first half's A under its first 16 MFMAs
        mfma_rows(fa, fb, 0, 4);
        mfma_rows(fa, fb, 4, 8);
        load_a(it, 32, 0, ga);         // second half (k 32..63) of stage it
        load_a(it, 32, 4, ga);
        load_b(it, 32, gb);
        if (it + 1 < nk) {
          wait_vm<0>();  // stage it + 1 landed (the only DMA in flight)
          asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // all reads of stage it done
          if (it + 2 < nk) issue(it % NBUF, it + 2);
          load_a(it + 1, 0, 0, fa);
          load_b(it + 1, 0, fb);
        }
        mfma_rows(ga, gb, 0, 8);
      }
    } else if constexpr (PP == 1) {
      static_assert(BK == 32 && NBUF == 4, "staggered groups: one k-step per stage, 4-slot ring");
      const int grp = __builtin_amdgcn_readfirstlane(wm);
      for (int g = 0; g <= nk; ++g) {
        if (g + 1 < nk) wait_vm<LPS>();  // stage g landed; stage g + 1 may stay in flight
        else wait_vm<0>();
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        if (g + 2 < nk) issue((g + 2) % NBUF, g + 2);
        const int st = g - grp;
        if (st >= 0 && st < nk) stage_compute(st);
      }
    } else {
      for (int it = 0; it < nk; ++it) {
        stage_sync(it);
        stage_compute(it);
      }
    }
    // acc[i][j][0..3] = C[m0 + wm*128 + 16i + (lane & 15)][n0 + wn*64 + 16j + 4 (lane >> 4) + 0..3]
    const int mrow = m0 + wm * 128 + (lane & 15);
    const int ncol4 = n0 + wn * 64 + 4 * (lane >> 4);
    if (P.splits == 1) {
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          if (mrow + 16 * i >= P.M) continue;
          const long ci = (long)(mrow + 16 * i) * P.ldc + ncol4 + 16 * j;
          f32x4 v = acc[i][j];
          if (P.c_f32) {
            float* cp = reinterpret_cast<float*>(P.C) + ci;
            if (P.beta) v += *reinterpret_cast<const f32x4*>(cp);
            *reinterpret_cast<f32x4*>(cp) = v;
          } else {
            uint16_t* cp = reinterpret_cast<uint16_t*>(P.C) + ci;
            if (P.beta) {
              const u16x4 c = *reinterpret_cast<const u16x4*>(cp);
              v += f32x4{bf2f(c.x), bf2f(c.y), bf2f(c.z), bf2f(c.w)};
            }
            const u16x4 o = {f2bf(v.x), f2bf(v.y), f2bf(v.z), f2bf(v.w)};
            *reinterpret_cast<u16x4*>(cp) = o;
          }
        }
    } else {
      float* W = P.ws + (long)s * P.M * P.N;
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if (mrow + 16 * i < P.M)
            *reinterpret_cast<f32x4*>(W + (long)(mrow + 16 * i) * P.N + ncol4 + 16 * j) = acc[i][j];
    }
    return;
  } else {
  f32x16 acc[4][NI];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  for (int it = 0; it < nk; ++it) {
    stage_sync(it);
    const uint16_t* As = lds + (it % NBUF) * 2 * TILE;
    const uint16_t* Bs = As + TILE;
    bf16x8v a[2][4], b[2][NI];
#pragma unroll
    for (int i = 0; i < 4; ++i) a[0][i] = frag(As, 0, wm * 128 + 32 * i, lane);
#pragma unroll
    for (int j = 0; j < NI; ++j) b[0][j] = frag(Bs, 0, wn * 32 * NI + 32 * j, lane);
#pragma unroll
    for (int ks = 0; ks < BK / 16; ++ks) {
      const int cur = ks & 1;
      if (ks + 1 < BK / 16) {  // next k-step's fragments in flight while this step's MFMAs run
#pragma unroll
        for (int i = 0; i < 4; ++i) a[cur ^ 1][i] = frag(As, 16 * (ks + 1), wm * 128 + 32 * i, lane);
#pragma unroll
        for (int j = 0; j < NI; ++j) b[cur ^ 1][j] = frag(Bs, 16 * (ks + 1), wn * 32 * NI + 32 * j, lane);
      }
      if (PRIO) __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < NI; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[cur][i], b[cur][j], acc[i][j], 0, 0, 0);
      if (PRIO) __builtin_amdgcn_s_setprio(0);
    }
  }

  // epilogue: lane owns column n0 + wn*32*NI + 32j + (lane & 31) of rows m0 + wm*128 + 32i + crow(reg)
  const int ncol = n0 + wn * 32 * NI + (lane & 31);
  if (P.splits == 1) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < NI; ++j)
#pragma unroll
        for (int reg = 0; reg < 16; ++reg) {
          const int m = m0 + wm * 128 + 32 * i + crow(reg, hh);
          if (m >= P.M) continue;
          const long ci = (long)m * P.ldc + ncol + 32 * j;
          float v = acc[i][j][reg];
          if (P.c_f32) {
            float* cp = reinterpret_cast<float*>(P.C) + ci;
            if (P.beta) v += *cp;
            *cp = v;
          } else {
            uint16_t* cp = reinterpret_cast<uint16_t*>(P.C) + ci;
            if (P.beta) v += bf2f(*cp);
            *cp = f2bf(v);
          }
        }
  } else {
    float* W = P.ws + (long)s * P.M * P.N;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < NI; ++j)
#pragma unroll
        for (int reg = 0; reg < 16; ++reg) {
          const int m = m0 + wm * 128 + 32 * i + crow(reg, hh);
          if (m < P.M) W[(long)m * P.N + ncol + 32 * j] = acc[i][j][reg];
        }
  }
  }  // MF == 32
}

// C[m][n] = sum_s ws[s][m][n] (+ C[m][n]), 8 columns per thread (N % 8 == 0); C bf16 or fp32 (TC)
template <typename TC>
__global__ __launch_bounds__(256) void splitk_reduce_kernel(const float* __restrict__ ws, TC* __restrict__ C,
                                                            long ldc, int M, int N, int splits, int beta) {
  const long n8 = (long)M * N / 8;
  const long slab = (long)M * N;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += (long)gridDim.x * blockDim.x) {
    const long e = i * 8;
    const int m = (int)(e / N), n = (int)(e % N);
    f32x4 a = *reinterpret_cast<const f32x4*>(ws + e);
    f32x4 b = *reinterpret_cast<const f32x4*>(ws + e + 4);
    for (int s = 1; s < splits; ++s) {
      a += *reinterpret_cast<const f32x4*>(ws + s * slab + e);
      b += *reinterpret_cast<const f32x4*>(ws + s * slab + e + 4);
    }
    TC* cp = C + (long)m * ldc + n;
    if constexpr (sizeof(TC) == 4) {
      if (beta) {
        a += *reinterpret_cast<const f32x4*>(cp);
        b += *reinterpret_cast<const f32x4*>(cp + 4);
      }
      *reinterpret_cast<f32x4*>(cp) = a;
      *reinterpret_cast<f32x4*>(cp + 4) = b;
    } else {
      if (beta) {
        const u16x8 c = *reinterpret_cast<const u16x8*>(cp);
        a.x += bf2f(c[0]); a.y += bf2f(c[1]); a.z += bf2f(c[2]); a.w += bf2f(c[3]);
        b.x += bf2f(c[4]); b.y += bf2f(c[5]); b.z += bf2f(c[6]); b.w += bf2f(c[7]);
      }
      const u16x8 o = {f2bf(a.x), f2bf(a.y), f2bf(a.z), f2bf(a.w), f2bf(b.x), f2bf(b.y), f2bf(b.z), f2bf(b.w)};
      *reinterpret_cast<u16x8*>(cp) = o;
    }
  }
}

template <int BK, int NBUF, bool PRIO = false, int NI = 2, int MF = 32, bool PRE = false, int PP = 0>
int launch_wgrad(const GemmWgradParams& p, hipStream_t st) {
  constexpr int threads = (256 / (32 * NI)) * 2 * 64;
  const size_t lds = (size_t)NBUF * 2 * BK * 256 * 2;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)gemm_wgrad_kernel<BK, NBUF, PRIO, NI, MF, PRE, PP>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr = true;
  }
  const int nblk = p.ntiles * p.splits;
  hipLaunchKernelGGL((gemm_wgrad_kernel<BK, NBUF, PRIO, NI, MF, PRE, PP>), dim3(nblk), dim3(threads), lds, st, p);
  DLLM_CHECK_LAUNCH();
  if (p.splits > 1) {
    const long n8 = (long)p.M * p.N / 8;
    const int blocks = (int)std::min<long>((n8 + 255) / 256, 2048);
    if (p.c_f32)
      hipLaunchKernelGGL(splitk_reduce_kernel<float>, dim3(blocks), dim3(256), 0, st, p.ws, (float*)p.C, p.ldc, p.M,
                         p.N, p.splits, p.beta);
    else
      hipLaunchKernelGGL(splitk_reduce_kernel<uint16_t>, dim3(blocks), dim3(256), 0, st, p.ws, (uint16_t*)p.C, p.ldc,
                         p.M, p.N, p.splits, p.beta);
    DLLM_CHECK_LAUNCH();
  }
  return 0;
}

}  // namespace

extern "C" int dllm_gemm_wgrad_bk() { return 64; }

// the split-K pass alone: C (+)= sum of p.splits fp32 slabs p.ws (the w4 weight-gradient kernel's, csrc/gemm_w4.hip)
extern "C" int dllm_wgrad_reduce(const GemmWgradParams* pp, hipStream_t st) {
  const GemmWgradParams& p = *pp;
  if (p.splits < 2 || p.ws == nullptr || p.N % 8 || p.M <= 0) return -4;
  const long n8 = (long)p.M * p.N / 8;
  const int blocks = (int)std::min<long>((n8 + 255) / 256, 2048);
  if (p.c_f32)
    hipLaunchKernelGGL(splitk_reduce_kernel<float>, dim3(blocks), dim3(256), 0, st, p.ws, (float*)p.C, p.ldc, p.M, p.N,
                       p.splits, p.beta);
  else
    hipLaunchKernelGGL(splitk_reduce_kernel<uint16_t>, dim3(blocks), dim3(256), 0, st, p.ws, (uint16_t*)p.C, p.ldc,
                       p.M, p.N, p.splits, p.beta);
  DLLM_CHECK_LAUNCH();
  return 0;
}

// variant: 0 = BK64 x 2 stages (128 KB LDS), 1 = BK32 x 4 stages (128 KB), 2 = BK32 x 3 stages (96 KB),
// 3 / 4 = variants 0 / 1 with s_setprio raised around the MFMA block,
// 5 / 6 = variants 0 / 1 with 4 waves of 128x128 (one wave per SIMD, accumulators in AGPRs),
// 7 / 8 / 9 = variants 0 / 4 / 3 on v_mfma_f32_16x16x32_bf16, 10 = variant 8 with staggered wave groups (PP = 1),
// 11 = variant 9 with the next stage's first fragments read across the barrier (PP = 2)
extern "C" int dllm_gemm_wgrad(const GemmWgradParams* pp, int variant, hipStream_t st) {
  const GemmWgradParams& p = *pp;
  if (p.M % 8 || p.M < 8 || p.N % BN || p.K <= 0 || p.splits < 1 || p.ntiles != ((p.M + BM - 1) / BM) * (p.N / BN))
    return -4;
  if (variant < 0)  // auto: 16x16x32 MFMA, BK=64 x 2, prioritised MFMA issue — fastest on every T5 / BART wgrad
    variant = 9;     // shape measured (profiles/r1_gemm_wgrad_bench_v3.jsonl: +3-11 % over the 32x32x16 variants)
  switch (variant) {
    case 1: return launch_wgrad<32, 4>(p, st);
    case 2: return launch_wgrad<32, 3>(p, st);
    case 3: return launch_wgrad<64, 2, true>(p, st);
    case 4: return launch_wgrad<32, 4, true>(p, st);
    case 5: return launch_wgrad<64, 2, false, 4>(p, st);
    case 6: return launch_wgrad<32, 4, false, 4>(p, st);
    case 7: return launch_wgrad<64, 2, false, 2, 16>(p, st);
    case 8: return launch_wgrad<32, 4, true, 2, 16>(p, st);
    case 9: return launch_wgrad<64, 2, true, 2, 16>(p, st);
    case 10: return launch_wgrad<32, 4, true, 2, 16, false, 1>(p, st);
    case 11: return launch_wgrad<64, 2, true, 2, 16, false, 2>(p, st);
    default: return launch_wgrad<64, 2>(p, st);
  }
}

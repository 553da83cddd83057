// Projection GEMMs with fused epilogues for gfx950 (MI355X / CDNA4):
//
//   NT (forward):  C[M][N] = epi( A[M][K] · B[N][K]^T )   A = activations [tokens][in], B = nn.Linear weight [out][in]
//   NN (dgrad):    C[M][N] = epi( A[M][K] · B[K][N] )     A = output grad [tokens][out], B = weight [out][in]
//
// Why a hand-written kernel when hipBLASLt runs these shapes well: the epilogue.  The T5 / BART FFN is
// `wo(dropout(act(wi x)))`; through the library every FFN costs two extra full passes over the
// [tokens, d_ff] activation (activation+dropout forward, activation+dropout backward, ~0.8-1.2 GB of HBM
// traffic each at t5-base b=64) and keeps BOTH the pre-activation and the activation alive for backward.
// Here the wi GEMM applies bias + activation + dropout before its store (the keep decision is the shared
// counter hash of ops/rng.py on the output element index), and the wo dgrad GEMM applies the activation /
// dropout backward to its accumulators before its store: for ReLU the mask is `H != 0` read back from the
// saved activation itself (ReLU and dropout both produce exact zeros), so the pre-activation is never
// stored at all.  GELU writes its derivative, dropout mask and scale applied, as a second output instead of the
// pre-activation: the backward epilogue is then a single multiply.
//
// Structure (same machinery as csrc/gemm.hip, the weight-gradient kernel):
// * 256x256 output tile per 512-thread workgroup, 8 waves as 2(M) x 4(N), 128x64 per wave = 4x2
//   v_mfma_f32_32x32x16_bf16 accumulators; operands staged global -> LDS by LDS-DMA
//   (global_load_lds_dwordx4, lane-linear, pre-swizzled source addresses), NBUF-deep ring, one barrier
//   per k-stage, counted vmcnt keeps the next stages in flight;
// * K-contiguous operands live in [256][BK] images (BK*2-byte rows); 16-B chunk c of row r sits at
//   chunk c ^ ((r / RPB) & (CPR-1)) (RPB = rows per 256-B bank row): the 16 rows one ds_read_b128 phase
//   touches land on 16 distinct bank slots.  N-contiguous B (dgrad) uses the k-major [BK][256] image with
//   hardware-transposed reads (ds_read_b64_tr_b16) exactly as the wgrad kernel;
// * the MFMA operand roles are swapped (C^T = B A^T per 32x32 sub-tile) so a lane's accumulators are 4
//   CONSECUTIVE output columns of one row: the epilogue does its math on f32x4 and stores 8 B per lane,
//   and dropout pairs (2 decisions per hash) fall inside one lane;
// * bijective XCD remap of the 1-D grid, tiles of one 256-row block of A consecutive (L2 reuse of A).
#include "common.h"

#include <cstdlib>
#include <type_traits>

using namespace dllm;

DLLM_SEED_STEP_TU(gemm_fused)

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8v;
typedef __attribute__((ext_vector_type(4))) short s16x4;

#include "gelu.h"
#include "gemm_params.h"

namespace {

constexpr int BM = 256, BN = 256, NT = 512;

enum Epi { EPI_NONE = 0, EPI_RELU = 1, EPI_GELU = 2, EPI_DRELU = 3, EPI_DGELU = 4, EPI_GELU_TANH = 5,
           EPI_DGELU_TANH = 6, EPI_DRELU_M = 7, EPI_GEGLU = 8, EPI_DGEGLU = 9 };

DLLM_DEVICE int xcd_remap(int bid, int nblk) {
  const int q = nblk / 8, r = nblk % 8, x = bid % 8;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + bid / 8;
}

// ---- k-major [BK][256] image (512-B rows), transposed reads (as csrc/gemm.hip).  Bit 3 of the k-row also enters
// the swizzle: the two 16-lane groups of one 16x16x32 fragment read (k-rows kk..kk+3 and kk+8..kk+11 of the same 16
// columns, one ds_read_b64_tr_b16) then land on distinct banks; the 32x32x16 reads stay conflict-free.
DLLM_DEVICE int gsw(int r) { return ((r & 3) << 2) ^ (((r >> 3) & 1) << 1); }
DLLM_DEVICE int loff_km(int r, int col) { return (r << 8) + (((col >> 3) ^ gsw(r)) << 3) + (col & 7); }

DLLM_DEVICE u16x4 ld_tr(const uint16_t* T, int r0, int c0, int i) {
  const int r = r0 + (i >> 2);
  const int col = c0 + 4 * (i & 3);
  s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(T + loff_km(r, col)));
  return __builtin_bit_cast(u16x4, v);
}

DLLM_DEVICE bf16x8v frag_km(const uint16_t* T, int kk, int cb, int lane) {
  const int g = lane >> 4;
  const int r0 = kk + 8 * (g >> 1);
  const int c0 = cb + 16 * (g & 1);
  const u16x4 lo = ld_tr(T, r0, c0, lane & 15);
  const u16x4 hi = ld_tr(T, r0 + 4, c0, lane & 15);
  const u16x8 v = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
  return __builtin_bit_cast(bf16x8v, v);
}

// 16x16x32 operand from the k-major image: lane l holds column cb + (l & 15), k = kk + 8 (l >> 4) + 0..7
DLLM_DEVICE bf16x8v frag_km16(const uint16_t* T, int kk, int cb, int lane) {
  const int r0 = kk + 8 * (lane >> 4);
  const u16x4 lo = ld_tr(T, r0, cb, lane & 15);
  const u16x4 hi = ld_tr(T, r0 + 4, cb, lane & 15);
  const u16x8 v = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
  return __builtin_bit_cast(bf16x8v, v);
}

// ---- row-major [256][BK] image (k contiguous)
// S16 (BK = 32 with 16x16x32 fragments): a ds_read_b128 lane group of frag16 touches rows {0-3, 12-15} at chunk c and
// rows 4-11 at chunk c^1 (rows 16 apart repeat the pattern); with 4 rows per 256-B bank row, chunk c ^ (2 * bit 3 of r)
// puts those 16 reads on 16 distinct bank slots (the BK = 32 32x32x16 swizzle (r / 4) & 3 would 2-way conflict).
template <int BK, bool S16 = false>
struct RowImg {
  static constexpr int CPR = BK / 8;          // 16-B chunks per row
  static constexpr int RPB = 256 / (BK * 2);  // rows per 256-B bank row
  static constexpr int RPI = 1024 / (BK * 2); // rows per 1-KB DMA wave-instruction
  static DLLM_DEVICE int swz(int r) {
    if constexpr (S16 && BK == 32) return ((r >> 3) & 1) << 1;
    else return (r / RPB) & (CPR - 1);
  }
  // 32x32x16 operand: lane l holds row cb + (l & 31), k = kk + 8 (l >> 5) + 0..7
  static DLLM_DEVICE bf16x8v frag(const uint16_t* T, int kk, int cb, int lane) {
    const int r = cb + (lane & 31);
    const int c = (kk >> 3) + (lane >> 5);
    const u16x8 v = *reinterpret_cast<const u16x8*>(T + r * BK + ((c ^ swz(r)) << 3));
    return __builtin_bit_cast(bf16x8v, v);
  }
  // 16x16x32 operand: lane l holds row cb + (l & 15), k = kk + 8 (l >> 4) + 0..7 (conflict-free at BK = 64)
  static DLLM_DEVICE bf16x8v frag16(const uint16_t* T, int kk, int cb, int lane) {
    const int r = cb + (lane & 15);
    const int c = (kk >> 3) + (lane >> 4);
    const u16x8 v = *reinterpret_cast<const u16x8*>(T + r * BK + ((c ^ swz(r)) << 3));
    return __builtin_bit_cast(bf16x8v, v);
  }
};

// GELU (erf, tanh) with its derivative: csrc/gelu.h (shared with csrc/gemm_w4.hip's GELU epilogues)
using dllm_gelu::gelu_pair;
using dllm_gelu::gelu_tanh_pair;

DLLM_DEVICE void store4(uint16_t* p, f32x4 v) {
  const u16x4 o = {f2bf(v.x), f2bf(v.y), f2bf(v.z), f2bf(v.w)};
  *reinterpret_cast<u16x4*>(p) = o;
}

DLLM_DEVICE f32x4 load4(const uint16_t* p) {
  const u16x4 r = *reinterpret_cast<const u16x4*>(p);
  return f32x4{bf2f(r.x), bf2f(r.y), bf2f(r.z), bf2f(r.w)};
}

// v = accumulators (+ bias, added by the caller from registers loaded once) for C[m][n .. n+3] (n % 4 == 0)
// GELU forwards write G = dropout'(.) * act'(U) (the keep mask and 1/(1-p) already applied) as the second output, so
// their backward epilogues are one multiply: dU = (dY Wo) * G — no activation math and no hash in the backward.
template <int EPI>
DLLM_DEVICE f32x4 epilogue4(const GemmFusedParams& P, uint32_t seed, int m, int n, f32x4 v) {
  const bool drop = P.p > 0.f;
  if (EPI == EPI_RELU) {
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = fmaxf(v[k], 0.f);
    // FFN activation dropout: the row-Weyl hash of (row m, column n) (common.h rw_*; the w4 epilogues' decisions)
    if (drop) rw_dropout4(v, mix32(seed, (uint32_t)m), rw_t2(P.thr), (uint32_t)n, P.scale);
  } else if (EPI == EPI_GELU || EPI == EPI_GELU_TANH) {
    f32x4 dg;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      float g, d;
      if (EPI == EPI_GELU) gelu_pair(v[k], g, d);
      else gelu_tanh_pair(v[k], g, d);
      v[k] = g;
      dg[k] = d;
    }
    if (drop) {  // row-Weyl decisions of (row m, columns n ..) as the ReLU branch
      const f32x4 sc = rw_scale4(rw_gbase(mix32(seed, (uint32_t)m), (uint32_t)n >> 1), rw_t2(P.thr), P.scale);
      v = v * sc;
      dg = dg * sc;
    }
    store4(P.aux_out + (long)m * P.ldaux + n, dg);
  } else if (EPI == EPI_DRELU) {
    // H = dropout(relu(u)) was stored by the forward: dH/du = (H != 0) * scale
    const u16x4 h = *reinterpret_cast<const u16x4*>(P.aux + (long)m * P.ldaux + n);
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = (h[k] & 0x7fff) ? v[k] * P.scale : 0.f;
  } else if (EPI == EPI_DGELU || EPI == EPI_DGELU_TANH) {
    v = v * load4(P.aux + (long)m * P.ldaux + n);
  } else if (EPI == EPI_DGEGLU) {
    // gated backward: dH (this GEMM, N = F columns) -> [d gate | d up] = [dH * G1 | dH * G2] in the [M][2F] layout of
    // the stacked wi output; G1 = s * gelu'(gate) * up, G2 = s * gelu(gate) stored by the forward (s = keep / (1 - p))
    const f32x4 g1 = load4(P.aux + (long)m * P.ldaux + n);
    const f32x4 g2 = load4(P.aux2 + (long)m * P.ldaux + n);
    store4(P.C + (long)m * P.ldc + P.N + n, v * g2);
    v = v * g1;
  }
  store4(P.C + (long)m * P.ldc + n, v);
  return v;
}

// Forward activation of epilogue4 without its stores (the ping-pong kernel's LDS-staged epilogue stores whole rows):
// returns act(v) with dropout, and in dg the GELU forwards' second output
template <int EPI>
DLLM_DEVICE f32x4 act4(const GemmFusedParams& P, uint32_t seed, int m, int n, f32x4 v, f32x4& dg) {
  const bool drop = P.p > 0.f;
  if (EPI == EPI_RELU) {
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = fmaxf(v[k], 0.f);
    // FFN activation dropout: the row-Weyl hash of (row m, column n) (common.h rw_*; the w4 epilogues' decisions)
    if (drop) rw_dropout4(v, mix32(seed, (uint32_t)m), rw_t2(P.thr), (uint32_t)n, P.scale);
  } else if (EPI == EPI_GELU || EPI == EPI_GELU_TANH) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      float g, d;
      if (EPI == EPI_GELU) gelu_pair(v[k], g, d);
      else gelu_tanh_pair(v[k], g, d);
      v[k] = g;
      dg[k] = d;
    }
    if (drop) {  // row-Weyl decisions of (row m, columns n ..) as the ReLU branch
      const f32x4 sc = rw_scale4(rw_gbase(mix32(seed, (uint32_t)m), (uint32_t)n >> 1), rw_t2(P.thr), P.scale);
      v = v * sc;
      dg = dg * sc;
    }
  }
  return v;
}

// PP_STAGE: the ping-pong kernel's GELU forward epilogues (two outputs) go through a 4 KB per-wave LDS scratch after
// the operand ring and leave as whole 128-B rows (A/B: -DPP_STAGE=0)
#ifndef PP_STAGE
#define PP_STAGE 1
#endif
#ifndef PP_STAGE_BWD
#define PP_STAGE_BWD 1
#endif

// MF = 32: v_mfma_f32_32x32x16_bf16, 4x2 accumulator tiles of 32x32 per wave;
// MF = 16: v_mfma_f32_16x16x32_bf16, 8x4 tiles of 16x16 (same cycles per FLOP; on random data the chip holds a
// higher clock on this shape, MI355X_MICROARCH.md "DVFS give-back" item 7) — both built, the faster picked by
// measurement (tools/gemm_fused_bench.py).
// PRE (16x16 only): all fragments of both 32-deep k-steps of a stage are read before the first MFMA, so the second
// k-step's LDS latency hides under the first k-step's MFMAs (+96 VGPRs of fragments instead of +48).
template <int BK, int NBUF, bool BKM, int EPI, int MF, bool PRE = false>
__global__ __launch_bounds__(NT, 1) void gemm_fused_kernel(GemmFusedParams P) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const uint32_t seed = P.p > 0.f ? eff_seed(P.seed) : P.seed;
  uint16_t* lds = reinterpret_cast<uint16_t*>(smem);  // [NBUF][A image | B image], BK*256 elements each
  using RI = RowImg<BK, MF == 16>;
  constexpr int TILE = BK * 256;
  constexpr int PW = BK / 16;  // 1-KB DMA instructions per wave per operand per stage
  constexpr int LPS = 2 * PW;
  static_assert(NBUF >= 2 && NBUF <= 5 && NBUF * 2 * TILE * 2 <= 160 * 1024, "ring depth");

  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63, hh = lane >> 5;
  const int wm = w >> 2, wn = w & 3;
  const int t = xcd_remap(blockIdx.x, gridDim.x);
  const int m0 = (t / P.tn) * BM, n0 = (t % P.tn) * BN;
  const int nk = P.K / BK;

  // DMA sources.  Row image: instruction q covers rows q*RPI .. +RPI, lane -> (row l / CPR, pos l % CPR).
  const uint16_t* Ag = P.A + (long)m0 * P.lda;
  const uint16_t* Bg = BKM ? P.B + n0 : P.B + (long)n0 * P.ldb;
  long aoff[PW], boff[PW];
#pragma unroll
  for (int i = 0; i < PW; ++i) {
    const int q = w * PW + i;
    const int r = q * RI::RPI + lane / RI::CPR;
    const int c = (lane % RI::CPR) ^ RI::swz(r);
    aoff[i] = (long)r * P.lda + c * 8;
    if (BKM) {  // k-major image: instruction q covers k-rows 2q, 2q+1; lane -> (row 2q + l/32, chunk l%32)
      const int kr = 2 * q + hh;
      boff[i] = (long)kr * P.ldb + (((lane & 31) ^ gsw(kr)) << 3);
    } else {
      boff[i] = (long)r * P.ldb + c * 8;
    }
  }
  const uint32_t lds0 = lds_addr(lds);
  auto issue = [&](int buf, int kt) {
    const long k0 = (long)kt * BK;
    const uint32_t Al = lds0 + (uint32_t)(buf * 2 * TILE) * 2u;
    const uint32_t Bl = Al + TILE * 2u;
    const uint16_t* Bk = BKM ? Bg + k0 * P.ldb : Bg + k0;
#pragma unroll
    for (int i = 0; i < PW; ++i) {
      const uint32_t q = __builtin_amdgcn_readfirstlane(w * PW + i);
      glds16(Ag + k0 + aoff[i], __builtin_amdgcn_readfirstlane(Al + q * 1024u));
      glds16(Bk + boff[i], __builtin_amdgcn_readfirstlane(Bl + q * 1024u));
    }
  };

#pragma unroll
  for (int p = 0; p < NBUF - 1; ++p)
    if (p < nk) issue(p, p);

  // stage `it` must have landed (stages it+1 .. it+NBUF-2 may stay in flight); every wave is done reading the
  // buffer about to be refilled; then the refill of that buffer is issued
  auto stage_sync = [&](int it) {
    const int ahead = min(NBUF - 2, nk - 1 - it);
    if (NBUF >= 5 && ahead >= 3) wait_vm<(NBUF >= 5 ? 3 * LPS : 0)>();
    else if (NBUF >= 4 && ahead >= 2) wait_vm<(NBUF >= 4 ? 2 * LPS : 0)>();
    else if (NBUF >= 3 && ahead >= 1) wait_vm<(NBUF >= 3 ? LPS : 0)>();
    else wait_vm<0>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (it + NBUF - 1 < nk) issue((it + NBUF - 1) % NBUF, it + NBUF - 1);
  };

  if constexpr (MF == 32) {
    f32x16 acc[4][2];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    auto bfrag = [&](const uint16_t* Bs, int kk, int j) {
      const int cb = wn * 64 + 32 * j;
      return BKM ? frag_km(Bs, kk, cb, lane) : RI::frag(Bs, kk, cb, lane);
    };

    for (int it = 0; it < nk; ++it) {
      stage_sync(it);
      const uint16_t* As = lds + (it % NBUF) * 2 * TILE;
      const uint16_t* Bs = As + TILE;
      bf16x8v a[2][4], b[2][2];
#pragma unroll
      for (int i = 0; i < 4; ++i) a[0][i] = RI::frag(As, 0, wm * 128 + 32 * i, lane);
#pragma unroll
      for (int j = 0; j < 2; ++j) b[0][j] = bfrag(Bs, 0, j);
#pragma unroll
      for (int ks = 0; ks < BK / 16; ++ks) {
        const int cur = ks & 1;
        if (ks + 1 < BK / 16) {
#pragma unroll
          for (int i = 0; i < 4; ++i) a[cur ^ 1][i] = RI::frag(As, 16 * (ks + 1), wm * 128 + 32 * i, lane);
#pragma unroll
          for (int j = 0; j < 2; ++j) b[cur ^ 1][j] = bfrag(Bs, 16 * (ks + 1), j);
        }
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)  // swapped roles: D = B_sub A_sub^T -> lane holds row m, 4 consecutive n
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(b[cur][j], a[cur][i], acc[i][j], 0, 0, 0);
        __builtin_amdgcn_s_setprio(0);
      }
    }

    // epilogue: acc[i][j][4g + 0..3] = C[m0 + wm*128 + 32i + (lane & 31)][n0 + wn*64 + 32j + 8g + 4hh + 0..3]
    const int mrow = m0 + wm * 128 + (lane & 31);
    f32x4 bv[2][4];
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int g = 0; g < 4; ++g)
        bv[j][g] = P.bias ? load4(P.bias + n0 + wn * 64 + 32 * j + 8 * g + 4 * hh) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const f32x4 v = {acc[i][j][4 * g], acc[i][j][4 * g + 1], acc[i][j][4 * g + 2], acc[i][j][4 * g + 3]};
          epilogue4<EPI>(P, seed, mrow + 32 * i, n0 + wn * 64 + 32 * j + 8 * g + 4 * hh, v + bv[j][g]);
        }
  } else {
    static_assert(MF == 16 && (BK == 64 || BK == 32) && (!PRE || BK == 64), "16x16x32 images: BK = 64, or 32 (S16)");
    f32x4 acc[8][4];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    auto mfma_block = [&](const bf16x8v (&a)[8], const bf16x8v (&b)[4]) {
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)  // swapped roles: lane holds row m = lane & 15, 4 consecutive n
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[j], a[i], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
    };
    auto load_k = [&](const uint16_t* As, const uint16_t* Bs, int kk, bf16x8v (&a)[8], bf16x8v (&b)[4]) {
#pragma unroll
      for (int i = 0; i < 8; ++i) a[i] = RI::frag16(As, kk, wm * 128 + 16 * i, lane);
#pragma unroll
      for (int j = 0; j < 4; ++j)
        b[j] = BKM ? frag_km16(Bs, kk, wn * 64 + 16 * j, lane) : RI::frag16(Bs, kk, wn * 64 + 16 * j, lane);
    };
    for (int it = 0; it < nk; ++it) {
      stage_sync(it);
      const uint16_t* As = lds + (it % NBUF) * 2 * TILE;
      const uint16_t* Bs = As + TILE;
      if constexpr (PRE) {
        bf16x8v a0[8], b0[4], a1[8], b1[4];
        load_k(As, Bs, 0, a0, b0);
        load_k(As, Bs, 32, a1, b1);
        mfma_block(a0, b0);
        mfma_block(a1, b1);
      } else {
#pragma unroll
        for (int ks = 0; ks < BK / 32; ++ks) {
          bf16x8v a[8], b[4];
          load_k(As, Bs, 32 * ks, a, b);
          mfma_block(a, b);
        }
      }
    }

    // epilogue: acc[i][j][0..3] = C[m0 + wm*128 + 16i + (lane & 15)][n0 + wn*64 + 16j + 4 (lane >> 4) + 0..3]
    const int mrow = m0 + wm * 128 + (lane & 15);
    const int ncol = n0 + wn * 64 + 4 * (lane >> 4);
    f32x4 bv[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) bv[j] = P.bias ? load4(P.bias + ncol + 16 * j) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) epilogue4<EPI>(P, seed, mrow + 16 * i, ncol + 16 * j, acc[i][j] + bv[j]);
  }
}

// ---- ping-pong kernel (variant 8; NT: A [M][K], B [N][K], both k-contiguous; BKM: B [K][N]) -----------------------
// Same 256x256 tile, 8 waves as 2(M) x 4(N), 16x16x32 MFMA, BK = 64 double-buffered [256][64] images (128 KB), but the
// k-tile is cut into 4 PHASES, one per 64x32 quadrant of a wave's 128x64 output (16 MFMAs each), and the two wave
// rows (wm = 0 / 1, one wave of each on every SIMD) run one barrier apart:
//
//   wave row 0:  | L(P)  |b| M(P)  |b| L(P+1) |b| M(P+1) |b| ...     L = ds_reads of the phase's fragments, one
//   wave row 1:  |b| ... | L(P)   |b| M(P)   |b| L(P+1)  |b| ...         8-KB DMA unit pair, counted vmcnt
//                                                                    M = 16 MFMAs of the quadrant
// so on every SIMD one wave's MFMAs cover the other wave's LDS reads and DMA issue (MI355X_MICROARCH.md: two
// waves per SIMD, MFMA and LDS pipes independent).  Quadrants run (m0,n0) (m0,n1) (m1,n1) (m1,n0): phase 0 reads the
// top 64 A rows + the n0 B fragments, phase 1 the n1 B fragments, phase 2 the bottom A rows, phase 3 nothing.
//
// DMA units: a k-tile is 8 units of 64 image rows (8 KB, one global_load_lds_dwordx4 per thread):
//   U0 A 0-63 | U1 A 128-191 | U2 B {0-31, 64-95} | U3 B {128-159, 192-223} | U4 B {32-63, 96-127} | U5 B {160-191,
//   224-255} | U6 A 64-127 | U7 A 192-255          (first read in phase 0, 0, 0, 0, 1, 1, 2, 2)
// Phase q of k-tile kt issues U4,U5 (q = 0) / U6,U7 (q = 1) of kt + 1 and U0,U1 (q = 2) / U2,U3 (q = 3) of kt + 2, then
// waits until everything issued 4 or more phases ago has landed (vmcnt = glds issued in the last 4 phases).  Every
// unit is issued >= 5 phases before its read (RAW: the wait sits in the L section before the read phase's barrier)
// and >= 2 phases after the previous read of its slot (WAR: the reads retire by lgkmcnt before the next barrier).
//
// BKM (dgrad, B = [K][N] k-major, [64][256] image with transposed reads): every quadrant's B fragments span all 64
// k-rows, so phase 0 reads both n0 and n1 B fragments and the B units are k-row quarters (16 rows x 512 B):
//   U0 A 0-63 | U1 A 128-191 | Bk0..Bk3 | U6 A 64-127 | U7 A 192-255 (first read 0, 0, 0 x 4, 2, 2).  Issue:
//   q0 U6 (kt + 1), q1 U7 (kt + 1), q2 U0, U1, Bk0 (kt + 2), q3 Bk1-3 (kt + 2) -> 1 + 1 + 3 + 3 = 8 glds per 4 phases, so the
//   same vmcnt(8) rule retires every unit >= 1 phase before its read, and every refill is >= 2 phases after its last read.
//
// PERSIST: one workgroup per CU walks tiles vt0, vt0 + vstep, ... (the 32 workgroups of an XCD on 32 consecutive
// virtual tiles, grouped as above); the DMA unit stream runs on across tile boundaries (global k-tile counter), so the
// next tile's first units are in flight while the wave rows run the previous tile's epilogue, each inside its own
// L slot (covered by the other row's MFMAs).  The epilogue's NST stores sit in the vmcnt queue between units: the 4
// phases after an epilogue wait for vmcnt(8 + NST) (an under-count when the epilogue also loads: conservative).
template <int EPI, bool BKM, bool PERSIST>
__global__ __launch_bounds__(NT, 1) void gemm_pp_kernel(GemmFusedParams P) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const uint32_t seed = P.p > 0.f ? eff_seed(P.seed) : P.seed;
  uint16_t* lds = reinterpret_cast<uint16_t*>(smem);  // [2][A image | B image], [256][64] each
  using RI = RowImg<64>;
  constexpr int TILE = 64 * 256;
  // staged store-only epilogues: 2 whole-row stores per 16-row block and output (32 instead of 64).  GELU forwards only
  // (two outputs): bart-large +0.45 %; the ReLU forward measured 1 % slower staged (profiles/r4_gemm_pp_stage_ab.txt)
  constexpr bool STAGED = PP_STAGE && (EPI == EPI_GELU || EPI == EPI_GELU_TANH);
  // GELU backward (one tile per workgroup): derivative loads and dU stores as whole rows through the same scratch
  constexpr bool STAGED_BWD = PP_STAGE_BWD && (EPI == EPI_DGELU || EPI == EPI_DGELU_TANH);
  // gated backward (persistent): G1 / G2 rows in and both output halves out as whole rows through the scratch
  constexpr bool STAGED_DGEGLU = PP_STAGE_BWD && EPI == EPI_DGEGLU;
  // (the staged gated backward's loads are consumed before its last stores: 32 stores stay queued)
  constexpr int NST = STAGED ? ((EPI == EPI_GELU || EPI == EPI_GELU_TANH) ? 32 : 16)
                      : STAGED_DGEGLU ? 32
                      : (EPI == EPI_GELU || EPI == EPI_GELU_TANH || EPI == EPI_DGEGLU) ? 64
                      : EPI == EPI_GEGLU ? 48 : 32;
  // gated forward (EPI_GEGLU, NT only): B = the stacked [wi_0; wi_1] weight [2F][K]; tile column block nb covers hidden
  // units f0 = 128 nb .. f0 + 127: image rows 0-127 are wi_0 rows f0.., rows 128-255 wi_1 rows f0.. (two DMA sources),
  // and each wave reads its fragments so that accumulator columns j = 0, 2 are gate and j = 1, 3 the matching up
  // values of the same 16 hidden units (brow below): gelu(gate) * up is formed in registers, the [M][2F] product is
  // never stored.
  constexpr bool GATED = EPI == EPI_GEGLU;
  static_assert(!GATED || !BKM, "gated forward is NT only");
  constexpr int VM_POST = 8 + NST <= 63 ? 8 + NST : 63;

  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  const int wm = w >> 2, wn = w & 3;
  const int T = P.tm * P.tn;
  const int nk = P.K / 64;
  int vt0, vstep, ntw;
  if constexpr (PERSIST) {
    const int G = gridDim.x, b = blockIdx.x, x = b % 8, slot = b / 8;
    const int nwx = G / 8 + (x < G % 8 ? 1 : 0);
    const int ntx = T / 8 + (x < T % 8 ? 1 : 0);
    vt0 = x * (T / 8) + min(x, T % 8) + slot;
    vstep = nwx;
    ntw = slot < ntx ? (ntx - slot + nwx - 1) / nwx : 0;
  } else {
    vt0 = xcd_remap(blockIdx.x, gridDim.x);
    vstep = 0;
    ntw = 1;
  }
  if (ntw == 0) return;
  auto tile_mn = [&](int i, int& tm0, int& tn0) {
    const int t = vt0 + i * vstep;
    int mb = t / P.tn, nb = t % P.tn;
    if (P.grp > 0) {  // the 32 tiles an XCD runs at once cover a grp x (32 / grp) block of tiles (L2 reuse of A, B)
      const int gs = P.grp * P.tn, g = t / gs, r = t % gs;
      const int rows = min(P.grp, P.tm - g * P.grp);
      mb = g * P.grp + r % rows;
      nb = r / rows;
    }
    tm0 = mb * BM;
    tn0 = nb * BN;
  };

  // per-thread DMA source offsets: A units are 64 contiguous rows, B units two 32-row segments 64 apart.  Unit bases
  // are multiples of 16 rows and the swizzle (r / 2) & 7 depends on r mod 16 only, so one chunk offset serves all.
  const int ra = 8 * w + (lane >> 3);
  const int rb = (w < 4 ? 0 : 64) + 8 * (w & 3) + (lane >> 3);
  const int cs = ((lane & 7) ^ RI::swz(ra)) * 8;
  // k-major B: wave-instruction w of a 16-row unit covers k-rows 2w, 2w+1; lane -> (row 2w + lane/32, chunk lane%32),
  // chunk pre-swizzled by gsw (depends on k-row mod 16 only)
  const int kr = 2 * w + (lane >> 5);
  // byte offsets of the thread's 16 B inside a unit: buffer_load ... lds with the unit's (scalar) base in the
  // descriptor keeps the whole address computation in SGPRs (2 VGPRs of offsets instead of 64-bit pointers per unit)
  const uint32_t offA = (uint32_t)(ra * P.lda + cs) * 2u;
  const uint32_t offB = (uint32_t)(BKM ? kr * P.ldb + (((lane & 31) ^ gsw(kr)) << 3) : rb * P.ldb + cs) * 2u;
  auto tile_a = [&](int tm0) { return P.A + (long)tm0 * P.lda; };
  auto tile_b = [&](int tn0) { return BKM ? P.B + tn0 : P.B + (long)(GATED ? tn0 / 2 : tn0) * P.ldb; };
  // gated: image rows 128.. come from wi_1 = rows F.. of B (F = N / 2)
  const long up_rows = GATED ? (long)(P.N / 2 - 128) * P.ldb : 0;
  int m0, n0, m1 = 0, n1 = 0;
  tile_mn(0, m0, n0);
  if (ntw > 1) tile_mn(1, m1, n1);
  const uint16_t *a_cur = tile_a(m0), *b_cur = tile_b(n0), *a_nxt = tile_a(m1), *b_nxt = tile_b(n1);
  int g_cur = 0;  // global k-tile index of the current tile's first k-tile
  const int total = ntw * nk;

  const uint32_t lds0 = lds_addr(lds);
  const uint32_t la = (uint32_t)(8 * w) * 128u;                              // wave's first image row, A units
  const uint32_t lb = (uint32_t)((w < 4 ? 0 : 64) + 8 * (w & 3)) * 128u;     // B units
  // global k-tile g -> (source tile bases, k-tile inside that tile); g is in the current or the next tile
  // (PERSIST launches only with nk >= 2)
  auto src = [&](int g, const uint16_t*& ab, const uint16_t*& bb) {
    int loc = g - g_cur;
    ab = a_cur;
    bb = b_cur;
    if (PERSIST && loc >= nk) {
      loc -= nk;
      ab = a_nxt;
      bb = b_nxt;
    }
    // opaque to the optimizer: otherwise it hoists every unit's descriptor for both tiles out of the loops and runs
    // out of SGPRs (spilling into VGPR lanes); rebuilding a descriptor costs a few SALU ops per unit
    asm volatile("" : "+s"(ab), "+s"(bb));
    return loc;
  };
  auto unitA = [&](int base, int g) {
    const uint16_t *ab, *bb;
    const int kt = src(g, ab, bb);
    const uint32_t dst = lds0 + (uint32_t)((g & 1) * 2 * TILE) * 2u + (uint32_t)base * 128u + la;
    bld16(ab + (long)base * P.lda + kt * 64, offA, __builtin_amdgcn_readfirstlane(dst));
  };
  auto unitB = [&](int base, int g) {
    const uint16_t *ab, *bb;
    const int kt = src(g, ab, bb);
    const uint32_t dst = lds0 + (uint32_t)((g & 1) * 2 * TILE + TILE) * 2u + (uint32_t)base * 128u + lb;
    bld16(bb + (long)base * P.ldb + (GATED && base >= 128 ? up_rows : 0) + kt * 64, offB,
          __builtin_amdgcn_readfirstlane(dst));
  };
  auto unitBk = [&](int u, int g) {  // k-rows 16u .. 16u+15 of global k-tile g
    const uint16_t *ab, *bb;
    const int kt = src(g, ab, bb);
    const uint32_t dst = lds0 + (uint32_t)((g & 1) * 2 * TILE + TILE) * 2u + (uint32_t)(16 * u + 2 * w) * 512u;
    bld16(bb + (long)(kt * 64 + 16 * u) * P.ldb, offB, __builtin_amdgcn_readfirstlane(dst));
  };
  auto issue_units = [&](int q, int k) {
    if constexpr (BKM) {
      switch (q) {
        case 0: unitA(64, k); break;
        case 1: unitA(192, k); break;
        case 2: unitA(0, k); unitA(128, k); unitBk(0, k); break;
        default: unitBk(1, k); unitBk(2, k); unitBk(3, k); break;
      }
    } else {
      switch (q) {
        case 0: unitB(32, k); unitB(160, k); break;
        case 1: unitA(64, k); unitA(192, k); break;
        case 2: unitA(0, k); unitA(128, k); break;
        default: unitB(0, k); unitB(128, k); break;
      }
    }
  };
  auto units_of = [](int q) { return BKM ? (q < 2 ? 1 : 3) : 2; };
  // phase p (p = 4 g + q, p >= -6) issues the units of global k-tile tgt(p)
  auto tgt = [](int p) { return (p >> 2) + ((p & 3) < 2 ? 1 : 2); };
  auto issue = [&](int p) {
    const int k = tgt(p);
    if (k < total) issue_units(p & 3, k);
  };
  // after phase p's issue: retire everything issued at phases <= p - 4; POST: an epilogue's NST stores are queued
  // between those units and this phase's
  auto retire = [&](int p, bool post) {
    int n = 0;
#pragma unroll
    for (int d = 0; d < 4; ++d) n += tgt(p - d) < total ? units_of((p - d) & 3) : 0;
    if (post) {
      // units of phases p-3 .. p-1 + NST stores + units of phase p may stay queued; n counts the units only
      switch (n) {
        case 8: wait_vm<(8 + NST <= 63 ? 8 + NST : 63)>(); break;
        case 7: wait_vm<(7 + NST <= 63 ? 7 + NST : 63)>(); break;
        case 6: wait_vm<(6 + NST <= 63 ? 6 + NST : 63)>(); break;
        case 5: wait_vm<(5 + NST <= 63 ? 5 + NST : 63)>(); break;
        case 4: wait_vm<(4 + NST <= 63 ? 4 + NST : 63)>(); break;
        case 3: wait_vm<(3 + NST <= 63 ? 3 + NST : 63)>(); break;
        case 2: wait_vm<(2 + NST <= 63 ? 2 + NST : 63)>(); break;
        case 1: wait_vm<(1 + NST <= 63 ? 1 + NST : 63)>(); break;
        default: wait_vm<0>(); break;
      }
      return;
    }
    switch (n) {
      case 8: wait_vm<8>(); break;
      case 7: wait_vm<7>(); break;
      case 6: wait_vm<6>(); break;
      case 5: wait_vm<5>(); break;
      case 4: wait_vm<4>(); break;
      case 3: wait_vm<3>(); break;
      case 2: wait_vm<2>(); break;
      case 1: wait_vm<1>(); break;
      default: wait_vm<0>(); break;
    }
  };

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8v a[4][2], b0[2][2], b1[2][2];

  // prologue: phases -6 .. -1 (issue only), then one barrier for everybody and the one-barrier stagger of wave row 1
#pragma unroll
  for (int p = -6; p < 0; ++p) issue(p);
  retire(-1, false);
  __builtin_amdgcn_s_barrier();
  if (wm == 1) __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);

  auto sync_l = [&]() {  // end of an L section
    __builtin_amdgcn_s_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
  };
  auto sync_m = [&]() {  // end of an M section
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };
  auto quad = [&](int qm, int qn, const bf16x8v (&bb)[2][2]) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[4 * qm + i][2 * qn + j] =
              __builtin_amdgcn_mfma_f32_16x16x32_bf16(bb[j][ks], a[i][ks], acc[4 * qm + i][2 * qn + j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };

  // one k-tile = 4 phases.  FULL: every unit of the 4 phases exists (g + 2 < total) -> unconditional issue, fixed vmcnt;
  // POST: first k-tile after an epilogue (its stores are queued between the units)
  // image row of the wave's B fragment for accumulator column block jq (0..3).  The DMA schedule fills image rows
  // {0-31, 64-95, 128-159, 192-223} (read by phase 0's b0) one phase earlier than {32-63, 96-127, 160-191, 224-255}
  // (phase 1's b1), so the gated placement keeps b0 inside the first set: wave wn's gate block for b0 is rows
  // 64 (wn >> 1) + 16 (wn & 1) .. + 15, its up block the same + 128, and b1 takes the blocks 32 rows further.
  auto brow = [&](int jq) {
    return GATED ? (jq & 1) * 128 + (wn >> 1) * 64 + (wn & 1) * 16 + 32 * (jq >> 1) : wn * 64 + 16 * jq;
  };
  auto ktile = [&](int g, auto full, bool post) {
    constexpr bool FULL = decltype(full)::value;
    const uint16_t* As = lds + (g & 1) * 2 * TILE;
    const uint16_t* Bs = As + TILE;
    const int p0 = 4 * g;
    auto iss = [&](int p) {
      if constexpr (FULL) {
        issue_units(p & 3, tgt(p));
        if (PERSIST && post) wait_vm<VM_POST>();
        else wait_vm<8>();
      } else {
        issue(p);
        retire(p, PERSIST && post);
      }
    };
    // phase 0: quadrant (m0, n0)
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
#pragma unroll
      for (int i = 0; i < 4; ++i) a[i][ks] = RI::frag16(As, 32 * ks, wm * 128 + 16 * i, lane);
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        if constexpr (BKM) {
          b0[j][ks] = frag_km16(Bs, 32 * ks, wn * 64 + 16 * j, lane);
          b1[j][ks] = frag_km16(Bs, 32 * ks, wn * 64 + 32 + 16 * j, lane);
        } else {
          b0[j][ks] = RI::frag16(Bs, 32 * ks, brow(j), lane);
        }
      }
    }
    iss(p0);
    sync_l();
    quad(0, 0, b0);
    sync_m();
    // phase 1: quadrant (m0, n1)
    if constexpr (!BKM) {
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int j = 0; j < 2; ++j) b1[j][ks] = RI::frag16(Bs, 32 * ks, brow(2 + j), lane);
    }
    iss(p0 + 1);
    sync_l();
    quad(0, 1, b1);
    sync_m();
    // phase 2: quadrant (m1, n1)
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < 4; ++i) a[i][ks] = RI::frag16(As, 32 * ks, wm * 128 + 64 + 16 * i, lane);
    iss(p0 + 2);
    sync_l();
    quad(1, 1, b1);
    sync_m();
    // phase 3: quadrant (m1, n0), no reads
    iss(p0 + 3);
    sync_l();
    quad(1, 0, b0);
    sync_m();
  };

  // ReLU derivative bit mask (P.mask): 128 bits per thread per tile, bit 16 i + 4 j + r <-> acc[i][j][r], stored as
  // one 16-B word at tile (mb * tn + nb), thread tid — the forward (EPI_RELU) writes it, the backward (EPI_DRELU_M)
  // stages it into LDS with one extra DMA unit at the start of the tile (double-buffered by tile parity) instead of
  // reading the [M, N] bf16 activation back in its epilogue.
  auto mask_word = [&](int tm0, int tn0) { return (long)((tm0 / BM) * P.tn + tn0 / BN) * NT * 4; };
  const uint32_t lds_mask = lds0 + (uint32_t)(4 * TILE) * 2u;  // after the two [A | B] buffers
  auto mask_unit = [&](int i, int tm0, int tn0) {
    bld16(P.mask + mask_word(tm0, tn0), (uint32_t)tid * 16u,
          __builtin_amdgcn_readfirstlane(lds_mask + (uint32_t)(i & 1) * 8192u + (uint32_t)w * 1024u));
  };

  // epilogue: acc[i][j][0..3] = C[m0 + wm*128 + 16i + (lane & 15)][n0 + wn*64 + 16j + 4 (lane >> 4) + 0..3]
  auto epilogue = [&](int tm0, int tn0, int ti) {
    // opaque lane id: otherwise the per-thread parts of the 32 store addresses are hoisted out of the tile loop
    // (PERSIST) and stay live through the main loop
    int ln = lane;
    asm volatile("" : "+v"(ln));
    const int mrow = tm0 + wm * 128 + (ln & 15);
    const int ncol = tn0 + wn * 64 + 4 * (ln >> 4);
    f32x4 bv[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) bv[j] = P.bias ? load4(P.bias + ncol + 16 * j) : f32x4{0.f, 0.f, 0.f, 0.f};
    if constexpr (GATED) {
      // acc[i][2 jj] = gate, acc[i][2 jj + 1] = up for hidden units f .. f + 3 (f - f0 = the gate block's image row, brow)
      const int F = P.N / 2;
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int jj = 0; jj < 2; ++jj) {
          const int m = mrow + 16 * i, f = tn0 / 2 + (wn >> 1) * 64 + (wn & 1) * 16 + 32 * jj + 4 * (ln >> 4);
          const f32x4 gt = acc[i][2 * jj], up = acc[i][2 * jj + 1];
          f32x4 h, g1, g2;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            float a, d;
            gelu_tanh_pair(gt[r], a, d);
            h[r] = a * up[r];
            g1[r] = d * up[r];
            g2[r] = a;
          }
          if (P.p > 0.f) {  // row-Weyl decision of the OUTPUT element (row m, column f), as csrc/act.hip's gated path
            const f32x4 s = rw_scale4(rw_gbase(mix32(seed, (uint32_t)m), (uint32_t)f >> 1), rw_t2(P.thr), P.scale);
            h = h * s;
            g1 = g1 * s;
            g2 = g2 * s;
          }
          store4(P.C + (long)m * P.ldc + f, h);
          store4(P.aux_out + (long)m * P.ldaux + f, g1);
          store4(P.aux_out2 + (long)m * P.ldaux + f, g2);
        }
    } else if constexpr (EPI == EPI_DRELU_M) {
      const u32x4 mw = *reinterpret_cast<const u32x4*>(smem + 4 * TILE * 2 + (ti & 1) * 8192 + tid * 16);
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          f32x4 v = acc[i][j];
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = (mw[i >> 1] >> ((i & 1) * 16 + 4 * j + r)) & 1u ? v[r] * P.scale : 0.f;
          store4(P.C + (long)(mrow + 16 * i) * P.ldc + ncol + 16 * j, v);
        }
    } else if constexpr (STAGED) {
      // per 16-row block: the wave's 16 x 64 outputs (and the GELU derivative) into its 4 KB scratch after the operand
      // ring (16-B chunks XOR-swizzled by row), then 2 whole-row stores per output: 8 full 128-B lines each
      unsigned char* scr = smem + 4 * TILE * 2 + w * 4096;
      constexpr bool TWO = EPI == EPI_GELU || EPI == EPI_GELU_TANH;
      u32x4 bits = {0u, 0u, 0u, 0u};
      const int rho = ln & 15, q = ln >> 4;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          f32x4 dg = {0.f, 0.f, 0.f, 0.f};
          const f32x4 v = act4<EPI>(P, seed, mrow + 16 * i, ncol + 16 * j, acc[i][j] + bv[j], dg);
          if (EPI == EPI_RELU) {
#pragma unroll
            for (int r = 0; r < 4; ++r) bits[i >> 1] |= (v[r] != 0.f ? 1u : 0u) << ((i & 1) * 16 + 4 * j + r);
          }
          const int off = rho * 128 + (((2 * j + (q >> 1)) ^ (rho & 7)) << 4) + 8 * (q & 1);
          *reinterpret_cast<u16x4*>(scr + off) = u16x4{f2bf(v.x), f2bf(v.y), f2bf(v.z), f2bf(v.w)};
          if (TWO) *reinterpret_cast<u16x4*>(scr + 2048 + off) = u16x4{f2bf(dg.x), f2bf(dg.y), f2bf(dg.z), f2bf(dg.w)};
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // other lanes of this wave read what these wrote
#pragma unroll
        for (int st = 0; st < 2; ++st) {
          const int row = 8 * st + (ln >> 3), ch = ln & 7;
          const int off = row * 128 + ((ch ^ (row & 7)) << 4);
          const long m = tm0 + wm * 128 + 16 * i + row;
          const int n = tn0 + wn * 64 + 8 * ch;
          *reinterpret_cast<u16x8*>(P.C + m * P.ldc + n) = *reinterpret_cast<const u16x8*>(scr + off);
          if (TWO) *reinterpret_cast<u16x8*>(P.aux_out + m * P.ldaux + n) = *reinterpret_cast<const u16x8*>(scr + 2048 + off);
        }
        // the next block's scratch writes must not overtake these reads (in-order LDS per wave; the barrier keeps
        // the compiler from moving them)
        __builtin_amdgcn_sched_barrier(0);
      }
      if (EPI == EPI_RELU && P.mask) *reinterpret_cast<u32x4*>(P.mask + mask_word(tm0, tn0) + tid * 4) = bits;
    } else {
      u32x4 bits = {0u, 0u, 0u, 0u};
      // GELU backward: column sums of the stored dU over the wave's 128 rows — the fc1 bias gradient — from registers
      // (otherwise a separate pass re-reads all of dU, [tokens, d_ff] bf16)
      constexpr bool CS = EPI == EPI_DGELU || EPI == EPI_DGELU_TANH;
      f32x4 cs[4] = {};
      if constexpr (STAGED_DGEGLU) {
        // per 16-row block: G1 / G2 rows in as whole 128-B rows (one block ahead) to the wave's scratch (G1 at 0, G2 at
        // 2 KB), dH * G1 / dH * G2 formed in place in the accumulator layout, both [M][2F] halves out as whole rows
        unsigned char* scr = smem + 4 * TILE * 2 + w * 4096;
        const int rho = ln & 15, q = ln >> 4, lrow = ln >> 3, lch = ln & 7;
        auto ldg = [&](int i, u16x8(&a)[4]) __attribute__((always_inline)) {
#pragma unroll
          for (int st = 0; st < 2; ++st) {
            const long m = tm0 + wm * 128 + 16 * i + 8 * st + lrow;
            const long o = m * P.ldaux + tn0 + wn * 64 + 8 * lch;
            a[st] = *reinterpret_cast<const u16x8*>(P.aux + o);
            a[2 + st] = *reinterpret_cast<const u16x8*>(P.aux2 + o);
          }
        };
        u16x8 cur[4], nxt[4];
        ldg(0, cur);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          if (i + 1 < 8) ldg(i + 1, nxt);
#pragma unroll
          for (int st = 0; st < 2; ++st) {
            const int row = 8 * st + lrow;
            const int off = row * 128 + ((lch ^ (row & 7)) << 4);
            *reinterpret_cast<u16x8*>(scr + off) = cur[st];
            *reinterpret_cast<u16x8*>(scr + 2048 + off) = cur[2 + st];
          }
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // other lanes of this wave read what these wrote
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int off = rho * 128 + (((2 * j + (q >> 1)) ^ (rho & 7)) << 4) + 8 * (q & 1);
            const u16x4 a1 = *reinterpret_cast<const u16x4*>(scr + off);
            const u16x4 a2 = *reinterpret_cast<const u16x4*>(scr + 2048 + off);
            const f32x4 v = acc[i][j] + bv[j];
            const f32x4 v1 = v * f32x4{bf2f(a1.x), bf2f(a1.y), bf2f(a1.z), bf2f(a1.w)};
            const f32x4 v2 = v * f32x4{bf2f(a2.x), bf2f(a2.y), bf2f(a2.z), bf2f(a2.w)};
            *reinterpret_cast<u16x4*>(scr + off) = u16x4{f2bf(v1.x), f2bf(v1.y), f2bf(v1.z), f2bf(v1.w)};
            *reinterpret_cast<u16x4*>(scr + 2048 + off) = u16x4{f2bf(v2.x), f2bf(v2.y), f2bf(v2.z), f2bf(v2.w)};
          }
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
          for (int st = 0; st < 2; ++st) {
            const int row = 8 * st + lrow;
            const int off = row * 128 + ((lch ^ (row & 7)) << 4);
            const long m = tm0 + wm * 128 + 16 * i + row;
            uint16_t* cp = P.C + m * P.ldc + tn0 + wn * 64 + 8 * lch;
            *reinterpret_cast<u16x8*>(cp) = *reinterpret_cast<const u16x8*>(scr + off);
            *reinterpret_cast<u16x8*>(cp + P.N) = *reinterpret_cast<const u16x8*>(scr + 2048 + off);
          }
          __builtin_amdgcn_sched_barrier(0);  // the next block's scratch writes stay after these reads
          if (i + 1 < 8) {
#pragma unroll
            for (int e = 0; e < 4; ++e) cur[e] = nxt[e];
          }
        }
      } else if constexpr (STAGED_BWD) {
        // GELU backward: per 16-row block the saved derivative rows come in as whole 128-B rows (prefetched one block
        // ahead) through the wave's 4 KB scratch, each lane multiplies its accumulator layout in place there, and dU
        // leaves as whole rows: 2 + 2 full-line accesses per block instead of 4 + 4 partial ones
        unsigned char* scr = smem + 4 * TILE * 2 + w * 4096;
        const int rho = ln & 15, q = ln >> 4, lrow = ln >> 3, lch = ln & 7;
        auto ldaux = [&](int i, u16x8(&a)[2]) __attribute__((always_inline)) {
#pragma unroll
          for (int st = 0; st < 2; ++st) {
            const long m = tm0 + wm * 128 + 16 * i + 8 * st + lrow;
            a[st] = *reinterpret_cast<const u16x8*>(P.aux + m * P.ldaux + tn0 + wn * 64 + 8 * lch);
          }
        };
        u16x8 cur[2], nxt[2];
        ldaux(0, cur);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          if (i + 1 < 8) ldaux(i + 1, nxt);
#pragma unroll
          for (int st = 0; st < 2; ++st) {
            const int row = 8 * st + lrow;
            *reinterpret_cast<u16x8*>(scr + row * 128 + ((lch ^ (row & 7)) << 4)) = cur[st];
          }
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // other lanes of this wave read what these wrote
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int off = rho * 128 + (((2 * j + (q >> 1)) ^ (rho & 7)) << 4) + 8 * (q & 1);
            const u16x4 a4 = *reinterpret_cast<const u16x4*>(scr + off);
            const f32x4 v = (acc[i][j] + bv[j]) * f32x4{bf2f(a4.x), bf2f(a4.y), bf2f(a4.z), bf2f(a4.w)};
            cs[j] += v;
            *reinterpret_cast<u16x4*>(scr + off) = u16x4{f2bf(v.x), f2bf(v.y), f2bf(v.z), f2bf(v.w)};
          }
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
          for (int st = 0; st < 2; ++st) {
            const int row = 8 * st + lrow;
            const long m = tm0 + wm * 128 + 16 * i + row;
            *reinterpret_cast<u16x8*>(P.C + m * P.ldc + tn0 + wn * 64 + 8 * lch) =
                *reinterpret_cast<const u16x8*>(scr + row * 128 + ((lch ^ (row & 7)) << 4));
          }
          __builtin_amdgcn_sched_barrier(0);  // the next block's scratch writes stay after these reads
          if (i + 1 < 8) {
            cur[0] = nxt[0];
            cur[1] = nxt[1];
          }
        }
      } else {
#pragma unroll
      for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const f32x4 v = epilogue4<EPI>(P, seed, mrow + 16 * i, ncol + 16 * j, acc[i][j] + bv[j]);
          if (EPI == EPI_RELU) {
#pragma unroll
            for (int r = 0; r < 4; ++r) bits[i >> 1] |= (v[r] != 0.f ? 1u : 0u) << ((i & 1) * 16 + 4 * j + r);
          }
          if constexpr (CS) cs[j] += v;
        }
      }
      if (EPI == EPI_RELU && P.mask) *reinterpret_cast<u32x4*>(P.mask + mask_word(tm0, tn0) + tid * 4) = bits;
      if constexpr (CS) {
        if (P.colsum) {  // the 16 lanes of a lane group hold the same 16 columns on 16 different rows
#pragma unroll
          for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              float x = cs[j][r];
              x += __shfl_xor(x, 1);
              x += __shfl_xor(x, 2);
              x += __shfl_xor(x, 4);
              x += __shfl_xor(x, 8);
              cs[j][r] = x;
            }
          if ((ln & 15) == 0) {
            float* cp = P.colsum + (long)(tm0 / 128 + wm) * P.N + ncol;
#pragma unroll
            for (int j = 0; j < 4; ++j) *reinterpret_cast<f32x4*>(cp + 16 * j) = cs[j];
          }
        }
      }
    }
  };

  int g = 0;
  for (int i = 0; i < ntw; ++i) {
    if constexpr (EPI == EPI_DRELU_M) mask_unit(i, m0, n0);  // lands long before the epilogue (>= 8 phases, nk >= 2)
    // post: first k-tile after an epilogue
    int kt = 0;
    for (; kt < nk && g + 2 < total; ++kt, ++g) ktile(g, std::true_type{}, i > 0 && kt == 0);
    for (; kt < nk; ++kt, ++g) ktile(g, std::false_type{}, i > 0 && kt == 0);
    if (i + 1 < ntw) {  // PERSIST only: epilogue inside the staggered stream, then the next tile becomes current
      __builtin_amdgcn_sched_barrier(0);
      epilogue(m0, n0, i);
      __builtin_amdgcn_sched_barrier(0);  // keep the accumulator reset (and the next fragments) after the epilogue
#pragma unroll
      for (int r = 0; r < 8; ++r)
#pragma unroll
        for (int c = 0; c < 4; ++c) acc[r][c] = f32x4{0.f, 0.f, 0.f, 0.f};
      __builtin_amdgcn_sched_barrier(0);
      m0 = m1;
      n0 = n1;
      a_cur = a_nxt;
      b_cur = b_nxt;
      g_cur += nk;
      if (i + 2 < ntw) {
        tile_mn(i + 2, m1, n1);
        a_nxt = tile_a(m1);
        b_nxt = tile_b(n1);
      }
    }
  }
  if (wm == 0) __builtin_amdgcn_s_barrier();  // undo the stagger: every wave has passed the same number of barriers
  if constexpr (EPI == EPI_DRELU_M) {  // last tile: its mask unit may be < 4 phases old when nk == 1
    wait_vm<0>();
    __builtin_amdgcn_s_barrier();
  }
  epilogue(m0, n0, ntw - 1);
}

int num_cus() {
  static int n = [] {
    int dev = 0, cus = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    return cus > 0 ? cus : 256;
  }();
  return n;
}

// persist: one workgroup per CU when there are >= 2 tiles per CU and >= 2 k-tiles per tile, for the store-only
// epilogues (none / ReLU / GELU forward / ReLU backward from the bit mask, whose only load is an LDS-DMA unit).  The
// GELU backward loads its aux tile in the epilogue: that first load waits in order behind the next tile's queued DMA
// units and the persistent form measured 7-17 % SLOWER (profiles/r1_gemm_experiments.md), so it keeps one tile per
// workgroup.
template <int EPI, bool BKM>
int launch_pp(const GemmFusedParams& p, bool persist, hipStream_t st) {
  constexpr bool staged = (PP_STAGE && (EPI == EPI_GELU || EPI == EPI_GELU_TANH)) ||
                          (PP_STAGE_BWD && (EPI == EPI_DGELU || EPI == EPI_DGELU_TANH || EPI == EPI_DGEGLU));
  const size_t lds = (size_t)2 * 2 * 64 * 256 * 2 + (EPI == EPI_DRELU_M ? 2 * 8192 : 0) + (staged ? 8 * 4096 : 0);
  const int T = p.tm * p.tn, cus = num_cus() / 8 * 8;
  // the gated forward is store-only too; its backward (two aux loads per accumulator block) measured 6-10 % faster
  // persistent as well (profiles/r2_geglu_bench.jsonl); the GELU forward (two stores, no loads) is persistent too:
  // +0.9 % on the bart-large b=256 step in round 4 (profiles/r4_gelu_persist_ab.txt)
  const bool light = EPI == EPI_NONE || EPI == EPI_RELU || EPI == EPI_DRELU_M || EPI == EPI_GEGLU ||
                     EPI == EPI_DGEGLU || EPI == EPI_GELU || EPI == EPI_GELU_TANH;
  if (light && persist && cus >= 8 && T >= 2 * cus && p.K >= 128) {
    static bool attr = false;
    if (!attr) {
      (void)hipFuncSetAttribute((const void*)gemm_pp_kernel<EPI, BKM, true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)lds);
      attr = true;
    }
    hipLaunchKernelGGL((gemm_pp_kernel<EPI, BKM, true>), dim3(cus), dim3(NT), lds, st, p);
  } else {
    static bool attr = false;
    if (!attr) {
      (void)hipFuncSetAttribute((const void*)gemm_pp_kernel<EPI, BKM, false>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
      attr = true;
    }
    hipLaunchKernelGGL((gemm_pp_kernel<EPI, BKM, false>), dim3(T), dim3(NT), lds, st, p);
  }
  DLLM_CHECK_LAUNCH();
  return 0;
}

template <int BK, int NBUF, bool BKM, int EPI, int MF, bool PRE = false>
int launch(const GemmFusedParams& p, hipStream_t st) {
  const size_t lds = (size_t)NBUF * 2 * BK * 256 * 2;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)gemm_fused_kernel<BK, NBUF, BKM, EPI, MF, PRE>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr = true;
  }
  hipLaunchKernelGGL((gemm_fused_kernel<BK, NBUF, BKM, EPI, MF, PRE>), dim3(p.tm * p.tn), dim3(NT), lds, st, p);
  DLLM_CHECK_LAUNCH();
  return 0;
}

template <bool BKM, int EPI>
int launch_v(const GemmFusedParams& p, int variant, hipStream_t st) {
  switch (variant) {
    case 1: return launch<32, 4, BKM, EPI, 32>(p, st);
    case 8: return launch_pp<EPI, BKM>(p, false, st);
    case 9: return launch_pp<EPI, BKM>(p, true, st);
    default: return -6;
  }
}

template <bool BKM>
int dispatch_epi(const GemmFusedParams& p, int variant, hipStream_t st) {
  switch (p.epi) {
    case EPI_NONE: return launch_v<BKM, EPI_NONE>(p, variant, st);
    case EPI_RELU: return launch_v<BKM, EPI_RELU>(p, variant, st);
    case EPI_GELU: return launch_v<BKM, EPI_GELU>(p, variant, st);
    case EPI_GELU_TANH: return launch_v<BKM, EPI_GELU_TANH>(p, variant, st);
    case EPI_DRELU: return launch_v<BKM, EPI_DRELU>(p, variant, st);
    case EPI_DGELU: return launch_v<BKM, EPI_DGELU>(p, variant, st);
    case EPI_DGELU_TANH: return launch_v<BKM, EPI_DGELU_TANH>(p, variant, st);
    case EPI_DRELU_M: return variant == 8 ? launch_pp<EPI_DRELU_M, BKM>(p, false, st)
                                          : variant == 9 ? launch_pp<EPI_DRELU_M, BKM>(p, true, st) : -6;
    case EPI_GEGLU:  // ping-pong kernel only (its fragment placement pairs gate and up), NT only
      if constexpr (BKM) return -6;
      else return variant == 8 || variant == 9 ? launch_pp<EPI_GEGLU, false>(p, variant == 9, st) : -6;
    case EPI_DGEGLU: return variant == 8 || variant == 9 ? launch_pp<EPI_DGEGLU, BKM>(p, variant == 9, st) : -6;
    default: return -5;
  }
}

}  // namespace

// variant: 1 = the staged kernel, BK32 x 4 stages, 32x32x16 MFMA (reduction lengths K % 64 != 0), 8 = ping-pong kernel
// gemm_pp_kernel, 9 = its persistent form (the default for K % 64 == 0).  Variants 0 and 2-7 (other BK / stage / MFMA
// shapes of the staged kernel, all slower than the ping-pong kernel on every T5 / BART shape,
// profiles/r1_gemm_experiments.md) were deleted in round 6.
extern "C" int dllm_gemm_fused(const GemmFusedParams* pp, int b_kmajor, int variant, hipStream_t st) {
  const GemmFusedParams& p = *pp;
  const int bk = variant >= 8 ? 64 : 32;
  if (p.M % BM || p.N % BN || p.K <= 0 || p.K % bk || p.tm * BM != p.M || p.tn * BN != p.N) return -4;
  return b_kmajor ? dispatch_epi<true>(p, variant, st) : dispatch_epi<false>(p, variant, st);
}

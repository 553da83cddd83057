// Projection GEMMs on ONE WAVE PER SIMD for gfx950 (MI355X / CDNA4):
//
//   NT (forward):  C[M][N] (+)= A[M][K] . B[N][K]^T (+ bias)   A = activations [tokens][in], B = nn.Linear weight [out][in]
//   NN (dgrad):    C[M][N] (+)= A[M][K] . B[K][N]              A = output gradient [tokens][out], B = weight (k-major)
//
// Why this shape of kernel (profiles/r2_gemm_pmc_pp_vs_hipblaslt.txt): the 8-wave ping-pong kernel of
// csrc/gemm_fused.hip re-reads A/B fragments for 128x64 sub-tiles, rebuilds buffer descriptors around every DMA
// (4x hipBLASLt's SALU count) and parks its waves 38 % of their cycles at barriers.  Here:
//
// * 256x256 output tile per 256-thread workgroup, 4 waves as 2(M) x 2(N), 128x128 per wave = 8x8
//   v_mfma_f32_16x16x32_bf16 accumulators: 256 fp32 per lane, which the allocator places in the AGPR half of the
//   unified 512-register file (__launch_bounds__(256, 1): one wave per SIMD).  Per 64-deep k-tile a wave issues 128
//   MFMAs against 32 fragment reads (ds_read_b128 / 2x ds_read_b64_tr_b16): 4 MFMAs per LDS read, twice the ratio of
//   the 8-wave kernel;
// * operands go global -> LDS by LDS-DMA (buffer_load_dwordx4 ... lds), 16 per wave per k-tile.  Descriptors are
//   built ONCE per tile in SGPRs, the per-lane offsets live in 16 VGPRs, the k-tile advance is one VALU add per DMA
//   and M0 is written by the DMA statement itself (no save / restore): 1 SALU per DMA;
// * two 64-KB LDS buffers (k-tile t in buffer t & 1), ONE barrier per k-tile, placed 8 MFMAs into the k-tile's
//   second 32-deep sub-step: after it the DMA of k-tile t+2 (into the buffer k-tile t just left) and the fragment
//   reads of k-tile t+1 are issued between the remaining 56 MFMAs, so the LDS latency of the next sub-step and the
//   DMA issue hide under matrix work and the DMA has one full k-tile of MFMAs to land;
// * the instruction interleave is pinned in 8-MFMA chunks (sched_barrier between chunks; inside a chunk the
//   compiler's own lgkmcnt bookkeeping places the waits);
// * ragged M / N: the descriptors' range check returns 0 for rows past the edge (NT) and per-lane offsets of columns
//   past N are pushed out of range (NN); stores are masked.  K % 64 == 0;
// * epilogue: accumulators of row blocks 2i / 2i+1 are packed to bf16 and exchanged between lane rows with
//   v_permlane16_swap, so every lane stores 16 contiguous bytes (32 stores per wave instead of 64 of 8 B,
//   cdna_hip_programming.md T21);
// * bijective XCD remap of the 1-D grid, tiles grouped grp x (32 / grp) per XCD for L2 reuse of A and B.
#include "common.h"

#include <algorithm>
#include <cstdlib>
#include <type_traits>

#include "gelu.h"
#include "gemm_params.h"
#include "route.h"

using namespace dllm;

DLLM_SEED_STEP_TU(gemm_w4)

namespace {

// epilogues: none; ReLU + dropout with the bit mask of kept positive outputs (forward, NT); the input gradient
// through that mask, dU = dH * scale where the bit is set (backward, NN).  The mask is what the backward needs of
// the forward: no re-read of H, no re-hash (T5 FFN, ops/ffn.py).
// LM-head cross-entropy (ops/lm_head.py): CEF = forward partials (no C), CEB = dlogits (gemm_params.h)
// Weight gradient (WG, "TN"): C[M][N] (+)= A^T B with BOTH operands token-major (A = dY [K][M], B = X [K][N]): the A
// image is k-major like the NN B operand (transposed fragment reads), K is split over workgroups (tile index = split x
// output tile, one tile per workgroup) and each split stores its fp32 product to a slab of ws (reduced into C by
// csrc/gemm.hip's split-K pass), or — one split — accumulates straight into the fp32 / bf16 C.
// GELU (erf) FFN: forward NT + bias writing h and its dropout-scaled derivative (two outputs, as csrc/gemm_fused.hip's
// epilogue 2), backward NN multiplying by that derivative and summing dU per 128 rows (csrc/gemm_fused.hip epilogue 4)
enum { W4_EPI_NONE = 0, W4_EPI_RELU = 1, W4_EPI_DRELU_M = 7, W4_EPI_CEF = 8, W4_EPI_CEB = 9, W4_EPI_WG = 10,
       W4_EPI_GELU = 11, W4_EPI_DGELU = 12 };

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8v;
typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef __attribute__((ext_vector_type(2))) uint32_t u32x2;

constexpr int NT = 256, BK = 64;
constexpr uint32_t kOOB = 0x80000000u;  // a buffer offset past every descriptor's range: the load returns 0

DLLM_DEVICE int xcd_remap(int bid, int nblk) {
  const int q = nblk / 8, r = nblk % 8, x = bid % 8;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + bid / 8;
}

// raw buffer descriptor over [base, base + bytes): offsets >= bytes read as 0 (stride 0 -> byte range check)
DLLM_DEVICE i32x4 make_srd(const void* base, uint32_t bytes) {
  const uint64_t a = (uint64_t)base;
  i32x4 r;
  r.x = __builtin_amdgcn_readfirstlane((int)(uint32_t)a);
  r.y = __builtin_amdgcn_readfirstlane((int)((uint32_t)(a >> 32) & 0xFFFFu));
  r.z = __builtin_amdgcn_readfirstlane((int)bytes);
  r.w = 0x00020000;
  return r;
}

// 16 B per lane from srd + voff + soff to LDS byte ldsb + IMM + 16 * lane.  The per-lane offset is fixed for the
// whole kernel, the k-tile advance is the wave-uniform soff, and M0 is formed by the DMA statement itself (written
// here and nowhere else; clobbered, not saved): 1 SALU + the M0 -> LDS-DMA wait state per DMA, no VALU.  Invisible to
// the compiler's vmcnt bookkeeping (as glds16 in common.h); retired by the explicit counted waits below.
template <uint32_t IMM>
DLLM_DEVICE void dma16(const i32x4& srd, uint32_t voff, uint32_t soff, uint32_t ldsb) {
  asm volatile("s_add_u32 m0, %3, %4\n\ts_nop 0\n\tbuffer_load_dwordx4 %0, %1, %2 offen lds"
               :
               : "v"(voff), "s"(srd), "s"(soff), "s"(ldsb), "i"(IMM)
               : "memory", "m0", "scc");
}

// descriptor moved forward by `bytes` (base up, range down): the k-major B operand's k-tile advance
DLLM_DEVICE i32x4 srd_advance(const i32x4& s, uint32_t bytes) {
  const uint64_t a = (((uint64_t)(uint32_t)s.y & 0xFFFFu) << 32 | (uint32_t)s.x) + bytes;
  i32x4 r;
  r.x = (int)(uint32_t)a;
  r.y = (int)((uint32_t)(a >> 32) & 0xFFFFu);
  r.z = (int)((uint32_t)s.z - bytes);
  r.w = s.w;
  return r;
}

// which of a chunk's n DMAs rides on its MFMA j (DMA k on MFMA 1 + 7 k / n), or -1
constexpr int dma_slot(int j, int n) {
  for (int k = 0; k < n; ++k)
    if (1 + 7 * k / n == j) return k;
  return -1;
}

template <int B, int E, typename F>
DLLM_DEVICE void sfor(F&& f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>{});
    sfor<B + 1, E>(f);
  }
}

// ---- k-major [64][256] image (512-B rows) of the NN B operand, transposed reads (csrc/gemm_fused.hip layout)
DLLM_DEVICE int gsw(int r) { return ((r & 3) << 2) ^ (((r >> 3) & 1) << 1); }
DLLM_DEVICE uint32_t boff_km(int r, int col) {  // byte offset of (k-row r, column col)
  return (uint32_t)((r << 9) + ((((col >> 3) ^ gsw(r)) << 3) + (col & 7)) * 2);
}

template <typename T>
DLLM_DEVICE T lds_ld(const unsigned char* smem, uint32_t off) {
  return *reinterpret_cast<const T*>(smem + off);
}

// 16x16x32 operand from the k-major image: lane l holds column cb + (l & 15), k = kk + 8 (l >> 4) + 0..7
DLLM_DEVICE bf16x8v frag_km16(const unsigned char* smem, uint32_t img, int kk, int cb, int lane) {
  const int i = lane & 15;
  const int r = kk + 8 * (lane >> 4) + (i >> 2);
  const int col = cb + 4 * (i & 3);
  typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(smem + img + boff_km(r, col)));
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(smem + img + boff_km(r + 4, col)));
  const s16x4 v0 = lo, v1 = hi;
  const u16x8 v = {(uint16_t)v0.x, (uint16_t)v0.y, (uint16_t)v0.z, (uint16_t)v0.w,
                   (uint16_t)v1.x, (uint16_t)v1.y, (uint16_t)v1.z, (uint16_t)v1.w};
  return __builtin_bit_cast(bf16x8v, v);
}

DLLM_DEVICE uint32_t pk2(float a, float b) { return pack_bf16x2(a, b); }

// ReLU of two packed bf16 (a set sign bit -> +0): one v_pk_max_i16
DLLM_DEVICE uint32_t relu2(uint32_t v) {
  uint32_t r;
  asm("v_pk_max_i16 %0, %1, 0" : "=v"(r) : "v"(v));
  return r;
}
// 1 in each nonzero 16-bit half, else 0: one v_pk_min_u16
DLLM_DEVICE uint32_t nz2(uint32_t v) {
  uint32_t r;
  asm("v_pk_min_u16 %0, %1, %2" : "=v"(r) : "v"(v), "s"(0x00010001u));
  return r;
}
// ReLU bit-mask layout (W4_EPI_RELU writes, W4_EPI_DRELU_M reads): in the 32-bit word of one accumulator row, element r
// of column group j (columns 16 j + 4 qd + r) is pair p = 2 j + (r >> 1) of the row, at bit p (even column) or 16 + p
// (odd column) — what nz2 of the packed pair shifted by p gives
DLLM_DEVICE constexpr int mbit(int j, int r) { return 2 * j + (r >> 1) + 16 * (r & 1); }
// 0xFFFF in the low / high half where bit p / 16 + p of w is set (p < 16): both bits moved to the halves' sign
// positions, then one v_pk_ashrrev_i16 by 15
DLLM_DEVICE uint32_t bits2(uint32_t w, int p) {
  uint32_t r;
  asm("v_pk_ashrrev_i16 %0, %1, %2" : "=v"(r) : "s"(0x000F000Fu), "v"(w << (15 - p)));
  return r;
}
// even bits of w to the low half (bit 2k -> k), odd bits to the high half (2k+1 -> 16+k) (Hacker's Delight 7-2
// unshuffle): the ping-pong kernel's 4 j + r bit order -> mbit order
DLLM_DEVICE uint32_t unshuffle32(uint32_t x) {
  uint32_t t = (x ^ (x >> 1)) & 0x22222222u;
  x ^= t ^ (t << 1);
  t = (x ^ (x >> 2)) & 0x0C0C0C0Cu;
  x ^= t ^ (t << 2);
  t = (x ^ (x >> 4)) & 0x00F000F0u;
  x ^= t ^ (t << 4);
  t = (x ^ (x >> 8)) & 0x0000FF00u;
  x ^= t ^ (t << 8);
  return x;
}

// c += b . a^T (16x16x32, bf16): inline asm so the accumulator is pinned to AGPRs ("+a") and the fragments to VGPRs.
// With the builtin, hipcc (ROCm 7.2) spreads the 256 accumulators and 128 fragment registers over both halves of the
// register file and spills ~200 VGPRs.  The asm is opaque to hipcc's hazard recognizer, so the kernel pads the two
// places the builtin would have been padded: after the accumulator zeroing (mfma_init) and before the epilogue reads.
DLLM_DEVICE void mfma(f32x4& c, const bf16x8v& b, const bf16x8v& a) {
  asm("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(c) : "v"(b), "v"(a));
}
// first k-step of a tile: C input 0 (no accumulator zeroing pass)
DLLM_DEVICE void mfma0(f32x4& c, const bf16x8v& b, const bf16x8v& a) {
  asm("v_mfma_f32_16x16x32_bf16 %0, %1, %2, 0" : "=a"(c) : "v"(b), "v"(a));
}
// c += b . a^T with an LDS-DMA riding on it: M0 is formed BEFORE the MFMA, which covers the M0 -> LDS-DMA wait state
// (no s_nop), and the DMA issues right behind it.  One wave per SIMD pays each DMA's issue in MFMA-pipe cycles
// (tools/mfma_dma_probe.hip, profiles/r6_mfma_dma_probe3.txt: ~28 cycles per 1-KB DMA beside 16x16x32 MFMAs, -6 with
// M0 formed early, more when DMAs issue back to back), so the kernel spreads its DMAs one per few MFMAs this way.
template <uint32_t IMM>
DLLM_DEVICE void mfma_dma(f32x4& c, const bf16x8v& b, const bf16x8v& a, const i32x4& srd, uint32_t voff, uint32_t soff,
                          uint32_t ldsb) {
  asm volatile("s_add_u32 m0, %5, %6\n\tv_mfma_f32_16x16x32_bf16 %0, %1, %2, %0\n\tbuffer_load_dwordx4 %3, %4, %7 offen lds"
               : "+a"(c)
               : "v"(b), "v"(a), "v"(voff), "s"(srd), "s"(ldsb), "i"(IMM), "s"(soff)
               : "memory", "m0", "scc");
}
// the first k-step's form of mfma_dma (C input 0)
template <uint32_t IMM>
DLLM_DEVICE void mfma0_dma(f32x4& c, const bf16x8v& b, const bf16x8v& a, const i32x4& srd, uint32_t voff, uint32_t soff,
                           uint32_t ldsb) {
  asm volatile("s_add_u32 m0, %5, %6\n\tv_mfma_f32_16x16x32_bf16 %0, %1, %2, 0\n\tbuffer_load_dwordx4 %3, %4, %7 offen lds"
               : "=a"(c)
               : "v"(b), "v"(a), "v"(voff), "s"(srd), "s"(ldsb), "i"(IMM), "s"(soff)
               : "memory", "m0", "scc");
}
DLLM_DEVICE void mfma_v(f32x4& c, const bf16x8v& b, const bf16x8v& a) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(c) : "v"(b), "v"(a));
}

// RS bit 0 = fragment read schedule: 0 spreads the 16 next-sub-step reads over the 8 chunks (2 per chunk), 1 issues
// them 4 per chunk in the first 4 chunks after they become legal (more MFMA cover for their latency).
// RS bit 1 = direct epilogue stores from the accumulator layout instead of the LDS-staged whole-row stores (A/B).
// RS bits 4..7 = ABLATIONS for timing studies only (results are garbage): 16 no k-loop DMAs, 32 no k-loop fragment
// reads, 64 no k-loop wait + barrier, 128 no epilogue stores (tools/gemm_w4_bench.py --ablate)
// RS bit 9 = buffer b released half-way through sub-step 0 (lgkmcnt(0) + a second barrier): the DMA of k-tile g+2 starts
// there, 8 pieces on sub-step 0's last 32 MFMAs and 8 on sub-step 1's, and sub-step 1's wait keeps those 8 in flight
// (vmcnt(8)) — the DMA issue spread over 88 MFMAs instead of 56 (-4.8 % summed kernel time, bit-identical outputs)
// RS bit 8 = k-loop DMAs fused into MFMAs (mfma_dma: M0 formed early, one DMA every few MFMAs) instead of 2-3 DMA
// statements back to back after each chunk
template <bool BKM, bool BIAS, bool ACC, int RS, int EPI = W4_EPI_NONE>
__global__ __launch_bounds__(NT, 1) void gemm_w4_kernel(GemmW4Params P) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr uint32_t TB = 256 * BK * 2;  // one operand image: 32 KB
  constexpr uint32_t BUF = 2 * TB;       // [A | B] of one k-tile: 64 KB; two buffers

  constexpr bool AKM = EPI == W4_EPI_WG;  // A k-major too (weight gradient)
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = w >> 1, wn = w & 1;

  // ---- tiles of this workgroup.  Blocks are dealt round-robin over the 8 XCDs (b % 8 share one), so XCD x takes a
  // contiguous range of virtual tiles and its slot-th workgroup walks vbase + slot, + nwx, ... (grid == #tiles: one
  // tile each, the bijective XCD remap); virtual tile -> (row block, column block) in groups of grp row blocks,
  // column-major inside a group, so the 32 tiles an XCD runs at once share A and B panels in its L2.
  // (WG: virtual tile = split * tm * tn + output tile, so an XCD's contiguous range shares the splits' k-ranges)
  const int Tmn = P.tm * P.tn, T = AKM ? Tmn * P.splits : Tmn, G = gridDim.x, bid = blockIdx.x, xcd = bid % 8,
            slot = bid / 8;
  const int nwx = G / 8 + (xcd < G % 8 ? 1 : 0);
  const int ntx = T / 8 + (xcd < T % 8 ? 1 : 0);
  const int vbase = xcd * (T / 8) + min(xcd, T % 8) + slot;
  const int ntw = slot < ntx ? (ntx - slot + nwx - 1) / nwx : 0;
  if (ntw == 0) return;
  auto tile_mn = [&](int i, int& m0, int& n0, int& ks) {
    int vt = vbase + i * nwx;
    ks = AKM ? vt / Tmn : 0;
    vt -= ks * Tmn;
    int mb = vt / P.tn, nb = vt % P.tn;
    if (P.grp > 0) {
      const int gs = P.grp * P.tn, g = vt / gs, r = vt % gs;
      const int rows = min(P.grp, P.tm - g * P.grp);
      mb = g * P.grp + r % rows;
      nb = r / rows;
    }
    m0 = mb * 256;
    n0 = nb * 256;
  };
  // k-rows of split ks (WG: of K, or of its deferred segment) / all of K; first k-row of the split's operands
  auto krows = [&](int ks) {
    if (!AKM) return P.K;
    return P.nseg > 0 ? min(P.kchunk, P.seg_rows - (ks % P.seg_chunks) * P.kchunk) : min(P.kchunk, P.K - ks * P.kchunk);
  };
  auto a_at = [&](int ks) {
    return P.nseg > 0 ? P.segA[ks / P.seg_chunks] + (long)(ks % P.seg_chunks) * P.kchunk * P.lda
                      : P.A + (long)ks * P.kchunk * P.lda;
  };
  auto b_at = [&](int ks) {
    if (!AKM) return P.B;
    return P.nseg > 0 ? P.segB[ks / P.seg_chunks] + (long)(ks % P.seg_chunks) * P.kchunk * P.ldb
                      : P.B + (long)ks * P.kchunk * P.ldb;
  };
  // k-major descriptors span the split's k-rows of the view (column overrun: see the DMA offsets below)
  auto srd_a = [&](int m0, int ks) {
    return AKM ? make_srd(a_at(ks) + m0, (uint32_t)(((long)(krows(ks) - 1) * P.lda + P.M - m0) * 2))
               : make_srd(P.A + (long)m0 * P.lda, (uint32_t)(min(P.M - m0, 256) * P.lda * 2));
  };
  auto srd_b = [&](int n0, int ks) {
    return BKM ? make_srd(b_at(ks) + n0, (uint32_t)(((long)(krows(ks) - 1) * P.ldb + P.N - n0) * 2))
               : make_srd(P.B + (long)n0 * P.ldb, (uint32_t)(min(P.N - n0, 256) * P.ldb * 2));
  };

  // ---- per-lane DMA offsets (tile- and k-invariant).  Row image ([256][64], 128-B rows): wave-instruction q covers
  // rows 8q .. 8q+7, lane -> (row 8q + l/8, 16-B chunk (l%8) ^ ((row/2)&7)); rows past M / N fall out of the tile's
  // descriptor range.  K-major image ([64][256], 512-B rows): instruction q covers k-rows 2q, 2q+1, lane -> (k-row
  // 2q + l/32, chunk (l%32) ^ gsw(k-row)).  K-major columns past N are NOT masked: they load neighbouring elements of
  // B's view (the descriptor spans exactly the view, so nothing past it), which only reach output columns >= N, and
  // those are never stored (column j of C depends on column j of B alone).
  uint32_t va[8], vb[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int q = w * 8 + i;
    const int r = 8 * q + (lane >> 3);
    const int c = (lane & 7) ^ ((r >> 1) & 7);
    const int kr = 2 * q + (lane >> 5);
    if (AKM) va[i] = (uint32_t)(kr * P.lda + ((lane & 31) ^ gsw(kr)) * 8) * 2u;
    else va[i] = (uint32_t)(r * P.lda + c * 8) * 2u;
    if (BKM) {
      vb[i] = (uint32_t)(kr * P.ldb + ((lane & 31) ^ gsw(kr)) * 8) * 2u;
    } else {
      vb[i] = (uint32_t)(r * P.ldb + c * 8) * 2u;
    }
  }
  const uint32_t lds0 = lds_addr(smem) + (uint32_t)w * 8192u;  // this wave's 8 KB slice of each operand image
  // the 16 DMAs of one k-tile: instruction d < 8 -> A image bytes (8 w + d) KB, d >= 8 -> B image (8 w + d - 8) KB.
  // Row images advance by soffset (k-tile * 128 B inside the row); the k-major image by moving its descriptor.
  struct Dma {
    i32x4 sa, sb;
    uint32_t soa, sob, ldsb;
  };
  auto dma_plan = [&](const i32x4& sa, const i32x4& sb, int kk, int b) {
    Dma r;
    if constexpr (AKM) {
      r.sa = srd_advance(sa, (uint32_t)kk * (uint32_t)(BK * P.lda * 2));
      r.soa = 0;
    } else {
      r.sa = sa;
      r.soa = (uint32_t)kk * (BK * 2);
    }
    if constexpr (BKM) {
      r.sb = srd_advance(sb, (uint32_t)kk * (uint32_t)(BK * P.ldb * 2));
      r.sob = 0;
    } else {
      r.sb = sb;
      r.sob = (uint32_t)kk * (BK * 2);
    }
    r.ldsb = lds0 + (uint32_t)b * BUF;
    return r;
  };
  auto dma = [&](const Dma& q, auto D) {
    constexpr int d = decltype(D)::value;
    if constexpr (d < 8) dma16<(uint32_t)d * 1024u>(q.sa, va[d], q.soa, q.ldsb);
    else dma16<TB + (uint32_t)(d - 8) * 1024u>(q.sb, vb[d - 8], q.sob, q.ldsb);
  };
  // MFMA (i, j) of a chunk carrying DMA d of k-tile plan q
  auto mfma_dma_d = [&](f32x4& c, const bf16x8v& b, const bf16x8v& a, const Dma& q, auto D) {
    constexpr int d = decltype(D)::value;
    if constexpr (d < 8) mfma_dma<(uint32_t)d * 1024u>(c, b, a, q.sa, va[d], q.soa, q.ldsb);
    else mfma_dma<TB + (uint32_t)(d - 8) * 1024u>(c, b, a, q.sb, vb[d - 8], q.sob, q.ldsb);
  };

  auto mfma_dma0_d = [&](f32x4& c, const bf16x8v& b, const bf16x8v& a, const Dma& q, auto D) {
    constexpr int d = decltype(D)::value;
    if constexpr (d < 8) mfma0_dma<(uint32_t)d * 1024u>(c, b, a, q.sa, va[d], q.soa, q.ldsb);
    else mfma0_dma<TB + (uint32_t)(d - 8) * 1024u>(c, b, a, q.sb, vb[d - 8], q.sob, q.ldsb);
  };

  // ---- fragment reads.  Row image: a[i] = rows wm*128 + 16 i + (l & 15), k chunk kk/8 + (l >> 4), swizzled by
  // ((row / 2) & 7), which does not depend on i: one base offset per 32-deep half, +2 KB per i.
  const int rl = lane & 15, qd = lane >> 4;
  const uint32_t arow = (uint32_t)(wm * 128 + rl), brow = (uint32_t)(wn * 128 + rl);
  const int asw = (int)((arow >> 1) & 7), bsw = (int)((brow >> 1) & 7);
  const uint32_t aoff[2] = {arow * 128u + (uint32_t)((qd ^ asw) << 4), arow * 128u + (uint32_t)(((qd + 4) ^ asw) << 4)};
  const uint32_t boff[2] = {brow * 128u + (uint32_t)((qd ^ bsw) << 4), brow * 128u + (uint32_t)(((qd + 4) ^ bsw) << 4)};
  auto rd_a = [&](int b, int h, int i) {
    if constexpr (AKM) return frag_km16(smem, (uint32_t)b * BUF, 32 * h, wm * 128 + 16 * i, lane);
    else return lds_ld<bf16x8v>(smem, (uint32_t)b * BUF + aoff[h] + (uint32_t)i * 2048u);
  };
  auto rd_b = [&](int b, int h, int j) {
    if constexpr (BKM) return frag_km16(smem, (uint32_t)b * BUF + TB, 32 * h, wn * 128 + 16 * j, lane);
    else return lds_ld<bf16x8v>(smem, (uint32_t)b * BUF + TB + boff[h] + (uint32_t)j * 2048u);
  };

  f32x4 acc[8][8];
  bf16x8v fa0[8], fb0[8], fa1[8], fb1[8];

  // ---- current / next tile.  The DMA stream runs on across tile boundaries: the last two k-tiles of a tile prefetch
  // the first two of the next, which land while the wave rows run the epilogue.  Persistent mode needs nk >= 2
  // (host-checked); with one tile per workgroup the prefetch past the end is clamped to the last k-tile.
  int m0, n0, ks0, m1 = 0, n1 = 0, ks1 = 0;
  tile_mn(0, m0, n0, ks0);
  if (ntw > 1) tile_mn(1, m1, n1, ks1);
  // k-tiles per tile: all of K, or (WG, one tile per workgroup) this split's
  const int nk = krows(ks0) / BK;
  i32x4 sa0 = srd_a(m0, ks0), sb0 = srd_b(n0, ks0), sa1 = srd_a(m1, ks1), sb1 = srd_b(n1, ks1);
  // DMA plan for k-tile kt + 2 of tile i (tile-local numbering; >= nk means the next tile) into buffer b
  auto plan_next = [&](int i, int kt, int b) {
    const int kn = kt + 2;
    const bool cross = kn >= nk && i + 1 < ntw;
    return dma_plan(cross ? sa1 : sa0, cross ? sb1 : sb0, cross ? kn - nk : min(kn, nk - 1), b);
  };

  // ---- mask of a tile for the DRELU_M epilogue: this wave's 64 threads x 32 B by LDS-DMA into the first 2 KB of its
  // output staging rows, issued when the tile starts; it lands under the k-loop (its waits retire it) and is read into
  // registers before the staging rows are reused.
  unsigned char* const scr = smem + 2 * BUF + (uint32_t)w * 8192u;  // this wave's staging rows [32][256 B]
  const uint32_t scr_lds = lds_addr(smem) + 2 * BUF + (uint32_t)w * 8192u;
  const i32x4 srd_mask = make_srd(P.mask, 0xFFFFFFF0u);
  // mask_pp: the ping-pong forward's layout (8 waves of 128x64, 16 B per thread per tile, bit 16 i + 4 j + r of its
  // acc[i][j][r]): this thread's elements of columns 16 j, j < 4 / >= 4, belong to ping-pong wave (wm, 2 wn) /
  // (wm, 2 wn + 1), same lane, same i — their 16-B words are DMA'd instead of this kernel's own 32 B
  const uint32_t pp_thread = (uint32_t)((wm * 4 + 2 * wn) * 64 + lane);
  auto mask_dma = [&](int tm0, int tn0) {
    if constexpr (EPI == W4_EPI_DRELU_M) {
      const uint32_t tile = (uint32_t)((tm0 / 256) * P.tn + tn0 / 256);
      const uint32_t a = P.mask_pp ? (tile * 512u + pp_thread) * 16u : (tile * 256u + (uint32_t)tid) * 32u;
      const uint32_t b = P.mask_pp ? a + 64u * 16u : a + 16u;
      dma16<0>(srd_mask, a, 0u, scr_lds);
      dma16<1024>(srd_mask, b, 0u, scr_lds);
    }
  };
  const uint32_t seed = ((EPI == W4_EPI_RELU || EPI == W4_EPI_GELU) && P.p > 0.f) ? eff_seed(P.seed) : P.seed;

  // ---- prologue: k-tiles 0 and 1 in flight, wait for k-tile 0, read its first half
  mask_dma(m0, n0);
  {
    const Dma q0 = dma_plan(sa0, sb0, 0, 0), q1 = plan_next(0, -1, 1);
    sfor<0, 16>([&](auto D) { dma(q0, D); });
    sfor<0, 16>([&](auto D) { dma(q1, D); });
  }
  wait_vm<16>();
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int j = 0; j < 8; ++j) fb0[j] = rd_b(0, 0, j);
#pragma unroll
  for (int i = 0; i < 8; ++i) fa0[i] = rd_a(0, 0, i);

  // one chunk = the 8 MFMAs of accumulator row i (swapped roles: lane holds row m = 16 i + (l & 15), 4 consecutive n)
  auto chunk = [&](const bf16x8v (&fa)[8], const bf16x8v (&fb)[8], int i) {
#pragma unroll
    for (int j = 0; j < 8; ++j) mfma(acc[i][j], fb[j], fa[i]);
  };
  // first 32-deep step of a tile: C = 0 in the instruction, so no 256-write accumulator zeroing pass
  auto chunk0 = [&](const bf16x8v (&fa)[8], const bf16x8v (&fb)[8], int i) {
#pragma unroll
    for (int j = 0; j < 8; ++j) mfma0(acc[i][j], fb[j], fa[i]);
  };

  int g = 0;  // global k-tile counter (buffer parity)
  int ti = 0;
  do {  // tiles
    // every k-tile runs the same branch-free body: a peeled last k-tile makes the allocator re-assign all 256 AGPRs
    // between loop and tail (~600 v_accvgpr copies), and with a zero-trip path it keeps a VGPR copy of the zeroed
    // accumulators alive (do-while, nk >= 1)
    int kt = 0;
    do {
      // the accumulator zeroing (v_accvgpr_write) must be 2+ wait states before the first asm MFMA reads it as C; hipcc
      // cannot see that read
      asm volatile("s_nop 2" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      const int b = g & 1;
      // RS bit 9 (A/B): buffer b is released by a barrier half-way through sub-step 0 (every wave's reads of its k 32..63
      // half returned), so the DMA of k-tile g+2 into it starts there: 8 of its 16 pieces ride on sub-step 0's last 32
      // MFMAs, 8 on sub-step 1's (the DMA issue spread over 88 MFMAs instead of 56)
      constexpr bool EARLY = (RS & 512) != 0;
      Dma q;
      // sub-step 0 (k 0..31, fragments fa0 / fb0): read the k 32..63 fragments into fa1 / fb1, two per chunk, B first
      // (the next sub-step's first chunk needs all of B and a[0])
      sfor<0, 8>([&](auto I) {
        constexpr int i = decltype(I)::value;
        if constexpr (EARLY && i >= 4) {
          if constexpr (i == 4) {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();
            __builtin_amdgcn_sched_barrier(0);
            q = plan_next(ti, kt, b);
          }
          // DMAs 2 (i - 4), 2 (i - 4) + 1 on MFMAs 1 and 5 of the chunk
          sfor<0, 8>([&](auto J) {
            constexpr int j = decltype(J)::value;
            constexpr int d = 2 * (i - 4) + (j == 5 ? 1 : 0);
            if (kt == 0) {
              if constexpr (j == 1 || j == 5) mfma_dma0_d(acc[i][j], fb0[j], fa0[i], q, std::integral_constant<int, d>{});
              else mfma0(acc[i][j], fb0[j], fa0[i]);
            } else {
              if constexpr (j == 1 || j == 5) mfma_dma_d(acc[i][j], fb0[j], fa0[i], q, std::integral_constant<int, d>{});
              else mfma_v(acc[i][j], fb0[j], fa0[i]);
            }
          });
        } else {
          if (kt == 0) chunk0(fa0, fb0, i);
          else chunk(fa0, fb0, i);
        }
        if constexpr ((RS & 32) != 0) {
        } else if constexpr ((RS & 1) == 0) {
          if (i < 4) {
            fb1[2 * i] = rd_b(b, 1, 2 * i);
            fb1[2 * i + 1] = rd_b(b, 1, 2 * i + 1);
          } else {
            fa1[2 * i - 8] = rd_a(b, 1, 2 * i - 8);
            fa1[2 * i - 7] = rd_a(b, 1, 2 * i - 7);
          }
        } else {
          if (i < 2) {
#pragma unroll
            for (int e = 0; e < 4; ++e) fb1[4 * i + e] = rd_b(b, 1, 4 * i + e);
          } else if (i < 4) {
#pragma unroll
            for (int e = 0; e < 4; ++e) fa1[4 * (i - 2) + e] = rd_a(b, 1, 4 * (i - 2) + e);
          }
        }
        __builtin_amdgcn_sched_barrier(0);
      });
      // sub-step 1 (k 32..63, fa1 / fb1).  After its first chunk: k-tile g+1 landed (its DMA was the last issued; after
      // an epilogue its 32 stores are queued behind it) and every wave is past its reads of buffer b -> barrier; then
      // DMA k-tile g+2 into buffer b and read k-tile g+1's first half into fa0 / fb0, spread over the remaining 7 chunks
      chunk(fa1, fb1, 0);
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (EARLY) {
        // k-tile g+1 landed: everything but the 8 pieces of g+2 issued in sub-step 0 retired (after an epilogue its 32
        // C stores are queued between them; modes whose epilogues issue other counts drain everything there)
        if (kt == 0 && g > 0) {
          if constexpr (!ACC && EPI != W4_EPI_CEF && EPI != W4_EPI_WG && EPI != W4_EPI_GELU && EPI != W4_EPI_DGELU)
            asm volatile("s_waitcnt vmcnt(40) lgkmcnt(0)" ::: "memory");
          else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
        } else {
          asm volatile("s_waitcnt vmcnt(8) lgkmcnt(0)" ::: "memory");
        }
        __builtin_amdgcn_s_barrier();
      } else if constexpr ((RS & 64) == 0) {
        // after an epilogue its 32 C stores are the youngest VMEM ops (CEF stores fewer: drain everything)
        if (kt == 0 && g > 0 && !ACC && EPI != W4_EPI_CEF && EPI != W4_EPI_WG && EPI != W4_EPI_GELU &&
            EPI != W4_EPI_DGELU)
          asm volatile("s_waitcnt vmcnt(32) lgkmcnt(0)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
      }
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (!EARLY) q = plan_next(ti, kt, b);
      sfor<1, 8>([&](auto I) {
        constexpr int i = decltype(I)::value;
        // DMA: instructions 0..7 of A then of B, spread over chunks 1..7 (2, 2, 2, 3, 2, 2, 3); EARLY: the remaining 8
        // (8..15), one per chunk and two in chunk 5
        constexpr int d0 = EARLY ? 8 + (i - 1) + (i > 5 ? 1 : 0) : (i - 1) * 16 / 7;
        constexpr int d1 = EARLY ? 8 + i + (i >= 5 ? 1 : 0) : i * 16 / 7;
        if constexpr ((RS & 256) != 0 && (RS & 16) == 0) {
          // DMA k of the chunk's n rides on MFMA 1 + 7 k / n (1, 4 or 1, 3, 5)
          sfor<0, 8>([&](auto J) {
            constexpr int j = decltype(J)::value;
            constexpr int n = d1 - d0;
            constexpr int k = dma_slot(j, n);
            if constexpr (k >= 0) mfma_dma_d(acc[i][j], fb1[j], fa1[i], q, std::integral_constant<int, d0 + k>{});
            else mfma_v(acc[i][j], fb1[j], fa1[i]);
          });
        } else {
          chunk(fa1, fb1, i);
          if constexpr ((RS & 16) == 0) sfor<d0, d1>([&](auto D) { dma(q, D); });
        }
        // fragments of k-tile g+1 (buffer b ^ 1), first half: B in chunks 1..4, A in chunks 5..7
        if constexpr ((RS & 32) != 0) {
        } else if constexpr ((RS & 1) == 0) {
          if (i <= 4) {
            fb0[2 * i - 2] = rd_b(b ^ 1, 0, 2 * i - 2);
            fb0[2 * i - 1] = rd_b(b ^ 1, 0, 2 * i - 1);
          } else if (i < 7) {
            fa0[3 * (i - 5)] = rd_a(b ^ 1, 0, 3 * (i - 5));
            fa0[3 * (i - 5) + 1] = rd_a(b ^ 1, 0, 3 * (i - 5) + 1);
            fa0[3 * (i - 5) + 2] = rd_a(b ^ 1, 0, 3 * (i - 5) + 2);
          } else {
            fa0[6] = rd_a(b ^ 1, 0, 6);
            fa0[7] = rd_a(b ^ 1, 0, 7);
          }
        } else {
          if (i <= 2) {
#pragma unroll
            for (int e = 0; e < 4; ++e) fb0[4 * (i - 1) + e] = rd_b(b ^ 1, 0, 4 * (i - 1) + e);
          } else if (i <= 4) {
#pragma unroll
            for (int e = 0; e < 4; ++e) fa0[4 * (i - 3) + e] = rd_a(b ^ 1, 0, 4 * (i - 3) + e);
          }
        }
        __builtin_amdgcn_sched_barrier(0);
      });
      ++g;
    } while (++kt < nk);

    // the last MFMAs' results are read by VALU below: 8-pass XDL write -> VALU read needs 11 wait states, which
    // hipcc cannot see through the asm
    asm volatile("s_nop 7\n\ts_nop 7" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    // ---- epilogue.  acc[i][j][r] = C[m0 + wm*128 + 16 i + (l & 15)][n0 + wn*128 + 16 j + 4 (l >> 4) + r].
    // Row blocks 2ii / 2ii+1 packed to bf16 and exchanged with v_permlane16_swap (odd 16-lane rows of X <-> even rows
    // of Y): afterwards lane l holds 8 consecutive columns 16 j + 8 (qd >> 1) of row 32 ii + 16 (qd & 1) + (l & 15).
    // STAGE (default): each 32-row group goes through this wave's 8 KB LDS scratch (row-major, 16-B chunks XOR-swizzled
    // by row: conflict-free both ways) and leaves as whole-row stores, 4 rows x 256 B per instruction = 8 full 128-B
    // lines, instead of 32 rows x 32 B = 32 partial lines from the accumulator layout (the store-bound part of the
    // kernel: tools/gemm_w4_bench.py --ablate).  Stores go through a buffer descriptor over the tile's rows: rows past
    // M fall out of its range, columns past N are pushed out per lane, so every wave issues exactly 32 stores (the
    // vmcnt(32) above counts them).
    if constexpr (EPI == W4_EPI_WG) {
      // ---- weight gradient: acc[i][j] = 4 fp32 of row m0 + wm*128 + 16 i + (l & 15), columns n0 + wn*128 + 16 j +
      // 4 qd .. + 3 (N % 256 == 0: no column edge) -> this split's slab of ws, or C (one split)
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int row = m0 + wm * 128 + 16 * i + rl;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          asm volatile("" : "+a"(acc[i][j]));
          f32x4 v = acc[i][j];
          const int col = n0 + wn * 128 + 16 * j + 4 * qd;
          if (row < P.M) {
            if (P.splits > 1) {
              *reinterpret_cast<f32x4*>(P.ws + ((long)ks0 * P.M + row) * P.N + col) = v;
            } else if (P.c_f32) {
              float* cp = reinterpret_cast<float*>(P.Cw) + (long)row * P.ldc + col;
              if (P.beta) v += *reinterpret_cast<const f32x4*>(cp);
              *reinterpret_cast<f32x4*>(cp) = v;
            } else {
              uint16_t* cp = reinterpret_cast<uint16_t*>(P.Cw) + (long)row * P.ldc + col;
              if (P.beta) {
                const u16x4 c = *reinterpret_cast<const u16x4*>(cp);
                v += f32x4{bf2f(c[0]), bf2f(c[1]), bf2f(c[2]), bf2f(c[3])};
              }
              *reinterpret_cast<u16x4*>(cp) = u16x4{f2bf(v[0]), f2bf(v[1]), f2bf(v[2]), f2bf(v[3])};
            }
          }
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    } else if constexpr (EPI == W4_EPI_CEF) {
      // ---- LM-head CE forward: per row of the tile and per 128-column half (this wave's wn), the online-softmax
      // partial {max, sum exp(x - max), sum x} of the valid vocabulary columns; the row's label logit from whichever
      // lane holds that column.  The 4 lanes qd = 0..3 of a row hold its 4 x 8 columns: shuffles over lane >> 4.
      const int nb = n0 + wn * 128 + 4 * qd;  // chunk-local column of acc[i][j][r]: nb + 16 j + r
      float cb[8][4];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int n = nb + 16 * j + r;
          cb[j][r] = (P.cbias != nullptr && n < P.N) ? P.cbias[P.c0 + n] : 0.f;
        }
      }
      const int pcol = (n0 + wn * 128) >> 7;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int row = m0 + wm * 128 + 16 * i + rl;
        const long yl = row < P.M ? P.labels[row] - (long)P.c0 - nb : -1;  // label column relative to this lane's
        float xs[8][4];
        float mx = -INFINITY;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          asm volatile("" : "+a"(acc[i][j]));
          const f32x4 a = acc[i][j];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int n = nb + 16 * j + r;
            const bool ok = n < P.N && n >= P.skip;
            xs[j][r] = ok ? a[r] + cb[j][r] : -INFINITY;
            mx = fmaxf(mx, xs[j][r]);
          }
        }
        mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
        mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
        float se = 0.f, sx = 0.f;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float x = xs[j][r];
            se += x == -INFINITY ? 0.f : __expf(x - mx);
            sx += x == -INFINITY ? 0.f : x;
            if (yl == 16 * j + r && x != -INFINITY) P.xlab[row] = x;
          }
        }
        se += __shfl_xor(se, 16, 64);
        se += __shfl_xor(se, 32, 64);
        sx += __shfl_xor(sx, 16, 64);
        sx += __shfl_xor(sx, 32, 64);
        // a 128-column half lying wholly past N has no partial slot (pcol == pstride would be the next row's slot 0)
        if (qd == 0 && row < P.M && pcol < P.pstride)
          *reinterpret_cast<f32x4*>(P.part + ((long)row * P.pstride + pcol) * 4) = f32x4{mx, se, sx, 0.f};
        __builtin_amdgcn_sched_barrier(0);
      }
    } else {
      // descriptor inputs made provably wave-uniform (readfirstlane), or hipcc wraps every store in a waterfall loop
      const uint64_t cb = (uint64_t)(P.C + (long)m0 * P.ldc);
      const uint32_t clo = __builtin_amdgcn_readfirstlane((uint32_t)cb), chi = __builtin_amdgcn_readfirstlane((uint32_t)(cb >> 32));
      const __amdgpu_buffer_rsrc_t srdC = __builtin_amdgcn_make_buffer_rsrc(
          (void*)(((uint64_t)chi << 32) | clo), (short)0,
          (int)__builtin_amdgcn_readfirstlane((uint32_t)(min(P.M - m0, 256) * P.ldc * 2)), 0x00020000);
      // GELU: the second output (forward) / the saved derivative (backward), rows m0 .. m0 + 255 of [M][ldaux]
      __amdgpu_buffer_rsrc_t srdX = srdC;
      if constexpr (EPI == W4_EPI_GELU || EPI == W4_EPI_DGELU) {
        const uint64_t xb = EPI == W4_EPI_GELU ? (uint64_t)(P.aux_out + (long)m0 * P.ldaux)
                                               : (uint64_t)(P.aux + (long)m0 * P.ldaux);
        const uint32_t xlo = __builtin_amdgcn_readfirstlane((uint32_t)xb), xhi = __builtin_amdgcn_readfirstlane((uint32_t)(xb >> 32));
        srdX = __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)xhi << 32) | xlo), (short)0,
                                                 (int)__builtin_amdgcn_readfirstlane((uint32_t)(min(P.M - m0, 256) * P.ldaux * 2)),
                                                 0x00020000);
      }
      f32x4 csum[8];  // DGELU: this lane's column sums (columns 16 j + 4 qd + r) over its rows of the wave's 128
#pragma unroll
      for (int j = 0; j < 8; ++j) csum[j] = f32x4{0.f, 0.f, 0.f, 0.f};
      const int mr = wm * 128 + 16 * (qd & 1) + rl;  // tile-local row of ii = 0
      const int nc = wn * 128 + 8 * (qd >> 1);       // tile-local column of j = 0
      uint32_t mw[8];  // mask words: bit 4 j + r of word i <-> acc[i][j][r]
      if constexpr (EPI == W4_EPI_DRELU_M) {
        // the tile's mask DMA is older than every DMA of the last k-tile: at most those 16 are still outstanding
        asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
        const u32x4 lo = *reinterpret_cast<const u32x4*>(scr + 16 * lane);
        const u32x4 hi = *reinterpret_cast<const u32x4*>(scr + 1024 + 16 * lane);
        if (P.mask_pp) {  // word i = [ping-pong (wm, 2wn) bits 16i..16i+15 | (wm, 2wn+1) bits 16i..16i+15]
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            const uint32_t a = (i >> 1) == 0 ? lo.x : (i >> 1) == 1 ? lo.y : (i >> 1) == 2 ? lo.z : lo.w;
            const uint32_t b = (i >> 1) == 0 ? hi.x : (i >> 1) == 1 ? hi.y : (i >> 1) == 2 ? hi.z : hi.w;
            mw[i] = unshuffle32((i & 1) ? ((a >> 16) | (b & 0xFFFF0000u)) : ((a & 0xFFFFu) | (b << 16)));
          }
        } else {
          mw[0] = lo.x; mw[1] = lo.y; mw[2] = lo.z; mw[3] = lo.w;
          mw[4] = hi.x; mw[5] = hi.y; mw[6] = hi.z; mw[7] = hi.w;
        }
      } else {
#pragma unroll
        for (int i = 0; i < 8; ++i) mw[i] = 0u;
      }
      // bias kept as packed bf16 (16 registers instead of 32 fp32), widened where added
      u32x2 bv[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        bv[j] = u32x2{0u, 0u};
        if constexpr (BIAS) {
          const int nb4 = n0 + wn * 128 + 16 * j + 4 * qd;
          if (nb4 < P.N) bv[j] = *reinterpret_cast<const u32x2*>(P.bias + nb4);
        }
      }
      auto bias4 = [&](int j) {
        return f32x4{bf2f((uint16_t)(bv[j].x & 0xFFFFu)), bf2f((uint16_t)(bv[j].x >> 16)),
                     bf2f((uint16_t)(bv[j].y & 0xFFFFu)), bf2f((uint16_t)(bv[j].y >> 16))};
      };
      auto add_c = [&](u32x4 o, uint32_t off) {  // ACC: o + C, in fp32, rounded once
        const u32x4 c = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(srdC, off, 0, 0));
        auto add2 = [](uint32_t u, uint32_t v) {
          return pk2(bf2f((uint16_t)(u & 0xFFFFu)) + bf2f((uint16_t)(v & 0xFFFFu)),
                     bf2f((uint16_t)(u >> 16)) + bf2f((uint16_t)(v >> 16)));
        };
        return u32x4{add2(o.x, c.x), add2(o.y, c.y), add2(o.z, c.z), add2(o.w, c.w)};
      };
      const int rowL = 16 * (qd & 1) + rl;                       // staging row written by this lane
      // CEB: this lane's 8 rows (ii, half): lse, label column relative to the tile's column 0, row gradient scale
      float ce_lse[8], ce_g[8];
      int ce_y[8];
      if constexpr (EPI == W4_EPI_CEB) {
        const float gs = *P.gscale;
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const int row = m0 + wm * 128 + 32 * (q >> 1) + 16 * (q & 1) + rl;
          const long y = row < P.M ? P.labels[row] : P.ignore;
          const bool valid = row < P.M && y != P.ignore && y >= 0 && y < P.V;
          ce_lse[q] = row < P.M ? P.lse[row] : 0.f;
          ce_g[q] = valid ? gs : 0.f;
          const long yt = y - (long)P.c0 - n0;
          ce_y[q] = (yt >= 0 && yt < 256) ? (int)yt : -1;
        }
      }
      const uint32_t t2 = rw_t2(P.thr);  // row-Weyl dropout threshold pair (ReLU forward)
#pragma unroll
      for (int ii = 0; ii < 4; ++ii) {
        // ReLU / GELU forward dropout: row-Weyl bases of this lane's rows 32 ii + rl (x) and + 16 (y) at column pair kp0
        uint32_t rwx = 0u, rwy = 0u;
        if constexpr (EPI == W4_EPI_RELU || EPI == W4_EPI_GELU) {
          if (P.p > 0.f) {
            const uint32_t rx = (uint32_t)(m0 + wm * 128 + 32 * ii + rl);
            const uint32_t kp0 = (uint32_t)(n0 + wn * 128 + 4 * qd) >> 1;
            rwx = rw_gbase(mix32(seed, rx), kp0);
            rwy = rw_gbase(mix32(seed, rx + 16u), kp0);
          }
        }
        u32x2 ga[8][2];  // GELU backward: the saved derivative at this lane's accumulator positions (rows ii, ii + 16)
        if constexpr (EPI == W4_EPI_DGELU) {
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const int col = n0 + wn * 128 + 16 * j + 4 * qd;
            const int row = wm * 128 + 32 * ii + rl;  // tile-local
            const uint32_t o0 = col < P.N ? (uint32_t)(row * P.ldaux + col) * 2u : kOOB;
            const uint32_t o1 = col < P.N ? (uint32_t)((row + 16) * P.ldaux + col) * 2u : kOOB;
            ga[j][0] = __builtin_bit_cast(u32x2, __builtin_amdgcn_raw_buffer_load_b64(srdX, o0, 0, 0));
            ga[j][1] = __builtin_bit_cast(u32x2, __builtin_amdgcn_raw_buffer_load_b64(srdX, o1, 0, 0));
          }
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          // opaque re-definition in place: the AGPR -> VGPR copies cannot be hoisted above this point (otherwise all 256
          // accumulators are copied out at the loop exit: 256 VGPRs + spills)
          asm volatile("" : "+a"(acc[2 * ii][j]), "+a"(acc[2 * ii + 1][j]));
          f32x4 xv = acc[2 * ii][j], yv = acc[2 * ii + 1][j];
          if constexpr (BIAS) {
            const f32x4 b4 = bias4(j);
            xv += b4;
            yv += b4;
          }
          if constexpr (EPI == W4_EPI_RELU) {
            // scaled in fp32 (rounded once, as before); ReLU, dropout and the mask bits follow on the packed pairs
            if (P.p > 0.f) {
              xv *= P.scale;
              yv *= P.scale;
            }
          } else if constexpr (EPI == W4_EPI_DRELU_M) {
            // scaled in fp32 (rounded once); the mask zeroes the packed pairs below
            if (P.p > 0.f) {
              xv *= P.scale;
              yv *= P.scale;
            }
          } else if constexpr (EPI == W4_EPI_GELU) {
            // h = s gelu(u), G = s gelu'(u), s = keep / (1 - p) with the keep bits of the [M][N] element index
            f32x4 gx, gy;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              float g, d;
              dllm_gelu::gelu_pair(xv[r], g, d);
              xv[r] = g;
              gx[r] = d;
              dllm_gelu::gelu_pair(yv[r], g, d);
              yv[r] = g;
              gy[r] = d;
            }
            if (P.p > 0.f) {  // row-Weyl decisions of column pairs kp0 + 8 j, + 1 (as the ReLU forward)
              const f32x4 sx = rw_scale4(rwx + (uint32_t)(8 * j) * RW_G, t2, P.scale);
              const f32x4 sy = rw_scale4(rwy + (uint32_t)(8 * j) * RW_G, t2, P.scale);
              xv *= sx;
              gx *= sx;
              yv *= sy;
              gy *= sy;
            }
            uint32_t g0 = pk2(gx.x, gx.y), g1 = pk2(gx.z, gx.w), h0 = pk2(gy.x, gy.y), h1 = pk2(gy.z, gy.w);
            const auto r0 = __builtin_amdgcn_permlane16_swap(g0, h0, false, false);
            const auto r1 = __builtin_amdgcn_permlane16_swap(g1, h1, false, false);
            // the derivative leaves directly from the swapped layout (16 B per lane, 8 consecutive columns of one
            // row): keeping all 8 for a second staging pass spilled the epilogue
            const int nl = nc + 16 * j;
            const uint32_t goff = n0 + nl < P.N ? (uint32_t)((mr + 32 * ii) * P.ldaux + n0 + nl) * 2u : kOOB;
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(i32x4, u32x4{r0[0], r1[0], r0[1], r1[1]}), srdX,
                                                   goff, 0, 0);
          } else if constexpr (EPI == W4_EPI_DGELU) {
            // dU = dH * G (fp32, rounded once); column sums of dU for the bias gradient
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const uint32_t wx = ga[j][0][r >> 1], wy = ga[j][1][r >> 1];
              xv[r] *= bf2f((uint16_t)((r & 1) ? (wx >> 16) : (wx & 0xFFFFu)));
              yv[r] *= bf2f((uint16_t)((r & 1) ? (wy >> 16) : (wy & 0xFFFFu)));
            }
            csum[j] += xv + yv;
          } else if constexpr (EPI == W4_EPI_CEB) {
            // dlogits = g (softmax - (1 - eps) onehot - eps / V); xv: row q = 2 ii, yv: row q = 2 ii + 1
            const float off = P.eps / (float)P.V, hit = 1.f - P.eps;
            const int nt = wn * 128 + 16 * j + 4 * qd;  // tile column of r = 0
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int n = n0 + nt + r;
              const bool ok = n < P.N && n >= P.skip;
              const float b = (P.cbias != nullptr && n < P.N) ? P.cbias[P.c0 + n] : 0.f;
              xv[r] = ok ? ce_g[2 * ii] * (__expf(xv[r] + b - ce_lse[2 * ii]) - off - (ce_y[2 * ii] == nt + r ? hit : 0.f))
                         : 0.f;
              yv[r] = ok ? ce_g[2 * ii + 1] *
                               (__expf(yv[r] + b - ce_lse[2 * ii + 1]) - off - (ce_y[2 * ii + 1] == nt + r ? hit : 0.f))
                         : 0.f;
            }
          }
          uint32_t x0 = pk2(xv.x, xv.y), x1 = pk2(xv.z, xv.w), y0 = pk2(yv.x, yv.y), y1 = pk2(yv.z, yv.w);
          if constexpr (EPI == W4_EPI_RELU) {
            // ReLU on the bf16 pairs (sign bit set -> 0), then the row-Weyl dropout of column pairs kp0 + 8 j (x0 / y0)
            // and kp0 + 8 j + 1 (x1 / y1), then the kept-and-positive bits: 9 VALU per pair in all (was ~13 per element
            // with fp32 ReLU, a mix32 per pair and per-element bit inserts)
            x0 = relu2(x0);
            x1 = relu2(x1);
            y0 = relu2(y0);
            y1 = relu2(y1);
            if (P.p > 0.f) {
              x0 &= ~rw_drop2(rw_pair_y(rwx + (uint32_t)(8 * j) * RW_G), t2);
              x1 &= ~rw_drop2(rw_pair_y(rwx + (uint32_t)(8 * j + 1) * RW_G), t2);
              y0 &= ~rw_drop2(rw_pair_y(rwy + (uint32_t)(8 * j) * RW_G), t2);
              y1 &= ~rw_drop2(rw_pair_y(rwy + (uint32_t)(8 * j + 1) * RW_G), t2);
            }
            mw[2 * ii] |= (nz2(x0) << (2 * j)) | (nz2(x1) << (2 * j + 1));
            mw[2 * ii + 1] |= (nz2(y0) << (2 * j)) | (nz2(y1) << (2 * j + 1));
          } else if constexpr (EPI == W4_EPI_DRELU_M) {
            // the pair's two mask bits widened to 16-bit halves (3 VALU per pair, was 4 per element)
            x0 &= bits2(mw[2 * ii], 2 * j);
            x1 &= bits2(mw[2 * ii], 2 * j + 1);
            y0 &= bits2(mw[2 * ii + 1], 2 * j);
            y1 &= bits2(mw[2 * ii + 1], 2 * j + 1);
          }
          {
            const auto r0 = __builtin_amdgcn_permlane16_swap(x0, y0, false, false);
            const auto r1 = __builtin_amdgcn_permlane16_swap(x1, y1, false, false);
            x0 = r0[0];
            y0 = r0[1];
            x1 = r1[0];
            y1 = r1[1];
          }
          u32x4 o = {x0, x1, y0, y1};
          if constexpr ((RS & 2) == 0) {  // staged: chunk 2j + (qd >> 1) of staging row rowL, swizzled by the row
            const int cj = 2 * j + (qd >> 1);
            *reinterpret_cast<u32x4*>(scr + rowL * 256 + ((cj ^ (rowL & 15)) << 4)) = o;
          } else {
            const int nl = nc + 16 * j;
            const uint32_t off = n0 + nl < P.N ? (uint32_t)((mr + 32 * ii) * P.ldc + n0 + nl) * 2u : kOOB;
            if constexpr (ACC) o = add_c(o, off);
            if constexpr ((RS & 128) == 0) __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(i32x4, o), srdC, off, 0, 0);
          }
          // bound the live ranges
          if (j & 1) __builtin_amdgcn_sched_barrier(0);
        }
        if constexpr ((RS & 2) == 0) {
          // read back row-major (the same wave's DS instructions execute in order: no barrier, and the next group's
          // writes cannot overtake these reads): store s covers staging rows 4s .. 4s+3, lane -> (row 4s + l/16,
          // 16-B chunk l%16)
#pragma unroll
          for (int s2 = 0; s2 < 8; ++s2) {
            const int r = 4 * s2 + (lane >> 4), c = lane & 15;
            u32x4 o = *reinterpret_cast<const u32x4*>(scr + r * 256 + ((c ^ (r & 15)) << 4));
            const int col = wn * 128 + 8 * c;
            const uint32_t off = n0 + col < P.N ? (uint32_t)((wm * 128 + 32 * ii + r) * P.ldc + n0 + col) * 2u : kOOB;
            if constexpr (ACC) o = add_c(o, off);
            if constexpr ((RS & 128) == 0) __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(i32x4, o), srdC, off, 0, 0);
          }
          __builtin_amdgcn_sched_barrier(0);
          if constexpr (EPI == W4_EPI_RELU) {  // this row group's 2 of the thread's 8 mask words of the tile
            uint32_t* mp = P.mask + (size_t)(((m0 / 256) * P.tn + n0 / 256) * 256 + tid) * 8;
            *reinterpret_cast<u32x2*>(mp + 2 * ii) = u32x2{mw[2 * ii], mw[2 * ii + 1]};
          }
        }
      }
      if constexpr (EPI == W4_EPI_DGELU) {
        // the 16 lanes rl = 0..15 of a quarter qd hold the same columns on 16 rows: fold them, lane rl = 0 stores the
        // wave's 128-row partial row (m0 / 128 + wm) of colsum
#pragma unroll
        for (int j = 0; j < 8; ++j) {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            float v = csum[j][r];
            v += __shfl_xor(v, 1, 64);
            v += __shfl_xor(v, 2, 64);
            v += __shfl_xor(v, 4, 64);
            v += __shfl_xor(v, 8, 64);
            csum[j][r] = v;
          }
        }
        if (rl == 0) {
          float* cp = P.colsum + (long)(m0 / 128 + wm) * P.N + n0 + wn * 128 + 4 * qd;
#pragma unroll
          for (int j = 0; j < 8; ++j)
            if (n0 + wn * 128 + 16 * j + 4 * qd < P.N) *reinterpret_cast<f32x4*>(cp + 16 * j) = csum[j];
        }
      }

    }
    __builtin_amdgcn_sched_barrier(0);
    // next tile becomes current
    m0 = m1;
    n0 = n1;
    ks0 = ks1;
    sa0 = sa1;
    sb0 = sb1;
    if (ti + 1 < ntw) mask_dma(m0, n0);  // the staging rows' reads above returned before their stores issued
    if (ti + 2 < ntw) {
      tile_mn(ti + 2, m1, n1, ks1);
      sa1 = srd_a(m1, ks1);
      sb1 = srd_b(n1, ks1);
    }
  } while (++ti < ntw);
  wait_vm<0>();  // clamped prefetches of the last tile may still be landing in LDS
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

// persist: one workgroup per CU (LDS and registers admit one) walking its tiles, when there are more tiles than CUs
// and at least 2 k-tiles per tile; otherwise one tile per workgroup
template <bool BKM, bool BIAS, bool ACC, int RS, int EPI = W4_EPI_NONE>
int launch_rs(const GemmW4Params& p, bool persist, hipStream_t st) {
  static_assert(EPI == W4_EPI_NONE || (RS & 2) == 0, "epilogues use the staging rows");
  constexpr size_t lds = 2 * 2 * 256 * BK * 2 + ((RS & 2) == 0 ? 4 * 8192 : 0);  // 128 KB (+ 32 KB output staging)
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)gemm_w4_kernel<BKM, BIAS, ACC, RS, EPI>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr = true;
  }
  const int T = p.tm * p.tn * (EPI == W4_EPI_WG ? p.splits : 1), cus = num_cus() / 8 * 8;
  const int grid = EPI != W4_EPI_WG && persist && p.K >= 2 * BK && cus >= 8 && T > cus ? cus : T;
  hipLaunchKernelGGL((gemm_w4_kernel<BKM, BIAS, ACC, RS, EPI>), dim3(grid), dim3(NT), lds, st, p);
  DLLM_CHECK_LAUNCH();
  return 0;
}

// DLLM_ROUTE w4_sched (kernel template RS; ops/routing.py), read per call so microbenchmarks can A/B it in one process;
// the ablation values (bits 4..7) exist for the plain forward only
template <bool BKM, bool BIAS, bool ACC>
int launch(const GemmW4Params& p, bool persist, hipStream_t st) {
  // default 769: early fragment reads, DMAs riding on MFMAs (profiles/r6_w4_dma_interleave_ab.txt), buffer released
  // half-way through sub-step 0 (profiles/r6_w4_early_release_ab.txt)
  const int rs = route_int("w4_sched", 769);
  if constexpr (!BKM && !BIAS && !ACC) {
    switch (rs) {
      case 16: return launch_rs<BKM, BIAS, ACC, 16>(p, persist, st);
      case 32: return launch_rs<BKM, BIAS, ACC, 32>(p, persist, st);
      case 64: return launch_rs<BKM, BIAS, ACC, 64>(p, persist, st);
      case 128: return launch_rs<BKM, BIAS, ACC, 128>(p, persist, st);
      case 112: return launch_rs<BKM, BIAS, ACC, 112>(p, persist, st);
      default: break;
    }
  }
  if (rs & 256) return (rs & 512) ? launch_rs<BKM, BIAS, ACC, 769>(p, persist, st) : launch_rs<BKM, BIAS, ACC, 257>(p, persist, st);
  switch (rs & 3) {  // bit 1: direct (unstaged) epilogue stores, for A/B
    case 0: return launch_rs<BKM, BIAS, ACC, 0>(p, persist, st);
    case 2: return launch_rs<BKM, BIAS, ACC, 2>(p, persist, st);
    case 3: return launch_rs<BKM, BIAS, ACC, 3>(p, persist, st);
    default: return launch_rs<BKM, BIAS, ACC, 1>(p, persist, st);
  }
}

template <bool BKM>
int dispatch(const GemmW4Params& p, bool persist, hipStream_t st) {
  if (p.accumulate) return p.bias ? launch<BKM, true, true>(p, persist, st) : launch<BKM, false, true>(p, persist, st);
  return p.bias ? launch<BKM, true, false>(p, persist, st) : launch<BKM, false, false>(p, persist, st);
}

}  // namespace

// epi: W4_EPI_NONE, W4_EPI_RELU (NT, optional bias, no accumulate), W4_EPI_DRELU_M (NN, no bias, no accumulate)
extern "C" int dllm_gemm_w4(const GemmW4Params* pp, int b_kmajor, int persist, int epi, hipStream_t st) {
  const GemmW4Params& p = *pp;
  const int rsb = route_int("w4_sched", 769);
  const bool il = (rsb & 256) != 0, early = il && (rsb & 512) != 0;
  // N % 8: 16-B C stores (CEF stores no C: any N)
  if (p.M <= 0 || p.N <= 0 || p.K <= 0 || p.K % BK || (p.N % 8 && epi != W4_EPI_CEF) || p.tm * 256 < p.M ||
      p.tn * 256 < p.N)
    return -4;
  if (epi == W4_EPI_RELU) {
    if (b_kmajor || p.accumulate || p.mask == nullptr) return -5;
    if (early)
      return p.bias ? launch_rs<false, true, false, 769, W4_EPI_RELU>(p, persist != 0, st)
                    : launch_rs<false, false, false, 769, W4_EPI_RELU>(p, persist != 0, st);
    if (il)
      return p.bias ? launch_rs<false, true, false, 257, W4_EPI_RELU>(p, persist != 0, st)
                    : launch_rs<false, false, false, 257, W4_EPI_RELU>(p, persist != 0, st);
    return p.bias ? launch_rs<false, true, false, 1, W4_EPI_RELU>(p, persist != 0, st)
                  : launch_rs<false, false, false, 1, W4_EPI_RELU>(p, persist != 0, st);
  }
  if (epi == W4_EPI_DRELU_M) {
    if (!b_kmajor || p.accumulate || p.bias || p.mask == nullptr) return -5;
    if (early) return launch_rs<true, false, false, 769, W4_EPI_DRELU_M>(p, persist != 0, st);
    if (il) return launch_rs<true, false, false, 257, W4_EPI_DRELU_M>(p, persist != 0, st);
    return launch_rs<true, false, false, 1, W4_EPI_DRELU_M>(p, persist != 0, st);
  }
  if (epi == W4_EPI_GELU) {  // NT, bias, two outputs; persistent (store-only epilogue)
    if (b_kmajor || p.accumulate || p.aux_out == nullptr || p.ldaux < p.N || p.ldaux % 8 || p.N % 8) return -5;
    return p.bias ? launch_rs<false, true, false, 1, W4_EPI_GELU>(p, persist != 0, st)
                  : launch_rs<false, false, false, 1, W4_EPI_GELU>(p, persist != 0, st);
  }
  if (epi == W4_EPI_DGELU) {  // NN; its derivative loads would queue behind a persistent tile's prefetch: one tile each
    if (!b_kmajor || p.accumulate || p.bias || p.aux == nullptr || p.colsum == nullptr || p.ldaux < p.N ||
        p.ldaux % 4 || p.M % 128 || p.N % 4)
      return -5;
    return launch_rs<true, false, false, 1, W4_EPI_DGELU>(p, false, st);
  }
  if (epi == W4_EPI_CEF || epi == W4_EPI_CEB) {
    if (b_kmajor || p.accumulate || p.bias || p.labels == nullptr || p.skip < 0 || p.V <= 0) return -5;
    if (epi == W4_EPI_CEF) {
      if (p.part == nullptr || p.xlab == nullptr || p.pstride < (p.N + 127) / 128) return -5;
      return launch_rs<false, false, false, 1, W4_EPI_CEF>(p, persist != 0, st);
    }
    if (p.lse == nullptr || p.gscale == nullptr) return -5;
    return launch_rs<false, false, false, 1, W4_EPI_CEB>(p, persist != 0, st);
  }
  if (epi == W4_EPI_WG) {
    // both operands k-major, one tile per workgroup; ws holds `splits` [M][N] fp32 slabs (splits > 1) or C is written
    if (!b_kmajor || p.accumulate || p.bias || p.N % 256 || p.splits < 1 || p.kchunk < BK || p.kchunk % BK ||
        (p.splits > 1 && p.ws == nullptr) || (p.splits == 1 && p.Cw == nullptr) ||
        (long)p.tm * p.tn * p.splits > 0x7fffffffL)
      return -5;
    if (p.nseg > 0) {  // deferred segments: seg_chunks splits of kchunk rows cover each segment exactly
      if (p.nseg > W4_MAX_SEGS || p.seg_chunks < 1 || p.splits != p.nseg * p.seg_chunks || p.seg_rows % BK ||
          (long)p.kchunk * p.seg_chunks < p.seg_rows || (long)p.kchunk * (p.seg_chunks - 1) >= p.seg_rows)
        return -5;
      for (int i = 0; i < p.nseg; ++i)
        if (p.segA[i] == nullptr || p.segB[i] == nullptr) return -5;
    } else if ((long)p.kchunk * p.splits < p.K || (long)p.kchunk * (p.splits - 1) >= p.K) {
      return -5;
    }
    // every split's k-major descriptors (k-rows x leading dimension) must fit their 32-bit byte range
    const long span = ((long)(p.kchunk - 1) * std::max(p.lda, p.ldb) + std::max(p.M, p.N)) * 2;
    if (span >= 0xFFFFFFFFL) return -6;
    if (early) return launch_rs<true, false, false, 769, W4_EPI_WG>(p, false, st);
    if (il) return launch_rs<true, false, false, 257, W4_EPI_WG>(p, false, st);
    return launch_rs<true, false, false, 1, W4_EPI_WG>(p, false, st);
  }
  if (epi != W4_EPI_NONE) return -5;
  return b_kmajor ? dispatch<true>(p, persist != 0, st) : dispatch<false>(p, persist != 0, st);
}

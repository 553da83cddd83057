// Shared tile helpers of the attention kernels (csrc/attn.hip): head dim 64, bf16 tiles of
// [rows][64] in LDS with an XOR swizzle that makes both row reads (ds_read_b128) and hardware-transposed reads
// (ds_read_b64_tr_b16) bank-conflict free, and the v_mfma_f32_32x32x16_bf16 operand / accumulator layouts.
#pragma once
#include "common.h"

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8v;
typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef __attribute__((ext_vector_type(8))) float f32x8;

namespace {

using namespace dllm;

constexpr int D = 64;
constexpr int TILE64 = 64 * D;  // elements of a 64-row tile (8 KB)
constexpr int TILE32 = 32 * D;  // elements of a 32-row tile (4 KB)
constexpr int FWD_BM = 128;     // query rows per forward / dQ workgroup (4 waves x 32)
constexpr int FWD_BN = 64;      // keys per K/V tile
constexpr int BWD_BK = 128;     // keys per dK/dV workgroup (4 waves x 32)
constexpr int BWD_BQ = 32;      // query rows per dK/dV tile
constexpr float LOG2E = 1.4426950408889634f;
constexpr float LN2 = 0.6931471805599453f;
constexpr float RESCALE_THR = 8.f;
constexpr uint32_t HG = 0x9E3779B1u;

DLLM_DEVICE bf16x8v as_frag(u16x8 v) { return __builtin_bit_cast(bf16x8v, v); }

// v_exp_f32 directly: libm exp2f wraps it in a denormal-range fix-up (compare, select, add, ldexp) that costs
// 5 extra VALU ops per score; softmax probabilities below 2^-126 are irrelevant (flushed to 0).
DLLM_DEVICE float fast_exp2(float x) { return __builtin_amdgcn_exp2f(x); }

// 8 consecutive accumulator registers -> one bf16 MFMA operand (4 v_cvt_pk_bf16_f32)
DLLM_DEVICE bf16x8v pack8(const f32x16& a, int base) {
  const f32x8 v = {a[base], a[base + 1], a[base + 2], a[base + 3], a[base + 4], a[base + 5], a[base + 6], a[base + 7]};
  return __builtin_convertvector(v, bf16x8v);
}

DLLM_DEVICE f32x16 mfma32(bf16x8v a, bf16x8v b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

// bijective XCD-aware remap (cdna_hip_programming.md §5 "XCD swizzle must be bijective")
DLLM_DEVICE int xcd_remap(int bid, int nblk) {
  const int q = nblk / 8, r = nblk % 8, x = bid % 8;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + bid / 8;
}

// row of the C/D accumulator held in register `reg` by lane-half `hh` (32x32x16 layout)
DLLM_DEVICE int crow(int reg, int hh) { return (reg & 3) + 8 * (reg >> 2) + 4 * hh; }

// ---- swizzled [rows][64] bf16 tiles
DLLM_DEVICE int swz(int r) { return (((r >> 1) & 1) << 2) | ((r >> 2) & 3); }
DLLM_DEVICE int toff(int r, int c) { return (r << 6) + ((c ^ swz(r)) << 3); }
DLLM_DEVICE u16x8 ld_row(const uint16_t* T, int r, int c) { return *reinterpret_cast<const u16x8*>(T + toff(r, c)); }
DLLM_DEVICE void st_row(uint16_t* T, int r, int c, u16x8 v) { *reinterpret_cast<u16x8*>(T + toff(r, c)) = v; }

// Transposed read (ds_read_b64_tr_b16): the calling lane's 16-lane group reads rows r0..r0+3 (r0 % 4 == 0) x
// columns c0..c0+15 (c0 % 16 == 0); group lane i receives column c0 + i of the 4 rows (row q in element q).
// Lane 4q+p supplies the address of row q, columns 4p..4p+3.  EXEC must be full (no divergence here).
DLLM_DEVICE u16x4 ld_tr(const uint16_t* T, int r0, int c0, int i) {
  const int r = r0 + (i >> 2);
  const int col = c0 + 4 * (i & 3);
  const int off = (r << 6) + (((col >> 3) ^ swz(r)) << 3) + (col & 4);
  s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(T + off));
  return __builtin_bit_cast(u16x4, v);
}

// A operand (32x32x16, k = sequence, permuted k order of an accumulator-fed B) for head-dim rows
// [32t, 32t+32) and sequence rows kb0.. (lo: kb0+0..3, hi: kb0+8..11) of a swizzled tile.
DLLM_DEVICE bf16x8v ld_tr_operand(const uint16_t* T, int kb0, int t, int r) {
  const int c0 = 32 * t + 16 * ((r >> 4) & 1);
  const u16x4 lo = ld_tr(T, kb0, c0, r & 15);
  const u16x4 hi = ld_tr(T, kb0 + 8, c0, r & 15);
  const u16x8 v = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
  return as_frag(v);
}

}  // namespace

// Parameter block for the attention kernels (csrc/attn.hip), filled by the host binding.
#pragma once
#include <stdint.h>

struct AttnParams {
  const uint16_t* q;
  const uint16_t* k;
  const uint16_t* v;
  const uint16_t* o;   // fwd output / bwd input
  const uint16_t* dout;
  uint16_t* o_out;
  float* lse;          // [B, H, Sq]
  float* delta;        // [B, H, Sq] (bwd, written by the dQ kernel)
  float* rowrec;       // [B*H][sq_pad / 64][4][64] per-row terms for dK/dV (written by the dQ kernel):
                       // -lse2, c_lo - lse2, c_hi - lse2, -delta (rows >= Sq: -inf, -inf, -inf, 0)
  uint16_t* dq;        // [B, Sq, H, D] strided (bwd)
  uint16_t* dk;        // [B, Sk, H, D]
  uint16_t* dv;
  float* dlut;         // [H, Sq + Sk - 1] fp32 (bwd)
  const uint8_t* kpm;  // [B, Sk] 1 = attend
  const float* lut;    // [H, Sq + Sk - 1]
  long q_sb, q_ss, q_sh;
  long k_sb, k_ss, k_sh;
  long v_sb, v_ss, v_sh;
  long o_sb, o_ss, o_sh;
  long do_sb, do_ss, do_sh;
  long dq_sb, dq_ss, dq_sh;
  long dk_sb, dk_ss, dk_sh;
  long dv_sb, dv_ss, dv_sh;
  int B, H, Sq, Sk;
  float scale;
  int causal;
  int causal_off;  // Sk - Sq
  float p_drop;
  uint32_t seed;
  uint32_t thr;
  int n_tiles;  // fwd: q tiles; bwd: key blocks
  int n_ktiles;  // 64-key tiles (key-mask array length / 64)
  int sq_pad;    // rows of the dropout bit-mask planes (query tiles x 128)
  uint32_t* dmask;  // [B*H][n_ktiles][2][sq_pad] dropout keep bits written by fwd, read by bwd
  int dmask_ready;  // fwd: planes already generated (attn_dropout_mask) -> read instead of hash
  // Saturated bias ranges (T5 relative buckets): LUT entries [0, sat_lo] all equal lut[0] and [sat_hi, L) all
  // equal lut[L-1], and the LUT gradient is only consumed per bucket.  A (forward, dQ, dK/dV) tile whose LUT
  // indices all fall in one range adds a scalar bias (no LDS lookups) and its dS sum is credited to lut[0] /
  // lut[L-1] (no diagonal shear).  Disabled: sat_lo = INT_MIN / 2, sat_hi = INT_MAX / 2.
  int sat_lo;
  int sat_hi;
  // bwd, optional: per-block column sums of dQ / dK / dV (the bias gradients of the projections that produced q / k /
  // v).  Row b * ceil(S / 128) + block (S = Sq for csq, Sk for csk / csv), columns h * 64 + d, row strides csq_ld /
  // cskv_ld floats; the host sums the rows (ops/attention.py).  nullptr: not wanted.
  float* csq;
  float* csk;
  float* csv;
  long csq_ld, cskv_ld;
};

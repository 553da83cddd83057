// Flash attention forward + backward for encoder-decoder models on gfx950 (MI355X / CDNA4).
//
// Head dim D = 64 (T5 d_kv, BART 1024/16, flan-t5-xl 2048/32).  bf16 in/out, fp32 accumulate,
// v_mfma_f32_32x32x16_bf16 (wave64).  Supports: softmax scale (BART d^-0.5, T5 1.0), T5 relative
// position bias as a per-head LUT over (j - i) staged in LDS, key-padding mask, causal mask
// (bottom-right aligned: key j visible to query i iff j <= i + Sk - Sq), attention-probability
// dropout regenerated from a counter-based hash (never stored).
//
// LDS tiles are [rows][64] bf16 with 128-B rows and no padding; 16-B chunk c of row r is stored at
// chunk c ^ swz(r), swz(r) = ((r>>1)&1)<<2 | ((r>>2)&3).  With that one image both access kinds the
// kernels need are bank-conflict free: row reads (ds_read_b128, MFMA operands whose k-dim is the head
// dim) and hardware-transposed reads (ds_read_b64_tr_b16, operands whose k-dim is the sequence) — so
// no tile is ever written transposed element by element.
//
// Scores are computed in log2 units: s2 = (q.k) * scale * log2(e) + bias * log2(e) (the LUT is
// pre-scaled when staged), softmax via exp2; the LSE handed from forward to backward is in log2 units.
// Online softmax defers the O/l rescale until the running max grows by more than 8 (P <= 2^8 in bf16).
//
// Forward (workgroup = 4 waves = 128 query rows of one (b, h); K/V tiles of 64 keys, double-buffered,
// next tile's global loads in flight during compute, one barrier per tile):
//   swapped QK^T: each wave computes S^T = K Q^T so a lane owns one query row; row max / sum are in-lane
//   + one xor-32 shuffle; the P^T accumulator registers, converted to bf16, are directly the B operand
//   of O^T = V^T P^T (cdna_hip_programming.md §3, accumulator as the next MFMA's operand); V^T comes
//   from transposed LDS reads.  1-D grid with a bijective XCD remap: q-tiles of one (b, h) share an XCD.
// Backward = two atomic-free kernels (P recomputed from LSE in both):
//   dQ kernel (query blocks, query on the lane): dS^T = P^T (dP^T - delta) feeds dQ^T += K^T dS^T as the
//   B operand (K^T by transposed reads); also computes delta = rowsum(dO * O).
//   dK/dV kernel (key blocks of 128, key on the lane): P and dS accumulators are the B operands of
//   dV^T += dO^T Pd and dK^T += Q^T dS (dO^T, Q^T by transposed reads); bias-LUT gradient = diagonal sums
//   of dS via a register shear + 2 LDS atomics per lane per tile.
// Saturated T5 bias tiles (AttnParams::sat_lo / sat_hi): a wave tile whose relative distances all lie beyond the
// last exact bucket (|j - i| >= 91 for bidirectional T5) sees one constant bias — it adds a scalar instead of
// reading the LUT, and dK/dV credits its whole dS sum to the range's end entry instead of shearing diagonals (the
// LUT gradient is consumed per bucket).  dK/dV -12..20 %, forward -2 % (interleaved A/B, r1_attn_bench_v8_ab).
#include "common.h"
#include "route.h"
#include "attn_params.h"
#include "attn_tile.h"
#include <stdlib.h>
#include <type_traits>

using namespace dllm;

DLLM_SEED_STEP_TU(attn)

// output tiles staged through LDS and stored as whole rows (store_rows_staged): forward O, dQ (A/B: -D..._STAGE=0)
#ifndef FWD_STAGE
#define FWD_STAGE 1
#endif
#ifndef DQ_STAGE
#define DQ_STAGE 1
#endif

namespace {

// attention dropout (ops/rng.py attention_keep_mask): the row-Weyl hash of common.h (rw_*) with one row per (b, h,
// query): per query row rh = mix32(seed, row); per key pair kp = key >> 1, g = (rh & 0xFFFFFF) * C24 + kp * HG, the
// xorshift + 24-bit multiply round (pair_y), and the two-key signed compare (drop_mask2).  The xorshift + multiply
// round matters: g alone is linear in kp and leaves lag-2 drops anti-correlated; with it every lag-1/2/3/16 joint drop
// rate and the row-count variance match independent Bernoulli draws (tests/test_training_cpu.py
// test_attention_dropout_hash_statistics).
static_assert(HG == RW_G, "attention Weyl step = the row-Weyl hash's");
DLLM_DEVICE uint32_t pair_y(uint32_t g) { return rw_pair_y(g); }
// per-lane, per-tile start of the Weyl sequence: g of pair kp0 + j is gbase + j * HG
DLLM_DEVICE uint32_t pair_gbase(uint32_t rh, uint32_t kp0) { return rw_gbase(rh, kp0); }
// t2 = (thr16 - 0x8000) in both 16-bit halves.  Returns the pair's DROP mask: 0xFFFF in the half of each dropped key
// (low half = even key, high half = odd key).
DLLM_DEVICE uint32_t drop_mask2(uint32_t y, uint32_t t2) { return rw_drop2(y, t2); }

// Keep-word layout of one (row, 64-key tile, lane half) — shared by the forward and both backward kernels: the lane's
// 16 key pairs are slots p = 0..15, pair slot p of accumulator register i of s0 (t = 0) or s1 (t = 1) being
// p = 8 t + (i >> 1) (the key pair kbase + 32 t + crow(i & ~1, hh) .. + 1); the even key's bit is p, the odd key's 16 + p.
DLLM_DEVICE constexpr int keep_bit(int t, int i) { return ((i & 1) << 4) + 8 * t + (i >> 1); }
DLLM_DEVICE uint32_t pair_slot_kp(int p) { return (uint32_t)((p & 1) + 4 * ((p & 7) >> 1) + 16 * (p >> 3)); }

// Dropout keep word of one (row, 64-key tile, lane half) in the keep_bit layout (ops/rng.py mirrors the decisions).
DLLM_DEVICE uint32_t dropout_word(uint32_t rh, int kbase, int hh, uint32_t thr) {
  const uint32_t gbase = pair_gbase(rh, (uint32_t)(kbase >> 1) + 2u * (uint32_t)hh);
  const uint32_t t2 = ((thr - 0x8000u) & 0xFFFFu) * 0x10001u;
  uint32_t drop = 0;
#pragma unroll
  for (int p = 0; p < 16; ++p) {
    const uint32_t m = drop_mask2(pair_y(gbase + pair_slot_kp(p) * HG), t2);
    drop |= (m & ((1u << p) | (0x10000u << p)));
  }
  return ~drop;
}

// One wave's 32 rows x 64 bf16 output tile in the MFMA accumulator layout (lane (r, hh) holds columns 32 t + 8 g + 4 hh
// .. + 3 of row r in a_t[4 g .. 4 g + 3]; times `mul`) through the wave's 4 KB LDS scratch (16-B chunks XOR-swizzled by
// row), stored as whole 128-B rows: 4 full-line stores instead of 8 per-lane 8-B stores touching 32 lines each.  Row rr
// goes to base + rr * row_stride (elements) for rr < nrows.  The caller has made the scratch free (barrier).
//
// Bias-gradient column sums (AttnParams csq / csk / csv): the staged rows are summed per column on their way to the row
// stores.  Lane (row group lane >> 3, 16-B chunk ch) adds the 8 bf16 values of each of its valid rows (the stored,
// rounded values: what a separate column reduction of dQ / dK / dV would read), cs_wave folds the 8 row groups with xor
// shuffles and writes the wave's 64 sums to `red` (LDS); after a barrier one thread per column adds the 4 waves' sums in
// a fixed order (deterministic) and stores one partial row of the [B * blocks][cols] fp32 buffer the host reduces.
DLLM_DEVICE void cs_add(float (&acc)[8], const u16x8& v) {
#pragma unroll
  for (int e = 0; e < 8; ++e) acc[e] += bf2f(v[e]);
}

DLLM_DEVICE void cs_wave(float (&acc)[8], int lane, float* red) {
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    float s = acc[e];
    s += __shfl_xor(s, 8, 64);
    s += __shfl_xor(s, 16, 64);
    s += __shfl_xor(s, 32, 64);
    acc[e] = s;
  }
  if (lane < 8) {
    *reinterpret_cast<float4*>(red + 8 * lane) = make_float4(acc[0], acc[1], acc[2], acc[3]);
    *reinterpret_cast<float4*>(red + 8 * lane + 4) = make_float4(acc[4], acc[5], acc[6], acc[7]);
  }
}

// `red` != nullptr: also the tile's column sums over its rows < nrows into red[0, 64) (cs_wave)
DLLM_DEVICE void store_rows_staged(unsigned char* scr, const f32x16& a0, const f32x16& a1, float mul, int r, int hh,
                                   int lane, uint16_t* base, long row_stride, int nrows, float* red = nullptr) {
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const f32x16& a = t == 0 ? a0 : a1;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const u16x4 pk = {f2bf(a[4 * g] * mul), f2bf(a[4 * g + 1] * mul), f2bf(a[4 * g + 2] * mul),
                        f2bf(a[4 * g + 3] * mul)};
      *reinterpret_cast<u16x4*>(scr + r * 128 + (((4 * t + g) ^ (r & 7)) << 4) + 8 * hh) = pk;
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // other lanes of this wave read what these wrote
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int st = 0; st < 4; ++st) {
    const int row = 8 * st + (lane >> 3), ch = lane & 7;
    const u16x8 v = *reinterpret_cast<const u16x8*>(scr + row * 128 + ((ch ^ (row & 7)) << 4));
    if (row < nrows) {
      *reinterpret_cast<u16x8*>(base + (long)row * row_stride + 8 * ch) = v;
      if (red != nullptr) cs_add(acc, v);
    }
  }
  if (red != nullptr) cs_wave(acc, lane, red);
}

// ================================================================================== dropout bit planes
// All keep decisions of one attention call, [B*H][n_ktiles][2][sq_pad] words, one thread per word (q fastest:
// coalesced stores).  Pure VALU + streaming stores, for generating the planes ahead of the forward on a side
// stream (ops/attention.py prefetch_dropout_mask) where they overlap the projection GEMM.
__global__ __launch_bounds__(256) void attn_dropout_mask_kernel(AttnParams P, long nwords) {
  for (long w = (long)blockIdx.x * blockDim.x + threadIdx.x; w < nwords; w += (long)gridDim.x * blockDim.x) {
    const int q = (int)(w % P.sq_pad);
    const long r = w / P.sq_pad;
    const int hh = (int)(r & 1);
    const long t2 = r >> 1;
    const int kt = (int)(t2 % P.n_ktiles);
    const long bh = t2 / P.n_ktiles;
    const uint32_t rh = mix32(eff_seed(P.seed), (uint32_t)(bh * P.Sq + q));
    P.dmask[w] = dropout_word(rh, kt * FWD_BN, hh, P.thr);
  }
}

// ================================================================================== forward
// DROP_IN: dropout keep bits are read from precomputed planes (attn_dropout_mask_kernel on a side stream);
// otherwise the forward hashes them itself (hidden in its MFMA/LDS latency) and stores the planes for backward.
// FNB = K/V ring depth: 3 (two tiles in flight, 2 workgroups per CU) or 2 (one tile in flight, a 2/3-size LDS
// footprint and a 168-VGPR budget so 3 workgroups share a CU: more waves to hide latency with).
template <bool HAS_BIAS, bool HAS_KPM, bool CAUSAL, bool DROP, bool DROP_IN, int FNB>
__global__ __launch_bounds__(256, FNB == 3 ? 2 : 3) void attn_fwd_kernel(AttnParams P) {
  static_assert(FNB == 2 || FNB == 3, "K/V ring depth");
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  uint16_t* KV = reinterpret_cast<uint16_t*>(smem);            // [FNB buffers][K tile | V tile]
  uint32_t* mwl = reinterpret_cast<uint32_t*>(KV + 2 * FNB * TILE64); // [FNB][4 waves][2 halves][32 rows] keep bits
  float* kmask = reinterpret_cast<float*>(mwl + FNB * 256);     // [ntiles * 64]: 0 or -inf per key
  int* tflag = reinterpret_cast<int*>(kmask + P.n_ktiles * FWD_BN);  // [ntiles]: tile has a masked key
  float* lut_s = reinterpret_cast<float*>(tflag + P.n_ktiles);   // [Sk + FWD_BM + FWD_BN], log2-scaled

  // w through readfirstlane: wave-uniform to the compiler, so per-wave tile decisions are scalar branches
  const int tid = threadIdx.x, w = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63, r = lane & 31,
            hh = lane >> 5;
  const int logical = xcd_remap(blockIdx.x, gridDim.x);
  const int qt = logical % P.n_tiles;
  const int bh = logical / P.n_tiles;
  const int h = bh % P.H, b = bh / P.H;
  const int q0 = qt * FWD_BM;
  const int qw0 = q0 + w * 32;
  const int qrow = qw0 + r;
  const bool qvalid = qrow < P.Sq;
  const float sl2 = P.scale * LOG2E;

  int kend = P.Sk;
  if (CAUSAL) {
    const int lim = q0 + FWD_BM + P.causal_off;  // keys <= last row + off
    kend = lim < kend ? lim : kend;
  }
  const int ntiles = kend > 0 ? (kend + FWD_BN - 1) / FWD_BN : 0;

  // ---- staging by LDS-DMA: wave w moves rows 16w .. 16w+15 of the K and V tiles (2 x 1 KB per operand);
  // lane L of DMA j lands at row 8j + L/8, physical chunk L%8 and fetches logical chunk (L%8) ^ swz(row).
  // Keys past Sk re-read row Sk-1 (finite values; masked to -inf / P = 0).  No staging VGPRs, no ds_write.
  const uint32_t kv_lds = lds_addr(KV);
  const uint32_t mw_lds = lds_addr(mwl);
  // buffer-descriptor DMA: wave-uniform (b, h) bases in SGPRs, per-lane 32-bit byte offsets from one v_mad_u32_u24
  // (the launcher checks strides and lengths fit), instead of 64-bit address arithmetic per DMA
  const uint16_t* kbase_p = P.k + b * P.k_sb + h * P.k_sh;
  const uint16_t* vbase_p = P.v + b * P.v_sb + h * P.v_sh;
  const uint32_t kss2 = (uint32_t)P.k_ss * 2u, vss2 = (uint32_t)P.v_ss * 2u;
  int drow[2];
  uint32_t dc16[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    drow[i] = 8 * (2 * w + i) + (lane >> 3);
    dc16[i] = (uint32_t)(((lane & 7) ^ swz(drow[i])) * 16);
  }
  auto issue_tile = [&](int buf, int kt) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int j = 2 * w + i;
      const uint32_t kk = (uint32_t)min(kt * FWD_BN + drow[i], P.Sk - 1);  // keys past Sk re-read row Sk-1
      const uint32_t dst = kv_lds + (uint32_t)(buf * 2 * TILE64 * 2 + j * 1024);
      bld16(kbase_p, __umul24(kk, kss2) + dc16[i], __builtin_amdgcn_readfirstlane(dst));
      bld16(vbase_p, __umul24(kk, vss2) + dc16[i], __builtin_amdgcn_readfirstlane(dst + TILE64 * 2));
    }
    if (DROP && DROP_IN)  // this wave's 32 rows x 2 lane halves of keep bits: lane L -> half L/32, row qw0 + L%32
      glds4(P.dmask + ((long)bh * P.n_ktiles * 2 + 2 * kt + hh) * P.sq_pad + qrow,
            __builtin_amdgcn_readfirstlane(mw_lds + (uint32_t)((buf * 256 + w * 64) * 4)));
  };
  // the first FNB - 1 tiles are issued before the prologue's global reads (bias LUT, Q fragments, key mask) so their
  // latencies overlap instead of adding up
  if (ntiles > 0) issue_tile(0, 0);
  if (FNB == 3 && ntiles > 1) issue_tile(1, 1);
  const int lut_base = P.Sq - 1 - (q0 + FWD_BM - 1);  // lut_s[i] = LUT[lut_base + i]
  float c_lo = 0.f, c_hi = 0.f;                        // saturated-range biases (log2-scaled)
  if (HAS_BIAS) {
    const int L = P.Sq + P.Sk - 1;
    const float* lrow = P.lut + (long)h * L;
    for (int i = tid; i < P.Sk + FWD_BM + FWD_BN; i += 256) {
      const int gi = lut_base + i;
      lut_s[i] = (gi >= 0 && gi < L) ? lrow[gi] * LOG2E : 0.f;
    }
    c_lo = lrow[0] * LOG2E;
    c_hi = lrow[L - 1] * LOG2E;
  }
  bf16x8v qf[4];
  {
    const uint16_t* qp = P.q + b * P.q_sb + (long)qrow * P.q_ss + h * P.q_sh;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      u16x8 t = {0, 0, 0, 0, 0, 0, 0, 0};
      if (qvalid) t = *reinterpret_cast<const u16x8*>(qp + 16 * s + 8 * hh);
      qf[s] = as_frag(t);
    }
  }
  const long row_g = (long)(b * P.H + h) * P.Sq + qrow;
  const uint32_t rh = DROP ? mix32(eff_seed(P.seed), (uint32_t)row_g) : 0u;
  const float dscale = DROP ? 1.f / (1.f - P.p_drop) : 1.f;
  const uint32_t t2drop = ((P.thr - 0x8000u) & 0xFFFFu) * 0x10001u;  // drop_mask2 threshold pair

  for (int t = w; t < ntiles; t += 4) {  // wave-per-tile: per-key mask + "tile has a masked key" flag
    const int j = t * FWD_BN + lane;
    bool ok = j < P.Sk;
    if (HAS_KPM && ok) ok = P.kpm[(long)b * P.Sk + j] != 0;
    kmask[j] = ok ? 0.f : -INFINITY;
    const unsigned long long m = __ballot(!ok);
    if (lane == 0) tflag[t] = m == 0ull ? 0 : (~m == 0ull ? 2 : 1);  // 2: every key masked -> tile skipped
  }

  f32x16 o0 = {}, o1 = {};
  float m_run = -INFINITY, l_run = 0.f;

  // S^T = K Q^T for the tile in LDS buffer `buf` (8 MFMAs, two independent accumulation chains)
  auto scores = [&](int buf, f32x16& s0, f32x16& s1) __attribute__((always_inline)) {
    const uint16_t* Kb = KV + buf * 2 * TILE64;
    s0 = f32x16{};
    s1 = f32x16{};
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      s0 = mfma32(as_frag(ld_row(Kb, r, 2 * s + hh)), qf[s], s0);
      s1 = mfma32(as_frag(ld_row(Kb, 32 + r, 2 * s + hh)), qf[s], s1);
    }
  };
  // online softmax of tile kt's scores (in s0/s1) and O^T += V^T P^T with V from buffer `buf`
  auto softmax_pv = [&](int kt, int buf, f32x16& s0, f32x16& s1) __attribute__((always_inline)) {
    const uint32_t mword = (DROP && DROP_IN) ? mwl[buf * 256 + w * 64 + hh * 32 + r] : 0u;
    const int kbase = kt * FWD_BN;
    const uint16_t* Vb = KV + buf * 2 * TILE64 + TILE64;
    const bool tile_causal = CAUSAL && (kbase + FWD_BN - 1 > qw0 + P.causal_off);
    const int climit = qrow + P.causal_off - kbase;  // key offsets above this are masked (causal)
    const float* lb = lut_s + (kbase - qrow + P.Sq - 1 - lut_base);
    // saturated tile (every LUT index of the wave's 32 rows x 64 keys in one constant-bias range): a scalar
    // bias, no LDS lookups.  One wave-uniform branch around two fully unrolled bodies.
    const int sat = !HAS_BIAS ? 0
                    : (kbase + FWD_BN - 1 - qw0 + P.Sq - 1 <= P.sat_lo ? 1
                       : (kbase - qw0 - 31 + P.Sq - 1 >= P.sat_hi ? 2 : 0));
    // Per score, in VALU instructions (the forward is VALU-bound: MI355X_MICROARCH.md issue costs): scale + bias 1
    // (LUT tiles 2), max 0.5 (v_max3), exp 1, row sum 1, dropout ~4, bf16 pack 0.5.  Saturated / bias-free tiles
    // stay in the raw QK^T domain until the exponent: max(s * sl2 + c) = max(s) * sl2 + c (sl2 > 0), and
    // p = exp2(fma(s, sl2, c - m)) is one FMA.
    const bool use_lut = HAS_BIAS && sat == 0;
    const float cb = sat == 1 ? c_lo : (sat == 2 ? c_hi : 0.f);
    if (use_lut) {
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        s0[i] = fmaf(s0[i], sl2, lb[crow(i, hh)]);
        s1[i] = fmaf(s1[i], sl2, lb[32 + crow(i, hh)]);
      }
    }
    if (CAUSAL && tile_causal) {
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int kl0 = crow(i, hh);
        s0[i] = kl0 > climit ? -INFINITY : s0[i];
        s1[i] = kl0 + 32 > climit ? -INFINITY : s1[i];
      }
    }
    // key mask (padding / past Sk): one uniform branch per tile around 8 vector LDS reads; a per-score `if`
    // made the compiler emit 16 branches each ending in s_waitcnt lgkmcnt(0)
    if ((HAS_KPM || kbase + FWD_BN > P.Sk) && tflag[kt] != 0) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const f32x4 m0 = *reinterpret_cast<const f32x4*>(kmask + kbase + 8 * g + 4 * hh);
        const f32x4 m1 = *reinterpret_cast<const f32x4*>(kmask + kbase + 32 + 8 * g + 4 * hh);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          s0[4 * g + e] += m0[e];
          s1[4 * g + e] += m1[e];
        }
      }
    }
    float ma = fmaxf(fmaxf(s0[0], s0[1]), s0[2]), mb = fmaxf(fmaxf(s1[0], s1[1]), s1[2]);
#pragma unroll
    for (int i = 3; i < 15; i += 2) {
      ma = fmaxf(fmaxf(ma, s0[i]), s0[i + 1]);
      mb = fmaxf(fmaxf(mb, s1[i]), s1[i + 1]);
    }
    float mloc = fmaxf(fmaxf(ma, mb), fmaxf(s0[15], s1[15]));
    mloc = fmaxf(mloc, __shfl_xor(mloc, 32, 64));
    if (!use_lut) mloc = fmaf(mloc, sl2, cb);  // -inf stays -inf
    // deferred rescale (T13): keep the running max unless the tile max exceeds it by > 8 (log2 units)
    const bool grow = mloc > m_run + RESCALE_THR;
    float alpha = 1.f;
    if (grow) {
      alpha = fast_exp2(m_run - mloc);
      m_run = mloc;
    }
    const float m_use = m_run == -INFINITY ? 0.f : m_run;
    float la = 0.f, lb2 = 0.f;
    if (use_lut) {
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        s0[i] = fast_exp2(s0[i] - m_use);
        s1[i] = fast_exp2(s1[i] - m_use);
        la += s0[i];
        lb2 += s1[i];
      }
    } else {
      const float cm = cb - m_use;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        s0[i] = fast_exp2(fmaf(s0[i], sl2, cm));
        s1[i] = fast_exp2(fmaf(s1[i], sl2, cm));
        la += s0[i];
        lb2 += s1[i];
      }
    }
    l_run = l_run * alpha + (la + lb2);
    if (__any(grow)) {
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        o0[i] *= alpha;
        o1[i] *= alpha;
      }
    }
    if (DROP && DROP_IN) {  // precomputed keep bits; the 1/(1-p) scale is applied once to O at the end
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        s0[i] = __uint_as_float(__float_as_uint(s0[i]) & (uint32_t)__builtin_amdgcn_sbfe((int)mword, keep_bit(0, i), 1));
        s1[i] = __uint_as_float(__float_as_uint(s1[i]) & (uint32_t)__builtin_amdgcn_sbfe((int)mword, keep_bit(1, i), 1));
      }
    }
    // P as bf16 pairs: pk[2 t + half] holds registers 8 half .. 8 half + 7 of s_t; its dword j is one adjacent key pair,
    // pair slot 4 (2 t + half) + j of the keep_bit layout
    bf16x8v pk[4] = {pack8(s0, 0), pack8(s0, 8), pack8(s1, 0), pack8(s1, 8)};
    if (DROP && !DROP_IN) {
      // keep decisions applied to the packed pairs (the 1/(1-p) scale is applied once to O at the end) and recorded as
      // one bit word per lane and tile for the backward kernels, which never re-hash.  Per key pair: one add (the
      // Weyl step is a constant), two 24-bit multiplies, two shift-xors, the two-key signed compare (drop_mask2: 2),
      // one bitwise op zeroing the dropped halves and one recording them — 10 VALU per two keys.
      const uint32_t gbase = pair_gbase(rh, (uint32_t)(kbase >> 1) + 2u * (uint32_t)hh);
      uint32_t drop = 0;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        u32x4 v = __builtin_bit_cast(u32x4, pk[q]);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int p = 4 * q + j;
          const uint32_t m = drop_mask2(pair_y(gbase + pair_slot_kp(p) * HG), t2drop);
          v[j] &= ~m;
          drop |= m & ((1u << p) | (0x10000u << p));
        }
        pk[q] = __builtin_bit_cast(bf16x8v, v);
      }
      P.dmask[((long)bh * P.n_ktiles * 2 + 2 * kt + hh) * P.sq_pad + qrow] = ~drop;
    }
    // O^T += V^T P^T
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
#pragma unroll
      for (int sp = 0; sp < 2; ++sp) {
        const int kb0 = kb * 32 + 16 * sp + 4 * hh;
        o0 = mfma32(ld_tr_operand(Vb, kb0, 0, r), pk[2 * kb + sp], o0);
        o1 = mfma32(ld_tr_operand(Vb, kb0, 1, r), pk[2 * kb + sp], o1);
      }
    }
  };

  // K/V ring: right after the barrier that retires tile kt - 1, tile kt + FNB - 1 is issued into the buffer tile
  // kt - 1 vacated (FNB = 3: a whole extra tile of compute to land); one barrier per tile.
  f32x16 sa0, sa1;
  wait_vm<0>();
  __syncthreads();
  // the ring slot of a tile is a compile-time constant (loop unrolled by the ring depth): every LDS read address is a
  // loop-invariant per-lane offset plus an immediate
  auto step = [&](int kt, auto buf_c) __attribute__((always_inline)) {
    constexpr int BUF = decltype(buf_c)::value;
    if (kt > 0) {
      // tile kt landed (FNB = 3: this wave's 4 DMAs of tile kt+1, issued one tile later, and then either its keep-word
      // DMA (DROP_IN) or tile kt-1's keep-word store (vmcnt counts stores too) may stay in flight)
      if (FNB == 3 && kt + 1 < ntiles) wait_vm<(DROP ? 5 : 4)>();
      else wait_vm<0>();
      __syncthreads();
    }
    if (kt + FNB - 1 < ntiles) issue_tile((BUF + FNB - 1) % FNB, kt + FNB - 1);
    if (!HAS_KPM || tflag[kt] != 2) {  // a fully padded key tile contributes exactly nothing
      scores(BUF, sa0, sa1);
      softmax_pv(kt, BUF, sa0, sa1);
    }
  };
  for (int kt = 0; kt < ntiles; kt += FNB) {
    step(kt, std::integral_constant<int, 0>{});
    if (kt + 1 < ntiles) step(kt + 1, std::integral_constant<int, 1>{});
    if constexpr (FNB == 3) {
      if (kt + 2 < ntiles) step(kt + 2, std::integral_constant<int, 2>{});
    }
  }

  const float l_tot = l_run + __shfl_xor(l_run, 32, 64);
  const float inv = l_tot > 0.f ? dscale / l_tot : 0.f;  // dropout's 1/(1-p) folded in
#if FWD_STAGE
  // every wave is done with the K/V ring (the last tile's DMAs were waited for): its first 16 KB stage the O tiles
  __syncthreads();
  store_rows_staged(smem + w * 4096, o0, o1, inv, r, hh, lane, P.o_out + b * P.o_sb + (long)qw0 * P.o_ss + h * P.o_sh,
                    P.o_ss, P.Sq - qw0);
#endif
  if (qvalid) {
#if !FWD_STAGE
    uint16_t* op = P.o_out + b * P.o_sb + (long)qrow * P.o_ss + h * P.o_sh;
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const f32x16& acc = t == 0 ? o0 : o1;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        u16x4 pk = {f2bf(acc[4 * g] * inv), f2bf(acc[4 * g + 1] * inv), f2bf(acc[4 * g + 2] * inv),
                    f2bf(acc[4 * g + 3] * inv)};
        *reinterpret_cast<u16x4*>(op + 32 * t + 8 * g + 4 * hh) = pk;
      }
    }
#endif
    if (hh == 0) {
      const float m_use = m_run == -INFINITY ? 0.f : m_run;
      P.lse[row_g] = l_tot > 0.f ? m_use + log2f(l_tot) : INFINITY;  // log2 units
    }
  }
}

// ================================================================================== backward: dQ
// OCC = workgroups per CU the register budget is cut for (2: 256 VGPRs, 3: 168)
// CS: also the dQ column sums (AttnParams csq; instantiated for the bias-free kernels only, so the T5 variants compile
// without any of that code)
template <bool HAS_BIAS, bool HAS_KPM, bool CAUSAL, bool DROP, int OCC, bool CS = false>
__global__ __launch_bounds__(256, OCC) void attn_bwd_dq_kernel(AttnParams P) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  uint16_t* KV = reinterpret_cast<uint16_t*>(smem);            // [2][K | V]
  float* kmask = reinterpret_cast<float*>(KV + 4 * TILE64);     // [ntiles * 64]: 0 or -inf per key
  int* tflag = reinterpret_cast<int*>(kmask + P.n_ktiles * FWD_BN);  // [ntiles]: tile has a masked key
  float* lut_s = reinterpret_cast<float*>(tflag + P.n_ktiles);   // [Sk + FWD_BM + FWD_BN]

  // w through readfirstlane: wave-uniform to the compiler, so per-wave tile decisions are scalar branches
  const int tid = threadIdx.x, w = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63, r = lane & 31,
            hh = lane >> 5;
  const int logical = xcd_remap(blockIdx.x, gridDim.x);
  const int qt = logical % P.n_tiles;
  const int bh = logical / P.n_tiles;
  const int h = bh % P.H, b = bh / P.H;
  const int q0 = qt * FWD_BM;
  const int qw0 = q0 + w * 32;
  const int qrow = qw0 + r;
  const bool qvalid = qrow < P.Sq;
  const float sl2 = P.scale * LOG2E;
  int kend = P.Sk;
  if (CAUSAL) {
    const int lim = q0 + FWD_BM + P.causal_off;
    kend = lim < kend ? lim : kend;
  }
  const int ntiles = kend > 0 ? (kend + FWD_BN - 1) / FWD_BN : 0;
  // K/V tiles by LDS-DMA into 2 buffers (see the forward kernel); per-key mask + tile flags up front
  const uint32_t kv_lds = lds_addr(KV);
  // buffer-descriptor DMA: wave-uniform (b, h) bases in SGPRs, per-lane 32-bit byte offsets from one v_mad_u32_u24
  // (the launcher checks strides and lengths fit), instead of 64-bit address arithmetic per DMA
  const uint16_t* kbase_p = P.k + b * P.k_sb + h * P.k_sh;
  const uint16_t* vbase_p = P.v + b * P.v_sb + h * P.v_sh;
  const uint32_t kss2 = (uint32_t)P.k_ss * 2u, vss2 = (uint32_t)P.v_ss * 2u;
  int drow[2];
  uint32_t dc16[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    drow[i] = 8 * (2 * w + i) + (lane >> 3);
    dc16[i] = (uint32_t)(((lane & 7) ^ swz(drow[i])) * 16);
  }
  auto issue_tile = [&](int buf, int kt) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int j = 2 * w + i;
      const uint32_t kk = (uint32_t)min(kt * FWD_BN + drow[i], P.Sk - 1);  // keys past Sk re-read row Sk-1
      const uint32_t dst = kv_lds + (uint32_t)(buf * 2 * TILE64 * 2 + j * 1024);
      bld16(kbase_p, __umul24(kk, kss2) + dc16[i], __builtin_amdgcn_readfirstlane(dst));
      bld16(vbase_p, __umul24(kk, vss2) + dc16[i], __builtin_amdgcn_readfirstlane(dst + TILE64 * 2));
    }
  };
  // tile 0 is issued before the prologue's global reads (bias LUT, Q / dO / O rows, lse, key mask) so their latencies
  // overlap instead of adding up
  if (ntiles > 0) issue_tile(0, 0);
  const int lut_base = P.Sq - 1 - (q0 + FWD_BM - 1);
  float c_lo = 0.f, c_hi = 0.f;
  if (HAS_BIAS) {
    const int L = P.Sq + P.Sk - 1;
    const float* lrow = P.lut + (long)h * L;
    for (int i = tid; i < P.Sk + FWD_BM + FWD_BN; i += 256) {
      const int gi = lut_base + i;
      lut_s[i] = (gi >= 0 && gi < L) ? lrow[gi] * LOG2E : 0.f;
    }
    c_lo = lrow[0] * LOG2E;
    c_hi = lrow[L - 1] * LOG2E;
  }
  bf16x8v qf[4], dof[4];
  float dpart = 0.f;
  {
    const uint16_t* qp = P.q + b * P.q_sb + (long)qrow * P.q_ss + h * P.q_sh;
    const uint16_t* dp = P.dout + b * P.do_sb + (long)qrow * P.do_ss + h * P.do_sh;
    const uint16_t* op = P.o + b * P.o_sb + (long)qrow * P.o_ss + h * P.o_sh;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      u16x8 a = {0, 0, 0, 0, 0, 0, 0, 0}, c = a, o8 = a;
      if (qvalid) {
        a = *reinterpret_cast<const u16x8*>(qp + 16 * s + 8 * hh);
        c = *reinterpret_cast<const u16x8*>(dp + 16 * s + 8 * hh);
        o8 = *reinterpret_cast<const u16x8*>(op + 16 * s + 8 * hh);
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) dpart += bf2f(c[j]) * bf2f(o8[j]);
      qf[s] = as_frag(a);
      dof[s] = as_frag(c);
    }
  }
  const float delta = dpart + __shfl_xor(dpart, 32, 64);
  const long row_g = (long)(b * P.H + h) * P.Sq + qrow;
  if (qvalid && hh == 0) P.delta[row_g] = delta;
  const float lse2 = qvalid ? P.lse[row_g] : INFINITY;
  if (P.rowrec != nullptr) {  // dK/dV's per-row terms, field-major per 64-row chunk (attn_bwd_dkdv2_kernel)
    float c0 = 0.f, c1 = 0.f;
    if (HAS_BIAS) {
      const int L = P.Sq + P.Sk - 1;
      c0 = P.lut[(long)h * L] * LOG2E;
      c1 = P.lut[(long)h * L + L - 1] * LOG2E;
    }
    float* rec = P.rowrec + ((long)bh * (P.sq_pad >> 6) + (qrow >> 6)) * 256 + (qrow & 63);
    const float f = hh == 0 ? -lse2 : (hh == 1 ? c0 - lse2 : 0.f);  // lanes 0-31: fields 0 / 3, 32-63: 1 / 2
    const float g = hh == 0 ? (qvalid ? -delta : 0.f) : c1 - lse2;
    rec[hh == 0 ? 0 : 64] = f;
    rec[hh == 0 ? 192 : 128] = g;
  }
  const float dscale = DROP ? 1.f / (1.f - P.p_drop) : 1.f;

  for (int t = w; t < ntiles; t += 4) {
    const int j = t * FWD_BN + lane;
    bool ok = j < P.Sk;
    if (HAS_KPM && ok) ok = P.kpm[(long)b * P.Sk + j] != 0;
    kmask[j] = ok ? 0.f : -INFINITY;
    const unsigned long long m = __ballot(!ok);
    if (lane == 0) tflag[t] = m == 0ull ? 0 : (~m == 0ull ? 2 : 1);  // 2: every key masked -> tile skipped
  }
  // dropout decisions: the bit words the forward stored (keep_bit layout: register i of key half kb -> keep_bit(kb, i))
  const uint32_t* mrow = DROP ? P.dmask + ((long)bh * P.n_ktiles * 2 + hh) * P.sq_pad + qrow : nullptr;
  const uint32_t dsbits = __float_as_uint(dscale);
  uint32_t mword = 0, mnext = 0;
  if (DROP && ntiles > 0) mnext = mrow[0];

  f32x16 dq0 = {}, dq1 = {};
  // the buffer of a tile is a compile-time constant (loop unrolled by 2): LDS read addresses are loop-invariant
  // per-lane offsets plus immediates
  auto step = [&](int kt, auto cur_c) __attribute__((always_inline)) {
    constexpr int cur = decltype(cur_c)::value;
    const int kbase = kt * FWD_BN;
    wait_vm<0>();
    __syncthreads();  // tile kt visible; every wave is done with tile kt-1 (buffer cur ^ 1)
    if (kt + 1 < ntiles) issue_tile(cur ^ 1, kt + 1);
    if (DROP) {
      mword = mnext;
      if (kt + 1 < ntiles) mnext = mrow[(long)(kt + 1) * 2 * P.sq_pad];
    }
    if (HAS_KPM && tflag[kt] == 2) return;  // fully padded key tile: P = 0, no dQ contribution
    const uint16_t* Kb = KV + cur * 2 * TILE64;
    const uint16_t* Vb = Kb + TILE64;
    const bool tile_causal = CAUSAL && (kbase + FWD_BN - 1 > qw0 + P.causal_off);
    const int climit = qrow + P.causal_off - kbase;
    const float* lb = lut_s + (kbase - qrow + P.Sq - 1 - lut_base);
    const int sat = !HAS_BIAS ? 0
                    : (kbase + FWD_BN - 1 - qw0 + P.Sq - 1 <= P.sat_lo ? 1
                       : (kbase - qw0 - 31 + P.Sq - 1 >= P.sat_hi ? 2 : 0));
    // P = exp2(s * sl2 + bias - lse): saturated / bias-free tiles fold the constant bias and the row's lse into one
    // FMA operand (cl), LUT tiles add the bias by FMA and subtract lse.  dS = P * (dP * keep / (1 - p) - delta).
    const bool use_lut = HAS_BIAS && sat == 0;
    const float cl = (sat == 1 ? c_lo : (sat == 2 ? c_hi : 0.f)) - lse2;
    const bool masked = (HAS_KPM || kbase + FWD_BN > P.Sk) && tflag[kt] != 0;
    // the tile's two 32-key halves one after the other: S / dP accumulators of one half live at a time (32 fewer
    // VGPRs: the kernel fits the 168-register budget of 3 workgroups per CU)
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
      f32x16 sv = {}, pv = {};
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        sv = mfma32(as_frag(ld_row(Kb, 32 * kb + r, 2 * s + hh)), qf[s], sv);
        pv = mfma32(as_frag(ld_row(Vb, 32 * kb + r, 2 * s + hh)), dof[s], pv);
      }
      if (use_lut) {
#pragma unroll
        for (int i = 0; i < 16; ++i) sv[i] = fmaf(sv[i], sl2, lb[32 * kb + crow(i, hh)]) - lse2;
      } else {
#pragma unroll
        for (int i = 0; i < 16; ++i) sv[i] = fmaf(sv[i], sl2, cl);
      }
      if (CAUSAL && tile_causal) {
#pragma unroll
        for (int i = 0; i < 16; ++i) sv[i] = crow(i, hh) + 32 * kb > climit ? -INFINITY : sv[i];
      }
      if (masked) {
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const f32x4 m = *reinterpret_cast<const f32x4*>(kmask + kbase + 32 * kb + 8 * g + 4 * hh);
#pragma unroll
          for (int e = 0; e < 4; ++e) sv[4 * g + e] += m[e];
        }
      }
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const float pr = fast_exp2(sv[i]);  // lse = +inf for rows >= Sq -> 0
        float kf = 1.f;
        if (DROP)  // sign-extended bit -> all-ones mask -> dscale or 0.0f
          kf = __uint_as_float((uint32_t)__builtin_amdgcn_sbfe((int)mword, keep_bit(kb, i), 1) & dsbits);
        sv[i] = pr * fmaf(pv[i], kf, -delta);
      }
      // dQ^T += K^T dS^T over this half's 32 keys
      const bf16x8v d0 = pack8(sv, 0), d1 = pack8(sv, 8);
#pragma unroll
      for (int sp = 0; sp < 2; ++sp) {
        const int kb0 = kb * 32 + 16 * sp + 4 * hh;
        dq0 = mfma32(ld_tr_operand(Kb, kb0, 0, r), sp == 0 ? d0 : d1, dq0);
        dq1 = mfma32(ld_tr_operand(Kb, kb0, 1, r), sp == 0 ? d0 : d1, dq1);
      }
    }
  };
  for (int kt = 0; kt < ntiles; kt += 2) {
    step(kt, std::integral_constant<int, 0>{});
    if (kt + 1 < ntiles) step(kt + 1, std::integral_constant<int, 1>{});
  }
#if DQ_STAGE
  // every wave is done with the K/V buffers (the last tile's DMAs were waited for): they stage the dQ tiles
  __syncthreads();
  // column sums: the 4 waves' 64 sums at smem + 16 KB (past the 4 staging tiles, still inside the K/V buffers)
  float* red = CS ? reinterpret_cast<float*>(smem + 4 * 4096) : nullptr;
  store_rows_staged(smem + w * 4096, dq0, dq1, P.scale, r, hh, lane,
                    P.dq + b * P.dq_sb + (long)qw0 * P.dq_ss + h * P.dq_sh, P.dq_ss, P.Sq - qw0,
                    CS ? red + w * 64 : nullptr);
  if constexpr (CS) {
    __syncthreads();
    if (tid < 64)
      P.csq[(long)(b * P.n_tiles + qt) * P.csq_ld + h * 64 + tid] = red[tid] + red[64 + tid] + red[128 + tid] +
                                                                     red[192 + tid];
  }
#else
  if (qvalid) {
    uint16_t* dqp = P.dq + b * P.dq_sb + (long)qrow * P.dq_ss + h * P.dq_sh;
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const f32x16& acc = t == 0 ? dq0 : dq1;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        u16x4 pk = {f2bf(acc[4 * g] * P.scale), f2bf(acc[4 * g + 1] * P.scale), f2bf(acc[4 * g + 2] * P.scale),
                    f2bf(acc[4 * g + 3] * P.scale)};
        *reinterpret_cast<u16x4*>(dqp + 32 * t + 8 * g + 4 * hh) = pk;
      }
    }
  }
#endif
}

// ================================================================================== backward: dK, dV (v2)
// Key blocks of 128 (4 waves x 32 keys, key on the lane as in v1), query tiles of 64 rows per pipeline stage: the
// Q / dO tile, the per-row terms (attn_bwd_dq_kernel's rowrec: -lse, c_lo - lse, c_hi - lse, -delta) and the dropout
// keep words of the tile are moved by LDS-DMA two stages ahead into a 3-slot ring (no VGPR staging, one barrier per
// 64 rows; v1 moved 32 rows per barrier through registers one tile ahead, and its waves sat parked on the barrier
// and on the per-score lse / delta arithmetic half the time, profiles/r1_attn_pmc.txt).  Per score (saturated /
// bias-free tile): P = exp2(fma(s, sl2, rt)), keep = sbfe & dscale bits, Pd = P keep, dS = P fma(dP, keep, -delta).
constexpr int K2_QT = 64;
#ifndef DKDV_OPERANDS_AHEAD
#define DKDV_OPERANDS_AHEAD 1
#endif
constexpr int K2_NBUF = 3;
// timing ablations of the dK/dV kernel (A/B builds only, results are wrong; profiles/r4_dkdv_ablations.txt): 1 no
// bias-gradient diagonal sums, 2 no LUT bias reads, 4 no stage barrier, 8 no dV/dK MFMAs, 16 no dropout keep bits,
// 32 no row-term reads, 64 no exp
#ifndef DKDV_ABLATE
#define DKDV_ABLATE 0
#endif
#ifndef DKDV_SQ_STAGE
#define DKDV_SQ_STAGE 1
#endif
#ifndef DKDV2_STAGE
#define DKDV2_STAGE 1
#endif
constexpr int K2_STAGE = 2 * 64 * D * 2 + 1024 + 1024;  // Q, dO [64][64] bf16 + rowrec [4][64] f32 + keep [4][64] u32

// NB = stage ring depth: 3 (two stages in flight, 2 workgroups per CU) or 2 (one in flight, a 168-VGPR budget so 3
// workgroups share a CU; taken for the bias-free variants, which fit it)
template <bool HAS_BIAS, bool HAS_KPM, bool CAUSAL, bool DROP, int NB, bool CS = false>
__global__ __launch_bounds__(256, NB == 3 ? 2 : 3) void attn_bwd_dkdv2_kernel(AttnParams P) {
  static_assert(NB == 2 || NB == 3, "stage ring depth");
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  float* kmask = reinterpret_cast<float*>(smem + NB * K2_STAGE);  // [128]
  float* lut_r = kmask + BWD_BK;                                       // [Sq + 128 + 64] reversed, log2-scaled
  float* dlut_s = lut_r + (HAS_BIAS ? P.Sq + BWD_BK + K2_QT : 0);      // [Sq + 128]

  const int tid = threadIdx.x, w = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63, r = lane & 31,
            hh = lane >> 5;
  const int logical = xcd_remap(blockIdx.x, gridDim.x);
  const int kblk = logical % P.n_tiles;
  const int bh = logical / P.n_tiles;
  const int h = bh % P.H, b = bh / P.H;
  const int k0 = kblk * BWD_BK;
  const int kw0 = k0 + w * 32;
  const int key = kw0 + r;
  const bool kvalid = key < P.Sk;
  const int L = P.Sq + P.Sk - 1;
  const int win = P.Sq + BWD_BK;
  const float sl2 = P.scale * LOG2E;

  int qt_begin = 0;
  if (CAUSAL) {
    const int qmin = k0 - P.causal_off;  // first query that can see key k0
    qt_begin = qmin > 0 ? qmin / K2_QT : 0;
  }
  const int nqt_all = (P.Sq + K2_QT - 1) / K2_QT;
  // ---- stage DMA (per wave and stage: 2 + 2 Q / dO pieces of 8 rows, a quarter of the rowrec chunk, one keep column)
  const uint32_t st_lds = lds_addr(smem);
  const uint16_t* qbase_p = P.q + b * P.q_sb + h * P.q_sh;
  const uint16_t* dbase_p = P.dout + b * P.do_sb + h * P.do_sh;
  const uint32_t qss2 = (uint32_t)P.q_ss * 2u, dss2 = (uint32_t)P.do_ss * 2u;
  int drow[2];
  uint32_t dc16[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    drow[i] = 8 * (2 * w + i) + (lane >> 3);
    dc16[i] = (uint32_t)(((lane & 7) ^ swz(drow[i])) * 16);
  }
  const float* rec_src = P.rowrec + (long)bh * (P.sq_pad >> 6) * 256 + w * 64 + lane;
  const int ktf = min((k0 >> 6) + (w >> 1), P.n_ktiles - 1);
  const uint32_t* keep_src = DROP ? P.dmask + (((long)bh * P.n_ktiles + ktf) * 2 + (w & 1)) * P.sq_pad + lane : nullptr;
  auto issue = [&](int slot, int qt) {
    const uint32_t base = st_lds + (uint32_t)(slot * K2_STAGE);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const uint32_t qq = (uint32_t)min(qt * K2_QT + drow[i], P.Sq - 1);
      const uint32_t dst = base + (uint32_t)((2 * w + i) * 1024);
      bld16(qbase_p, __umul24(qq, qss2) + dc16[i], __builtin_amdgcn_readfirstlane(dst));
      bld16(dbase_p, __umul24(qq, dss2) + dc16[i], __builtin_amdgcn_readfirstlane(dst + TILE64 * 2));
    }
    glds4(rec_src + (long)qt * 256, __builtin_amdgcn_readfirstlane(base + 4 * TILE64 + w * 256));
    if (DROP) glds4(keep_src + qt * K2_QT, __builtin_amdgcn_readfirstlane(base + 4 * TILE64 + 1024 + w * 256));
  };
  constexpr int DPT = DROP ? 6 : 5;  // DMAs per wave and stage

  // the first two stages are issued before the prologue's global reads (bias LUT, key mask, K / V fragments): their
  // latencies overlap instead of adding up (short-Sq cross-attention blocks are prologue-bound).  A block whose keys
  // are all padding drains them unused (wait_vm<0> below) before it exits.
  if (qt_begin < nqt_all) issue(0, qt_begin);
  if (NB == 3 && qt_begin + 1 < nqt_all) issue(1, qt_begin + 1);
  if (HAS_BIAS) {
    const float* lrow = P.lut + (long)h * L;
    for (int t = tid; t < win + K2_QT; t += 256) {
      const int i = win - 1 - t, gi = k0 + i;
      lut_r[t] = (i >= 0 && gi < L) ? lrow[gi] * LOG2E : 0.f;
    }
    for (int i = tid; i < win; i += 256) dlut_s[i] = 0.f;
  }
  float sat_acc_lo = 0.f, sat_acc_hi = 0.f;
  bool key_ok = false;
  if (tid < BWD_BK) {
    const int kk = k0 + tid;
    key_ok = kk < P.Sk;
    if (HAS_KPM && key_ok) key_ok = P.kpm[(long)b * P.Sk + kk] != 0;
    kmask[tid] = key_ok ? 0.f : -INFINITY;
  }
  const bool block_live = !HAS_KPM || __syncthreads_or(key_ok ? 1 : 0);
  // some key of the block is padding or past Sk: the exponent gets the per-key mask (else nothing to add)
  const bool block_masked = __syncthreads_or((tid < BWD_BK && !key_ok) ? 1 : 0);
  bf16x8v kf[4], vf[4];
  {
    const uint16_t* kp = P.k + b * P.k_sb + (long)key * P.k_ss + h * P.k_sh;
    const uint16_t* vp = P.v + b * P.v_sb + (long)key * P.v_ss + h * P.v_sh;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      u16x8 a = {0, 0, 0, 0, 0, 0, 0, 0}, c = a;
      if (kvalid) {
        a = *reinterpret_cast<const u16x8*>(kp + 16 * s + 8 * hh);
        c = *reinterpret_cast<const u16x8*>(vp + 16 * s + 8 * hh);
      }
      kf[s] = as_frag(a);
      vf[s] = as_frag(c);
    }
  }
  // retire the fragment loads here: left pending, hipcc's waitcnt pass (blind to the asm DMAs) waits for them before
  // their first use inside the stage loop (vmcnt(0) in every ring-depth unrolled copy), draining the DMA ring
  asm volatile("" ::"v"(kf[0]), "v"(kf[1]), "v"(kf[2]), "v"(kf[3]), "v"(vf[0]), "v"(vf[1]), "v"(vf[2]), "v"(vf[3]));
  const float km = kmask[w * 32 + r];
  // this lane's dropout bit: the forward's lane (hh_f) and register (bit) that held (q, key)
  const int kl = key - k0, kc = kl & 31;
  const int mcol = (kl >> 6) * 2 + ((kc >> 2) & 1);
  const int mbit = keep_bit((kl >> 5) & 1, (kc & 3) + 4 * (kc >> 3));
  const float dscale = DROP ? 1.f / (1.f - P.p_drop) : 1.f;
  const uint32_t dsbits = __float_as_uint(dscale);

  const int nqt = block_live ? nqt_all : qt_begin;
  if (!block_live) wait_vm<0>();
  f32x16 dv0 = {}, dv1 = {}, dk0 = {}, dk1 = {};
  // one pipeline stage; the ring slot is a compile-time constant (the loop below is unrolled by the ring depth) so
  // every LDS read address is a loop-invariant per-lane offset plus an immediate: no per-stage address arithmetic
  auto stage = [&](int qt, auto slot_c) __attribute__((always_inline)) {
    constexpr int SLOT = decltype(slot_c)::value;
    if (NB == 3 && qt + 1 < nqt) wait_vm<DPT>();
    else wait_vm<0>();
    if constexpr ((DKDV_ABLATE & 4) == 0)
      __syncthreads();  // stage qt landed for every wave; every wave is done with stage qt - 1 (the slot refilled next)
    if (qt + NB - 1 < nqt) issue((SLOT + NB - 1) % NB, qt + NB - 1);
    const unsigned char* stg = smem + SLOT * K2_STAGE;
    const uint16_t* Qb = reinterpret_cast<const uint16_t*>(stg);
    const uint16_t* dOb = Qb + TILE64;
    const float* rec = reinterpret_cast<const float*>(stg + 4 * TILE64);
    const uint32_t* mwd = reinterpret_cast<const uint32_t*>(stg + 4 * TILE64 + 1024);
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int q0 = qt * K2_QT + 32 * u;
      f32x16 sacc = {}, dpacc = {};
      if constexpr (NB == 3 && DKDV_OPERANDS_AHEAD) {
        // all 8 operand rows in flight before the first MFMA (one LDS round trip; hipcc otherwise waits before each)
        bf16x8v qa[4], da[4];
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          qa[s] = as_frag(ld_row(Qb, 32 * u + r, 2 * s + hh));
          da[s] = as_frag(ld_row(dOb, 32 * u + r, 2 * s + hh));
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          sacc = mfma32(qa[s], kf[s], sacc);
          dpacc = mfma32(da[s], vf[s], dpacc);
        }
      } else {
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          sacc = mfma32(as_frag(ld_row(Qb, 32 * u + r, 2 * s + hh)), kf[s], sacc);
          dpacc = mfma32(as_frag(ld_row(dOb, 32 * u + r, 2 * s + hh)), vf[s], dpacc);
        }
      }
      const int sat = !HAS_BIAS ? 0
                      : (kw0 + 31 - q0 + P.Sq - 1 <= P.sat_lo ? 1 : (kw0 - q0 - 31 + P.Sq - 1 >= P.sat_hi ? 2 : 0));
      const bool use_lut = HAS_BIAS && sat == 0 && (DKDV_ABLATE & 2) == 0;
      f32x16 pd, ds;
      if constexpr (NB == 3) {  // all 16 row terms read up front: their LDS latency hides under the MFMAs
        // rows 32u + crow(i, hh): four consecutive rows per 16-B read
        const float* rt_row = rec + (use_lut ? 0 : (sat == 1 ? 64 : 128)) + 32 * u + 4 * hh;
        const float* nd_row = rec + 192 + 32 * u + 4 * hh;
        float rt[16], nd[16];
        uint32_t mw[16];
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          f32x4 a = {0.f, -1.f, 0.5f, 0.25f}, c = a;
          if constexpr ((DKDV_ABLATE & 32) == 0) {
            a = *reinterpret_cast<const f32x4*>(rt_row + 8 * g);
            c = *reinterpret_cast<const f32x4*>(nd_row + 8 * g);
          }
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            rt[4 * g + e] = a[e];
            nd[4 * g + e] = c[e];
          }
          if (DROP && (DKDV_ABLATE & 16) == 0) {
            const u32x4 v = *reinterpret_cast<const u32x4*>(mwd + mcol * 64 + 32 * u + 8 * g + 4 * hh);
#pragma unroll
            for (int e = 0; e < 4; ++e) mw[4 * g + e] = v[e];
          }
        }
        if (use_lut) {  // bias per (key - row) from the reversed LUT: immediate ds_read offsets per register
          const float* lrow_t = lut_r + (win - 1 - (key - q0 - 4 * hh + P.Sq - 1 - k0));
#pragma unroll
          for (int i0 = 0; i0 < 16; i0 += 8) {  // 8 reads in flight per batch (hipcc otherwise waits on each in turn)
            float lv[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) lv[i] = lrow_t[crow(i0 + i, 0)];
#pragma unroll
            for (int i = 0; i < 8; ++i) rt[i0 + i] += lv[i];
          }
        }
        if (block_masked) {  // padding / tail keys: -inf on the lane's whole column
#pragma unroll
          for (int i = 0; i < 16; ++i) rt[i] += km;
        }
        const bool tile_causal = CAUSAL && (kw0 + 31 > q0 + P.causal_off);
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const float x = fmaf(sacc[i], sl2, rt[i]);
          float pr = (DKDV_ABLATE & 64) ? x : fast_exp2(x);  // rows >= Sq: rt = -inf -> 0
          if (CAUSAL && tile_causal && key > q0 + crow(i, hh) + P.causal_off) pr = 0.f;
          float keepf = 1.f;
          if (DROP && (DKDV_ABLATE & 16) == 0) keepf = __uint_as_float((uint32_t)__builtin_amdgcn_sbfe((int)mw[i], mbit, 1) & dsbits);
          pd[i] = pr * keepf;
          ds[i] = pr * fmaf(dpacc[i], keepf, nd[i]);
        }
      } else {  // 2-deep ring at 168 VGPRs: row terms consumed group by group, P / dS in place
        // rows 32u + crow(i, hh): four consecutive rows per 16-B read, consumed group by group (12 live registers of
        // row terms instead of 48); P keep -> sacc, dS -> dpacc in place
        const float* rt_row = rec + (use_lut ? 0 : (sat == 1 ? 64 : 128)) + 32 * u + 4 * hh;
        const float* nd_row = rec + 192 + 32 * u + 4 * hh;
        const float* lrow_t = lut_r + (win - 1 - (key - q0 - 4 * hh + P.Sq - 1 - k0));
        const bool tile_causal = CAUSAL && (kw0 + 31 > q0 + P.causal_off);
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          f32x4 rt4 = *reinterpret_cast<const f32x4*>(rt_row + 8 * g);
          const f32x4 nd4 = *reinterpret_cast<const f32x4*>(nd_row + 8 * g);
          u32x4 mw4 = {0u, 0u, 0u, 0u};
          if (DROP) mw4 = *reinterpret_cast<const u32x4*>(mwd + mcol * 64 + 32 * u + 8 * g + 4 * hh);
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int i = 4 * g + e;
            float t = rt4[e];
            if (use_lut) t += lrow_t[crow(i, 0)];  // bias per (key - row) from the reversed LUT (immediate offsets)
            if (block_masked) t += km;             // padding / tail keys: -inf on the lane's whole column
            float pr = fast_exp2(fmaf(sacc[i], sl2, t));  // rows >= Sq: rt = -inf -> 0
            if (CAUSAL && tile_causal && key > q0 + crow(i, hh) + P.causal_off) pr = 0.f;
            float keepf = 1.f;
            if (DROP) keepf = __uint_as_float((uint32_t)__builtin_amdgcn_sbfe((int)mw4[e], mbit, 1) & dsbits);
            sacc[i] = pr * keepf;
            dpacc[i] = pr * fmaf(dpacc[i], keepf, nd4[e]);
          }
        }
        pd = sacc;
        ds = dpacc;
      }
      if (HAS_BIAS && sat != 0) {
        float t = 0.f;
#pragma unroll
        for (int i = 0; i < 16; ++i) t += ds[i];
        if (sat == 1) sat_acc_lo += t;
        else sat_acc_hi += t;
      } else if (HAS_BIAS && (DKDV_ABLATE & 1) == 0) {
        // diagonal sums of the wave's 32x32 dS tile: rotate register i (row rho = crow(i, hh)) left by rho
        // lanes so lane r receives element (rho, (r + rho) & 31) whose diagonal (col - row) is r or r - 32.
        // The rotations go out in batches of 8 before any is consumed (one LDS round trip per batch: issued one by one,
        // hipcc waited on each), the wrapped part is split off by one select per register (tot / neg), and the two sums
        // leave by one LDS atomic per lane, no divergent branch: lanes 0-31 add diagonal r, lanes 32-63 diagonal r - 32.
        const int rb = r + 4 * hh;  // r + rho = rb + crow(i, 0)
        float tot = 0.f, neg = 0.f;
#pragma unroll
        for (int i0 = 0; i0 < 16; i0 += 8) {
          float v[8];
#pragma unroll
          for (int i = 0; i < 8; ++i) v[i] = __shfl(ds[i0 + i], ((rb + crow(i0 + i, 0)) & 31) + 32 * hh, 64);
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            tot += v[i];
            neg += rb + crow(i0 + i, 0) < 32 ? 0.f : v[i];
          }
        }
        tot += __shfl_xor(tot, 32, 64);
        neg += __shfl_xor(neg, 32, 64);
        const int li = w * 32 + r - q0 + P.Sq - 1;
        const int la = hh == 0 ? li : li - 32;
        const float va = hh == 0 ? tot - neg : (li >= 32 ? neg : 0.f);
        atomicAdd(&dlut_s[la < 0 ? 0 : la], va);  // la < 0: rows past Sq only (dS = 0)
      }
      const bf16x8v pf0 = pack8(pd, 0), pf1 = pack8(pd, 8), sf0 = pack8(ds, 0), sf1 = pack8(ds, 8);
      if constexpr ((DKDV_ABLATE & 8) != 0) {
        asm volatile("" ::"v"(pf0), "v"(pf1), "v"(sf0), "v"(sf1));
      } else if constexpr (NB == 3 && DKDV_OPERANDS_AHEAD) {  // the 8 transposed operands (16 reads) in flight together
        bf16x8v ot[2][2], qtr[2][2];
#pragma unroll
        for (int sp = 0; sp < 2; ++sp) {
          const int c0 = 32 * u + 16 * sp + 4 * hh;
#pragma unroll
          for (int t = 0; t < 2; ++t) {
            ot[sp][t] = ld_tr_operand(dOb, c0, t, r);
            qtr[sp][t] = ld_tr_operand(Qb, c0, t, r);
          }
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int sp = 0; sp < 2; ++sp) {
          const bf16x8v pfv = sp == 0 ? pf0 : pf1, sfv = sp == 0 ? sf0 : sf1;
          dv0 = mfma32(ot[sp][0], pfv, dv0);
          dv1 = mfma32(ot[sp][1], pfv, dv1);
          dk0 = mfma32(qtr[sp][0], sfv, dk0);
          dk1 = mfma32(qtr[sp][1], sfv, dk1);
        }
      } else {
#pragma unroll
        for (int sp = 0; sp < 2; ++sp) {
          const int c0 = 32 * u + 16 * sp + 4 * hh;
          const bf16x8v pfv = sp == 0 ? pf0 : pf1, sfv = sp == 0 ? sf0 : sf1;
          dv0 = mfma32(ld_tr_operand(dOb, c0, 0, r), pfv, dv0);
          dv1 = mfma32(ld_tr_operand(dOb, c0, 1, r), pfv, dv1);
          dk0 = mfma32(ld_tr_operand(Qb, c0, 0, r), sfv, dk0);
          dk1 = mfma32(ld_tr_operand(Qb, c0, 1, r), sfv, dk1);
        }
      }
    }
  };
  for (int qt = qt_begin; qt < nqt; qt += NB) {  // unrolled by the ring depth
    stage(qt, std::integral_constant<int, 0>{});
    if (qt + 1 < nqt) stage(qt + 1, std::integral_constant<int, 1>{});
    if constexpr (NB == 3) {
      if (qt + 2 < nqt) stage(qt + 2, std::integral_constant<int, 2>{});
    }
  }

#if DKDV2_STAGE
  {
    // every wave is done with the stage ring (its last stage drained the DMAs): reuse it to stage the wave's 32 x 64 dK
    // and dV tiles (16-B chunks XOR-swizzled by row) and store whole 128-B key rows, 8 full-line stores per wave
    // instead of 16 per-lane stores touching 32 lines each (as attn_bwd_dkdv_sq_kernel)
    __syncthreads();
    unsigned char* scr = smem + w * 8192;
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const f32x16& ak = t == 0 ? dk0 : dk1;
      const f32x16& av = t == 0 ? dv0 : dv1;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        u16x4 pk = {f2bf(ak[4 * g] * P.scale), f2bf(ak[4 * g + 1] * P.scale), f2bf(ak[4 * g + 2] * P.scale),
                    f2bf(ak[4 * g + 3] * P.scale)};
        u16x4 pv = {f2bf(av[4 * g]), f2bf(av[4 * g + 1]), f2bf(av[4 * g + 2]), f2bf(av[4 * g + 3])};
        const int off = r * 128 + (((4 * t + g) ^ (r & 7)) << 4) + 8 * hh;
        *reinterpret_cast<u16x4*>(scr + off) = pk;
        *reinterpret_cast<u16x4*>(scr + 4096 + off) = pv;
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // other lanes of this wave read what these wrote
    float ak[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, av[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int st = 0; st < 4; ++st) {
      const int row = 8 * st + (lane >> 3), ch = lane & 7;
      const int off = row * 128 + ((ch ^ (row & 7)) << 4);
      const u16x8 vk = *reinterpret_cast<const u16x8*>(scr + off);
      const u16x8 vv = *reinterpret_cast<const u16x8*>(scr + 4096 + off);
      const int ks = kw0 + row;
      if (ks < P.Sk) {
        *reinterpret_cast<u16x8*>(P.dk + b * P.dk_sb + (long)ks * P.dk_ss + h * P.dk_sh + 8 * ch) = vk;
        *reinterpret_cast<u16x8*>(P.dv + b * P.dv_sb + (long)ks * P.dv_ss + h * P.dv_sh + 8 * ch) = vv;
        if constexpr (CS) {
          cs_add(ak, vk);
          cs_add(av, vv);
        }
      }
    }
    if constexpr (CS) {
      // column sums (cs_wave): [wave][dK 64 | dV 64] at smem + 32 KB, past the 4 waves' 8 KB staging areas and
      // inside the drained stage ring (NB * K2_STAGE >= 36 KB)
      float* red = reinterpret_cast<float*>(smem + 4 * 8192);
      cs_wave(ak, lane, red + w * 128);
      cs_wave(av, lane, red + w * 128 + 64);
      __syncthreads();
      if (tid < 128) {
        const int c = tid & 63, which = tid >> 6;
        const float s = red[which * 64 + c] + red[128 + which * 64 + c] + red[256 + which * 64 + c] +
                        red[384 + which * 64 + c];
        (which == 0 ? P.csk : P.csv)[(long)(b * P.n_tiles + kblk) * P.cskv_ld + h * 64 + c] = s;
      }
    }
  }
#else
  if (kvalid) {
    uint16_t* dkp = P.dk + b * P.dk_sb + (long)key * P.dk_ss + h * P.dk_sh;
    uint16_t* dvp = P.dv + b * P.dv_sb + (long)key * P.dv_ss + h * P.dv_sh;
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const f32x16& ak = t == 0 ? dk0 : dk1;
      const f32x16& av = t == 0 ? dv0 : dv1;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        u16x4 pk = {f2bf(ak[4 * g] * P.scale), f2bf(ak[4 * g + 1] * P.scale), f2bf(ak[4 * g + 2] * P.scale),
                    f2bf(ak[4 * g + 3] * P.scale)};
        u16x4 pv = {f2bf(av[4 * g]), f2bf(av[4 * g + 1]), f2bf(av[4 * g + 2]), f2bf(av[4 * g + 3])};
        *reinterpret_cast<u16x4*>(dkp + 32 * t + 8 * g + 4 * hh) = pk;
        *reinterpret_cast<u16x4*>(dvp + 32 * t + 8 * g + 4 * hh) = pv;
      }
    }
  }
#endif
  if (HAS_BIAS) {
    __syncthreads();
    float* grow = P.dlut + (long)h * L;
    for (int i = tid; i < win; i += 256) {
      const int gi = k0 + i;
      const float v = dlut_s[i];
      if (gi < L && v != 0.f) atomicAdd(grow + gi, v);
    }
    const float a_lo = wave_sum(sat_acc_lo), a_hi = wave_sum(sat_acc_hi);
    if (lane == 0) {
      if (a_lo != 0.f) atomicAdd(grow, a_lo);
      if (a_hi != 0.f) atomicAdd(grow + L - 1, a_hi);
    }
  }
}

// ================================================================================== backward: dK, dV, short queries
// Cross-attention (T5 / BART decoder queries against the encoder keys: Sq <= 128, no bias, no causal mask).  The whole
// query side of one (b, h) — Q, dO and the per-row terms, two 64-row stages — stays in LDS while one workgroup walks MB
// consecutive key blocks of 128, loading block j + 1's K / V fragments, key flags and dropout keep words while block
// j computes.  attn_bwd_dkdv2_kernel starts one workgroup per key block instead, each re-staging the query side and
// waiting on its own K / V loads before two short stages: prologue-latency bound at this shape.  Per score: the
// bias-free body of attn_bwd_dkdv2_kernel (P = exp2(fma(s, sl2, rt)), Pd = P keep, dS = P fma(dP, keep, -delta)).
template <bool HAS_KPM, bool DROP, int MB, bool CS = false>
__global__ __launch_bounds__(256, 2) void attn_bwd_dkdv_sq_kernel(AttnParams P) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  // [2 stages of K2_STAGE: Q | dO | row terms (1 KB) | unused], keep words [2 parities][2 stages][1 KB], key mask [128],
  // (DKDV_SQ_STAGE) per-wave 8 KB store staging
  const uint32_t* keepb = reinterpret_cast<const uint32_t*>(smem + 2 * K2_STAGE);
  float* kmask = reinterpret_cast<float*>(smem + 2 * K2_STAGE + 4096);

  const int tid = threadIdx.x, w = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63, r = lane & 31,
            hh = lane >> 5;
  const int ngrp = (P.n_tiles + MB - 1) / MB;
  const int logical = xcd_remap(blockIdx.x, gridDim.x);
  const int grp = logical % ngrp;
  const int bh = logical / ngrp;
  const int h = bh % P.H, b = bh / P.H;
  const int kb_begin = grp * MB;
  const int kb_end = min(kb_begin + MB, P.n_tiles);
  const float sl2 = P.scale * LOG2E;
  const int nqt = (P.Sq + K2_QT - 1) / K2_QT;  // 1 or 2: the launcher takes this kernel for Sq <= 128 only
  const uint32_t st_lds = lds_addr(smem);

  // query side, once: Q / dO pieces and the row terms of every stage (the DMA pieces of attn_bwd_dkdv2_kernel)
  {
    const uint16_t* qbase_p = P.q + b * P.q_sb + h * P.q_sh;
    const uint16_t* dbase_p = P.dout + b * P.do_sb + h * P.do_sh;
    const uint32_t qss2 = (uint32_t)P.q_ss * 2u, dss2 = (uint32_t)P.do_ss * 2u;
    const float* rec_src = P.rowrec + (long)bh * (P.sq_pad >> 6) * 256 + w * 64 + lane;
    for (int qt = 0; qt < nqt; ++qt) {
      const uint32_t base = st_lds + (uint32_t)(qt * K2_STAGE);
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int drow = 8 * (2 * w + i) + (lane >> 3);
        const uint32_t dc16 = (uint32_t)(((lane & 7) ^ swz(drow)) * 16);
        const uint32_t qq = (uint32_t)min(qt * K2_QT + drow, P.Sq - 1);
        const uint32_t dst = base + (uint32_t)((2 * w + i) * 1024);
        bld16(qbase_p, __umul24(qq, qss2) + dc16, __builtin_amdgcn_readfirstlane(dst));
        bld16(dbase_p, __umul24(qq, dss2) + dc16, __builtin_amdgcn_readfirstlane(dst + TILE64 * 2));
      }
      glds4(rec_src + (long)qt * 256, __builtin_amdgcn_readfirstlane(base + 4 * TILE64 + w * 256));
    }
  }
  // this lane's key inside a block and its dropout bit (the forward's lane half and register that held (q, key))
  const int kl = w * 32 + r, kc = kl & 31;
  const int mcol = (kl >> 6) * 2 + ((kc >> 2) & 1);
  const int mbit = keep_bit((kl >> 5) & 1, (kc & 3) + 4 * (kc >> 3));
  const uint32_t dsbits = __float_as_uint(DROP ? 1.f / (1.f - P.p_drop) : 1.f);

  // per key block: wave w's keep-word column (64-key tile 2 kb + w / 2, lane half w & 1) for every stage
  auto issue_keep = [&](int kb, int par) __attribute__((always_inline)) {
    if constexpr (DROP) {
      const int ktf = min(2 * kb + (w >> 1), P.n_ktiles - 1);
      const uint32_t* src = P.dmask + (((long)bh * P.n_ktiles + ktf) * 2 + (w & 1)) * P.sq_pad + lane;
      for (int qt = 0; qt < nqt; ++qt)
        glds4(src + qt * K2_QT,
              __builtin_amdgcn_readfirstlane(st_lds + 2 * K2_STAGE + (uint32_t)((par * 2 + qt) * 1024 + w * 256)));
    }
  };
  auto load_kv = [&](int kb, bf16x8v(&kf)[4], bf16x8v(&vf)[4]) __attribute__((always_inline)) {
    const int key = kb * BWD_BK + kl;
    const bool kvalid = key < P.Sk;
    const uint16_t* kp = P.k + b * P.k_sb + (long)key * P.k_ss + h * P.k_sh;
    const uint16_t* vp = P.v + b * P.v_sb + (long)key * P.v_ss + h * P.v_sh;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      u16x8 a = {0, 0, 0, 0, 0, 0, 0, 0}, c = a;
      if (kvalid) {
        a = *reinterpret_cast<const u16x8*>(kp + 16 * s + 8 * hh);
        c = *reinterpret_cast<const u16x8*>(vp + 16 * s + 8 * hh);
      }
      kf[s] = as_frag(a);
      vf[s] = as_frag(c);
    }
  };
  auto key_flag = [&](int kb) __attribute__((always_inline)) {
    const int kk = kb * BWD_BK + tid;
    bool ok = tid < BWD_BK && kk < P.Sk;
    if (HAS_KPM && ok) ok = P.kpm[(long)b * P.Sk + kk] != 0;
    return ok;
  };

  // Each block: key flags -> mask, prefetch of the next block, stages, then ONE drain (wait_vm<0>: the prefetch and the
  // previous block's dK / dV stores, both issued a whole block earlier) and barrier before this block's stores — the
  // barrier also retires every wave's reads of the key mask and keep slot the next block's writes reuse.  Waiting on
  // everything (not a counted vmcnt) keeps it correct when a wave skips loads or stores for keys past Sk.
  bf16x8v kf[4], vf[4], kfn[4], vfn[4];
  issue_keep(kb_begin, 0);
  load_kv(kb_begin, kf, vf);
  bool key_ok = key_flag(kb_begin);
  wait_vm<0>();
  __syncthreads();
  for (int kb = kb_begin; kb < kb_end; ++kb) {
    const int par = (kb - kb_begin) & 1;
    const int key = kb * BWD_BK + kl;
    if (tid < BWD_BK) kmask[tid] = key_ok ? 0.f : -INFINITY;
    const bool block_live = !HAS_KPM || __syncthreads_or(key_ok ? 1 : 0);
    const bool block_masked = __syncthreads_or((tid < BWD_BK && !key_ok) ? 1 : 0);
    const float km = block_masked ? kmask[kl] : 0.f;
    const bool more = kb + 1 < kb_end;
    if (more) {  // next block's inputs, in flight during this block's stages
      issue_keep(kb + 1, par ^ 1);
      load_kv(kb + 1, kfn, vfn);
      key_ok = key_flag(kb + 1);
    }
    f32x16 dv0 = {}, dv1 = {}, dk0 = {}, dk1 = {};
    if (block_live) {
      for (int qt = 0; qt < nqt; ++qt) {
        const unsigned char* stg = smem + qt * K2_STAGE;
        const uint16_t* Qb = reinterpret_cast<const uint16_t*>(stg);
        const uint16_t* dOb = Qb + TILE64;
        const float* rec = reinterpret_cast<const float*>(stg + 4 * TILE64);
        const uint32_t* mwd = keepb + (par * 2 + qt) * 256;
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          f32x16 sacc = {}, dpacc = {};
#pragma unroll
          for (int s = 0; s < 4; ++s) {
            sacc = mfma32(as_frag(ld_row(Qb, 32 * u + r, 2 * s + hh)), kf[s], sacc);
            dpacc = mfma32(as_frag(ld_row(dOb, 32 * u + r, 2 * s + hh)), vf[s], dpacc);
          }
          // row terms of rows 32 u + crow(i, hh): the bias-free -lse at 128.., -delta at 192..
          const float* rt_row = rec + 128 + 32 * u + 4 * hh;
          const float* nd_row = rec + 192 + 32 * u + 4 * hh;
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            const f32x4 rt4 = *reinterpret_cast<const f32x4*>(rt_row + 8 * g);
            const f32x4 nd4 = *reinterpret_cast<const f32x4*>(nd_row + 8 * g);
            u32x4 mw4 = {0u, 0u, 0u, 0u};
            if (DROP) mw4 = *reinterpret_cast<const u32x4*>(mwd + mcol * 64 + 32 * u + 8 * g + 4 * hh);
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const int i = 4 * g + e;
              const float pr = fast_exp2(fmaf(sacc[i], sl2, rt4[e] + km));  // rows >= Sq: rt = -inf -> 0
              float keepf = 1.f;
              if (DROP) keepf = __uint_as_float((uint32_t)__builtin_amdgcn_sbfe((int)mw4[e], mbit, 1) & dsbits);
              sacc[i] = pr * keepf;
              dpacc[i] = pr * fmaf(dpacc[i], keepf, nd4[e]);
            }
          }
          const bf16x8v pf0 = pack8(sacc, 0), pf1 = pack8(sacc, 8), sf0 = pack8(dpacc, 0), sf1 = pack8(dpacc, 8);
#pragma unroll
          for (int sp = 0; sp < 2; ++sp) {
            const int c0 = 32 * u + 16 * sp + 4 * hh;
            const bf16x8v pfv = sp == 0 ? pf0 : pf1, sfv = sp == 0 ? sf0 : sf1;
            dv0 = mfma32(ld_tr_operand(dOb, c0, 0, r), pfv, dv0);
            dv1 = mfma32(ld_tr_operand(dOb, c0, 1, r), pfv, dv1);
            dk0 = mfma32(ld_tr_operand(Qb, c0, 0, r), sfv, dk0);
            dk1 = mfma32(ld_tr_operand(Qb, c0, 1, r), sfv, dk1);
          }
        }
      }
    }
    wait_vm<0>();
    __syncthreads();
#if DKDV_SQ_STAGE
    {
      // the wave's 32 x 64 dK and dV tiles through its LDS scratch (16-B chunks XOR-swizzled by row), then whole
      // 128-B key rows: 8 full-line stores per wave instead of 16 stores of 16 B into 32 lines each
      unsigned char* scr = smem + 2 * K2_STAGE + 4096 + BWD_BK * 4 + w * 8192;
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const f32x16& ak = t == 0 ? dk0 : dk1;
        const f32x16& av = t == 0 ? dv0 : dv1;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          u16x4 pk = {f2bf(ak[4 * g] * P.scale), f2bf(ak[4 * g + 1] * P.scale), f2bf(ak[4 * g + 2] * P.scale),
                      f2bf(ak[4 * g + 3] * P.scale)};
          u16x4 pv = {f2bf(av[4 * g]), f2bf(av[4 * g + 1]), f2bf(av[4 * g + 2]), f2bf(av[4 * g + 3])};
          const int off = r * 128 + (((4 * t + g) ^ (r & 7)) << 4) + 8 * hh;
          *reinterpret_cast<u16x4*>(scr + off) = pk;
          *reinterpret_cast<u16x4*>(scr + 4096 + off) = pv;
        }
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // other lanes of this wave read what these wrote
      float ak[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, av[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int st = 0; st < 4; ++st) {
        const int row = 8 * st + (lane >> 3), ch = lane & 7;
        const int off = row * 128 + ((ch ^ (row & 7)) << 4);
        const u16x8 vk = *reinterpret_cast<const u16x8*>(scr + off);
        const u16x8 vv = *reinterpret_cast<const u16x8*>(scr + 4096 + off);
        const int ks = kb * BWD_BK + w * 32 + row;
        if (ks < P.Sk) {
          *reinterpret_cast<u16x8*>(P.dk + b * P.dk_sb + (long)ks * P.dk_ss + h * P.dk_sh + 8 * ch) = vk;
          *reinterpret_cast<u16x8*>(P.dv + b * P.dv_sb + (long)ks * P.dv_ss + h * P.dv_sh + 8 * ch) = vv;
          if constexpr (CS) {
            cs_add(ak, vk);
            cs_add(av, vv);
          }
        }
      }
      if constexpr (CS) {
        // column sums (cs_wave): [wave][dK 64 | dV 64] in the 2 KB past the staging areas (lds_sq); the next key
        // block's writes come after its own barrier above
        float* red = reinterpret_cast<float*>(smem + 2 * K2_STAGE + 4096 + BWD_BK * 4 + 4 * 8192);
        cs_wave(ak, lane, red + w * 128);
        cs_wave(av, lane, red + w * 128 + 64);
        __syncthreads();
        if (tid < 128) {
          const int c = tid & 63, which = tid >> 6;
          const float s = red[which * 64 + c] + red[128 + which * 64 + c] + red[256 + which * 64 + c] +
                          red[384 + which * 64 + c];
          (which == 0 ? P.csk : P.csv)[(long)(b * P.n_tiles + kb) * P.cskv_ld + h * 64 + c] = s;
        }
      }
    }
#else
    if (key < P.Sk) {
      uint16_t* dkp = P.dk + b * P.dk_sb + (long)key * P.dk_ss + h * P.dk_sh;
      uint16_t* dvp = P.dv + b * P.dv_sb + (long)key * P.dv_ss + h * P.dv_sh;
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const f32x16& ak = t == 0 ? dk0 : dk1;
        const f32x16& av = t == 0 ? dv0 : dv1;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          u16x4 pk = {f2bf(ak[4 * g] * P.scale), f2bf(ak[4 * g + 1] * P.scale), f2bf(ak[4 * g + 2] * P.scale),
                      f2bf(ak[4 * g + 3] * P.scale)};
          u16x4 pv = {f2bf(av[4 * g]), f2bf(av[4 * g + 1]), f2bf(av[4 * g + 2]), f2bf(av[4 * g + 3])};
          *reinterpret_cast<u16x4*>(dkp + 32 * t + 8 * g + 4 * hh) = pk;
          *reinterpret_cast<u16x4*>(dvp + 32 * t + 8 * g + 4 * hh) = pv;
        }
      }
    }
#endif
    if (more) {
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        kf[s] = kfn[s];
        vf[s] = vfn[s];
      }
    }
  }
}

#define DISPATCH4(FN, hb, hk, ca, dr, ...)                                              \
  do {                                                                                  \
    if (hb) {                                                                           \
      if (hk) { if (ca) { if (dr) FN<true, true, true, true>(__VA_ARGS__); else FN<true, true, true, false>(__VA_ARGS__); } \
                else { if (dr) FN<true, true, false, true>(__VA_ARGS__); else FN<true, true, false, false>(__VA_ARGS__); } } \
      else { if (ca) { if (dr) FN<true, false, true, true>(__VA_ARGS__); else FN<true, false, true, false>(__VA_ARGS__); } \
             else { if (dr) FN<true, false, false, true>(__VA_ARGS__); else FN<true, false, false, false>(__VA_ARGS__); } } \
    } else {                                                                            \
      if (hk) { if (ca) { if (dr) FN<false, true, true, true>(__VA_ARGS__); else FN<false, true, true, false>(__VA_ARGS__); } \
                else { if (dr) FN<false, true, false, true>(__VA_ARGS__); else FN<false, true, false, false>(__VA_ARGS__); } } \
      else { if (ca) { if (dr) FN<false, false, true, true>(__VA_ARGS__); else FN<false, false, true, false>(__VA_ARGS__); } \
             else { if (dr) FN<false, false, false, true>(__VA_ARGS__); else FN<false, false, false, false>(__VA_ARGS__); } } \
    }                                                                                   \
  } while (0)

template <bool HB, bool HK, bool CA, bool DR>
void launch_fwd_t(const AttnParams& p, int nblk, size_t lds, hipStream_t st) {
  // lds was sized for the 3-deep ring; the 2-deep one drops one K/V buffer pair and one keep-bit slot
  const size_t lds2 = lds - (size_t)2 * TILE64 * 2 - 256 * 4;
  // 3 workgroups per CU on the 2-deep ring: t5-base encoder forward -10 % (profiles/r2_attn_fwd_occ3.txt)
  if (3 * lds2 <= 160 * 1024) {
    if (DR && p.dmask_ready)
      hipLaunchKernelGGL((attn_fwd_kernel<HB, HK, CA, DR, true, 2>), dim3(nblk), dim3(256), lds2, st, p);
    else
      hipLaunchKernelGGL((attn_fwd_kernel<HB, HK, CA, DR, false, 2>), dim3(nblk), dim3(256), lds2, st, p);
    return;
  }
  if (DR && p.dmask_ready)
    hipLaunchKernelGGL((attn_fwd_kernel<HB, HK, CA, DR, true, 3>), dim3(nblk), dim3(256), lds, st, p);
  else
    hipLaunchKernelGGL((attn_fwd_kernel<HB, HK, CA, DR, false, 3>), dim3(nblk), dim3(256), lds, st, p);
}
template <bool HB, bool HK, bool CA, bool DR>
void launch_bwd_dq_t(const AttnParams& p, int nblk, size_t lds, hipStream_t st) {
  // 2 workgroups per CU (3 measured equal, profiles/r2_ab_attn_dq_halves.txt and r5_dq_occ_rounds_ab.txt)
  if constexpr (!HB) {
    if (p.csq != nullptr) {  // column sums for the q-projection bias (BART)
      hipLaunchKernelGGL((attn_bwd_dq_kernel<HB, HK, CA, DR, 2, true>), dim3(nblk), dim3(256), lds, st, p);
      return;
    }
  }
  hipLaunchKernelGGL((attn_bwd_dq_kernel<HB, HK, CA, DR, 2>), dim3(nblk), dim3(256), lds, st, p);
}
template <bool HB, bool HK, bool CA, bool DR>
void launch_bwd_dkdv2_t(const AttnParams& p, int nblk, size_t lds, hipStream_t st) {
  const size_t lds2 = lds - K2_STAGE;  // lds was sized for the 3-deep ring
  // bias- and dropout-free variants: they fit 168 VGPRs without spills (BART-large shapes: bwd -4..6 %, bench
  // +0.8 %, profiles/r2_attn_dkdv_occ3.txt).  The dropout variant spills (7 VGPRs bias-free) and measured 2 % slower on
  // self-attention, but short-query (Sq <= 256) bias-free calls — T5 cross-attention, two 64-row stages per key block,
  // prologue-latency bound — gain from the third workgroup: step -0.5 % (profiles/r3_cross_dkdv_occ3_ab.txt);
  if (!HB && (!DR || p.Sq <= 256) && 3 * lds2 <= 160 * 1024) {
    if constexpr (!HB) {
      if (p.csk != nullptr) {  // column sums for the k / v projection biases (BART)
        hipLaunchKernelGGL((attn_bwd_dkdv2_kernel<HB, HK, CA, DR, 2, true>), dim3(nblk), dim3(256), lds2, st, p);
        return;
      }
    }
    hipLaunchKernelGGL((attn_bwd_dkdv2_kernel<HB, HK, CA, DR, 2>), dim3(nblk), dim3(256), lds2, st, p);
    return;
  }
  if constexpr (!HB) {
    if (p.csk != nullptr) {
      hipLaunchKernelGGL((attn_bwd_dkdv2_kernel<HB, HK, CA, DR, 3, true>), dim3(nblk), dim3(256), lds, st, p);
      return;
    }
  }
  static size_t attr = 64 * 1024;  // dynamic LDS above 64 KB (long sequences with bias) must be opted into
  if (lds > attr) {
    (void)hipFuncSetAttribute((const void*)attn_bwd_dkdv2_kernel<HB, HK, CA, DR, 3>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr = lds;
  }
  hipLaunchKernelGGL((attn_bwd_dkdv2_kernel<HB, HK, CA, DR, 3>), dim3(nblk), dim3(256), lds, st, p);
}

template <bool HK, bool DR, int MB, bool CS>
void launch_bwd_dkdv_sq_cs(const AttnParams& p, dim3 grid, size_t lds, hipStream_t st) {
  static bool attr = false;  // the staged epilogue puts the dynamic LDS above the 64 KB default
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)attn_bwd_dkdv_sq_kernel<HK, DR, MB, CS>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    attr = true;
  }
  hipLaunchKernelGGL((attn_bwd_dkdv_sq_kernel<HK, DR, MB, CS>), grid, dim3(256), lds, st, p);
}

template <bool HK, bool DR, int MB>
void launch_bwd_dkdv_sq_mb(const AttnParams& p, dim3 grid, size_t lds, hipStream_t st) {
  if (p.csk != nullptr) launch_bwd_dkdv_sq_cs<HK, DR, MB, true>(p, grid, lds, st);
  else launch_bwd_dkdv_sq_cs<HK, DR, MB, false>(p, grid, lds, st);
}

template <bool HK, bool DR>
void launch_bwd_dkdv_sq_t(const AttnParams& p, int mb, size_t lds, hipStream_t st) {
  const long ng = (p.n_tiles + mb - 1) / mb;
  const dim3 grid((unsigned)(ng * p.H * p.B));
  if (mb >= 8) launch_bwd_dkdv_sq_mb<HK, DR, 8>(p, grid, lds, st);
  else if (mb >= 4) launch_bwd_dkdv_sq_mb<HK, DR, 4>(p, grid, lds, st);
  else launch_bwd_dkdv_sq_mb<HK, DR, 2>(p, grid, lds, st);
}

}  // namespace

// The K/V tile DMA addresses rows with 32-bit byte offsets from v_mad_u32_u24 (csrc/attn.hip issue_tile).
static bool kv_offsets_fit(const AttnParams& p) {
  const long kss2 = p.k_ss * 2, vss2 = p.v_ss * 2;
  return kss2 > 0 && vss2 > 0 && kss2 < (1L << 24) && vss2 < (1L << 24) && p.Sk < (1 << 24) &&
         (long)p.Sk * (kss2 > vss2 ? kss2 : vss2) + 256 < (1L << 31);
}

extern "C" int dllm_attn_fwd(AttnParams* pp, hipStream_t st) {
  AttnParams p = *pp;
  if (!kv_offsets_fit(p)) return -6;
  p.thr = drop_threshold(p.p_drop);
  p.n_tiles = (p.Sq + FWD_BM - 1) / FWD_BM;
  const long nblk = (long)p.n_tiles * p.H * p.B;
  p.n_ktiles = (p.Sk + FWD_BN - 1) / FWD_BN;
  p.sq_pad = p.n_tiles * FWD_BM;
  if (p.p_drop > 0.f && p.dmask == nullptr) return -5;  // the caller allocates the dropout bit planes
  // 3 K/V buffers + per-key mask + bias LUT window
  size_t lds = (size_t)6 * TILE64 * 2 + 3 * 256 * 4 + (size_t)p.n_ktiles * (FWD_BN + 1) * 4;
  if (p.lut) lds += (size_t)(p.Sk + FWD_BM + FWD_BN) * 4;
  if (nblk <= 0 || nblk > 0x7fffffff || lds > 160 * 1024) return -4;
  DISPATCH4(launch_fwd_t, p.lut != nullptr, p.kpm != nullptr, p.causal != 0, p.p_drop > 0.f, p, (int)nblk, lds, st);
  DLLM_CHECK_LAUNCH();
  return 0;
}

extern "C" int dllm_attn_bwd(AttnParams* pp, hipStream_t st) {
  AttnParams p = *pp;
  if (!kv_offsets_fit(p)) return -6;
  p.thr = drop_threshold(p.p_drop);
  // 1) dQ (+ delta): query blocks, forward geometry
  p.n_tiles = (p.Sq + FWD_BM - 1) / FWD_BM;
  p.n_ktiles = (p.Sk + FWD_BN - 1) / FWD_BN;
  p.sq_pad = p.n_tiles * FWD_BM;
  if (p.p_drop > 0.f && p.dmask == nullptr) return -5;
  // column sums need the staged stores of all three kernels (and the v2 / short-query dK/dV kernels)
  // (the column-sum variants are instantiated for the bias-LUT-free kernels only)
  if ((p.csq != nullptr || p.csk != nullptr) &&
      (!DQ_STAGE || !DKDV2_STAGE || !DKDV_SQ_STAGE || p.rowrec == nullptr || p.lut != nullptr))
    return -7;
  if ((p.csk == nullptr) != (p.csv == nullptr)) return -7;
  long nblk = (long)p.n_tiles * p.H * p.B;
  // 2 K/V buffers + per-key mask + tile flags + bias LUT window
  size_t lds = (size_t)4 * TILE64 * 2 + (size_t)p.n_ktiles * (FWD_BN + 1) * 4;
  if (p.lut) lds += (size_t)(p.Sk + FWD_BM + FWD_BN) * 4;
  if (nblk <= 0 || nblk > 0x7fffffff || lds > 160 * 1024) return -4;
  DISPATCH4(launch_bwd_dq_t, p.lut != nullptr, p.kpm != nullptr, p.causal != 0, p.p_drop > 0.f, p, (int)nblk, lds,
            st);
  DLLM_CHECK_LAUNCH();
  // 2) dK, dV (+ bias-LUT gradient): key blocks
  p.n_tiles = (p.Sk + BWD_BK - 1) / BWD_BK;
  nblk = (long)p.n_tiles * p.H * p.B;
  // short-query cross-attention (Sq <= 128, no bias, not causal): one workgroup walks MB key blocks with the query
  // side resident (attn_bwd_dkdv_sq_kernel) — the largest MB in {4, 2} that still launches 6 workgroups per CU (3
  // rounds at 2 per CU); smaller launches keep one workgroup per key block (dkdv2).  Batch sweep at the T5 cross
  // shape: dkdv2 wins at batch 8 / 16, MB 2 at 32, MB 4 from 64.  In the t5-base b=512 step: 15.34 -> 13.50 ms/step
  // (MB 8: 14.10), profiles/r4_dkdv_sq_ab.txt
  constexpr int sq_cap = 4;
  static const int cus = [] {
    int dev = 0, n = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev);
    return n > 0 ? n : 256;
  }();
  // DLLM_ROUTE attn_dkdv_sq_force=1 (read per call; tests): the largest allowed MB whatever the launch size
  const bool force = route_int("attn_dkdv_sq_force", 0) == 1;
  int mb = 0;
  for (int m = 8; m >= 2; m /= 2)
    if (m <= sq_cap && mb == 0 && (force || (long)((p.n_tiles + m - 1) / m) * p.H * p.B >= 6L * cus)) mb = m;
  if (p.rowrec != nullptr && p.lut == nullptr && !p.causal && p.Sq <= 2 * K2_QT && mb > 1 && p.n_tiles >= 2) {
    const size_t lds_sq = (size_t)2 * K2_STAGE + 4096 + BWD_BK * 4 + (DKDV_SQ_STAGE ? 4 * 8192 + 2048 : 0);
    if ((long)((p.n_tiles + mb - 1) / mb) * p.H * p.B > 0x7fffffff) return -4;
    if (p.kpm != nullptr) {
      if (p.p_drop > 0.f) launch_bwd_dkdv_sq_t<true, true>(p, mb, lds_sq, st);
      else launch_bwd_dkdv_sq_t<true, false>(p, mb, lds_sq, st);
    } else {
      if (p.p_drop > 0.f) launch_bwd_dkdv_sq_t<false, true>(p, mb, lds_sq, st);
      else launch_bwd_dkdv_sq_t<false, false>(p, mb, lds_sq, st);
    }
    DLLM_CHECK_LAUNCH();
    return 0;
  }
  // v2: 64-row stages through an LDS-DMA ring (per-row terms from the dQ kernel).  Round 6 deleted the v1 kernel
  // (32-row register-staged stages), reachable only through an A/B switch since round 2.
  if (p.rowrec == nullptr) return -5;
  lds = (size_t)K2_NBUF * K2_STAGE + BWD_BK * 4;
  if (p.lut) lds += (size_t)(2 * (p.Sq + BWD_BK) + K2_QT) * 4;
  if (nblk <= 0 || nblk > 0x7fffffff || lds > 160 * 1024) return -4;
  DISPATCH4(launch_bwd_dkdv2_t, p.lut != nullptr, p.kpm != nullptr, p.causal != 0, p.p_drop > 0.f, p, (int)nblk,
            lds, st);
  DLLM_CHECK_LAUNCH();
  return 0;
}

// keep-bit planes only (same layout/decisions the forward would produce); p.dmask preallocated by the caller
extern "C" int dllm_attn_dropout_mask(AttnParams* pp, hipStream_t st) {
  AttnParams p = *pp;
  if (p.p_drop <= 0.f || p.dmask == nullptr) return -5;
  p.thr = drop_threshold(p.p_drop);
  p.n_ktiles = (p.Sk + FWD_BN - 1) / FWD_BN;
  p.sq_pad = (p.Sq + FWD_BM - 1) / FWD_BM * FWD_BM;
  const long nwords = (long)p.B * p.H * p.n_ktiles * 2 * p.sq_pad;
  const int blocks = (int)std::min<long>((nwords + 255) / 256, 65536);
  hipLaunchKernelGGL(attn_dropout_mask_kernel, dim3(blocks), dim3(256), 0, st, p, nwords);
  DLLM_CHECK_LAUNCH();
  return 0;
}

extern "C" int dllm_attn_params_size() { return (int)sizeof(AttnParams); }

// Flash attention forward + backward for encoder-decoder models on gfx950 (MI355X / CDNA4).
//
// Head dim D = 64 (T5 d_kv, BART 1024/16, flan-t5-xl 2048/32).  bf16 in/out, fp32 accumulate, MFMA
// v_mfma_f32_32x32x16_bf16 (wave64).  Supports: softmax scale (BART d^-0.5, T5 1.0), T5 relative
// position bias as a per-head LUT over (j - i) staged in LDS, key-padding mask, causal mask
// (bottom-right aligned: key j visible to query i iff j <= i + Sk - Sq), attention-probability
// dropout with the counter-based mask of common.h (regenerated in backward, never stored).
//
// Forward (one workgroup = 4 waves = 128 query rows of one (b, h); KV tiles of 64 keys):
//   "swapped" QK^T: each wave computes S^T = K Q^T so one lane owns one query column and holds 16 of
//   its 32 scores per 32-key subtile in registers -> row max / row sum are in-lane + one xor-32 shuffle.
//   The S^T accumulator is converted to bf16 and fed straight back as the B operand of O^T = V^T P^T
//   (no LDS round trip for P; cdna_hip_programming.md §3 "accumulator tile as the next MFMA's operand").
//   K is staged row-major in LDS with a 16-B row pad (conflict-free ds_read_b128), V transposed
//   (V^T, 8-B pad, conflict-free ds_read_b64).  Grid is 1-D with an XCD-aware bijective remap so the
//   q-tiles of one (b, h) land on one XCD and share K/V through its L2.
//
// Backward = two atomic-free kernels (recompute P from the forward's LSE in both):
//   dQ kernel (query blocks, query on the lane, like the forward): dS^T = P^T (dP^T - delta) stays in
//   registers and feeds dQ^T += K^T dS^T as the B operand; it also computes delta = rowsum(dO * O).
//   dK/dV kernel (key blocks of 128, key on the lane): S = Q K^T and dPd = dO V^T come out with the key
//   on the MFMA column, so P and dS are directly the B operands of dV^T += dO^T Pd and dK^T += Q^T dS
//   (K and V of the wave's 32 keys stay in registers).  The extra recompute (2 of 7 GEMMs) buys no
//   fp32 dQ atomics, no dS round trip through LDS and no cross-wave reduction.  The relative-bias
//   gradient is the sum of dS along diagonals: LDS float atomics into a window of the LUT, then one
//   global atomic per entry per workgroup.
#include "common.h"
#include "attn_params.h"

using namespace dllm;

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8v;

namespace {

constexpr int D = 64;
constexpr int FWD_BM = 128;  // 4 waves x 32 query rows
constexpr int FWD_BN = 64;   // keys per KV tile
constexpr int KS_STRIDE = 72;  // bf16 elements per K row in LDS (64 + 8 pad = 144 B)
constexpr int VT_STRIDE = 68;  // bf16 elements per V^T row (64 keys + 4 pad = 136 B)
constexpr float LOG2E = 1.4426950408889634f;

// AttnParams: csrc/attn_params.h (shared with the host binding)

DLLM_DEVICE bf16x8v as_frag(u16x8 v) { return __builtin_bit_cast(bf16x8v, v); }

DLLM_DEVICE bf16x8v pack8(const f32x16& a, int base) {
  u16x8 r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = f2bf(a[base + j]);
  return as_frag(r);
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

// ================================================================================== forward
template <bool HAS_BIAS, bool HAS_KPM, bool CAUSAL, bool DROP>
__global__ __launch_bounds__(256) void attn_fwd_kernel(AttnParams P) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  uint16_t* Ks = reinterpret_cast<uint16_t*>(smem);                 // [64][KS_STRIDE]
  uint16_t* Vt = Ks + FWD_BN * KS_STRIDE;                             // [64 d][VT_STRIDE]
  float* kmask = reinterpret_cast<float*>(Vt + D * VT_STRIDE);        // [64]
  float* lut_s = kmask + FWD_BN;                                      // [Sk + FWD_BM + FWD_BN]

  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63, r = lane & 31, hh = lane >> 5;
  const int logical = xcd_remap(blockIdx.x, gridDim.x);
  const int qt = logical % P.n_tiles;
  const int bh = logical / P.n_tiles;
  const int h = bh % P.H, b = bh / P.H;
  const int q0 = qt * FWD_BM;
  const int qrow = q0 + w * 32 + r;
  const bool qvalid = qrow < P.Sq;

  // LUT window: idx = key - q + Sq - 1, key in [0,Sk), q in [q0, q0+127]
  const int lut_base = P.Sq - 1 - (q0 + FWD_BM - 1);
  if (HAS_BIAS) {
    const int L = P.Sq + P.Sk - 1;
    const float* lrow = P.lut + (long)h * L;
    for (int i = tid; i < P.Sk + FWD_BM + FWD_BN; i += 256) {
      const int gi = lut_base + i;
      lut_s[i] = (gi >= 0 && gi < L) ? lrow[gi] : 0.f;
    }
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

  f32x16 o0 = {}, o1 = {};
  float m_run = -INFINITY, l_run = 0.f;
  int kend = P.Sk;
  if (CAUSAL) {
    const int lim = q0 + FWD_BM - 1 + P.causal_off + 1;
    kend = lim < kend ? lim : kend;
  }
  const int ntiles = kend > 0 ? (kend + FWD_BN - 1) / FWD_BN : 0;
  const float dscale = DROP ? 1.f / (1.f - P.p_drop) : 1.f;
  const long drop_row = ((long)(b * P.H + h) * P.Sq + qrow) * ((P.Sk + 1) & ~1);  // Sk rounded to even

  for (int kt = 0; kt < ntiles; ++kt) {
    const int kbase = kt * FWD_BN;
    __syncthreads();
    // ---- stage K (row-major) and V^T into LDS
#pragma unroll
    for (int pass = 0; pass < 2; ++pass) {
      const int key = (tid >> 3) + 32 * pass, ch = tid & 7;
      const int kk = kbase + key;
      u16x8 kv = {0, 0, 0, 0, 0, 0, 0, 0}, vv = {0, 0, 0, 0, 0, 0, 0, 0};
      if (kk < P.Sk) {
        kv = *reinterpret_cast<const u16x8*>(P.k + b * P.k_sb + (long)kk * P.k_ss + h * P.k_sh + ch * 8);
        vv = *reinterpret_cast<const u16x8*>(P.v + b * P.v_sb + (long)kk * P.v_ss + h * P.v_sh + ch * 8);
      }
      *reinterpret_cast<u16x8*>(Ks + key * KS_STRIDE + ch * 8) = kv;
#pragma unroll
      for (int e = 0; e < 8; ++e) Vt[(ch * 8 + e) * VT_STRIDE + key] = vv[e];
    }
    if (tid < FWD_BN) {
      const int kk = kbase + tid;
      bool ok = kk < P.Sk;
      if (HAS_KPM && ok) ok = P.kpm[(long)b * P.Sk + kk] != 0;
      kmask[tid] = ok ? 0.f : -INFINITY;
    }
    __syncthreads();

    // ---- S^T = K Q^T for two 32-key subtiles
    f32x16 s0 = {}, s1 = {};
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      bf16x8v a0 = as_frag(*reinterpret_cast<const u16x8*>(Ks + r * KS_STRIDE + 16 * s + 8 * hh));
      bf16x8v a1 = as_frag(*reinterpret_cast<const u16x8*>(Ks + (32 + r) * KS_STRIDE + 16 * s + 8 * hh));
      s0 = mfma32(a0, qf[s], s0);
      s1 = mfma32(a1, qf[s], s1);
    }
    // ---- scale, bias, masks; running max
    float mloc = -INFINITY;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int kl0 = crow(i, hh), kl1 = 32 + crow(i, hh);
      float v0 = s0[i] * P.scale + kmask[kl0];
      float v1 = s1[i] * P.scale + kmask[kl1];
      if (HAS_BIAS) {
        v0 += lut_s[kbase + kl0 - qrow + P.Sq - 1 - lut_base];
        v1 += lut_s[kbase + kl1 - qrow + P.Sq - 1 - lut_base];
      }
      if (CAUSAL) {
        if (kbase + kl0 > qrow + P.causal_off) v0 = -INFINITY;
        if (kbase + kl1 > qrow + P.causal_off) v1 = -INFINITY;
      }
      s0[i] = v0;
      s1[i] = v1;
      mloc = fmaxf(mloc, fmaxf(v0, v1));
    }
    mloc = fmaxf(mloc, __shfl_xor(mloc, 32, 64));
    const float m_new = fmaxf(m_run, mloc);
    const float m_use = m_new == -INFINITY ? 0.f : m_new;
    const float alpha = exp2f((m_run - m_use) * LOG2E);
    float lsum = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const float p0 = exp2f((s0[i] - m_use) * LOG2E);
      const float p1 = exp2f((s1[i] - m_use) * LOG2E);
      lsum += p0 + p1;
      s0[i] = p0;
      s1[i] = p1;
    }
    if (DROP) {
      // registers (i, i+1), i even, hold keys (2m, 2m+1): one hash per pair
#pragma unroll
      for (int i = 0; i < 16; i += 2) {
        const uint32_t e0 = (uint32_t)(drop_row + kbase + crow(i, hh));
        bool a0, a1, c0, c1;
        keep_two(P.seed, P.thr, e0, a0, a1);
        keep_two(P.seed, P.thr, e0 + 32u, c0, c1);
        s0[i] = a0 ? s0[i] * dscale : 0.f;
        s0[i + 1] = a1 ? s0[i + 1] * dscale : 0.f;
        s1[i] = c0 ? s1[i] * dscale : 0.f;
        s1[i + 1] = c1 ? s1[i + 1] * dscale : 0.f;
      }
    }
    l_run = l_run * alpha + lsum;
    m_run = m_new;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      o0[i] *= alpha;
      o1[i] *= alpha;
    }
    // ---- O^T += V^T P^T  (P^T accumulator registers reused as the B operand)
    const bf16x8v pa0 = pack8(s0, 0), pa1 = pack8(s0, 8), pb0 = pack8(s1, 0), pb1 = pack8(s1, 8);
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const uint16_t* vrow = Vt + (32 * t + r) * VT_STRIDE;
      f32x16 acc = t == 0 ? o0 : o1;
#pragma unroll
      for (int kb = 0; kb < 2; ++kb) {
#pragma unroll
        for (int sp = 0; sp < 2; ++sp) {
          const int kb0 = kb * 32 + 16 * sp + 4 * hh;
          u16x4 lo = *reinterpret_cast<const u16x4*>(vrow + kb0);
          u16x4 hi = *reinterpret_cast<const u16x4*>(vrow + kb0 + 8);
          u16x8 av = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
          const bf16x8v pf = kb == 0 ? (sp == 0 ? pa0 : pa1) : (sp == 0 ? pb0 : pb1);
          acc = mfma32(as_frag(av), pf, acc);
        }
      }
      if (t == 0) o0 = acc; else o1 = acc;
    }
  }

  // ---- epilogue
  const float l_tot = l_run + __shfl_xor(l_run, 32, 64);
  const float inv = l_tot > 0.f ? 1.f / l_tot : 0.f;
  if (qvalid) {
    uint16_t* op = P.o_out + b * P.o_sb + (long)qrow * P.o_ss + h * P.o_sh;
#pragma unroll
    for (int t = 0; t < 2; ++t) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const f32x16& acc = t == 0 ? o0 : o1;
        u16x4 pk = {f2bf(acc[4 * g] * inv), f2bf(acc[4 * g + 1] * inv), f2bf(acc[4 * g + 2] * inv),
                    f2bf(acc[4 * g + 3] * inv)};
        *reinterpret_cast<u16x4*>(op + 32 * t + 8 * g + 4 * hh) = pk;
      }
    }
    if (hh == 0) {
      const float m_use = m_run == -INFINITY ? 0.f : m_run;
      P.lse[(long)(b * P.H + h) * P.Sq + qrow] = l_tot > 0.f ? m_use + logf(l_tot) : INFINITY;
    }
  }
}

// ================================================================================== backward
constexpr int BWD_BK = 128;    // dK/dV kernel: keys per workgroup (4 waves x 32)
constexpr int BWD_BQ = 32;     // dK/dV kernel: query rows per tile
constexpr int QS_STRIDE = 72;  // [32 q][64 d] bf16 rows (144 B)
constexpr int QT_STRIDE = 36;  // [64 d][32 q] bf16 rows (72 B: 8-B reads conflict-free)

// ---- dQ kernel.  One workgroup = 128 query rows (4 waves x 32, query on the lane); loop over 64-key tiles.
// S^T = K Q^T and dP^T = V dO^T (swapped, like the forward), dS^T = P^T (dP^T - delta) in registers, and
// dQ^T += K^T dS^T takes the dS^T accumulators directly as B operands.  Also computes and stores
// delta = rowsum(dO * O) (one dot per lane pair) for the dK/dV kernel.  No atomics.
template <bool HAS_BIAS, bool HAS_KPM, bool CAUSAL, bool DROP>
__global__ __launch_bounds__(256, 2) void attn_bwd_dq_kernel(AttnParams P) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  uint16_t* Ks = reinterpret_cast<uint16_t*>(smem);             // [64][KS_STRIDE]
  uint16_t* Vs = Ks + FWD_BN * KS_STRIDE;                        // [64][KS_STRIDE]
  uint16_t* Kt = Vs + FWD_BN * KS_STRIDE;                        // [64 d][VT_STRIDE]
  float* kmask = reinterpret_cast<float*>(Kt + D * VT_STRIDE);   // [64]
  float* lut_s = kmask + FWD_BN;                                 // [Sk + FWD_BM + FWD_BN]

  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63, r = lane & 31, hh = lane >> 5;
  const int logical = xcd_remap(blockIdx.x, gridDim.x);
  const int qt = logical % P.n_tiles;
  const int bh = logical / P.n_tiles;
  const int h = bh % P.H, b = bh / P.H;
  const int q0 = qt * FWD_BM;
  const int qrow = q0 + w * 32 + r;
  const bool qvalid = qrow < P.Sq;
  const int lut_base = P.Sq - 1 - (q0 + FWD_BM - 1);
  if (HAS_BIAS) {
    const int L = P.Sq + P.Sk - 1;
    const float* lrow = P.lut + (long)h * L;
    for (int i = tid; i < P.Sk + FWD_BM + FWD_BN; i += 256) {
      const int gi = lut_base + i;
      lut_s[i] = (gi >= 0 && gi < L) ? lrow[gi] : 0.f;
    }
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
  const long row_off = (long)(b * P.H + h) * P.Sq + qrow;
  if (qvalid && hh == 0) P.delta[row_off] = delta;
  const float lse_q = qvalid ? P.lse[row_off] : INFINITY;

  f32x16 dq0 = {}, dq1 = {};
  int kend = P.Sk;
  if (CAUSAL) {
    const int lim = q0 + FWD_BM - 1 + P.causal_off + 1;
    kend = lim < kend ? lim : kend;
  }
  const int ntiles = kend > 0 ? (kend + FWD_BN - 1) / FWD_BN : 0;
  const float dscale = DROP ? 1.f / (1.f - P.p_drop) : 1.f;
  const long drop_row = row_off * ((P.Sk + 1) & ~1);

  for (int kt = 0; kt < ntiles; ++kt) {
    const int kbase = kt * FWD_BN;
    __syncthreads();
#pragma unroll
    for (int pass = 0; pass < 2; ++pass) {
      const int key = (tid >> 3) + 32 * pass, ch = tid & 7;
      const int kk = kbase + key;
      u16x8 kv = {0, 0, 0, 0, 0, 0, 0, 0}, vv = kv;
      if (kk < P.Sk) {
        kv = *reinterpret_cast<const u16x8*>(P.k + b * P.k_sb + (long)kk * P.k_ss + h * P.k_sh + ch * 8);
        vv = *reinterpret_cast<const u16x8*>(P.v + b * P.v_sb + (long)kk * P.v_ss + h * P.v_sh + ch * 8);
      }
      *reinterpret_cast<u16x8*>(Ks + key * KS_STRIDE + ch * 8) = kv;
      *reinterpret_cast<u16x8*>(Vs + key * KS_STRIDE + ch * 8) = vv;
#pragma unroll
      for (int e = 0; e < 8; ++e) Kt[(ch * 8 + e) * VT_STRIDE + key] = kv[e];
    }
    if (tid < FWD_BN) {
      const int kk = kbase + tid;
      bool ok = kk < P.Sk;
      if (HAS_KPM && ok) ok = P.kpm[(long)b * P.Sk + kk] != 0;
      kmask[tid] = ok ? 0.f : -INFINITY;
    }
    __syncthreads();

    f32x16 s0 = {}, s1 = {}, p0 = {}, p1 = {};
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      bf16x8v a0 = as_frag(*reinterpret_cast<const u16x8*>(Ks + r * KS_STRIDE + 16 * s + 8 * hh));
      bf16x8v a1 = as_frag(*reinterpret_cast<const u16x8*>(Ks + (32 + r) * KS_STRIDE + 16 * s + 8 * hh));
      bf16x8v v0 = as_frag(*reinterpret_cast<const u16x8*>(Vs + r * KS_STRIDE + 16 * s + 8 * hh));
      bf16x8v v1 = as_frag(*reinterpret_cast<const u16x8*>(Vs + (32 + r) * KS_STRIDE + 16 * s + 8 * hh));
      s0 = mfma32(a0, qf[s], s0);
      s1 = mfma32(a1, qf[s], s1);
      p0 = mfma32(v0, dof[s], p0);
      p1 = mfma32(v1, dof[s], p1);
    }
    // dS^T = P^T * (dP^T * keep - delta), P^T = exp(S^T * scale + bias - lse)
#pragma unroll
    for (int i = 0; i < 16; i += 2) {
      float kf0[2] = {1.f, 1.f}, kf1[2] = {1.f, 1.f};
      if (DROP) {
        const uint32_t e0 = (uint32_t)(drop_row + kbase + crow(i, hh));
        bool a0, a1, c0, c1;
        keep_two(P.seed, P.thr, e0, a0, a1);
        keep_two(P.seed, P.thr, e0 + 32u, c0, c1);
        kf0[0] = a0 ? dscale : 0.f;
        kf0[1] = a1 ? dscale : 0.f;
        kf1[0] = c0 ? dscale : 0.f;
        kf1[1] = c1 ? dscale : 0.f;
      }
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int ii = i + u;
        const int kl0 = crow(ii, hh), kl1 = 32 + kl0;
        float v0 = s0[ii] * P.scale + kmask[kl0];
        float v1 = s1[ii] * P.scale + kmask[kl1];
        if (HAS_BIAS) {
          v0 += lut_s[kbase + kl0 - qrow + P.Sq - 1 - lut_base];
          v1 += lut_s[kbase + kl1 - qrow + P.Sq - 1 - lut_base];
        }
        if (CAUSAL) {
          if (kbase + kl0 > qrow + P.causal_off) v0 = -INFINITY;
          if (kbase + kl1 > qrow + P.causal_off) v1 = -INFINITY;
        }
        const float pr0 = exp2f((v0 - lse_q) * LOG2E);
        const float pr1 = exp2f((v1 - lse_q) * LOG2E);
        s0[ii] = pr0 * (p0[ii] * kf0[u] - delta);
        s1[ii] = pr1 * (p1[ii] * kf1[u] - delta);
      }
    }
    // dQ^T += K^T dS^T
    const bf16x8v da0 = pack8(s0, 0), da1 = pack8(s0, 8), db0 = pack8(s1, 0), db1 = pack8(s1, 8);
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const uint16_t* krow = Kt + (32 * t + r) * VT_STRIDE;
      f32x16 acc = t == 0 ? dq0 : dq1;
#pragma unroll
      for (int kb = 0; kb < 2; ++kb) {
#pragma unroll
        for (int sp = 0; sp < 2; ++sp) {
          const int kb0 = kb * 32 + 16 * sp + 4 * hh;
          u16x4 lo = *reinterpret_cast<const u16x4*>(krow + kb0);
          u16x4 hi = *reinterpret_cast<const u16x4*>(krow + kb0 + 8);
          u16x8 av = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
          const bf16x8v bf = kb == 0 ? (sp == 0 ? da0 : da1) : (sp == 0 ? db0 : db1);
          acc = mfma32(as_frag(av), bf, acc);
        }
      }
      if (t == 0) dq0 = acc; else dq1 = acc;
    }
  }
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
}

// ---- dK/dV kernel.  One workgroup = 128 keys (4 waves x 32, key on the lane); loop over 32-row query tiles.
// S = Q K^T and dPd = dO V^T come out with the key on the MFMA column, so P and dS are directly the B
// operands of dV^T += dO^T Pd and dK^T += Q^T dS (K and V of the wave's keys stay in registers).  The
// relative-bias gradient (sum of dS along diagonals) goes through LDS float atomics, then one global
// atomic per LUT entry per workgroup.  Needs delta from the dQ kernel.
template <bool HAS_BIAS, bool HAS_KPM, bool CAUSAL, bool DROP>
__global__ __launch_bounds__(256, 2) void attn_bwd_dkdv_kernel(AttnParams P) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  uint16_t* Qs = reinterpret_cast<uint16_t*>(smem);        // [32][72]
  uint16_t* dOs = Qs + BWD_BQ * QS_STRIDE;                   // [32][72]
  uint16_t* Qt = dOs + BWD_BQ * QS_STRIDE;                   // [64][36]
  uint16_t* dOt = Qt + D * QT_STRIDE;                        // [64][36]
  float* lse_s = reinterpret_cast<float*>(dOt + D * QT_STRIDE);  // [32]
  float* del_s = lse_s + BWD_BQ;                             // [32]
  float* kmask = del_s + BWD_BQ;                             // [128]
  float* lut_s = kmask + BWD_BK;                             // [Sq + 128]
  float* dlut_s = lut_s + (HAS_BIAS ? P.Sq + BWD_BK : 0);    // [Sq + 128]

  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63, r = lane & 31, hh = lane >> 5;
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

  if (HAS_BIAS) {
    const float* lrow = P.lut + (long)h * L;
    for (int i = tid; i < win; i += 256) {
      const int gi = k0 + i;
      lut_s[i] = gi < L ? lrow[gi] : 0.f;
      dlut_s[i] = 0.f;
    }
  }
  if (tid < BWD_BK) {
    const int kk = k0 + tid;
    bool ok = kk < P.Sk;
    if (HAS_KPM && ok) ok = P.kpm[(long)b * P.Sk + kk] != 0;
    kmask[tid] = ok ? 0.f : -INFINITY;
  }
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

  f32x16 dv0 = {}, dv1 = {}, dk0 = {}, dk1 = {};
  const float dscale = DROP ? 1.f / (1.f - P.p_drop) : 1.f;
  int qt_begin = 0;
  if (CAUSAL) {
    const int qmin = k0 - P.causal_off;  // first query that can see key k0
    qt_begin = qmin > 0 ? qmin / BWD_BQ : 0;
  }
  const int nqt = (P.Sq + BWD_BQ - 1) / BWD_BQ;
  const long bh_rows = (long)(b * P.H + h) * P.Sq;
  const float* lse_row = P.lse + bh_rows;
  const float* del_row = P.delta + bh_rows;
  const long sk2 = (P.Sk + 1) & ~1;

  for (int qt = qt_begin; qt < nqt; ++qt) {
    const int q0 = qt * BWD_BQ;
    __syncthreads();
    {
      const int qq = tid >> 3, ch = tid & 7;
      const int qg = q0 + qq;
      u16x8 a = {0, 0, 0, 0, 0, 0, 0, 0}, c = a;
      if (qg < P.Sq) {
        a = *reinterpret_cast<const u16x8*>(P.q + b * P.q_sb + (long)qg * P.q_ss + h * P.q_sh + ch * 8);
        c = *reinterpret_cast<const u16x8*>(P.dout + b * P.do_sb + (long)qg * P.do_ss + h * P.do_sh + ch * 8);
      }
      *reinterpret_cast<u16x8*>(Qs + qq * QS_STRIDE + ch * 8) = a;
      *reinterpret_cast<u16x8*>(dOs + qq * QS_STRIDE + ch * 8) = c;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        Qt[(ch * 8 + e) * QT_STRIDE + qq] = a[e];
        dOt[(ch * 8 + e) * QT_STRIDE + qq] = c[e];
      }
      if (tid < BWD_BQ) {
        const int qg2 = q0 + tid;
        lse_s[tid] = qg2 < P.Sq ? lse_row[qg2] : INFINITY;
        del_s[tid] = qg2 < P.Sq ? del_row[qg2] : 0.f;
      }
    }
    __syncthreads();

    f32x16 sacc = {}, dpacc = {};
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      bf16x8v qa = as_frag(*reinterpret_cast<const u16x8*>(Qs + r * QS_STRIDE + 16 * s + 8 * hh));
      bf16x8v da = as_frag(*reinterpret_cast<const u16x8*>(dOs + r * QS_STRIDE + 16 * s + 8 * hh));
      sacc = mfma32(qa, kf[s], sacc);
      dpacc = mfma32(da, vf[s], dpacc);
    }
    f32x16 pd, ds;
    const float km = kmask[w * 32 + r];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int ql = crow(i, hh);
      const int qg = q0 + ql;
      float sv = sacc[i] * P.scale + km;
      if (HAS_BIAS) {
        int li = key - qg + P.Sq - 1 - k0;
        li = li < 0 ? 0 : li;
        sv += lut_s[li];
      }
      if (CAUSAL && key > qg + P.causal_off) sv = -INFINITY;
      const float pr = exp2f((sv - lse_s[ql]) * LOG2E);  // lse = +inf for q >= Sq -> 0
      float keepf = 1.f;
      if (DROP) keepf = keep_one(P.seed, P.thr, (uint32_t)((bh_rows + qg) * sk2 + key)) ? dscale : 0.f;
      pd[i] = pr * keepf;
      ds[i] = pr * (dpacc[i] * keepf - del_s[ql]);
    }
    if (HAS_BIAS) {
      // Diagonal sums of this wave's 32x32 dS tile without per-element atomics: rotate register i
      // (tile row rho = crow(i, hh)) left by rho lanes so lane r receives element (rho, (r + rho) & 31),
      // whose diagonal (col - row) is r (no wrap) or r - 32 (wrapped).  Masked / out-of-range
      // elements are exactly 0 (P = 0), so no guards are needed.
      float pos = 0.f, neg = 0.f;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int rho = crow(i, hh);
        const float v = __shfl(ds[i], ((r + rho) & 31) + 32 * hh, 64);
        if (r + rho < 32) pos += v; else neg += v;
      }
      pos += __shfl_xor(pos, 32, 64);
      neg += __shfl_xor(neg, 32, 64);
      if (hh == 0) {
        const int li = w * 32 + r - q0 + P.Sq - 1;  // LUT index (window-local) of diagonal r
        atomicAdd(&dlut_s[li], pos);
        if (li >= 32) atomicAdd(&dlut_s[li - 32], neg);
      }
    }
    const bf16x8v pf0 = pack8(pd, 0), pf1 = pack8(pd, 8), sf0 = pack8(ds, 0), sf1 = pack8(ds, 8);
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const uint16_t* drow = dOt + (32 * t + r) * QT_STRIDE;
      const uint16_t* qrw = Qt + (32 * t + r) * QT_STRIDE;
      f32x16 av = t == 0 ? dv0 : dv1;
      f32x16 ak = t == 0 ? dk0 : dk1;
#pragma unroll
      for (int sp = 0; sp < 2; ++sp) {
        const int c0 = 16 * sp + 4 * hh;
        u16x4 lo = *reinterpret_cast<const u16x4*>(drow + c0);
        u16x4 hi = *reinterpret_cast<const u16x4*>(drow + c0 + 8);
        u16x8 a8 = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
        av = mfma32(as_frag(a8), sp == 0 ? pf0 : pf1, av);
        u16x4 lo2 = *reinterpret_cast<const u16x4*>(qrw + c0);
        u16x4 hi2 = *reinterpret_cast<const u16x4*>(qrw + c0 + 8);
        u16x8 b8 = {lo2.x, lo2.y, lo2.z, lo2.w, hi2.x, hi2.y, hi2.z, hi2.w};
        ak = mfma32(as_frag(b8), sp == 0 ? sf0 : sf1, ak);
      }
      if (t == 0) { dv0 = av; dk0 = ak; } else { dv1 = av; dk1 = ak; }
    }
  }

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
  if (HAS_BIAS) {
    __syncthreads();
    float* grow = P.dlut + (long)h * L;
    for (int i = tid; i < win; i += 256) {
      const int gi = k0 + i;
      const float v = dlut_s[i];
      if (gi < L && v != 0.f) atomicAdd(grow + gi, v);
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
  hipLaunchKernelGGL((attn_fwd_kernel<HB, HK, CA, DR>), dim3(nblk), dim3(256), lds, st, p);
}
template <bool HB, bool HK, bool CA, bool DR>
void launch_bwd_dq_t(const AttnParams& p, int nblk, size_t lds, hipStream_t st) {
  hipLaunchKernelGGL((attn_bwd_dq_kernel<HB, HK, CA, DR>), dim3(nblk), dim3(256), lds, st, p);
}
template <bool HB, bool HK, bool CA, bool DR>
void launch_bwd_dkdv_t(const AttnParams& p, int nblk, size_t lds, hipStream_t st) {
  hipLaunchKernelGGL((attn_bwd_dkdv_kernel<HB, HK, CA, DR>), dim3(nblk), dim3(256), lds, st, p);
}

}  // namespace

extern "C" int dllm_attn_fwd(AttnParams* pp, hipStream_t st) {
  AttnParams p = *pp;
  p.thr = drop_threshold(p.p_drop);
  p.n_tiles = (p.Sq + FWD_BM - 1) / FWD_BM;
  const long nblk = (long)p.n_tiles * p.H * p.B;
  if (nblk <= 0 || nblk > 0x7fffffff) return -3;
  size_t lds = (size_t)FWD_BN * KS_STRIDE * 2 + (size_t)D * VT_STRIDE * 2 + FWD_BN * 4;
  if (p.lut) lds += (size_t)(p.Sk + FWD_BM + FWD_BN) * 4;
  if (lds > 160 * 1024) return -4;
  DISPATCH4(launch_fwd_t, p.lut != nullptr, p.kpm != nullptr, p.causal != 0, p.p_drop > 0.f, p, (int)nblk, lds, st);
  DLLM_CHECK_LAUNCH();
  return 0;
}

extern "C" int dllm_attn_bwd(AttnParams* pp, hipStream_t st) {
  AttnParams p = *pp;
  p.thr = drop_threshold(p.p_drop);
  // 1) dQ (+ delta): query blocks, same geometry as the forward
  p.n_tiles = (p.Sq + FWD_BM - 1) / FWD_BM;
  long nblk = (long)p.n_tiles * p.H * p.B;
  size_t lds = (size_t)2 * FWD_BN * KS_STRIDE * 2 + (size_t)D * VT_STRIDE * 2 + FWD_BN * 4;
  if (p.lut) lds += (size_t)(p.Sk + FWD_BM + FWD_BN) * 4;
  if (nblk <= 0 || nblk > 0x7fffffff || lds > 160 * 1024) return -4;
  DISPATCH4(launch_bwd_dq_t, p.lut != nullptr, p.kpm != nullptr, p.causal != 0, p.p_drop > 0.f, p, (int)nblk, lds,
            st);
  DLLM_CHECK_LAUNCH();
  // 2) dK, dV (+ bias-LUT gradient): key blocks
  p.n_tiles = (p.Sk + BWD_BK - 1) / BWD_BK;
  nblk = (long)p.n_tiles * p.H * p.B;
  lds = (size_t)2 * BWD_BQ * QS_STRIDE * 2 + (size_t)2 * D * QT_STRIDE * 2 + 2 * BWD_BQ * 4 + BWD_BK * 4;
  if (p.lut) lds += (size_t)2 * (p.Sq + BWD_BK) * 4;
  if (nblk <= 0 || nblk > 0x7fffffff || lds > 160 * 1024) return -4;
  DISPATCH4(launch_bwd_dkdv_t, p.lut != nullptr, p.kpm != nullptr, p.causal != 0, p.p_drop > 0.f, p, (int)nblk, lds,
            st);
  DLLM_CHECK_LAUNCH();
  return 0;
}

extern "C" int dllm_attn_params_size() { return (int)sizeof(AttnParams); }

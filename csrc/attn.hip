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
// Backward (one workgroup = 4 waves = 128 keys; loop over 32-row query tiles):
//   "key on the lane": S = Q K^T and dPd = dO V^T come out with the key on the MFMA column, so the
//   P / dS accumulators are directly the B operands of dV^T += dO^T Pd and dK^T += Q^T dS (K and V of
//   the wave's 32 keys stay in registers).  dS crosses LDS once (per wave) for dQ = dS K; the four
//   waves' dQ partials are summed in LDS and added to an fp32 dQ buffer with 256-B-contiguous atomics.
//   The relative-bias gradient is the sum of dS along diagonals: LDS float atomics into a window of
//   the LUT, then one global atomic per entry per workgroup.
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
  const long drop_row = ((long)(b * P.H + h) * P.Sq + qrow) * P.Sk;

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
      float p0 = exp2f((s0[i] - m_use) * LOG2E);
      float p1 = exp2f((s1[i] - m_use) * LOG2E);
      lsum += p0 + p1;
      if (DROP) {
        const int kl0 = crow(i, hh), kl1 = 32 + crow(i, hh);
        p0 = (mix32(P.seed, (uint32_t)(drop_row + kbase + kl0)) >= P.thr) ? p0 * dscale : 0.f;
        p1 = (mix32(P.seed, (uint32_t)(drop_row + kbase + kl1)) >= P.thr) ? p1 * dscale : 0.f;
      }
      s0[i] = p0;
      s1[i] = p1;
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
// delta[b,h,q] = sum_d dO * O
__global__ __launch_bounds__(256) void attn_bwd_delta_kernel(AttnParams P) {
  const int wid = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  const long nrows = (long)P.B * P.H * P.Sq;
  if (wid >= nrows) return;
  const int q = wid % P.Sq;
  const int bh = wid / P.Sq;
  const int h = bh % P.H, b = bh / P.H;
  const float a = bf2f(P.dout[b * P.do_sb + (long)q * P.do_ss + h * P.do_sh + lane]);
  const float c = bf2f(P.o[b * P.o_sb + (long)q * P.o_ss + h * P.o_sh + lane]);
  const float s = wave_sum(a * c);
  if (lane == 0) const_cast<float*>(P.delta)[wid] = s;
}

constexpr int BWD_BK = 128;  // keys per workgroup (4 waves x 32)
constexpr int BWD_BQ = 32;   // query rows per tile
constexpr int QS_STRIDE = 72;  // [32 q][64 d] rows, bf16
constexpr int QT_STRIDE = 36;  // [64 d][32 q] rows, bf16 (72 B)
constexpr int KT_STRIDE = 40;  // [64 d][32 keys] rows per wave, bf16 (80 B)
constexpr int DS_STRIDE = 40;  // [32 q][32 keys] rows per wave, bf16

template <bool HAS_BIAS, bool HAS_KPM, bool CAUSAL, bool DROP>
__global__ __launch_bounds__(256) void attn_bwd_kernel(AttnParams P) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  uint16_t* Qs = reinterpret_cast<uint16_t*>(smem);        // [32][72]
  uint16_t* dOs = Qs + BWD_BQ * QS_STRIDE;                   // [32][72]
  uint16_t* Qt = dOs + BWD_BQ * QS_STRIDE;                   // [64][36]
  uint16_t* dOt = Qt + D * QT_STRIDE;                        // [64][36]
  uint16_t* Kt = dOt + D * QT_STRIDE;                        // [4 waves][64][40]
  uint16_t* dSs = Kt + 4 * D * KT_STRIDE;                    // [4 waves][32][40]
  float* dQs = reinterpret_cast<float*>(dSs + 4 * BWD_BQ * DS_STRIDE);  // [4][32][64]
  float* lse_s = dQs + 4 * BWD_BQ * D;                       // [32]
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
  const int key = kw0 + r;  // this lane's key column
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
  // K, V fragments of this wave's 32 keys (B operands of S = Q K^T and dPd = dO V^T), K^T image for dQ
  bf16x8v kf[4], vf[4];
  {
    const uint16_t* kp = P.k + b * P.k_sb + (long)key * P.k_ss + h * P.k_sh;
    const uint16_t* vp = P.v + b * P.v_sb + (long)key * P.v_ss + h * P.v_sh;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      u16x8 a = {0, 0, 0, 0, 0, 0, 0, 0}, c = {0, 0, 0, 0, 0, 0, 0, 0};
      if (kvalid) {
        a = *reinterpret_cast<const u16x8*>(kp + 16 * s + 8 * hh);
        c = *reinterpret_cast<const u16x8*>(vp + 16 * s + 8 * hh);
      }
      kf[s] = as_frag(a);
      vf[s] = as_frag(c);
      uint16_t* ktw = Kt + w * D * KT_STRIDE;
#pragma unroll
      for (int e = 0; e < 8; ++e) ktw[(16 * s + 8 * hh + e) * KT_STRIDE + r] = a[e];
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
  const float* lse_row = P.lse + (long)(b * P.H + h) * P.Sq;
  const float* del_row = P.delta + (long)(b * P.H + h) * P.Sq;
  const long drop_base = (long)(b * P.H + h) * P.Sq;

  for (int qt = qt_begin; qt < nqt; ++qt) {
    const int q0 = qt * BWD_BQ;
    __syncthreads();
    // ---- stage Q, dO (row-major and transposed), lse, delta
    {
      const int qq = tid >> 3, ch = tid & 7;  // 32 rows x 8 chunks
      const int qg = q0 + qq;
      u16x8 a = {0, 0, 0, 0, 0, 0, 0, 0}, c = {0, 0, 0, 0, 0, 0, 0, 0};
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

    // ---- S = Q K^T, dPd = dO V^T   (C layout: row q = crow(i,hh), column key = r)
    f32x16 sacc = {}, dpacc = {};
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      bf16x8v qa = as_frag(*reinterpret_cast<const u16x8*>(Qs + r * QS_STRIDE + 16 * s + 8 * hh));
      bf16x8v da = as_frag(*reinterpret_cast<const u16x8*>(dOs + r * QS_STRIDE + 16 * s + 8 * hh));
      sacc = mfma32(qa, kf[s], sacc);
      dpacc = mfma32(da, vf[s], dpacc);
    }
    // ---- P, Pd, dS
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
      if (DROP) keepf = (mix32(P.seed, (uint32_t)((drop_base + qg) * P.Sk + key)) >= P.thr) ? dscale : 0.f;
      pd[i] = pr * keepf;
      const float dp = dpacc[i] * keepf;
      ds[i] = pr * (dp - del_s[ql]);
    }
    if (HAS_BIAS) {
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int qg = q0 + crow(i, hh);
        if (qg < P.Sq && kvalid) atomicAdd(&dlut_s[key - qg + P.Sq - 1 - k0], ds[i]);
      }
    }
    // ---- dV^T += dO^T Pd ; dK^T += Q^T dS   (A from transposed LDS images, B = accumulators)
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
    // ---- dQ partial = dS K  (dS through this wave's LDS tile, K^T image as B)
    uint16_t* dsw = dSs + w * BWD_BQ * DS_STRIDE;
#pragma unroll
    for (int i = 0; i < 16; ++i) dsw[crow(i, hh) * DS_STRIDE + r] = f2bf(ds[i]);
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): this wave's LDS writes visible to its reads
    __builtin_amdgcn_wave_barrier();
    f32x16 q0acc = {}, q1acc = {};
    const uint16_t* ktw = Kt + w * D * KT_STRIDE;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      bf16x8v a = as_frag(*reinterpret_cast<const u16x8*>(dsw + r * DS_STRIDE + 16 * s + 8 * hh));
      bf16x8v b0 = as_frag(*reinterpret_cast<const u16x8*>(ktw + r * KT_STRIDE + 16 * s + 8 * hh));
      bf16x8v b1 = as_frag(*reinterpret_cast<const u16x8*>(ktw + (32 + r) * KT_STRIDE + 16 * s + 8 * hh));
      q0acc = mfma32(a, b0, q0acc);
      q1acc = mfma32(a, b1, q1acc);
    }
    // dQ partial C layout: row q = crow(i,hh), column d = 32t + r
    float* dqw = dQs + w * BWD_BQ * D;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      dqw[crow(i, hh) * D + r] = q0acc[i];
      dqw[crow(i, hh) * D + 32 + r] = q1acc[i];
    }
    __syncthreads();
    // sum the 4 wave partials; fp32 atomics, 256 contiguous bytes per wave-instruction
#pragma unroll
    for (int it = 0; it < (BWD_BQ * D) / 256; ++it) {
      const int e = it * 256 + tid;
      const int ql = e >> 6, dd = e & 63;
      const int qg = q0 + ql;
      const float v = dQs[e] + dQs[BWD_BQ * D + e] + dQs[2 * BWD_BQ * D + e] + dQs[3 * BWD_BQ * D + e];
      if (qg < P.Sq) atomicAdd(P.dq_acc + (((long)b * P.Sq + qg) * P.H + h) * D + dd, v);
    }
  }

  // ---- store dK (scaled), dV:  C layout row d = 32t + crow(i,hh), column key = r
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

// dq (bf16, strided [B,Sq,H,D]) = scale * dq_acc (fp32 contiguous [B,Sq,H,D])
__global__ __launch_bounds__(256) void attn_dq_convert_kernel(const float* __restrict__ acc, uint16_t* __restrict__ dq,
                                                              long n4, int Sq, int H, long sb, long ss, long sh,
                                                              float scale) {
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n4; i += (long)gridDim.x * 256) {
    const int dc = (int)(i % (D / 4));
    long t = i / (D / 4);
    const int h = (int)(t % H);
    t /= H;
    const int q = (int)(t % Sq);
    const long b = t / Sq;
    f32x4 v = *reinterpret_cast<const f32x4*>(acc + i * 4) * scale;
    u16x4 o = {f2bf(v.x), f2bf(v.y), f2bf(v.z), f2bf(v.w)};
    *reinterpret_cast<u16x4*>(dq + b * sb + (long)q * ss + h * sh + dc * 4) = o;
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
void launch_bwd_t(const AttnParams& p, int nblk, size_t lds, hipStream_t st) {
  hipLaunchKernelGGL((attn_bwd_kernel<HB, HK, CA, DR>), dim3(nblk), dim3(256), lds, st, p);
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
  // delta
  const long rows = (long)p.B * p.H * p.Sq;
  hipLaunchKernelGGL(attn_bwd_delta_kernel, dim3((rows + 3) / 4), dim3(256), 0, st, p);
  p.n_tiles = (p.Sk + BWD_BK - 1) / BWD_BK;
  const long nblk = (long)p.n_tiles * p.H * p.B;
  size_t lds = (size_t)2 * BWD_BQ * QS_STRIDE * 2 + (size_t)2 * D * QT_STRIDE * 2 + (size_t)4 * D * KT_STRIDE * 2 +
               (size_t)4 * BWD_BQ * DS_STRIDE * 2 + (size_t)4 * BWD_BQ * D * 4 + 2 * BWD_BQ * 4 + BWD_BK * 4;
  if (p.lut) lds += (size_t)2 * (p.Sq + BWD_BK) * 4;
  if (lds > 160 * 1024) return -4;
  DISPATCH4(launch_bwd_t, p.lut != nullptr, p.kpm != nullptr, p.causal != 0, p.p_drop > 0.f, p, (int)nblk, lds, st);
  DLLM_CHECK_LAUNCH();
  return 0;
}

extern "C" int dllm_attn_dq_convert(const float* acc, void* dq, int B, int Sq, int H, long sb, long ss, long sh,
                                    float scale, hipStream_t st) {
  const long n4 = (long)B * Sq * H * (D / 4);
  long g = (n4 + 255) / 256;
  if (g > 8192) g = 8192;
  if (g < 1) g = 1;
  hipLaunchKernelGGL(attn_dq_convert_kernel, dim3((int)g), dim3(256), 0, st, acc, (uint16_t*)dq, n4, Sq, H, sb, ss,
                     sh, scale);
  DLLM_CHECK_LAUNCH();
  return 0;
}

extern "C" int dllm_attn_params_size() { return (int)sizeof(AttnParams); }

// fp32 flash attention (forward + backward) on the gfx950 f32-input matrix cores (v_mfma_f32_16x16x4_f32: exact
// f32 products, one rounding per product, fp32 accumulation — the reference's own precision, ref/train-torchrun.py
// 115-128 trains in fp32).  Same feature set and semantics as the bf16 kernels of csrc/attn.hip / ops/attention.py:
// T5 relative-position bias LUT [H, Sq + Sk - 1] (+ its gradient), key-padding mask, causal mask, softmax scale and
// attention-probability dropout with the exact keep decisions of ops/rng.py attention_keep_mask.  O(S) memory:
// probabilities are never materialised (the fp32 composite it replaces stored [B, H, Sq, Sk] scores + masks).
//
// Layout trick (no transposes through LDS for P or dS): the 16x16x4 f32 MFMA's C/D map puts rows 4g .. 4g+3
// (g = lane >> 4) of column (lane & 15) in a lane's 4 registers, and its A/B maps take reduction index k = g from
// lane group g.  Computing S^T = K Q^T (keys on the MFMA's M side) leaves each lane with keys 16t + 4g + i of ONE query
// row; feeding register i as the k-step-i operand of the next product reduces over keys {16t + 4g + i : g} — any key
// order is a valid reduction order as long as the other operand is read in the same order (its LDS image is laid out
// for that read: one ds_read_b128 per 4 k-steps).
//
//   forward    grid (Sq/64, B*H), 4 waves x 16 query rows; per 64-key block: K (row-major) and V (transposed) staged in
//              LDS, S^T = K Q^T (64 MFMAs / wave), online softmax + dropout in registers, O^T += V^T P^T (64 MFMAs).
//   dQ         grid (Sq/64, B*H): S^T, dP^T = V dO^T, dS = P (dP_kept - delta), dQ^T += K^T dS^T; the bias gradient is
//              summed per diagonal of the block's dS tile in LDS and added to dlut once per block (fp32 atomics).
//   dK / dV    grid (Sk/64, B*H), 4 waves x 16 keys: S = Q K^T, dP = dO V^T, dV += P_kept^T dO, dK += dS^T Q.
#include "common.h"

#include "attn_f32_params.h"

using namespace dllm;

DLLM_SEED_STEP_TU(attn_f32)

namespace {

constexpr int D = 64, BQ = 64, BKY = 64, NT = 256;
constexpr uint32_t C24 = 0x9E3779u, C24B = 0x85EBCBu, HG = 0x9E3779B1u;  // ops/rng.py attention_keep_mask

DLLM_DEVICE f32x4 mma(float a, float b, f32x4 c) { return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0); }

// keep decision of key j of the row whose hash is rh (ops/rng.py attention_keep_mask, bit-exact)
DLLM_DEVICE bool keep_key(uint32_t rh, int j, uint32_t thr) {
  const uint32_t g = __umul24(rh, C24) + (uint32_t)(j >> 1) * HG;
  const uint32_t hh = __umul24(g ^ (g >> 15), C24B);
  const uint32_t y = hh ^ (hh >> 16);
  const uint32_t half = (j & 1) ? (y >> 16) : (y & 0xFFFFu);
  return (half ^ 0x8000u) >= thr;
}
// keep bits of keys j0 .. j0 + 3 (j0 % 4 == 0): bit i <-> key j0 + i; two hashes (one per key pair)
DLLM_DEVICE uint32_t keep4(uint32_t rh, int j0, uint32_t thr) {
  const uint32_t g0 = __umul24(rh, C24) + (uint32_t)(j0 >> 1) * HG;
  uint32_t bits = 0;
#pragma unroll
  for (int pp = 0; pp < 2; ++pp) {
    const uint32_t g = g0 + (uint32_t)pp * HG;
    const uint32_t hh = __umul24(g ^ (g >> 15), C24B);
    const uint32_t y = hh ^ (hh >> 16);
    bits |= (((y & 0xFFFFu) ^ 0x8000u) >= thr ? 1u : 0u) << (2 * pp);
    bits |= (((y >> 16) ^ 0x8000u) >= thr ? 1u : 0u) << (2 * pp + 1);
  }
  return bits;
}

// [64][64] fp32 image, row-major, 16-B chunks XOR-swizzled by (row & 15)
DLLM_DEVICE int rm_off(int r, int c4) { return r * 64 + ((c4 ^ (r & 15)) << 2); }
// [64 cols][64 rows] transposed image of a row-major tile X[r][col]: element (col, r) at col * 64 + chunk(r>>2) ^ (col&15)
DLLM_DEVICE int tr_off(int col, int r) { return col * 64 + ((((r >> 2) ^ (col & 15))) << 2) + (r & 3); }

// stage rows [r0, r0 + 64) of a [*, S, H, 64] view into LDS: row-major image `rm` and/or transposed image `tr`
// (rows >= S read as 0).  256 threads, 4 x 16-B chunks each.
template <bool RM, bool TR>
DLLM_DEVICE void stage(const float* base, long ss, int r0, int S, float* rm, float* tr, int tid) {
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int idx = tid + NT * j, r = idx >> 4, c4 = idx & 15;
    f32x4 v = {0.f, 0.f, 0.f, 0.f};
    if (r0 + r < S) v = *reinterpret_cast<const f32x4*>(base + (long)(r0 + r) * ss + 4 * c4);
    if constexpr (RM) *reinterpret_cast<f32x4*>(rm + rm_off(r, c4)) = v;
    if constexpr (TR) {
      tr[tr_off(4 * c4 + 0, r)] = v.x;
      tr[tr_off(4 * c4 + 1, r)] = v.y;
      tr[tr_off(4 * c4 + 2, r)] = v.z;
      tr[tr_off(4 * c4 + 3, r)] = v.w;
    }
  }
}

// 16 floats of row r, columns 16 g .. 16 g + 15, from a row-major image
DLLM_DEVICE void rd_row16(const float* rm, int r, int g, float (&out)[16]) {
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const f32x4 v = *reinterpret_cast<const f32x4*>(rm + rm_off(r, 4 * g + j));
    out[4 * j] = v.x;
    out[4 * j + 1] = v.y;
    out[4 * j + 2] = v.z;
    out[4 * j + 3] = v.w;
  }
}
// 4 consecutive rows r4 .. r4 + 3 (r4 % 4 == 0) of column col, from a transposed image
DLLM_DEVICE f32x4 rd_col4(const float* tr, int col, int r4) {
  return *reinterpret_cast<const f32x4*>(tr + col * 64 + ((((r4 >> 2) ^ (col & 15))) << 2));
}

DLLM_DEVICE float grp_max(float v) {  // over the 4 lane groups (same lane & 15)
  v = fmaxf(v, __shfl_xor(v, 16, 64));
  return fmaxf(v, __shfl_xor(v, 32, 64));
}
DLLM_DEVICE float grp_sum(float v) {
  v += __shfl_xor(v, 16, 64);
  return v + __shfl_xor(v, 32, 64);
}

// key in range and not padding (the causal test is per (row, key), done by the callers)
DLLM_DEVICE bool key_ok(const AttnF32Params& P, int b, int key) {
  return key < P.Sk && (P.kpm == nullptr || P.kpm[(long)b * P.Sk + key] != 0);
}

// ================================================================================================ forward
template <bool DROP>
__global__ __launch_bounds__(NT) void attn_f32_fwd_kernel(AttnF32Params P) {
  __shared__ __attribute__((aligned(16))) float Ks[BKY * D];
  __shared__ __attribute__((aligned(16))) float Vt[D * BKY];
  __shared__ float Ls[2 * BKY];
  __shared__ uint8_t Mk[BKY];  // 1: key valid (in range, not padding)
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g = lane >> 4, c = lane & 15;
  const int bh = blockIdx.y, b = bh / P.H, h = bh % P.H;
  const int q0 = blockIdx.x * BQ;
  const int row = q0 + 16 * w + c;
  const int rowc = min(row, P.Sq - 1);
  const long L = (long)P.Sq + P.Sk - 1;
  float qf[16];
  {
    const float* qp = P.q + (long)b * P.q_sb + (long)rowc * P.q_ss + (long)h * P.q_sh + 16 * g;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const f32x4 v = *reinterpret_cast<const f32x4*>(qp + 4 * j);
      qf[4 * j] = v.x;
      qf[4 * j + 1] = v.y;
      qf[4 * j + 2] = v.z;
      qf[4 * j + 3] = v.w;
    }
  }
  const uint32_t rh = DROP ? mix32(eff_seed(P.seed), (uint32_t)((long)bh * P.Sq + rowc)) : 0u;
  const float dscale = DROP ? 1.f / (1.f - P.p_drop) : 1.f;
  float m = -INFINITY, l = 0.f;
  f32x4 acc[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  const float* kb = P.k + (long)b * P.k_sb + (long)h * P.k_sh;
  const float* vb = P.v + (long)b * P.v_sb + (long)h * P.v_sh;
  int kend = P.Sk;
  if (P.causal) kend = min(P.Sk, max(0, q0 + BQ + P.causal_off));
  for (int k0 = 0; k0 < kend; k0 += BKY) {
    __syncthreads();  // the previous block's LDS reads are done
    stage<true, false>(kb, P.k_ss, k0, P.Sk, Ks, nullptr, tid);
    stage<false, true>(vb, P.v_ss, k0, P.Sk, nullptr, Vt, tid);
    if (P.lut && tid < 2 * BKY - 1) {  // bias of (key, row) at Ls[key - row - (k0 - q0 - 63)]
      long idx = (long)k0 - q0 - 63 + tid + P.Sq - 1;
      idx = idx < 0 ? 0 : (idx >= L ? L - 1 : idx);
      Ls[tid] = P.lut[(long)h * L + idx];
    }
    if (tid < BKY) Mk[tid] = key_ok(P, b, k0 + tid);
    __syncthreads();
    f32x4 st[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      float kf[16];
      rd_row16(Ks, 16 * t + c, g, kf);
      st[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < 16; ++s) st[t] = mma(kf[s], qf[s], st[t]);
    }
    // st[t][i] = S[row][key = k0 + 16 t + 4 g + i]
    float mx = -INFINITY;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int key = k0 + 16 * t + 4 * g + i;
        float x = st[t][i] * P.scale;
        if (P.lut) x += Ls[key - row - (k0 - q0 - 63)];
        if (!Mk[16 * t + 4 * g + i] || (P.causal && key > row + P.causal_off)) x = -INFINITY;
        st[t][i] = x;
        mx = fmaxf(mx, x);
      }
    }
    mx = grp_max(mx);
    const float mn = fmaxf(m, mx);
    const float mu = mn == -INFINITY ? 0.f : mn;
    const float alpha = __expf(m - mu);
    float ls = 0.f;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const uint32_t kb4 = DROP ? keep4(rh, k0 + 16 * t + 4 * g, P.thr) : 0xFu;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float pr = __expf(st[t][i] - mu);
        ls += pr;
        st[t][i] = DROP ? (((kb4 >> i) & 1u) ? pr * dscale : 0.f) : pr;
      }
    }
    ls = grp_sum(ls);
    l = l * alpha + ls;
    m = mn;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) acc[dt] *= alpha;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        const f32x4 va = rd_col4(Vt, 16 * dt + c, 16 * t + 4 * g);
        acc[dt] = mma(va.x, st[t][0], acc[dt]);
        acc[dt] = mma(va.y, st[t][1], acc[dt]);
        acc[dt] = mma(va.z, st[t][2], acc[dt]);
        acc[dt] = mma(va.w, st[t][3], acc[dt]);
      }
    }
  }
  if (row < P.Sq) {
    const float inv = l > 0.f ? 1.f / l : 0.f;
    float* op = P.o_out + (long)b * P.o_sb + (long)row * P.o_ss + (long)h * P.o_sh;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) *reinterpret_cast<f32x4*>(op + 16 * dt + 4 * g) = acc[dt] * inv;
    if (g == 0) P.lse[(long)bh * P.Sq + row] = l > 0.f ? m + __logf(l) : INFINITY;
  }
}

// ================================================================================================ backward
// delta[bh][row] = sum_d dO * O; one 16-lane group per row
__global__ __launch_bounds__(NT) void attn_f32_delta_kernel(AttnF32Params P) {
  const long rows = (long)P.B * P.H * P.Sq;
  const long r = (long)blockIdx.x * (NT / 16) + (threadIdx.x >> 4);
  const int j = threadIdx.x & 15;
  float s = 0.f;
  if (r < rows) {
    const int row = (int)(r % P.Sq);
    const long bh = r / P.Sq;
    const int b = (int)(bh / P.H), h = (int)(bh % P.H);
    const f32x4 o = *reinterpret_cast<const f32x4*>(P.o + (long)b * P.o_sb + (long)row * P.o_ss + (long)h * P.o_sh + 4 * j);
    const f32x4 d = *reinterpret_cast<const f32x4*>(P.dout + (long)b * P.do_sb + (long)row * P.do_ss +
                                                    (long)h * P.do_sh + 4 * j);
    s = o.x * d.x + o.y * d.y + o.z * d.z + o.w * d.w;
  }
#pragma unroll
  for (int mm = 8; mm >= 1; mm >>= 1) s += __shfl_xor(s, mm, 16);
  if (r < rows && j == 0) P.delta[r] = s;
}

template <bool DROP>
__global__ __launch_bounds__(NT) void attn_f32_dq_kernel(AttnF32Params P) {
  __shared__ __attribute__((aligned(16))) float Ks[BKY * D];
  __shared__ __attribute__((aligned(16))) float Kt[D * BKY];
  __shared__ __attribute__((aligned(16))) float Vs[BKY * D];
  __shared__ float Ls[2 * BKY];
  __shared__ float Ds[BQ * (BKY + 1)];  // dS tile of the block, row stride 65: a diagonal walk is bank-conflict free
  __shared__ uint8_t Mk[BKY];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g = lane >> 4, c = lane & 15;
  const int bh = blockIdx.y, b = bh / P.H, h = bh % P.H;
  const int q0 = blockIdx.x * BQ;
  const int row = q0 + 16 * w + c;
  const int rowc = min(row, P.Sq - 1);
  const bool row_ok = row < P.Sq;
  const long L = (long)P.Sq + P.Sk - 1;
  float qf[16], dof[16];
  {
    const float* qp = P.q + (long)b * P.q_sb + (long)rowc * P.q_ss + (long)h * P.q_sh + 16 * g;
    const float* dp = P.dout + (long)b * P.do_sb + (long)rowc * P.do_ss + (long)h * P.do_sh + 16 * g;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const f32x4 v = *reinterpret_cast<const f32x4*>(qp + 4 * j);
      const f32x4 d = *reinterpret_cast<const f32x4*>(dp + 4 * j);
      qf[4 * j] = v.x; qf[4 * j + 1] = v.y; qf[4 * j + 2] = v.z; qf[4 * j + 3] = v.w;
      dof[4 * j] = d.x; dof[4 * j + 1] = d.y; dof[4 * j + 2] = d.z; dof[4 * j + 3] = d.w;
    }
  }
  const float lse = row_ok ? P.lse[(long)bh * P.Sq + row] : INFINITY;
  const float dlt = row_ok ? P.delta[(long)bh * P.Sq + row] : 0.f;
  const uint32_t rh = DROP ? mix32(eff_seed(P.seed), (uint32_t)((long)bh * P.Sq + rowc)) : 0u;
  const float dscale = DROP ? 1.f / (1.f - P.p_drop) : 1.f;
  const bool want_dlut = P.dlut != nullptr && P.lut != nullptr;
  f32x4 acc[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  const float* kb = P.k + (long)b * P.k_sb + (long)h * P.k_sh;
  const float* vb = P.v + (long)b * P.v_sb + (long)h * P.v_sh;
  int kend = P.Sk;
  if (P.causal) kend = min(P.Sk, max(0, q0 + BQ + P.causal_off));
  for (int k0 = 0; k0 < kend; k0 += BKY) {
    __syncthreads();
    stage<true, true>(kb, P.k_ss, k0, P.Sk, Ks, Kt, tid);
    stage<true, false>(vb, P.v_ss, k0, P.Sk, Vs, nullptr, tid);
    if (P.lut && tid < 2 * BKY - 1) {
      long idx = (long)k0 - q0 - 63 + tid + P.Sq - 1;
      idx = idx < 0 ? 0 : (idx >= L ? L - 1 : idx);
      Ls[tid] = P.lut[(long)h * L + idx];
    }
    if (tid < BKY) Mk[tid] = key_ok(P, b, k0 + tid);
    __syncthreads();
    f32x4 st[4], dpt[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      float kf[16], vf[16];
      rd_row16(Ks, 16 * t + c, g, kf);
      rd_row16(Vs, 16 * t + c, g, vf);
      st[t] = f32x4{0.f, 0.f, 0.f, 0.f};
      dpt[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < 16; ++s) {
        st[t] = mma(kf[s], qf[s], st[t]);
        dpt[t] = mma(vf[s], dof[s], dpt[t]);
      }
    }
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const uint32_t kb4 = DROP ? keep4(rh, k0 + 16 * t + 4 * g, P.thr) : 0xFu;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int key = k0 + 16 * t + 4 * g + i;
        const int di = key - row - (k0 - q0 - 63);
        float x = st[t][i] * P.scale;
        if (P.lut) x += Ls[di];
        const bool msk = !Mk[16 * t + 4 * g + i] || (P.causal && key > row + P.causal_off);
        const float pr = msk ? 0.f : __expf(x - lse);
        const float dpk = DROP ? (((kb4 >> i) & 1u) ? dpt[t][i] * dscale : 0.f) : dpt[t][i];
        const float ds = pr * (dpk - dlt);
        st[t][i] = ds;
        if (want_dlut) Ds[(16 * w + c) * (BKY + 1) + 16 * t + 4 * g + i] = ds;  // 0 for rows >= Sq (lse = inf)
      }
    }
#pragma unroll
    for (int t = 0; t < 4; ++t) {
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        const f32x4 ka = rd_col4(Kt, 16 * dt + c, 16 * t + 4 * g);
        acc[dt] = mma(ka.x, st[t][0], acc[dt]);
        acc[dt] = mma(ka.y, st[t][1], acc[dt]);
        acc[dt] = mma(ka.z, st[t][2], acc[dt]);
        acc[dt] = mma(ka.w, st[t][3], acc[dt]);
      }
    }
    if (want_dlut) {
      // bias gradient: per diagonal d = key - row + 63 of the 64x64 block, one thread walks its diagonal in the dS
      // tile (LDS reads, no atomics) and adds the sum to dlut once
      __syncthreads();
      if (tid < 2 * BKY - 1) {
        const int d = tid;
        const int r0 = d < 63 ? 63 - d : 0, r1 = d < 63 ? 63 : 126 - d;
        float v = 0.f;
        for (int r = r0; r <= r1; ++r) v += Ds[r * (BKY + 1) + r + d - 63];
        const long idx = (long)k0 - q0 - 63 + d + P.Sq - 1;
        if (v != 0.f && idx >= 0 && idx < L) atomicAdd(&P.dlut[(long)h * L + idx], v);
      }
    }
  }
  if (row_ok) {
    float* dqp = P.dq + (long)b * P.dq_sb + (long)row * P.dq_ss + (long)h * P.dq_sh;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) *reinterpret_cast<f32x4*>(dqp + 16 * dt + 4 * g) = acc[dt] * P.scale;
  }
}

template <bool DROP>
__global__ __launch_bounds__(NT) void attn_f32_dkdv_kernel(AttnF32Params P) {
  __shared__ __attribute__((aligned(16))) float Qs[BQ * D];
  __shared__ __attribute__((aligned(16))) float Qt[D * BQ];
  __shared__ __attribute__((aligned(16))) float Os[BQ * D];  // dO, row-major
  __shared__ __attribute__((aligned(16))) float Ot[D * BQ];  // dO, transposed
  __shared__ float Ls[2 * BQ];
  __shared__ float Rl[BQ], Rd[BQ];
  __shared__ uint32_t Rh[BQ];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g = lane >> 4, c = lane & 15;
  const int bh = blockIdx.y, b = bh / P.H, h = bh % P.H;
  const int k0 = blockIdx.x * BKY;
  const int key = k0 + 16 * w + c;
  const int keyc = min(key, P.Sk - 1);
  const long L = (long)P.Sq + P.Sk - 1;
  float kf[16], vf[16];
  {
    const float* kp = P.k + (long)b * P.k_sb + (long)keyc * P.k_ss + (long)h * P.k_sh + 16 * g;
    const float* vp = P.v + (long)b * P.v_sb + (long)keyc * P.v_ss + (long)h * P.v_sh + 16 * g;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const f32x4 a = *reinterpret_cast<const f32x4*>(kp + 4 * j);
      const f32x4 v = *reinterpret_cast<const f32x4*>(vp + 4 * j);
      kf[4 * j] = a.x; kf[4 * j + 1] = a.y; kf[4 * j + 2] = a.z; kf[4 * j + 3] = a.w;
      vf[4 * j] = v.x; vf[4 * j + 1] = v.y; vf[4 * j + 2] = v.z; vf[4 * j + 3] = v.w;
    }
  }
  const float dscale = DROP ? 1.f / (1.f - P.p_drop) : 1.f;
  const uint32_t seed = DROP ? eff_seed(P.seed) : 0u;
  const bool kok = key_ok(P, b, key);
  f32x4 dk[4], dv[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    dk[i] = f32x4{0.f, 0.f, 0.f, 0.f};
    dv[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  const float* qb = P.q + (long)b * P.q_sb + (long)h * P.q_sh;
  const float* ob = P.dout + (long)b * P.do_sb + (long)h * P.do_sh;
  int qstart = 0;
  if (P.causal) qstart = max(0, (k0 - P.causal_off) / BQ * BQ);
  for (int q0 = qstart; q0 < P.Sq; q0 += BQ) {
    __syncthreads();
    stage<true, true>(qb, P.q_ss, q0, P.Sq, Qs, Qt, tid);
    stage<true, true>(ob, P.do_ss, q0, P.Sq, Os, Ot, tid);
    if (P.lut && tid < 2 * BQ - 1) {  // bias of (key, row) at Ls[key - row - (k0 - q0 - 63)]
      long idx = (long)k0 - q0 - 63 + tid + P.Sq - 1;
      idx = idx < 0 ? 0 : (idx >= L ? L - 1 : idx);
      Ls[tid] = P.lut[(long)h * L + idx];
    }
    if (tid < BQ) {
      const int r = q0 + tid;
      const bool ok = r < P.Sq;
      Rl[tid] = ok ? P.lse[(long)bh * P.Sq + r] : INFINITY;
      Rd[tid] = ok ? P.delta[(long)bh * P.Sq + r] : 0.f;
      if (DROP) Rh[tid] = mix32(seed, (uint32_t)((long)bh * P.Sq + min(r, P.Sq - 1)));
    }
    __syncthreads();
    f32x4 sc[4], dp[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      float qf[16], of[16];
      rd_row16(Qs, 16 * t + c, g, qf);
      rd_row16(Os, 16 * t + c, g, of);
      sc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
      dp[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < 16; ++s) {
        sc[t] = mma(qf[s], kf[s], sc[t]);
        dp[t] = mma(of[s], vf[s], dp[t]);
      }
    }
    // sc[t][i] = S[row = q0 + 16 t + 4 g + i][key]; pd = kept P, sc <- dS
    f32x4 pd[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int rl = 16 * t + 4 * g + i, row = q0 + rl;
        float x = sc[t][i] * P.scale;
        if (P.lut) x += Ls[key - row - (k0 - q0 - 63)];
        const bool msk = !kok || (P.causal && key > row + P.causal_off);
        const float pr = msk ? 0.f : __expf(x - Rl[rl]);
        const bool kp = DROP ? keep_key(Rh[rl], key, P.thr) : true;
        const float dpk = kp ? dp[t][i] * dscale : 0.f;
        pd[t][i] = kp ? pr * dscale : 0.f;
        sc[t][i] = pr * (dpk - Rd[rl]);
      }
    }
#pragma unroll
    for (int t = 0; t < 4; ++t) {
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        const f32x4 oa = rd_col4(Ot, 16 * dt + c, 16 * t + 4 * g);
        const f32x4 qa = rd_col4(Qt, 16 * dt + c, 16 * t + 4 * g);
        dv[dt] = mma(pd[t][0], oa.x, dv[dt]);
        dv[dt] = mma(pd[t][1], oa.y, dv[dt]);
        dv[dt] = mma(pd[t][2], oa.z, dv[dt]);
        dv[dt] = mma(pd[t][3], oa.w, dv[dt]);
        dk[dt] = mma(sc[t][0], qa.x, dk[dt]);
        dk[dt] = mma(sc[t][1], qa.y, dk[dt]);
        dk[dt] = mma(sc[t][2], qa.z, dk[dt]);
        dk[dt] = mma(sc[t][3], qa.w, dk[dt]);
      }
    }
  }
  // dk[dt][i] = dK[key = k0 + 16 w + 4 g + i][d = 16 dt + c]
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int kr = k0 + 16 * w + 4 * g + i;
    if (kr >= P.Sk) continue;
    float* dkp = P.dk + (long)b * P.dk_sb + (long)kr * P.dk_ss + (long)h * P.dk_sh;
    float* dvp = P.dv + (long)b * P.dv_sb + (long)kr * P.dv_ss + (long)h * P.dv_sh;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      dkp[16 * dt + c] = dk[dt][i] * P.scale;
      dvp[16 * dt + c] = dv[dt][i];
    }
  }
}

}  // namespace

extern "C" int dllm_attn_f32_fwd(AttnF32Params* pp, hipStream_t st) {
  const AttnF32Params& P = *pp;
  dim3 grid((P.Sq + BQ - 1) / BQ, P.B * P.H);
  if (P.p_drop > 0.f) hipLaunchKernelGGL(attn_f32_fwd_kernel<true>, grid, dim3(NT), 0, st, P);
  else hipLaunchKernelGGL(attn_f32_fwd_kernel<false>, grid, dim3(NT), 0, st, P);
  DLLM_CHECK_LAUNCH();
  return 0;
}

extern "C" int dllm_attn_f32_bwd(AttnF32Params* pp, hipStream_t st) {
  const AttnF32Params& P = *pp;
  const long rows = (long)P.B * P.H * P.Sq;
  hipLaunchKernelGGL(attn_f32_delta_kernel, dim3((unsigned)((rows + NT / 16 - 1) / (NT / 16))), dim3(NT), 0, st, P);
  DLLM_CHECK_LAUNCH();
  dim3 gq((P.Sq + BQ - 1) / BQ, P.B * P.H), gk((P.Sk + BKY - 1) / BKY, P.B * P.H);
  if (P.p_drop > 0.f) {
    hipLaunchKernelGGL(attn_f32_dq_kernel<true>, gq, dim3(NT), 0, st, P);
    hipLaunchKernelGGL(attn_f32_dkdv_kernel<true>, gk, dim3(NT), 0, st, P);
  } else {
    hipLaunchKernelGGL(attn_f32_dq_kernel<false>, gq, dim3(NT), 0, st, P);
    hipLaunchKernelGGL(attn_f32_dkdv_kernel<false>, gk, dim3(NT), 0, st, P);
  }
  DLLM_CHECK_LAUNCH();
  return 0;
}

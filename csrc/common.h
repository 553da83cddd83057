// Shared device helpers for the gfx950 (MI355X / CDNA4) kernel library.
// Wave64 everywhere: lane = threadIdx.x & 63, reductions over 64 lanes.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define DLLM_HOST_DEVICE __host__ __device__ __forceinline__
#define DLLM_DEVICE __device__ __forceinline__

typedef uint16_t bf16_raw;
typedef __attribute__((ext_vector_type(2))) float f32x2;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(8))) short bf16x8;   // MFMA A/B fragment (8 x bf16)
typedef __attribute__((ext_vector_type(4))) short bf16x4;
typedef __attribute__((ext_vector_type(4))) uint16_t u16x4;
typedef __attribute__((ext_vector_type(8))) uint16_t u16x8;
typedef __attribute__((ext_vector_type(4))) uint32_t u32x4;

namespace dllm {

constexpr int kWave = 64;

DLLM_DEVICE float bf2f(uint16_t v) { return __uint_as_float(((uint32_t)v) << 16); }

// Round-to-nearest-even f32 -> bf16.  A plain cast to __bf16 lowers to v_cvt_pk_bf16_f32 on gfx950
// (keeps NaN a NaN: MI355X_MICROARCH.md "Correctness boundaries").
DLLM_DEVICE uint16_t f2bf(float f) {
  __bf16 b = (__bf16)f;
  return __builtin_bit_cast(uint16_t, b);
}

// one v_cvt_pk_bf16_f32 (RNE, as f2bf); the scalar form costs 2 converts + shift + or
typedef __attribute__((ext_vector_type(2))) __bf16 dllm_bf16x2;
DLLM_DEVICE uint32_t pack_bf16x2(float lo, float hi) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(f32x2{lo, hi}, dllm_bf16x2));
}

// ---- generic element access for bf16 (uint16 storage) / fp32 --------------------------------
template <typename T> struct Elem;
template <> struct Elem<float> {
  static DLLM_DEVICE float load(const float* p) { return *p; }
  static DLLM_DEVICE void store(float* p, float v) { *p = v; }
  static DLLM_DEVICE f32x4 load4(const float* p) { return *reinterpret_cast<const f32x4*>(p); }
  static DLLM_DEVICE void store4(float* p, f32x4 v) { *reinterpret_cast<f32x4*>(p) = v; }
  static DLLM_DEVICE float round(float v) { return v; }
};
template <> struct Elem<uint16_t> {
  static DLLM_DEVICE float load(const uint16_t* p) { return bf2f(*p); }
  static DLLM_DEVICE void store(uint16_t* p, float v) { *p = f2bf(v); }
  static DLLM_DEVICE f32x4 load4(const uint16_t* p) {
    u16x4 r = *reinterpret_cast<const u16x4*>(p);
    return f32x4{bf2f(r.x), bf2f(r.y), bf2f(r.z), bf2f(r.w)};
  }
  static DLLM_DEVICE void store4(uint16_t* p, f32x4 v) {
    const uint32_t lo = pack_bf16x2(v.x, v.y), hi = pack_bf16x2(v.z, v.w);
    *reinterpret_cast<uint2*>(p) = make_uint2(lo, hi);
  }
  static DLLM_DEVICE float round(float v) { return bf2f(f2bf(v)); }
};

// ---- counter-based dropout hash (mirrors ops/rng.py mix32) ------------------------------------
DLLM_HOST_DEVICE uint32_t mix32(uint32_t seed, uint32_t idx) {
  uint32_t x = (idx * 0x9E3779B1u) ^ seed;
  x ^= x >> 16;
  x *= 0x85EBCA6Bu;
  x ^= x >> 13;
  x *= 0xC2B2AE35u;
  x ^= x >> 16;
  return x;
}

// 16-bit threshold: element e is kept iff half (e & 1) of mix32(seed, e >> 1) >= thr16.
inline uint32_t drop_threshold(float p) {
  double t = (double)p * 65536.0;
  return t >= 65535.0 ? 0xFFFFu : (uint32_t)t;
}

DLLM_DEVICE bool keep_one(uint32_t seed, uint32_t thr16, uint32_t e) {
  const uint32_t h = mix32(seed, e >> 1);
  return ((e & 1u) ? (h >> 16) : (h & 0xFFFFu)) >= thr16;
}

// e_even must be even: decisions for elements e_even and e_even + 1 from one hash
DLLM_DEVICE void keep_two(uint32_t seed, uint32_t thr16, uint32_t e_even, bool& k0, bool& k1) {
  const uint32_t h = mix32(seed, e_even >> 1);
  k0 = (h & 0xFFFFu) >= thr16;
  k1 = (h >> 16) >= thr16;
}

// v[k] (elements e4 .. e4+3, e4 even) -> dropped or scaled
DLLM_DEVICE void dropout4(f32x4& v, uint32_t seed, uint32_t thr16, uint32_t e4, float scale) {
  bool k0, k1, k2, k3;
  keep_two(seed, thr16, e4, k0, k1);
  keep_two(seed, thr16, e4 + 2u, k2, k3);
  v.x = k0 ? v.x * scale : 0.f;
  v.y = k1 ? v.y * scale : 0.f;
  v.z = k2 ? v.z * scale : 0.f;
  v.w = k3 ? v.w * scale : 0.f;
}

// ---- row-Weyl dropout hash (attention probabilities and the FFN activations; ops/rng.py rowwise_keep_mask) ---------
// For tensors whose kernels walk rows: rh = mix32(seed, row) once per row; per column pair kp = col >> 1,
// g = (rh & 0xFFFFFF) * C24 + kp * G (mod 2^32: a Weyl sequence along the row, one add per pair), h = ((g ^ (g >> 15)) &
// 0xFFFFFF) * C24B (full-rate v_mul_u32_u24), y = h ^ (h >> 16); the even column keeps iff ((y & 0xFFFF) ^ 0x8000) >=
// thr16, the odd one iff ((y >> 16) ^ 0x8000) >= thr16.  ~7 VALU per pair, against mix32's three quarter-rate
// v_mul_lo_u32 per pair; statistics: tests/test_training_cpu.py test_attention_dropout_hash_statistics.
constexpr uint32_t RW_C24 = 0x9E3779u, RW_C24B = 0x85EBCBu, RW_G = 0x9E3779B1u;
DLLM_DEVICE uint32_t rw_pair_y(uint32_t g) {
  const uint32_t h = __umul24(g ^ (g >> 15), RW_C24B);
  return h ^ (h >> 16);
}
// g of column pair kp0 of the row with hash rh (pair kp0 + j: + j * RW_G)
DLLM_DEVICE uint32_t rw_gbase(uint32_t rh, uint32_t kp0) { return __umul24(rh, RW_C24) + kp0 * RW_G; }
// (thr16 - 0x8000) in both 16-bit halves: the threshold operand of rw_drop2
DLLM_HOST_DEVICE uint32_t rw_t2(uint32_t thr16) { return ((thr16 - 0x8000u) & 0xFFFFu) * 0x10001u; }
// DROP mask of a pair: 0xFFFF in the half of each dropped column (low half = even column): saturating signed difference,
// then its sign spread over the half
DLLM_DEVICE uint32_t rw_drop2(uint32_t y, uint32_t t2) {
  uint32_t d, m;
  asm("v_pk_sub_i16 %0, %1, %2 clamp" : "=v"(d) : "v"(y), "s"(t2));  // t2: wave-uniform (kernel arguments)
  asm("v_pk_ashrrev_i16 %0, %1, %2" : "=v"(m) : "s"(0x000F000Fu), "v"(d));  // per-half count (an inline 15 would
                                                                            // shift the high half by 0)
  return m;
}
// per-element factors (scale if kept, else 0) of the 4 columns of the two pairs starting at Weyl value g
DLLM_DEVICE f32x4 rw_scale4(uint32_t g, uint32_t t2, float scale) {
  const uint32_t m0 = rw_drop2(rw_pair_y(g), t2), m1 = rw_drop2(rw_pair_y(g + RW_G), t2);
  return f32x4{(m0 & 0xFFFFu) ? 0.f : scale, (m0 >> 16) ? 0.f : scale, (m1 & 0xFFFFu) ? 0.f : scale,
               (m1 >> 16) ? 0.f : scale};
}
// fp32 form for 4 consecutive columns col .. col+3 (col even) of the row with hash rh: kept ones scaled, dropped zeroed
DLLM_DEVICE void rw_dropout4(f32x4& v, uint32_t rh, uint32_t t2, uint32_t col, float scale) {
  const uint32_t g = rw_gbase(rh, col >> 1);
  const uint32_t m0 = rw_drop2(rw_pair_y(g), t2), m1 = rw_drop2(rw_pair_y(g + RW_G), t2);
  v.x = (m0 & 0xFFFFu) ? 0.f : v.x * scale;
  v.y = (m0 >> 16) ? 0.f : v.y * scale;
  v.z = (m1 & 0xFFFFu) ? 0.f : v.z * scale;
  v.w = (m1 >> 16) ? 0.f : v.w * scale;
}

// ---- graph-replayable dropout seeds ----------------------------------------------------------------------------
// A captured HIP graph replays its kernel arguments verbatim, so a per-site seed passed by value would draw the SAME
// mask every replayed step.  Every translation unit with dropout therefore keeps a device pointer to ONE 32-bit step
// counter (set once by dllm_set_seed_step_<tu>, bumped on the device by a captured add each step): kernels use
// mix32(site_seed, *step) when it is set, the site seed itself when not (eager mode: identical masks to before).
#define DLLM_SEED_STEP_TU(TU)                                                                           \
  namespace {                                                                                           \
  __device__ const uint32_t* g_seed_step = nullptr;                                                     \
  DLLM_DEVICE uint32_t eff_seed(uint32_t seed) {                                                        \
    const uint32_t* p = g_seed_step;                                                                    \
    return p ? dllm::mix32(seed, *p) : seed;                                                            \
  }                                                                                                     \
  }                                                                                                     \
  extern "C" int dllm_set_seed_step_##TU(const uint32_t* p) {                                           \
    return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_seed_step), &p, sizeof(p));                              \
  }

// ---- wave64 reductions -------------------------------------------------------------------------
DLLM_DEVICE float wave_sum(float v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m, 64);
  return v;
}
DLLM_DEVICE float wave_max(float v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v = fmaxf(v, __shfl_xor(v, m, 64));
  return v;
}

// Block-wide sum for blockDim.x == NT (multiple of 64). `red` must hold NT/64 floats.
template <int NT>
DLLM_DEVICE float block_sum(float v, float* red) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  v = wave_sum(v);
  __syncthreads();
  if (lane == 0) red[w] = v;
  __syncthreads();
  float r = 0.f;
#pragma unroll
  for (int i = 0; i < NT / 64; ++i) r += red[i];
  return r;
}
template <int NT>
DLLM_DEVICE float block_max(float v, float* red) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  v = wave_max(v);
  __syncthreads();
  if (lane == 0) red[w] = v;
  __syncthreads();
  float r = -INFINITY;
#pragma unroll
  for (int i = 0; i < NT / 64; ++i) r = fmaxf(r, red[i]);
  return r;
}

// ---- LDS-DMA (global_load_lds_dwordx4) ---------------------------------------------------------
// LDS-DMA of 16 B per lane: lane i's bytes land at LDS byte address `lds_byte` + 16 i (wave-uniform base in
// M0).  Inline asm, not the builtin: hipcc treats the builtin as an LDS store and waits vmcnt(0) before the
// next ds_read of ANY buffer, which would drain the ring every stage; the asm load is invisible to its
// bookkeeping and is retired by the explicit counted waits in the k-loop (cdna_hip_programming.md §6).
DLLM_DEVICE void glds16(const uint16_t* g, uint32_t lds_byte) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(g), "s"(lds_byte)
               : "memory");
}

// 4 B per lane variant (lane i -> lds_byte + 4 i)
DLLM_DEVICE void glds4(const void* g, uint32_t lds_byte) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(g), "s"(lds_byte)
               : "memory");
}

// LDS-DMA through a buffer descriptor: 16 B per lane from base + voff (bytes) to LDS lds_byte + 16 * lane.  base is
// wave-uniform (the descriptor lives in SGPRs, so the address math is scalar and only the 32-bit voff is per lane);
// num_records = 2^32 - 1, so voff only has to stay below 4 GB; soffset 0.  Inline asm for the same reason as glds16:
// the llvm.amdgcn.raw.buffer.load.lds intrinsic makes hipcc wait vmcnt(0) before the next transposed LDS read.
typedef __attribute__((ext_vector_type(4))) int i32x4;
DLLM_DEVICE void bld16(const void* base, uint32_t voff, uint32_t lds_byte) {
  const uint64_t a = (uint64_t)base;
  i32x4 r;
  r.x = (int)(uint32_t)a;
  r.y = (int)((uint32_t)(a >> 32) & 0xFFFFu);
  r.z = -1;
  r.w = 0x00020000;
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds\n\t"
               "s_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(voff), "s"(r), "s"(lds_byte)
               : "memory");
}

DLLM_DEVICE uint32_t lds_addr(const void* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}

template <int N_>
DLLM_DEVICE void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N_) : "memory");
}

}  // namespace dllm

#define DLLM_CHECK_LAUNCH() \
  do { hipError_t e__ = hipGetLastError(); if (e__ != hipSuccess) return (int)e__; } while (0)

// What an LDS-DMA costs a one-wave-per-SIMD MFMA stream on gfx950 (the projection GEMM's k-loop shape,
// csrc/gemm_w4.hip: 128 MFMA 16x16x32 + 16 buffer_load_dwordx4 ... lds + 32 ds_read_b128 per 64-deep k-tile and wave).
//
// One 256-thread workgroup per CU (LDS request forces it), 4 waves, accumulators pinned to AGPRs, random operands.
// Each loop iteration is 256 MFMA cycles: 16 x 16x16x32 or 8 x 32x32x16, plus D DMAs (1 KiB per wave each) placed
// evenly ("spread") or back to back after the first MFMA ("burst"), plus R ds_read_b128 whose results feed the next
// iteration's MFMAs.  DMA source: "hot" = a 64 KiB window per workgroup (L2 / L1 resident), "cold" = a 1 GiB stream.
// Output: ns per iteration (median over interleaved rounds) and the MFMA-busy fraction against the no-DMA body.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/mfma_dma_probe.hip -o build/mfma_dma_probe
//   build/mfma_dma_probe [iters] [rounds]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8v;
typedef __attribute__((ext_vector_type(4))) int i32x4;
typedef __attribute__((ext_vector_type(4))) uint32_t u32x4;

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));      \
      exit(1);                                                                       \
    }                                                                                \
  } while (0)

__device__ __forceinline__ void mf16(f32x4& c, const bf16x8v& a, const bf16x8v& b) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(c) : "v"(a), "v"(b));
}
__device__ __forceinline__ void mf32(f32x16& c, const bf16x8v& a, const bf16x8v& b) {
  asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+a"(c) : "v"(a), "v"(b));
}

// the w4 DMA statement: M0 formed by the statement, buffer descriptor in SGPRs, wave-uniform soffset
template <uint32_t IMM>
__device__ __forceinline__ void dma_buf(const i32x4& srd, uint32_t voff, uint32_t soff, uint32_t ldsb) {
  asm volatile("s_add_u32 m0, %3, %4\n\ts_nop 0\n\tbuffer_load_dwordx4 %0, %1, %2 offen lds"
               :
               : "v"(voff), "s"(srd), "s"(soff), "s"(ldsb), "i"(IMM)
               : "memory", "m0", "scc");
}
template <uint32_t IMM>
__device__ __forceinline__ void dma_glb(const void* p, uint32_t ldsb) {
  asm volatile("s_add_u32 m0, %1, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off"
               :
               : "v"(p), "s"(ldsb), "i"(IMM)
               : "memory", "m0", "scc");
}

template <int N_>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N_) : "memory");
}

// MF: 16 or 32; DM: 0 none, 1 buffer lds, 2 global lds; D: DMAs per iteration; BURST; HOT: 0 cold (HBM), 1 hot
// (64 KiB per workgroup, L2), 2 MALL (512 KiB per workgroup, 128 MiB in all); R: ds_reads per iteration;
// BAR: s_barrier every BAR iterations (0 = none)
template <int MF, int DM, int D, bool BURST, int HOT, int R, int BAR, int NW = 4>
__global__ __launch_bounds__(NW * 64, 1) void probe(const uint16_t* src, long wg_bytes, float* out, int iters,
                                                     unsigned long long* clk) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  // MFMAs per wave and iteration: 256 cycles of matrix pipe per SIMD, shared by NW / 4 waves per SIMD
  constexpr int NM = (MF == 16 ? 16 : 8) * 4 / NW;
  constexpr int DW = D * 4 / NW;  // DMAs per wave and iteration (the same per-SIMD density)
  const unsigned char* base = (const unsigned char*)src + (long)blockIdx.x * wg_bytes;
  const uint64_t a64 = (uint64_t)base;
  i32x4 srd;
  srd.x = __builtin_amdgcn_readfirstlane((int)(uint32_t)a64);
  srd.y = __builtin_amdgcn_readfirstlane((int)((uint32_t)(a64 >> 32) & 0xFFFFu));
  srd.z = -1;
  srd.w = 0x00020000;
  const uint32_t lds0 = (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)smem + (uint32_t)(w & 3) * 16384u +
                        (uint32_t)(w >> 2) * 65536u;
  const uint32_t voff = (uint32_t)lane * 16u + (uint32_t)w * 1024u;
  u32x4 sink = {0u, 0u, 0u, 0u};
  const uint32_t window = HOT == 1 ? 65536u : HOT == 2 ? 524288u : (uint32_t)std::min<long>(wg_bytes, 0x7fff0000L);

  bf16x8v a[4], b[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    for (int e = 0; e < 8; ++e) {
      a[i][e] = (__bf16)(((lane * 7 + i * 13 + e * 3) % 17) * 0.0625f - 0.5f);
      b[i][e] = (__bf16)(((lane * 5 + i * 11 + e * 7) % 19) * 0.0625f - 0.55f);
    }
  }
  f32x4 c16[16];
  f32x16 c32[4];
#pragma unroll
  for (int i = 0; i < 16; ++i) c16[i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int i = 0; i < 4; ++i) c32[i] = f32x16{};
  asm volatile("s_nop 4" ::: "memory");

  const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  uint32_t soff = 0;
  uint32_t roff = (uint32_t)lane * 16u + (uint32_t)w * 16384u;
  for (int it = 0; it < iters; ++it) {
    const uint32_t ldsb = lds0 + (uint32_t)(it & 7) * 2048u;
    bf16x8v rd[R > 0 ? R : 1];
#pragma unroll
    for (int m = 0; m < NM; ++m) {
      // DM 3: M0 for the DMA after this MFMA is formed BEFORE it (the MFMA covers the M0 -> LDS-DMA wait state)
      if constexpr (DM == 3) {
#pragma unroll
        for (int d = 0; d < DW; ++d) {
          if (BURST ? (m == 0 && d == 0) : (m == (d * NM) / DW))
            asm volatile("s_add_u32 m0, %0, %1" ::"s"(ldsb), "i"(0) : "m0", "scc");
        }
      }
      if constexpr (MF == 16) mf16(c16[m % 16], a[m & 3], b[(m >> 2) & 3]);
      else mf32(c32[m & 3], a[m & 3], b[(m >> 2) & 1]);
      // DMA slots: spread = evenly over the iteration; burst = all after MFMA 0
      if constexpr (DM != 0) {
#pragma unroll
        for (int d = 0; d < DW; ++d) {
          const bool here = BURST ? (m == 0) : (m == (d * NM) / DW);
          if (here) {
            const uint32_t o = (soff + (uint32_t)d * 4096u) % window;
            if constexpr (DM == 1) dma_buf<0>(srd, voff, o, ldsb + (uint32_t)(d & 1) * 1024u);
            else if constexpr (DM == 2) dma_glb<0>(base + o + voff, ldsb + (uint32_t)(d & 1) * 1024u);
            else if constexpr (DM == 3)
              asm volatile("buffer_load_dwordx4 %0, %1, %2 offen lds" ::"v"(voff), "s"(srd), "s"(o) : "memory", "m0");
            else {
              u32x4 v;
              asm volatile("buffer_load_dwordx4 %0, %1, %2, %3 offen" : "=v"(v) : "v"(voff), "s"(srd), "s"(o) : "memory");
              sink ^= v;
            }
          }
        }
      }
      if constexpr (R > 0) {
#pragma unroll
        for (int r = 0; r < R; ++r) {
          if (m == (r * NM) / R) {
            rd[r] = *reinterpret_cast<const bf16x8v*>(smem + ((roff + (uint32_t)r * 1024u) & 0xFFF0u));
          }
        }
      }
    }
    if constexpr (R > 0) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
      for (int r = 0; r < R && r < 4; ++r) b[r] = rd[r];
    }
    if constexpr (DM != 0) wait_vm<16>();
    if constexpr (BAR > 0) {
      if ((it % BAR) == BAR - 1) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
      }
    }
    soff += (uint32_t)DW * 4096u;
    roff += 64u;
  }
  wait_vm<0>();
  const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  if (tid == 0) {  // diagnostic stamps: their own buffer, never an output
    clk[2 * blockIdx.x] = t1 - t0;
    clk[2 * blockIdx.x + 1] = r1 - r0;
  }
  asm volatile("s_nop 7\n\ts_nop 7" ::: "memory");
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 16; ++i) s += c16[i][0] + c16[i][3];
#pragma unroll
  for (int i = 0; i < 4; ++i) s += c32[i][0] + c32[i][15];
  if constexpr (DM == 4) {
    wait_vm<0>();
    s += (float)(sink.x ^ sink.y ^ sink.z ^ sink.w);
  }
  out[blockIdx.x * NW * 64 + tid] = s;
}

struct Variant {
  const char* name;
  void (*fn)(const uint16_t*, long, float*, int, unsigned long long*);
  int threads = 256;
};

#define V(NAME, ...) Variant{NAME, probe<__VA_ARGS__>}
#define V8(NAME, ...) Variant{NAME, probe<__VA_ARGS__, 8>, 512}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 4000;
  const int rounds = argc > 2 ? atoi(argv[2]) : 5;
  int dev = 0, cus = 0;
  CK(hipGetDevice(&dev));
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  const int grid = cus;
  const long total = 1L << 30;  // 1 GiB source
  const long wg_bytes = total / grid / 4096 * 4096;
  uint16_t* src;
  float* out;
  unsigned long long* clk;
  CK(hipMalloc(&clk, (size_t)grid * 2 * 8));
  std::vector<unsigned long long> hclk((size_t)grid * 2);
  CK(hipMalloc(&src, total));
  CK(hipMalloc(&out, (size_t)grid * 512 * 4));
  {
    std::vector<uint16_t> h(1 << 20);
    for (size_t i = 0; i < h.size(); ++i) h[i] = (uint16_t)(0x3c00 + (i * 2654435761u >> 20) % 512);
    for (long o = 0; o < total; o += (long)h.size() * 2) CK(hipMemcpy((char*)src + o, h.data(), h.size() * 2, hipMemcpyHostToDevice));
  }
  const size_t lds = 136 * 1024;  // one workgroup per CU (8 waves: two 64 KB halves)
  std::vector<Variant> vs = {
      V("mf16 nodma", 16, 0, 2, false, 2, 0, 0),
      V("mf16 buf2 spread hot", 16, 1, 2, false, 1, 0, 0),
      V("mf16 buf2 burst hot", 16, 1, 2, true, 1, 0, 0),
      V("mf16 buf2 spread hot m0early", 16, 3, 2, false, 1, 0, 0),
      V("mf16 vld2 spread hot", 16, 4, 2, false, 1, 0, 0),
      V("mf16 glb2 spread hot", 16, 2, 2, false, 1, 0, 0),
      V("mf16 buf4 spread hot", 16, 1, 4, false, 1, 0, 0),
      V("mf16 buf2 spread mall", 16, 1, 2, false, 2, 0, 0),
      V("mf32 nodma", 32, 0, 2, false, 2, 0, 0),
      V("mf32 buf2 spread hot", 32, 1, 2, false, 1, 0, 0),
      V8("w8 mf16 nodma", 16, 0, 2, false, 2, 0, 0),
      V8("w8 mf16 buf2 spread hot", 16, 1, 2, false, 1, 0, 0),
      V8("w8 mf16 buf4 spread hot", 16, 1, 4, false, 1, 0, 0),
      V8("w8 mf16 buf2 spread mall", 16, 1, 2, false, 2, 0, 0),
      V8("w8 mf16 buf2 spread hot bar1", 16, 1, 2, false, 1, 0, 1),
      V("mf16 buf2 spread hot bar1", 16, 1, 2, false, 1, 0, 1),
  };

  for (auto& v : vs) CK(hipFuncSetAttribute((const void*)v.fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::vector<std::vector<float>> ts(vs.size());
  std::vector<std::vector<double>> ghz(vs.size()), cyc(vs.size());
  for (int r = 0; r < rounds; ++r) {
    for (size_t i = 0; i < vs.size(); ++i) {
      hipLaunchKernelGGL(vs[i].fn, dim3(grid), dim3(vs[i].threads), lds, 0, src, wg_bytes, out, iters, clk);
      CK(hipEventRecord(e0));
      hipLaunchKernelGGL(vs[i].fn, dim3(grid), dim3(vs[i].threads), lds, 0, src, wg_bytes, out, iters, clk);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms = 0.f;
      CK(hipEventElapsedTime(&ms, e0, e1));
      ts[i].push_back(ms);
      CK(hipMemcpy(hclk.data(), clk, hclk.size() * 8, hipMemcpyDeviceToHost));
      std::vector<double> g, c;
      for (int b = 0; b < grid; ++b) {
        g.push_back((double)hclk[2 * b] / (double)hclk[2 * b + 1] * 0.1);  // GHz (memrealtime: 100 MHz)
        c.push_back((double)hclk[2 * b] / iters);
      }
      std::sort(g.begin(), g.end());
      std::sort(c.begin(), c.end());
      ghz[i].push_back(g[g.size() / 2]);
      cyc[i].push_back(c[c.size() / 2]);
    }
  }
  double base16 = 0, base32 = 0;
  printf("# %d CUs, %d iterations of 256 matrix-pipe cycles per wave, median of %d rounds\n", cus, iters, rounds);
  printf("%-34s %10s %10s %10s %10s %10s\n", "variant", "ns/iter", "rel", "TF/s", "cyc/iter", "GHz");
  for (size_t i = 0; i < vs.size(); ++i) {
    std::sort(ts[i].begin(), ts[i].end());
    const double ms = ts[i][ts[i].size() / 2];
    const double ns = ms * 1e6 / iters;
    if (i == 0) base16 = ns;
    if (std::string(vs[i].name) == "mf32 nodma") base32 = ns;
    const double flop = (double)grid * 4 * iters * 16 * (16.0 * 16 * 32 * 2);
    const double ref = std::string(vs[i].name).find("mf32") == 0 && base32 > 0 ? base32 : base16;
    std::sort(ghz[i].begin(), ghz[i].end());
    std::sort(cyc[i].begin(), cyc[i].end());
    printf("%-34s %10.2f %10.3f %10.1f %10.1f %10.3f\n", vs[i].name, ns, ns / ref, flop / (ms * 1e-3) / 1e12,
           cyc[i][cyc[i].size() / 2], ghz[i][ghz[i].size() / 2]);
  }
  CK(hipFree(clk));
  CK(hipFree(src));
  CK(hipFree(out));
  return 0;
}
